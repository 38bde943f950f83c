#!/bin/bash
# round 3 session 2 checkpoint after the k_pway changes (own kernels for big-endian bodies, K_SCAN early
# stores, per-shape load groups): whole GPU suite, smoke, N=1 bench + kernel trace, the stagger A/B
# (library default vs each G), N>1 rehearsals (world-1 RCCL/IPC, 4 rank processes on one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03zl_pytest.log" 2>&1 && tail -2 "$OUT/r03zl_pytest.log" &&
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r03zl_smoke.log" 2>&1 && tail -1 "$OUT/r03zl_smoke.log" &&
echo "== bench n1" && timeout -k 10 400 python bench.py > "$OUT/r03zl_bench_n1.json" 2> "$OUT/r03zl_bench_n1.err" && tail -c 300 "$OUT/r03zl_bench_n1.json" &&
echo "== rocprof" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03zl_prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 > "$OUT/r03zl_rocprof.log" 2>&1) &&
echo "== world-1 allreduce" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/r03zl_bench_ar1.json" 2> "$OUT/r03zl_bench_ar1.err" && tail -c 300 "$OUT/r03zl_bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/r03zl_bench_od4.json" 2> "$OUT/r03zl_bench_od4.err" && tail -c 300 "$OUT/r03zl_bench_od4.json"
