#!/bin/bash
# round 3 checkpoint B: N=1 bench, its rocprofv3 kernel trace, the N>1 rehearsals
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== bench n1" && timeout -k 10 400 python bench.py > "$OUT/r03j_bench_n1.json" 2> "$OUT/r03j_bench_n1.err" && tail -c 600 "$OUT/r03j_bench_n1.json" &&
echo "== rocprof" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03j_prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 > "$OUT/r03j_rocprof.log" 2>&1) &&
echo "== world-1 allreduce" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/r03j_bench_ar1.json" 2> "$OUT/r03j_bench_ar1.err" && tail -c 300 "$OUT/r03j_bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/r03j_bench_od4.json" 2> "$OUT/r03j_bench_od4.err" && tail -c 300 "$OUT/r03j_bench_od4.json"
