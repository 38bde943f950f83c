#!/bin/bash
# round 3: phase-timing test; N=1 bench (with the MST CPU baseline); world-1 RCCL Allreduce rehearsal and
# 4 rank processes on one GPU (IPC) — the N>1 bench flow with its new parity/phases/e2e fields
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v -x -k "phase_timing or rccl_transport or pipelined or config5" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r03d_pytest.log" 2>&1
rc=$?; tail -6 "$OUT/r03d_pytest.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench n1" && timeout -k 10 400 python bench.py > "$OUT/r03d_bench_n1.json" 2> "$OUT/r03d_bench_n1.err" && tail -c 1500 "$OUT/r03d_bench_n1.json" &&
echo "== world-1 allreduce" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/r03d_bench_ar1.json" 2> "$OUT/r03d_bench_ar1.err" && tail -c 1500 "$OUT/r03d_bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/r03d_bench_od4.json" 2> "$OUT/r03d_bench_od4.err" && tail -c 1500 "$OUT/r03d_bench_od4.json"
