#!/bin/bash
# round 3: re-run the N>1 bench rehearsals after the stream-sync fix (world-1 RCCL/IPC, 4 procs on one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
echo "== world-1 allreduce" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/r03f_bench_ar1.json" 2> "$OUT/r03f_bench_ar1.err" && tail -c 400 "$OUT/r03f_bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/r03f_bench_od4.json" 2> "$OUT/r03f_bench_od4.err" && tail -c 400 "$OUT/r03f_bench_od4.json"
