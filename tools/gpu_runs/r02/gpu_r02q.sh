#!/bin/bash
# round-2 GPU step: the N>1 bench flow after the cold-operand changes — world-size-1 Allreduce rehearsal
# (RCCL engine at P = 1) and 4 rank processes on one GPU (IPC engines, hbm_combine with cycled sets).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== world-1 allreduce" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/bench_ar1.json" 2> "$OUT/bench_ar1.err" && tail -c 2500 "$OUT/bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/bench_od4.json" 2> "$OUT/bench_od4.err" && tail -c 3000 "$OUT/bench_od4.json"
