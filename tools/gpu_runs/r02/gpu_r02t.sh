#!/bin/bash
# round-2 GPU step after the lazy cross-stream ordering event: full suite + smoke + N=1 bench + rocprof
# trace, then the world-1 Allreduce rehearsal (every engine through the N>1 bench flow).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
bash tools/gpu_check.sh || exit $?
echo "== world-1 allreduce" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/bench_ar1.json" 2> "$OUT/bench_ar1.err" && tail -c 1200 "$OUT/bench_ar1.json"
