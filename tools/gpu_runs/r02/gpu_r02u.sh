#!/bin/bash
# round-2 final GPU step: full suite + smoke + N=1 bench + rocprof trace (tools/gpu_check.sh), configs[0]
# CPU vs GPU, the world-1 Allreduce rehearsal and 4 rank processes on one GPU (the N>1 bench flow).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
bash tools/gpu_check.sh || exit $?
echo "== configs[0]" && timeout -k 10 200 python tools/cpu_baseline_c1.py > "$OUT/config0.json" 2>&1 && tail -1 "$OUT/config0.json" &&
echo "== world-1 allreduce" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/bench_ar1.json" 2> "$OUT/bench_ar1.err" && tail -c 600 "$OUT/bench_ar1.json" &&
echo "== one-device x4" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > "$OUT/bench_od4.json" 2> "$OUT/bench_od4.err" && tail -c 600 "$OUT/bench_od4.json"
