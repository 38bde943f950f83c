#!/bin/bash
# Run tools/ipc_stress as P rank processes on one GPU: ipc_stress.sh P ITERATIONS [DEVICE]
# (MPJX_IPC_MODE / MPJX_IPC_STAGE_ALLOC pass through). Exit 0 when every rank saw every result right.
export MPJX_IPC_OVERSUBSCRIBE=${MPJX_IPC_OVERSUBSCRIBE:-1}  # rank processes share one GPU
P=${1:-8}; IT=${2:-500}; DEV=${3:-0}
cd "$(dirname "$0")"
ID=$(head -c 128 /dev/urandom | od -An -tx1 -v | tr -d ' \n')
pids=()
for ((r = 0; r < P; r++)); do
  timeout -k 10 300 ./ipc_stress "$r" "$P" "$DEV" "$ID" "$IT" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "ipc_stress P=$P it=$IT mode=${MPJX_IPC_MODE:-push} alloc=${MPJX_IPC_STAGE_ALLOC:-coarse}: rc=$rc"
exit $rc
