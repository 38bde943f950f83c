#!/bin/bash
# ipc_stress.sh over staging allocation classes and modes; stops at a fault or time limit (any exit
# other than 0 = clean or 5 = wrong results seen).
cd "$(dirname "$0")"
P=${1:-8}; IT=${2:-400}
shift 2
for combo in "${@:-coarse:push coarse:pull fine:push uncached:push}"; do
  for c in $combo; do
    export MPJX_IPC_STAGE_ALLOC=${c%%:*} MPJX_IPC_MODE=${c##*:}
    ./ipc_stress.sh "$P" "$IT" 2>&1 | grep -v "^rank .*0 bad calls" | head -40
    rc=${PIPESTATUS[0]}
    [ "$rc" -eq 0 ] || [ "$rc" -eq 5 ] || exit "$rc"
  done
done
