#!/bin/bash
# Infinity-Cache reuse check: every timed kernel shape on the same buffers every launch (rotate 1, the
# bench's pattern) against R independent buffer sets cycled per launch (nothing left in the 256 MiB
# cache from the previous launch). Each step under its own time limit; the chain stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cold
mkdir -p "$OUT"
for R in 1 4; do
  echo "== 256 MiB rotate $R" && timeout -k 10 120 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 \
      --combine --copies --iters 24 --rotate $R >> "$OUT/pway256.jsonl" || exit $?
done
for R in 1 8; do
  echo "== 32 MiB rotate $R" && timeout -k 10 120 python tools/bench_pway.py --mib-per-slice 32 \
      --cases MST:8,SCAN:8,FOLD:2,SCAN:2,MST:4 --copies --iters 40 --rotate $R >> "$OUT/pway32.jsonl" || exit $?
done
cat "$OUT"/*.jsonl
