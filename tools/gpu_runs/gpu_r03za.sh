#!/bin/bash
# the load-group sweep in the RCCL exchange engine's layout (input slots contiguous: skew 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
echo "== tune_stagger skew 0" && timeout -k 10 300 tools/tuning/tune_stagger 7 0 > "$OUT/r03za_stagger_skew0.jsonl" 2>&1 && grep library "$OUT/r03za_stagger_skew0.jsonl"
