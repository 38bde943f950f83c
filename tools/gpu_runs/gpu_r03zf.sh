#!/bin/bash
# K_SCAN P=8 with contiguous input slots and skewed output slots (the RCCL engine's Scan layout)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
echo "== tune_stagger in 0 / out 4096" && timeout -k 10 300 tools/tuning/tune_stagger 7 0 4096 > "$OUT/r03zf_stagger_in0_out4k.jsonl" 2>&1 && grep library "$OUT/r03zf_stagger_in0_out4k.jsonl" &&
echo "== split_lib in 0" && SKEW=0 timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03zf_lib_in0.jsonl" 2>&1 && grep '^{' "$OUT/r03zf_lib_in0.jsonl"
