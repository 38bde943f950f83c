#!/bin/bash
# the library's combine at BASELINE configs[3]/[4] shapes for N = 2/4/8 in the RCCL engine's layout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
echo "== config_shapes" && timeout -k 10 300 python tools/tuning/config_shapes.py > "$OUT/r03zd_config_shapes.jsonl" 2>&1 && grep '^{' "$OUT/r03zd_config_shapes.jsonl"
