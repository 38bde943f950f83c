#!/bin/bash
# kernel-trace durations (no launch gaps) of the library's P-way kernels vs the tune_split harness kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
echo "== rocprof split_lib" && ITERS=30 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03t_prof_lib" -o lib -- python3 "$R/tools/tuning/split_lib.py" > "$OUT/r03t_lib.jsonl" 2>&1 &&
echo "== rocprof tune_split" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03t_prof_harness" -o h -- "$R/tools/tuning/tune_split" 3 > "$OUT/r03t_harness.jsonl" 2>&1 &&
echo done
