#!/bin/bash
# load-issue pattern experiment (tune_stagger) + library-vs-harness A/B (tune_split), then kernel-trace
# durations of the stagger variants (no launch gaps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tune_stagger" && timeout -k 10 300 tools/tuning/tune_stagger 7 > "$OUT/r03u_stagger.jsonl" 2>&1 && cat "$OUT/r03u_stagger.jsonl" &&
echo "== tune_split" && timeout -k 10 300 tools/tuning/tune_split 5 > "$OUT/r03u_split.jsonl" 2>&1 && grep -E "64MiB|P8" "$OUT/r03u_split.jsonl" &&
cd /tmp && echo "== rocprof stagger" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03u_prof" -o st -- "$R/tools/tuning/tune_stagger" 2 > "$OUT/r03u_prof.log" 2>&1 && echo done
