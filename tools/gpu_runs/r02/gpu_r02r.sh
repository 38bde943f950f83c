#!/bin/bash
# round-2 GPU step on the final build: native combine bench (the /opt/rocm runtime pairing), full GPU
# suite + smoke, N=1 bench, its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== native combine" && timeout -k 10 120 tools/combine_bench 20 5 4 > "$OUT/combine_bench.json" 2>&1 && cat "$OUT/combine_bench.json" &&
timeout -k 10 120 tools/combine_bench 20 5 4 >> "$OUT/combine_bench.json" 2>&1 && tail -1 "$OUT/combine_bench.json" &&
bash tools/gpu_check.sh
