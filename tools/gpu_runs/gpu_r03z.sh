#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) of the round-3 session-2 k_pway kernels at
# the engines' combine shapes (tools/tuning/split_lib.py: library path, skewed slots, cold sets)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
echo "== fetch" && ITERS=5 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/r03z_fetch" -o lib -- python3 "$R/tools/tuning/split_lib.py" > "$OUT/r03z_fetch.log" 2>&1 &&
echo "== write" && ITERS=5 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/r03z_write" -o lib -- python3 "$R/tools/tuning/split_lib.py" > "$OUT/r03z_write.log" 2>&1 &&
echo done
