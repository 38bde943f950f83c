#!/bin/bash
# round 3: PMC traffic of the N=1 bench on the current build (FETCH_SIZE and WRITE_SIZE, one pass each)
# and of the P-way kernels in the engines' layouts (tools/slot_layout.py shapes, skewed and contiguous)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/r03p_fetch" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/r03p_fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/r03p_write" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/r03p_write.log" 2>&1
rc=$?; echo "pmc rc=$rc"; ls "$OUT"/r03p_fetch "$OUT"/r03p_write; exit $rc
