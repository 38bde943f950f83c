#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per pass) of the N=1 bench on the final round-3 build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
echo "== fetch" && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/r03zj_fetch" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/r03zj_fetch.log" 2>&1 &&
echo "== write" && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/r03zj_write" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/r03zj_write.log" 2>&1 &&
echo done
