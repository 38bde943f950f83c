#!/bin/bash
# rocprofv3 passes over the N=1 bench: kernel trace + stats, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950). Outputs under gpurun_out/prof_*.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_trace" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 > "$OUT/prof_trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/prof_fetch" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/prof_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/prof_write" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/prof_write.log" 2>&1
rc=$?; echo "profile rc=$rc"; exit $rc
