#!/bin/bash
# round-2 GPU step: PMC traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) of the cold-retuned
# kernels at every shape the bench reports, plus the N=1 bench's kernel trace (tools/profile.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/profile.sh || exit $?
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=0
  for args in "--mib-per-slice 32 --cases MST:8,SCAN:8,SCAN:2,FOLD:2 --copies" "--mib-per-slice 8 --cases MST:8" \
              "--mib-per-slice 128 --cases FOLD:2" "--mib-per-slice 64 --cases MST:4" \
              "--mib-per-slice 256 --cases FOLD:2 --big-endian"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_cold_${i}_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 $args > "$OUT/pmc_cold_${i}_$ctr.log" 2>&1 || exit $?
  done
done
echo pmc done
