#!/bin/bash
# PMC traffic of the P-way 32 MiB shapes under the round-2 policies (POL 3 below the 512 MiB threshold)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_pol3_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 32 --cases MST:8,SCAN:8,SCAN:2,FOLD:2 --copies > "$OUT/pmc_pol3_$ctr.log" 2>&1 || exit $?
done
echo pmc done
