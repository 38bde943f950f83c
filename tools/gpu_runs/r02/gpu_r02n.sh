#!/bin/bash
# PMC traffic of the hbm_combine shapes of the N=2 and N=4 bench lines (FOLD P=2 on 128 MiB slices,
# MST P=4 on 64 MiB slices), one counter per pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_n24_a_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 128 --cases FOLD:2 > "$OUT/pmc_n24_a_$ctr.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_n24_b_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 64 --cases MST:4 > "$OUT/pmc_n24_b_$ctr.log" 2>&1 || exit $?
done
echo pmc done
