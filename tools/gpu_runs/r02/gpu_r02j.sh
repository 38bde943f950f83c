#!/bin/bash
# round-2 GPU step: P-way kernels after the 512 MiB non-temporal threshold (timing + PMC of the N=8
# combine shape), then the whole suite, smoke, bench, rocprof trace + PMC of the N=1 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pway" && for mib in 8 32 256; do timeout -k 10 200 python tools/bench_pway.py --mib-per-slice $mib --copies > "$OUT/pway_thr512_$mib.jsonl" 2>&1 || exit $?; done && cat "$OUT"/pway_thr512_*.jsonl | grep '^{' &&
(cd /tmp && for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_thr512_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 32 --cases MST:8,SCAN:8,SCAN:2,FOLD:2 > "$OUT/pmc_thr512_$ctr.log" 2>&1 || exit $?
done) &&
bash tools/gpu_check.sh && bash tools/profile.sh
