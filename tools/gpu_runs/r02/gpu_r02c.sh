#!/bin/bash
# round-2 GPU step: full GPU suite + smoke, configs[4] pipeline overlap (timing + kernel trace), the
# P-way combine at the pipeline-chunk shape (8 MiB slices) with its PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== c5 overlap" && timeout -k 10 300 python tools/c5_overlap.py --calls 3 > "$OUT/c5_overlap.json" 2> "$OUT/c5_overlap.err" && cat "$OUT/c5_overlap.json" &&
echo "== pway 8 MiB" && timeout -k 10 300 python tools/bench_pway.py --mib-per-slice 8 --cases MST:8,MST:4,FOLD:2 --iters 50 > "$OUT/pway_8.jsonl" 2>&1 && cat "$OUT/pway_8.jsonl" &&
cd /tmp &&
echo "== c5 trace" && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c5_trace" -o c5 -- python3 "$R/tools/c5_overlap.py" --trace-run > "$OUT/c5_trace.log" 2>&1 &&
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr" &&
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_pway8_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 8 --cases MST:8 > "$OUT/pmc_pway8_$ctr.log" 2>&1 || exit $?
done
echo "rc=$?"
