#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pway" && for mib in 8 32 256; do timeout -k 10 200 python tools/bench_pway.py --mib-per-slice $mib --copies > "$OUT/pway_pol3_$mib.jsonl" 2>&1 || exit $?; done && cat "$OUT"/pway_pol3_*.jsonl | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  %-5s P=%d %4d MiB %8.1f us %.3f' % (d['order'], d['P'], d['slice_MiB'], d['us'], d['frac_8TBps']))" &&
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_pol3.json" 2>&1 && grep '^{' "$OUT/bench_pol3.json" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_us'], d['roofline']['frac'], d['allreduce_p1']['frac'], d['parity'])" &&
echo "== pytest" && timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_combine.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_pol3.log" 2>&1; rc=$?; tail -2 "$OUT/pytest_pol3.log"; exit $rc
