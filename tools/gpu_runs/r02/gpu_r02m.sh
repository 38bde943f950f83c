#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pway" && for mib in 8 32 256; do timeout -k 10 200 python tools/bench_pway.py --mib-per-slice $mib --cases MST:5,MST:8,FOLD:6,FOLD:8,SCAN:5,SCAN:8 > "$OUT/pway_u2_$mib.jsonl" 2>&1 || exit $?; done && cat "$OUT"/pway_u2_*.jsonl | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  %-5s P=%d %4d MiB %8.1f us %.3f' % (d['order'], d['P'], d['slice_MiB'], d['us'], d['frac_8TBps']))"
