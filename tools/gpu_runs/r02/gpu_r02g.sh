#!/bin/bash
# cache-policy sweep of the real kernels: default threshold vs higher NT thresholds, in-place policy on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
C=MST:8,MST:4,FOLD:2,FOLD:4,SCAN:2,SCAN:8
for cfg in "64 1" "64 0" "320 1" "1024 1"; do
  set -- $cfg
  echo "== NT_MIN_MIB=$1 INPLACE=$2"
  for mib in 8 32 256; do
    MPJX_NT_MIN_MIB=$1 MPJX_INPLACE_POLICY=$2 timeout -k 10 200 python tools/bench_pway.py --mib-per-slice $mib --cases $C --iters 20 > "$OUT/pol_$1_$2_$mib.jsonl" 2>&1 || exit $?
    grep '^{' "$OUT/pol_$1_$2_$mib.jsonl" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  %-5s P=%d %4d MiB %8.1f us %.3f' % (d['order'], d['P'], d['slice_MiB'], d['us'], d['frac_8TBps']))"
  done
done
echo "== bench N=1 (in-place policy on)" && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_pol.json" 2>&1 && grep '^{' "$OUT/bench_pol.json" | tail -c 700
echo "== bench N=1 (in-place policy off)" && MPJX_INPLACE_POLICY=0 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_pol0.json" 2>&1 && grep '^{' "$OUT/bench_pol0.json" | tail -c 700
