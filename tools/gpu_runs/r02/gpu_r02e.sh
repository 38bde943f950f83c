#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest mpjbuf" && timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -k "mpjbuf" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest_mpjbuf.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_mpjbuf.log"; [ $rc -eq 0 ] || exit $rc
echo "== mpjbuf timing" && timeout -k 10 300 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 --mpjbuf > "$OUT/pway_mpjbuf.jsonl" 2>&1 && cat "$OUT/pway_mpjbuf.jsonl" &&
echo "== e2e" && timeout -k 10 300 python tools/e2e_bench.py > "$OUT/e2e.json" 2>&1 && cat "$OUT/e2e.json"
