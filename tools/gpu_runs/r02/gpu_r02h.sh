#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tune_policy3" && timeout -k 10 200 ./tools/tune_policy3 7 > "$OUT/tune_policy3_fixed.txt" 2>&1 && cat "$OUT/tune_policy3_fixed.txt" &&
echo "== bench N=1" && timeout -k 10 300 python bench.py > "$OUT/bench_pol2.json" 2> "$OUT/bench_pol2.err" && grep '^{' "$OUT/bench_pol2.json" | tail -c 1400 &&
echo "== pway" && timeout -k 10 200 python tools/bench_pway.py --copies --cases FOLD:2,MST:8 > "$OUT/pway_after.jsonl" 2>&1 && grep '^{' "$OUT/pway_after.jsonl" &&
echo "== pytest" && timeout -k 10 600 python -u -m pytest tests/test_gpu_combine.py tests/test_gpu_collectives.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_pol2.log" 2>&1; rc=$?; tail -2 "$OUT/pytest_pol2.log"; exit $rc
