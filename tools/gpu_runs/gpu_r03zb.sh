#!/bin/bash
# layout-aware load group (K_MST P=8 staggered in pairs when the operand streams are congruent mod 16 MiB):
# parity of the combine/collective tests, the library path in both slot layouts, the sweep at skew 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest combine + collectives" && timeout -k 10 900 python -u -m pytest tests/test_gpu_combine.py tests/test_gpu_collectives.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03zb_pytest.log" 2>&1 && tail -2 "$OUT/r03zb_pytest.log" &&
echo "== split_lib skew 0" && SKEW=0 timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03zb_lib_skew0.jsonl" 2>&1 && grep '^{' "$OUT/r03zb_lib_skew0.jsonl" &&
echo "== split_lib skew 4096" && timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03zb_lib_skew4k.jsonl" 2>&1 && grep '^{' "$OUT/r03zb_lib_skew4k.jsonl" &&
echo "== tune_stagger skew 0" && timeout -k 10 300 tools/tuning/tune_stagger 7 0 > "$OUT/r03zb_stagger_skew0.jsonl" 2>&1 && grep library "$OUT/r03zb_stagger_skew0.jsonl"
