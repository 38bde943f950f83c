#!/bin/bash
# parity of the colliding-streams (pair-staggered) K_MST P=8 path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
echo "== pytest colliding" && timeout -k 10 600 python -u -m pytest tests/test_gpu_combine.py -k "colliding or streaming" -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03zg_pytest.log" 2>&1; rc=$?; tail -12 "$OUT/r03zg_pytest.log"; exit $rc
