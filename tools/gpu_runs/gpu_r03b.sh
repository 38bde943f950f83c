#!/bin/bash
# round 3: faithful-mode buffer side effects (every rank's recvbuf, BKT sendbuf), then the whole GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v -x -k "faithful" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r03b_faithful.log" 2>&1
rc=$?; tail -15 "$OUT/r03b_faithful.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r03b_pytest_gpu.log" 2>&1
rc=$?; tail -15 "$OUT/r03b_pytest_gpu.log"; exit $rc
