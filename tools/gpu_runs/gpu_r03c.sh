#!/bin/bash
# round 3: new tests (IPC Split, caller stream destroyed, smp devices mismatch, faithful buffers) + N=1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_ipc.py -m gpu -v -x -k "split or destroyed or mismatches or faithful or jgf" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r03c_pytest.log" 2>&1
rc=$?; tail -12 "$OUT/r03c_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/r03c_bench.json" 2> "$OUT/r03c_bench.err"
rc=$?; tail -c 3000 "$OUT/r03c_bench.json"; exit $rc
