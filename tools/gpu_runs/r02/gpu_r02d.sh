#!/bin/bash
# round-2 GPU step: C++ KATs (incl. the RCCL engine bound to /opt/rocm), mpjbuf combine timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest cpp" && timeout -k 10 600 python -u -m pytest tests/test_gpu_cpp.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_cpp.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_cpp.log"; [ $rc -eq 0 ] || exit $rc
echo "== mpjbuf" && timeout -k 10 300 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 --mpjbuf > "$OUT/pway_mpjbuf.jsonl" 2>&1 && cat "$OUT/pway_mpjbuf.jsonl"
