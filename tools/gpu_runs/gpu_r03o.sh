#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_cpp.py -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r03o_pytest_cpp.log 2>&1
rc=$?; tail -12 gpurun_out/r03o_pytest_cpp.log; timeout -k 10 300 tests/cpp/jgf_tests 1 4 | tee gpurun_out/r03o_jgf_native.txt; exit $rc
