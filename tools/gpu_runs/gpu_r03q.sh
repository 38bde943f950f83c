#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_ipc.py -m gpu -v -k "microbenchmark or faithful" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03q_pytest.log 2>&1
rc=$?; tail -16 gpurun_out/r03q_pytest.log; exit $rc
