#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v -k "int32_range or slot_skew or rccl_transport" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03l_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r03l_pytest.log; exit $rc
