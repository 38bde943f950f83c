#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug/c4_check.py 2>&1 | tee gpurun_out/r03e_c4.txt
