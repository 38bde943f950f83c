#!/bin/bash
# round 3: the JGF SparseMatmult refval pin and the topo/map KAT on the GPU path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v -k "jgf or topo" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r03a_pytest.log" 2>&1
rc=$?; tail -30 "$OUT/r03a_pytest.log"; exit $rc
