#!/bin/bash
# round 3: JGF MolDyn refval through libmpjx (in-place Allreduces), then the JGF SparseMatmult pin again
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v -k "moldyn or jgf" -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03g_pytest.log" 2>&1
rc=$?; tail -45 "$OUT/r03g_pytest.log"; exit $rc
