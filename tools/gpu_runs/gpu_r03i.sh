#!/bin/bash
# round 3 checkpoint A: smoke + the whole GPU suite on the current build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r03i_smoke.log" 2>&1 && tail -2 "$OUT/r03i_smoke.log" &&
echo "== pytest gpu" && timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03i_pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/r03i_pytest_gpu.log"; exit $rc
