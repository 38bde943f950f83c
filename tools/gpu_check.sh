#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel stats. Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
(rocm-smi --showproductname; nproc; lscpu | head -20) > "$OUT/host.txt" 2>&1 || true
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 ;
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 && cat "$OUT/bench.log" &&
echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rc=$rc"; exit $rc
