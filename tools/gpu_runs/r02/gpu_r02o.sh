#!/bin/bash
# round-2 GPU step after the cold-operand retune (1024-lane non-temporal streaming tiles, no cache-reuse
# policies): the library's kernels cold and warm, the full GPU suite + smoke, the N=1 bench (cold
# operand sets), its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_cold.sh > "$OUT/cold.log" 2>&1 || { tail -5 "$OUT/cold.log"; exit 1; }
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 170 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 && tail -c 3000 "$OUT/bench.log" &&
echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rc=$rc"; exit $rc
