#!/bin/bash
# big-endian bodies as kernels of their own (native streaming kernels at full occupancy): parity of the
# combine + byte-order tests, smoke, stagger/library A/B, the library's engine-shape timings, N=1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r03w_smoke.log" 2>&1 && tail -1 "$OUT/r03w_smoke.log" &&
echo "== pytest combine + byte order" && timeout -k 10 900 python -u -m pytest tests/test_gpu_combine.py tests/test_gpu_collectives.py -k "combine or endian or mpjbuf or streaming or swap or scan or Scan" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03w_pytest.log" 2>&1 && tail -2 "$OUT/r03w_pytest.log" &&
echo "== tune_stagger" && timeout -k 10 300 tools/tuning/tune_stagger 7 > "$OUT/r03w_stagger.jsonl" 2>&1 && cat "$OUT/r03w_stagger.jsonl" &&
echo "== split_lib" && timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03w_lib.jsonl" 2>&1 && grep '^{' "$OUT/r03w_lib.jsonl" &&
echo "== bench n1" && timeout -k 10 400 python bench.py > "$OUT/r03w_bench_n1.json" 2> "$OUT/r03w_bench_n1.err" && tail -c 300 "$OUT/r03w_bench_n1.json"
