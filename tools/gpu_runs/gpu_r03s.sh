#!/bin/bash
# round 3 re-entry: rebuilt tree sanity (smoke, N=1 bench) + split/region experiment for K_MST P=4 64 MiB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r03s_smoke.log" 2>&1 && tail -1 "$OUT/r03s_smoke.log" &&
echo "== tune_split" && timeout -k 10 300 tools/tuning/tune_split 7 > "$OUT/r03s_tune_split.jsonl" 2>&1 && cat "$OUT/r03s_tune_split.jsonl" &&
echo "== split_lib" && timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03s_split_lib_none.jsonl" 2>&1 &&
MPJX_PWAY_SPLIT_KIB=32768 timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03s_split_lib_32.jsonl" 2>&1 &&
MPJX_PWAY_SPLIT_KIB=16384 timeout -k 10 200 python tools/tuning/split_lib.py > "$OUT/r03s_split_lib_16.jsonl" 2>&1 &&
cat "$OUT"/r03s_split_lib_*.jsonl &&
echo "== bench n1" && timeout -k 10 400 python bench.py > "$OUT/r03s_bench_n1.json" 2> "$OUT/r03s_bench_n1.err" && tail -c 600 "$OUT/r03s_bench_n1.json"
