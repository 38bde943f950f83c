#!/bin/bash
# streaming form without the grid-stride loop: parity (combine + collectives), library A/B, N=1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest combine + collectives" && timeout -k 10 900 python -u -m pytest tests/test_gpu_combine.py tests/test_gpu_collectives.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/r03zi_pytest.log" 2>&1 && tail -2 "$OUT/r03zi_pytest.log" &&
echo "== tune_stagger" && timeout -k 10 300 tools/tuning/tune_stagger 9 > "$OUT/r03zi_stagger.jsonl" 2>&1 && grep -E "default|G2 \(both|G8 \(all|G4 \(all" "$OUT/r03zi_stagger.jsonl" &&
echo "== bench n1" && timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/r03zi_bench_n1.json" 2> "$OUT/r03zi_bench_n1.err" && python -c "import json;d=json.loads(open('$OUT/r03zi_bench_n1.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_us'],d['roofline']['frac'],d['parity'])"
