#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest" && timeout -k 10 900 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_collectives.py tests/test_gpu_combine.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_copy.log" 2>&1; rc=$?
tail -2 "$OUT/pytest_copy.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_copy.json" 2>&1 && grep '^{' "$OUT/bench_copy.json" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_us'], d['roofline']['frac'], d['allreduce_p1'])"
