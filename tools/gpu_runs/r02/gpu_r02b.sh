#!/bin/bash
# round-2 GPU step: fused big-endian kernels (parity), collectives/combine regression, N=1 bench,
# P-way kernel timings (native and big-endian) and their PMC traffic (one counter per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest" && timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_combine.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_be.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_be.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_b.json" 2> "$OUT/bench_b.err" && tail -c 600 "$OUT/bench_b.json" &&
echo "== bench world-1 allreduce rehearsal" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --allreduce --steps 10 --warmup 3 > "$OUT/bench_ar1.json" 2> "$OUT/bench_ar1.err" && tail -c 1500 "$OUT/bench_ar1.json" &&
echo "== pway" && timeout -k 10 300 python tools/bench_pway.py --copies > "$OUT/pway_32.jsonl" 2>&1 &&
timeout -k 10 300 python tools/bench_pway.py --big-endian > "$OUT/pway_32_be.jsonl" 2>&1 &&
timeout -k 10 300 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 > "$OUT/pway_256.jsonl" 2>&1 &&
timeout -k 10 300 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 --big-endian > "$OUT/pway_256_be.jsonl" 2>&1 &&
cat "$OUT"/pway_*.jsonl &&
cd /tmp &&
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr" &&
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_pway32_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --cases MST:8,SCAN:8,SCAN:2,FOLD:2 --copies > "$OUT/pmc_pway32_$ctr.log" 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_pway256be_$ctr" -o p -- python3 "$R/tools/bench_pway.py" --iters 3 --mib-per-slice 256 --cases FOLD:2 --big-endian > "$OUT/pmc_pway256be_$ctr.log" 2>&1 || exit $?
done
echo "rc=$?"
