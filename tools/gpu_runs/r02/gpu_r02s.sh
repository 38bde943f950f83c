#!/bin/bash
# round-2 GPU step: every op family / element width through the streaming kernels on cold operands
# (N=8 combine shape K_MST P=8 on 32 MiB slices, Scan P=8, and the 2 x 256 MiB fold).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
for ot in 3:8 1:7 6:5 10:6 3:1 1:3 4:6 2:2 5:4 11:0x108 12:0x105; do
  op=${ot%%:*}; ty=${ot##*:}
  timeout -k 10 120 python tools/bench_pway.py --mib-per-slice 32 --cases MST:8,SCAN:8 --rotate 4 --op $op --type $ty --iters 20 >> "$OUT/types_cold.jsonl" || exit $?
  timeout -k 10 120 python tools/bench_pway.py --mib-per-slice 256 --cases FOLD:2 --combine --rotate 4 --op $op --type $ty --iters 20 >> "$OUT/types_cold.jsonl" || exit $?
done
cat "$OUT/types_cold.jsonl"
