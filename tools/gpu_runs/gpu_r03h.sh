#!/bin/bash
# round 3: operand-slot placement experiment
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
SKEW_SET=fine timeout -k 10 700 python tools/slot_skew.py --iters 30 2>&1 | tee gpurun_out/r03h_slot_skew_fine.jsonl
