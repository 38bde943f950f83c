#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python tools/slot_layout.py 2>&1 | tee gpurun_out/r03k_slot_layout.jsonl
