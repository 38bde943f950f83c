#!/bin/bash
# round 3: the chunk pipeline's two lanes on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--lanes 4 --chunk-mib 64" "--lanes 8 --chunk-mib 64" "--lanes 4 --chunk-mib 16"; do
  timeout -k 10 300 python tools/c5_overlap.py $args --calls 3 >> gpurun_out/r03m_lanes.jsonl 2> gpurun_out/r03m_lanes.err || exit $?
done
cut -c1-700 gpurun_out/r03m_lanes.jsonl
