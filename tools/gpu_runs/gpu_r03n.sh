#!/bin/bash
# round 3: the two-lane pipeline with more hardware queues per process (multicore ranks share ONE
# process here, so 4 queues serialise their streams; one process per GPU uses 3-4 streams)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--lanes 2 --chunk-mib 64" "--lanes 4 --chunk-mib 64"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python tools/c5_overlap.py $args --calls 3 >> gpurun_out/r03n_lanes_hwq16.jsonl 2> gpurun_out/r03n.err || exit $?
done
cut -c1-600 gpurun_out/r03n_lanes_hwq16.jsonl
