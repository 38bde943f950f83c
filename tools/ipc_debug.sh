#!/bin/bash
# Debug helper: run the IPC test cases for P ranks directly (worker stderr kept per rank).
P=${1:-2}
OUT=gpurun_out/ipc_dbg
mkdir -p $OUT
python - <<PY
import json, sys
sys.path[:0] = ["tests", "oracle"]
import test_gpu_ipc as T
json.dump(T.cases_for($P), open("$OUT/cases.json", "w"))
PY
UID_HEX=$(python -c "import os; print(os.urandom(128).hex())")
pids=()
for ((r=0; r<P; r++)); do
  MPJX_IPC_DEBUG=1 MPJX_IPC_TIMEOUT_S=30 timeout -k 5 120 python -u tests/ipc_worker.py $r $P $UID_HEX $OUT/cases.json $OUT > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "workers rc=$rc"
python tools/ipc_check.py $P $OUT > $OUT/check.txt 2>&1; grep -v " ok" $OUT/check.txt | head -40
rm -f $OUT/*.npy
exit $rc
