#!/bin/bash
# Debug helper: BASELINE-size collectives through the IPC engine, P ranks on one GPU (no output check).
P=${1:-2}
OUT=gpurun_out/ipc_big
mkdir -p $OUT
cat > $OUT/cases.json <<JSON
[{"id": "ar_f64_256m", "kind": "allreduce", "op": 3, "type": 8, "n": 33554432, "seed": 1, "nosave": true},
 {"id": "rs_band_64m", "kind": "reduce_scatter", "op": 6, "type": 5, "recvcounts": [$(python -c "print(','.join(['%d' % ((16<<20)//$P)]*$P))")], "seed": 2, "nosave": true},
 {"id": "scan_bxor_64m", "kind": "scan", "op": 10, "type": 5, "n": 16777216, "seed": 3, "nosave": true},
 {"id": "ar_max_f32_1g", "kind": "allreduce", "op": 1, "type": 7, "n": 268435456, "seed": 4, "nosave": true}]
JSON
UID_HEX=$(python -c "import os; print(os.urandom(128).hex())")
pids=()
for ((r=0; r<P; r++)); do
  MPJX_IPC_DEBUG=1 MPJX_IPC_TIMEOUT_S=60 timeout -k 5 150 python -u tests/ipc_worker.py $r $P $UID_HEX $OUT/cases.json $OUT > $OUT/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "workers rc=$rc"
exit $rc
