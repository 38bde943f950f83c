#!/bin/bash
# The JNI shim's RCCL scenario (tests/jni_driver.py rccl: P = 3 rank threads, fake JVM in copy mode, the
# RCCL stand-in) up to six times in one GPU call, stopping at the first failure; each run under its own
# limit and the driver's watchdog (tests/watchdog.py: blocking syscalls, native and Python stacks of every
# thread, then exit 3). Used to find the round-6 hang (profiles/r06/jni_rccl_hang_stacks_diag1.txt) and to
# check its fix (profiles/r06/jni_rccl_diag_q.txt). Outputs: gpurun_out/jni_rccl_diag_<i>.{out,err}.
set -o pipefail
export MPJX_JNI_DRIVER_SO=tests/jni/libmpjx_jni_fake_standin.so RSI_TIMEOUT_S=30 MPJX_RCCL_TIMEOUT_S=30 MPJX_JNI_DRIVER_WATCHDOG_S=45 MPJX_JNI_DRIVER_VERBOSE=1
mkdir -p gpurun_out
for i in 1 2 3 4 5 6; do
  echo "== run $i $(date +%T)"
  timeout -k 10 80 python -u tests/jni_driver.py rccl > gpurun_out/jni_rccl_diag_$i.out 2> gpurun_out/jni_rccl_diag_$i.err
  rc=$?
  echo "   rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
