#!/bin/bash
# Host-side AddressSanitizer build of libmpjx and the C++ known-answer harness (tests/cpp/ccl_tests.cpp),
# for the host code that the GPU parity tests cannot see: the multicore rendezvous (SmpWorld), the
# IPC shared-memory world and staging windows, the host pipelines, argument checks. Device code is
# compiled exactly as in the product (no GPU ASan, no xnack): every -fsanitize= sits behind
# -Xarch_host. Output in tools/asan/ (git-ignored).
#   build here:   tools/asan_check.sh build
#   run (GPU box): tools/asan_check.sh run      -> multicore P=8 and IPC P=4 KATs under ASan
#   jni (here, CPU): tools/asan_check.sh jni    -> the JNI shim + tests/jni/fakejvm.c under ASan + UBSan,
#                  driven through tests/jni_driver.py's CPU scenarios (bounds, exceptions, no pinning)
export MPJX_IPC_OVERSUBSCRIBE=${MPJX_IPC_OVERSUBSCRIBE:-1}  # rank processes share one GPU
set -euo pipefail
cd "$(dirname "$0")/.."
# SANITIZER=thread builds a ThreadSanitizer variant instead (tools/tsan/), for the multicore rendezvous
KIND=${SANITIZER:-address}
OUT=tools/asan
[ "$KIND" = thread ] && OUT=tools/tsan
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=$KIND -Xarch_host -fno-omit-frame-pointer"
case "${1:-build}" in
jni)
  mkdir -p "$OUT"
  gcc -std=gnu11 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -shared -Wall -Wextra -Werror \
    -Itests/jni -Iinclude integration/jni/mpi_HipIntracomm.c tests/jni/fakejvm.c -o "$OUT/libmpjx_jni_fake.so" \
    -Lmpjexpress_amd/lib -lmpjx -lpthread -Wl,-rpath,"$PWD/mpjexpress_amd/lib"
  ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=halt_on_error=1 \
    LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
    MPJX_JNI_DRIVER_SO="$OUT/libmpjx_jni_fake.so" python tests/jni_driver.py cpu
  ;;
build)
  mkdir -p "$OUT"
  pids=()
  for f in mpjexpress_amd/csrc/*.hip; do
    "$HIPCC" -O2 -Xarch_host -gline-tables-only -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude $SAN -c "$f" -o "$OUT/$(basename "$f" .hip).o" &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p"; done
  # the .so leaves the ASan runtime to the executable (no --no-undefined here)
  "$HIPCC" --offload-arch=gfx950 -shared -o "$OUT/libmpjx.so" "$OUT"/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  "$HIPCC" -O1 -Xarch_host -gline-tables-only -std=c++17 --offload-arch=gfx950 -Iinclude $SAN tests/cpp/ccl_tests.cpp -o "$OUT/ccl_tests" \
    -L"$OUT" -lmpjx -Wl,-rpath,'$ORIGIN'
  echo "built $OUT/ccl_tests"
  ;;
run)
  # ROCm's ASan runtime trips its own CHECK (sanitizer_allocator_device.h, "dev_runtime_unloaded_")
  # when libhsa-runtime frees memory from __cxa_finalize at process exit, after the tests are done;
  # so the verdict is read from the output: every KAT passed and no AddressSanitizer ERROR report.
  export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1
  # exitcode=0: a report does not fail the KAT run by itself; reports are counted from the output
  export TSAN_OPTIONS=halt_on_error=0:report_signal_unsafe=0:exitcode=0:report_thread_leaks=0:suppressions=$PWD/tools/tsan.supp
  LOG=${GRAFT_REPO_ROOT:-.}/gpurun_out/$KIND
  mkdir -p "$LOG"
  timeout -k 10 300 stdbuf -oL -eL "$OUT/ccl_tests" 8 > "$LOG/asan_multicore.log" 2>&1 || true
  MPJX_IPC_TIMEOUT_S=120 timeout -k 10 300 stdbuf -oL -eL "$OUT/ccl_tests" ipc 4 > "$LOG/asan_ipc.log" 2>&1 || true
  ok=0
  for f in "$LOG/asan_multicore.log" "$LOG/asan_ipc.log"; do
    if grep -q "ALL CCL TESTS PASSED" "$f" && ! grep -q "ERROR: AddressSanitizer\|WARNING: ThreadSanitizer" "$f"; then
      echo "$(basename "$f"): all KATs passed, no $KIND sanitizer report"
    else
      echo "$(basename "$f"): FAILED"; grep -m5 "ERROR: AddressSanitizer\|FAIL\|bad" "$f" || true; ok=1
    fi
  done
  exit $ok
  ;;
esac
