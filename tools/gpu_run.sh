#!/bin/bash
# One GPU-box pass, steps chosen on the command line (replaces round 3's 56 one-off scripts):
#   tools/gpu_run.sh TAG STEP [STEP ...]
# Outputs go to gpurun_out/TAG_<step>.*; each GPU step runs under its own time limit and the chain
# stops at the first failure (no GPU step runs after a fault, an abort or a time limit).
# Steps:
#   pytest        the whole -m gpu suite              pytest_k:EXPR   the -m gpu tests matching EXPR
#   smoke         __graft_entry__.smoke()             bench           python bench.py (N = 1 line)
#   rocprof       rocprofv3 --kernel-trace --stats of the N = 1 bench
#   pmc_bench     rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, of the N = 1 bench (one counter per pass)
#   ar1           N > 1 bench flow at world size 1 (torchrun, --allreduce: preflights, every engine)
#   ar1_fail      the same with MPJX_PREFLIGHT_FAIL=rccl (the RCCL engines skipped, IPC still measured)
#   od4           N > 1 bench flow, 4 rank processes on one GPU (--one-device: IPC engines)
#   launch1       `python bench.py --launch --allreduce`: bench.py starts its own torchrun child (world 1)
#   launch1_budget  the same with --budget-s 30: optional phases skipped, the line still printed
#   od4_launch    `python bench.py --gpus 4 --one-device` WITHOUT a launcher: the self-launched 4 ranks
#   od8_launch    the same with 8 rank processes on the one GPU
#   launch1_budget5 / launch1_hard  world-1 self-launch with --budget-s 5 (optional phases skipped) /
#                 --hard-s 30 with the e2e_host phase stalled (MPJX_BENCH_STALL_PHASE): the line so far, cut_short
#   jni_latency   configs[0] (1 MiB, P = 4 rank threads) through the JNI shim + stand-in JNIEnv, per call
#   host_once_ab / host_once_prof  the same with MPJX_HOST_ONCE=1/0 alternated / their kernel stats
#   census        tools/queue_census.py: hardware queues of the P = 8 one-GPU IPC worlds vs what the GPU maps
#   load_cost     tools/load_cost: dlopen / runtime init / comm init / first and later calls (no torch)
#   load_cost_ab  the same, 3 x alternating the shipped library and mpjexpress_amd/lib_cz (compressed fatbin)
#   shapes        tools/tuning/config_shapes.py (configs[3]/[4] combine shapes, RCCL layout)
#   shapes_warm   the same with the input slots rewritten before every combine (MODE=after_write)
#   shapes_sizes  RS BAND int32 K_MST P=8 over slice sizes 4 KiB .. 64 MiB (MODE=sizes)
#   pmc_shapes    FETCH_SIZE / WRITE_SIZE passes of config_shapes.py; shapes_prof  its rocprofv3 kernel trace
#   tune_short    tools/tuning/tune_short (short-launch structures at the configs[3] shapes)
#   tune_short_skew  the same with 4 KiB-skewed input slots; tune_short_prof  under rocprofv3 --kernel-trace
#   tune_streams  read-only vs read+write HBM streams, 1-8 operand streams (tools/tuning/tune_streams.hip)
#   tune_stores   read-8-write-1 with the store's cache policy (nt / plain / sc1 / sc0 sc1 / buffer nt / sc1 nt), 8-32 MiB slices
#   pcie          host link: DMA / kernel / mixed copies one way and both ways, host staging threads
#                 (tools/tuning/pcie_probe.hip); e2e  tools/e2e_bench.py (the host path's rates)
# (tuning harnesses are built on the box into /tmp/mpjx_tune: their binaries do not travel)
#   latency_fuse  the IPC fused forms' size limit: MPJX_IPC_FUSE_KIB = 512 (default) / 2048 / 0, 8 B .. 2 MiB
#   latency       tools/latency multicore sweep (LATENCY_ARGS, default P = 4)
#   latency_ipc   tools/latency over 4 IPC rank processes, device sync: round 3's launches (MPJX_IPC_FUSED=share),
#                 the fence flags fused into the copy-out (=fence), the default (+ the flag stored from the
#                 combine kernel's tail), then host sync
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:?usage: gpu_run.sh TAG STEP...}
shift
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run() {  # run NAME SECONDS CMD... : one step, its own limit; a nonzero status ends the chain
  local name=$1 lim=$2
  shift 2
  echo "== $TAG $name ($(date +%T))"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "   $name rc=$rc"
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
tbuild() {  # tbuild NAME [extra sources]: build a tuning harness on the box (binaries do not travel)
  local n=$1
  shift
  mkdir -p /tmp/mpjx_tune
  run "build_$n" 300 hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude "tools/tuning/$n.hip" "$@" -o "/tmp/mpjx_tune/$n" -lpthread
}
T=/tmp/mpjx_tune
for step in "$@"; do
  case $step in
    pytest) run pytest 1000 bash -c "python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread --durations=25 > '$OUT/${TAG}_pytest.log' 2>&1"
            tail -2 "$OUT/${TAG}_pytest.log" ;;
    pytest_k:*) run pytest_k 600 bash -c "python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread --durations=25 -k '${step#pytest_k:}' > '$OUT/${TAG}_pytest_k.log' 2>&1"
            tail -2 "$OUT/${TAG}_pytest_k.log" ;;
    smoke) run smoke 300 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > '$OUT/${TAG}_smoke.log' 2>&1"
           tail -1 "$OUT/${TAG}_smoke.log" ;;
    bench) run bench 400 bash -c "python bench.py > '$OUT/${TAG}_bench_n1.json' 2> '$OUT/${TAG}_bench_n1.err'"
           head -c 600 "$OUT/${TAG}_bench_n1.json"; echo ;;
    rocprof) run rocprof 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_prof' -o bench -- python3 '$R/bench.py' --no-cpu-baseline --steps 20 > '$OUT/${TAG}_rocprof.log' 2>&1" ;;
    pmc_bench)
      run pmc_fetch 300 bash -c "cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d '$OUT/${TAG}_pmcb_fetch' -o bench -- python3 '$R/bench.py' --no-cpu-baseline --steps 5 --warmup 1 > '$OUT/${TAG}_pmcb_fetch.log' 2>&1"
      run pmc_write 300 bash -c "cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d '$OUT/${TAG}_pmcb_write' -o bench -- python3 '$R/bench.py' --no-cpu-baseline --steps 5 --warmup 1 > '$OUT/${TAG}_pmcb_write.log' 2>&1" ;;
    ar1) run ar1 500 bash -c "$TR --nproc-per-node 1 --master-port 29612 bench.py --allreduce --steps 10 --warmup 3 > '$OUT/${TAG}_bench_ar1.json' 2> '$OUT/${TAG}_bench_ar1.err'"
         head -c 400 "$OUT/${TAG}_bench_ar1.json"; echo ;;
    ar1_fail) run ar1_fail 500 bash -c "MPJX_PREFLIGHT_FAIL=rccl $TR --nproc-per-node 1 --master-port 29613 bench.py --allreduce --steps 5 --warmup 2 > '$OUT/${TAG}_bench_ar1_fail.json' 2> '$OUT/${TAG}_bench_ar1_fail.err'"
         head -c 400 "$OUT/${TAG}_bench_ar1_fail.json"; echo ;;
    od4) run od4 600 bash -c "$TR --nproc-per-node 4 --master-port 29614 bench.py --gpus 4 --one-device --steps 5 --warmup 2 > '$OUT/${TAG}_bench_od4.json' 2> '$OUT/${TAG}_bench_od4.err'"
         head -c 400 "$OUT/${TAG}_bench_od4.json"; echo ;;
    launch1) run launch1 500 bash -c "python bench.py --launch --allreduce --steps 10 --warmup 3 > '$OUT/${TAG}_bench_launch1.json' 2> '$OUT/${TAG}_bench_launch1.err'"
         head -c 400 "$OUT/${TAG}_bench_launch1.json"; echo ;;
    launch1_budget) run launch1_budget 400 bash -c "python bench.py --launch --allreduce --steps 5 --warmup 2 --budget-s 30 > '$OUT/${TAG}_bench_launch1_budget.json' 2> '$OUT/${TAG}_bench_launch1_budget.err'"
         head -c 400 "$OUT/${TAG}_bench_launch1_budget.json"; echo ;;
    launch1_budget5) run launch1_budget5 400 bash -c "python bench.py --launch --allreduce --steps 5 --warmup 2 --budget-s 5 > '$OUT/${TAG}_bench_launch1_budget5.json' 2> '$OUT/${TAG}_bench_launch1_budget5.err'"
         head -c 400 "$OUT/${TAG}_bench_launch1_budget5.json"; echo ;;
    launch1_hard) run launch1_hard 400 bash -c "MPJX_BENCH_STALL_PHASE=e2e_host python bench.py --launch --allreduce --steps 5 --warmup 2 --no-preflight --hard-s 30 > '$OUT/${TAG}_bench_launch1_hard.json' 2> '$OUT/${TAG}_bench_launch1_hard.err'"
         head -c 400 "$OUT/${TAG}_bench_launch1_hard.json"; echo ;;
    od8_launch) run od8_launch 600 bash -c "python bench.py --gpus 8 --one-device --steps 5 --warmup 2 > '$OUT/${TAG}_bench_od8_launch.json' 2> '$OUT/${TAG}_bench_od8_launch.err'"
         head -c 400 "$OUT/${TAG}_bench_od8_launch.json"; echo ;;
    od4_launch) run od4_launch 600 bash -c "python bench.py --gpus 4 --one-device --steps 5 --warmup 2 > '$OUT/${TAG}_bench_od4_launch.json' 2> '$OUT/${TAG}_bench_od4_launch.err'"
         head -c 400 "$OUT/${TAG}_bench_od4_launch.json"; echo ;;
    jni_latency) run jni_latency 200 bash -c "python tests/jni_driver.py latency > '$OUT/${TAG}_jni_latency.json' 2> '$OUT/${TAG}_jni_latency.err'"
         cat "$OUT/${TAG}_jni_latency.json" ;;
    jni_latency_ab)  # the host-direct form on / off (MPJX_HOST_DIRECT), alternated
      for i in 1 2; do
        run jni_latency_on$i 200 bash -c "python tests/jni_driver.py latency >> '$OUT/${TAG}_jni_latency_ab.jsonl' 2>> '$OUT/${TAG}_jni_latency_ab.err'"
        run jni_latency_off$i 200 bash -c "MPJX_HOST_DIRECT=0 python tests/jni_driver.py latency >> '$OUT/${TAG}_jni_latency_ab.jsonl' 2>> '$OUT/${TAG}_jni_latency_ab.err'"
      done
      cat "$OUT/${TAG}_jni_latency_ab.jsonl" ;;
    jni_latency_prof)  # kernel stats of the host-direct form alone (page-locked callers), then of the staged form
      run jni_prof_direct 200 bash -c "cd /tmp && MPJX_JNI_LATENCY_ONLY=pinned MPJX_JNI_LATENCY_CALLS=200 rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_jni_prof_direct' -o jni -- python3 '$R/tests/jni_driver.py' latency > '$OUT/${TAG}_jni_prof_direct.log' 2>&1" &&
      run jni_prof_staged 200 bash -c "cd /tmp && MPJX_HOST_DIRECT=0 MPJX_JNI_LATENCY_ONLY=pinned MPJX_JNI_LATENCY_CALLS=200 rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_jni_prof_staged' -o jni -- python3 '$R/tests/jni_driver.py' latency > '$OUT/${TAG}_jni_prof_staged.log' 2>&1" ;;
    census_forced) run census_forced 900 bash -c "python tools/queue_census.py '$OUT/${TAG}_census_forced.json' forced > '$OUT/${TAG}_census_forced.log' 2>&1"
            tail -9 "$OUT/${TAG}_census_forced.log" ;;
    census) run census 600 bash -c "python tools/queue_census.py '$OUT/${TAG}_census.json' > '$OUT/${TAG}_census.log' 2>&1"
            tail -3 "$OUT/${TAG}_census.log" ;;
    host_once_ab)  # host-direct Allreduce result across the link once (MPJX_HOST_ONCE=1) or to every rank (0), alternated
      for i in 1 2 3; do
        run once_on$i 200 bash -c "MPJX_HOST_ONCE=1 python tests/jni_driver.py latency >> '$OUT/${TAG}_host_once_ab.jsonl' 2>> '$OUT/${TAG}_host_once_ab.err'"
        run once_off$i 200 bash -c "MPJX_HOST_ONCE=0 python tests/jni_driver.py latency >> '$OUT/${TAG}_host_once_ab.jsonl' 2>> '$OUT/${TAG}_host_once_ab.err'"
      done
      cat "$OUT/${TAG}_host_once_ab.jsonl" ;;
    host_once_prof)  # kernel stats of the host-direct Allreduce (page-locked callers), result once vs to every rank
      run once_prof_on 200 bash -c "cd /tmp && MPJX_HOST_ONCE=1 MPJX_JNI_LATENCY_ONLY=pinned MPJX_JNI_LATENCY_CALLS=200 rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_once_prof_on' -o jni -- python3 '$R/tests/jni_driver.py' latency > '$OUT/${TAG}_once_prof_on.log' 2>&1" &&
      run once_prof_off 200 bash -c "cd /tmp && MPJX_HOST_ONCE=0 MPJX_JNI_LATENCY_ONLY=pinned MPJX_JNI_LATENCY_CALLS=200 rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_once_prof_off' -o jni -- python3 '$R/tests/jni_driver.py' latency > '$OUT/${TAG}_once_prof_off.log' 2>&1" ;;
    probe_host) run build_probe_host 200 hipcc --offload-arch=gfx950 -O2 tools/probe_host_range.cpp -o /tmp/probe_host_range
                run probe_host 60 bash -c "/tmp/probe_host_range > '$OUT/${TAG}_probe_host.jsonl' 2>&1"
                cat "$OUT/${TAG}_probe_host.jsonl" ;;
    load_cost) run load_cost 120 bash -c "tools/load_cost > '$OUT/${TAG}_load_cost.json' 2> '$OUT/${TAG}_load_cost.err'"
         cat "$OUT/${TAG}_load_cost.json" ;;
    load_cost_ab)  # the shipped library and a compressed-fatbin build of it (mpjexpress_amd/lib_cz), alternated
      for i in 1 2 3; do
        run load_cost_a$i 120 bash -c "tools/load_cost >> '$OUT/${TAG}_load_cost_ab.jsonl' 2>> '$OUT/${TAG}_load_cost_ab.err'"
        run load_cost_cz$i 120 bash -c "tools/load_cost mpjexpress_amd/lib_cz/libmpjx.so >> '$OUT/${TAG}_load_cost_ab.jsonl' 2>> '$OUT/${TAG}_load_cost_ab.err'"
      done
      cat "$OUT/${TAG}_load_cost_ab.jsonl" ;;
    shapes) run shapes 300 bash -c "python tools/tuning/config_shapes.py > '$OUT/${TAG}_shapes.jsonl' 2>&1"
            cat "$OUT/${TAG}_shapes.jsonl" ;;
    shapes_warm) run shapes_warm 300 bash -c "MODE=after_write python tools/tuning/config_shapes.py > '$OUT/${TAG}_shapes_warm.jsonl' 2>&1"
            cat "$OUT/${TAG}_shapes_warm.jsonl" ;;
    shapes_sizes) run shapes_sizes 300 bash -c "MODE=sizes python tools/tuning/config_shapes.py > '$OUT/${TAG}_shapes_sizes.jsonl' 2>&1"
            cat "$OUT/${TAG}_shapes_sizes.jsonl" ;;
    shapes_prof) run shapes_prof 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_prof_shapes' -o shapes -- python3 '$R/tools/tuning/config_shapes.py' > '$OUT/${TAG}_prof_shapes.log' 2>&1" ;;
    pmc_shapes)
      run pmc_shapes_fetch 300 bash -c "cd /tmp && ITERS=5 rocprofv3 --pmc FETCH_SIZE --output-format csv -d '$OUT/${TAG}_pmcs_fetch' -o shapes -- python3 '$R/tools/tuning/config_shapes.py' > '$OUT/${TAG}_pmcs_fetch.log' 2>&1"
      run pmc_shapes_write 300 bash -c "cd /tmp && ITERS=5 rocprofv3 --pmc WRITE_SIZE --output-format csv -d '$OUT/${TAG}_pmcs_write' -o shapes -- python3 '$R/tools/tuning/config_shapes.py' > '$OUT/${TAG}_pmcs_write.log' 2>&1" ;;
    tune_short) tbuild tune_short mpjexpress_amd/csrc/mpjx_k_util.hip
            run tune_short 300 bash -c "$T/tune_short ${TUNE_ROUNDS:-7} > '$OUT/${TAG}_tune_short.jsonl' 2>&1"
                cat "$OUT/${TAG}_tune_short.jsonl" ;;
    tune_short_skew) [ -x $T/tune_short ] || tbuild tune_short mpjexpress_amd/csrc/mpjx_k_util.hip
            run tune_short_skew 300 bash -c "SKEW=4096 $T/tune_short ${TUNE_ROUNDS:-7} > '$OUT/${TAG}_tune_short_skew4k.jsonl' 2>&1" ;;
    tune_short_prof) [ -x $T/tune_short ] || tbuild tune_short mpjexpress_amd/csrc/mpjx_k_util.hip
            run tune_short_prof 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/${TAG}_prof_short' -o short -- $T/tune_short 3 > '$OUT/${TAG}_prof_short.log' 2>&1" ;;
    tune_streams) tbuild tune_streams
                  run tune_streams 200 bash -c "$T/tune_streams 7 > '$OUT/${TAG}_tune_streams.jsonl' 2>&1"
                  cat "$OUT/${TAG}_tune_streams.jsonl" ;;
    tune_stores) tbuild tune_streams
                 run tune_stores 300 bash -c "$T/tune_streams 7 20 stores > '$OUT/${TAG}_tune_stores.jsonl' 2>&1"
                 cat "$OUT/${TAG}_tune_stores.jsonl" ;;
    pcie) tbuild pcie_probe
          run pcie 300 bash -c "$T/pcie_probe 5 > '$OUT/${TAG}_pcie.jsonl' 2>&1"
          cat "$OUT/${TAG}_pcie.jsonl" ;;
    e2e_trace)  # memory-copy + kernel trace of the host pipeline, pinned then pageable callers
      run e2e_trace_pinned 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d '$OUT/${TAG}_e2e_trace_pinned' -o e2e -- python3 '$R/tools/e2e_bench.py' --only pinned --iters 3 > '$OUT/${TAG}_e2e_trace_pinned.log' 2>&1"
      run e2e_trace_pageable 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d '$OUT/${TAG}_e2e_trace_pageable' -o e2e -- python3 '$R/tools/e2e_bench.py' --only pageable --iters 3 > '$OUT/${TAG}_e2e_trace_pageable.log' 2>&1" ;;
    e2e) run e2e 300 bash -c "python tools/e2e_bench.py > '$OUT/${TAG}_e2e.json' 2>&1"
         cat "$OUT/${TAG}_e2e.json" ;;
    latency) run latency 300 bash -c "tools/latency ${LATENCY_ARGS:-} > '$OUT/${TAG}_latency.json' 2>&1"
             tail -c 600 "$OUT/${TAG}_latency.json" ;;
    latency_ipc)
      run latency_ipc_r3 300 bash -c "MPJX_IPC_SYNC=device-shared MPJX_IPC_FUSED=share tools/latency ipc 4 16 > '$OUT/${TAG}_latency_ipc_dsync_r3.json' 2>&1"
      run latency_ipc_fence 300 bash -c "MPJX_IPC_SYNC=device-shared MPJX_IPC_FUSED=fence tools/latency ipc 4 16 > '$OUT/${TAG}_latency_ipc_dsync_fence.json' 2>&1"
      run latency_ipc_new 300 bash -c "MPJX_IPC_SYNC=device-shared tools/latency ipc 4 16 > '$OUT/${TAG}_latency_ipc_dsync.json' 2>&1"
      run latency_ipc_host 300 bash -c "MPJX_IPC_SYNC=host tools/latency ipc 4 16 > '$OUT/${TAG}_latency_ipc_host.json' 2>&1"
      tail -c 400 "$OUT/${TAG}_latency_ipc_dsync.json" ;;
    latency_fuse)  # the fused forms' size limit (MPJX_IPC_FUSE_KIB): default 512 KiB vs 2 MiB vs never, device sync
      run latency_fuse_512 300 bash -c "MPJX_IPC_SYNC=device-shared tools/latency ipc 4 2 > '$OUT/${TAG}_latency_fuse512.json' 2>&1"
      run latency_fuse_2048 300 bash -c "MPJX_IPC_SYNC=device-shared MPJX_IPC_FUSE_KIB=2048 tools/latency ipc 4 2 > '$OUT/${TAG}_latency_fuse2048.json' 2>&1"
      run latency_fuse_0 300 bash -c "MPJX_IPC_SYNC=device-shared MPJX_IPC_FUSE_KIB=0 tools/latency ipc 4 2 > '$OUT/${TAG}_latency_fuse0.json' 2>&1"
      tail -c 500 "$OUT/${TAG}_latency_fuse2048.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $TAG done"
