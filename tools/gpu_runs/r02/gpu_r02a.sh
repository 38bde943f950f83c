# round-2 GPU step: IPC tests (incl. the shared-GPU guard and the platform-envelope probe), configs[0]
# parity, then the N=1 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_cpp.py "tests/test_gpu_collectives.py::test_config0_allreduce_sum_double_1mib_p4" -x -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_ipc_r02.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_ipc_r02.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_n1_r02a.json 2> gpurun_out/bench_n1_r02a.err; rc=$?
tail -c 1500 gpurun_out/bench_n1_r02a.json; exit $rc
