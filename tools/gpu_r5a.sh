set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_elim_route.py tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py > gpurun_out/r5a/pytest_elim.log 2>&1
echo "exit $?"
tail -5 gpurun_out/r5a/pytest_elim.log
