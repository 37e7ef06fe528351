set -e
mkdir -p gpurun_out/r3k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bounds.py tests/test_gpu_join_sort_window.py tests/test_gpu_analytic.py > gpurun_out/r3k/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k/new -o run -- python3 tools/run_window.py 1000000000 3 > gpurun_out/r3k/new.log 2>&1
