set -e
mkdir -p gpurun_out/r3y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_join_algo.py tests/test_gpu_join_sort_window.py tests/test_gpu_distributed.py tests/test_gpu_props.py > gpurun_out/r3y/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3y/t -o run -- python3 tools/run_join.py 3 > gpurun_out/r3y/t.log 2>&1
MGDK_PJ_STAGE16=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3y/t0 -o run -- python3 tools/run_join.py 3 > gpurun_out/r3y/t0.log 2>&1
