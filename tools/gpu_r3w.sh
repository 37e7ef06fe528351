set -e
mkdir -p gpurun_out/r3w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py tests/test_gpu_firstn.py tests/test_gpu_ops.py > gpurun_out/r3w/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w/prof -o run -- python3 tools/opbench.py --only other_ops > gpurun_out/r3w/opbench.json 2> gpurun_out/r3w/opbench.err
