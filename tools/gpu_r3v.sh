set -e
mkdir -p gpurun_out/r3v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_join_algo.py tests/test_gpu_join_sort_window.py tests/test_gpu_group_sorted.py tests/test_gpu_props.py tests/test_gpu_distributed.py tests/test_gpu_sort_qsort.py tests/test_gpu_ops.py tests/test_gpu_group_str.py > gpurun_out/r3v/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3v/prof -o run -- python3 tools/opbench.py --only config3 other_ops > gpurun_out/r3v/opbench.json 2> gpurun_out/r3v/opbench.err
