set -e
mkdir -p gpurun_out/r3x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py tests/test_gpu_firstn.py tests/test_gpu_ops.py tests/test_gpu_distributed.py tests/test_gpu_group_sorted.py"
MGDK_SORT_MSD_MIN=2000 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/r3x/tests_msd_small.log 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/r3x/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3x/prof -o run -- python3 tools/opbench.py --only other_ops > gpurun_out/r3x/opbench.json 2> gpurun_out/r3x/opbench.err
