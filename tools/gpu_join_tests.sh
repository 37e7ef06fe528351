set -e
mkdir -p gpurun_out/j1
timeout -k 10 400 python -u -m pytest tests/test_join_algo.py tests/test_gpu_join_sort_window.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j1/tests.log 2>&1
