set -e
mkdir -p gpurun_out/r3f
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bounds.py tests/test_gpu_join_sort_window.py tests/test_gpu_analytic.py tests/test_gpu_distributed.py > gpurun_out/r3f/tests.log 2>&1
timeout -k 10 300 python tools/opbench.py --only config5 > gpurun_out/r3f/opbench_config5.json 2>/dev/null
MGDK_WIN_LEAN=0 timeout -k 10 300 python tools/opbench.py --only config5 > gpurun_out/r3f/opbench_config5_old.json 2>/dev/null
