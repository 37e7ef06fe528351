set -e
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bounds.py tests/test_gpu_join_sort_window.py tests/test_gpu_analytic.py tests/test_gpu_aggr_sorted.py > gpurun_out/r3e/tests.log 2>&1
timeout -k 10 300 python tools/opbench.py --only config5 > gpurun_out/r3e/opbench_config5.json 2>/dev/null
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3e/bench.json 2> gpurun_out/r3e/bench.err
