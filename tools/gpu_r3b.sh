# aggregates finished on the device: parity tests + dist group profile
set -e
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_analytic.py tests/test_gpu_distributed.py tests/test_gpu_exchange_ops.py tests/test_gpu_group_str.py tests/test_gpu_group_sorted.py > gpurun_out/r3b/tests.log 2>&1
timeout -k 10 200 python tools/prof_dist_group.py 6000000 > gpurun_out/r3b/p6m.json 2>&1
timeout -k 10 300 python tools/prof_dist_group.py 60000000 > gpurun_out/r3b/p60m.json 2>&1
