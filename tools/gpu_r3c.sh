set -e
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_distributed.py > gpurun_out/r3c/tests.log 2>&1
timeout -k 10 300 python tools/prof_dist_group.py 60000000 > gpurun_out/r3c/p60m.json 2>&1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err
