set -e
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_distributed.py tests/test_gpu_join_sort_window.py > gpurun_out/r3d/tests.log 2>&1
timeout -k 10 300 python tools/prof_dist_group.py 60000000 > gpurun_out/r3d/p60m.json 2>/dev/null
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err
