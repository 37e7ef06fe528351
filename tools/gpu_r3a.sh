# Round-3 check: new GPU tests, bench with the config-4/5 legs (1 GPU), a
# world-2 gloo rehearsal of the bench on the one GPU.
set -e
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group_sorted.py tests/test_gpu_distributed.py tests/test_c_abi.py tests/test_gpu_ops.py tests/test_gpu_join_sort_window.py > gpurun_out/r3a/tests.log 2>&1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --sf 10 --window-rows 200000000 --no-cpu > gpurun_out/r3a/bench_n2_gloo.json 2> gpurun_out/r3a/bench_n2_gloo.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bounds.py tests/test_gpu_join_sort_window.py -k "window or bounds or range" > gpurun_out/r3a/window_tests.log 2>&1
timeout -k 10 300 python tools/opbench.py --only config5 > gpurun_out/r3a/opbench_config5.json 2>&1
