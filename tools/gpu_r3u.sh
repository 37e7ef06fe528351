set -e
mkdir -p gpurun_out/r3u
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group_sorted.py tests/test_gpu_group_str.py tests/test_gpu_threads.py tests/test_gpu_distributed.py tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_aggr_sorted.py tests/test_gpu_join_sort_window.py > gpurun_out/r3u/tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --sf 10 --window-rows 200000000 --no-cpu > gpurun_out/r3u/bench_n2_gloo.json 2> gpurun_out/r3u/bench_n2_gloo.err
