set -e
mkdir -p gpurun_out/r3z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_distributed.py tests/test_gpu_exchange_ops.py > gpurun_out/r3z/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z/prof -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r3z/bench.json 2> gpurun_out/r3z/bench.err
