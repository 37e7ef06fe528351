set -e
mkdir -p gpurun_out/r3p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_distributed.py tests/test_gpu_exchange_ops.py > gpurun_out/r3p/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p/t -o run -- python3 tools/run_gsorted.py > gpurun_out/r3p/t.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p/prof -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r3p/bench.json 2> gpurun_out/r3p/bench.err
