set -e
mkdir -p gpurun_out/r3m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py tests/test_gpu_group_sorted.py tests/test_gpu_ops.py tests/test_gpu_distributed.py tests/test_gpu_props.py > gpurun_out/r3m/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m/t -o run -- python3 tools/run_gsorted.py > gpurun_out/r3m/t.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3m/w -o run -- python3 tools/run_gsorted.py 600000000 1 > gpurun_out/r3m/w.log 2>&1
