set -e
mkdir -p gpurun_out/r3n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py tests/test_gpu_ops.py tests/test_gpu_props.py > gpurun_out/r3n/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n/t -o run -- python3 tools/run_gsorted.py > gpurun_out/r3n/t.log 2>&1
MGDK_GS_STAGE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n/t0 -o run -- python3 tools/run_gsorted.py > gpurun_out/r3n/t0.log 2>&1
