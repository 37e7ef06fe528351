set -e
mkdir -p gpurun_out/r3aa
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for u in 16 8 32; do
  MGDK_GS_DIRECT_U=$u timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3aa/u$u -o run -- python3 tools/run_gsorted.py > gpurun_out/r3aa/u$u.log 2>&1
done
MGDK_GS_DIRECT_U=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py > gpurun_out/r3aa/tests_u8.log 2>&1
MGDK_GS_DIRECT_U=32 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_aggr_sorted.py > gpurun_out/r3aa/tests_u32.log 2>&1
