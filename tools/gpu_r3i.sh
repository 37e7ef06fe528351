set -e
mkdir -p gpurun_out/r3i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_analytic.py tests/test_gpu_join_sort_window.py > gpurun_out/r3i/tests.log 2>&1
for v in base noxcd fr16 fr4; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i/$v -o run -- python3 tools/run_window.py 1000000000 3 > gpurun_out/r3i/$v.log 2>&1
done
