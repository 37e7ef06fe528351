# targeted GPU tests, then the probe-pass shape probe
set -e
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_msk_cands.py tests/test_join_algo.py tests/test_gpu_group_sorted.py tests/test_gpu_sort_qsort.py > gpurun_out/quick/tests.log 2>&1
timeout -k 10 120 tools/probes/l2probe > gpurun_out/quick/l2probe.log 2>&1
timeout -k 10 120 tools/probes/l2probe 36608 >> gpurun_out/quick/l2probe.log 2>&1
