# fused ordered group sums (LDS-staged loads): parity + kernel times at SF100
set -e
export TMPDIR=/tmp
O=gpurun_out/gs2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_sums.py > $O/tests.log 2>&1 || { echo "TESTS FAILED" >> $O/tests.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/prof_dist_group.py 600121500 > $O/prof.log 2>&1
