# join: partitions of 16 Ki build rows (144 KiB LDS tables) vs 8 Ki, old path
set -e
export TMPDIR=/tmp
O=gpurun_out/j5
mkdir -p $O
MGDK_JOIN_RP=0 MGDK_PJ_ROWS=16384 timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_join_sort_window.py -k "join" > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
MGDK_JOIN_RP=0 timeout -k 10 300 python tools/opbench.py --only config3 > $O/join_p2048.json 2>&1
MGDK_JOIN_RP=0 MGDK_PJ_ROWS=16384 timeout -k 10 300 python tools/opbench.py --only config3 > $O/join_p1024.json 2>&1
MGDK_JOIN_RP=0 MGDK_PJ_ROWS=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/opbench.py --only config3 > $O/prof.log 2>&1
