# join work: parity tests, shape probe, SF10 join old vs new path, rocprof of the new path
set -e
export TMPDIR=/tmp
O=gpurun_out/j4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_msk_cands.py tests/test_join_algo.py tests/test_gpu_join_sort_window.py -k "join or msk or ordered" > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 120 tools/probes/l2probe > $O/l2probe.log 2>&1
timeout -k 10 120 tools/probes/l2probe 36608 >> $O/l2probe.log 2>&1
MGDK_JOIN_RP=0 timeout -k 10 300 python tools/opbench.py --only config3 > $O/join_old.json 2>&1
timeout -k 10 300 python tools/opbench.py --only config3 > $O/join_rp.json 2>&1
MGDK_JOIN_RP_CBITS=8 timeout -k 10 300 python tools/opbench.py --only config3 > $O/join_rp8.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/opbench.py --only config3 > $O/prof.log 2>&1
