# local pass: wait / instruction counters, and the time without its LDS passes
set -e
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 tools/run_sort.py 100000000 1 > $O/sq.log 2>&1
MGDK_LIB=$PWD/tools/variants/libmgdk_nopass.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_nopass -o run -- python3 tools/run_sort.py > $O/p_nopass.log 2>&1
MGDK_SORT_LOCALXG=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_xg0 -o run -- python3 tools/run_sort.py > $O/p_xg0.log 2>&1
