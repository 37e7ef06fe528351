# PMC of the sort's local pass (SQ counters; one pass, one sort)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq -o run -- python3 tools/run_sort.py 100000000 1 > $O/sq.log 2>&1
