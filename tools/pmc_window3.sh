set -e
mkdir -p gpurun_out/pmcw3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcw3/s -o run -- python3 tools/run_window.py 1000000000 2 > gpurun_out/pmcw3/s.log 2>&1
MGDK_WIN_LEAN=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcw3/o -o run -- python3 tools/run_window.py 1000000000 2 > gpurun_out/pmcw3/o.log 2>&1
