set -e
mkdir -p gpurun_out/pmcj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcj/s -o run -- python3 tools/run_join.py 1 > gpurun_out/pmcj/s.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcj/t -o run -- python3 tools/run_join.py 3 > gpurun_out/pmcj/t.log 2>&1
