set -e
mkdir -p gpurun_out/pmcw2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmcw2/s -o run -- python3 tools/run_window.py 1000000000 2 > gpurun_out/pmcw2/s.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcw2/k -o run -- python3 tools/run_window.py 1000000000 3 > gpurun_out/pmcw2/k.log 2>&1
