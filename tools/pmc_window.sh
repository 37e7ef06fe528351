set -e
mkdir -p gpurun_out/pmcw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcw/f -o run -- python3 tools/run_window.py > gpurun_out/pmcw/f.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw/w -o run -- python3 tools/run_window.py > gpurun_out/pmcw/w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcw/s -o run -- python3 tools/run_window.py > gpurun_out/pmcw/s.log 2>&1
