set -e
mkdir -p gpurun_out/pmcg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcg/t -o run -- python3 tools/run_gsorted.py > gpurun_out/pmcg/t.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmcg/s -o run -- python3 tools/run_gsorted.py 600000000 1 > gpurun_out/pmcg/s.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcg/f -o run -- python3 tools/run_gsorted.py 600000000 1 > gpurun_out/pmcg/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcg/w -o run -- python3 tools/run_gsorted.py 600000000 1 > gpurun_out/pmcg/w.log 2>&1
