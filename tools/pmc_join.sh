# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the SF10 hash join
# (BASELINE config 3) plus its kernel trace; output under gpurun_out/pmcj
set -e
out=gpurun_out/pmcj
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/opbench.py --only config3_hashjoin_sf10 > $out/opbench.json 2> $out/trace.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/opbench.py --only config3_hashjoin_sf10 > $out/f.json 2> $out/f.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/opbench.py --only config3_hashjoin_sf10 > $out/w.json 2> $out/w.err
