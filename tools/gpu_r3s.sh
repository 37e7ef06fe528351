set -e
mkdir -p gpurun_out/r3s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s/prof -o run -- python3 tools/opbench.py --only other_ops config3 config1 > gpurun_out/r3s/opbench.json 2> gpurun_out/r3s/opbench.err
