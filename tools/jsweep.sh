set -e
mkdir -p gpurun_out/jsweep
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 110 130 160 200 300; do
  MGDK_JOIN_CAP_PCT=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jsweep/c$c -o run -- python3 tools/opbench.py --only hashjoin > gpurun_out/jsweep/c$c.json 2> gpurun_out/jsweep/c$c.err
done
