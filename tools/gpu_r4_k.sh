# XCD group size sweep for the radix scatter passes; kernel stats of the other ops
set -e
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
for g in 32 128 256; do
  MGDK_SORT_XCDG=$g timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_xg$g.json 2> $O/opbench_xg$g.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/opbench.py --only other_ops > $O/prof.log 2>&1
