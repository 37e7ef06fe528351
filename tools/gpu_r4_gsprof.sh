# config-4 local step under the kernel trace (SF100 rows)
set -e
export TMPDIR=/tmp
O=gpurun_out/gsprof
mkdir -p $O
timeout -k 10 300 python tools/prof_dist_group.py 600121500 > $O/dist.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/prof_dist_group.py 600121500 > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run -- python tools/opbench.py --only other_ops > $O/prof2.log 2>&1
