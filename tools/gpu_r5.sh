# round-5 GPU steps: bash tools/gpu_r5.sh <step> [...]; each step writes under
# gpurun_out/r5/<step>/ and runs under its own time limit; the first failing
# step ends the call
set -e
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
for step in "$@"; do
O=gpurun_out/r5/$step
mkdir -p $O
case $step in
sort)
	timeout -k 10 600 $T tests/test_gpu_sort_progress.py tests/test_gpu_join_sort_window.py -k "sort" > $O/tests.log 2>&1
	for xg in 0 32 64 128 256; do
		MGDK_SORT_XCDG=$xg timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench_xg$xg.json 2> $O/opbench_xg$xg.err
	done
	;;
sortvar)
	# sort tile variants (tools/variant_build.py): opbench other_ops per variant x XCD group
	for v in $SORTVARS; do
		for xg in ${XGS:-32}; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so MGDK_SORT_XCDG=$xg timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench_${v}_xg$xg.json 2> $O/opbench_${v}_xg$xg.err
		done
	done
	;;
join)
	timeout -k 10 600 $T -x tests/test_gpu_join_sort_window.py tests/test_join_algo.py tests/test_join_str.py tests/test_msk_cands.py -k "join" > $O/tests.log 2>&1
	for v in 1 3; do
		MGDK_JOIN_PART=$v timeout -k 10 200 python tools/opbench.py --only config3 > $O/opbench_part$v.json 2> $O/opbench_part$v.err
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only config3 > $O/prof.log 2>&1
	;;
gsums)
	timeout -k 10 600 $T tests/test_gpu_group_sums.py > $O/tests.log 2>&1
	for r in a b; do
		for f in 0 1; do
			MGDK_GS_FUSED=$f timeout -k 10 200 python tools/opbench.py --only config4_group_sums > $O/opbench_f$f$r.json 2> $O/opbench_f$f$r.err
		done
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only config4_group_sums > $O/prof.log 2>&1
	MGDK_GS_FUSED=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fused -o run -- python3 tools/opbench.py --only config4_group_sums > $O/prof_fused.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/opbench.py --only config4_group_sums > $O/pmc_f.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/opbench.py --only config4_group_sums > $O/pmc_w.log 2>&1
	;;
gsvar)
	# group-sums variants (tools/variant_build.py): tests on the default build, then opbench
	# config4_group_sums alternating default / variants twice
	timeout -k 10 600 $T -x tests/test_gpu_group_sums.py > $O/tests.log 2>&1
	for r in a b; do
		timeout -k 10 200 python tools/opbench.py --only config4_group_sums > $O/default_$r.json 2> $O/default_$r.err
		for v in $GSVARS; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/opbench.py --only config4_group_sums > $O/${v}_$r.json 2> $O/${v}_$r.err
		done
	done
	;;
jk)
	timeout -k 10 600 $T tests/test_join_kinds.py tests/test_cand_algebra.py tests/test_theta_join.py > $O/tests.log 2>&1
	;;
stats)
	timeout -k 10 600 $T tests/test_group_stats.py tests/test_window_stats.py tests/test_gpu_window_funcs.py > $O/tests.log 2>&1
	;;
grp)
	timeout -k 10 600 $T tests/test_gpu_ops.py tests/test_gpu_group_sorted.py tests/test_gpu_group_str.py tests/test_gpu_props.py tests/test_msk_cands.py > $O/tests.log 2>&1
	;;
selvar)
	# select variants (tools/variant_build.py): the select suites on the default build, then
	# selgrp_trace alternating default / variants twice, then a kernel trace of the default
	timeout -k 10 600 $T -x tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_msk_cands.py tests/test_cand_algebra.py tests/test_gpu_threads.py tests/test_c_abi.py > $O/tests.log 2>&1
	for r in a b; do
		timeout -k 10 200 python tools/selgrp_trace.py > $O/default_$r.json 2> $O/default_$r.err
		for v in $SELVARS; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/selgrp_trace.py > $O/${v}_$r.json 2> $O/${v}_$r.err
		done
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/selgrp_trace.py > $O/prof.log 2>&1
	;;
selgrp)
	timeout -k 10 200 python tools/selgrp_trace.py > $O/plain.json 2> $O/plain.err
	for gg in 256 512 1024; do
		MGDK_GROUP_GRID=$gg MGDK_SEL_WGRID=$((gg * 2)) timeout -k 10 200 python tools/selgrp_trace.py > $O/grid$gg.json 2> $O/grid$gg.err
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/selgrp_trace.py > $O/prof.log 2>&1
	;;
markjoin)
	timeout -k 10 300 $T tests/test_join_kinds.py -k markjoin > $O/tests.log 2>&1
	;;
cand)
	timeout -k 10 600 $T tests/test_cand_algebra.py tests/test_gpu_window_funcs.py > $O/tests.log 2>&1
	;;
sortsuite)
	timeout -k 10 900 $T tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py tests/test_gpu_sort_hybrid.py tests/test_gpu_firstn.py tests/test_gpu_group_str.py tests/test_gpu_sort_progress.py > $O/tests.log 2>&1
	;;
all)
	timeout -k 10 1100 $T tests > $O/tests.log 2>&1
	;;
smoke)
	timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
	;;
bench)
	timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
	;;
opbench)
	timeout -k 10 600 python tools/opbench.py > $O/opbench.json 2> $O/opbench.err
	;;
soa)
	for p in 10 11; do
		timeout -k 10 120 tools/probes/join_soa_probe $p >> $O/soa.log 2>&1
	done
	;;
place)
	for p in 1024 2048 4096; do
		timeout -k 10 120 tools/probes/place_probe $p >> $O/place.log 2>&1
	done
	;;
joinlf)
	for v in "80 1" "80 0" "65 0" "50 0"; do
		set -- $v
		MGDK_PJ_LF=$1 MGDK_PJ2_OCC=$2 timeout -k 10 200 python tools/opbench.py --only config3 > $O/opbench_lf$1_occ$2.json 2> $O/opbench_lf$1_occ$2.err
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	MGDK_PJ_LF=50 MGDK_PJ2_OCC=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof50 -o run -- python3 tools/opbench.py --only config3 > $O/prof50.log 2>&1
	;;
joinpb)
	timeout -k 10 600 $T -x tests/test_gpu_join_sort_window.py -k "partitioned" > $O/tests.log 2>&1
	for v in ${PBV:-"0 80" "1 80" "1 70"}; do
		set -- $v
		MGDK_PJ2_PB=$1 MGDK_PJ_LF=$2 timeout -k 10 200 python tools/opbench.py --only config3 > $O/opbench_pb$1_lf$2.json 2> $O/opbench_pb$1_lf$2.err
	done
	cd /tmp && cd $GRAFT_REPO_ROOT
	MGDK_PJ2_PB=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only config3 > $O/prof.log 2>&1
	;;
joinpmc)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_sq -o run -- python3 tools/opbench.py --only config3 > $O/pmc_sq.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/opbench.py --only config3 > $O/pmc_f.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/opbench.py --only config3 > $O/pmc_w.log 2>&1
	;;
joinvar)
	# join variants (tools/variant_build.py): opbench config3 per variant
	for v in $JVARS; do
		MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/opbench.py --only config3 > $O/opbench_$v.json 2> $O/opbench_$v.err
	done
	;;
grpvar)
	for v in $GVARS; do
		MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/selgrp_trace.py > $O/selgrp_$v.json 2> $O/selgrp_$v.err
	done
	;;
sortprof)
	timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench.json 2> $O/opbench.err
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only other_ops > $O/prof.log 2>&1
	;;
final)
	# round-end evidence: suite, smoke, bench, rocprof of the bench, PMC passes
	timeout -k 10 1000 $T tests > $O/gpu_tests.log 2>&1
	timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
	timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu > $O/prof_bench.json 2> $O/prof_bench.err
	timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_f.log 2>&1
	timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_w.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_jf -o run -- python3 tools/opbench.py --only config3 config4_group_sums > $O/pmc_jf.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_jw -o run -- python3 tools/opbench.py --only config3 config4_group_sums > $O/pmc_jw.log 2>&1
	timeout -k 10 300 python tools/opbench.py > $O/opbench.json 2> $O/opbench.err
	;;
sortlb)
	for v in 1 0 1 0; do
		MGDK_SORT_LB=$v timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench_lb$v.json 2> $O/opbench_lb$v.err
		echo "lb=$v $(grep -h '"kernel_ms"' $O/opbench_lb$v.json | head -1)" >> $O/summary.txt
	done
	;;
sortdirect)
	for v in 0 1 0 1; do
		MGDK_SORT_DIRECT=$v timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench_d$v.json 2> $O/opbench_d$v.err
		grep -h '"kernel_ms"' $O/opbench_d$v.json | head -1 >> $O/summary.txt
	done
	;;
*)
	echo "unknown step $step"; exit 2
	;;
esac
done
