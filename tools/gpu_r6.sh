# round-6 GPU steps: bash tools/gpu_r6.sh <step> [...]; each step writes under
# gpurun_out/r6/<step>/ and runs under its own time limit; the first failing
# step ends the call, except that a test step whose pytest exits 1 (tests
# failed, nothing crashed) lets the next steps run
set -e
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
tests() {
	local rc=0
	timeout -k 10 "$@" || rc=$?
	if [ $rc -eq 1 ]; then echo "tests failed (rc 1), continuing"; return 0; fi
	return $rc
}
for step in "$@"; do
O=gpurun_out/r6/$step
mkdir -p $O
case $step in
gputests)
	tests 900 $T -x tests > $O/tests.log 2>&1
	;;
dist)
	tests 300 $T -x tests/test_gpu_distributed.py > $O/tests.log 2>&1
	;;
jk)
	tests 600 $T -x tests/test_join_kinds.py tests/test_cand_algebra.py tests/test_theta_join.py tests/test_leftjoin_multi.py > $O/tests.log 2>&1
	;;
tests_*)
	tests 600 $T -x ${TESTS} > $O/tests.log 2>&1
	;;
jvar)
	# join variants (tools/variant_build.py): opbench config3, default / variants alternating twice
	for r in a b; do
		timeout -k 10 200 python tools/opbench.py --only config3 > $O/default_$r.json 2> $O/default_$r.err
		for v in $JVARS; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/opbench.py --only config3 > $O/${v}_$r.json 2> $O/${v}_$r.err
		done
	done
	;;
svar)
	# select variants: opbench config1, default / variants alternating twice
	for r in a b; do
		timeout -k 10 200 python tools/opbench.py --only config1 > $O/default_$r.json 2> $O/default_$r.err
		for v in $SVARS; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/opbench.py --only config1 > $O/${v}_$r.json 2> $O/${v}_$r.err
		done
	done
	;;
final_a)
	# round-end evidence, part 1: the GPU suite and the smoke test
	tests 1000 $T tests > $O/gpu_tests.log 2>&1
	timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
	;;
final_b)
	# round-end evidence, part 2: the driver line, rocprof of it, PMC passes, the op legs
	timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu > $O/prof_bench.json 2> $O/prof_bench.err
	timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_f.log 2>&1
	timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_w.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_jf -o run -- python3 tools/opbench.py --only config3 config4_group_sums > $O/pmc_jf.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_jw -o run -- python3 tools/opbench.py --only config3 config4_group_sums > $O/pmc_jw.log 2>&1
	timeout -k 10 300 python tools/opbench.py > $O/opbench.json 2> $O/opbench.err
	;;
sprof)
	# kernel trace of opbench config1 (the select legs)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default -o run -- python3 tools/opbench.py --only config1 > $O/default.log 2>&1
	;;
q1prof)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/q1op_prof.py 3 > $O/q1.log 2>&1
	;;
benchrep)
	# the driver line twice more on one box (run-to-run spread)
	timeout -k 10 420 python bench.py > $O/bench_1.json 2> $O/bench_1.err
	timeout -k 10 420 python bench.py > $O/bench_2.json 2> $O/bench_2.err
	;;
bench)
	timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
	;;
benchprof)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-parity > $O/bench.json 2> $O/bench.err
	;;
jprof)
	# per-kernel times of opbench config3 for the default library and each of $JVARS
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default -o run -- python3 tools/opbench.py --only config3 > $O/default.log 2>&1
	for v in $JVARS; do
		MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/opbench.py --only config3 > $O/$v.log 2>&1
	done
	;;
join)
	timeout -k 10 200 python tools/opbench.py --only config3 > $O/opbench.json 2> $O/opbench.err
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only config3 > $O/prof.log 2>&1
	;;
joinpmc)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq -o run -- python3 tools/opbench.py --only config3 > $O/pmc_sq.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- python3 tools/opbench.py --only config3 > $O/pmc_tcc.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/opbench.py --only config3 > $O/pmc_f.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/opbench.py --only config3 > $O/pmc_w.log 2>&1
	;;
sortenv)
	# sort under environment switches, alternating: default, LB=0, HYBRID=1
	for r in a b; do
		timeout -k 10 200 python tools/opbench.py --only other_ops > $O/default_$r.json 2> $O/default_$r.err
		MGDK_SORT_LB=0 timeout -k 10 200 python tools/opbench.py --only other_ops > $O/lb0_$r.json 2> $O/lb0_$r.err
		MGDK_SORT_HYBRID=1 timeout -k 10 200 python tools/opbench.py --only other_ops > $O/hy_$r.json 2> $O/hy_$r.err
	done
	;;
fpcliff)
	timeout -k 10 600 python tools/fp_cliff.py > $O/fp_cliff.json 2> $O/fp_cliff.err
	;;
fpprof)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/fp_cliff.py 100000000 par > $O/prof.log 2>&1
	;;
envvar)
	# opbench legs under environment switches, alternating (ENVLEG: opbench --only key; ENVS: NAME=VAR=VALUE ...)
	for r in a b; do
		timeout -k 10 300 python tools/opbench.py --only $ENVLEG > $O/default_$r.json 2> $O/default_$r.err
		for ev in $ENVS; do
			nm=${ev%%=*}; kv=${ev#*=}
			env $kv timeout -k 10 300 python tools/opbench.py --only $ENVLEG > $O/${nm}_$r.json 2> $O/${nm}_$r.err
		done
	done
	;;
sortvar)
	# sort variants (tools/variant_build.py): opbench other_ops, default / variants alternating twice
	for r in a b; do
		timeout -k 10 200 python tools/opbench.py --only other_ops > $O/default_$r.json 2> $O/default_$r.err
		for v in $SVARS; do
			MGDK_LIB=$PWD/tools/variants/libmgdk_$v.so timeout -k 10 200 python tools/opbench.py --only other_ops > $O/${v}_$r.json 2> $O/${v}_$r.err
		done
	done
	;;
sortpmc)
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq -o run -- python3 tools/run_sort.py 100000000 2 > $O/pmc_sq.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- python3 tools/run_sort.py 100000000 2 > $O/pmc_tcc.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/run_sort.py 100000000 2 > $O/pmc_f.log 2>&1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/run_sort.py 100000000 2 > $O/pmc_w.log 2>&1
	timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/run_sort.py 100000000 2 > $O/prof.log 2>&1
	;;
sort)
	timeout -k 10 200 python tools/opbench.py --only other_ops > $O/opbench.json 2> $O/opbench.err
	cd /tmp && cd $GRAFT_REPO_ROOT
	timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/opbench.py --only other_ops > $O/prof.log 2>&1
	;;
*)
	echo "unknown step $step"; exit 2
	;;
esac
echo "step $step done"
done
