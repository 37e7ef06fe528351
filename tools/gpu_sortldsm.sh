# sort ranking: per-wave LDS lane masks (variant ldsm) vs 8 ballots (default);
# the variant's sort parity tests first, then the op bench alternating
set -e
out=gpurun_out/sortldsm
mkdir -p $out
lib=$PWD/tools/variants/libmgdk_ldsm.so
MGDK_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py tests/test_gpu_firstn.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/ldsm.tests.log 2>&1
for v in base ldsm base ldsm; do
  if [ $v = base ]; then l=""; else l=$lib; fi
  MGDK_LIB=$l timeout -k 10 120 python tools/opbench.py --only other_ops >> $out/$v.json 2>> $out/$v.err
done
