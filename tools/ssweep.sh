# sort scatter shape sweep: waves per workgroup x rows per wave (variant
# libraries from tools/variant_build.py); sort parity tests, then the op bench
set -e
mkdir -p gpurun_out/ssweep
for v in base ${@:-w8r16 w4r16 w8r8 w16r8}; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py -m gpu -q -x -k "sort or order" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ssweep/$v.tests.log 2>&1
  MGDK_LIB=$lib timeout -k 10 120 python tools/opbench.py --only other_ops > gpurun_out/ssweep/$v.json 2> gpurun_out/ssweep/$v.err
done
