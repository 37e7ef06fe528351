# select: scan fused into the write pass vs the separate scan kernel (the
# round-3 experiment behind profiles/r03/select_fuse; the fused variant was
# dropped, so both legs now run the same library unless a variant is rebuilt)
set -e
out=gpurun_out/selfuse
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_exchange_ops.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
for v in fused nofuse fused nofuse; do
  if [ $v = fused ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 120 python tools/opbench.py --only config1_thetaselect config2_q6 >> $out/$v.json 2>> $out/$v.err
done
