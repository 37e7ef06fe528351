# sort tile-size sweep (variant libraries from tools/variant_build.py)
set -e
mkdir -p gpurun_out/ssweep
for v in base; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 120 python tools/opbench.py --only other_ops > gpurun_out/ssweep/$v.json 2> gpurun_out/ssweep/$v.err
done
