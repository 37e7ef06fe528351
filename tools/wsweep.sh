# RANGE window bounds tile-size sweep (variant libraries from tools/variant_build.py)
set -e
mkdir -p gpurun_out/wsweep
for v in base fr8h128 fr16h256 fr16h128 fr4h128; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 120 python tools/opbench.py --only window > gpurun_out/wsweep/$v.json 2> gpurun_out/wsweep/$v.err
done
