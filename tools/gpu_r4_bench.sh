# Round 4: the reworked bench (every config leg + full-size parity) at N=1,
# then the self-spawned 2-rank rehearsal over gloo on the one GPU.
set -e
out=gpurun_out/${1:-r4bench}
mkdir -p $out
timeout -k 10 500 python -u bench.py > $out/n1.json 2> $out/n1.err
timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo --sf 20 --no-cpu --window-rows 200000000 > $out/n2_gloo.json 2> $out/n2_gloo.err
