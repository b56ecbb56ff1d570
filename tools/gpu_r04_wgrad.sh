#!/bin/bash
# Round 4: weight-gradient tests, then the Winograd wgrad microbench and the DSM train phase
# with the 128-cout (two N-blocks per wave) kernel vs the 64-cout variant build, interleaved.
mkdir -p gpurun_out; export TMPDIR=/tmp
# the variant library is built on the CPU side (tools/build_variant.sh) and travels with the tree
[ -f b-pinn-kalman-filter_amd/lib/variants/libbpk_nb1.so ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "weight_gradient or wgrad" > gpurun_out/t_wgrad.log 2>&1 || { tail -30 gpurun_out/t_wgrad.log; exit 1; }
tail -1 gpurun_out/t_wgrad.log
for v in new nb1 new nb1; do
  lib=""; [ $v = nb1 ] && lib="BPK_LIB=$PWD/b-pinn-kalman-filter_amd/lib/variants/libbpk_nb1.so"
  env $lib timeout -k 10 200 python tools/bench_wgrad.py > gpurun_out/wgrad_$v.log 2>&1 || { tail gpurun_out/wgrad_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/wgrad_$v.log | cut -c1-160
done
for v in new nb1; do
  lib=""; [ $v = nb1 ] && lib="BPK_LIB=$PWD/b-pinn-kalman-filter_amd/lib/variants/libbpk_nb1.so"
  env $lib timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --cifar-steps 6 > gpurun_out/train_$v.log 2>/dev/null || exit 1
  echo "== train $v"; python tools/show_line.py gpurun_out/train_$v.log
done
