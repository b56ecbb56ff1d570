#!/bin/bash
# Round 4: per-shape A/B of the Winograd PRE mix (tools/bench_wino_mix.py, B = 64 and 8): the
# 16-cin one-workgroup-per-CU kernel (default) vs the 8-cin forms (variant -DWINO_NO_K16: the
# 8-wave form for PRE+stats, the 4-wave two-workgroups-per-CU form for the residual tail),
# interleaved twice.
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -f b-pinn-kalman-filter_amd/lib/variants/libbpk_nok16.so ] || exit 1
for r in 1 2; do for v in k16 nok16; do for b in 64 8; do
  lib=""; [ $v = nok16 ] && lib="BPK_LIB=$PWD/b-pinn-kalman-filter_amd/lib/variants/libbpk_nok16.so"
  env $lib B=$b timeout -k 10 200 python tools/bench_wino_mix.py > gpurun_out/wmix_${v}_b${b}_$r.log 2>&1 || { tail gpurun_out/wmix_${v}_b${b}_$r.log; exit 1; }
  echo "== $v B=$b run $r: $(tail -1 gpurun_out/wmix_${v}_b${b}_$r.log | cut -c1-200)"
done; done; done
