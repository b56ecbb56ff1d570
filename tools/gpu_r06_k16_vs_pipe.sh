#!/bin/bash
# Round 6 (session 2): per-shape K16 vs the 8-cin pipelined form (variant WINO_NO_K16) on the
# NCSN++ PRE mix, interleaved x2, B = 64 and 8.  The variant library is built beforehand, in
# this container: tools/build_variant.sh nok16 "-DWINO_NO_K16=1", then copied to
# b-pinn-kalman-filter_amd/lib/libbpk_nok16_ab.so (lib/variants/ does not travel to the box).
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in default nok16; do
    if [ $v = nok16 ]; then export BPK_LIB=$PWD/b-pinn-kalman-filter_amd/lib/libbpk_nok16_ab.so; else unset BPK_LIB; fi
    for b in 64 8; do
      B=$b timeout -k 10 300 python3 tools/bench_wino_mix.py > $O/${v}_b${b}_$r.log 2>&1 || { tail -5 $O/${v}_b${b}_$r.log; exit 1; }
      tail -1 $O/${v}_b${b}_$r.log
    done
  done
done
