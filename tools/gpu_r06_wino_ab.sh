#!/bin/bash
# Round 6 Winograd K16 A/B (tools/build_variant.sh): PRE shape-mix microbench at B=64, the base
# library against variants, interleaved x2 on one box; then one parity pass per variant.
set -o pipefail
O=gpurun_out/r06wino; mkdir -p $O; export TMPDIR=/tmp
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base ss pl2ss pl2; do
    lib=$PWD/$L/variants/libbpk_$v.so; [ $v = base ] && lib=$PWD/$L/libbpk_base.so
    BPK_LIB=$lib timeout -k 10 300 python3 tools/bench_wino_mix.py > $O/mix_${v}_$r.log 2>&1 || { tail $O/mix_${v}_$r.log; exit 1; }
    echo "$v $r: $(tail -1 $O/mix_${v}_$r.log | cut -c1-300)"
  done
done
for v in ss pl2ss; do
  BPK_LIB=$PWD/$L/variants/libbpk_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "winograd or wino" > $O/tests_$v.log 2>&1 || { tail -20 $O/tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/tests_$v.log)"
done
