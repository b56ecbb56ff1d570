#!/bin/bash
# persistent 16-cin Winograd kernel (one workgroup per CU walking the items) vs one workgroup per
# item: conv parity tests on the persistent build, then the PRE shape mix and the sampler phase,
# interleaved x2 on one box
set -o pipefail
O=gpurun_out/r06persist; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/b-pinn-kalman-filter_amd/lib/variants
BPK_LIB=$L/libbpk_persist.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "conv or wino or gn or group or ncsnpp or ddpm or net" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
SAMPLER="--no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline --steps 10 --warmup 2"
for r in 1 2; do
  for v in np persist; do
    BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python3 tools/bench_wino_mix.py > $O/mix_${v}_$r.log 2>&1 || { tail $O/mix_${v}_$r.log; exit 1; }
    BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python3 bench.py $SAMPLER > $O/s_${v}_$r.json 2> $O/s_${v}_$r.err || { tail $O/s_${v}_$r.err; exit 1; }
    echo "$v $r: mix $(tail -1 $O/mix_${v}_$r.log | grep -o '"ms_per_forward_mix": [0-9.]*') sampler $(grep -o '"value": [0-9.]*' $O/s_${v}_$r.json)"
  done
done
