#!/bin/bash
# persistent K16 item order: rr (round-robin rounds of G items) vs xr (each XCD walks a contiguous
# eighth of the items) vs np (one workgroup per item): PRE mix time, sampler, mix HBM fetch
set -o pipefail
O=gpurun_out/r06persist2; mkdir -p $O; export TMPDIR=/tmp; export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
L=$PWD/b-pinn-kalman-filter_amd/lib/variants
BPK_LIB=$L/libbpk_xr.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_ops.py -k "conv or wino" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
SAMPLER="--no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline --steps 10 --warmup 2"
for r in 1 2; do
  for v in np rr xr; do
    BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python3 tools/bench_wino_mix.py > $O/mix_${v}_$r.log 2>&1 || { tail $O/mix_${v}_$r.log; exit 1; }
    BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python3 bench.py $SAMPLER > $O/s_${v}_$r.json 2> $O/s_${v}_$r.err || { tail $O/s_${v}_$r.err; exit 1; }
    echo "$v $r: mix $(tail -1 $O/mix_${v}_$r.log | grep -o '"ms_per_forward_mix": [0-9.]*') sampler $(grep -o '"value": [0-9.]*' $O/s_${v}_$r.json)"
  done
done
for v in np rr xr; do
  BPK_LIB=$L/libbpk_$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o pmc --output-format csv -- python3 tools/prof_r02.py mix > $O/f_$v.log 2>&1 || { tail -5 $O/f_$v.log; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$O/f_$v/**/*counter_collection*.csv',recursive=True)[0]
v=sum(float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'wino_f23' in r['Kernel_Name'])
print('$v mix FETCH_SIZE x2 GB', round(2*v*1024/1e9,2))"
done
