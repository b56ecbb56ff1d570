#!/bin/bash
# Same-box A/B of two libbpk.so builds (lib/libbpk_A.so vs lib/libbpk_B.so) on the PINN
# train step (and the short sampler line that always runs).
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
L=$PWD/b-pinn-kalman-filter_amd/lib
for i in 1 2; do for v in A B; do
  BPK_LIB=$L/libbpk_$v.so timeout -k 10 400 python bench.py --steps 3 --no-train --no-dps --no-cpu-baseline --pinn-steps 8 > gpurun_out/pab_$v$i.log 2> gpurun_out/pab_$v$i.err || { tail -5 gpurun_out/pab_$v$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pab_$v$i.log'));print('$v', d['value'], d['pinn_train_steps_per_s'], d['pinn_losses'])"
done; done
