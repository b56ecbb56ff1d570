#!/bin/bash
# Round 6 (session 2): in-launch split-K combine -- parity tests, split census, PINN B=8 / B=64
# graph step with the combine off (BPK_SPLITK_FUSE_MAX=0) and on (default).
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "igemm or wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/census_splitk.py 8 > $O/census_b8.json 2> $O/census_b8.err || { tail -20 $O/census_b8.err; exit 1; }
for f in 0 16; do
  BPK_SPLITK_FUSE_MAX=$f timeout -k 10 300 python3 tools/prof_pinn.py graph 8 30 > $O/b8_f$f.log 2>&1 || { tail -20 $O/b8_f$f.log; exit 1; }
  echo "fuse $f B=8: $(tail -1 $O/b8_f$f.log | cut -c1-200)"
done
for f in 0 16; do
  BPK_SPLITK_FUSE_MAX=$f timeout -k 10 300 python3 tools/prof_pinn.py graph 1 20 > $O/b64_f$f.log 2>&1 || { tail -20 $O/b64_f$f.log; exit 1; }
  echo "fuse $f B=64: $(tail -1 $O/b64_f$f.log | cut -c1-200)"
done
