#!/bin/bash
# Round 6: native spatial embedding (+ derivatives), batched timestep embeddings, ResidualBlock
# skip add in conv2's epilogue: parity tests, then PINN graph-step timing (B=8, B=64).
set -o pipefail
O=gpurun_out/r06emb; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pinn.py tests/test_gpu_configs.py -k "pinn or spatial" tests/test_gpu_graph.py > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
run() { # name per-rank-of env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python3 tools/prof_pinn.py graph $n 20 > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(grep -o "'pinn_train_steps_per_s': [0-9.]*" $O/$name.log) $(grep -o "'pinn_losses': [^]]*" $O/$name.log)"
}
run b8 8
run b8_old 8 BPK_SEMB_FUSED=0 BPK_RES_TAIL=0
run b64 1
run b64_old 1 BPK_SEMB_FUSED=0 BPK_RES_TAIL=0
run b16 4
run b32 2
run b32_c4 2 BPK_PINN_COPIES=4
