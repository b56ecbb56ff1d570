#!/bin/bash
# final tree: the GPU test tier + smoke, the driver's default bench command twice, the per-rank
# work of the 8-GPU point, and rocprofv3 summaries of the sampler (B=64 / B=8) and DPS
set -o pipefail
O=gpurun_out/r06final2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1500 python3 -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 900 python3 bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  grep -o '"value": [0-9.]*' $O/bench_$r.json | head -1
done
timeout -k 10 900 python3 bench.py --per-rank-of 8 > $O/per_rank_of_8.json 2> $O/per_rank_of_8.err || { tail -20 $O/per_rank_of_8.err; exit 1; }
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
SAMPLER="--no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline"
for n in b64 b8; do
  gb=64; [ $n = b8 ] && gb=8
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$n -o $n --output-format csv -- python3 bench.py --steps 4 --warmup 2 --global-batch $gb $SAMPLER > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  rm -f $O/$n/${n}_kernel_trace.csv
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dps -o dps --output-format csv -- python3 tools/prof_dps.py 2 > $O/dps.log 2>&1 || { tail -5 $O/dps.log; exit 1; }
rm -f $O/dps/dps_kernel_trace.csv
echo done
