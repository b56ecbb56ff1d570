#!/bin/bash
# Round 5: the persistent 16-cin Winograd form -- bit-identity / fp64 tests, then the PRE mix
# A/B (BPK_WINO_PERSIST=0 vs default) and the sampler line.
mkdir -p gpurun_out/r05d; export TMPDIR=/tmp
O=gpurun_out/r05d
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "persistent_form or winograd_split_k or pair_form" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1 0 1; do
  BPK_WINO_PERSIST=$v timeout -k 10 200 python tools/bench_wino_mix.py > $O/mix_$v.log 2>&1 || { tail -5 $O/mix_$v.log; exit 1; }
  echo "persist=$v $(tail -1 $O/mix_$v.log)"
done
grep 128@128 $O/mix_0.log $O/mix_1.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log
# the PC sampler's step graph with eager large-argument work between steps, same prior:
# with graph packet capture forced on (the runtime default) and with the package setting
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 240 python -u tools/audit_pinn_graph.py pc redlarge_item > $O/pc_pcap1.log 2>&1 || { tail -5 $O/pc_pcap1.log; exit 1; }
grep RESULT $O/pc_pcap1.log
timeout -k 10 240 python -u tools/audit_pinn_graph.py pc redlarge_item > $O/pc_pcap0.log 2>&1 || { tail -5 $O/pc_pcap0.log; exit 1; }
grep RESULT $O/pc_pcap0.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "graph or pair_form or weight_gradient or sharded_pinn or native_leaky" > $O/pytest_graph.log 2>&1 || { tail -30 $O/pytest_graph.log; exit 1; }
tail -2 $O/pytest_graph.log
