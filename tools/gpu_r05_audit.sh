#!/bin/bash
# Round 5, VERDICT r04 items 1-2: audit of the captured PINN step, fixed-parameter replays
# with different eager work between them, a rocprofv3 kernel summary of DPS NFEs, then
# (last: a profiler crash ends the call) a PMC FETCH_SIZE pass over the DPS step.
mkdir -p gpurun_out/r05a; export TMPDIR=/tmp
O=gpurun_out/r05a
timeout -k 10 400 python -u tools/audit_pinn_graph.py audit 64 > $O/audit.log 2>&1 || { tail -20 $O/audit.log; exit 1; }
tail -40 $O/audit.log
for m in ${MODES:-none memset0 memsetx redlarge redsmall d2h redlarge_item}; do
  timeout -k 10 240 python -u tools/audit_pinn_graph.py iso $m 64 > $O/iso_$m.log 2>&1 || { tail -5 $O/iso_$m.log; exit 1; }
  grep RESULT $O/iso_$m.log
done
cd /tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dps_prof -o dps --output-format csv -- python3 tools/prof_dps.py 2 > $O/dps_prof.log 2>&1 || { tail -5 $O/dps_prof.log; exit 1; }
tail -2 $O/dps_prof.log
if [ -n "$PMC" ]; then
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/dps_fetch -o pmc --output-format csv -- python3 tools/prof_steps.py dps > $O/dps_fetch.log 2>&1 || { tail -5 $O/dps_fetch.log; exit 1; }
  echo "dps fetch pass ok"
fi
