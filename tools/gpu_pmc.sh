#!/bin/bash
# PMC passes: one counter group per rocprofv3 run, each under its own limit; output
# directories are named <mode>_<group> under gpurun_out/pmc_$TAG (summarise with
# tools/pmc_summary.py gpurun_out/pmc_$TAG $TAG on the same tree: it records the kernel
# sources' sha1, which bench.py checks before it uses an entry).
# $1 = kernels (single-kernel passes) | steps (whole-step traffic; $2 = modes)
TAG=${TAG:-r06}
D=gpurun_out/pmc_$TAG
# the profiler's preloaded library starts the HIP runtime before Python runs: the graph
# packet-capture setting must come from the environment (op/_hipenv.py is too late there).
# Rounds 4-5 ran without it and needed a 64 MB kernel-argument pool to keep the PINN / DPS
# passes from dying with SIGSEGV inside a launch; with the setting in effect the DPS pass runs
# at the default pool (round 6, profiles/r06_pmc_dps_default_pool.txt)
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
mkdir -p $D; export TMPDIR=/tmp
run() {  # script mode group counters...
  local script=$1 mode=$2 grp=$3; shift 3
  timeout -s KILL ${PMC_LIMIT:-240} rocprofv3 --pmc "$@" -d $D/${mode}_$grp -o pmc --output-format csv -- python $script $mode > $D/${mode}_$grp.log 2>&1 || { echo "pass $mode $grp failed"; grep -v "^[WE]2026\|^    @" $D/${mode}_$grp.log | tail -12; exit 1; }
  echo "pass $mode $grp ok"
}
if [ "${1:-kernels}" = kernels ]; then
run tools/prof_r02.py wino_one sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run tools/prof_r02.py wino_one sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run tools/prof_r02.py mix fetch FETCH_SIZE
run tools/prof_r02.py mix write WRITE_SIZE
run tools/prof_r02.py upfirdn fetch FETCH_SIZE
run tools/prof_r02.py upfirdn write WRITE_SIZE
run tools/prof_r02.py ns fetch FETCH_SIZE
run tools/prof_r02.py ns write WRITE_SIZE
run tools/prof_r02.py ns sq SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
else
for m in ${2:-train cifar pinn dps}; do
  run tools/prof_steps.py $m fetch FETCH_SIZE
  python tools/pmc_summary.py $D $TAG reduce-step $m FETCH_SIZE && rm -rf $D/${m}_fetch
  run tools/prof_steps.py $m write WRITE_SIZE
  python tools/pmc_summary.py $D $TAG reduce-step $m WRITE_SIZE && rm -rf $D/${m}_write
done
fi
echo PMC_DONE
