#!/bin/bash
# Round 5: whole-step PMC traffic of the PINN and DPS steps only (re-run of the passes of
# tools/gpu_r05_pmc.sh whose profiler run crashed).
export TAG=r05
bash tools/gpu_pmc.sh steps "${MODES:-pinn dps}"
