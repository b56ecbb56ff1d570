#!/bin/bash
# Round 5: whole-step PMC traffic on the final kernels (the single-kernel passes of
# tools/gpu_r05_pmc.sh still match their sources).
export TAG=r05
bash tools/gpu_pmc.sh steps "train cifar pinn dps"
