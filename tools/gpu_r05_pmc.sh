#!/bin/bash
# Round 5 PMC re-collection on the final kernels: single-kernel passes, then whole-step traffic
# of the four steps (the kernel-argument pool at 64 MB, tools/gpu_pmc.sh).
export TAG=r05
bash tools/gpu_pmc.sh kernels && bash tools/gpu_pmc.sh steps "train cifar pinn dps"
