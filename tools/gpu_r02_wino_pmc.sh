#!/bin/bash
bash tools/gpu_wino_ab.sh || exit 1
bash tools/gpu_pmc_r02.sh || exit 1
