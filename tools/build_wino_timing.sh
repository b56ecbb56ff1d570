#!/bin/bash
# Builds the timing-instrumented Winograd library (conv_winograd.hip -DWINO_TIMING + extra
# defines) for tools/wino_timing.py: tools/build_wino_timing.sh <name> [-DFOO=1 ...]
# -> b-pinn-kalman-filter_amd/lib/libbpk_wino_timing<name>.so
set -e
cd "$(dirname "$0")/../b-pinn-kalman-filter_amd/csrc"
name=$1; shift
d=$(mktemp -d)
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -munsafe-fp-atomics"
$H -DWINO_TIMING -fno-slp-vectorize "$@" -c conv_winograd.hip -o $d/w.o
$H -c bpk_common.hip -o $d/c.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/w.o $d/c.o -o ../lib/libbpk_wino_timing$name.so
rm -rf $d
