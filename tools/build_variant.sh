#!/bin/bash
# Build a variant of libbpk.so with extra -D flags on one source (A/B runs; SRC=conv_winograd
# by default):
#   [SRC=upfirdn2d] tools/build_variant.sh NAME "-DWINO_PRIO8=1 ..."  ->  lib/variants/libbpk_NAME.so
set -e
cd "$(dirname "$0")/../b-pinn-kalman-filter_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
out=../lib/variants; mkdir -p $out/obj_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../../include \
  -munsafe-fp-atomics -fno-slp-vectorize $@ -c ${SRC:-conv_winograd}.hip -o $out/obj_$name/${SRC:-conv_winograd}.o
objs=$(ls ../lib/obj/*.o | grep -v "/${SRC:-conv_winograd}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $out/obj_$name/${SRC:-conv_winograd}.o -o $out/libbpk_$name.so
rm -rf $out/obj_$name
echo built $out/libbpk_$name.so
