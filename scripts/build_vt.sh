#!/bin/bash
# build_vt.sh NAME [-DMACRO ...] -- experiment library build/exp/libvt_NAME.so: vtrace.hip
# recompiled with the given macros, linked with the product objects of `make` (A/B only).
set -e
cd "$(dirname "$0")/.."
n=$1; shift
mkdir -p build/exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ifreeimpala_amd/csrc \
  -Wno-unused-result -Wno-unused-value "$@" -c freeimpala_amd/csrc/vtrace.hip -o build/exp/vt_$n.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/exp/libvt_$n.so build/exp/vt_$n.o \
  build/obj/gemm_f32.hip.o build/obj/misc.hip.o build/obj/atari.hip.o build/obj/atari_fr.hip.o \
  build/obj/fc_gemm.hip.o build/obj/farmer.hip.o build/obj/learner.cpp.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
