#!/bin/bash
# build_exp.sh NAME [-DMACRO ...] -- experiment library build/ab/lib_NAME.so: atari_fr.hip
# (or SRC=<file>) recompiled with the given macros, linked with the product objects of `make`
# (A/B only; build/ab travels to the GPU box, build/exp does not).
set -e
cd "$(dirname "$0")/.."
n=$1; shift
SRC=${SRC:-freeimpala_amd/csrc/atari_fr.hip}
mkdir -p build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ifreeimpala_amd/csrc \
  -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics "$@" -x hip -c "$SRC" -o build/ab/fr_$n.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/lib_$n.so build/obj/farmer.hip.o build/obj/vtrace.hip.o \
  build/obj/gemm_f32.hip.o build/obj/misc.hip.o build/obj/atari.hip.o build/ab/fr_$n.o build/obj/fc_gemm.hip.o \
  build/obj/fc_blaslt.cpp.o build/obj/learner.cpp.o -L/opt/rocm/lib -lrccl -lhipblaslt -Wl,-rpath,/opt/rocm/lib
