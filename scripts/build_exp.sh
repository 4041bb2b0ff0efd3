#!/bin/bash
# build_exp.sh NAME [-DMACRO ...] -- experiment library build/ab/lib_NAME.so: one source
# (SRC=<file>, default freeimpala_amd/csrc/atari_fr.hip) recompiled with the given macros and
# linked with the product objects of `make` in place of that source's own object (A/B only;
# build/ab travels to the GPU box, build/exp does not).
set -e
cd "$(dirname "$0")/.."
n=$1; shift
SRC=${SRC:-freeimpala_amd/csrc/atari_fr.hip}
base=$(basename "$SRC")
case " farmer.hip vtrace.hip gemm_f32.hip misc.hip atari.hip atari_fr.hip fc_gemm.hip learner.cpp " in
  *" $base "*) ;;
  *) echo "build_exp.sh: $SRC must be named after the product source it replaces" >&2; exit 2 ;;
esac
mkdir -p build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ifreeimpala_amd/csrc \
  -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics "$@" -x hip -c "$SRC" -o build/ab/x_$n.o
objs=""
for o in farmer.hip vtrace.hip gemm_f32.hip misc.hip atari.hip atari_fr.hip fc_gemm.hip learner.cpp; do
  if [ "$o" = "$base" ]; then objs="$objs build/ab/x_$n.o"; else objs="$objs build/obj/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/lib_$n.so $objs \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
