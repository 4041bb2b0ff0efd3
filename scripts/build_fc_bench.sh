#!/bin/bash
# builds build/fc_bench (scripts/fc_bench.hip) against the in-tree libfi_learner.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ifreeimpala_amd/csrc scripts/fc_bench.hip \
    -o build/fc_bench -Lfreeimpala_amd/lib -lfi_learner '-Wl,-rpath,$ORIGIN/../freeimpala_amd/lib' -Wl,-rpath,/opt/rocm/lib
