#!/usr/bin/env python3
"""Timing-only copy of atari_fr.hip with per-phase clock sums in conv12_fwd_fr (waves 0 and 4),
written to build/exp2/atari_fr.hip; build it with
  SRC=build/exp2/atari_fr.hip bash scripts/build_exp.sh c12ph 
The launcher prints '[phases conv12_fwd_fr wave W] clk/frame: B1 phaseA phaseB B2' on the 4th call.
Buckets: 1 = B1 wait, 2 = phase A, 3 = phase B, 4 = B2 wait."""
import os, re
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "freeimpala_amd/csrc/atari_fr.hip")).read()
macros = r'''
#include <cstdio>
#include <vector>
__device__ unsigned long long fi_phases[1024 * 16];
#define PH_DECL unsigned long long ph_[6] = {0, 0, 0, 0, 0, 0}, pt_ = __builtin_amdgcn_s_memtime(), rt0_ = __builtin_amdgcn_s_memrealtime(), ct0_ = pt_; int pn_ = 0;
#define PH(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph_[k] += t_ - pt_; pt_ = t_; } while (0)
#define PH_ITER() (++pn_)
#define PH_FLUSH() do { const int w_ = wave_id(); if ((threadIdx.x & 63) == 0 && (w_ == 0 || w_ == 4) && blockIdx.x < 1024) { \
    for (int k_ = 0; k_ < 6; ++k_) fi_phases[blockIdx.x * 16 + (w_ ? 8 : 0) + k_] = ph_[k_]; \
    fi_phases[blockIdx.x * 16 + (w_ ? 8 : 0) + 7] = pn_; \
    fi_phases[blockIdx.x * 16 + (w_ ? 8 : 0) + 6] = ((__builtin_amdgcn_s_memtime() - ct0_) << 20) / max(1ull, __builtin_amdgcn_s_memrealtime() - rt0_); } } while (0)
static void ph_report(const char* name, int grid) {
    static int calls = 0;
    if (++calls != 4) return;
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(1024 * 16);
    (void)hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(fi_phases), h.size() * 8);
    for (int r = 0; r < 2; ++r) {
        double sum[6] = {0}, n = 0, mhz = 0;
        for (int b = 0; b < grid && b < 1024; ++b) {
            for (int k = 0; k < 6; ++k) sum[k] += (double)h[b * 16 + 8 * r + k];
            n += (double)h[b * 16 + 8 * r + 7];
            mhz += (double)h[b * 16 + 8 * r + 6] / (1 << 20) * 100.0;
        }
        std::fprintf(stderr, "[phases %s wave %d] clk/frame: B1 %.0f  A %.0f  B %.0f  B2 %.0f  clock %.0f MHz\n", name, 4 * r,
                     sum[1] / n, sum[2] / n, sum[3] / n, sum[4] / n, mhz / grid);
    }
}
'''
src = src.replace('namespace fi {\n', 'namespace fi {\n' + macros, 1)
k0 = src.index('void conv12_fwd_fr(')
k1 = src.index('int conv12_fwd_fr_launch(')
ker = src[k0:k1]
def sub(old, new, count):
    global ker
    assert ker.count(old) == count, (old, ker.count(old))
    ker = ker.replace(old, new)
sub('        for (int it = 0; it <= nmine; ++it) {\n', '        PH_DECL\n        for (int it = 0; it <= nmine; ++it) {\n            PH(3);\n            PH_ITER();\n', 2)
sub('            lds_barrier();  // B1: image(it) complete; the conv2 image read by conv2(it-2)\n',
    '            lds_barrier();  // B1: image(it) complete; the conv2 image read by conv2(it-2)\n            PH(1);\n', 1)
sub('            lds_barrier();  // B1\n', '            lds_barrier();  // B1\n            PH(1);\n', 1)
sub('            lds_barrier();  // B2: the conv2 image complete\n', '            PH(2);\n            lds_barrier();  // B2: the conv2 image complete\n            PH(4);\n', 1)
sub('            lds_barrier();  // B2: a1(it-1) in the conv2 image\n', '            PH(2);\n            lds_barrier();  // B2: a1(it-1) in the conv2 image\n            PH(4);\n', 1)
sub('        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n', '        PH(3);\n        PH_FLUSH();\n        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n', 2)
src = src[:k0] + ker + src[k1:]
src = src.replace('                       a1_planar);\n    FI_HIP_CHECK(hipGetLastError());\n    return FI_OK;\n}',
                  '                       a1_planar);\n    FI_HIP_CHECK(hipGetLastError());\n    ph_report("conv12_fwd_fr", grid);\n    return FI_OK;\n}', 1)
os.makedirs(os.path.join(ROOT, "build/exp2"), exist_ok=True)
open(os.path.join(ROOT, "build/exp2/atari_fr.hip"), "w").write(src)
print("wrote build/exp2/atari_fr.hip")
