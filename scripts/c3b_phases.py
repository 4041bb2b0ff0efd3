#!/usr/bin/env python3
"""Timing-only copy of atari_fr.hip with per-phase clock sums in conv3_bwd_fr, written to
build/exp2/atari_fr.hip; build it with
  SRC=build/exp2/atari_fr.hip bash scripts/build_exp.sh c3bph
The launcher prints, on the 4th call, the mean clocks per frame of waves 0, 2 (weight gradient
+ DMA issue, 5 and 4 k-tiles), 4 and 6 (data gradient) in the buckets of c3_frames' loop:
  bar = lds_barrier wait, vm = the issuer's vmcnt wait for its next pieces,
  reshuffle, issue = the DMA issue of frame it + 3, work = the wave's MFMA body (dgrad: with its stores).
s_memtime forces an lgkmcnt wait at each stamp, so the sums are an upper bound of each phase."""
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "freeimpala_amd/csrc/atari_fr.hip")).read()
macros = r'''
#include <cstdio>
#include <vector>
__device__ unsigned long long fi_phases[1024 * 32];
__device__ unsigned long long fi_dg[1024 * 8];  // dgrad waves 4, 6: MFMA loop / epilogue clock sums
#define PH_DECL unsigned long long ph_[6] = {0, 0, 0, 0, 0, 0}, pt_ = __builtin_amdgcn_s_memtime(), rt0_ = __builtin_amdgcn_s_memrealtime(), ct0_ = pt_; int pn_ = 0;
#define PH(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph_[k] += t_ - pt_; pt_ = t_; } while (0)
#define PH_ITER() (++pn_)
#define PH_FLUSH() do { const int w_ = wave_id(); if ((threadIdx.x & 63) == 0 && (w_ & 1) == 0 && blockIdx.x < 1024) { \
    const int s_ = blockIdx.x * 32 + 8 * (w_ >> 1); \
    for (int k_ = 0; k_ < 6; ++k_) fi_phases[s_ + k_] = ph_[k_]; \
    fi_phases[s_ + 7] = pn_; \
    fi_phases[s_ + 6] = ((__builtin_amdgcn_s_memtime() - ct0_) << 20) / max(1ull, __builtin_amdgcn_s_memrealtime() - rt0_); } } while (0)
static void ph_report(const char* name, int grid) {
    static int calls = 0;
    if (++calls != 4) return;
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(1024 * 32);
    (void)hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(fi_phases), h.size() * 8);
    for (int r = 0; r < 4; ++r) {
        double sum[6] = {0}, n = 0, mhz = 0;
        for (int b = 0; b < grid && b < 1024; ++b) {
            for (int k = 0; k < 6; ++k) sum[k] += (double)h[b * 32 + 8 * r + k];
            n += (double)h[b * 32 + 8 * r + 7];
            mhz += (double)h[b * 32 + 8 * r + 6] / (1 << 20) * 100.0;
        }
        std::fprintf(stderr, "[phases %s wave %d] clk/frame: bar %.0f  vm %.0f  reshuffle %.0f  issue %.0f  work %.0f  total %.0f  clock %.0f MHz\n",
                     name, 2 * r, sum[1] / n, sum[2] / n, sum[5] / n, sum[3] / n, sum[4] / n,
                     (sum[1] + sum[2] + sum[3] + sum[4] + sum[5]) / n, mhz / grid);
    }
    std::vector<unsigned long long> d(1024 * 8);
    (void)hipMemcpyFromSymbol(d.data(), HIP_SYMBOL(fi_dg), d.size() * 8);
    for (int r = 0; r < 2; ++r) {
        double a = 0, b = 0, n = 0;
        for (int g = 0; g < grid && g < 1024; ++g) { a += d[g * 8 + 4 * r]; b += d[g * 8 + 4 * r + 1]; n += d[g * 8 + 4 * r + 2]; }
        std::fprintf(stderr, "[phases %s wave %d] dgrad work split: mfma loop %.0f  epilogue %.0f clk/frame\n", name, 4 + 2 * r, a / n, b / n);
    }
}
'''
src = src.replace('namespace fi {\n', 'namespace fi {\n' + macros, 1)
k0 = src.index('__device__ __forceinline__ void c3_frames(')
k1 = src.index('// weight gradient of one wave, taps t = 2i + B')
ker = src[k0:k1]


def sub(old, new, count=1):
    global ker
    assert ker.count(old) == count, (old, ker.count(old))
    ker = ker.replace(old, new)


sub('    for (int it = 0; it < nmine; ++it) {\n', '    PH_DECL\n    for (int it = 0; it < nmine; ++it) {\n')
sub('        lds_barrier();  // frame it in slot it&1; every wave done with frame it-1 (slot (it+1)&1)\n',
    '        PH(0);\n        lds_barrier();  // frame it in slot it&1; every wave done with frame it-1 (slot (it+1)&1)\n        PH(1);\n')
sub('            wait_vmcnt(issued - mA);  // own pieces of frame it+1 landed\n',
    '            wait_vmcnt(issued - mA);  // own pieces of frame it+1 landed\n            PH(2);\n')
sub('            mA = mB;\n            mB = mC;\n        }\n        work(X, f);\n        issued += nst;\n',
    '            mA = mB;\n            mB = mC;\n            PH(3);\n        }\n        work(X, f);\n        PH(4);\n        PH_ITER();\n        issued += nst;\n')
sub('            reshuffle((it + 1) & 1, (it + 1) & 1);\n            int mC = issued;\n',
    '            reshuffle((it + 1) & 1, (it + 1) & 1);\n            PH(5);\n            int mC = issued;\n')
sub('    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n}\n',
    '    PH_FLUSH();\n    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n}\n')
src = src[:k0] + ker + src[k1:]
k0 = src.index('__global__ __launch_bounds__(512, 2) void conv3_bwd_fr(')
k1 = src.index('int conv3_bwd_fr_launch(')
ker = src[k0:k1]
sub('        auto work = [&](auto phc, const char* X, int f) {\n',
    '        unsigned long long dg_m = 0, dg_e = 0, dg_n = 0;\n        auto work = [&](auto phc, const char* X, int f) {\n            const unsigned long long tq0 = __builtin_amdgcn_s_memtime();\n')
sub('            u32x4* dst = (u32x4*)(ctx.da2 + (size_t)f * 5184);\n',
    '            const unsigned long long tq1 = __builtin_amdgcn_s_memtime();\n            dg_m += tq1 - tq0;\n            u32x4* dst = (u32x4*)(ctx.da2 + (size_t)f * 5184);\n')
sub('        c3_frames<false>(ctx, smem, 3, [&](const char* X, int f) {\n            if (ph) work(std::integral_constant<int, 1>{}, X, f);\n            else work(std::integral_constant<int, 0>{}, X, f);\n        });\n',
    '        c3_frames<false>(ctx, smem, 3, [&](const char* X, int f) {\n            const unsigned long long te0 = __builtin_amdgcn_s_memtime();\n            if (ph) work(std::integral_constant<int, 1>{}, X, f);\n            else work(std::integral_constant<int, 0>{}, X, f);\n            (void)te0;\n            dg_e += __builtin_amdgcn_s_memtime() - te0;\n            ++dg_n;\n        });\n'
    '        if (lane == 0 && (w == 4 || w == 6) && blockIdx.x < 1024) {\n            fi_dg[blockIdx.x * 8 + 4 * ((w - 4) >> 1)] = dg_m;\n            fi_dg[blockIdx.x * 8 + 4 * ((w - 4) >> 1) + 1] = dg_e - dg_m;\n            fi_dg[blockIdx.x * 8 + 4 * ((w - 4) >> 1) + 2] = dg_n;\n        }\n')
src = src[:k0] + ker + src[k1:]
old = '''    hipLaunchKernelGGL(conv3_bwd_fr, dim3(grid), dim3(512), 0, s, a2, da3, a3, w3d, da2,
                       slab, cs_slab, cs2, nframes);
    FI_HIP_CHECK(hipGetLastError());
'''
assert src.count(old) == 1
src = src.replace(old, old + '    ph_report("conv3_bwd_fr", grid);\n')
os.makedirs(os.path.join(ROOT, "build/exp2"), exist_ok=True)
open(os.path.join(ROOT, "build/exp2/atari_fr.hip"), "w").write(src)
print("wrote build/exp2/atari_fr.hip")
