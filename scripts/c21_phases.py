#!/usr/bin/env python3
"""Timing-only copy of atari_fr.hip with per-phase clock sums in conv21_bwd_fr, written to
build/exp2/c21ph/atari_fr.hip; build it with
  SRC=build/exp2/c21ph/atari_fr.hip bash scripts/build_exp.sh c21ph
The launcher prints, on the 4th call, the mean clocks per frame of waves 0, 2 (conv2 weight
gradient, raw-frame conversion, all DMA) and 4, 6 (conv2 data gradient -> da1 in LDS, then conv1's
weight gradient) in these buckets:
  waves 0-3: vm (wait for da2(it)), B1, wgrad2, convert, B2, dma (issue of da2(it+1), a1(it+2))
  waves 4-7: B1, dgrad2 (with its epilogues), B2, wgrad1 (with the segment flush)
s_memtime forces an lgkmcnt wait at each stamp, so the sums are an upper bound of each phase."""
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "freeimpala_amd/csrc/atari_fr.hip")).read()
macros = r'''
#include <cstdio>
#include <vector>
__device__ unsigned long long fi_phases[1024 * 32];
#define PH_DECL unsigned long long ph_[7] = {0, 0, 0, 0, 0, 0, 0}, pt_ = __builtin_amdgcn_s_memtime(), rt0_ = __builtin_amdgcn_s_memrealtime(), ct0_ = pt_; int pn_ = 0;
#define PH(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph_[k] += t_ - pt_; pt_ = t_; } while (0)
#define PH_ITER() (++pn_)
#define PH_FLUSH() do { const int w_ = wave_id(); if ((threadIdx.x & 63) == 0 && (w_ & 1) == 0 && blockIdx.x < 1024) { \
    const int s_ = blockIdx.x * 32 + 8 * (w_ >> 1); \
    for (int k_ = 0; k_ < 6; ++k_) fi_phases[s_ + k_] = ph_[k_ + 1]; \
    fi_phases[s_ + 7] = pn_; \
    fi_phases[s_ + 6] = ((__builtin_amdgcn_s_memtime() - ct0_) << 20) / max(1ull, __builtin_amdgcn_s_memrealtime() - rt0_); } } while (0)
static void ph_report(const char* name, int grid) {
    static int calls = 0;
    if (++calls != 4) return;
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(1024 * 32);
    (void)hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(fi_phases), h.size() * 8);
    static const char* names[2][6] = {{"vm", "B1", "wgrad2", "convert", "B2", "dma"},
                                      {"B1", "dgrad2", "B2", "wgrad1", "-", "-"}};
    for (int r = 0; r < 4; ++r) {
        double sum[6] = {0}, n = 0, mhz = 0, tot = 0;
        for (int b = 0; b < grid && b < 1024; ++b) {
            for (int k = 0; k < 6; ++k) sum[k] += (double)h[b * 32 + 8 * r + k];
            n += (double)h[b * 32 + 8 * r + 7];
            mhz += (double)h[b * 32 + 8 * r + 6] / (1 << 20) * 100.0;
        }
        std::fprintf(stderr, "[phases %s wave %d] clk/frame:", name, 2 * r);
        for (int k = 0; k < 6; ++k) { std::fprintf(stderr, " %s %.0f", names[r >= 2][k], sum[k] / n); tot += sum[k] / n; }
        std::fprintf(stderr, "  total %.0f  clock %.0f MHz\n", tot, mhz / grid);
    }
}
'''
src = src.replace('namespace fi {\n', 'namespace fi {\n' + macros, 1)
k0 = src.index('__global__ __launch_bounds__(512, 2) void conv21_bwd_fr(')
k1 = src.index('int conv21_bwd_fr_launch(')
ker = src[k0:k1]


def sub(old, new, count=1):
    global ker
    assert ker.count(old) == count, (old, ker.count(old))
    ker = ker.replace(old, new)


# waves 0-3 (buckets 1..6: vm, B1, wgrad2, convert, B2, dma)
sub('''        for (int it = 0; it < nmine; ++it) {
            wait_vmcnt(issued - m_dy);  // own pieces of da2(it) landed (a1(it) is older)
            lds_barrier();  // B1: frame it's images in LDS; frame it-1's D and image consumed
''', '''        PH_DECL
        for (int it = 0; it < nmine; ++it) {
            PH(0);
            wait_vmcnt(issued - m_dy);  // own pieces of da2(it) landed (a1(it) is older)
            PH(1);
            lds_barrier();  // B1: frame it's images in LDS; frame it-1's D and image consumed
            PH(2);
''')
sub('''#pragma unroll
            for (int i = 0; i < c21::NRAW_A; ++i) {  // raw(it) -> bf16 pair-plane image (free since B1)''',
    '''            PH(3);
#pragma unroll
            for (int i = 0; i < c21::NRAW_A; ++i) {  // raw(it) -> bf16 pair-plane image (free since B1)''')
sub('''            lds_barrier();  // B2: D and the image complete; da2 image and a1 slot it&1 consumed
''', '''            PH(4);
            lds_barrier();  // B2: D and the image complete; da2 image and a1 slot it&1 consumed
            PH(5);
''')
sub('''            if (it + 2 < nmine) issued += issue_ax(it + 2, it & 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
''', '''            if (it + 2 < nmine) issued += issue_ax(it + 2, it & 1);
            PH(6);
            PH_ITER();
        }
        PH_FLUSH();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
''')
# waves 4-7 (buckets 1..4: B1, dgrad2, B2, wgrad1)
sub('''        for (int it = 0; it < nmine; ++it) {
            const int f = frame_of(it);
            lds_barrier();  // B1
''', '''        PH_DECL
        for (int it = 0; it < nmine; ++it) {
            const int f = frame_of(it);
            PH(4);
            lds_barrier();  // B1
            PH(1);
''')
sub('''            lds_barrier();  // B2: D and the image complete
            if (it + 1 < nmine) load_raw(it + 1);
''', '''            PH(2);
            lds_barrier();  // B2: D and the image complete
            PH(3);
            if (it + 1 < nmine) load_raw(it + 1);
''')
sub('''            if (__builtin_expect(it == seg_last(sg, nmine), 0)) c1_flush();
        }
''', '''            if (__builtin_expect(it == seg_last(sg, nmine), 0)) c1_flush();
            PH(4);
            PH_ITER();
        }
        PH_FLUSH();
''')
src = src[:k0] + ker + src[k1:]
old = '''                           cs2, slab1, cs1, nframes, a1_planar);
    FI_HIP_CHECK(hipGetLastError());
'''
assert src.count(old) == 1
src = src.replace(old, old + '    ph_report("conv21_bwd_fr", grid);\n')
os.makedirs(os.path.join(ROOT, "build/exp2/c21ph"), exist_ok=True)
open(os.path.join(ROOT, "build/exp2/c21ph/atari_fr.hip"), "w").write(src)
print("wrote build/exp2/c21ph/atari_fr.hip")
