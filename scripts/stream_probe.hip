// stream_probe.hip -- calibration: how fast can ONE launch move the V-trace kernel's bytes?
// Reads two (T,B,A) fp32 tensors + four (T,B) tensors and writes one (T,B,A) + three (T,B)
// tensors (= 244 B per (t,b) at A = 18, the V-trace algorithmic traffic) with plain
// 16-byte loads/stores, grid-stride, various grid sizes. Prints us/launch and GB/s, WARM
// (the same set every launch: it stays in the 256 MB Infinity Cache) and COLD (launches
// rotate over 6 disjoint sets = 600 MB, as bench.py's roofline_vtrace does), with plain and
// with non-temporal stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const f4* __restrict__ a, const f4* __restrict__ b,
                                                     f4* __restrict__ o, size_t n4,
                                                     const f4* __restrict__ s0, const f4* __restrict__ s1,
                                                     const f4* __restrict__ s2, const f4* __restrict__ s3,
                                                     f4* __restrict__ o0, f4* __restrict__ o1,
                                                     f4* __restrict__ o2, size_t m4) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) st<NT>(o + i, a[i] + b[i]);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m4; i += stride) {
        const f4 x = s0[i] + s1[i] + s2[i] + s3[i];
        st<NT>(o0 + i, x); st<NT>(o1 + i, x * 2.f); st<NT>(o2 + i, x * 3.f);
    }
}

struct Set { float *a, *b, *o, *s[4], *oo[3]; };

int main() {
    const size_t T = 100, B = 4096, A = 18;
    const size_t n = T * B * A, m = T * B;
    const int NSETS = 6;
    std::vector<Set> sets(NSETS);
    for (auto& S : sets) {
        hipMalloc(&S.a, n * 4); hipMalloc(&S.b, n * 4); hipMalloc(&S.o, n * 4);
        for (auto& p : S.s) { hipMalloc(&p, m * 4); hipMemset(p, 0, m * 4); }
        for (auto& p : S.oo) hipMalloc(&p, m * 4);
        hipMemset(S.a, 0, n * 4); hipMemset(S.b, 0, n * 4);
    }
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double bytes = 244.0 * T * B;
    for (int nt = 0; nt < 2; ++nt)
        for (int cold = 0; cold < 2; ++cold)
            for (int grid : {512, 1024, 2048, 4096, 8192}) {
                auto go = [&](int i) {
                    const Set& S = sets[cold ? i % NSETS : 0];
                    auto k = nt ? stream_kernel<true> : stream_kernel<false>;
                    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const f4*)S.a, (const f4*)S.b, (f4*)S.o, n / 4,
                                       (const f4*)S.s[0], (const f4*)S.s[1], (const f4*)S.s[2], (const f4*)S.s[3],
                                       (f4*)S.oo[0], (f4*)S.oo[1], (f4*)S.oo[2], m / 4);
                };
                for (int i = 0; i < 6; ++i) go(i);
                hipEventRecord(e0);
                for (int i = 0; i < 60; ++i) go(i);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                ms /= 60;
                printf("%s %s grid %5d: %.2f us/launch  %.0f GB/s (%.1f%% of 8 TB/s)\n", cold ? "cold" : "warm",
                       nt ? "nt-store" : "store   ", grid, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
                       100 * bytes / (ms * 1e-3) / 8e12);
            }
    return 0;
}
