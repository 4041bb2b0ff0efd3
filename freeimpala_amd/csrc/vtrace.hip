// vtrace.hip -- fused V-trace targets + IMPALA loss + analytic gradients (gfx950).
//
// Replaces nothing in the reference line-for-line: the reference learner step
// (include/freeimpala/learner.h:32-49) is sleep + random bytes. The numerics follow the
// IMPALA spec as restated in SURVEY.md 8(a) (and in oracle/impala_oracle.c, the checker):
//   log_rho = log pi(a) - log mu(a); rho = min(rho_bar, e^log_rho); c = lambda*min(c_bar, e^.)
//   acc_t = rho_t (r_t + g_t V_{t+1} - V_t) + g_t c_t acc_{t+1};  vs_t = V_t + acc_t
//   pg_adv_t = min(pg_rho_bar, e^log_rho)(r_t + g_t vs_{t+1} - V_t)
//   dL/dz = -pg_adv (onehot - pi) + ec pi (log pi - sum pi log pi);  dL/dV_t = bc (V_t - vs_t)
//
// Kernel 1 (vtrace_lds_kernel, the hot one): one 256-thread workgroup owns 16 batch
// columns for all T and walks time BACKWARDS in chunks of 16 steps. Each chunk's
// (16 t x 16 b) slices of pi/mu logits and of the action/reward/discount/value rows are
// contiguous 1 KiB-multiples in the (T,B,A)/(T,B) layouts, so they are staged into LDS
// with LDS-DMA (global_load_lds_dwordx4), three chunks in flight in a ring, counted vmcnt
// and raw s_barrier (no vmcnt(0) drains). Thread (tl, c) = (4*wave + lane/16, lane%16)
// reads its logits row conflict-free, computes the log-softmaxes, and the reverse-time
// affine recurrence acc_t = d_t + g_t acc_{t+1} is solved with a 2-step wavefront
// shuffle suffix scan over the 4 timesteps of a wave plus a 4-entry LDS combine across
// waves and a carried value across chunks. dlogits go back through LDS and leave as
// coalesced 16-byte stores. Algorithmic HBM traffic: 12A+28 bytes per (t,b).
//
// Kernel 2 (vtrace_column_kernel): one lane per column, serial over t; any A <= 64, any B.
#include "fi_common.h"
#include "kernels.h"

#include <algorithm>
#include <cmath>

namespace fi {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct VtArgs {
    int T, B, A;
    const float* __restrict__ pi;
    const float* __restrict__ mu;
    const int32_t* __restrict__ act;
    const float* __restrict__ rew;
    const float* __restrict__ disc;
    const float* __restrict__ val;
    float* vs;
    float* adv;
    float* dlog;
    float* dval;
    double* part;  // [nblk][3]
    float* sink;   // 2048 floats of scratch for masked-off stores
    fi_vtrace_hparams hp;
};

constexpr size_t kSinkFloats = 2048;

__device__ __forceinline__ void block_reduce3(double pg, double base, double ent, double* red,
                                              double* out) {
    pg = wave_sum(pg);
    base = wave_sum(base);
    ent = wave_sum(ent);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        red[w * 3 + 0] = pg;
        red[w * 3 + 1] = base;
        red[w * 3 + 2] = ent;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
        const int nw = blockDim.x >> 6;
        for (int i = 0; i < nw; ++i) s += red[i * 3 + threadIdx.x];
        out[threadIdx.x] = s;
    }
}

// ------------------------------------------------------------------------------------
// Kernel 2: one column per lane (reference-shaped, used for odd A / ragged B)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void vtrace_column_kernel(VtArgs a) {
    __shared__ double red[4 * 3];
    const int b = blockIdx.x * 256 + threadIdx.x;
    const int T = a.T, B = a.B, A = a.A;
    double pg = 0, base = 0, ent = 0;
    if (b < B) {
        float v_next = a.val[(size_t)T * B + b];
        float acc_next = 0.f;
        float vs_next = v_next;
        a.dval[(size_t)T * B + b] = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            const size_t e = (size_t)t * B + b;
            const float* zp = a.pi + e * A;
            const float* zm = a.mu + e * A;
            int at = a.act[e];
            at = at < 0 ? 0 : (at >= A ? A - 1 : at);
            float mx = -INFINITY, mm = -INFINITY;
            for (int i = 0; i < A; ++i) { mx = fmaxf(mx, zp[i]); mm = fmaxf(mm, zm[i]); }
            float sp = 0.f, sm = 0.f;
            for (int i = 0; i < A; ++i) { sp += expf(zp[i] - mx); sm += expf(zm[i] - mm); }
            const float lse = mx + logf(sp), lsem = mm + logf(sm);
            const float lpa = zp[at] - lse, lma = zm[at] - lsem;
            const float ratio = expf(lpa - lma);
            const float rho = fminf(a.hp.rho_bar, ratio);
            const float cc = a.hp.lambda_ * fminf(a.hp.c_bar, ratio);
            const float pgr = fminf(a.hp.pg_rho_bar, ratio);
            const float r = a.rew[e], g = a.disc[e], v = a.val[e];
            const float acc = rho * (r + g * v_next - v) + g * cc * acc_next;
            const float vs = v + acc;
            const float adv = pgr * (r + g * vs_next - v);
            if (a.vs) a.vs[e] = vs;
            if (a.adv) a.adv[e] = adv;
            float plogp = 0.f;
            for (int i = 0; i < A; ++i) {
                const float lp = zp[i] - lse;
                plogp += expf(lp) * lp;
            }
            float* dz = a.dlog + e * A;
            for (int i = 0; i < A; ++i) {
                const float lp = zp[i] - lse;
                const float p = expf(lp);
                dz[i] = -adv * ((i == at ? 1.f : 0.f) - p) + a.hp.entropy_cost * p * (lp - plogp);
            }
            a.dval[e] = -a.hp.baseline_cost * acc;
            pg += (double)(-adv * lpa);
            base += 0.5 * (double)acc * (double)acc;
            ent += (double)plogp;
            acc_next = acc;
            v_next = v;
            vs_next = vs;
        }
    }
    block_reduce3(pg, base, ent, red, a.part + (size_t)blockIdx.x * 3);
}

// ------------------------------------------------------------------------------------
// Kernel 1: LDS-staged reverse-time chunks, LDS-DMA ring, shuffle scan
// ------------------------------------------------------------------------------------
template <int A>
struct VtLayout {
    static constexpr int NB = 16;                      // batch columns per workgroup
    static constexpr int TC = 16;                      // timesteps per chunk
    static constexpr int ROWF = NB * A;                // floats per t-row of a logits tile
    static constexpr int ROW4 = ROWF / 4;              // float4 per t-row (= 4A)
    static constexpr int LOGB = TC * ROWF * 4;         // bytes per logits tile (= 1024*A)
    static constexpr int SCB = TC * NB * 4;            // bytes per scalar tile (= 1 KiB)
    static constexpr int SLOT = 2 * LOGB + 4 * SCB;    // pi | mu | act | rew | disc | val
    static constexpr int RING = 3;                     // chunks in flight
    static constexpr int OFF_DLOG = RING * SLOT;       // dlogits staging tile
    static constexpr int OFF_SMALL = OFF_DLOG + LOGB;  // carry/vnext/wave totals/reduce
    static constexpr int SMALL = (2 * NB + 2 * NB + 4 * NB + 4 * NB) * 4 + 4 * 3 * 8;
    static constexpr int TOTAL = OFF_SMALL + SMALL;
    static constexpr int NINSTR = 2 * A + 4;           // 1-KiB LDS-DMA pieces per chunk
    static constexpr int G = NINSTR / 4;               // per wave
    static_assert(A % 2 == 0, "fast V-trace kernel needs even A");
    static_assert(TOTAL <= 160 * 1024, "LDS budget");
};

template <int A>
__device__ __forceinline__ void vt_issue_chunk(const VtArgs& a, uint32_t lds0, int slot, int t0,
                                               int b0, int w, int lane) {
    using L = VtLayout<A>;
    const uint32_t base = lds0 + (uint32_t)(slot * L::SLOT);
#pragma unroll
    for (int i = 0; i < L::G; ++i) {
        const int j = w + 4 * i;  // wave-uniform piece index
        if (j < 2 * A) {
            const int which = j >= A ? 1 : 0;
            const int jj = j - which * A;
            const int q = jj * 64 + lane;  // float4 index inside the [TC][ROW4] tile
            const int tl = q / L::ROW4, c4 = q - tl * L::ROW4;
            const int t = max(t0 + tl, 0);
            const float* arr = which ? a.mu : a.pi;
            const float* src = arr + ((size_t)t * a.B + b0) * A + c4 * 4;
            glds16(src, base + which * L::LOGB + jj * 1024);
        } else {
            const int s = j - 2 * A;  // 0 act, 1 rew, 2 disc, 3 val
            const int tl = lane >> 2, qd = lane & 3;
            const int t = max(t0 + tl, 0);
            const char* arr = s == 0 ? (const char*)a.act
                              : s == 1 ? (const char*)a.rew
                              : s == 2 ? (const char*)a.disc
                                       : (const char*)a.val;
            const char* src = arr + ((size_t)t * a.B + b0) * 4 + qd * 16;
            glds16(src, base + 2 * L::LOGB + s * L::SCB);
        }
    }
}

template <int A>
__global__ __launch_bounds__(256, 1) void vtrace_lds_kernel(VtArgs a) {
    using L = VtLayout<A>;
    __shared__ __attribute__((aligned(16))) char smem[L::TOTAL];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = wave_id();
    const int cb = xcd_remap(blockIdx.x, gridDim.x);
    const int b0 = cb * L::NB;
    const int T = a.T, B = a.B;
    const int nchunks = (T + L::TC - 1) / L::TC;
    const int tl = w * 4 + (lane >> 4), c = lane & 15;
    const int b = b0 + c;
    const uint32_t lds0 = lds_addr(smem);

    float* carry = (float*)(smem + L::OFF_SMALL);  // [2][NB]
    float* vnext = carry + 2 * L::NB;              // [2][NB]
    float* totd = vnext + 2 * L::NB;               // [4][NB]
    float* totg = totd + 4 * L::NB;                // [4][NB]
    double* red = (double*)(totg + 4 * L::NB);     // [4][3]
    float* dstage = (float*)(smem + L::OFF_DLOG);

    if (tid < L::NB) {
        carry[tid] = 0.f;
        vnext[tid] = a.val[(size_t)T * B + b0 + tid];  // bootstrap V_T
        a.dval[(size_t)T * B + b0 + tid] = 0.f;
    }

    // prologue: up to RING chunks in flight; marks = VMEM ops issued after each chunk
    int issued = 0, m0 = 0, m1 = 0, m2 = 0;
    vt_issue_chunk<A>(a, lds0, 0, T - L::TC, b0, w, lane);
    issued += L::G;
    m0 = issued;
    if (nchunks > 1) {
        vt_issue_chunk<A>(a, lds0, 1, T - 2 * L::TC, b0, w, lane);
        issued += L::G;
        m1 = issued;
    }
    if (nchunks > 2) {
        vt_issue_chunk<A>(a, lds0, 2, T - 3 * L::TC, b0, w, lane);
        issued += L::G;
        m2 = issued;
    }
    const int n_dst = (A - w + 3) / 4;  // dlogits float4 stores per wave per chunk
    const fi_vtrace_hparams hp = a.hp;

    float pg = 0.f, base = 0.f, ent = 0.f;
    for (int k = 0; k < nchunks; ++k) {
        const int slot = k % 3;
        const int t0 = T - L::TC * (k + 1);
        wait_vmcnt(issued - m0);
        lds_barrier();  // B1: chunk k landed for every wave

        const char* sl = smem + slot * L::SLOT;
        const float* zpi = (const float*)sl + tl * L::ROWF + c * A;
        const float* zmu = (const float*)(sl + L::LOGB) + tl * L::ROWF + c * A;
        const int* sact = (const int*)(sl + 2 * L::LOGB);
        const float* srew = (const float*)(sl + 2 * L::LOGB + L::SCB);
        const float* sdisc = (const float*)(sl + 2 * L::LOGB + 2 * L::SCB);
        const float* sval = (const float*)(sl + 2 * L::LOGB + 3 * L::SCB);
        const int t = t0 + tl;
        const bool valid = t >= 0;

        float zp[A], zm[A];
#pragma unroll
        for (int i = 0; i < A; i += 2) {
            const float2 p2 = *(const float2*)(zpi + i);
            const float2 m2v = *(const float2*)(zmu + i);
            zp[i] = p2.x; zp[i + 1] = p2.y;
            zm[i] = m2v.x; zm[i + 1] = m2v.y;
        }
        int at = sact[tl * L::NB + c];
        at = at < 0 ? 0 : (at >= A ? A - 1 : at);
        const float r = srew[tl * L::NB + c];
        const float g = sdisc[tl * L::NB + c];
        const float v = sval[tl * L::NB + c];
        const float vn = (tl == L::TC - 1) ? vnext[(k & 1) * L::NB + c] : sval[(tl + 1) * L::NB + c];

        float mx = zp[0], mm = zm[0];
#pragma unroll
        for (int i = 1; i < A; ++i) { mx = fmaxf(mx, zp[i]); mm = fmaxf(mm, zm[i]); }
        float sp = 0.f, sm = 0.f;
#pragma unroll
        for (int i = 0; i < A; ++i) { sp += expf(zp[i] - mx); sm += expf(zm[i] - mm); }
        const float lse = mx + logf(sp), lsem = mm + logf(sm);
        float zpa = 0.f, zma = 0.f;
#pragma unroll
        for (int i = 0; i < A; ++i) {
            zpa = (i == at) ? zp[i] : zpa;
            zma = (i == at) ? zm[i] : zma;
        }
        const float lpa = zpa - lse, lma = zma - lsem;
        const float ratio = expf(lpa - lma);
        const float rho = fminf(hp.rho_bar, ratio);
        const float cc = hp.lambda_ * fminf(hp.c_bar, ratio);
        const float pgr = fminf(hp.pg_rho_bar, ratio);
        float d = valid ? rho * (r + g * vn - v) : 0.f;
        float gg = valid ? g * cc : 1.f;

        // inclusive suffix composition over the wave's 4 timesteps (lanes +16, +32)
        {
            const float d2 = __shfl_down(d, 16, 64), g2 = __shfl_down(gg, 16, 64);
            if (lane < 48) { d = d + gg * d2; gg = gg * g2; }
        }
        {
            const float d2 = __shfl_down(d, 32, 64), g2 = __shfl_down(gg, 32, 64);
            if (lane < 32) { d = d + gg * d2; gg = gg * g2; }
        }
        if (lane < 16) {
            totd[w * L::NB + c] = d;
            totg[w * L::NB + c] = gg;
        }
        lds_barrier();  // B2: wave totals visible

        float acc_in = carry[(k & 1) * L::NB + c];  // acc at t0 + 16
        for (int w2 = 3; w2 > w; --w2) acc_in = totd[w2 * L::NB + c] + totg[w2 * L::NB + c] * acc_in;
        const float acc = d + gg * acc_in;
        const float acc_up = __shfl_down(acc, 16, 64);
        const float acc_nx = (lane >= 48) ? acc_in : acc_up;
        const float vs_t = v + acc;
        const float vs_n = vn + acc_nx;
        const float adv = pgr * (r + g * vs_n - v);
        const float dv = -hp.baseline_cost * acc;

        float plogp = 0.f;
#pragma unroll
        for (int i = 0; i < A; ++i) {
            const float lp = zp[i] - lse;
            plogp += expf(lp) * lp;
        }
        float* dz = dstage + tl * L::ROWF + c * A;
#pragma unroll
        for (int i = 0; i < A; i += 2) {
            float2 o;
            {
                const float lp = zp[i] - lse, p = expf(lp);
                o.x = -adv * ((i == at ? 1.f : 0.f) - p) + hp.entropy_cost * p * (lp - plogp);
            }
            {
                const float lp = zp[i + 1] - lse, p = expf(lp);
                o.y = -adv * ((i + 1 == at ? 1.f : 0.f) - p) + hp.entropy_cost * p * (lp - plogp);
            }
            *(float2*)(dz + i) = o;
        }
        if (valid) {
            pg += -adv * lpa;
            base += 0.5f * acc * acc;
            ent += plogp;
        }
        {  // always-executed stores (masked rows go to the sink) keep vmcnt counts exact
            const size_t e = (size_t)(valid ? t : 0) * B + b;
            float* pvs = valid ? a.vs + e : a.sink + tid;
            float* padv = valid ? a.adv + e : a.sink + 256 + tid;
            float* pdv = valid ? a.dval + e : a.sink + 512 + tid;
            __builtin_nontemporal_store(vs_t, pvs);
            __builtin_nontemporal_store(adv, padv);
            __builtin_nontemporal_store(dv, pdv);
            issued += 3;
        }
        if (tl == 0) {
            carry[((k + 1) & 1) * L::NB + c] = acc;
            vnext[((k + 1) & 1) * L::NB + c] = v;
        }
        lds_barrier();  // B3: dlogits staged; ring slot k%3 is free

        // dlogits: LDS -> coalesced 16-byte stores (one (t, 16 columns) row = 4A float4)
        for (int q = tid; q < 64 * A; q += 256) {
            const int rtl = q / L::ROW4, c4 = q - rtl * L::ROW4;
            const int rt = t0 + rtl;
            const f32x4 val = ((const f32x4*)dstage)[q];
            f32x4* dst = rt >= 0 ? (f32x4*)(a.dlog + ((size_t)rt * B + b0) * A) + c4
                                 : (f32x4*)(a.sink + 1024) + tid;
            __builtin_nontemporal_store(val, dst);
        }
        issued += n_dst;

        int m3 = 0;
        if (k + 3 < nchunks) {
            vt_issue_chunk<A>(a, lds0, slot, T - L::TC * (k + 4), b0, w, lane);
            issued += L::G;
            m3 = issued;
        }
        m0 = m1;
        m1 = m2;
        m2 = m3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    block_reduce3((double)pg, (double)base, (double)ent, red, a.part + (size_t)blockIdx.x * 3);
}

__global__ __launch_bounds__(256) void vtrace_finalize_kernel(const double* __restrict__ part,
                                                              int nblk, double* losses) {
    __shared__ double red[4 * 3];
    double s0 = 0, s1 = 0, s2 = 0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        s0 += part[(size_t)i * 3];
        s1 += part[(size_t)i * 3 + 1];
        s2 += part[(size_t)i * 3 + 2];
    }
    block_reduce3(s0, s1, s2, red, losses);
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static size_t vt_nblk_max(int B) { return (size_t)std::max((B + 15) / 16, (B + 255) / 256); }

size_t vtrace_workspace_bytes(int T, int B, int A) {
    (void)T;
    (void)A;
    return kSinkFloats * sizeof(float) + ((vt_nblk_max(B) * 3 * sizeof(double) + 255) & ~(size_t)255);
}

template <int A>
static void launch_lds(const VtArgs& a, int nblk, hipStream_t s) {
    hipLaunchKernelGGL(vtrace_lds_kernel<A>, dim3(nblk), dim3(256), 0, s, a);
}

static bool lds_supported(int A, int B) { return B % 16 == 0 && A % 2 == 0 && A >= 2 && A <= 20; }

int vtrace_launch(int variant, int T, int B, int A, const float* pi, const float* mu,
                  const int32_t* act, const float* rew, const float* disc, const float* val,
                  const fi_vtrace_hparams& hp, float* vs, float* adv, float* dlog, float* dval,
                  double* losses, void* ws, size_t ws_bytes, hipStream_t stream, bool finalize,
                  int* nblk_out) {
    FI_REQUIRE(T >= 1 && B >= 1 && A >= 1 && A <= 64, "vtrace: bad shape");
    FI_REQUIRE(pi && mu && act && rew && disc && val && dlog && dval && losses && ws,
               "vtrace: null pointer");
    FI_REQUIRE(ws_bytes >= vtrace_workspace_bytes(T, B, A), "vtrace: workspace too small");
    VtArgs a;
    a.T = T; a.B = B; a.A = A;
    a.pi = pi; a.mu = mu; a.act = act; a.rew = rew; a.disc = disc; a.val = val;
    a.vs = vs; a.adv = adv; a.dlog = dlog; a.dval = dval;
    a.sink = (float*)ws;
    a.part = (double*)((char*)ws + kSinkFloats * sizeof(float));
    a.hp = hp;
    bool use_lds = variant == 1 || (variant == 0 && lds_supported(A, B));
    FI_REQUIRE(!(variant == 1 && !lds_supported(A, B)), "vtrace: LDS kernel needs B%16==0, even A<=20");
    int nblk;
    if (use_lds) {
        FI_REQUIRE(vs && adv, "vtrace: LDS kernel writes vs and pg_adv (non-null)");
        FI_REQUIRE(((uintptr_t)pi | (uintptr_t)mu | (uintptr_t)dlog) % 16 == 0 &&
                   ((uintptr_t)act | (uintptr_t)rew | (uintptr_t)disc | (uintptr_t)val) % 16 == 0,
                   "vtrace: LDS kernel needs 16-byte aligned tensors");
        nblk = B / 16;
        switch (A) {
            case 2: launch_lds<2>(a, nblk, stream); break;
            case 4: launch_lds<4>(a, nblk, stream); break;
            case 6: launch_lds<6>(a, nblk, stream); break;
            case 8: launch_lds<8>(a, nblk, stream); break;
            case 10: launch_lds<10>(a, nblk, stream); break;
            case 12: launch_lds<12>(a, nblk, stream); break;
            case 14: launch_lds<14>(a, nblk, stream); break;
            case 16: launch_lds<16>(a, nblk, stream); break;
            case 18: launch_lds<18>(a, nblk, stream); break;
            case 20: launch_lds<20>(a, nblk, stream); break;
            default: return fail(FI_ERR_UNSUPPORTED, "vtrace: A not instantiated");
        }
    } else {
        nblk = (B + 255) / 256;
        hipLaunchKernelGGL(vtrace_column_kernel, dim3(nblk), dim3(256), 0, stream, a);
    }
    FI_HIP_CHECK(hipGetLastError());
    if (nblk_out) *nblk_out = nblk;
    if (finalize) return vtrace_finalize_launch(ws, nblk, losses, stream);
    return FI_OK;
}

int vtrace_finalize_launch(void* ws, int nblk, double* losses, hipStream_t stream) {
    const double* part = (const double*)((char*)ws + kSinkFloats * sizeof(float));
    hipLaunchKernelGGL(vtrace_finalize_kernel, dim3(1), dim3(256), 0, stream, part, nblk, losses);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

}  // namespace fi

extern "C" size_t fi_vtrace_workspace_bytes(int T, int B, int A) {
    return fi::vtrace_workspace_bytes(T, B, A);
}

extern "C" int fi_vtrace_loss_fp32_variant(int variant, int T, int B, int A, const float* pi,
                                           const float* mu, const int32_t* act, const float* rew,
                                           const float* disc, const float* val,
                                           const fi_vtrace_hparams* hp, float* vs, float* adv,
                                           float* dlog, float* dval, double* losses, void* ws,
                                           size_t ws_bytes, void* stream) {
    if (!hp) return fi::fail(FI_ERR_INVALID, "vtrace: null hparams");
    return fi::vtrace_launch(variant, T, B, A, pi, mu, act, rew, disc, val, *hp, vs, adv, dlog,
                             dval, losses, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int fi_vtrace_loss_fp32(int T, int B, int A, const float* pi, const float* mu,
                                   const int32_t* act, const float* rew, const float* disc,
                                   const float* val, const fi_vtrace_hparams* hp, float* vs,
                                   float* adv, float* dlog, float* dval, double* losses, void* ws,
                                   size_t ws_bytes, void* stream) {
    return fi_vtrace_loss_fp32_variant(0, T, B, A, pi, mu, act, rew, disc, val, hp, vs, adv, dlog,
                                       dval, losses, ws, ws_bytes, stream);
}
