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
// Kernel 1 (vtrace_lds_kernel<A>, the hot one): one 256-thread workgroup (4 waves) owns
// 8 batch columns for all T and walks time BACKWARDS in chunks of 32 steps; wave w owns
// rows 8w..8w+7 of a chunk (lane = 8*row + column). Each chunk's pi/mu logits tiles
// (32 rows x 8 columns x A floats) and the action/reward/discount/value tiles are
// contiguous pieces of the (T,B,A)/(T,B) layouts and arrive by LDS-DMA
// (buffer_load_dwordx4 ... nt lds: read once, so not kept in the caches) into a 2-slot ring
// (81,920 B at A=18, two workgroups per CU); the next chunk is issued right after the landing
// barrier, with counted vmcnt waits.
// Per element: packed-fp32 softmax statistics, one v_exp_f32 per logit. The reverse
// recurrence acc_t = d_t + g_t c_t acc_{t+1} is an affine suffix scan: a 3-step butterfly
// inside the wave (DPP row_ror:8, v_permlane16_swap, v_permlane32_swap: no LDS round trip),
// a 4-entry combine across waves through LDS and a carry kept in registers across chunks.
// dlogits are written over the wave's own pi rows in LDS and leave as full-wave 16-byte
// stores; the loss partials are reduced in-wave by DPP/permlane and written per workgroup
// (summed in a fixed order by the grad-norm kernel). Algorithmic HBM traffic: 12A+28 bytes
// per (t,b). Requires B % 8 == 0, A in {2..64 compiled set} and T*B*A*4 < 2^31 (32-bit
// buffer offsets; vtrace_launch falls back to kernel 2 above that).
//
// Kernel 2 (vtrace_column_kernel): one lane per column, serial over t; any A <= 64, any B.
#include "fi_common.h"
#include "kernels.h"

#include <atomic>
#include <algorithm>
#include <cmath>
#include <mutex>

namespace fi {

#define VT_EXP(x) __expf(x)
#define VT_LOG(x) __logf(x)
#define VT_EXP2(x) __builtin_amdgcn_exp2f(x)
#define VT_LOG2(x) __builtin_amdgcn_logf(x)
#ifdef FI_VT_NT
#define VT_ST(v, p) __builtin_nontemporal_store((v), (p))
#else
#define VT_ST(v, p) (*(p) = (v))
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// max of three through v_max3_f32 directly: fmaxf() under the kernels' IEEE mode makes hipcc
// quiet every LDS-loaded operand first (one v_max_f32 x, x, x each), doubling the row-max cost
__device__ __forceinline__ float vt_max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

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
    int* bad;      // count of actions outside [0, A) (those rows use a clamped action)
    fi_vtrace_hparams hp;
};

constexpr size_t kSinkFloats = 2048;

// wave-wide double sum in VALU cross-lane moves (no ds_bpermute round trips in the
// workgroup's tail): rotations 8, 4, 2, 1 inside each 16-lane row by DPP, then the row pairs
// and halves by gfx950's v_permlane16_swap / v_permlane32_swap. The summation order is
// fixed, so the result is deterministic; lane 0 holds the total the callers use.
template <int CTRL>
__device__ __forceinline__ double vt_dpp_d(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int S>
__device__ __forceinline__ double vt_xor_d(double v, int lane) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    unsigned rlo, rhi;
    if constexpr (S == 16) {
        const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        rlo = (lane & 16) ? a[0] : a[1];
        rhi = (lane & 16) ? b[0] : b[1];
    } else {
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        rlo = (lane & 32) ? a[0] : a[1];
        rhi = (lane & 32) ? b[0] : b[1];
    }
    return __longlong_as_double((long long)(((unsigned long long)rhi << 32) | rlo));
}
__device__ __forceinline__ double vt_wave_sum(double v) {
    const int lane = threadIdx.x & 63;
    v += vt_dpp_d<0x128>(v);  // row_ror:8
    v += vt_dpp_d<0x124>(v);  // row_ror:4
    v += vt_dpp_d<0x122>(v);  // row_ror:2
    v += vt_dpp_d<0x121>(v);  // row_ror:1
    v += vt_xor_d<16>(v, lane);
    v += vt_xor_d<32>(v, lane);
    return v;
}

__device__ __forceinline__ void block_reduce3(double pg, double base, double ent, double* red,
                                              double* out) {
    pg = vt_wave_sum(pg);
    base = vt_wave_sum(base);
    ent = vt_wave_sum(ent);
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
            if ((unsigned)at >= (unsigned)A) atomicAdd(a.bad, 1);
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
// Kernel 1: LDS-staged reverse-time chunks, LDS-DMA double buffer, shuffle scan.
// Workgroup = 8 batch columns x all T, 256 threads, two workgroups per CU (81,920 B of LDS
// each) so one workgroup's arithmetic overlaps the other's DMA waits. A chunk is 32
// timesteps; wave w owns rows 8w..8w+7 of it (lane = 8 * row + column), reads only its own
// rows of the logits tiles, writes its dlogits back over its own pi rows and its scan total
// over its own mu rows, and stores its own dlogits rows -- so a chunk needs two barriers
// (data landed, wave totals visible). Pieces of the partial (earliest) chunk that hold no
// valid timestep are not fetched.
// ------------------------------------------------------------------------------------
#ifndef FI_VT_NW
#define FI_VT_NW 4
#endif
template <int A>
struct VtLayout {
    static constexpr int NW = FI_VT_NW;                // waves per workgroup (8 rows each)
    static constexpr int NB = 8;                       // batch columns per workgroup
    static constexpr int TC = 8 * NW;                  // timesteps per chunk
    static constexpr int ROWF = NB * A;                // floats per t-row of a logits tile
    static constexpr int ROWB = ROWF * 4;              // bytes per t-row (= 32A)
    static constexpr int LOGB = TC * ROWB;             // bytes per logits tile (= 256*NW*A)
    static constexpr int SCB = TC * NB * 4;            // bytes per scalar tile (= 256*NW)
    static constexpr int PT = LOGB / 1024;             // 1-KiB pieces per logits tile
    static constexpr int MUB = LOGB;
    static constexpr int TOTB = 0;
    static constexpr int GLOG = 2 * PT / NW;           // logits pieces per wave per chunk
    static constexpr int SCO = LOGB + MUB;             // scalar tiles' offset in a slot
    static constexpr int SLOT = SCO + 4 * SCB + TOTB;  // pi | mu | act | rew | disc | val [| tot]
    static constexpr int RING = 2;
    static constexpr int TOTAL = RING * SLOT;
    static constexpr int WPS0 = (163840 / TOTAL) * NW / 4;  // waves per SIMD the LDS allows
    static constexpr int WPS = WPS0 < 1 ? 1 : (WPS0 > 8 ? 8 : WPS0);
    static_assert(A % 2 == 0, "fast V-trace kernel needs even A");
    static_assert((NW == 2 || NW == 4) && LOGB % 1024 == 0 && (2 * PT) % NW == 0 && SCB == 256 * NW, "tiling");
    static_assert(TOTAL <= 160 * 1024, "LDS budget");
};

// queue chunk (rows t0 .. t0+31) into ring slot `slot`; returns the pieces this wave issued
// (pieces I0 <= i < I1 of this wave's list: logits pieces 0..GLOG-1, then its scalar piece;
// the list is issued in groups between arithmetic so the TA drains between them)
struct VtRsrc {  // buffer descriptors of the six input tensors (built once per workgroup)
    fi_i32x4 pi, mu, act, rew, disc, val;
};
__device__ __forceinline__ VtRsrc vt_rsrc(const VtArgs& a) {
    const uint32_t lbytes = (uint32_t)a.T * a.B * a.A * 4, sbytes = (uint32_t)a.T * a.B * 4;
    return VtRsrc{make_rsrc(a.pi, lbytes), make_rsrc(a.mu, lbytes), make_rsrc(a.act, sbytes),
                  make_rsrc(a.rew, sbytes), make_rsrc(a.disc, sbytes), make_rsrc(a.val, sbytes + a.B * 4)};
}

template <int A, int I0, int I1>
__device__ __forceinline__ int vt_issue_chunk(const VtArgs& a, const VtRsrc& rs, uint32_t lds0, int slot,
                                              int t0, int b0, int w, int lane) {
    using L = VtLayout<A>;
    const uint32_t base = lds0 + (uint32_t)(slot * L::SLOT);
    const int first_row = t0 < 0 ? -t0 : 0;  // rows above hold t < 0: not needed
    int n = 0;
#pragma unroll
    for (int i = I0; i < (I1 < L::GLOG ? I1 : L::GLOG); ++i) {
        const int j = w + L::NW * i;  // wave-uniform piece index: pi (0..PT-1), mu (PT..2PT-1)
        const int jj = j < L::PT ? j : j - L::PT;
        const int last_row = (jj * 1024 + 1023) / L::ROWB;
        if (last_row < first_row) continue;
        const int q = jj * 1024 + 16 * lane;  // byte inside the tile
        const int tl = q / L::ROWB, cb = q - tl * L::ROWB;
        const int t = max(t0 + tl, 0);
        // 32-bit buffer offsets (a (T, B, A) fp32 tensor is far below 4 GiB): no 64-bit
        // address arithmetic per piece
        blds16_nt(j < L::PT ? rs.pi : rs.mu, (uint32_t)((t * a.B + b0) * A * 4 + cb),
               base + (j < L::PT ? 0 : L::LOGB) + jj * 1024);
        ++n;
    }
    if (I1 > L::GLOG) {  // scalar tiles (TC rows x 8 columns x 4 B): wave w's piece holds 4/NW of them,
       // lane -> (tile, row, 16-B half of the row)
        constexpr int LPT = 16 * L::NW;  // lanes per tile
        const int s = w * (4 / L::NW) + lane / LPT;
        const int t = max(t0 + ((lane % LPT) >> 1), 0);
        // the piece's 4/NW tiles come from up to 4 tensors: one descriptor per tile, lanes select
        const uint32_t off = (uint32_t)((t * a.B + b0) * 4 + (lane & 1) * 16);
        if constexpr (L::NW == 4) {
            blds16_nt(w == 0 ? rs.act : w == 1 ? rs.rew : w == 2 ? rs.disc : rs.val, off, base + L::SCO + w * 1024);
        } else {
            const char* arr = s == 0 ? (const char*)a.act
                              : s == 1 ? (const char*)a.rew
                              : s == 2 ? (const char*)a.disc
                                       : (const char*)a.val;
            glds16(arr + ((size_t)t * a.B + b0) * 4 + (lane & 1) * 16, base + L::SCO + w * 1024);
        }
        ++n;
    }
    return n;
}

// v from lane ^ S, in VALU cross-lane ops (no LDS round trip): S = 8 by DPP row_ror:8 inside
// each 16-lane row, S = 16 / 32 by gfx950's v_permlane16_swap / v_permlane32_swap
template <int S>
__device__ __forceinline__ float vt_xor(float v, int lane) {
    const unsigned u = __float_as_uint(v);
    if constexpr (S == 8) {
        return __uint_as_float(__builtin_amdgcn_update_dpp(0u, u, 0x128, 0xf, 0xf, false));
    } else if constexpr (S == 16) {
        const auto q = __builtin_amdgcn_permlane16_swap(u, u, false, false);
        return __uint_as_float((lane & 16) ? q[0] : q[1]);
    } else {
        const auto q = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        return __uint_as_float((lane & 32) ? q[0] : q[1]);
    }
}
template <int S>
__device__ __forceinline__ void vt_xscan_step(float& sd, float& sg, float& ed, float& eg, int lane) {
    const float pd = vt_xor<S>(sd, lane), pg = vt_xor<S>(sg, lane);
    const bool later = (lane & S) == 0;  // partner segment holds later rows
    ed = later ? ed + eg * pd : ed;
    eg = later ? eg * pg : eg;
    sd = later ? sd + sg * pd : pd + pg * sd;
    sg = sg * pg;
}

template <int A>
__global__ __launch_bounds__(64 * VtLayout<A>::NW, VtLayout<A>::WPS) void vtrace_lds_kernel(VtArgs a) {
    using L = VtLayout<A>;
    __shared__ __attribute__((aligned(16))) char smem[L::TOTAL];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = wave_id();
    const int cb = xcd_remap(blockIdx.x, gridDim.x);
    const int b0 = cb * L::NB;
    const int T = a.T, B = a.B;
    const int nchunks = (T + L::TC - 1) / L::TC;
    const int r = lane >> 3, c = lane & 7;
    const int tl = 8 * w + r;
    const int b = b0 + c;
    const uint32_t lds0 = lds_addr(smem);

    float vnext = a.val[(size_t)T * B + b];  // V at the row after the chunk (bootstrap first)
    float carry = 0.f;                       // acc at the row after the chunk
    if (tid < L::NB) a.dval[(size_t)T * B + b0 + tid] = 0.f;

    constexpr int NP = L::GLOG + 1, G1 = NP / 3, G2 = 2 * NP / 3;  // issue groups
    const VtRsrc rs = vt_rsrc(a);
    int issued = vt_issue_chunk<A, 0, NP>(a, rs, lds0, 0, T - L::TC, b0, w, lane);
    int mark = issued;  // VMEM ops issued once the chunk being waited for was queued
    const fi_vtrace_hparams hp = a.hp;

    float pg = 0.f, base = 0.f, ent = 0.f;
#define VT_STAMP()
    for (int k = 0; k < nchunks; ++k) {
        const int slot = k & 1;
        const int t0 = T - L::TC * (k + 1);
        wait_vmcnt(issued - mark);
        lds_barrier();  // B1: chunk k landed for every wave; slot (k+1)&1 fully consumed
        VT_STAMP();
        const bool more = k + 1 < nchunks;
        if (more) issued += vt_issue_chunk<A, 0, G1>(a, rs, lds0, slot ^ 1, t0 - L::TC, b0, w, lane);
        VT_STAMP();
        char* sl = smem + slot * L::SLOT;
        float* zpi = (float*)sl + tl * L::ROWF + c * A;
        float* zmu = (float*)(sl + L::LOGB) + tl * L::ROWF + c * A;
        const int* sact = (const int*)(sl + L::SCO);
        const float* srew = (const float*)(sl + L::SCO + L::SCB);
        const float* sdisc = (const float*)(sl + L::SCO + 2 * L::SCB);
        const float* sval = (const float*)(sl + L::SCO + 3 * L::SCB);
        const int t = t0 + tl;
        const bool valid = t >= 0;

        // packed-fp32 softmax statistics: e_i = 2^(z_i log2e - max log2e) (one v_pk_fma +
        // one v_exp_f32 per logit), pi_i = e_i / sum e, H = sum pi log pi = (sum e z)/sum e - lse
        constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
        f32x2 zp2[A / 2], zm2[A / 2];
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            zp2[i] = *(const f32x2*)(zpi + 2 * i);
            zm2[i] = *(const f32x2*)(zmu + 2 * i);
        }
        int at = sact[tl * L::NB + c];
        if (valid && (unsigned)at >= (unsigned)A) atomicAdd(a.bad, 1);
        at = at < 0 ? 0 : (at >= A ? A - 1 : at);
        const float zpa = zpi[at], zma = zmu[at];
        const float rw = srew[tl * L::NB + c];
        const float g = sdisc[tl * L::NB + c];
        const float v = sval[tl * L::NB + c];
        const float vn = (tl == L::TC - 1) ? vnext : sval[(tl + 1) * L::NB + c];
        const float vrow0 = sval[c];  // V at this chunk's first row: next chunk's vnext

        float mx = vt_max3(zp2[0].x, zp2[0].y, zp2[0].y), mm = vt_max3(zm2[0].x, zm2[0].y, zm2[0].y);
#pragma unroll
        for (int i = 1; i < A / 2; ++i) {
            mx = vt_max3(mx, zp2[i].x, zp2[i].y);
            mm = vt_max3(mm, zm2[i].x, zm2[i].y);
        }
        const f32x2 nmx = {-mx * L2E, -mx * L2E}, nmm = {-mm * L2E, -mm * L2E};
        f32x2 e2[A / 2];
        f32x2 sp2 = {0.f, 0.f}, sm2 = {0.f, 0.f}, sz2 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            const f32x2 ap = zp2[i] * L2E + nmx;
            const f32x2 am = zm2[i] * L2E + nmm;
            e2[i] = f32x2{VT_EXP2(ap.x), VT_EXP2(ap.y)};
            sp2 += e2[i];
            sz2 += e2[i] * zp2[i];
            sm2 += f32x2{VT_EXP2(am.x), VT_EXP2(am.y)};
        }
        if (more) issued += vt_issue_chunk<A, G1, G2>(a, rs, lds0, slot ^ 1, t0 - L::TC, b0, w, lane);
        const float sp = sp2.x + sp2.y, sm = sm2.x + sm2.y;
        const float lse = mx + VT_LOG2(sp) * LN2, lsem = mm + VT_LOG2(sm) * LN2;
        const float inv = __builtin_amdgcn_rcpf(sp);
        const float plogp = (sz2.x + sz2.y) * inv - lse;
        const float lpa = zpa - lse, lma = zma - lsem;
        const float ratio = VT_EXP(lpa - lma);
        const float rho = fminf(hp.rho_bar, ratio);
        const float cc = hp.lambda_ * fminf(hp.c_bar, ratio);
        const float pgr = fminf(hp.pg_rho_bar, ratio);
        float d = valid ? rho * (rw + g * vn - v) : 0.f;
        float gg = valid ? g * cc : 1.f;

        // butterfly over the wave's 8 rows (lane ^ 8, ^ 16, ^ 32): (sd, sg) = the composition
        // of the lane's current row segment, (ed, eg) = the composition of the rows after this
        // one inside it; at the end (sd, sg) is the wave total in every row
        const float d_own = d, g_own = gg;
        float ed = 0.f, eg = 1.f;
        vt_xscan_step<8>(d, gg, ed, eg, lane);
        vt_xscan_step<16>(d, gg, ed, eg, lane);
        vt_xscan_step<32>(d, gg, ed, eg, lane);
        if (more) issued += vt_issue_chunk<A, G2, NP>(a, rs, lds0, slot ^ 1, t0 - L::TC, b0, w, lane);
        mark = issued;  // the wait for chunk k+1 ignores the stores issued after this point
        // wave total -> this wave's own first mu row (no other wave reads it)
        float* tot = (float*)(sl + L::LOGB) + (8 * w) * L::ROWF;
        if (lane < 8) {
            tot[c] = d;
            tot[8 + c] = gg;
        }
        lds_barrier();  // B2: wave totals visible
        VT_STAMP();

        float acc_in = carry;  // acc at row 8(w+1): compose the later waves onto the carry
        float carry_new = carry;
#pragma unroll
        for (int w2 = L::NW - 1; w2 >= 0; --w2) {
            const float* t2 = (const float*)(sl + L::LOGB) + (8 * w2) * L::ROWF;
            carry_new = t2[c] + t2[8 + c] * carry_new;
            if (w2 == w + 1) acc_in = carry_new;
        }
        if (w == L::NW - 1) acc_in = carry;
        const float acc_nx = ed + eg * acc_in;
        const float acc = d_own + g_own * acc_nx;
        const float vs_t = v + acc;
        const float vs_n = vn + acc_nx;
        const float adv = pgr * (rw + g * vs_n - v);
        const float dv = -hp.baseline_cost * acc;
        carry = carry_new;
        vnext = vrow0;

        // dlogits over this wave's own pi rows:
        //   dz_i = pi_i (adv + ec (log pi_i - H)) - adv [i = a_t] = e_i (alpha + beta z_i) - adv [i = a_t]
        {
            const float ec = hp.entropy_cost;
            const float al = inv * (adv - ec * (plogp + lse)), be = inv * ec;
            const f32x2 al2 = {al, al};
#pragma unroll
            for (int i = 0; i < A / 2; ++i) *(f32x2*)(zpi + 2 * i) = e2[i] * (zp2[i] * be + al2);
            zpi[at] -= adv;
        }
        if (valid) {
            pg += -adv * lpa;
            base += 0.5f * acc * acc;
            ent += plogp;
        }
        // Stores. Every chunk but the last (the only one holding t < 0) stores with the full
        // wave, so the per-wave VMEM count used by the next chunk's wait is exact; the last
        // chunk masks freely (nothing waits on its count). Rows: vs/pg_adv/dvalue 32 B per
        // t-row of the block, merged with the neighbouring blocks' segments in L2.
        if (valid) {
            const size_t e = (size_t)t * B + b;
            VT_ST(vs_t, a.vs + e);
            VT_ST(adv, a.adv + e);
            VT_ST(dv, a.dval + e);
        }
        issued += 3;
        {  // this wave's 8 dlogits rows (8 * 2A float4 = 4 full-wave x4 stores + one x2)
            const float* srcf = (const float*)sl + (8 * w) * L::ROWF;
            float* dst0 = a.dlog + ((size_t)(t0 + 8 * w) * B + b0) * A;  // row stride B*A
            constexpr int N4 = 8 * L::ROWF / 4, NF4 = N4 / 64;         // 288, 4 (A = 18)
            constexpr int R4 = L::ROWF / 4;                            // float4 per row
#pragma unroll
            for (int i = 0; i < NF4; ++i) {
                const int q = i * 64 + lane, rr = q / R4, c4 = q - rr * R4;
                if (t0 + 8 * w + rr >= 0)
                    VT_ST(((const f32x4*)srcf)[q], (f32x4*)(dst0 + (size_t)rr * B * A) + c4);
            }
            issued += NF4;
            constexpr int REM2 = (N4 - NF4 * 64) * 2;  // remaining float2 (0..126)
            if constexpr (REM2 > 0) {
#pragma unroll
                for (int i = 0; i < (REM2 + 63) / 64; ++i) {
                    const int q2 = NF4 * 128 + i * 64 + lane;  // float2 index
                    const int rr = q2 / (2 * R4), c2 = q2 - rr * 2 * R4;
                    if (i * 64 + lane < REM2 && t0 + 8 * w + rr >= 0)
                        VT_ST(((const f32x2*)srcf)[q2], (f32x2*)(dst0 + (size_t)rr * B * A) + c2);
                }
                issued += (REM2 + 63) / 64;
            }
        }
        VT_STAMP();
    }
    // no vmcnt(0) here: the last chunk issues no LDS-DMA (only global stores are in flight),
    // so the loss-partial reduction below can overlap the store drain
    VT_STAMP();
    __syncthreads();
    // per-workgroup loss partials; summed in a fixed order by vtrace_finalize_kernel or, in
    // the learner step, by the gradient-norm kernel that runs anyway (no extra launch, no
    // serial tail at the end of this kernel)
    block_reduce3((double)pg, (double)base, (double)ent, (double*)smem, a.part + (size_t)blockIdx.x * 3);
}

// ------------------------------------------------------------------------------------
// Kernel 4 (vtrace_stream_kernel<A>): no chain of time chunks. A persistent
// 512-thread workgroup (one per CU, 132 KB of LDS) walks column GROUPS of 4 batch columns,
// g = lg, lg + G, ...; a group's whole sequence (pi and mu tiles: T rows x 288 B; act / rew /
// disc: T rows x 16 B; val: T+1 rows) is DMA'd into one of two slots, and the NEXT group's DMA
// is issued right after this one landed, so the loads of group g+1 stream while group g is
// computed and stored. Thread (t, c) = (tid >> 2, tid & 3) owns one (t, b) row:
//   A  every carry-independent quantity as the slot lands (softmax statistics of pi and mu,
//      rho, c, pg-rho, delta, gamma c);
//   B  one affine suffix scan over t per column: butterfly inside the wave (lanes 4, 8, 16, 32
//      apart hold rows 1, 2, 4, 8 later), wave totals combined through LDS;
//   C  vs, pg_adv, dvalue and dlogits (written over the thread's own pi row, then stored as
//      the tile's full 16-B pieces: 288-B row runs, the global layout's).
// Stores always issue (rows t >= T go to the scratch sink), so every wave issues exactly the
// same VMEM count per group and the wait for group g+1's DMA leaves group g's stores in flight.
// Requires T <= 127 (thread row T writes the bootstrap dvalue), B % 4 == 0, even A <= 20.
// ------------------------------------------------------------------------------------
template <int A>
struct VtStr {
    static constexpr int NC = 4;                        // batch columns per group
    static constexpr int NT = 512;                      // threads: (t, c) = (tid >> 2, tid & 3)
    static constexpr int TMAX = NT / NC - 1;            // 127 (thread row T carries the bootstrap dvalue)
    static constexpr int ROWB = NC * A * 4;             // bytes per t-row of a logits tile (288 at A=18)
    static constexpr int PPR = ROWB / 16;               // 16-B pieces per t-row
    static constexpr int NW = NT / 64;                  // 8 waves
    static constexpr int NST = 4 + 3;                   // stores per wave per group (dlogits + vs/adv/dval)
    static_assert(A % 2 == 0 && ROWB % 16 == 0, "pieces");
    __host__ __device__ static constexpr int logp(int T) { return (T * ROWB + 1023) / 1024; }  // pieces per logits tile
    __host__ __device__ static constexpr int scp(int T) { return (T * 16 + 1023) / 1024; }      // per scalar tile
    __host__ __device__ static constexpr int valp(int T) { return ((T + 1) * 16 + 1023) / 1024; }
    __host__ __device__ static constexpr int pieces(int T) { return 2 * logp(T) + 3 * scp(T) + valp(T); }
    __host__ __device__ static constexpr int slot_bytes(int T) { return 1024 * pieces(T); }
    __host__ __device__ static constexpr int lds_bytes(int T) { return 2 * slot_bytes(T) + NW * NC * 2 * 4; }
};

// piece j (< pieces(T)) of group b0's slot: the tensor it comes from and the byte offsets
template <int A>
__device__ __forceinline__ void vt_str_issue(const VtRsrc& rs, uint32_t slot_lds, int T, int B, int b0, int w, int lane) {
    using L = VtStr<A>;
    const int LP = L::logp(T), SP = L::scp(T), NPc = L::pieces(T);
    const int per_wave = (NPc + L::NW - 1) / L::NW;
    for (int i = 0; i < per_wave; ++i) {
        int j = w + L::NW * i;
        if (j >= NPc) j = w;  // pad the wave's count: a duplicate of its first piece (same bytes, same place)
        const int q0 = 16 * lane;
        if (j < 2 * LP) {  // pi | mu
            const int jj = j < LP ? j : j - LP;
            int q = jj * 1024 + q0;
            if (q >= T * L::ROWB) q = q0 % L::ROWB;  // past the tile: row 0 again, lands in the padding
            const int t = q / L::ROWB, cb = q - t * L::ROWB;
            blds16_nt(j < LP ? rs.pi : rs.mu, (uint32_t)((t * B + b0) * A * 4 + cb), slot_lds + 1024u * j);
        } else {  // act | rew | disc (T rows x 16 B) | val (T + 1 rows)
            const int k = j - 2 * LP, s = k / SP < 3 ? k / SP : 3;
            const int jj = k - s * SP, rows = s == 3 ? T + 1 : T;
            int q = jj * 1024 + q0;
            if (q >= rows * 16) q = q0 % 16;
            const int t = q >> 4, cb = q & 15;
            blds16_nt(s == 0 ? rs.act : s == 1 ? rs.rew : s == 2 ? rs.disc : rs.val,
                      (uint32_t)((t * B + b0) * 4 + cb), slot_lds + 1024u * j);
        }
    }
}

template <int S>
__device__ __forceinline__ float vt_shx(float v) { return __shfl_xor(v, S, 64); }
template <int S>
__device__ __forceinline__ void vt_str_scan_step(float& sd, float& sg, float& ed, float& eg, int lane) {
    const float pd = vt_shx<S>(sd), pg = vt_shx<S>(sg);
    const bool later = (lane & S) == 0;  // the partner segment holds later rows
    ed = later ? ed + eg * pd : ed;
    eg = later ? eg * pg : eg;
    sd = later ? sd + sg * pd : pd + pg * sd;
    sg = sg * pg;
}

template <int A>
__global__ __launch_bounds__(512, 1) void vtrace_stream_kernel(VtArgs a) {
    using L = VtStr<A>;
    extern __shared__ __attribute__((aligned(16))) char vsm[];
    const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
    const int T = a.T, B = a.B;
    const int tt = tid >> 2, c = tid & 3;
    const bool valid = tt < T;
    const int G = gridDim.x, lg = xcd_remap(blockIdx.x, G);
    const int ngroups = B / L::NC;
    const int SB = L::slot_bytes(T), LP = L::logp(T), SP = L::scp(T);
    const uint32_t lds0 = lds_addr(vsm);
    float* tot = (float*)(vsm + 2 * SB);  // [NW][NC][2] wave totals
    const VtRsrc rs = vt_rsrc(a);
    const fi_vtrace_hparams hp = a.hp;
    constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
    float pg = 0.f, base = 0.f, ent = 0.f;
    float* const sink = a.sink + tid;
    int k = 0;
    if (lg < ngroups) vt_str_issue<A>(rs, lds0, T, B, L::NC * lg, w, lane);
    for (int grp = lg; grp < ngroups; grp += G, ++k) {
        const int b0 = L::NC * grp, b = b0 + c;
        char* const sl = vsm + (k & 1) * SB;
        // this group's pieces landed (the previous group's NST stores may still be in flight)
        wait_vmcnt(k == 0 ? 0 : L::NST);
        lds_barrier();  // B1: every wave's pieces landed; the other slot's last reads are done
        if (grp + G < ngroups) vt_str_issue<A>(rs, lds0 + ((k + 1) & 1) * SB, T, B, L::NC * (grp + G), w, lane);

        // ---- A: carry-independent work of row (tt, b)
        const int tr = valid ? tt : 0;
        float* zpi = (float*)(sl + tr * L::ROWB + c * A * 4);
        const float* zmu = (const float*)(sl + 1024 * LP + tr * L::ROWB + c * A * 4);
        const int* sact = (const int*)(sl + 2048 * LP);
        const float* srew = (const float*)(sl + 2048 * LP + 1024 * SP);
        const float* sdisc = (const float*)(sl + 2048 * LP + 2048 * SP);
        const float* sval = (const float*)(sl + 2048 * LP + 3072 * SP);
        f32x2 zp2[A / 2], zm2[A / 2];
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            zp2[i] = *(const f32x2*)(zpi + 2 * i);
            zm2[i] = *(const f32x2*)(zmu + 2 * i);
        }
        int at = sact[4 * tr + c];
        if (valid && (unsigned)at >= (unsigned)A) atomicAdd(a.bad, 1);
        at = at < 0 ? 0 : (at >= A ? A - 1 : at);
        const float zpa = zpi[at], zma = zmu[at];
        const float rw = srew[4 * tr + c], g = sdisc[4 * tr + c], v = sval[4 * tr + c], vn = sval[4 * tr + 4 + c];
        float mx = vt_max3(zp2[0].x, zp2[0].y, zp2[0].y), mm = vt_max3(zm2[0].x, zm2[0].y, zm2[0].y);
#pragma unroll
        for (int i = 1; i < A / 2; ++i) {
            mx = vt_max3(mx, zp2[i].x, zp2[i].y);
            mm = vt_max3(mm, zm2[i].x, zm2[i].y);
        }
        const f32x2 nmx = {-mx * L2E, -mx * L2E}, nmm = {-mm * L2E, -mm * L2E};
        f32x2 sp2 = {0.f, 0.f}, sm2 = {0.f, 0.f}, sz2 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            const f32x2 ap = zp2[i] * L2E + nmx;
            const f32x2 am = zm2[i] * L2E + nmm;
            const f32x2 e = f32x2{VT_EXP2(ap.x), VT_EXP2(ap.y)};
            sp2 += e;
            sz2 += e * zp2[i];
            sm2 += f32x2{VT_EXP2(am.x), VT_EXP2(am.y)};
        }
        const float sp = sp2.x + sp2.y, sm = sm2.x + sm2.y;
        const float lse = mx + VT_LOG2(sp) * LN2, lsem = mm + VT_LOG2(sm) * LN2;
        const float inv = __builtin_amdgcn_rcpf(sp);
        const float plogp = (sz2.x + sz2.y) * inv - lse;
        const float lpa = zpa - lse, lma = zma - lsem;
        const float ratio = VT_EXP(lpa - lma);
        const float rho = fminf(hp.rho_bar, ratio);
        const float cc = hp.lambda_ * fminf(hp.c_bar, ratio);
        const float pgr = fminf(hp.pg_rho_bar, ratio);
        const float d_own = valid ? rho * (rw + g * vn - v) : 0.f;
        const float g_own = valid ? g * cc : 1.f;

        // ---- B: reverse affine scan over t (rows 16w .. 16w + 15 of this wave, 4 lanes apart)
        float sd = d_own, sg = g_own, ed = 0.f, eg = 1.f;
        vt_str_scan_step<4>(sd, sg, ed, eg, lane);
        vt_str_scan_step<8>(sd, sg, ed, eg, lane);
        vt_str_scan_step<16>(sd, sg, ed, eg, lane);
        vt_str_scan_step<32>(sd, sg, ed, eg, lane);
        if (lane < L::NC) {
            tot[(w * L::NC + c) * 2] = sd;
            tot[(w * L::NC + c) * 2 + 1] = sg;
        }
        lds_barrier();  // B2: wave totals visible
        float acc_in = 0.f;  // acc at row 16(w + 1): the later waves composed onto acc_T = 0
#pragma unroll
        for (int w2 = L::NW - 1; w2 > 0; --w2)
            if (w2 > w) acc_in = tot[(w2 * L::NC + c) * 2] + tot[(w2 * L::NC + c) * 2 + 1] * acc_in;
        const float acc_nx = ed + eg * acc_in;
        const float acc = d_own + g_own * acc_nx;

        // ---- C: targets, gradients, stores
        const float vs_t = v + acc;
        const float vs_n = vn + acc_nx;
        const float adv = pgr * (rw + g * vs_n - v);
        const float dv = -hp.baseline_cost * acc;
        {  // dlogits over this thread's own pi row
            const float ec = hp.entropy_cost;
            const float al = inv * (adv - ec * (plogp + lse)), be = inv * ec;
            const f32x2 al2 = {al, al};
#pragma unroll
            for (int i = 0; i < A / 2; ++i) {
                const f32x2 ap = zp2[i] * L2E + nmx;
                const f32x2 e = f32x2{VT_EXP2(ap.x), VT_EXP2(ap.y)};
                if (valid) *(f32x2*)(zpi + 2 * i) = e * (zp2[i] * be + al2);
            }
            if (valid) zpi[at] -= adv;
        }
        if (valid) {
            pg += -adv * lpa;
            base += 0.5f * acc * acc;
            ent += plogp;
        }
        {  // vs / pg_adv / dvalue of the thread's row; thread row T writes the bootstrap dvalue 0
            const size_t e = (size_t)tt * B + b;
            VT_ST(vs_t, valid ? a.vs + e : sink);
            VT_ST(adv, valid ? a.adv + e : sink);
            VT_ST(valid ? dv : 0.f, tt <= T ? a.dval + e : sink);
        }
        lds_barrier();  // B3: the dlogits rows are complete
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // the tile's T * PPR pieces, 4 rounds of 512
            const int q = L::NT * i + tid;
            const int row = q / L::PPR, pc = q - row * L::PPR;
            const f32x4 d4 = *(const f32x4*)(sl + 16 * (q < T * L::PPR ? q : 0));
            VT_ST(d4, q < T * L::PPR ? (f32x4*)(a.dlog + (size_t)(row * B + b0) * A) + pc : (f32x4*)(a.sink + 4 * tid));
        }
    }
    __syncthreads();
    block_reduce3((double)pg, (double)base, (double)ent, (double*)vsm, a.part + (size_t)blockIdx.x * 3);
}

// ------------------------------------------------------------------------------------
// Kernel 3 (vtrace_seq_kernel<A>, on request only -- measured slower than kernel 1, DESIGN.md
// section 5): a persistent 256-thread
// workgroup walks column PAIRS p = lg, lg + G, ... and owns each pair for the WHOLE sequence,
// so the only serial dependency of V-trace (the scalar carry acc_{t+1}) is resolved by one
// in-register scan plus one cross-wave combine per pair -- no chain of time chunks.
// A pair's data (pi and mu tiles: T rows x 144 B; the act / rew / disc / val columns:
// T (+1) rows x 8 B) arrives by LDS-DMA into one of two slots (32 KB each at T = 100); the
// next pair's DMA is issued right after the landing barrier, so it streams in while this
// pair is computed. Two workgroups per CU (8 waves, 4 pair-slots of LDS). Pairs adjacent in
// memory go to workgroups on the same XCD (xcd_remap), whose 144-B row runs share L2 lines.
// Lane map: lane = j + 32 c, column c = lane >> 5, j = 0..31 the wave's rows in REVERSE time
// (t = 32 w + 31 - j), so the reverse recurrence acc_t = d_t + g_t acc_{t+1} is a prefix
// scan in lane order inside each 32-lane half: DPP row_shr:1/2/4/8 inside 16-lane rows, then
// row_bcast:15 into the upper row (the classic gfx9 scan, affine operator), identity (0, 1)
// shifted in at the edges. Wave totals cross waves through LDS (one barrier).
// dlogits are written over the lane's own pi row in the slot and leave as 16-byte stores in
// the global layout's 144-B runs. Loss partials stay in registers across pairs and are
// reduced once per workgroup. vmcnt is counted per wave: every store instruction always
// issues (lanes with t >= T write the scratch sink), so the wait for pair k+1's DMA leaves
// exactly pair k's stores outstanding. Algorithmic HBM traffic: 12A+28 bytes per (t,b).
// ------------------------------------------------------------------------------------
template <int A>
struct VtSeq {
    static constexpr int NB = 2;                // batch columns per pair
    static constexpr int NT = 256;              // threads: 4 waves x 32 rows x 2 columns
    static constexpr int TMAX = NT / NB;        // 128 timesteps
    static constexpr int ROWB = NB * A * 4;     // bytes per t-row of a logits tile (144 at A=18)
    static constexpr int PPR = ROWB / 16;       // 16-B pieces per t-row
    static_assert(A % 2 == 0 && ROWB % 16 == 0, "pieces");
    // slot: pi [T][ROWB] | mu [T][ROWB] | act [T][NB] | rew [T][NB] | disc [T][NB] | val [T+1][NB],
    // each region padded to whole DMA instructions (1 KiB / 256 B), so the lanes of a tile's last
    // instruction that run past its end read zeros (out-of-range offset) into the padding and
    // every lane can issue
    __host__ __device__ static int tile_bytes(int T) { return (T * ROWB + 1023) & ~1023; }
    __host__ __device__ static int col_bytes(int T) { return (T * NB * 4 + NB * 4 + 255) & ~255; }
    __host__ __device__ static int slot_bytes(int T) { return 2 * tile_bytes(T) + 4 * col_bytes(T); }
    // two slots | wave totals [4][2][NB] | loss scratch [4][3] doubles
    static size_t lds_bytes(int T) { return (size_t)2 * slot_bytes(T) + 4 * 2 * NB * 4 + 4 * 3 * 8; }
};

// identity-filled DPP move of a float (lanes whose source is out of range get `idf`)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float vt_dppf(float v, float idf) {
    return __uint_as_float(__builtin_amdgcn_update_dpp(__float_as_uint(idf), __float_as_uint(v), CTRL, ROWMASK, 0xf, false));
}
// one Hillis-Steele step of the affine prefix composition (D, G) <- (D + G D', G G'),
// (D', G') = the value CTRL moves in (identity (0, 1) where there is none)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ void vt_affine_step(float& D, float& G) {
    const float pd = vt_dppf<CTRL, ROWMASK>(D, 0.f), pg = vt_dppf<CTRL, ROWMASK>(G, 1.f);
    D = fmaf(G, pd, D);
    G = G * pg;
}

// DMA of one pair into a slot: the pi and mu tiles' 1-KiB pieces ii = w, w + 4, ... (16 B per
// lane, the piece's 64 lanes cover 7 1/9 rows of 144 B), and scalar column w (act / rew / disc /
// val for waves 0..3: 4 B per lane, 256 B per instruction). Lanes past a tile's end read zeros
// (FI_OOB) into the slot's padding, so every instruction issues with all lanes. Offsets need a
// constant division (by 9) only; the stores' vmcnt bookkeeping does not depend on this count.
template <int A>
__device__ __forceinline__ void vt_seq_issue(const fi_i32x4 (&rs)[6], uint32_t slot_lds, int T, int B, int w,
                                             int lane, int b0) {
    using L = VtSeq<A>;
    const int np = T * L::PPR, nl = (np + 63) / 64;
    const uint32_t dl = (uint32_t)b0 * A * 4;
    for (int ii = w; ii < nl; ii += 4) {
        const int q = 64 * ii + lane;
        const int row = q / L::PPR, pc = q - row * L::PPR;
        const uint32_t voff = q < np ? (uint32_t)(row * B * A * 4 + pc * 16) + dl : FI_OOB;
        blds16(rs[0], voff, __builtin_amdgcn_readfirstlane(slot_lds + 1024 * ii));
        blds16(rs[1], voff, __builtin_amdgcn_readfirstlane(slot_lds + L::tile_bytes(T) + 1024 * ii));
    }
    const int lim = w < 3 ? 2 * T : 2 * (T + 1), ncl = (2 * (T + 1) + 63) / 64;
    fi_i32x4 rc = w == 0 ? rs[2] : (w == 1 ? rs[3] : (w == 2 ? rs[4] : rs[5]));
#pragma unroll
    for (int e = 0; e < 4; ++e) rc[e] = __builtin_amdgcn_readfirstlane(rc[e]);
    const uint32_t cbase = slot_lds + 2 * L::tile_bytes(T) + w * L::col_bytes(T);
    for (int ii = 0; ii < ncl; ++ii) {
        const int q = 64 * ii + lane;
        const uint32_t voff = q < lim ? (uint32_t)(((q >> 1) * B + b0 + (q & 1)) * 4) : FI_OOB;
        blds4(rc, voff, __builtin_amdgcn_readfirstlane(cbase + 256 * ii));
    }
}

template <int A>
__global__ __launch_bounds__(256, 2) void vtrace_seq_kernel(VtArgs a) {
    using L = VtSeq<A>;
    extern __shared__ __attribute__((aligned(16))) char vsm[];
    const int T = a.T, B = a.B;
    const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
    const int G = gridDim.x, lg = xcd_remap(blockIdx.x, G);
    const int npairs = B / L::NB;
    const int j = lane & 31, c = lane >> 5;
    const int t = 32 * w + 31 - j;
    const bool valid = t < T;
    const int tt = valid ? t : T - 1;  // rows past T read a valid row, contribute identity
    const int SB = L::slot_bytes(T);
    float* const tot = (float*)(vsm + 2 * SB);
    const uint32_t lds0 = lds_addr(vsm);
    fi_i32x4 rs[6];
    {
        const uint32_t lbytes = (uint32_t)T * B * A * 4, sbytes = (uint32_t)T * B * 4;
        rs[0] = make_rsrc(a.pi, lbytes);
        rs[1] = make_rsrc(a.mu, lbytes);
        rs[2] = make_rsrc(a.act, sbytes);
        rs[3] = make_rsrc(a.rew, sbytes);
        rs[4] = make_rsrc(a.disc, sbytes);
        rs[5] = make_rsrc(a.val, sbytes + (uint32_t)B * 4);
    }
    const fi_vtrace_hparams hp = a.hp;
    // per-wave store instructions of one pair: vs, adv, dval + this wave's dlogits pieces
    const int np = T * L::PPR;
    int n_dl = 0;
    for (int i = w; 64 * i < np; i += 4) ++n_dl;
    const int n_st = 3 + n_dl;
    float pg = 0.f, base = 0.f, ent = 0.f;
    float* const sink = a.sink + tid;  // stores of lanes with t >= T

    int k = 0;
    int p = lg;
    if (p < npairs) vt_seq_issue<A>(rs, lds0, T, B, w, lane, L::NB * p);
    for (; p < npairs; p += G, ++k) {
        const int b0 = L::NB * p, b = b0 + c;
        char* const sl = vsm + (k & 1) * SB;
        // this pair's DMA landed (the previous pair's stores may still be in flight)
        wait_vmcnt(k > 0 ? n_st : 0);
        lds_barrier();  // B1: slot k&1 landed for every wave; slot (k+1)&1's last reads done
        if (p + G < npairs) vt_seq_issue<A>(rs, lds0 + ((k + 1) & 1) * SB, T, B, w, lane, L::NB * (p + G));
        if (tid < L::NB) a.dval[(size_t)T * B + b0 + tid] = 0.f;  // the bootstrap row (not counted: see below)

        // scalars of the lane's (t, b)
        const int* sact = (const int*)(sl + 2 * L::tile_bytes(T));
        const float* srew = (const float*)(sl + 2 * L::tile_bytes(T) + L::col_bytes(T));
        const float* sdisc = (const float*)(sl + 2 * L::tile_bytes(T) + 2 * L::col_bytes(T));
        const float* sval = (const float*)(sl + 2 * L::tile_bytes(T) + 3 * L::col_bytes(T));
        int at = sact[2 * tt + c];
        const float rw = srew[2 * tt + c], g = sdisc[2 * tt + c], v = sval[2 * tt + c], vn = sval[2 * tt + 2 + c];
        if (valid && (unsigned)at >= (unsigned)A) atomicAdd(a.bad, 1);
        at = at < 0 ? 0 : (at >= A ? A - 1 : at);

        // softmax statistics of the lane's own row (as kernel 1)
        constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
        float* const zpi = (float*)(sl + (size_t)tt * L::ROWB) + c * A;
        const float* const zmu = (const float*)(sl + L::tile_bytes(T) + (size_t)tt * L::ROWB) + c * A;
        f32x2 zp2[A / 2], zm2[A / 2];
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            zp2[i] = *(const f32x2*)(zpi + 2 * i);
            zm2[i] = *(const f32x2*)(zmu + 2 * i);
        }
        const float zpa = zpi[at], zma = zmu[at];
        float mx = vt_max3(zp2[0].x, zp2[0].y, zp2[0].y), mm = vt_max3(zm2[0].x, zm2[0].y, zm2[0].y);
#pragma unroll
        for (int i = 1; i < A / 2; ++i) {
            mx = vt_max3(mx, zp2[i].x, zp2[i].y);
            mm = vt_max3(mm, zm2[i].x, zm2[i].y);
        }
        const f32x2 nmx = {-mx * L2E, -mx * L2E}, nmm = {-mm * L2E, -mm * L2E};
        f32x2 e2[A / 2];
        f32x2 sp2 = {0.f, 0.f}, sm2 = {0.f, 0.f}, sz2 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
            const f32x2 ap = zp2[i] * L2E + nmx;
            const f32x2 am = zm2[i] * L2E + nmm;
            e2[i] = f32x2{VT_EXP2(ap.x), VT_EXP2(ap.y)};
            sp2 += e2[i];
            sz2 += e2[i] * zp2[i];
            sm2 += f32x2{VT_EXP2(am.x), VT_EXP2(am.y)};
        }
        const float sp = sp2.x + sp2.y, sm = sm2.x + sm2.y;
        const float lse = mx + VT_LOG2(sp) * LN2, lsem = mm + VT_LOG2(sm) * LN2;
        const float inv = __builtin_amdgcn_rcpf(sp);
        const float plogp = (sz2.x + sz2.y) * inv - lse;
        const float lpa = zpa - lse, lma = zma - lsem;
        const float ratio = VT_EXP(lpa - lma);
        const float rho = fminf(hp.rho_bar, ratio);
        const float cc = hp.lambda_ * fminf(hp.c_bar, ratio);
        const float pgr = fminf(hp.pg_rho_bar, ratio);
        const float d_own = valid ? rho * (rw + g * vn - v) : 0.f;
        const float g_own = valid ? g * cc : 1.f;

        // prefix composition in lane order (= reverse time) inside each 32-lane column half
        float D = d_own, Gm = g_own;
        vt_affine_step<0x111>(D, Gm);       // row_shr:1
        vt_affine_step<0x112>(D, Gm);       // row_shr:2
        vt_affine_step<0x114>(D, Gm);       // row_shr:4
        vt_affine_step<0x118>(D, Gm);       // row_shr:8
        vt_affine_step<0x142, 0xa>(D, Gm);  // row_bcast:15 into rows 1 and 3 (lanes 16-31, 48-63)
        // exclusive composition (the rows after t inside the wave): one lane up, identity at j = 0
        float Dx = vt_dppf<0x138>(D, 0.f), Gx = vt_dppf<0x138>(Gm, 1.f);  // wave_shr:1
        if (j == 0) {
            Dx = 0.f;
            Gx = 1.f;
        }
        if (j == 31) {  // the wave's total for column c
            tot[(w * 2 + 0) * L::NB + c] = D;
            tot[(w * 2 + 1) * L::NB + c] = Gm;
        }
        lds_barrier();  // B2: wave totals visible
        float x = 0.f;  // acc at t = 32 (w + 1): later waves composed onto the bootstrap acc_T = 0
#pragma unroll
        for (int w2 = 3; w2 >= 0; --w2)
            if (w2 > w) x = tot[(w2 * 2 + 0) * L::NB + c] + tot[(w2 * 2 + 1) * L::NB + c] * x;
        const float acc_nx = Dx + Gx * x;  // acc_{t+1}
        const float acc = d_own + g_own * acc_nx;
        const float vs_t = v + acc;
        const float adv = pgr * (rw + g * (vn + acc_nx) - v);
        const float dv = -hp.baseline_cost * acc;

        // dlogits over the lane's own pi row: dz_i = e_i (alpha + beta z_i) - adv [i = a_t]
        {
            const float ec = hp.entropy_cost;
            const float al = inv * (adv - ec * (plogp + lse)), be = inv * ec;
            const f32x2 al2 = {al, al};
            if (valid) {
#pragma unroll
                for (int i = 0; i < A / 2; ++i) *(f32x2*)(zpi + 2 * i) = e2[i] * (zp2[i] * be + al2);
                zpi[at] -= adv;
            }
        }
        if (valid) {
            pg += -adv * lpa;
            base += 0.5f * acc * acc;
            ent += plogp;
        }
        {  // every lane stores (the sink takes rows t >= T), so each wave issues exactly 3 here
            const size_t e = (size_t)tt * B + b;
            VT_ST(vs_t, valid ? a.vs + e : sink);
            VT_ST(adv, valid ? a.adv + e : sink);
            VT_ST(dv, valid ? a.dval + e : sink);
        }
        lds_barrier();  // B3: the slot's dlogits rows complete

        // the dlogits tile out in the global layout (144-B runs), 16 B per lane
        for (int i = w; 64 * i < np; i += 4) {
            const int q = 64 * i + lane;
            if (q < np) {
                const int row = q / L::PPR, pc = q - row * L::PPR;
                const f32x4 d4 = *(const f32x4*)(sl + 16 * q);
                VT_ST(d4, (f32x4*)(a.dlog + (size_t)(row * B + b0) * A) + pc);
            }
        }
        // the bootstrap-row store above is the one VMEM op not in n_st: it was issued BEFORE
        // this pair's stores, i.e. it is older than them and retired by the next wait as well
    }
    __syncthreads();
    // per-workgroup loss partials (summed in a fixed order later, as kernel 1)
    block_reduce3((double)pg, (double)base, (double)ent, (double*)(tot + 4 * 2 * L::NB),
                  a.part + (size_t)blockIdx.x * 3);
}

__global__ __launch_bounds__(256) void vtrace_finalize_kernel(const double* __restrict__ part,
                                                              int nblk, double* losses,
                                                              const int* bad) {
    __shared__ double red[4 * 3];
    double s0 = 0, s1 = 0, s2 = 0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        s0 += part[(size_t)i * 3];
        s1 += part[(size_t)i * 3 + 1];
        s2 += part[(size_t)i * 3 + 2];
    }
    block_reduce3(s0, s1, s2, red, losses);
    // an action outside [0, A) anywhere in the batch poisons the loss scalars (the oracle
    // rejects such a batch; the standalone entry point has no synchronous status to return)
    if (threadIdx.x < 3 && bad && *bad != 0) losses[threadIdx.x] = __builtin_nan("");
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static size_t vt_nblk_max(int B) { return (size_t)std::max({(B + 7) / 8, (B + 255) / 256, 2 * 1024}); }

// workspace: [sink floats][loss partials, 256-B padded][int bad-action counter, 256 B]
static size_t vt_part_bytes(int B) { return (vt_nblk_max(B) * 3 * sizeof(double) + 255) & ~(size_t)255; }
size_t vtrace_workspace_bytes(int T, int B, int A) {
    (void)T;
    (void)A;
    return kSinkFloats * sizeof(float) + vt_part_bytes(B) + 256;
}
static int* vt_bad_counter(void* ws, int B) {
    return (int*)((char*)ws + kSinkFloats * sizeof(float) + vt_part_bytes(B));
}

template <int A>
static void launch_lds(const VtArgs& a, int nblk, hipStream_t s) {
    hipLaunchKernelGGL(vtrace_lds_kernel<A>, dim3(nblk), dim3(64 * VtLayout<A>::NW), 0, s, a);
}
template <int A>
static void launch_seq(const VtArgs& a, int nblk, hipStream_t s) {
    hipLaunchKernelGGL(vtrace_seq_kernel<A>, dim3(nblk), dim3(VtSeq<A>::NT), VtSeq<A>::lds_bytes(a.T), s, a);
}
// persistent grid of the sequence kernel: two workgroups per CU (LDS: two pair slots each)
// (the CU count is read from the calling thread's current device each time: handles on
// different devices launch from their own threads, so no cached process-wide value)
static int seq_grid(int B) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, std::min(B / 2, 2 * cus));
}

static bool lds_supported(int A, int B) { return B % 8 == 0 && A % 2 == 0 && A >= 2 && A <= 20; }

template <int A>
static int launch_str(const VtArgs& a, int nblk, hipStream_t s) {
    // more than 64 KB of dynamic LDS: the kernel's limit is raised once per device (a bit per
    // device id; handles on different devices launch from their own threads)
    static std::atomic<uint64_t> raised{0};
    int dev = 0;
    FI_HIP_CHECK(hipGetDevice(&dev));
    const uint64_t bit = dev < 64 ? (uint64_t)1 << dev : 0;
    if (!bit || !(raised.load(std::memory_order_acquire) & bit)) {
        const hipError_t e = hipFuncSetAttribute((const void*)vtrace_stream_kernel<A>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess)
            return fail(FI_ERR_HIP, std::string("vtrace: the streaming kernel needs 160 KB of LDS per workgroup "
                                                "(hipFuncSetAttribute MaxDynamicSharedMemorySize: ") +
                                        hipGetErrorString(e) + ")");
        raised.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(vtrace_stream_kernel<A>, dim3(nblk), dim3(VtStr<A>::NT), VtStr<A>::lds_bytes(a.T), s, a);
    return FI_OK;
}
// persistent grid of the streaming kernel: one workgroup per CU (132 KB of LDS at T = 100)
static int str_grid(int B) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, std::min(B / 4, cus));
}
// (the two slots hold the whole sequence of a group: T <= 124 at A = 18 within 160 KB of LDS)
static int str_lds_bytes(int T, int A) {
    const int logp = (T * 4 * A * 4 + 1023) / 1024, scp = (T * 16 + 1023) / 1024, valp = ((T + 1) * 16 + 1023) / 1024;
    return 2 * 1024 * (2 * logp + 3 * scp + valp) + 8 * 4 * 2 * 4;
}
// the dlogits tile leaves in 4 rounds of NT = 512 pieces of 16 B (VtStr::NST counts them), so
// T * PPR = T * A pieces must fit 2,048 (T <= 113 at A = 18, T <= 102 at A = 20)
static bool str_supported(int T, int A, int B) {
    return B % 4 == 0 && A % 2 == 0 && A >= 2 && A <= 20 && T <= VtStr<2>::TMAX && T * A <= 4 * VtStr<2>::NT &&
           str_lds_bytes(T, A) <= 160 * 1024;
}

int vtrace_launch(int variant, int T, int B, int A, const float* pi, const float* mu,
                  const int32_t* act, const float* rew, const float* disc, const float* val,
                  const fi_vtrace_hparams& hp, float* vs, float* adv, float* dlog, float* dval,
                  double* losses, void* ws, size_t ws_bytes, hipStream_t stream, bool finalize,
                  int* nblk_out, int* bad) {
    FI_REQUIRE(T >= 1 && B >= 1 && A >= 1 && A <= 64, "vtrace: bad shape");
    FI_REQUIRE(pi && mu && act && rew && disc && val && dlog && dval && ws, "vtrace: null pointer");
    finalize = finalize && losses;  // losses == NULL: partials stay in the workspace
    FI_REQUIRE(ws_bytes >= vtrace_workspace_bytes(T, B, A), "vtrace: workspace too small");
    VtArgs a;
    a.T = T; a.B = B; a.A = A;
    a.pi = pi; a.mu = mu; a.act = act; a.rew = rew; a.disc = disc; a.val = val;
    a.vs = vs; a.adv = adv; a.dlog = dlog; a.dval = dval;
    a.sink = (float*)ws;
    a.part = (double*)((char*)ws + kSinkFloats * sizeof(float));
    a.hp = hp;
    a.bad = bad;
    if (!bad) {  // standalone call: count into the workspace, finalize turns it into NaN losses
        a.bad = vt_bad_counter(ws, B);
        FI_HIP_CHECK(hipMemsetAsync(a.bad, 0, sizeof(int), stream));
    }
    // the LDS kernel's buffer descriptors and DMA offsets are 32-bit: T*B*A*4 must stay
    // below 2^31 bytes (else the column kernel, 64-bit indexing, runs)
    const bool fits32 = (size_t)T * B * A * sizeof(float) < ((size_t)1 << 31);
    // variant 3 (whole-sequence workgroups) on request only: measured slower than the chunked
    // kernel 1 ("V-trace: the whole-sequence kernel")
    const bool seq_ok = lds_supported(A, B) && fits32 && T <= 128 && B % 2 == 0;
    FI_REQUIRE(!(variant == 3 && !seq_ok), "vtrace: sequence kernel needs T<=128, B%8==0, even A<=20");
    if (variant == 3) {
        FI_REQUIRE(vs && adv, "vtrace: sequence kernel writes vs and pg_adv (non-null)");
        FI_REQUIRE(((uintptr_t)pi | (uintptr_t)mu | (uintptr_t)dlog) % 16 == 0, "vtrace: needs 16-byte aligned logits");
        const int nblk = seq_grid(B);
        switch (A) {
            case 2: launch_seq<2>(a, nblk, stream); break;
            case 4: launch_seq<4>(a, nblk, stream); break;
            case 6: launch_seq<6>(a, nblk, stream); break;
            case 8: launch_seq<8>(a, nblk, stream); break;
            case 10: launch_seq<10>(a, nblk, stream); break;
            case 12: launch_seq<12>(a, nblk, stream); break;
            case 14: launch_seq<14>(a, nblk, stream); break;
            case 16: launch_seq<16>(a, nblk, stream); break;
            case 18: launch_seq<18>(a, nblk, stream); break;
            case 20: launch_seq<20>(a, nblk, stream); break;
            default: return fail(FI_ERR_UNSUPPORTED, "vtrace: A not instantiated");
        }
        FI_HIP_CHECK(hipGetLastError());
        if (nblk_out) *nblk_out = nblk;
        if (finalize) return vtrace_finalize_launch(ws, nblk, losses, stream, a.bad);
        return FI_OK;
    }
    if (variant == 4) {
        FI_REQUIRE(str_supported(T, A, B) && fits32,
                   "vtrace: streaming kernel needs B%4==0, even A<=20, T*A<=2048 and the whole sequence of 4 columns in 160 KB of LDS");
        FI_REQUIRE(vs && adv, "vtrace: streaming kernel writes vs and pg_adv (non-null)");
        FI_REQUIRE(((uintptr_t)pi | (uintptr_t)mu | (uintptr_t)dlog) % 16 == 0 &&
                   ((uintptr_t)act | (uintptr_t)rew | (uintptr_t)disc | (uintptr_t)val) % 16 == 0,
                   "vtrace: streaming kernel needs 16-byte aligned tensors");
        const int nblk = str_grid(B);
        switch (A) {
            case 2: FI_TRY(launch_str<2>(a, nblk, stream)); break;
            case 4: FI_TRY(launch_str<4>(a, nblk, stream)); break;
            case 6: FI_TRY(launch_str<6>(a, nblk, stream)); break;
            case 8: FI_TRY(launch_str<8>(a, nblk, stream)); break;
            case 10: FI_TRY(launch_str<10>(a, nblk, stream)); break;
            case 12: FI_TRY(launch_str<12>(a, nblk, stream)); break;
            case 14: FI_TRY(launch_str<14>(a, nblk, stream)); break;
            case 16: FI_TRY(launch_str<16>(a, nblk, stream)); break;
            case 18: FI_TRY(launch_str<18>(a, nblk, stream)); break;
            case 20: FI_TRY(launch_str<20>(a, nblk, stream)); break;
            default: return fail(FI_ERR_UNSUPPORTED, "vtrace: A not instantiated");
        }
        FI_HIP_CHECK(hipGetLastError());
        if (nblk_out) *nblk_out = nblk;
        if (finalize) return vtrace_finalize_launch(ws, nblk, losses, stream, a.bad);
        return FI_OK;
    }
    bool use_lds = variant == 1 || (variant == 0 && lds_supported(A, B) && fits32);
    FI_REQUIRE(!(variant == 1 && !lds_supported(A, B)), "vtrace: LDS kernel needs B%8==0, even A<=20");
    FI_REQUIRE(!(variant == 1 && !fits32), "vtrace: LDS kernel needs T*B*A*4 < 2^31 bytes");
    int nblk;
    if (use_lds) {
        FI_REQUIRE(vs && adv, "vtrace: LDS kernel writes vs and pg_adv (non-null)");
        FI_REQUIRE(((uintptr_t)pi | (uintptr_t)mu | (uintptr_t)dlog) % 16 == 0 &&
                   ((uintptr_t)act | (uintptr_t)rew | (uintptr_t)disc | (uintptr_t)val) % 16 == 0,
                   "vtrace: LDS kernel needs 16-byte aligned tensors");
        nblk = B / 8;
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
    if (finalize) return vtrace_finalize_launch(ws, nblk, losses, stream, a.bad);
    return FI_OK;
}

const double* vtrace_partials(const void* ws) {
    return (const double*)((const char*)ws + kSinkFloats * sizeof(float));
}

int vtrace_finalize_launch(void* ws, int nblk, double* losses, hipStream_t stream, const int* bad) {
    const double* part = (const double*)((char*)ws + kSinkFloats * sizeof(float));
    hipLaunchKernelGGL(vtrace_finalize_kernel, dim3(1), dim3(256), 0, stream, part, nblk, losses, bad);
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
