// gemm_f32.hip -- fp32 GEMMs on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32) for the
// MLP policy of config #2 (fp32 parity mode). No reference counterpart (the reference
// learner has no network, learner.h:32-49); shapes follow SURVEY.md 8(a) "Policy network".
//
// C[M][N] = sum_k A(m,k) B(k,n), one 256-thread workgroup per 128x64 tile, BK = 16.
// Both operands are staged in LDS "k-major" ([BK][W]) so that every MFMA operand read is
// one conflict-free ds_read_b32 per lane (lane l: A[m=l&31][k=l>>5], B[k=l>>5][n=l&31]).
// Loaders translate the source layout (row-major with k or with m/n contiguous, or the
// split logits|value arrays of the heads) into that image; register prefetch of tile k+1
// overlaps the MFMAs of tile k. Epilogues fuse bias+ReLU, the heads split, the ReLU
// mask of the backward pass, or write split-K partial slabs (weight gradients).
#include "fi_common.h"

#include "kernels.h"

namespace fi {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 128, GBN = 64, GBK = 16;
constexpr int GLDA = GBM + 4, GLDB = GBN + 4;  // padded LDS row strides (floats)

// ---------------- loaders: fill a [GBK][W] k-major tile ---------------------------------
// KMajor: element(k, w) = p[k*ld + w]   (rows of the source are the reduction index)
// WMajor: element(k, w) = p[w*ld + k]   (rows of the source are the output index)
// Both vectorize with float4 when vec (ld % 4 == 0 and 16-byte aligned base).
template <int W>
struct KMajor {
    const float* p;
    int ld, krows, wcols;  // bounds: k < krows, w < wcols
    bool vec;
    static constexpr int PER = GBK * W / 4 / 256;  // float4 per thread
    __device__ void fetch(float4* r, int k0, int w0) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int k = idx / (W / 4), w = (idx % (W / 4)) * 4;
            const int gk = k0 + k, gw = w0 + w;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gk < krows) {
                const float* s = p + (size_t)gk * ld + gw;
                if (vec && gw + 3 < wcols) {
                    v = *(const float4*)s;
                } else {
                    if (gw < wcols) v.x = s[0];
                    if (gw + 1 < wcols) v.y = s[1];
                    if (gw + 2 < wcols) v.z = s[2];
                    if (gw + 3 < wcols) v.w = s[3];
                }
            }
            r[i] = v;
        }
    }
    __device__ void store(float* lds, int ldl, const float4* r) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int k = idx / (W / 4), w = (idx % (W / 4)) * 4;
            float* d = lds + k * ldl + w;
            d[0] = r[i].x; d[1] = r[i].y; d[2] = r[i].z; d[3] = r[i].w;
        }
    }
};

template <int W>
struct WMajor {
    const float* p;
    int ld, wrows, kcols;  // bounds: w < wrows, k < kcols
    bool vec;
    static constexpr int PER = GBK * W / 4 / 256;
    __device__ void fetch(float4* r, int k0, int w0) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int w = idx / (GBK / 4), k = (idx % (GBK / 4)) * 4;
            const int gw = w0 + w, gk = k0 + k;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gw < wrows) {
                const float* s = p + (size_t)gw * ld + gk;
                if (vec && gk + 3 < kcols) {
                    v = *(const float4*)s;
                } else {
                    if (gk < kcols) v.x = s[0];
                    if (gk + 1 < kcols) v.y = s[1];
                    if (gk + 2 < kcols) v.z = s[2];
                    if (gk + 3 < kcols) v.w = s[3];
                }
            }
            r[i] = v;
        }
    }
    __device__ void store(float* lds, int ldl, const float4* r) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int w = idx / (GBK / 4), k = (idx % (GBK / 4)) * 4;
            lds[(k + 0) * ldl + w] = r[i].x;
            lds[(k + 1) * ldl + w] = r[i].y;
            lds[(k + 2) * ldl + w] = r[i].z;
            lds[(k + 3) * ldl + w] = r[i].w;
        }
    }
};

// The heads' upstream gradient as a virtual [rows][A+1] matrix: columns 0..A-1 are
// dlogits (T,B,A) for rows < TB (zero on the bootstrap rows), column A is dvalue.
__device__ __forceinline__ float dout_get(const HeadsGrad& g, int row, int col) {
    if (row >= g.rows) return 0.f;
    if (col < g.A) return row < g.TB ? g.dlog[(size_t)row * g.A + col] : 0.f;
    return col == g.A ? g.dval[row] : 0.f;
}

template <int W>
struct DoutWMajor {  // element(k = o, w = m)
    HeadsGrad g;
    static constexpr int PER = GBK * W / 256;
    __device__ void fetch(float* r, int k0, int w0) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int w = idx / GBK, k = idx % GBK;
            r[i] = dout_get(g, w0 + w, k0 + k);
        }
    }
    __device__ void store(float* lds, int ldl, const float* r) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            lds[(idx % GBK) * ldl + idx / GBK] = r[i];
        }
    }
};

template <int W>
struct DoutKMajor {  // element(k = m, w = o)
    HeadsGrad g;
    static constexpr int PER = GBK * W / 256;
    __device__ void fetch(float* r, int k0, int w0) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            const int k = idx / W, w = idx % W;
            r[i] = dout_get(g, k0 + k, w0 + w);
        }
    }
    __device__ void store(float* lds, int ldl, const float* r) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            lds[(idx / W) * ldl + idx % W] = r[i];
        }
    }
};

template <class L>
struct RegsOf {
    typedef float4 type;
    static constexpr int N = L::PER;
};
template <int W>
struct RegsOf<DoutWMajor<W>> {
    typedef float type;
    static constexpr int N = DoutWMajor<W>::PER;
};
template <int W>
struct RegsOf<DoutKMajor<W>> {
    typedef float type;
    static constexpr int N = DoutKMajor<W>::PER;
};

// ---------------- epilogues ---------------------------------------------------------
struct EpiBiasRelu {  // C = relu(acc + bias) (relu optional)
    float* C;
    int ldc;
    const float* bias;
    int relu;
    __device__ void operator()(int m, int n, float v) const {
        v += bias ? bias[n] : 0.f;
        if (relu) v = fmaxf(v, 0.f);
        C[(size_t)m * ldc + n] = v;
    }
};
struct EpiHeads {  // logits (rows, A) | values (rows)
    float* logits;
    float* values;
    const float* bias;
    int A;
    __device__ void operator()(int m, int n, float v) const {
        v += bias[n];
        if (n < A) logits[(size_t)m * A + n] = v;
        else values[m] = v;
    }
};
struct EpiMask {  // C = (act > 0) ? acc : 0  -- ReLU backward through the post-activation
    float* C;
    int ldc;
    const float* act;
    __device__ void operator()(int m, int n, float v) const {
        const size_t i = (size_t)m * ldc + n;
        C[i] = act[i] > 0.f ? v : 0.f;
    }
};
struct EpiSlab {  // split-K partial slab: C[split][m][n]
    float* C;
    int ldc;
    size_t split_stride;
    int z = 0;  // this workgroup's split (set by the kernel)
    __device__ void operator()(int m, int n, float v) const {
        C[z * split_stride + (size_t)m * ldc + n] = v;
    }
};
template <class E>
__device__ __forceinline__ void epi_set_split(E&, int) {}
__device__ __forceinline__ void epi_set_split(EpiSlab& e, int z) { e.z = z; }

// ---------------- the kernel --------------------------------------------------------
// COLSUM: blocks of the first M-tile also sum the B tile over k (the bias gradient of a
// weight-gradient GEMM, B = dY) into colsum[split][N] -- no separate column-sum pass.
template <class LA, class LB, class Epi, bool COLSUM>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(LA la, LB lb, Epi epi, int M, int N,
                                                          int K, int k_per_split, float* colsum) {
    __shared__ __attribute__((aligned(16))) float As[2][GBK * GLDA];
    __shared__ __attribute__((aligned(16))) float Bs[2][GBK * GLDB];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // tile order: the N-tiles of one (M-tile, split) get consecutive logical ids on ONE XCD
    // (xcd_remap), so the A rows they share are fetched from HBM once and hit that XCD's L2
    // for the others (in launch order they were gridDim.x workgroups apart)
    const int gx = gridDim.x, gy = gridDim.y;
    const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int lg = xcd_remap(lin, gx * gy * gridDim.z);
    const int by = lg % gy, bx = (lg / gy) % gx, bz = lg / (gx * gy);
    epi_set_split(epi, bz);
    const int m0 = bx * GBM, n0 = by * GBN;
    const int kbeg = bz * k_per_split;
    const int kend = min(K, kbeg + k_per_split);
    f32x16 acc0 = {}, acc1 = {};
    float cs = 0.f;
    const bool do_cs = COLSUM && bx == 0 && threadIdx.x < GBN;
    typename RegsOf<LA>::type ra[RegsOf<LA>::N];
    typename RegsOf<LB>::type rb[RegsOf<LB>::N];
    int buf = 0;
    if (kbeg < kend) {
        la.fetch(ra, kbeg, m0);
        lb.fetch(rb, kbeg, n0);
        la.store(As[0], GLDA, ra);
        lb.store(Bs[0], GLDB, rb);
    }
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += GBK) {
        const bool more = k0 + GBK < kend;
        if (more) {
            la.fetch(ra, k0 + GBK, m0);
            lb.fetch(rb, k0 + GBK, n0);
        }
        const float* as = As[buf];
        const float* bs = Bs[buf];
#pragma unroll
        for (int kp = 0; kp < GBK / 2; ++kp) {
            const int kk = 2 * kp + (lane >> 5);
            const float a = as[kk * GLDA + w * 32 + (lane & 31)];
            const float b0 = bs[kk * GLDB + (lane & 31)];
            const float b1 = bs[kk * GLDB + 32 + (lane & 31)];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
        }
        if (do_cs) {
#pragma unroll
            for (int kk = 0; kk < GBK; ++kk) cs += bs[kk * GLDB + threadIdx.x];
        }
        if (more) {
            la.store(As[buf ^ 1], GLDA, ra);
            lb.store(Bs[buf ^ 1], GLDB, rb);
        }
        __syncthreads();
        buf ^= 1;
    }
    if (do_cs && n0 + (int)threadIdx.x < N) colsum[(size_t)bz * N + n0 + threadIdx.x] = cs;
    // C/D map of 32x32 tiles: row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + w * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + (lane & 31);
        if (m < M) {
            if (n < N) epi(m, n, acc0[r]);
            if (n + 32 < N) epi(m, n + 32, acc1[r]);
        }
    }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <class LA, class LB, class Epi>
static int launch(LA la, LB lb, Epi epi, int M, int N, int K, int splits, hipStream_t s,
                  float* colsum = nullptr) {
    const int kps = ((K + splits - 1) / splits + GBK - 1) / GBK * GBK;
    dim3 grid((M + GBM - 1) / GBM, (N + GBN - 1) / GBN, splits);
    if (colsum)
        hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, Epi, true>), grid, dim3(256), 0, s, la, lb, epi, M,
                           N, K, kps, colsum);
    else
        hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, Epi, false>), grid, dim3(256), 0, s, la, lb, epi,
                           M, N, K, kps, colsum);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// Y[M][N] = X[M][K] W[K][N] + b (ReLU)
int f32_linear_fwd(const float* X, int M, int K, const float* W, const float* bias, int N,
                   bool relu, float* Y, hipStream_t s) {
    WMajor<GBM> la{X, K, M, K, K % 4 == 0 && aligned16(X)};
    KMajor<GBN> lb{W, N, K, N, N % 4 == 0 && aligned16(W)};
    return launch(la, lb, EpiBiasRelu{Y, N, bias, relu ? 1 : 0}, M, N, K, 1, s);
}

// heads: out = X Wh + bh split into logits (M, A) and values (M)
int f32_heads_fwd(const float* X, int M, int K, const float* W, const float* bias, int A,
                  float* logits, float* values, hipStream_t s) {
    const int N = A + 1;
    WMajor<GBM> la{X, K, M, K, K % 4 == 0 && aligned16(X)};
    KMajor<GBN> lb{W, N, K, N, N % 4 == 0 && aligned16(W)};
    return launch(la, lb, EpiHeads{logits, values, bias, A}, M, N, K, 1, s);
}

// dX[M][K] = dY[M][N] W[K][N]^T, masked by (act > 0) when act != null
int f32_linear_dgrad(const float* dY, int M, int N, const float* W, int K, const float* act,
                     float* dX, hipStream_t s) {
    WMajor<GBM> la{dY, N, M, N, N % 4 == 0 && aligned16(dY)};
    WMajor<GBN> lb{W, N, K, N, N % 4 == 0 && aligned16(W)};
    if (act) return launch(la, lb, EpiMask{dX, K, act}, M, K, N, 1, s);
    return launch(la, lb, EpiBiasRelu{dX, K, nullptr, 0}, M, K, N, 1, s);
}

// heads backward: dX[M][K] = dout[M][A+1] Wh[K][A+1]^T masked by act
int f32_heads_dgrad(const HeadsGrad& g, const float* W, int K, const float* act, float* dX,
                    hipStream_t s) {
    const int N = g.A + 1;
    DoutWMajor<GBM> la{g};
    WMajor<GBN> lb{W, N, K, N, false};
    return launch(la, lb, EpiMask{dX, K, act}, g.rows, K, N, 1, s);
}

// partial weight gradients: slab[split][I][N] = sum_{m in split} X[m][I] dY[m][N]
// slab[split][I][N] = sum_{m in split} X[m][I] dY[m][N];  cs_slab[split][N] = sum_m dY[m][N]
int f32_linear_wgrad_partial(const float* X, int M, int I, const float* dY, int N, int splits,
                             float* slab, float* cs_slab, hipStream_t s) {
    KMajor<GBM> la{X, I, M, I, I % 4 == 0 && aligned16(X)};
    KMajor<GBN> lb{dY, N, M, N, N % 4 == 0 && aligned16(dY)};
    return launch(la, lb, EpiSlab{slab, N, (size_t)I * N}, I, N, M, splits, s, cs_slab);
}

int f32_heads_wgrad_partial(const float* X, int I, const HeadsGrad& g, int splits, float* slab,
                            float* cs_slab, hipStream_t s) {
    const int N = g.A + 1;
    KMajor<GBM> la{X, I, g.rows, I, I % 4 == 0 && aligned16(X)};
    DoutKMajor<GBN> lb{g};
    return launch(la, lb, EpiSlab{slab, N, (size_t)I * N}, I, N, g.rows, splits, s, cs_slab);
}

// ---- MLP heads backward, fused (H = 256, O = A + 1 outputs): one pass over h2 computes both
// the heads' weight gradient (slab[block][H][O] = sum over the block's rows of h2[r][j] dout[r][o],
// plus the bias partials sum_r dout[r][o]) and the data gradient dz2[r][j] = (h2[r][j] > 0) *
// sum_o dout[r][o] Wh[j][o]. The two GEMM launches it replaces read h2 twice and ran the skinny
// O = 19 side padded to a 64-wide MFMA tile (1.0 ms at R = 413,696 against a 0.85 GB memory
// floor). A wave takes one row at a time (lane: 4 consecutive columns, the row's upstream
// gradient in scalar registers), rows r = its global wave index + k * (all waves); the block's 4
// waves are combined in a fixed order (deterministic), the blocks by reduce_slabs.
template <int O>
__global__ __launch_bounds__(256, 2) void heads_bwd_fused_f32(HeadsGrad g, const float* __restrict__ h2,
                                                              const float* __restrict__ Wh,  // [256][O]
                                                              float* __restrict__ dz2, float* __restrict__ slab,
                                                              float* __restrict__ cs_slab) {
    constexpr int H = 256, A = O - 1;
    __shared__ float red[H * O];
    __shared__ float bred[4][O];
    const int lane = threadIdx.x & 63, w = wave_id(), j0 = 4 * lane;
    float wv[4][O], acc[4][O], bs[O];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int o = 0; o < O; ++o) {
            wv[jj][o] = Wh[(size_t)(j0 + jj) * O + o];
            acc[jj][o] = 0.f;
        }
#pragma unroll
    for (int o = 0; o < O; ++o) bs[o] = 0.f;
    const int nw = gridDim.x * 4;
    auto row_in = [&](int r, float (&d)[O], float4& hv) {
#pragma unroll
        for (int o = 0; o < A; ++o) d[o] = r < g.TB ? g.dlog[(size_t)r * A + o] : 0.f;
        d[A] = g.dval[r];
        hv = *(const float4*)(h2 + (size_t)r * H + j0);
    };
    int r = blockIdx.x * 4 + w;
    float d[O];
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < g.rows) row_in(r, d, hv);
    for (; r < g.rows; r += nw) {
        float dn[O];  // the next row's inputs, loaded while this row computes
        float4 hn = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r + nw < g.rows) row_in(r + nw, dn, hn);
        const float hx[4] = {hv.x, hv.y, hv.z, hv.w};
        float dx[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            float a = 0.f;
#pragma unroll
            for (int o = 0; o < O; ++o) {
                a = fmaf(d[o], wv[jj][o], a);
                acc[jj][o] = fmaf(hx[jj], d[o], acc[jj][o]);
            }
            dx[jj] = hx[jj] > 0.f ? a : 0.f;
        }
        *(float4*)(dz2 + (size_t)r * H + j0) = make_float4(dx[0], dx[1], dx[2], dx[3]);
#pragma unroll
        for (int o = 0; o < O; ++o) {
            bs[o] += d[o];
            d[o] = dn[o];
        }
        hv = hn;
    }
    for (int i = threadIdx.x; i < H * O; i += 256) red[i] = 0.f;
    __syncthreads();
    for (int ww = 0; ww < 4; ++ww) {  // fixed-order combine of the block's waves
        if (w == ww) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int o = 0; o < O; ++o) red[(j0 + jj) * O + o] += acc[jj][o];
            if (lane == 0)
#pragma unroll
                for (int o = 0; o < O; ++o) bred[ww][o] = bs[o];
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < H * O; i += 256) slab[(size_t)blockIdx.x * H * O + i] = red[i];
    if (threadIdx.x < O)
        cs_slab[(size_t)blockIdx.x * O + threadIdx.x] =
            (bred[0][threadIdx.x] + bred[1][threadIdx.x]) + (bred[2][threadIdx.x] + bred[3][threadIdx.x]);
}

bool f32_heads_bwd_fused_supported(int H, int A) { return H == 256 && A == 18; }

int f32_heads_bwd_fused(const HeadsGrad& g, const float* h2, const float* Wh, int H, float* dz2, float* slab,
                        float* cs_slab, int grid, hipStream_t s) {
    FI_REQUIRE(f32_heads_bwd_fused_supported(H, g.A), "heads_bwd_fused: H = 256, A = 18 only");
    FI_REQUIRE(aligned16(h2) && aligned16(dz2), "heads_bwd_fused: 16-byte aligned h2 / dz2");
    hipLaunchKernelGGL(heads_bwd_fused_f32<19>, dim3(grid), dim3(256), 0, s, g, h2, Wh, dz2, slab, cs_slab);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// ---- PyTorch-layout weights (W[N][K], nn.Linear): the FarmerLstm torso (farmer.hip)
// Y[M][N] = X[M][K] W[N][K]^T + b (ReLU); ldx = row stride of X
int f32_gemm_nt(const float* X, int ldx, int M, int K, const float* W, const float* bias, int N,
                bool relu, float* Y, hipStream_t s) {
    WMajor<GBM> la{X, ldx, M, K, ldx % 4 == 0 && K % 4 == 0 && aligned16(X)};
    WMajor<GBN> lb{W, K, N, K, K % 4 == 0 && aligned16(W)};
    return launch(la, lb, EpiBiasRelu{Y, N, bias, relu ? 1 : 0}, M, N, K, 1, s);
}

// dX[M][K] = dY[M][N] W[N][K], masked by (act > 0) when act != null (act: [M][K])
int f32_gemm_nn_dgrad(const float* dY, int M, int N, const float* W, int K, const float* act, float* dX,
                      hipStream_t s) {
    WMajor<GBM> la{dY, N, M, N, N % 4 == 0 && aligned16(dY)};
    KMajor<GBN> lb{W, K, N, K, K % 4 == 0 && aligned16(W)};
    if (act) return launch(la, lb, EpiMask{dX, K, act}, M, K, N, 1, s);
    return launch(la, lb, EpiBiasRelu{dX, K, nullptr, 0}, M, K, N, 1, s);
}

// weight-gradient partials in PyTorch layout: slab[split][N][K] = sum_{m in split} dY[m][N] X[m][K]
int f32_gemm_tn_wgrad(const float* dY, int M, int N, const float* X, int ldx, int K, int splits, float* slab,
                      hipStream_t s) {
    KMajor<GBM> la{dY, N, M, N, N % 4 == 0 && aligned16(dY)};
    KMajor<GBN> lb{X, ldx, M, K, ldx % 4 == 0 && K % 4 == 0 && aligned16(X)};
    return launch(la, lb, EpiSlab{slab, K, (size_t)N * K}, N, K, M, splits, s);
}

}  // namespace fi
