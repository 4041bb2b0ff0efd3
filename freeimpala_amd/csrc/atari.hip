// atari.hip -- the Atari-shaped conv policy of config #3 on bf16 MFMA (gfx950).
//
// No reference counterpart: the reference learner has no network (learner.h:32-49). The
// architecture is the SURVEY.md 8(a) "Policy network" row (Nature-DQN torso as used by
// IMPALA/torchbeast): frames u8 (84,84,4)/255 -> conv 8x8/4 32 -> conv 4x4/2 64 ->
// conv 3x3/1 64 -> fc 3136->512 -> heads (A logits | value). NHWC everywhere, activations
// and upstream gradients in bf16, fp32 accumulation, fp32 master weights / grads / Adam.
//
// Every layer is one of two MFMA (v_mfma_f32_32x32x16_bf16) kernels:
//  * bf16_gemm  -- C[m][n] = sum_k A(m,k) B(n,k): forward convs as implicit GEMM (A gathered
//    from the NHWC input 16 bytes = 8 channels at a time; conv1 gathers 8 u8 = 2 pixels x 4
//    channels), fc/heads, and data-gradients (dgrad of a strided conv is split into S*S
//    parity classes so every M-tile uses one weight slice). Both operands are staged through
//    padded LDS rows (80 B: conflict-free ds_read_b128 fragment reads), register prefetch of
//    the next K-tile overlaps the MFMAs. Epilogues fuse bias + ReLU (+1/255 scale), the
//    heads split, and the ReLU mask of the backward pass.
//  * bf16_wgrad -- weight gradients C[i][j] = sum_m A(m,i) B(m,j): the reduction runs over
//    output pixels, so tiles are staged [m][i] and fed to the MFMA with the gfx950 transpose
//    read ds_read_b64_tr_b16 (no shuffles); split over m into fp32 slabs reduced in a fixed
//    order (deterministic); the bias gradient (column sums of B) rides along.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "atari.h"
#include "fi_common.h"
#include "kernels.h"

namespace fi {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ geometry
namespace geo {
constexpr int C1K = 256, C1O = 32;           // conv1: k = (ky,kx,ci) 8*8*4
constexpr int C2K = 512, C2O = 64;           // conv2: 4*4*32
constexpr int C3K = 576, C3O = 64;           // conv3: 3*3*64
constexpr int FCK = 3136, FCO = 512;         // fc
constexpr int HP = 32;                       // heads padded output width (A+1 <= 32)
constexpr int P1 = 400, P2 = 81, P3 = 49;    // output pixels per frame
}  // namespace geo

struct Offsets {  // offsets into the fp32 parameter blob (== oracle layout)
    size_t c1w, c1b, c2w, c2b, c3w, c3b, fcw, fcb, hw, hb, total;
    explicit Offsets(int A) {
        size_t o = 0;
        c1w = o; o += 8 * 8 * 4 * 32; c1b = o; o += 32;
        c2w = o; o += 4 * 4 * 32 * 64; c2b = o; o += 64;
        c3w = o; o += 3 * 3 * 64 * 64; c3b = o; o += 64;
        fcw = o; o += (size_t)3136 * 512; fcb = o; o += 512;
        hw = o; o += (size_t)512 * (A + 1); hb = o; o += A + 1;
        total = o;
    }
};

size_t atari_param_count(int A) { return Offsets(A).total; }

void atari_init_params(int A, uint64_t seed, std::vector<float>& p) {
    // Glorot-uniform (fan_in = kh*kw*cin, fan_out = kh*kw*cout), zero biases.
    Offsets off(A);
    p.assign(off.total, 0.f);
    uint64_t st = seed ^ 0xA7A21ull;
    auto next = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto fill = [&](size_t o, size_t n, double fi, double fo) {
        const double lim = std::sqrt(6.0 / (fi + fo));
        for (size_t i = 0; i < n; ++i) {
            const double u = (double)(next() >> 11) * (1.0 / 9007199254740992.0);
            p[o + i] = (float)((2.0 * u - 1.0) * lim);
        }
    };
    fill(off.c1w, 8192, 256, 64 * 32);
    fill(off.c2w, 32768, 512, 16 * 64);
    fill(off.c3w, 36864, 576, 9 * 64);
    fill(off.fcw, (size_t)3136 * 512, 3136, 512);
    fill(off.hw, (size_t)512 * (A + 1), 512, A + 1);
}

// ------------------------------------------------------------------ operand loaders
// Each returns 8 consecutive k (or i) values of row r as 8 packed bf16 (16 bytes), zero
// outside the matrix. kc = k / 8.
__device__ __forceinline__ u32x4 zero4() { return u32x4{0u, 0u, 0u, 0u}; }

struct RowsBf16 {  // plain row-major bf16 matrix [rows][ld]
    const __bf16* p;
    int rows, ld;
    __device__ void set_tile(int) {}
    __device__ u32x4 load(int r, int kc) const {
        if (r >= rows || kc * 8 >= ld) return zero4();
        return *(const u32x4*)(p + (size_t)r * ld + kc * 8);
    }
};

// conv1 input: frames u8 [N][84][84][4]; k = (ky*8 + kx)*4 + c, a k-chunk = 2 pixels x 4 ch
struct Conv1Gather {
    const uint8_t* fr;
    int rows;  // N*400
    __device__ void set_tile(int) {}
    __device__ u32x4 load(int m, int kc) const {
        if (m >= rows) return zero4();
        const int n = m / 400, pix = m - n * 400;
        const int oy = pix / 20, ox = pix - oy * 20;
        const int ky = kc >> 2, kx = (kc & 3) * 2;
        const uint2 v = *(const uint2*)(fr + (((size_t)n * 84 + oy * 4 + ky) * 84 + ox * 4 + kx) * 4);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[j] = (__bf16)(float)((v.x >> (8 * j)) & 0xffu);
            o[4 + j] = (__bf16)(float)((v.y >> (8 * j)) & 0xffu);
        }
        return __builtin_bit_cast(u32x4, o);
    }
};

// NHWC bf16 conv input, kernel KS, stride S, channels C (multiple of 8), output OH x OH
template <int H, int C, int KS, int S, int OH>
struct ConvGather {
    const __bf16* x;
    int rows;  // N * OH * OH
    __device__ void set_tile(int) {}
    __device__ u32x4 load(int m, int kc) const {
        if (m >= rows || kc * 8 >= KS * KS * C) return zero4();
        const int n = m / (OH * OH), pix = m - n * (OH * OH);
        const int oy = pix / OH, ox = pix - oy * OH;
        const int k = kc * 8;
        const int ky = k / (KS * C), kx = (k / C) % KS, c = k % C;
        return *(const u32x4*)(x + (((size_t)n * H + oy * S + ky) * H + ox * S + kx) * C + c);
    }
};

// dgrad of a conv (kernel KS, stride S, in IH x IH x Ci, out OH x OH x Co): rows are input
// pixels grouped by parity class (py,px); a class occupies `cstride` rows (>= N*Q*Q, padded
// to the M-tile) with Q = IH / S. k = (ty, tx, co), ky = py + S*ty, oy = iy' - ty.
template <int IH, int KS, int S, int OH, int CO>
struct DgradGather {
    const __bf16* dy;  // [N][OH][OH][CO]
    int nf, cstride;
    static constexpr int Q = IH / S, TT = KS / S;
    __device__ void set_tile(int) {}
    __device__ u32x4 load(int m, int kc) const {
        const int cls = m / cstride, r = m - cls * cstride;
        if (cls >= S * S || r >= nf * Q * Q) return zero4();
        const int n = r / (Q * Q), q2 = r - n * (Q * Q);
        const int iyq = q2 / Q, ixq = q2 - iyq * Q;
        const int k = kc * 8;
        const int tap = k / CO, co = k - tap * CO;
        if (tap >= TT * TT) return zero4();
        const int ty = tap / TT, tx = tap - ty * TT;
        const int oy = iyq - ty, ox = ixq - tx;
        if (oy < 0 || oy >= OH || ox < 0 || ox >= OH) return zero4();
        return *(const u32x4*)(dy + (((size_t)n * OH + oy) * OH + ox) * CO + co);
    }
};

// dgrad weights for parity class of the current M-tile: [cls][ci][k]
struct ClassRows {
    const __bf16* p;
    int rows, ld, cstride;
    size_t cls_stride;
    const __bf16* cur;
    __device__ void set_tile(int m0) { cur = p + (size_t)(m0 / cstride) * cls_stride; }
    __device__ u32x4 load(int r, int kc) const {
        if (r >= rows || kc * 8 >= ld) return zero4();
        return *(const u32x4*)(cur + (size_t)r * ld + kc * 8);
    }
};

// ------------------------------------------------------------------ epilogues
struct EpiAct {  // out[m][n] = bf16(relu(acc*scale + bias[n]))
    __bf16* out;
    int ld;
    const float* bias;
    float scale;
    __device__ void operator()(int m, int n, float v) const {
        v = fmaxf(v * scale + bias[n], 0.f);
        out[(size_t)m * ld + n] = (__bf16)v;
    }
};
struct EpiHeadsOut {
    float* logits;
    float* values;
    const float* bias;
    int A;
    __device__ void operator()(int m, int n, float v) const {
        if (n > A) return;
        v += bias[n];
        if (n < A) logits[(size_t)m * A + n] = v;
        else values[m] = v;
    }
};
template <int IH, int S>
struct EpiDgrad {  // class-ordered row -> input pixel; masked by the input activation
    __bf16* out;
    const __bf16* act;
    int nf, cstride, ci;
    static constexpr int Q = IH / S;
    __device__ void operator()(int m, int n, float v) const {
        const int cls = m / cstride, r = m - cls * cstride;
        if (r >= nf * Q * Q) return;
        const int b = r / (Q * Q), q2 = r - b * (Q * Q);
        const int iy = (q2 / Q) * S + cls / S, ix = (q2 % Q) * S + cls % S;
        const size_t i = (((size_t)b * IH + iy) * IH + ix) * ci + n;
        out[i] = (float)act[i] > 0.f ? (__bf16)v : (__bf16)0.f;
    }
};

// ------------------------------------------------------------------ bf16_gemm
constexpr int KB = 32;         // k per LDS stage
constexpr int LROW = KB + 8;   // padded LDS row (bf16): 80 bytes

template <int BM, int BN, int WM, int WN, class LA, class LB, class Epi>
__global__ __launch_bounds__(256) void bf16_gemm(LA la, LB lb, Epi epi, int M, int N, int K) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int CA = BM * (KB / 8) / 256;  // 16-byte chunks per thread
    constexpr int CBT = BN * (KB / 8);
    constexpr int CB = (CBT + 255) / 256;
    static_assert(TM >= 1 && TN >= 1 && WM * WN == 4 && CA >= 1, "tile");
    __shared__ __attribute__((aligned(16))) __bf16 sA[2][BM * LROW];
    __shared__ __attribute__((aligned(16))) __bf16 sB[2][BN * LROW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WN, wn = w % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    la.set_tile(m0);
    lb.set_tile(m0);
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
    u32x4 ra[CA], rb[CB];
    auto fetch = [&](int kc0) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int idx = tid + 256 * i;
            ra[i] = la.load(m0 + (idx >> 2), kc0 + (idx & 3));
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int idx = tid + 256 * i;
            if (idx < CBT) rb[i] = lb.load(n0 + (idx >> 2), kc0 + (idx & 3));
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int idx = tid + 256 * i;
            *(u32x4*)&sA[buf][(idx >> 2) * LROW + (idx & 3) * 8] = ra[i];
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int idx = tid + 256 * i;
            if (idx < CBT) *(u32x4*)&sB[buf][(idx >> 2) * LROW + (idx & 3) * 8] = rb[i];
        }
    };
    const int nk = (K + KB - 1) / KB;
    fetch(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) fetch((kt + 1) * (KB / 8));
#pragma unroll
        for (int ks = 0; ks < KB / 16; ++ks) {
            bf16x8 af[TM], bfv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *(const bf16x8*)&sA[buf][(wm * (BM / WM) + i * 32 + (lane & 31)) * LROW + ks * 16 +
                                                 (lane >> 5) * 8];
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfv[j] = *(const bf16x8*)&sB[buf][(wn * (BN / WN) + j * 32 + (lane & 31)) * LROW + ks * 16 +
                                                  (lane >> 5) * 8];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int n = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
                if (m < M && n < N) epi(m, n, acc[i][j][r]);
            }
}

template <int BM, int BN, int WM, int WN, class LA, class LB, class Epi>
static int gemm(LA la, LB lb, Epi epi, int M, int N, int K, hipStream_t s) {
    dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN);
    hipLaunchKernelGGL((bf16_gemm<BM, BN, WM, WN, LA, LB, Epi>), grid, dim3(256), 0, s, la, lb, epi, M,
                       N, K);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// ------------------------------------------------------------------ bf16_wgrad
// C[i][j] = scale * sum_m A(m, i) B(m, j) for m in [split*mps, (split+1)*mps)
// LDS rows are m; pitch chosen so the transposed b64 reads are bank-conflict free.
constexpr int MC = 32;  // m per LDS stage (2 MFMA K-steps)
template <int W>
struct TrPitch {
    static constexpr int value = (W % 128 == 0) ? W + 32 : (W % 64 == 0 ? W + 32 : W);
};

__device__ __forceinline__ bf16x8 tr_frag(const __bf16* base, int pitch, int lane) {
    // operand fragment of a 32x32x16 MFMA whose K index runs down the LDS rows:
    // lane l gets column (l&15) + 16*((l>>4)&1) of rows 8*(l>>5) + 0..7
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const __bf16* a0 = base + (8 * (g >> 1) + q) * pitch + 16 * (g & 1) + 4 * p;
    typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 4 * pitch));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BI, int BJ, int WI, int WJ, class LA, class LB>
__global__ __launch_bounds__(256) void bf16_wgrad(LA la, LB lb, float* __restrict__ slab,
                                                  float* __restrict__ cs_slab, int M, int I, int J,
                                                  int mps, float scale) {
    constexpr int TI = BI / WI / 32, TJ = BJ / WJ / 32;
    constexpr int PA = TrPitch<BI>::value, PB = TrPitch<BJ>::value;
    constexpr int CA = MC * (BI / 8) / 256, CBT = MC * (BJ / 8);
    constexpr int CB = (CBT + 255) / 256;
    static_assert(TI >= 1 && TJ >= 1 && WI * WJ == 4 && CA >= 1, "tile");
    __shared__ __attribute__((aligned(16))) __bf16 sA[2][MC * PA];
    __shared__ __attribute__((aligned(16))) __bf16 sB[2][MC * PB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w / WJ, wj = w % WJ;
    const int i0 = blockIdx.x * BI, j0 = blockIdx.y * BJ;
    const int mb = blockIdx.z * mps, me = min(M, mb + mps);
    const bool do_cs = blockIdx.x == 0 && tid < BJ;
    float cs = 0.f;
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b) acc[a][b] = f32x16{};
    u32x4 ra[CA], rb[CB];
    constexpr int AQ = BI / 8, BQ = BJ / 8;  // 16-byte chunks per LDS row
    auto fetch = [&](int mm) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            const int idx = tid + 256 * c;
            const int r = idx / AQ, q = idx - r * AQ;
            ra[c] = (mm + r < me) ? la.load(mm + r, i0 / 8 + q) : zero4();
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int idx = tid + 256 * c;
            const int r = idx / BQ, q = idx - r * BQ;
            if (idx < CBT) rb[c] = (mm + r < me) ? lb.load(mm + r, j0 / 8 + q) : zero4();
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            const int idx = tid + 256 * c;
            const int r = idx / AQ, q = idx - r * AQ;
            *(u32x4*)&sA[buf][r * PA + q * 8] = ra[c];
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int idx = tid + 256 * c;
            const int r = idx / BQ, q = idx - r * BQ;
            if (idx < CBT) *(u32x4*)&sB[buf][r * PB + q * 8] = rb[c];
        }
    };
    if (mb < me) {
        fetch(mb);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int mm = mb; mm < me; mm += MC) {
        const bool more = mm + MC < me;
        if (more) fetch(mm + MC);
#pragma unroll
        for (int ks = 0; ks < MC / 16; ++ks) {
            bf16x8 af[TI], bfv[TJ];
#pragma unroll
            for (int a = 0; a < TI; ++a)
                af[a] = tr_frag(&sA[buf][ks * 16 * PA + wi * (BI / WI) + a * 32], PA, lane);
#pragma unroll
            for (int b = 0; b < TJ; ++b)
                bfv[b] = tr_frag(&sB[buf][ks * 16 * PB + wj * (BJ / WJ) + b * 32], PB, lane);
#pragma unroll
            for (int a = 0; a < TI; ++a)
#pragma unroll
                for (int b = 0; b < TJ; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfv[b], acc[a][b], 0, 0, 0);
        }
        if (do_cs) {
#pragma unroll 8
            for (int r = 0; r < MC; ++r) cs += (float)sB[buf][r * PB + tid];
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    float* out = slab + (size_t)blockIdx.z * I * J;
#pragma unroll
    for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + wi * (BI / WI) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int j = j0 + wj * (BJ / WJ) + b * 32 + (lane & 31);
                if (i < I && j < J) out[(size_t)i * J + j] = acc[a][b][r] * scale;
            }
    if (do_cs && j0 + tid < J) cs_slab[(size_t)blockIdx.z * J + j0 + tid] = cs;
}

template <int BI, int BJ, int WI, int WJ, class LA, class LB>
static int wgrad(LA la, LB lb, float* slab, float* cs_slab, int M, int I, int J, int splits,
                 float scale, hipStream_t s) {
    const int mps = ((M + splits - 1) / splits + MC - 1) / MC * MC;
    dim3 grid((I + BI - 1) / BI, (J + BJ - 1) / BJ, splits);
    hipLaunchKernelGGL((bf16_wgrad<BI, BJ, WI, WJ, LA, LB>), grid, dim3(256), 0, s, la, lb, slab, cs_slab,
                       M, I, J, mps, scale);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// y *= (m > 0) elementwise (generic path only; the frame-resident conv3 backward masks in LDS)
__global__ void relu_mask_bf16_kernel(__bf16* __restrict__ y, const __bf16* __restrict__ m, size_t n8) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
        bf16x8 v = ((bf16x8*)y)[i];
        const bf16x8 k = ((const bf16x8*)m)[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (float)k[j] > 0.f ? v[j] : (__bf16)0.f;
        ((bf16x8*)y)[i] = v;
    }
}

static int relu_mask_bf16(__bf16* y, const __bf16* m, size_t n, hipStream_t s) {
    FI_REQUIRE(n % 8 == 0, "relu_mask_bf16: n % 8");
    hipLaunchKernelGGL(relu_mask_bf16_kernel, dim3(2048), dim3(256), 0, s, y, m, n / 8);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// ------------------------------------------------------------------ heads backward (VALU)
// The heads are a 512 x (A+1) layer: K = A+1 <= 19 is far too thin for MFMA tiles, so both
// backward products run on packed fp32 VALU with the weights / accumulators in registers.
// A wave owns one row at a time (the row's upstream gradient dout[A+1] is wave-uniform:
// scalar loads), each lane 8 consecutive hidden units.
//   dgrad: dh[r][j] = (h[r][j] > 0) * sum_o dout[r][o] Wh[j][o]
//   wgrad: dWh[j][o] = sum_r h[r][j] dout[r][o],  dbh[o] = sum_r dout[r][o]
template <int O>
__device__ __forceinline__ void heads_dout_row(const float* __restrict__ dlog, const float* __restrict__ dval,
                                               int r, int TB, float (&d)[O]) {
    constexpr int A = O - 1;
    if (r < TB) {
#pragma unroll
        for (int o = 0; o < A; ++o) d[o] = dlog[(size_t)r * A + o];
    } else {
#pragma unroll
        for (int o = 0; o < A; ++o) d[o] = 0.f;
    }
    d[A] = dval[r];
}

template <int O>
__global__ __launch_bounds__(256, 2) void heads_dgrad_valu(const float* __restrict__ dlog,
                                                           const float* __restrict__ dval,
                                                           const float* __restrict__ wh,  // [512][O] fp32
                                                           const __bf16* __restrict__ h,
                                                           __bf16* __restrict__ dh, int R, int TB,
                                                           float* __restrict__ fcb_slab) {  // [grid][512]
    __shared__ float cred[4][512];
    const int lane = threadIdx.x & 63, j0 = 8 * lane;
    float cs8[8] = {};  // the fc bias gradient = column sums of dh, as stored (bf16)
    float w[8][O];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
        for (int o = 0; o < O; ++o) w[jj][o] = wh[(size_t)(j0 + jj) * O + o];
    const int nw = gridDim.x * (blockDim.x >> 6);
    int r = blockIdx.x * (blockDim.x >> 6) + wave_id();
    float d[O];
    if (r < R) heads_dout_row<O>(dlog, dval, r, TB, d);
    for (; r < R; r += nw) {
        float dn[O];  // next row's upstream gradient, loaded while this row computes
        if (r + nw < R) heads_dout_row<O>(dlog, dval, r + nw, TB, dn);
        float acc[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            float a = 0.f;
#pragma unroll
            for (int o = 0; o < O; ++o) a = fmaf(d[o], w[jj][o], a);
            acc[jj] = a;
        }
        const bf16x8 hv = *(const bf16x8*)(h + (size_t)r * 512 + j0);
        bf16x8 out;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) out[jj] = (float)hv[jj] > 0.f ? (__bf16)acc[jj] : (__bf16)0.f;
        *(bf16x8*)(dh + (size_t)r * 512 + j0) = out;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) cs8[jj] += (float)out[jj];
#pragma unroll
        for (int o = 0; o < O; ++o) d[o] = dn[o];
    }
    // the block's 4 waves hold the same columns: fixed-order sum, one partial row per block
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) cred[wave_id()][j0 + jj] = cs8[jj];
    __syncthreads();
    for (int c = threadIdx.x; c < 512; c += blockDim.x)
        fcb_slab[(size_t)blockIdx.x * 512 + c] = ((cred[0][c] + cred[1][c]) + cred[2][c]) + cred[3][c];
}

template <int O>
__global__ __launch_bounds__(256, 1) void heads_wgrad_valu(const float* __restrict__ dlog,
                                                           const float* __restrict__ dval,
                                                           const __bf16* __restrict__ h,
                                                           float* __restrict__ slab,     // [grid][512][O]
                                                           float* __restrict__ cs_slab,  // [grid][O]
                                                           int R, int TB) {
    __shared__ float red[512 * O];
    __shared__ float bred[4][O];
    const int lane = threadIdx.x & 63, j0 = 8 * lane, w = wave_id();
    float acc[8][O], bs[O];
#pragma unroll
    for (int o = 0; o < O; ++o) {
        bs[o] = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) acc[jj][o] = 0.f;
    }
    const int nw = gridDim.x * (blockDim.x >> 6);
    int r = blockIdx.x * (blockDim.x >> 6) + w;
    float d[O];
    if (r < R) heads_dout_row<O>(dlog, dval, r, TB, d);
    for (; r < R; r += nw) {
        float dn[O];  // next row's upstream gradient, loaded while this row accumulates
        if (r + nw < R) heads_dout_row<O>(dlog, dval, r + nw, TB, dn);
        const bf16x8 hv = *(const bf16x8*)(h + (size_t)r * 512 + j0);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const float x = (float)hv[jj];
#pragma unroll
            for (int o = 0; o < O; ++o) acc[jj][o] = fmaf(x, d[o], acc[jj][o]);
        }
#pragma unroll
        for (int o = 0; o < O; ++o) {
            bs[o] += d[o];
            d[o] = dn[o];
        }
    }
    // fixed-order combine of the block's 4 waves, then one slab per block
    for (int i = threadIdx.x; i < 512 * O; i += blockDim.x) red[i] = 0.f;
    __syncthreads();
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj)
#pragma unroll
                for (int o = 0; o < O; ++o) red[(j0 + jj) * O + o] += acc[jj][o];
            if (lane == 0)
#pragma unroll
                for (int o = 0; o < O; ++o) bred[ww][o] = bs[o];
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < 512 * O; i += blockDim.x) slab[(size_t)blockIdx.x * 512 * O + i] = red[i];
    if (threadIdx.x < O)
        cs_slab[(size_t)blockIdx.x * O + threadIdx.x] =
            (bred[0][threadIdx.x] + bred[1][threadIdx.x]) + (bred[2][threadIdx.x] + bred[3][threadIdx.x]);
}

constexpr int kHeadsGrid = 512;
constexpr int kHeadsDgradGrid = 1024;

// O = A + 1 outputs as a template argument (the rows live in registers): every Atari action
// set, A = 2..18 (the full ALE set is 18; Breakout 4, Pong 6, Ms. Pac-Man 9)
template <class F>
static int heads_dispatch(int O, F&& f) {
    switch (O) {
#define FI_HEADS_CASE(o) case o: return f(std::integral_constant<int, o>{});
        FI_HEADS_CASE(3) FI_HEADS_CASE(4) FI_HEADS_CASE(5) FI_HEADS_CASE(6) FI_HEADS_CASE(7)
        FI_HEADS_CASE(8) FI_HEADS_CASE(9) FI_HEADS_CASE(10) FI_HEADS_CASE(11) FI_HEADS_CASE(12)
        FI_HEADS_CASE(13) FI_HEADS_CASE(14) FI_HEADS_CASE(15) FI_HEADS_CASE(16) FI_HEADS_CASE(17)
        FI_HEADS_CASE(18) FI_HEADS_CASE(19)
#undef FI_HEADS_CASE
        default: return fail(FI_ERR_INVALID, "atari heads: A + 1 = " + std::to_string(O) + " outside [3, 19]");
    }
}

static int heads_wgrad_launch(int O, const float* dlog, const float* dval, const __bf16* h, float* slab, float* cs,
                              int R, int TB, hipStream_t s) {
    FI_TRY(heads_dispatch(O, [&](auto o) {
        hipLaunchKernelGGL(heads_wgrad_valu<decltype(o)::value>, dim3(kHeadsGrid), dim3(256), 0, s, dlog, dval, h,
                           slab, cs, R, TB);
        return FI_OK;
    }));
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

static int heads_dgrad_launch(int O, const float* dlog, const float* dval, const float* wh, const __bf16* h,
                              __bf16* dh, int R, int TB, float* fcb_slab, hipStream_t s) {
    FI_TRY(heads_dispatch(O, [&](auto o) {
        hipLaunchKernelGGL(heads_dgrad_valu<decltype(o)::value>, dim3(kHeadsDgradGrid), dim3(256), 0, s, dlog,
                           dval, wh, h, dh, R, TB, fcb_slab);
        return FI_OK;
    }));
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// ------------------------------------------------------------------ weight layouts (bf16)
struct WeightsBf16 {
    __bf16 *c1T, *c2T, *c3T, *fcT, *hT;  // forward B operands [out][k]
    __bf16 *c2D, *c3D, *fcB;             // dgrad B operands
};

__global__ void weights_bf16_kernel(const float* __restrict__ p, Offsets o, int A, WeightsBf16 w) {
    const int O = A + 1;
    // segment sizes
    const size_t n1 = 32 * 256, n2 = 64 * 512, n3 = 64 * 576, nf = (size_t)512 * 3136,
                 nh = 32 * 512, n2d = 4 * 32 * 256, n3d = 64 * 576, nfb = nf;
    const size_t total = n1 + n2 + n3 + nf + nh + n2d + n3d + nfb;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
         t += (size_t)gridDim.x * blockDim.x) {
        size_t i = t;
        if (i < n1) { const int co = i / 256, k = i % 256; w.c1T[i] = (__bf16)p[o.c1w + (size_t)k * 32 + co]; continue; }
        i -= n1;
        if (i < n2) { const int co = i / 512, k = i % 512; w.c2T[i] = (__bf16)p[o.c2w + (size_t)k * 64 + co]; continue; }
        i -= n2;
        if (i < n3) { const int co = i / 576, k = i % 576; w.c3T[i] = (__bf16)p[o.c3w + (size_t)k * 64 + co]; continue; }
        i -= n3;
        if (i < nf) { const size_t j = i / 3136, k = i % 3136; w.fcT[i] = (__bf16)p[o.fcw + k * 512 + j]; continue; }
        i -= nf;
        if (i < nh) { const int oo = i / 512, j = i % 512; w.hT[i] = (__bf16)(oo < O ? p[o.hw + (size_t)j * O + oo] : 0.f); continue; }
        i -= nh;
        if (i < n2d) {  // [cls][ci][(ty,tx,co)]
            const int cls = i / (32 * 256), r = i % (32 * 256), ci = r / 256, k = r % 256;
            const int tap = k / 64, co = k % 64, ty = tap / 2, tx = tap % 2;
            const int ky = cls / 2 + 2 * ty, kx = cls % 2 + 2 * tx;
            w.c2D[i] = (__bf16)p[o.c2w + (((size_t)ky * 4 + kx) * 32 + ci) * 64 + co];
            continue;
        }
        i -= n2d;
        if (i < n3d) {  // [ci][(ky,kx,co)]
            const int ci = i / 576, k = i % 576, tap = k / 64, co = k % 64;
            w.c3D[i] = (__bf16)p[o.c3w + ((size_t)tap * 64 + ci) * 64 + co];
            continue;
        }
        i -= n3d;
        w.fcB[i] = (__bf16)p[o.fcw + i];
    }
}

// ------------------------------------------------------------------ the net
struct AtariImpl {
    int N = 0, A = 0, TB = 0;
    Offsets off{18};
    WeightsBf16 wb{};
    __bf16 *a1 = nullptr, *a2 = nullptr, *a3 = nullptr, *h = nullptr;
    __bf16 *da1 = nullptr, *da2 = nullptr, *da3 = nullptr, *dh = nullptr;
    float* slab = nullptr;
    size_t slab_floats = 0;
    const float* params = nullptr;  // last synced fp32 params (for biases)
    std::vector<void*> allocs;
    int cs2 = 0, cs3 = 0;  // class strides for the dgrad GEMMs
    bool fr = true;        // frame-resident kernels (FI_ATARI_GENERIC=1 -> generic GEMMs)
    bool fuse12 = true;    // conv1+conv2 forward in one kernel (FI_FWD_UNFUSED=1 -> two kernels)
    bool fuse21 = true;    // conv2 backward + conv1 wgrad in one kernel (FI_BWD_UNFUSED=1 -> two)
    bool keep_da1 = false; // fused backward also stores da1 to HBM (FI_KEEP_DA1=1; parity checks)
    bool a1_planar = true; // fused fwd + bwd: a1 stored in conv21's image order (FI_A1_NHWC=1 -> NHWC)
    int fr_grid = 256;     // persistent frame-resident workgroups, 1 per CU (FI_FR_GRID=g: tests put
                           // many frames on each workgroup at small N to reach the steady state)
};

int conv1_fwd_fr_launch(const uint8_t* frames, const __bf16* w1t, const float* bias, __bf16* a1,
                        int nframes, int grid, hipStream_t s);
int conv2_fwd_fr_launch(const __bf16* a1, const __bf16* w2t, const float* bias, __bf16* a2, int nframes,
                        int grid, hipStream_t s);
int conv3_fwd_fr_launch(const __bf16* a2, const __bf16* w3t, const float* bias, __bf16* a3, int nframes,
                        int grid, hipStream_t s);
int conv12_fwd_fr_launch(const uint8_t* frames, const __bf16* w1t, const float* b1, const __bf16* w2t,
                         const float* b2, __bf16* a1, __bf16* a2, int nframes, int grid, hipStream_t s,
                         int a1_planar);
int conv1_wgrad_fr_launch(const uint8_t* frames, const __bf16* da1, float* slab, float* cs_slab,
                          int nframes, int grid, hipStream_t s);
int conv21_bwd_fr_launch(const __bf16* a1, const __bf16* da2, const __bf16* w2d, const uint8_t* frames,
                         __bf16* da1_out, float* slab2, float* cs2, float* slab1, float* cs1, int nframes,
                         int grid, hipStream_t s, int a1_planar);
int conv2_bwd_fr_launch(const __bf16* a1, const __bf16* da2, const __bf16* w2d, __bf16* da1, float* slab,
                        float* cs_slab, int nframes, int grid, hipStream_t s);
int conv3_bwd_fr_launch(const __bf16* a2, const __bf16* da3, const __bf16* a3, const __bf16* w3d, __bf16* da2,
                        float* slab, float* cs_slab, float* cs2, int nframes, int grid, hipStream_t s);

static AtariImpl* impl(AtariNet* n) { return (AtariImpl*)n->impl; }

template <typename T>
static bool dmalloc(AtariImpl* I, T** p, size_t n) {
    if (hipMalloc((void**)p, n * sizeof(T) + 16) != hipSuccess) {
        *p = nullptr;
        return false;
    }
    I->allocs.push_back(*p);
    return true;
}

// split factors (blocks over the reduction) per weight-gradient GEMM
constexpr int SPL_FC = 9, SPL_C3 = 160, SPL_C2 = 256, SPL_C1 = 512;
// the fused conv2 backward + conv1 weight gradient's slabs: conv2 [grid][512][64], then conv1
// [grid][kC1Segs][256][32] (kC1Segs: atari.h, shared with atari_fr.hip's writer)
constexpr int GBM = 128;  // M-tile of the dgrad GEMMs (class stride granularity)

AtariNet* atari_create(int B, int T, int A) {
    if (A < 2 || A > 18) {  // the heads backward keeps a row of A + 1 outputs in registers
        set_error("atari: 2 <= A <= 18 (the full ALE action set is 18)");
        return nullptr;
    }
    AtariNet* n = new AtariNet();
    AtariImpl* I = new AtariImpl();
    n->impl = I;
    n->B = B; n->T = T; n->A = A; n->N = (T + 1) * B;
    I->N = n->N; I->A = A; I->TB = T * B; I->off = Offsets(A);
    const size_t N = n->N;
    I->fr = std::getenv("FI_ATARI_GENERIC") == nullptr;
    I->fuse12 = std::getenv("FI_FWD_UNFUSED") == nullptr;
    I->fuse21 = std::getenv("FI_BWD_UNFUSED") == nullptr;
    I->keep_da1 = std::getenv("FI_KEEP_DA1") != nullptr;
    // only conv21_bwd_fr reads a1 when both fused kernels run; every other consumer wants NHWC
    I->a1_planar = I->fr && I->fuse12 && I->fuse21 && std::getenv("FI_A1_NHWC") == nullptr;
    if (const char* g = std::getenv("FI_FR_GRID")) I->fr_grid = std::max(1, std::min(256, std::atoi(g)));
    I->cs2 = (int)(((N * 100) + GBM - 1) / GBM * GBM);
    I->cs3 = (int)(((N * 81) + GBM - 1) / GBM * GBM);
    bool ok = dmalloc(I, &I->a1, N * 400 * 32) && dmalloc(I, &I->a2, N * 81 * 64) &&
              dmalloc(I, &I->a3, N * 3136) && dmalloc(I, &I->h, N * 512) &&
              dmalloc(I, &I->da1, N * 400 * 32) && dmalloc(I, &I->da2, N * 81 * 64) &&
              dmalloc(I, &I->da3, N * 3136) && dmalloc(I, &I->dh, N * 512) &&
              dmalloc(I, &I->wb.c1T, 32 * 256) && dmalloc(I, &I->wb.c2T, 64 * 512) &&
              dmalloc(I, &I->wb.c3T, 64 * 576) && dmalloc(I, &I->wb.fcT, (size_t)512 * 3136) &&
              dmalloc(I, &I->wb.hT, 32 * 512) && dmalloc(I, &I->wb.c2D, 4 * 32 * 256) &&
              dmalloc(I, &I->wb.c3D, 64 * 576) && dmalloc(I, &I->wb.fcB, (size_t)3136 * 512);
    const size_t s_fc = (size_t)SPL_FC * 3136 * 512, s_c3 = (size_t)SPL_C3 * 576 * 64,
                 s_c2 = (size_t)SPL_C2 * (512 * 64 + kC1Segs * 256 * 32), s_c1 = (size_t)SPL_C1 * 256 * 32,
                 s_h = (size_t)kHeadsGrid * 512 * 19;  // heads_wgrad_valu's [grid][512][O]
    I->slab_floats = std::max(std::max(s_fc, s_c3), std::max(std::max(s_c2, s_c1), s_h)) + 1024 * 512;
    ok = ok && dmalloc(I, &I->slab, I->slab_floats);
    if (!ok) {
        set_error("atari: hipMalloc failed for activations");
        atari_destroy(n);
        return nullptr;
    }
    hipStream_t s0;
    if (hipStreamCreate(&s0) != hipSuccess) {
        set_error("atari: hipStreamCreate failed");
        atari_destroy(n);
        return nullptr;
    }
    // the data-gradient rows T*B.. (dh, da3, da2, da1) are never written by the backward (it walks
    // T*B frames): zeros, so those tensors read as the exact gradients (0) there -- on the
    // creation stream and waited for (no legacy-stream memset racing the learner's stream)
    if (hipMemsetAsync(I->dh, 0, N * 512 * sizeof(__bf16), s0) != hipSuccess ||
        hipMemsetAsync(I->da3, 0, N * 3136 * sizeof(__bf16), s0) != hipSuccess ||
        hipMemsetAsync(I->da2, 0, N * 81 * 64 * sizeof(__bf16), s0) != hipSuccess ||
        hipMemsetAsync(I->da1, 0, N * 400 * 32 * sizeof(__bf16), s0) != hipSuccess || hipStreamSynchronize(s0) != hipSuccess) {
        set_error("atari: hipMemsetAsync failed");
        (void)hipStreamDestroy(s0);
        atari_destroy(n);
        return nullptr;
    }
    (void)hipStreamDestroy(s0);
    return n;
}

void atari_destroy(AtariNet* n) {
    if (!n) return;
    AtariImpl* I = impl(n);
    if (I) {
        for (void* p : I->allocs) (void)hipFree(p);
        delete I;
    }
    delete n;
}

int atari_sync_weights(AtariNet* n, const float* params, hipStream_t s) {
    // fp32 master params -> the bf16 operand layouts of every forward / dgrad GEMM
    AtariImpl* I = impl(n);
    I->params = params;
    hipLaunchKernelGGL(weights_bf16_kernel, dim3(2048), dim3(256), 0, s, params, I->off, I->A, I->wb);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

int atari_forward(AtariNet* n, const uint8_t* frames, float* logits, float* values, hipStream_t s,
                  KernelTagger* tg) {
    AtariImpl* I = impl(n);
    const int N = I->N;
    const float* p = I->params;
    const Offsets& o = I->off;
    using namespace geo;
    int rc;
    if (I->fr && I->fuse12) {
        TagScope ts(tg, "conv12_fwd");
        rc = conv12_fwd_fr_launch(frames, I->wb.c1T, p + o.c1b, I->wb.c2T, p + o.c2b, I->a1, I->a2, N,
                                  std::min(N, I->fr_grid), s, I->a1_planar);
    } else if (I->fr) {
        TagScope ts(tg, "conv1_fwd");
        rc = conv1_fwd_fr_launch(frames, I->wb.c1T, p + o.c1b, I->a1, N, std::min(N, I->fr_grid), s);
    } else { TagScope ts(tg, "conv1_fwd"); rc = gemm<256, 32, 4, 1>(Conv1Gather{frames, N * P1}, RowsBf16{I->wb.c1T, C1O, C1K},
                             EpiAct{I->a1, C1O, p + o.c1b, 1.0f / 255.0f}, N * P1, C1O, C1K, s); }
    if (rc) return rc;
    if (I->fr && I->fuse12) {
        // conv2 ran inside conv12_fwd
    } else if (I->fr) {
        TagScope ts(tg, "conv2_fwd");
        rc = conv2_fwd_fr_launch(I->a1, I->wb.c2T, p + o.c2b, I->a2, N, std::min(N, I->fr_grid), s);
    } else { TagScope ts(tg, "conv2_fwd"); rc = gemm<128, 64, 2, 2>(ConvGather<20, 32, 4, 2, 9>{I->a1, N * P2}, RowsBf16{I->wb.c2T, C2O, C2K},
                             EpiAct{I->a2, C2O, p + o.c2b, 1.0f}, N * P2, C2O, C2K, s); }
    if (rc) return rc;
    if (I->fr) {
        TagScope ts(tg, "conv3_fwd");
        rc = conv3_fwd_fr_launch(I->a2, I->wb.c3T, p + o.c3b, I->a3, N, std::min(N, I->fr_grid), s);
    } else { TagScope ts(tg, "conv3_fwd"); rc = gemm<128, 64, 2, 2>(ConvGather<9, 64, 3, 1, 7>{I->a2, N * P3}, RowsBf16{I->wb.c3T, C3O, C3K},
                             EpiAct{I->a3, C3O, p + o.c3b, 1.0f}, N * P3, C3O, C3K, s); }
    if (rc) return rc;
    {
        TagScope ts(tg, "fc_fwd");
        rc = fc_fwd_launch(I->a3, I->wb.fcT, p + o.fcb, I->h, N, s);
    }
    if (rc) return rc;
    { TagScope ts(tg, "heads_fwd"); rc = gemm<128, 32, 4, 1>(RowsBf16{I->h, N, FCO}, RowsBf16{I->wb.hT, HP, FCO},
                             EpiHeadsOut{logits, values, p + o.hb, I->A}, N, HP, FCO, s); }
    return rc;
}

int atari_backward(AtariNet* n, const uint8_t* frames, const float* dlogits, const float* dvalue,
                   float* grads, hipStream_t s, KernelTagger* tg, GradReadyHook* gr) {
    AtariImpl* I = impl(n);
    const int N = I->N, A = I->A, O = A + 1;
    // the last B frames (t = T) only give the bootstrap value: their dlogits do not exist and
    // their dvalue is 0, so every gradient they would add is exactly 0 -- the frame-resident
    // backward kernels walk the first T*B frames only (dh rows T*B.. stay the zeros written at
    // creation, for the generic path's conv GEMMs that read all N rows)
    const int Nb = I->TB;
    const Offsets& o = I->off;
    using namespace geo;
    float* slab = I->slab;
    float* cs = I->slab + I->slab_floats - 1024 * 512;
    int rc;
#define FI_A(tag, x) do { TagScope ts_(tg, tag); rc = (x); if (rc) return rc; } while (0)
    // heads: wgrad [512][O] + bias, dgrad -> dh (masked by h), both packed-fp32 VALU kernels
    // (K = A + 1 <= 19 is too thin for MFMA); the dgrad also leaves the fc bias partials
    // (column sums of dh) in the slab
    FI_A("heads_wgrad", heads_wgrad_launch(O, dlogits, dvalue, I->h, slab, cs, Nb, I->TB, s));
    FI_A("reduce_slabs", reduce_slabs(slab, kHeadsGrid, (size_t)FCO * O, grads + o.hw, s));
    FI_A("reduce_slabs", reduce_slabs(cs, kHeadsGrid, (size_t)O, grads + o.hb, s));
    FI_A("heads_dgrad", heads_dgrad_launch(O, dlogits, dvalue, I->params + o.hw, I->h, I->dh, Nb, I->TB, slab, s));
    FI_A("reduce_slabs", reduce_slabs(slab, kHeadsDgradGrid, (size_t)FCO, grads + o.fcb, s));
    // fc: wgrad [3136][512] + bias, dgrad -> da3 (masked by a3)
    // fc: wgrad (fc_gemm.hip) as fp32 slabs reduced into the gradient blob, bias = column
    // sums of dh (left by heads dgrad), dgrad -> da3 unmasked (conv3's backward applies the
    // a3 ReLU mask as it loads da3)
    FI_A("fc_wgrad", fc_wgrad_launch(I->a3, I->dh, slab, grads + o.fcw, Nb, s));
    // buckets in reverse layer order: fc + heads (95 % of the gradient bytes) reduce while
    // fc dgrad, conv3 and conv2/conv1 backward run
    if (gr && (rc = gr->ready(o.fcw, o.total - o.fcw))) return rc;
    FI_A("fc_dgrad", fc_dgrad_launch(I->dh, I->wb.fcB, I->da3, I->fr ? Nb : N, s));  // the GEMM path reads all N
    // conv3: wgrad [576][64] + bias, dgrad -> da2 (masked by a2)
    if (I->fr) {
        const int grid = std::min(N, I->fr_grid);
        // conv2's bias partials ([grid][2][64] at cs + 3 grid 64, past c3b [grid][64] and
        // c1b [grid][4][32]) come from conv3_bwd (FI_C2B_C3) or from conv21_bwd
        FI_A("conv3_bwd", conv3_bwd_fr_launch(I->a2, I->da3, I->a3, I->wb.c3D, I->da2, slab, cs, cs + (size_t)3 * grid * C2O,
                                              Nb, grid, s));
        FI_A("reduce_slabs", reduce_slabs(slab, grid, (size_t)C3K * C3O, grads + o.c3w, s));
        FI_A("reduce_slabs", reduce_slabs(cs, grid, (size_t)C3O, grads + o.c3b, s));
        if (gr && (rc = gr->ready(o.c3w, o.fcw - o.c3w))) return rc;
    } else {
        FI_A("relu_mask", relu_mask_bf16(I->da3, I->a3, (size_t)N * FCK, s));
        FI_A("conv3_wgrad", (wgrad<128, 64, 2, 2>(ConvGather<9, 64, 3, 1, 7>{I->a2, N * P3}, RowsBf16{I->da3, N * P3, C3O},
                                   slab, cs, N * P3, C3K, C3O, SPL_C3, 1.f, s)));
        FI_A("reduce_slabs", reduce_slabs(slab, SPL_C3, (size_t)C3K * C3O, grads + o.c3w, s));
        FI_A("reduce_slabs", reduce_slabs(cs, SPL_C3, (size_t)C3O, grads + o.c3b, s));
        FI_A("conv3_dgrad", (gemm<128, 64, 2, 2>(DgradGather<9, 3, 1, 7, 64>{I->da3, N, I->cs3},
                                  ClassRows{I->wb.c3D, 64, C3K, I->cs3, (size_t)64 * C3K, nullptr},
                                  EpiDgrad<9, 1>{I->da2, I->a2, N, I->cs3, 64}, I->cs3, 64, C3K, s)));
        if (gr && (rc = gr->ready(o.c3w, o.fcw - o.c3w))) return rc;
    }
    // conv2 backward + conv1 wgrad fused: da1 stays in LDS (written to HBM only with FI_KEEP_DA1)
    if (I->fr && I->fuse21) {
        const int grid = std::min(N, I->fr_grid);
        float* slab1 = slab + (size_t)grid * C2K * C2O;
        float* cs1 = cs + (size_t)grid * C2O;
        FI_A("conv21_bwd", conv21_bwd_fr_launch(I->a1, I->da2, I->wb.c2D, frames, I->keep_da1 ? I->da1 : nullptr,
                                                slab, cs + (size_t)3 * grid * C2O, slab1, cs1, Nb, grid, s, I->a1_planar));
        FI_A("reduce_slabs", reduce_slabs(slab, grid, (size_t)C2K * C2O, grads + o.c2w, s));
        FI_A("reduce_slabs", reduce_slabs(cs + (size_t)3 * grid * C2O, 2 * grid, (size_t)C2O, grads + o.c2b, s));
        FI_A("reduce_slabs", reduce_slabs(slab1, grid * kC1Segs, (size_t)C1K * C1O, grads + o.c1w, s));
        FI_A("reduce_slabs", reduce_slabs(cs1, 4 * grid, (size_t)C1O, grads + o.c1b, s));
        if (gr && (rc = gr->ready(0, o.c3w))) return rc;
        return FI_OK;
    }
    // conv2: wgrad [512][64] + bias, dgrad -> da1 (4 parity classes, masked by a1)
    if (I->fr) {
        const int grid = std::min(N, I->fr_grid);
        FI_A("conv2_bwd", conv2_bwd_fr_launch(I->a1, I->da2, I->wb.c2D, I->da1, slab, cs + (size_t)3 * grid * C2O, Nb,
                                              grid, s));
        FI_A("reduce_slabs", reduce_slabs(slab, grid, (size_t)C2K * C2O, grads + o.c2w, s));
        // the bias partials in the fused path's layout and place (bit-identical gradients)
        FI_A("reduce_slabs", reduce_slabs(cs + (size_t)3 * grid * C2O, 2 * grid, (size_t)C2O, grads + o.c2b, s));
    } else {
        FI_A("conv2_wgrad", (wgrad<128, 64, 2, 2>(ConvGather<20, 32, 4, 2, 9>{I->a1, N * P2}, RowsBf16{I->da2, N * P2, C2O},
                               slab, cs, N * P2, C2K, C2O, SPL_C2, 1.f, s)));
        FI_A("reduce_slabs", reduce_slabs(slab, SPL_C2, (size_t)C2K * C2O, grads + o.c2w, s));
        FI_A("reduce_slabs", reduce_slabs(cs, SPL_C2, (size_t)C2O, grads + o.c2b, s));
        FI_A("conv2_dgrad", (gemm<128, 32, 4, 1>(DgradGather<20, 4, 2, 9, 64>{I->da2, N, I->cs2},
                              ClassRows{I->wb.c2D, 32, 256, I->cs2, (size_t)32 * 256, nullptr},
                              EpiDgrad<20, 2>{I->da1, I->a1, N, I->cs2, 32}, 4 * I->cs2, 32, 256, s)));
    }
    // conv1: wgrad [256][32] (+1/255 input scale) + bias
    if (I->fr) {
        const int grid = std::min(N, I->fr_grid);
        FI_A("conv1_wgrad", conv1_wgrad_fr_launch(frames, I->da1, slab, cs, Nb, grid, s));
        FI_A("reduce_slabs", reduce_slabs(slab, grid, (size_t)C1K * C1O, grads + o.c1w, s));
        FI_A("reduce_slabs", reduce_slabs(cs, grid, (size_t)C1O, grads + o.c1b, s));
    } else {
        FI_A("conv1_wgrad", (wgrad<128, 32, 4, 1>(Conv1Gather{frames, N * P1}, RowsBf16{I->da1, N * P1, C1O}, slab, cs,
                                   N * P1, C1K, C1O, SPL_C1, 1.0f / 255.0f, s)));
        FI_A("reduce_slabs", reduce_slabs(slab, SPL_C1, (size_t)C1K * C1O, grads + o.c1w, s));
        FI_A("reduce_slabs", reduce_slabs(cs, SPL_C1, (size_t)C1O, grads + o.c1b, s));
    }
    if (gr && (rc = gr->ready(0, o.c3w))) return rc;
#undef FI_A
    return FI_OK;
}

bool atari_tensor(AtariNet* n, const char* name, void** p, size_t* bytes) {
    AtariImpl* I = impl(n);
    const size_t N = I->N;
    struct E {
        const char* nm;
        void* p;
        size_t b;
    } t[] = {{"a1", I->a1, N * 400 * 32 * 2}, {"a2", I->a2, N * 81 * 64 * 2},
             {"a3", I->a3, N * 3136 * 2},     {"h", I->h, N * 512 * 2},
             {"da1", I->da1, N * 400 * 32 * 2}, {"da2", I->da2, N * 81 * 64 * 2},
             {"da3", I->da3, N * 3136 * 2},   {"dh", I->dh, N * 512 * 2}};
    for (auto& e : t)
        if (std::string(e.nm) == name) {
            *p = e.p;
            *bytes = e.b;
            return true;
        }
    return false;
}

}  // namespace fi
