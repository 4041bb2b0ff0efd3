// atari_fr.hip -- frame-resident conv kernels for the Atari policy (gfx950).
//
// The generic implicit GEMM (atari.hip) re-gathers conv inputs per K-tile and waits on
// memory latency every 32-deep K step. Every per-frame conv problem here is small enough
// to keep the WHOLE frame on chip instead: a persistent workgroup stages one frame into
// LDS with fully coalesced 16-byte loads (the next frame's loads are issued before the
// current frame is computed, so HBM latency hides behind a frame of MFMAs), all MFMA
// operands are then read from LDS, and outputs leave through an LDS staging tile as
// coalesced 16-byte stores. HBM traffic is one read of each input byte and one write of
// each output byte.
//
// conv1 (8x8/4, 4 -> 32 channels, u8 frames):
//   LDS frame image: bf16, two "pair planes". A pair = 2 adjacent pixels x 4 channels =
//   16 bytes; pair index q = x/2 goes to plane q&1 at slot y*21 + q/2. A 16-byte global
//   load u of the frame (4 pixels) lands exactly in slot u of both planes. A forward A
//   fragment (8 k = 2 pixels x 4 channels of one tap pair) of output pixel (oy, ox) is
//   plane h, slot (4oy+ky)*21 + ox + (ks&1): consecutive output pixels hit consecutive
//   16-byte slots (including across output-row wraps: 4*21 - 19 = 65 = 1 mod 16), so
//   ds_read_b128 is bank-conflict free.
#include "atari.h"
#include "fi_common.h"
#include "kernels.h"

namespace fi {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

namespace c1 {
constexpr int FRAME_LOADS = 84 * 84 * 4 / 16;       // 1764 16-byte loads per frame
constexpr int PER_T = (FRAME_LOADS + 255) / 256;    // 7
constexpr int PLANE = 84 * 21 * 16 + 64;            // bytes (+64: plane 1 shifted 4 slots)
constexpr int IMG = 2 * PLANE;                      // 56,576 B
constexpr int OUT = 400 * 32 * 2;                   // 25,600 B output / dY tile
constexpr int OUT_CH = OUT / 16;                    // 1600 16-byte chunks
constexpr int OUT_PER_T = (OUT_CH + 255) / 256;     // 7
}  // namespace c1

__device__ __forceinline__ void u8x16_to_bf16(u32x4 v, bf16x8& lo, bf16x8& hi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lo[j] = (__bf16)(float)((v[j >> 2] >> (8 * (j & 3))) & 0xffu);
        hi[j] = (__bf16)(float)((v[2 + (j >> 2)] >> (8 * (j & 3))) & 0xffu);
    }
}

__device__ __forceinline__ void c1_fetch_frame(const uint8_t* fr, u32x4 (&r)[c1::PER_T]) {
    const u32x4* src = (const u32x4*)fr;
#pragma unroll
    for (int i = 0; i < c1::PER_T; ++i) {
        const int u = threadIdx.x + 256 * i;
        r[i] = u < c1::FRAME_LOADS ? __builtin_nontemporal_load(src + u) : u32x4{0, 0, 0, 0};
    }
}

__device__ __forceinline__ void c1_store_image(char* img, const u32x4 (&r)[c1::PER_T]) {
#pragma unroll
    for (int i = 0; i < c1::PER_T; ++i) {
        const int u = threadIdx.x + 256 * i;
        if (u < c1::FRAME_LOADS) {
            bf16x8 lo, hi;
            u8x16_to_bf16(r[i], lo, hi);
            *(bf16x8*)(img + 16 * u) = lo;
            *(bf16x8*)(img + c1::PLANE + 16 * u) = hi;
        }
    }
}

// ---------------------------------------------------------------------------------
// conv1 forward: a1[f] = bf16(relu(conv(frames[f]) / 255 + b)), persistent over frames
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 1) void conv1_fwd_fr(const uint8_t* __restrict__ frames,
                                                       const __bf16* __restrict__ w1t,  // [32][256]
                                                       const float* __restrict__ bias,
                                                       __bf16* __restrict__ a1, int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c1::IMG + c1::OUT];
    char* img = smem;
    __bf16* out = (__bf16*)(smem + c1::IMG);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, col = lane & 31;
    // B fragments of all 16 K-steps stay in registers: lane holds W[n=col][k=16ks+8h..+8]
    bf16x8 bw[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bw[ks] = *(const bf16x8*)(w1t + col * 256 + ks * 16 + h * 8);
    const float bcol = bias[col];
    const float inv255 = 1.0f / 255.0f;

    u32x4 pre[c1::PER_T];
    int f = blockIdx.x;
    if (f < nframes) c1_fetch_frame(frames + (size_t)f * 28224, pre);
    for (; f < nframes; f += gridDim.x) {
        c1_store_image(img, pre);
        const int fn = f + gridDim.x;
        if (fn < nframes) c1_fetch_frame(frames + (size_t)fn * 28224, pre);
        __syncthreads();  // image ready, previous out tile drained
        // 13 row tiles of 32 output pixels: wave w takes tiles w, w+4, ...
        for (int t = w; t < 13; t += 4) {
            const int m = min(t * 32 + col, 399);
            const int oy = m / 20, ox = m - oy * 20;
            const char* abase = img + h * c1::PLANE + 16 * (oy * 4 * 21 + ox);
            f32x16 acc = {};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                const bf16x8 a = *(const bf16x8*)(abase + 16 * ((ks >> 1) * 21 + (ks & 1)));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bw[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < 400) out[row * 32 + col] = (__bf16)fmaxf(acc[r] * inv255 + bcol, 0.f);
            }
        }
        __syncthreads();  // out tile complete, image free
        u32x4* dst = (u32x4*)(a1 + (size_t)f * 12800);
#pragma unroll
        for (int i = 0; i < c1::OUT_PER_T; ++i) {
            const int c = threadIdx.x + 256 * i;
            if (c < c1::OUT_CH) __builtin_nontemporal_store(((const u32x4*)out)[c], dst + c);
        }
    }
}

// ---------------------------------------------------------------------------------
// conv1 weight gradient: dW1[k][co] = 1/255 sum_{f,m} im2col(frame_f)[m][k] da1_f[m][co]
// A^T fragments come from the frame image through ds_read_b64_tr_b16 with per-lane
// gather addresses (each lane names one output pixel's 4 channels of one tap); da1 is
// staged as [m][co] and read the same way. Each workgroup accumulates over its frames in
// registers and writes one fp32 partial slab [256][32] + bias partial [32].
// ---------------------------------------------------------------------------------
__device__ __forceinline__ bf16x8 tr2(const char* p0, const char* p1) {
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p1);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ __launch_bounds__(256, 1) void conv1_wgrad_fr(const uint8_t* __restrict__ frames,
                                                         const __bf16* __restrict__ da1,
                                                         float* __restrict__ slab,
                                                         float* __restrict__ cs_slab, int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c1::IMG + c1::OUT];
    char* img = smem;
    char* dy = smem + c1::IMG;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    // per-lane tr-read column: k = k0 + 16*(g&1) + 4p, i.e. tap = k0/4 + 4*(g&1) + p
    f32x16 acc0 = {}, acc1 = {};
    float csum[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // bias grad partial: co = 8*(chunk%4) + j

    u32x4 pre[c1::PER_T], pdy[c1::OUT_PER_T];
    auto fetch = [&](int ff) {
        c1_fetch_frame(frames + (size_t)ff * 28224, pre);
        const u32x4* s = (const u32x4*)(da1 + (size_t)ff * 12800);
#pragma unroll
        for (int i = 0; i < c1::OUT_PER_T; ++i) {
            const int c = threadIdx.x + 256 * i;
            pdy[i] = c < c1::OUT_CH ? __builtin_nontemporal_load(s + c) : u32x4{0, 0, 0, 0};
        }
    };
    // tap geometry of this lane for the two k-tiles of this wave (k0 = 64w + 32t)
    int toff[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int tap = (64 * w + 32 * t) / 4 + 4 * (g & 1) + p;
        const int ky = tap >> 3, kx = tap & 7;
        toff[t] = ky * 84 + kx;  // pixel offset of the tap relative to (4oy, 4ox)
    }
    // frame-invariant per-lane LDS offsets of every transposed read: A [ms][t][lo/hi], B [ms][lo/hi]
    int wao[25][2][2], wbo[25][2];
#pragma unroll
    for (int ms = 0; ms < 25; ++ms) {
        const int m_lo = ms * 16 + 8 * (g >> 1) + q;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int m = m_lo + 4 * hh;
            const int oy = m / 20, ox = m - oy * 20;
            wbo[ms][hh] = m * 64 + (16 * (g & 1) + 4 * p) * 2;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int P = oy * 4 * 84 + ox * 4 + toff[t];
                const int y = P / 84, x = P - y * 84;
                wao[ms][t][hh] = ((x >> 1) & 1) * c1::PLANE + 16 * (y * 21 + (x >> 2)) + 8 * (x & 1);
            }
        }
    }
    int f = blockIdx.x;
    if (f < nframes) fetch(f);
    for (; f < nframes; f += gridDim.x) {
        c1_store_image(img, pre);
#pragma unroll
        for (int i = 0; i < c1::OUT_PER_T; ++i) {
            const int c = threadIdx.x + 256 * i;
            if (c < c1::OUT_CH) {
                *(u32x4*)(dy + 16 * c) = pdy[i];
                const bf16x8 v = __builtin_bit_cast(bf16x8, pdy[i]);
#pragma unroll
                for (int j = 0; j < 8; ++j) csum[j] += (float)v[j];
            }
        }
        const int fn = f + gridDim.x;
        if (fn < nframes) fetch(fn);
        __syncthreads();
#pragma unroll
        for (int ms = 0; ms < 25; ++ms) {
            const bf16x8 bfr = tr2(dy + wbo[ms][0], dy + wbo[ms][1]);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr2(img + wao[ms][0][0], img + wao[ms][0][1]), bfr, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr2(img + wao[ms][1][0], img + wao[ms][1][1]), bfr, acc1, 0, 0, 0);
        }
        __syncthreads();
    }
    // partial slab: rows k = 64w + 32t + (r&3) + 8(r>>2) + 4(lane>>5), col co = lane&31
    float* out = slab + (size_t)blockIdx.x * 256 * 32;
    const float inv255 = 1.0f / 255.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = 64 * w + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        out[k * 32 + (lane & 31)] = acc0[r] * inv255;
        out[(k + 32) * 32 + (lane & 31)] = acc1[r] * inv255;
    }
    // bias partial: thread's chunks all have co octet = (threadIdx.x % 4) (256 % 4 == 0)
    __syncthreads();
    float* red = (float*)smem;  // [256][8]
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = csum[j];
    __syncthreads();
    if (threadIdx.x < 32) {
        const int oct = threadIdx.x >> 3, j = threadIdx.x & 7;
        float s = 0.f;
        for (int t = oct; t < 256; t += 4) s += red[t * 8 + j];
        cs_slab[(size_t)blockIdx.x * 32 + threadIdx.x] = s;
    }
}

int conv1_fwd_fr_launch(const uint8_t* frames, const __bf16* w1t, const float* bias, __bf16* a1,
                        int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv1_fwd_fr, dim3(grid), dim3(256), 0, s, frames, w1t, bias, a1, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

int conv1_wgrad_fr_launch(const uint8_t* frames, const __bf16* da1, float* slab, float* cs_slab,
                          int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv1_wgrad_fr, dim3(grid), dim3(256), 0, s, frames, da1, slab, cs_slab, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}


// =====================================================================================
// conv2 backward, fused and frame-resident (4x4 / stride 2, 32 -> 64 channels, 20x20 -> 9x9)
//   in : X = a1[f] (20,20,32) bf16 (layer input = ReLU mask),  dY = da2[f] (9,9,64) bf16
//   out: da1[f] = (X > 0) * dgrad(dY, W2)   (written in place over X in LDS, then stored)
//        dW2 += im2col(X)^T dY  (512 x 64, registers across frames),  db2 += sum dY
// LDS ring of 3 frames, filled by LDS-DMA (global_load_lds_dwordx4), counted vmcnt.
//   X image : pixel p at 256*(p>>2) + 64*sigma(p), sigma(p) = ((p&3) + ((p>>2)&1)) & 3
//             -> the four stride-2 pixels a transposed read gathers sit in different
//                quarters of a 256-byte bank row (conflict-free ds_read_b64_tr_b16)
//   dY tile : row r (output pixel) at 128*r, 16-byte chunk c at 16*(c ^ f(r)),
//             f(r) = (((r>>1)&1)<<2) | ((r>>2)&3): conflict-free both for the b128 row
//             reads of the dgrad and the transposed reads of the wgrad.
// wgrad: wave w owns taps (ky=w, kx=0..3) = k rows [128w, 128w+128) x 64 co.
// dgrad: wave w owns parity class (py, px) = (w>>1, w&1): 100 input pixels (4 row tiles),
//        K = (ty, tx, co) = 256, W2 class slice kept in registers (64 VGPRs).
// =====================================================================================
namespace c2 {
constexpr int XB = 20 * 20 * 32 * 2;         // 25,600
constexpr int DYROWS = 96;                   // 81 rows padded to 6 MFMA K-steps
constexpr int DYB = DYROWS * 128;            // 12,288
constexpr int SLOT = XB + DYB;               // 37,888
constexpr int RING = 3;
constexpr int NX = XB / 1024;                // 25 LDS-DMA pieces (1 KiB each)
constexpr int NDY = DYB / 1024;              // 12
constexpr int NPIECE = NX + NDY;             // 37
constexpr int OUT_CH = XB / 16;              // 1600 16-byte chunks of da1
constexpr int OUTT = 4 * 128 * 32 * 2;       // 32 KiB dgrad tile in accumulator order
}  // namespace c2

__device__ __forceinline__ int c2_sigma(int p) { return ((p & 3) + ((p >> 2) & 1)) & 3; }
__device__ __forceinline__ int c2_xaddr(int p) { return 256 * (p >> 2) + 64 * c2_sigma(p); }
__device__ __forceinline__ int c2_f(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int c2_dyaddr(int r, int c) { return 128 * r + 16 * (c ^ c2_f(r)); }

__device__ __forceinline__ void c2_issue(const __bf16* x, const __bf16* dy, uint32_t slot_lds,
                                         int w, int lane) {
#pragma unroll
    for (int i = 0; i < (c2::NPIECE + 3) / 4; ++i) {
        const int j = w + 4 * i;
        if (j >= c2::NPIECE) break;
        if (j < c2::NX) {
            const int P = j * 64 + lane;  // physical 16-byte piece of the X image
            const int G = P >> 4, s = (P >> 2) & 3, c = P & 3;
            const int p = 4 * G + ((s - (G & 1)) & 3);
            glds16((const char*)x + p * 64 + c * 16, slot_lds + j * 1024);
        } else {
            const int P = (j - c2::NX) * 64 + lane;  // physical piece of the dY tile
            const int r = P >> 3, pc = P & 7;
            const int rs = r < 81 ? r : 80;
            glds16((const char*)dy + rs * 128 + 16 * (pc ^ c2_f(r)), slot_lds + c2::XB + (j - c2::NX) * 1024);
        }
    }
}

__global__ __launch_bounds__(256, 1) void conv2_bwd_fr(const __bf16* __restrict__ a1,
                                                       const __bf16* __restrict__ da2,
                                                       const __bf16* __restrict__ w2d,  // [4][32][256]
                                                       __bf16* __restrict__ da1,
                                                       float* __restrict__ slab,   // [grid][512][64]
                                                       float* __restrict__ cs_slab,  // [grid][64]
                                                       int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c2::RING * c2::SLOT + c2::OUTT];
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, h = lane >> 5, col = lane & 31;
    __bf16* outt = (__bf16*)(smem + c2::RING * c2::SLOT);  // [cls][128][32], unmasked dX
    const uint32_t lds0 = lds_addr(smem);

    // dgrad B fragments (class w): W[k = 16ks + 8h + j][ci = col]
    bf16x8 bw[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bw[ks] = *(const bf16x8*)(w2d + ((size_t)(w * 32 + col)) * 256 + ks * 16 + h * 8);
    f32x16 accw[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) { accw[t][0] = f32x16{}; accw[t][1] = f32x16{}; }
    float bsum0 = 0.f, bsum1 = 0.f;

    // ---- frame-invariant LDS addresses (byte offsets inside a ring slot), per lane
    // wgrad B (dY, tr reads): [ms][ct][lo/hi]
    int wb_addr[6][2][2];
    // wgrad A (X image, tr reads): [ms][tap kx][lo/hi]
    int wa_addr[6][4][2];
#pragma unroll
    for (int ms = 0; ms < 6; ++ms) {
        const int mlo = ms * 16 + 8 * (g >> 1) + q, mhi = mlo + 4;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const int c = 4 * ct + 2 * (g & 1) + (p4 >> 1);
            wb_addr[ms][ct][0] = c2::XB + c2_dyaddr(mlo, c) + 8 * (p4 & 1);
            wb_addr[ms][ct][1] = c2::XB + c2_dyaddr(mhi, c) + 8 * (p4 & 1);
        }
        const int ml = min(mlo, 80), mh = min(mhi, 80);
        const int oyl = ml / 9, oxl = ml - oyl * 9, oyh = mh / 9, oxh = mh - oyh * 9;
        const int ci = 16 * (g & 1) + 4 * p4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            wa_addr[ms][t][0] = c2_xaddr((2 * oyl + w) * 20 + 2 * oxl + t) + 2 * ci;
            wa_addr[ms][t][1] = c2_xaddr((2 * oyh + w) * 20 + 2 * oxh + t) + 2 * ci;
        }
    }
    // lanes whose B rows m = 80 + 8*(g>>1) + j pass 81 in the last K-step get zeroed there
    const int mb5 = 80 + 8 * (g >> 1);
    // dgrad A (dY rows, b128): [rt][ks] address and validity bit
    int da_addr[4][16];
    uint64_t da_ok = 0;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
        const int r = min(rt * 32 + col, 99);
        const int iyq = r / 10, ixq = r - iyq * 10;
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
            const int tap = ks >> 2, ty = tap >> 1, tx = tap & 1;
            const int oy = iyq - ty, ox = ixq - tx;
            const bool ok = oy >= 0 && ox >= 0 && oy < 9 && ox < 9;
            da_addr[rt][ks] = c2::XB + c2_dyaddr(ok ? oy * 9 + ox : 0, 2 * (ks & 3) + h);
            if (ok) da_ok |= 1ull << (rt * 16 + ks);
        }
    }
    const int npw = (c2::NPIECE - w + 3) / 4;  // LDS-DMA pieces per wave per frame
    constexpr int STORES = c2::OUT_CH / 256;   // 6 store instructions every wave surely issues
    int issued = 0, m0 = 0, m1 = 0, m2 = 0;
    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    for (int i = 0; i < 3 && i < nmine; ++i) {
        const int f = blockIdx.x + i * gridDim.x;
        c2_issue(a1 + (size_t)f * 12800, da2 + (size_t)f * 5184, lds0 + i * c2::SLOT, w, lane);
        issued += npw;
        if (i == 0) m0 = issued; else if (i == 1) m1 = issued; else m2 = issued;
    }
    for (int it = 0; it < nmine; ++it) {
        const int f = blockIdx.x + it * gridDim.x;
        const int slot = it % 3;
        char* X = smem + slot * c2::SLOT;
        wait_vmcnt(issued - m0);
        lds_barrier();

        // ---------------- weight gradient: A^T = im2col(X) (tr reads), B = dY (tr reads)
#pragma unroll
        for (int ms = 0; ms < 6; ++ms) {
            bf16x8 bfr[2];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                bf16x8 v = tr2(X + wb_addr[ms][ct][0], X + wb_addr[ms][ct][1]);
                if (ms == 5) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (mb5 + j >= 81) v[j] = (__bf16)0.f;
                }
                bfr[ct] = v;
                if (w == 0) {
                    float sacc = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) sacc += (float)v[j];
                    if (ct == 0) bsum0 += sacc; else bsum1 += sacc;
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const bf16x8 afr = tr2(X + wa_addr[ms][t][0], X + wa_addr[ms][t][1]);
                accw[t][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, bfr[0], accw[t][0], 0, 0, 0);
                accw[t][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, bfr[1], accw[t][1], 0, 0, 0);
            }
        }

        // ---------------- data gradient of class (py, px): rows = 100 input pixels
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
            f32x16 acc = {};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                bf16x8 a = *(const bf16x8*)(X + da_addr[rt][ks]);
                if (!((da_ok >> (rt * 16 + ks)) & 1)) a = bf16x8{};
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bw[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ri = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                outt[(w * 128 + ri) * 32 + col] = (__bf16)acc[r];
            }
        }
        lds_barrier();  // dgrad tile complete
        {  // da1 = (X > 0) * dX, in NHWC order: chunk P = pixel P/4, channels 8*(P%4)..+8
            u32x4* dst = (u32x4*)(da1 + (size_t)f * 12800);
#pragma unroll
            for (int i = 0; i < (c2::OUT_CH + 255) / 256; ++i) {
                const int P = threadIdx.x + 256 * i;
                if (P < c2::OUT_CH) {
                    const int pix = P >> 2, c = P & 3;
                    const int iy = pix / 20, ix = pix - iy * 20;
                    const int cls = ((iy & 1) << 1) | (ix & 1), ri = (iy >> 1) * 10 + (ix >> 1);
                    const bf16x8 v = *(const bf16x8*)(outt + (cls * 128 + ri) * 32 + 8 * c);
                    const bf16x8 m = *(const bf16x8*)(X + c2_xaddr(pix) + 16 * c);
                    bf16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] = (float)m[j] > 0.f ? v[j] : (__bf16)0.f;
                    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), dst + P);
                }
            }
            issued += STORES;  // (wave 0 issues one more; counting fewer only waits longer)
        }
        lds_barrier();  // slot fully consumed
        int m3 = 0;
        if (it + 3 < nmine) {
            const int fn = blockIdx.x + (it + 3) * gridDim.x;
            c2_issue(a1 + (size_t)fn * 12800, da2 + (size_t)fn * 5184, lds0 + slot * c2::SLOT, w, lane);
            issued += npw;
            m3 = issued;
        }
        m0 = m1;
        m1 = m2;
        m2 = m3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // weight-gradient partial: k = 128w + 32t + row, co = 32ct + col
    float* out = slab + (size_t)blockIdx.x * 512 * 64;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 128 * w + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
                out[k * 64 + 32 * ct + col] = accw[t][ct][r];
            }
    // bias: wave 0 lanes l and l+32 hold the same co (16*(g&1) + (l&15)), different m halves
    if (w == 0) {
        const float o0 = __shfl_xor(bsum0, 32, 64), o1 = __shfl_xor(bsum1, 32, 64);
        if (lane < 32) {
            cs_slab[(size_t)blockIdx.x * 64 + lane] = bsum0 + o0;
            cs_slab[(size_t)blockIdx.x * 64 + 32 + lane] = bsum1 + o1;
        }
    }
}

int conv2_bwd_fr_launch(const __bf16* a1, const __bf16* da2, const __bf16* w2d, __bf16* da1,
                        float* slab, float* cs_slab, int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv2_bwd_fr, dim3(grid), dim3(256), 0, s, a1, da2, w2d, da1, slab, cs_slab,
                       nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}


// =====================================================================================
// conv3 backward, fused and frame-resident (3x3 / stride 1, 64 -> 64 channels, 9x9 -> 7x7)
//   in : X = a2[f] (9,9,64), dY = da3[f] (7,7,64);  out: da2[f] = (X>0) * dgrad(dY, W3),
//        dW3 (576 x 64) and db3 accumulated in registers across frames.
// X image : pixel p at 128p, its 64-byte channel halves swapped when (p>>1)&1 -> the four
//           consecutive pixels of a transposed read land in distinct bank quarters.
// dY tile : 64 rows (49 valid) x 128 B, chunk swizzle c ^ f(r) as in conv2.
// wgrad: 32x32x16 MFMA, k-tile kt = (tap, 32-channel half), waves take kt = w, w+4, ...
// dgrad: 16x16x32 MFMA, wave w owns input channels 16w..16w+15 for all 6 row tiles of 16
//        input pixels; its W3 slice (18 K-steps) lives in registers; taps that fall
//        outside the 7x7 output read a 16-byte zero row instead of being masked.
// =====================================================================================
namespace c3 {
constexpr int XB = 11 * 1024;                // 81 px * 128 B = 10,368, padded to 11 KiB
constexpr int DYB = 64 * 128;                // 8 KiB
constexpr int SLOT = XB + DYB;               // 19,456
constexpr int RING = 3;
constexpr int NX = 11, NDY = 8, NPIECE = NX + NDY;   // 19 LDS-DMA pieces
constexpr int OUTT = 96 * 128;               // dgrad tile [96 rows][64 ci] bf16
constexpr int ZERO = 64;                     // zero row (16 B used)
constexpr int OUT_CH = 81 * 8;               // 648 16-byte chunks of da2
}  // namespace c3

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int c3_xaddr(int p, int ci) {  // byte offset of (pixel, channel)
    return 128 * p + 64 * ((ci >> 5) ^ ((p >> 1) & 1)) + 2 * (ci & 31);
}

__device__ __forceinline__ void c3_issue(const __bf16* x, const __bf16* dy, uint32_t slot_lds,
                                         int w, int lane) {
#pragma unroll
    for (int i = 0; i < (c3::NPIECE + 3) / 4; ++i) {
        const int j = w + 4 * i;
        if (j >= c3::NPIECE) break;
        if (j < c3::NX) {
            const int P = j * 64 + lane;         // physical 16-byte piece of the X image
            const int p = min(P >> 3, 80), pc = P & 7;
            const int lc = 4 * ((pc >> 2) ^ ((p >> 1) & 1)) + (pc & 3);  // logical chunk
            glds16((const char*)x + p * 128 + 16 * lc, slot_lds + j * 1024);
        } else {
            const int P = (j - c3::NX) * 64 + lane;
            const int r = P >> 3, pc = P & 7;
            const int rs = r < 49 ? r : 48;
            glds16((const char*)dy + rs * 128 + 16 * (pc ^ c2_f(r)), slot_lds + c3::XB + (j - c3::NX) * 1024);
        }
    }
}

__global__ __launch_bounds__(256, 1) void conv3_bwd_fr(const __bf16* __restrict__ a2,
                                                       const __bf16* __restrict__ da3,
                                                       const __bf16* __restrict__ w3d,  // [64 ci][576]
                                                       __bf16* __restrict__ da2,
                                                       float* __restrict__ slab,     // [grid][576][64]
                                                       float* __restrict__ cs_slab,  // [grid][64]
                                                       int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c3::RING * c3::SLOT + c3::OUTT + c3::ZERO];
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, h = lane >> 5;
    const uint32_t lds0 = lds_addr(smem);
    __bf16* outt = (__bf16*)(smem + c3::RING * c3::SLOT);
    char* zero = smem + c3::RING * c3::SLOT + c3::OUTT;
    if (threadIdx.x < 16) ((uint32_t*)zero)[threadIdx.x] = 0u;

    // dgrad B (16x16x32): lane holds W[k = 32ks + 8*(lane>>4) + j][ci = 16w + (lane&15)]
    s16x8 bw[18];
#pragma unroll
    for (int ks = 0; ks < 18; ++ks)
        bw[ks] = *(const s16x8*)(w3d + (size_t)(16 * w + (lane & 15)) * 576 + 32 * ks + 8 * g);

    // ---- frame-invariant per-lane LDS offsets (relative to the slot base)
    int wb_addr[4][2][2];  // wgrad B tr reads [ms][ct][lo/hi]
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
        const int mlo = ms * 16 + 8 * (g >> 1) + q, mhi = mlo + 4;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const int c = 4 * ct + 2 * (g & 1) + (p4 >> 1);
            wb_addr[ms][ct][0] = c3::XB + c2_dyaddr(mlo, c) + 8 * (p4 & 1);
            wb_addr[ms][ct][1] = c3::XB + c2_dyaddr(mhi, c) + 8 * (p4 & 1);
        }
    }
    const int mb3 = 48 + 8 * (g >> 1);  // last K-step: element j <-> m = mb3 + j
    int wa_addr[5][4][2];  // wgrad A tr reads [i-th k-tile of this wave][ms][lo/hi]
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int kt = min(w + 4 * i, 17);
        const int tap = kt >> 1, ky = tap / 3, kx = tap - 3 * ky;
        const int ci = 32 * (kt & 1) + 16 * (g & 1) + 4 * p4;
#pragma unroll
        for (int ms = 0; ms < 4; ++ms) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int m = min(ms * 16 + 8 * (g >> 1) + q + 4 * hh, 48);
                const int oy = m / 7, ox = m - 7 * oy;
                wa_addr[i][ms][hh] = c3_xaddr((oy + ky) * 9 + ox + kx, ci);
            }
        }
    }
    const int nkt = (18 - w + 3) / 4;  // k-tiles of this wave: 5,5,4,4
    // dgrad A (16x16x32): row = input pixel rt*16 + (lane&15), k = 32ks + 8g -> tap ks>>1
    uint32_t da_addr[6][9];  // [rt][tap] byte offset of the dY row (or the zero row) + chunk base
#pragma unroll
    for (int rt = 0; rt < 6; ++rt) {
        const int pix = min(rt * 16 + (lane & 15), 80);
        const int iy = pix / 9, ix = pix - 9 * iy;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap - 3 * ky;
            const int oy = iy - ky, ox = ix - kx;
            const bool ok = oy >= 0 && ox >= 0 && oy < 7 && ox < 7;
            da_addr[rt][tap] = ok ? (uint32_t)((oy * 7 + ox) | 0x10000) : 0u;  // row | valid
        }
    }

    f32x16 accw[5][2];
#pragma unroll
    for (int i = 0; i < 5; ++i) { accw[i][0] = f32x16{}; accw[i][1] = f32x16{}; }
    float bsum0 = 0.f, bsum1 = 0.f;

    const int npw = (c3::NPIECE - w + 3) / 4;
    constexpr int STORES = c3::OUT_CH / 256;  // 2 (waves 0..1 issue a third)
    int issued = 0, m0 = 0, m1 = 0, m2 = 0;
    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    for (int i = 0; i < 3 && i < nmine; ++i) {
        const int f = blockIdx.x + i * gridDim.x;
        c3_issue(a2 + (size_t)f * 5184, da3 + (size_t)f * 3136, lds0 + i * c3::SLOT, w, lane);
        issued += npw;
        if (i == 0) m0 = issued; else if (i == 1) m1 = issued; else m2 = issued;
    }
    for (int it = 0; it < nmine; ++it) {
        const int f = blockIdx.x + it * gridDim.x;
        const int slot = it % 3;
        char* X = smem + slot * c3::SLOT;
        wait_vmcnt(issued - m0);
        lds_barrier();

        // ---------------- weight gradient (32x32x16, tr reads)
#pragma unroll
        for (int ms = 0; ms < 4; ++ms) {
            bf16x8 bfr[2];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                bf16x8 v = tr2(X + wb_addr[ms][ct][0], X + wb_addr[ms][ct][1]);
                if (ms == 3) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (mb3 + j >= 49) v[j] = (__bf16)0.f;
                }
                bfr[ct] = v;
                if (w == 0) {
                    float sacc = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) sacc += (float)v[j];
                    if (ct == 0) bsum0 += sacc; else bsum1 += sacc;
                }
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                if (i < nkt) {
                    const bf16x8 afr = tr2(X + wa_addr[i][ms][0], X + wa_addr[i][ms][1]);
                    accw[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, bfr[0], accw[i][0], 0, 0, 0);
                    accw[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, bfr[1], accw[i][1], 0, 0, 0);
                }
            }
        }

        // ---------------- data gradient (16x16x32): channels 16w.., 6 row tiles
#pragma unroll
        for (int rt = 0; rt < 6; ++rt) {
            f32x4 acc = {};
#pragma unroll
            for (int ks = 0; ks < 18; ++ks) {
                const uint32_t e = da_addr[rt][ks >> 1];
                const int row = e & 0xffff;
                const int c = 4 * (ks & 1) + g;  // co chunk: co0 = 32*(ks&1) + 8g
                const char* src = (e >> 16) ? X + c3::XB + c2_dyaddr(row, c) : zero;
                const s16x8 a = *(const s16x8*)src;
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                             __builtin_bit_cast(bf16x8, bw[ks]), acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rt * 16 + 4 * g + r;
                outt[row * 64 + 16 * w + (lane & 15)] = (__bf16)acc[r];
            }
        }
        lds_barrier();  // dgrad tile complete
        {
            u32x4* dst = (u32x4*)(da2 + (size_t)f * 5184);
#pragma unroll
            for (int i = 0; i < (c3::OUT_CH + 255) / 256; ++i) {
                const int P = threadIdx.x + 256 * i;
                if (P < c3::OUT_CH) {
                    const int pix = P >> 3, c = P & 7;
                    const bf16x8 v = *(const bf16x8*)(outt + pix * 64 + 8 * c);
                    const bf16x8 m = *(const bf16x8*)(X + c3_xaddr(pix, 8 * c));
                    bf16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] = (float)m[j] > 0.f ? v[j] : (__bf16)0.f;
                    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), dst + P);
                }
            }
            issued += STORES;
        }
        lds_barrier();  // slot fully consumed
        int m3 = 0;
        if (it + 3 < nmine) {
            const int fn = blockIdx.x + (it + 3) * gridDim.x;
            c3_issue(a2 + (size_t)fn * 5184, da3 + (size_t)fn * 3136, lds0 + slot * c3::SLOT, w, lane);
            issued += npw;
            m3 = issued;
        }
        m0 = m1;
        m1 = m2;
        m2 = m3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float* out = slab + (size_t)blockIdx.x * 576 * 64;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        if (i < nkt) {
            const int kt = w + 4 * i;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int k = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h;
                    out[k * 64 + 32 * ct + (lane & 31)] = accw[i][ct][r];
                }
        }
    }
    if (w == 0) {
        const float o0 = __shfl_xor(bsum0, 32, 64), o1 = __shfl_xor(bsum1, 32, 64);
        if (lane < 32) {
            cs_slab[(size_t)blockIdx.x * 64 + lane] = bsum0 + o0;
            cs_slab[(size_t)blockIdx.x * 64 + 32 + lane] = bsum1 + o1;
        }
    }
}

int conv3_bwd_fr_launch(const __bf16* a2, const __bf16* da3, const __bf16* w3d, __bf16* da2,
                        float* slab, float* cs_slab, int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv3_bwd_fr, dim3(grid), dim3(256), 0, s, a2, da3, w3d, da2, slab, cs_slab,
                       nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

}  // namespace fi
