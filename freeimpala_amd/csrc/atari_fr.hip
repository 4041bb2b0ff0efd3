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
#include <type_traits>

#include "atari.h"
#include "fi_common.h"
#include "kernels.h"

namespace fi {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;



namespace c1 {
constexpr int FRAME_LOADS = 84 * 84 * 4 / 16;       // 1764 16-byte loads per frame
constexpr int PLANE = 84 * 21 * 16 + 64;            // bytes (+64: plane 1 shifted 4 slots)
constexpr int IMG = 2 * PLANE;                      // 56,576 B
constexpr int OUT = 400 * 32 * 2;                   // 25,600 B output / dY tile
}  // namespace c1

// Where the bias sums go (A/B switches; the layout of the partials is the same either way):
//   FI_C2B_C3   conv2's bias partials summed by conv3_bwd's data-gradient epilogue (from the da2
//               it stores) instead of by conv21's weight-gradient waves (48 v_dot2 per frame)
//   FI_C1B_PH2  conv1's bias partials from the B fragments of conv1's weight gradient in phase 2
//               (m-steps split over the four waves at compile time) instead of the phase-1
//               epilogue (16 VALU per tile)
//   FI_C21_PKMASK  the da1 ReLU mask per 32-bit word (relu_mask_pair) instead of per element
#ifndef FI_C2B_C3
#define FI_C2B_C3 0
#endif
#ifndef FI_C1B_PH2
#define FI_C1B_PH2 1
#endif
#ifndef FI_C21_PKMASK
#define FI_C21_PKMASK 1
#endif

// Blocked fp32 accumulation of conv1's persistent weight gradient. A workgroup walks ~1,616
// frames at the bench size; one fp32 accumulator chain over all of them (25 MFMA steps per
// frame, ~40k accumulate roundings per element) measured 1.8e-5 relative L2 against fp64
// (tests/test_gpu_atari.py, full size) -- over SURVEY.md's 1e-5 bar. conv21_bwd_fr's conv1 waves
// therefore write a partial slab at the end of each of SEGS contiguous segments of their frames
// (segment k ends after frame seg_last(k); empty segments write zero slabs) and reduce_slabs sums
// them in a fixed order. conv2's weight gradient (6 MFMA steps per frame) stays one chain: it
// measures 1.3e-6 with two segments and is within the bar whole. Measured alternatives
// (profiles/r05_blocked_accumulation_ab.txt): a second conv1 register set, conv2 slabs flushed
// from inside the frame loop, and both roles walking a segment loop nest cost conv21 0.14, 0.17
// and 0.5 ms.
constexpr int SEGS = kC1Segs;  // atari.h: the slab count atari.hip allocates and reduces
__device__ __forceinline__ int seg_last(int k, int nmine) { return ((k + 1) * nmine) / SEGS - 1; }

// one conv2 weight-gradient slab [512][64] from a wave's accumulators (kernel row wr), zeroing
// them; with `drain` the stores (and every other outstanding VMEM op of the wave) complete
// before the frame loop's counted vmcnt waits resume
// (buffer stores: one per-lane offset register, the wave-uniform rest in soffset -- 128 flat
// stores with 64-bit addresses each spilled the frame loop's registers)
__device__ __forceinline__ void c2w_flush(f32x16 (&accw)[4][2], float* out, int wr, int h, int col, bool drain) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)128 * wr * 64, 0, 128 * 64 * 4, 0x00020000);
    const int vo = fi_opaque((4 * h * 64 + col) * 4);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                const float v = accw[t][ct][rr];
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, vo,
                                                      ((32 * t + (rr & 3) + 8 * (rr >> 2)) * 64 + 32 * ct) * 4, 0);
            }
            accw[t][ct] = f32x16{};
        }
    if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// sum of a fragment's 8 bf16 values into acc: 4 v_dot2c_f32_bf16 against (1, 1) instead of 8
// conversions + 8 adds (the weight-gradient waves' bias column sums of dY)
__device__ __forceinline__ float sum8_bf16(const bf16x8& v, float acc) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    struct P4 { bf16x2 p[4]; };
    const P4 pv = __builtin_bit_cast(P4, v);
    const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_fdot2_f32_bf16(pv.p[j], one, acc, false);
    return acc;
}

// bf16 pair {bf16(a), bf16(b)} with each half zeroed where the matching s16 half of `mask` is
// not > 0 (ReLU derivative of a stored bf16 activation; -0 and negatives count as off):
// 0 - m with signed saturation is negative exactly for m > 0, its arithmetic shift by 15 the
// half-word mask
__device__ __forceinline__ uint32_t relu_mask_pair(float a, float b, uint32_t mask) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 v = {(__bf16)a, (__bf16)b};
    // (the shift count comes from a register: an inline constant of a packed instruction feeds
    // its high half from the constant's upper 16 bits, i.e. 0 for 15)
    uint32_t t;
    asm("v_pk_sub_i16 %0, 0, %1 clamp\n\tv_pk_ashrrev_i16 %0, %2, %0" : "=&v"(t) : "v"(mask), "v"(0x000F000Fu));
    return __builtin_bit_cast(uint32_t, v) & t;
}

__device__ __forceinline__ void u8x16_to_bf16(u32x4 v, bf16x8& lo, bf16x8& hi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lo[j] = (__bf16)(float)((v[j >> 2] >> (8 * (j & 3))) & 0xffu);
        hi[j] = (__bf16)(float)((v[2 + (j >> 2)] >> (8 * (j & 3))) & 0xffu);
    }
}

// ---------------------------------------------------------------------------------
// conv1 forward: a1[f] = bf16(relu(conv(frames[f]) / 255 + b)), persistent over frames.
// The raw u8 frames stream through a 2-slot LDS-DMA ring (two frames in flight while one is
// computed); each frame is converted once into the bf16 pair-plane image.
// ---------------------------------------------------------------------------------
namespace c1 {
constexpr int RAW = 28 * 1024;          // one raw frame (28,224 B) in 28 1-KiB DMA pieces
}

// 8 waves: wave w DMAs raw pieces j = w + 8i (< 28)
__device__ __forceinline__ int c1_issue_raw(const uint8_t* fr, uint32_t slot_lds, int w, int lane) {
    const fi_i32x4 rr = make_rsrc(fr, 28224);  // bytes past the frame read as zeros
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = w + 8 * i;
        if (i < 3 || j < 28) blds16(rr, 16 * lane + 1024 * j, slot_lds + 1024 * j);
    }
    return w < 4 ? 4 : 3;
}

// 512 threads = two waves per SIMD. Wave w computes all 32 output channels of the pixel
// tiles w, w+8, w+16 (and 24 for wave 0): 16x16x32 MFMAs with the weights as the A operand,
// D[channel][pixel]; A row i of channel tile nt is channel 8(i>>2) + 4nt + (i&3), so lane
// group g ends with channels 8g..8g+7 of its pixel and stores them straight to a1 (16 B).
// Lane i of a tile holds pixel 16t + sig(i) (lanes 8..15 swapped by 4): with the image's
// plane offset of 8 units (mod 16) both 16-lane groups of every B read are conflict-free.
// The next tile's 8 B fragments are read between the current tile's MFMAs.
struct f32x4x2 {
    f32x4 a, b;
};

__global__ __launch_bounds__(512, 2) void conv1_fwd_fr(const uint8_t* __restrict__ frames,
                                                       const __bf16* __restrict__ w1t,  // [32][256]
                                                       const float* __restrict__ bias,
                                                       __bf16* __restrict__ a1, int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[2 * c1::RAW + c1::IMG];
    char* img = smem + 2 * c1::RAW;
    const int lane = threadIdx.x & 63, w = wave_id();
    const uint32_t lds0 = lds_addr(smem);
    const int g = lane >> 4, c16 = lane & 15, si = c16 ^ ((c16 >> 1) & 4);
    bf16x8 bw[2][8];  // lane holds W[8(i>>2) + 4nt + (i&3), i = lane&15][k = 32ks + 8g..+8]
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
            bw[nt][ks] = *(const bf16x8*)(w1t + (8 * (c16 >> 2) + 4 * nt + (c16 & 3)) * 256 + 32 * ks + 8 * g);
    float bch[8];  // bias of the lane's output channels 8g + j
#pragma unroll
    for (int j = 0; j < 8; ++j) bch[j] = bias[8 * g + j];
    const float inv255 = 1.0f / 255.0f;
    const int nst = w == 0 ? 4 : 3;  // a1 stores per frame (one per tile)

    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    int issued = 0, m0 = 0, m1 = 0;
    if (nmine > 0) issued += c1_issue_raw(frames + (size_t)blockIdx.x * 28224, lds0, w, lane);
    m0 = issued;
    if (nmine > 1) issued += c1_issue_raw(frames + (size_t)(blockIdx.x + gridDim.x) * 28224, lds0 + c1::RAW, w, lane);
    m1 = issued;
    for (int it = 0; it < nmine; ++it) {
        const int f = blockIdx.x + it * gridDim.x;
        const char* raw = smem + (it & 1) * c1::RAW;
        wait_vmcnt(issued - m0);
        lds_barrier();  // raw frame landed; every wave done with the previous image
#pragma unroll
        for (int i = 0; i < (c1::FRAME_LOADS + 511) / 512; ++i) {
            const int u = threadIdx.x + 512 * i;
            if (u < c1::FRAME_LOADS) {
                bf16x8 lo, hi;
                u8x16_to_bf16(*(const u32x4*)(raw + 16 * u), lo, hi);
                *(bf16x8*)(img + 16 * u) = lo;
                *(bf16x8*)(img + c1::PLANE + 16 * u) = hi;
            }
        }
        lds_barrier();  // image ready; raw slot free
        int m2 = issued;
        if (it + 2 < nmine) {
            issued += c1_issue_raw(frames + (size_t)(f + 2 * gridDim.x) * 28224, lds0 + (it & 1) * c1::RAW, w, lane);
            m2 = issued;
        }
        u32x4* dst = (u32x4*)(a1 + (size_t)f * 12800);
        // B fragments of tile t: pixel pair (4ox + 2g..+1) of input row 4oy + ks -> plane g&1,
        // unit (4oy + ks) * 21 + ox + (g>>1)
        auto load = [&](int t, bf16x8* d) {
            const int q = t * 16 + si, oy = q / 20, ox = q - 20 * oy;
            const char* ab = img + (g & 1) * c1::PLANE + 16 * (oy * 84 + ox + (g >> 1));
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) d[ks] = *(const bf16x8*)(ab + 16 * 21 * ks);
        };
        auto tile = [&](const bf16x8* cur) {
            f32x4x2 d = {f32x4{}, f32x4{}};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                d.a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[0][ks], cur[ks], d.a, 0, 0, 0);
                d.b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[1][ks], cur[ks], d.b, 0, 0, 0);
            }
            return d;
        };
        auto store = [&](int t, const f32x4x2& d) {
            const int q = t * 16 + si;
            bf16x8 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                o[r] = (__bf16)fmaxf(d.a[r] * inv255 + bch[r], 0.f);
                o[4 + r] = (__bf16)fmaxf(d.b[r] * inv255 + bch[4 + r], 0.f);
            }
            FI_ST16(__builtin_bit_cast(u32x4, o), dst + 4 * q + g);
        };
        bf16x8 fb[2][8];
        load(w, fb[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) {
            const int t = w + 8 * tt;
            if (tt < 2) load(t + 8, fb[(tt + 1) & 1]);
            else if (w == 0) load(24, fb[1]);  // wave 0 also takes tile 24
            const f32x4x2 d = tile(fb[tt & 1]);
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            store(t, d);
        }
        if (w == 0) store(24, tile(fb[1]));
        issued += nst;
        m0 = m1;
        m1 = m2;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// 8 waves: wave w accumulates k-tiles 4kg..4kg+3 (kg = w&1; k-tile = kernel row ky: 8 taps x
// 4 channels = 32 k) over the m-steps ms = mg, mg+4, ... (mg = w>>1) of every frame, so each
// da1 fragment read feeds four MFMAs (LDS reads per MFMA: 1.25 KB instead of 2). The four
// m-groups' partial sums are reduced in LDS in a fixed order at the end. Per frame: the raw
// u8 frame (1 slot, issued as soon as the previous one is converted) and the da1 tile
// (3-slot ring, two frames ahead) arrive by LDS-DMA; the frame is converted once into the
// bf16 pair-plane image; both MFMA operands come from transposed LDS reads, the next
// m-step's issued between the current one's MFMAs. Two barriers per frame: past the first,
// every wave is done with the previous frame (image and its da1 slot free); past the second,
// the image is complete (raw slot free).
__global__ __launch_bounds__(512, 2) void conv1_wgrad_fr(const uint8_t* __restrict__ frames,
                                                         const __bf16* __restrict__ da1,
                                                         float* __restrict__ slab,
                                                         float* __restrict__ cs_slab, int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c1::RAW + 3 * c1::OUT + c1::IMG];
    char* raw = smem;
    char* img = smem + c1::RAW + 3 * c1::OUT;
    const uint32_t lds0 = lds_addr(smem);
    const int lane = threadIdx.x & 63, w = wave_id(), tid = threadIdx.x;
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int kg = w & 1, mg = w >> 1;
    // lane's tr column: k = 32ky + 16(g&1) + 4p = tap (ky, kx = 4(g&1) + p) x 4 channels;
    // ky = 4kg + kt, the kt step is +21 image units (+336 B)
    const int toff = 4 * kg * 84 + 4 * (g & 1) + p;  // pixel offset of the tap relative to (4oy, 4ox)
    int wao[7][2];  // image offset of the A^T (im2col) transposed read, per own m-step / half
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int ms = min(mg + 4 * j, 24);
            const int m = ms * 16 + 8 * (g >> 1) + q + 4 * hh;
            const int oy = m / 20, ox = m - oy * 20;
            const int P = oy * 4 * 84 + ox * 4 + toff;
            const int y = P / 84, x = P - y * 84;
            wao[j][hh] = ((x >> 1) & 1) * c1::PLANE + 16 * (y * 21 + (x >> 2)) + 8 * (x & 1);
        }
    // da1 tile [m][32 co]: B read of rows m = 16ms + 8(g>>1) + q + 4hh -> base_hh + 1024 ms
    const int wb0 = (8 * (g >> 1) + q) * 64 + (16 * (g & 1) + 4 * p) * 2 + 1024 * mg;  // half hh: +256
    f32x16 acc[4] = {};
    float bsum = 0.f;

    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    auto issue_raw = [&](int k) {
        const fi_i32x4 rr = make_rsrc(frames + (size_t)(blockIdx.x + k * gridDim.x) * 28224, 28224);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = w + 8 * i;
            if (j < 28) blds16(rr, 16 * lane + 1024 * j, lds0 + 1024 * j);
        }
        return w < 4 ? 4 : 3;
    };
    auto issue_dy = [&](int k) {
        const fi_i32x4 dr = make_rsrc(da1 + (size_t)(blockIdx.x + k * gridDim.x) * 12800, 25600);
        const uint32_t base = lds0 + c1::RAW + (k % 3) * c1::OUT;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = w + 8 * i;
            if (j < 25) blds16(dr, 16 * lane + 1024 * j, base + 1024 * j);
        }
        return w == 0 ? 4 : 3;
    };
    // issue order: raw(0) dy(0) dy(1) | per frame it: dy(it+2) after the first barrier,
    // raw(it+1) after the second. mk_*: issue counts just after each frame's pieces.
    int issued = 0, mk_raw = 0, mk_dy0 = 0, mk_dy1 = 0;
    if (nmine > 0) { issued += issue_raw(0); mk_raw = issued; issued += issue_dy(0); mk_dy0 = issued; }
    if (nmine > 1) { issued += issue_dy(1); mk_dy1 = issued; }
    for (int it = 0; it < nmine; ++it) {
        const char* dy = smem + c1::RAW + (it % 3) * c1::OUT;
        wait_vmcnt(issued - max(mk_raw, mk_dy0));
        lds_barrier();  // raw frame + da1 tile landed; previous frame consumed by every wave
        int mk_dy2 = 0;
        if (it + 2 < nmine) { issued += issue_dy(it + 2); mk_dy2 = issued; }
#pragma unroll
        for (int i = 0; i < (c1::FRAME_LOADS + 511) / 512; ++i) {
            const int u = tid + 512 * i;
            if (u < c1::FRAME_LOADS) {
                bf16x8 lo, hi;
                u8x16_to_bf16(*(const u32x4*)(raw + 16 * u), lo, hi);
                *(bf16x8*)(img + 16 * u) = lo;
                *(bf16x8*)(img + c1::PLANE + 16 * u) = hi;
            }
        }
        lds_barrier();  // image ready; raw slot free
        if (it + 1 < nmine) { issued += issue_raw(it + 1); mk_raw = issued; }
        const char* DB = dy + wb0;
        auto load = [&](int j, bf16x8* d) {  // [0] da1, [1..4] A of k-tiles kt = 0..3
            d[0] = tr2(DB + 4096 * j, DB + 256 + 4096 * j);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) d[1 + kt] = tr2(img + wao[j][0] + 336 * kt, img + wao[j][1] + 336 * kt);
        };
        auto step = [&](const bf16x8* cur) {
            if (kg == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum += (float)cur[0][j];
            }
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
                acc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[1 + kt], cur[0], acc[kt], 0, 0, 0);
        };
        bf16x8 fb[2][5];
        load(0, fb[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            if (j < 5) load(j + 1, fb[(j + 1) & 1]);
            else if (mg == 0) load(6, fb[0]);  // m-group 0 also takes step 24
            step(fb[j & 1]);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (j < 5) {
                    if (kt < 2) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                    else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
            }
        }
        if (mg == 0) step(fb[0]);
        mk_dy0 = mk_dy1;
        mk_dy1 = mk_dy2;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // reduce the four m-groups in LDS (fixed order mg = 0..3), one k-group per round:
    // red[mg][kt][r][lane] -> slab rows k = 32(4kg + kt) + (r&3) + 8(r>>2) + 4(lane>>5), col lane&31
    float* red = (float*)smem;
    float* out = slab + (size_t)blockIdx.x * 256 * 32;
    const float inv255 = 1.0f / 255.0f;
#pragma unroll
    for (int round = 0; round < 2; ++round) {
        __syncthreads();
        if (kg == round) {
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[((mg * 4 + kt) * 16 + r) * 64 + lane] = acc[kt][r];
        }
        __syncthreads();
        for (int e = tid; e < 4 * 16 * 64; e += 512) {  // e = (kt * 16 + r) * 64 + l
            const float v = ((red[e] + red[4096 + e]) + red[8192 + e]) + red[12288 + e];
            const int l = e & 63, r = (e >> 6) & 15, kt = e >> 10;
            const int k = 32 * (4 * round + kt) + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            out[k * 32 + (l & 31)] = v * inv255;
        }
    }
    // bias partials: lanes l and l+32 hold the same co (tr column), other m half; the k-group 0
    // waves hold disjoint m-steps -> [4][32] in LDS, summed in m-group order
    __syncthreads();
    const float o = bsum + __shfl_xor(bsum, 32, 64);
    if (kg == 0 && lane < 32) red[32 * mg + lane] = o;
    __syncthreads();
    if (w == 0 && lane < 32) {
        const float t = ((red[lane] + red[32 + lane]) + red[64 + lane]) + red[96 + lane];
        cs_slab[(size_t)blockIdx.x * 32 + lane] = t;
    }
}

int conv1_fwd_fr_launch(const uint8_t* frames, const __bf16* w1t, const float* bias, __bf16* a1,
                        int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv1_fwd_fr, dim3(grid), dim3(512), 0, s, frames, w1t, bias, a1, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

int conv1_wgrad_fr_launch(const uint8_t* frames, const __bf16* da1, float* slab, float* cs_slab,
                          int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv1_wgrad_fr, dim3(grid), dim3(512), 0, s, frames, da1, slab, cs_slab, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}


// =====================================================================================
// Frame-resident forward of conv2 (4x4/2, 32 -> 64) and conv3 (3x3/1, 64 -> 64).
// 8 waves = 2 channel halves chh (32 output channels: two 16-channel A-operand tiles of the
// weight slice in registers, so D = [channel][pixel]) x 4 pixel-tile groups pg; each B
// fragment read feeds two MFMAs. A row i of channel tile ct is channel
// 32chh + 8(i>>2) + 4ct + (i&3), so lane group g ends with channels 32chh + 8g..+8 of its
// pixel and stores them straight from registers (16 B).
// Output pixels are walked on an s-grid whose pitch equals the LDS image's row pitch
// (conv2: s = 10oy + ox over the 10-wide parity-class planes; conv3: s = 9oy + ox over the
// 9-wide image; the extra columns are computed and dropped), so a B read of tile pixels s
// hits image units s + const: with chunk offsets Z(c) (chunks c, c+1 8 units apart) and the
// tile lanes permuted (sig) every ds_read_b128 is conflict-free, and every fragment
// address is a base register plus an immediate.
//   conv2 image: unit = pos + 100 P + 416 c + Z(c), P = 2(iy&1) + (ix&1), pos = (iy>>1)*10 + (ix>>1)
//   conv3 image: unit = p + 96 c + Z(c), p = 9 iy + ix
// Input frames arrive by LDS-DMA in their own byte order (1 KiB contiguous per wave
// instruction: a gather straight into the chunk-planar image cost ~15% of conv2's kernel in
// memory requests) into STG staging buffers, and each issuing wave moves its own landed
// pieces into the other of two image slots (ds_read/ds_write_b128) after the iteration's
// MFMAs, behind a counted vmcnt that lets the output stores fly. One barrier per iteration.
// =====================================================================================
__host__ __device__ constexpr int fz(int c) { return 8 * (c & 1) + 4 * ((c >> 1) & 1); }

// 16-byte unit i of an input frame (pixel i/4 or i/8, chunk i%4 or i%8) -> image unit
__device__ __forceinline__ int f2_dst(int i) {
    const int p = i >> 2, c = i & 3, iy = p / 20, ix = p - 20 * iy;
    return ((iy >> 1) * 10 + (ix >> 1)) + 100 * (2 * (iy & 1) + (ix & 1)) + 416 * c + fz(c);
}
__device__ __forceinline__ int f3_dst(int i) {
    const int p = i >> 3, c = i & 7;
    return p < 81 ? p + 96 * c + fz(c) : 0;
}
// Reshuffle lane order for the pixel-major (8 chunks per pixel) conv3 inputs: lane L moves
// unit rs_lane(L) of a 64-unit piece. In the identity order the 8 lanes of a ds_write_b128
// bank group (8 contiguous lanes, bank (a/4) mod 32) hold one pixel's 8 chunks, whose image
// units p + 96c + fz(c) fall on 2 distinct 16-B bank slots: 4-way conflicts (the conv3
// kernels' SQ_LDS_BANK_CONFLICT). This order gives each write group 8 pixels of one chunk
// pair pattern -- 8 distinct slots -- and keeps the staging ds_read_b128 groups conflict-free
// (scripts/lds_conflicts.py model: 331 -> 88 LDS cycles per frame for the X image; the
// bordered dY image 203 -> 104).
__device__ __forceinline__ int rs_lane(int L) { return 8 * (L & 7) + ((2 * (L & 7) + (L >> 3)) & 7); }

template <int L>  // L = 2 (conv2) or 3 (conv3)
struct FwdGeo;
template <>
struct FwdGeo<2> {  // two frames per iteration: 12 pixel tiles = 4 groups x 3
    static constexpr int XB = 1680 * 16;           // image units per frame
    static constexpr int IN_BYTES = 25600, OUT_ELEMS = 5184, IN_ELEMS = 12800, KS = 16, NT = 6;
    static constexpr int SW = 10, OW = 9;  // s-grid pitch, output width (= height)
    static constexpr int FPI = 2, STG = 1;  // frames per iteration, staging buffers (iterations ahead)
};
template <>
struct FwdGeo<3> {  // two frames per iteration: 8 pixel tiles = 4 groups x 2
    static constexpr int XB = 768 * 16;
    static constexpr int IN_BYTES = 10368, OUT_ELEMS = 3136, IN_ELEMS = 5184, KS = 18, NT = 4;
    static constexpr int SW = 9, OW = 7;
    static constexpr int FPI = 2, STG = 2;
};

template <int L>
__global__ __launch_bounds__(512, 2) void conv_fwd_fr(const __bf16* __restrict__ x,    // NHWC input frames
                                                      const __bf16* __restrict__ wt,   // [64][K] (ky,kx,ci)
                                                      const float* __restrict__ bias,  // [64]
                                                      __bf16* __restrict__ y,          // NHWC output frames
                                                      int nframes) {
    using G = FwdGeo<L>;
    constexpr int K = G::KS * 32, FPI = G::FPI, STG = G::STG;
    constexpr int TPW = G::NT * FPI / 4;                // pixel tiles per wave
    constexpr int NLP = (G::IN_BYTES + 1023) / 1024;   // 1-KiB pieces per input frame
    constexpr int PPW = (NLP + 7) / 8;                  // pieces per wave per frame (at most)
    constexpr int IMG = 2 * FPI * G::XB, SBUF = FPI * NLP * 1024;
    __shared__ __attribute__((aligned(16))) char smem[IMG + STG * SBUF + NLP * 64 * 2];
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int w = wave_id(), chh = w >> 2, pg = w & 3;
    const int g = lane >> 4, c16 = lane & 15, si = c16 ^ ((c16 >> 1) & 4);
    const uint32_t lds0 = lds_addr(smem);
    // image unit of every 16-byte unit of the input frame
    uint16_t* dstu = (uint16_t*)(smem + IMG + STG * SBUF);
    for (int i = tid; i < NLP * 64; i += 512) dstu[i] = (uint16_t)(L == 2 ? f2_dst(i) : f3_dst(i));
    for (int i = tid; i < IMG / 16; i += 512) ((u32x4*)smem)[i] = u32x4{0, 0, 0, 0};  // gap units

    // A operand: lane holds W[co = 32chh + 8(i>>2) + 4ct + (i&3), i = c16][k = 32ks + 8g..+8]
    bf16x8 wa[2][G::KS];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks)
            wa[ct][ks] = *(const bf16x8*)(wt + (size_t)(32 * chh + 8 * (c16 >> 2) + 4 * ct + (c16 & 3)) * K +
                                          32 * ks + 8 * g);
    float bch[8];  // bias of the lane's channels 32chh + 8g + j
#pragma unroll
    for (int j = 0; j < 8; ++j) bch[j] = bias[32 * chh + 8 * g + j];
    // this wave's tiles: global tile t = TPW*pg + i over the FPI frames of an iteration;
    // lane pixel s = 16 tt + sig(c16) of frame fi; B unit = s + chunk offset + tap immediate
    int bbase[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = TPW * pg + i, fi = t / G::NT, tt = t - fi * G::NT, s = 16 * tt + si;
        bbase[i] = fi * G::XB + 16 * (s + (L == 2 ? 416 : 96) * g + fz(g));
    }
    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int niter = (nmine + FPI - 1) / FPI;
    // iteration i2's frames: wave w DMAs pieces j = w + 8i of each frame, in the frame's own
    // byte order (fully coalesced), into staging buffer i2 % STG; returns the pieces issued
    auto issue = [&](int i2) {
        int n = 0;
#pragma unroll
        for (int u = 0; u < FPI; ++u) {
            const int k = FPI * i2 + u;
            if (k < nmine) {
                const fi_i32x4 xr = make_rsrc(x + (size_t)(blockIdx.x + k * gridDim.x) * G::IN_ELEMS, G::IN_BYTES);
                const uint32_t sb = lds0 + IMG + (i2 % STG) * SBUF + u * NLP * 1024;
#pragma unroll
                for (int i = 0; i < PPW; ++i) {
                    const int j = w + 8 * i;
                    if (j < NLP) {
                        blds16(xr, 1024 * j + 16 * lane, sb + 1024 * j);
                        ++n;
                    }
                }
            }
        }
        return n;
    };
    // the issuing wave moves its own landed pieces of iteration i2 into image slot i2 & 1
    // (all reads first, then all writes: one LDS round trip, not one per piece)
    const int sl = L == 3 ? rs_lane(lane) : lane;  // conv3: bank-conflict-free write groups
    auto reshuffle = [&](int i2) {
        u32x4 d[FPI][PPW];
        int du[FPI][PPW];
#pragma unroll
        for (int u = 0; u < FPI; ++u)
#pragma unroll
            for (int i = 0; i < PPW; ++i) {
                const int j = min(w + 8 * i, NLP - 1);
                d[u][i] = *(const u32x4*)(smem + IMG + (i2 % STG) * SBUF + u * NLP * 1024 + 1024 * j + 16 * sl);
                du[u][i] = dstu[64 * j + sl];
            }
#pragma unroll
        for (int u = 0; u < FPI; ++u) {
            const int k = FPI * i2 + u;
            if (k < nmine) {
                char* im = smem + ((i2 & 1) * FPI + u) * G::XB;
#pragma unroll
                for (int i = 0; i < PPW; ++i) {
                    const int j = w + 8 * i, b = 1024 * j + 16 * sl;
                    if (j < NLP && b < G::IN_BYTES) *(u32x4*)(im + 16 * du[u][i]) = d[u][i];
                }
            }
        }
    };
    __syncthreads();  // table and zeroed image ready
    // issue order: DMA(0), then per iteration: stores, DMA(it + 1 + STG) after reshuffle(it + 1).
    // mk[q]: issue count right after DMA(it + 1 + q), q < STG
    int issued = 0, mk[STG];
    if (niter > 0) {
        issued += issue(0);
        wait_vmcnt(0);
        reshuffle(0);
    }
#pragma unroll
    for (int q = 0; q < STG; ++q) {
        if (1 + q < niter) issued += issue(1 + q);
        mk[q] = issued;
    }
    auto imm = [&](int ks) {
        if (L == 2) {  // tap = ks (32 channels = chunks 0..3): class plane + position shift
            const int ky = ks >> 2, kx = ks & 3;
            return 16 * (10 * (ky >> 1) + (kx >> 1) + 100 * (2 * (ky & 1) + (kx & 1)));
        } else {       // tap = ks/2, channel half ks&1 -> chunk + 4
            const int tap = ks >> 1, ky = tap / 3, kx = tap - 3 * ky;
            return 16 * (9 * ky + kx + 384 * (ks & 1));
        }
    };
    constexpr int NSTEP = TPW * G::KS;  // (tile, k-step) steps per iteration
    for (int it = 0; it < niter; ++it) {
        const char* X = smem + (it & 1) * FPI * G::XB;
        lds_barrier();  // iteration it's image written; iteration it-1 consumed by every wave
        // tile-outer steps: each tile's 2*KS MFMAs end in its 16-byte store; B fragments are
        // read PD steps ahead of their MFMAs
        constexpr int PD = 4;
        bf16x8 fb[PD + 1];
#pragma unroll
        for (int st = 0; st < PD; ++st) fb[st] = *(const bf16x8*)(X + bbase[st / G::KS] + imm(st % G::KS));
        __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
        f32x4 acc0 = f32x4{}, acc1 = f32x4{};
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            const int i = st / G::KS, ks = st % G::KS;
            if (st + PD < NSTEP)
                fb[(st + PD) % (PD + 1)] = *(const bf16x8*)(X + bbase[(st + PD) / G::KS] + imm((st + PD) % G::KS));
            const bf16x8 b = fb[st % (PD + 1)];
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][ks], b, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][ks], b, acc1, 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            if (st + PD < NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (ks == G::KS - 1) {  // tile i done: bias, ReLU, one 16-byte store (its frame present)
                const int t = TPW * pg + i, fi = t / G::NT, tt = t - fi * G::NT, s = 16 * tt + si;
                const int k = FPI * it + fi;
                if (k < nmine) {
                    ++issued;
                    const int oy = s / G::SW, ox = s - G::SW * oy;
                    if (oy < G::OW && ox < G::OW) {
                        bf16x8 ov;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            ov[r] = (__bf16)fmaxf(acc0[r] + bch[r], 0.f);
                            ov[4 + r] = (__bf16)fmaxf(acc1[r] + bch[4 + r], 0.f);
                        }
                        u32x4* dst = (u32x4*)(y + (size_t)(blockIdx.x + k * gridDim.x) * G::OUT_ELEMS);
                        FI_ST16(__builtin_bit_cast(u32x4, ov), dst + 8 * (G::OW * oy + ox) + 4 * chh + g);
                    }
                }
                acc0 = f32x4{};
                acc1 = f32x4{};
            }
        }
        if (it + 1 < niter) {
            wait_vmcnt(issued - mk[0]);  // own pieces of iteration it + 1 landed (stores may fly)
            reshuffle(it + 1);           // image slot (it+1)&1 was last read in iteration it-1
        }
        int mnew = issued;
        if (it + 1 + STG < niter) {
            issued += issue(it + 1 + STG);  // into the staging buffer just emptied
            mnew = issued;
        }
#pragma unroll
        for (int q = 0; q + 1 < STG; ++q) mk[q] = mk[q + 1];
        mk[STG - 1] = mnew;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int conv2_fwd_fr_launch(const __bf16* a1, const __bf16* w2t, const float* bias, __bf16* a2, int nframes,
                        int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv_fwd_fr<2>, dim3(grid), dim3(512), 0, s, a1, w2t, bias, a2, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

int conv3_fwd_fr_launch(const __bf16* a2, const __bf16* w3t, const float* bias, __bf16* a3, int nframes,
                        int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv_fwd_fr<3>, dim3(grid), dim3(512), 0, s, a2, w3t, bias, a3, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// =====================================================================================
// Fused conv1 + conv2 forward (frame-resident): a1 is written to HBM once (conv2's backward
// needs it) but never read back for conv2 -- conv2 takes it from LDS. 8 waves, two per SIMD:
//   waves 0-3 (conv1 role): conv1 exactly as conv1_fwd_fr (W1 in registers, 16x16x32,
//     D = [channel][pixel]; pixel tiles w, w+4, ... of the 25); each lane's 16-byte a1
//     result goes to HBM at once and is HELD in registers until the next iteration writes it
//     into the conv2 input image (conv_fwd_fr<2>'s chunk-planar class-plane layout);
//   waves 4-7 (conv2 role): conv2 of the PREVIOUS frame from that image as conv_fwd_fr<2>
//     (W2 channel half chh in registers, s-grid tiles 3pg..3pg+2).
// The u8 -> bf16 conversion of frame it+1 overlaps frame it: two conv1 images (frame it is read
// by the conv1 MFMAs while frame it+1 is written), the raw bytes by plain 16-byte loads into
// registers one frame ahead, each unit's register reloaded right after its conversion.
// Iteration it: [B1] phase A: the conv1 role writes a1(it-1) into the conv2 image and converts
// NCA units per lane of raw(it+1); the conv2 role converts NA units per lane  [B2] phase B:
// conv1(it) MFMAs on waves 0-3 beside conv2(it-1) MFMAs on waves 4-7 (sharing each SIMD's
// matrix pipe), the conv1 role converting its remaining NC - NCA units between its tiles.
// (Round 5; before, two raw LDS-DMA slots and one image: the whole conversion in a phase of its
// own, 1.4k clocks per frame without MFMAs. Measured splits, conv12_fwd ms vs 5.86-6.02 for the
// old kernel in the same runs (scripts/r05_gpu_batch.sh, profiles/r05_conv12_split_ab.txt):
// NCA/NC/NA/NB = 1/3/4/0 5.65-5.75 (kept), 2/3/4/0 5.69-5.76, 0/3/4/0 5.70-5.80, 3/3/4/0
// 5.77-5.86, 0/2/3/2 5.81-5.83, 0/3/3/1 5.71-5.80, 0/2/2/3 6.54-6.56: units converted between
// the conv2 MFMAs (NB) cost ~650 clocks each, between the conv1 MFMAs ~390, in phase A ~300;
// raw units DMA'd into an LDS staging area instead of registers 6.03-6.07; s_setprio 1 on
// either role neutral / +0.15 ms.)
// LDS: 2 conv1 images (113,152) + conv2 image (26,880) = 140,032 B.
// HBM per frame: 28,224 (frame) + 25,600 (a1) + 10,368 (a2) = 64,192 B (vs 89,792 B for the
// two kernels separately).
// =====================================================================================
namespace c12 {
constexpr int X2 = 1680 * 16;             // conv2 input image (FwdGeo<2>::XB)
constexpr int LDS = 2 * c1::IMG + X2;     // 140,032 B
// raw units per lane: NC by the conv1 role (units tid + 256i; the first NCA in phase A), NA by
// the conv2 role (units 256 NC + t4 + 256i) in phase A
constexpr int NCA = 1, NC = 3, NA = 4;
static_assert(256 * (NC + NA) >= c1::FRAME_LOADS && 256 * (NC + NA - 1) < c1::FRAME_LOADS, "units");
static_assert(NCA <= NC && NC <= 6, "conv1-role units: one per tile");
}  // namespace c12

__device__ __forceinline__ void c12_cvt_unit(u32x4 v, char* img, int u) {
    bf16x8 lo, hi;
    u8x16_to_bf16(v, lo, hi);
    *(bf16x8*)(img + 16 * u) = lo;
    *(bf16x8*)(img + c1::PLANE + 16 * u) = hi;
}

__global__ __launch_bounds__(512, 2) void conv12_fwd_fr(const uint8_t* __restrict__ frames,
                                                        const __bf16* __restrict__ w1t,  // [32][256]
                                                        const float* __restrict__ b1,
                                                        const __bf16* __restrict__ w2t,  // [64][512]
                                                        const float* __restrict__ b2,
                                                        __bf16* __restrict__ a1, __bf16* __restrict__ a2,
                                                        int nframes, int a1_planar) {
    __shared__ __attribute__((aligned(16))) char smem[c12::LDS];
    char* x2 = smem + 2 * c1::IMG;
    const int lane = threadIdx.x & 63, tid = threadIdx.x, w = wave_id();
    const int g = lane >> 4, c16 = lane & 15, si = c16 ^ ((c16 >> 1) & 4);
    for (int i = tid; i < c12::X2 / 16; i += 512) ((u32x4*)x2)[i] = u32x4{0, 0, 0, 0};  // gap units
    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    auto raw_of = [&](int k) { return (const u32x4*)(frames + (size_t)(blockIdx.x + k * gridDim.x) * 28224); };
    auto img_of = [&](int k) { return smem + (k & 1) * c1::IMG; };

    if (w < 4) {
        // ---------------- conv1 role
        bf16x8 bw[2][8];  // lane holds W1[8(i>>2) + 4nt + (i&3), i = lane&15][k = 32ks + 8g..+8]
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
                bw[nt][ks] = *(const bf16x8*)(w1t + (8 * (c16 >> 2) + 4 * nt + (c16 & 3)) * 256 + 32 * ks + 8 * g);
        float bch[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bch[j] = b1[8 * g + j];
        const float inv255 = 1.0f / 255.0f;
        const int ntile = w == 0 ? 7 : 6;  // tiles w + 4tt < 25
        u32x4 held[7];                     // a1 of the previous frame, tile tt
        u32x4 rr[c12::NC];                 // raw units tid + 256i of the next frame to convert
        if (nmine > 0) {
            const u32x4* src = raw_of(0);
#pragma unroll
            for (int i = 0; i < c12::NC; ++i) rr[i] = src[tid + 256 * i];
#pragma unroll
            for (int i = 0; i < c12::NC; ++i) c12_cvt_unit(rr[i], img_of(0), tid + 256 * i);
        }
        if (nmine > 1) {
            const u32x4* src = raw_of(1);
#pragma unroll
            for (int i = 0; i < c12::NC; ++i) rr[i] = src[tid + 256 * i];
        }
        // every prologue load landed: the compiler's waits in the frame loop then follow only the
        // loop's own loads (it merges the preheader's pending loads into the loop head otherwise and
        // waits for all of them, stores included, in every frame). The builtin, not asm: the
        // compiler's wait pass reads it
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        for (int it = 0; it <= nmine; ++it) {
            const int f = blockIdx.x + it * gridDim.x;
            const bool cvt = it + 1 < nmine, rel = it + 2 < nmine;  // convert raw(it+1); reload for it+2
            const u32x4* nsrc = raw_of(rel ? it + 2 : it);
            char* nimg = img_of(it + 1);
            lds_barrier();  // B1: image(it) complete; the conv2 image read by conv2(it-2)
            if (it >= 1) {  // a1(it-1) -> conv2 image (pixel q, chunk g)
#pragma unroll
                for (int tt = 0; tt < 7; ++tt)
                    if (tt < ntile) *(u32x4*)(x2 + 16 * f2_dst(4 * ((w + 4 * tt) * 16 + si) + g)) = held[tt];
            }
            if (cvt) {
#pragma unroll
                for (int i = 0; i < c12::NCA; ++i) {
                    c12_cvt_unit(rr[i], nimg, tid + 256 * i);
                    if (rel) rr[i] = nsrc[tid + 256 * i];
                }
            }
            lds_barrier();  // B2: the conv2 image complete
            if (it < nmine) {
                const char* img = img_of(it);
                u32x4* dst = (u32x4*)(a1 + (size_t)f * 12800);
                auto load = [&](int t, bf16x8* d) {
                    const int q = t * 16 + si, oy = q / 20, ox = q - 20 * oy;
                    const char* ab = img + (g & 1) * c1::PLANE + 16 * (oy * 84 + ox + (g >> 1));
#pragma unroll
                    for (int ks = 0; ks < 8; ++ks) d[ks] = *(const bf16x8*)(ab + 16 * 21 * ks);
                };
                bf16x8 fb[2][8];
                load(w, fb[0]);
                __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
                for (int tt = 0; tt < 7; ++tt) {
                    if (tt < ntile) {
                        const int t = w + 4 * tt;
                        if (tt + 1 < ntile) load(t + 4, fb[(tt + 1) & 1]);
                        const bf16x8* cur = fb[tt & 1];
                        f32x4 da = f32x4{}, db = f32x4{};
#pragma unroll
                        for (int ks = 0; ks < 8; ++ks) {
                            da = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[0][ks], cur[ks], da, 0, 0, 0);
                            db = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[1][ks], cur[ks], db, 0, 0, 0);
                        }
                        const bool unit_here = tt >= c12::NCA && tt < c12::NC;  // tile tt converts unit tt
                        if (unit_here && cvt) {
                            c12_cvt_unit(rr[tt], nimg, tid + 256 * tt);
                            if (rel) rr[tt] = nsrc[tid + 256 * tt];
                        }
#pragma unroll
                        for (int ks = 0; ks < 8; ++ks) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                            if (tt + 1 < ntile) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                            if (unit_here) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                        }
                        bf16x8 o;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            o[r] = (__bf16)fmaxf(da[r] * inv255 + bch[r], 0.f);
                            o[4 + r] = (__bf16)fmaxf(db[r] * inv255 + bch[4 + r], 0.f);
                        }
                        held[tt] = __builtin_bit_cast(u32x4, o);
                        // a1 in HBM: NHWC, or (a1_planar) in conv21's image order -- parity-class
                        // plane P = 2(iy&1) + (ix&1), position (iy>>1)*10 + (ix>>1), chunk g -- so
                        // that conv21 loads it by linear DMA (c2_x_src)
                        const int q = t * 16 + si, iy = q / 20, ix = q - 20 * iy;
                        const int u = a1_planar ? 400 * (2 * (iy & 1) + (ix & 1)) + 4 * ((iy >> 1) * 10 + (ix >> 1)) + g
                                                : 4 * q + g;
                        FI_ST16(held[tt], dst + u);
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        // ---------------- conv2 role
        const int wr = w - 4, chh = wr & 1, pg = wr >> 1, t4 = tid - 256;
        bf16x8 wa[2][16];  // lane holds W2[co = 32chh + 8(i>>2) + 4ct + (i&3), i = c16][k = 32ks + 8g..+8]
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int ks = 0; ks < 16; ++ks)
                wa[ct][ks] = *(const bf16x8*)(w2t + (size_t)(32 * chh + 8 * (c16 >> 2) + 4 * ct + (c16 & 3)) * 512 +
                                              32 * ks + 8 * g);
        float bch[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bch[j] = b2[32 * chh + 8 * g + j];
        int bbase[3];  // tile i: s = 16 (3pg + i) + sig(c16) on the pitch-10 s-grid, chunk g
#pragma unroll
        for (int i = 0; i < 3; ++i) bbase[i] = 16 * (16 * (3 * pg + i) + si + 416 * g + fz(g));
        auto imm = [](int ks) {  // tap ks = (ky, kx): class plane + position shift
            const int ky = ks >> 2, kx = ks & 3;
            return 16 * (10 * (ky >> 1) + (kx >> 1) + 100 * (2 * (ky & 1) + (kx & 1)));
        };
        auto unit = [&](int i) { return 256 * c12::NC + t4 + 256 * i; };
        auto valid = [&](int i) { return i + 1 < c12::NA || unit(i) < c1::FRAME_LOADS; };
        u32x4 rr[c12::NA];
        if (nmine > 0) {
            const u32x4* src = raw_of(0);
#pragma unroll
            for (int i = 0; i < c12::NA; ++i)
                if (valid(i)) rr[i] = src[unit(i)];
#pragma unroll
            for (int i = 0; i < c12::NA; ++i)
                if (valid(i)) c12_cvt_unit(rr[i], img_of(0), unit(i));
        }
        if (nmine > 1) {
            const u32x4* src = raw_of(1);
#pragma unroll
            for (int i = 0; i < c12::NA; ++i)
                if (valid(i)) rr[i] = src[unit(i)];
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), as the conv1 role
        for (int it = 0; it <= nmine; ++it) {
            lds_barrier();  // B1
            if (it + 1 < nmine) {  // raw(it+1) -> the next image (free since B1)
                const bool rel = it + 2 < nmine;
                const u32x4* nsrc = raw_of(rel ? it + 2 : it);
#pragma unroll
                for (int i = 0; i < c12::NA; ++i) {
                    if (valid(i)) {
                        c12_cvt_unit(rr[i], img_of(it + 1), unit(i));
                        if (rel) rr[i] = nsrc[unit(i)];
                    }
                }
            }
            lds_barrier();  // B2: a1(it-1) in the conv2 image
            if (it >= 1) {  // conv2 of frame it-1 from the a1 image
                const int k = it - 1;
                u32x4* dst = (u32x4*)(a2 + (size_t)(blockIdx.x + k * gridDim.x) * 5184);
                constexpr int PD = 4, NSTEP = 3 * 16;
                bf16x8 fb[PD + 1];
#pragma unroll
                for (int st = 0; st < PD; ++st) fb[st] = *(const bf16x8*)(x2 + bbase[st / 16] + imm(st % 16));
                __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
                f32x4 acc0 = f32x4{}, acc1 = f32x4{};
#pragma unroll
                for (int st = 0; st < NSTEP; ++st) {
                    const int i = st / 16, ks = st % 16;
                    if (st + PD < NSTEP)
                        fb[(st + PD) % (PD + 1)] = *(const bf16x8*)(x2 + bbase[(st + PD) / 16] + imm((st + PD) % 16));
                    const bf16x8 b = fb[st % (PD + 1)];
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][ks], b, acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][ks], b, acc1, 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    if (st + PD < NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    if (ks == 15) {  // tile i done: bias, ReLU, one 16-byte store
                        const int s = 16 * (3 * pg + i) + si, oy = s / 10, ox = s - 10 * oy;
                        if (oy < 9 && ox < 9) {
                            bf16x8 ov;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                ov[r] = (__bf16)fmaxf(acc0[r] + bch[r], 0.f);
                                ov[4 + r] = (__bf16)fmaxf(acc1[r] + bch[4 + r], 0.f);
                            }
                            FI_ST16(__builtin_bit_cast(u32x4, ov), dst + 8 * (9 * oy + ox) + 4 * chh + g);
                        }
                        acc0 = f32x4{};
                        acc1 = f32x4{};
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

int conv12_fwd_fr_launch(const uint8_t* frames, const __bf16* w1t, const float* b1, const __bf16* w2t,
                         const float* b2, __bf16* a1, __bf16* a2, int nframes, int grid, hipStream_t s,
                         int a1_planar) {
    hipLaunchKernelGGL(conv12_fwd_fr, dim3(grid), dim3(512), 0, s, frames, w1t, b1, w2t, b2, a1, a2, nframes,
                       a1_planar);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// =====================================================================================
// Fused, frame-resident conv backward kernels (dgrad + wgrad + bias of one layer).
// Per frame, LDS holds the layer input X (= ReLU mask of the data gradient) and the
// upstream gradient dY; the kernel writes dX = (X > 0) * dgrad(dY, W) once and keeps
// dW / db accumulating in registers across its frames (one fp32 partial slab per
// workgroup, reduced in a fixed order afterwards). Frames stream through a 3-deep LDS ring
// filled by LDS-DMA gathers (buffer_load_dwordx4 ... lds, per-lane source offsets from an
// LDS table; border units read out of range and land as zeros) with counted vmcnt waits.
//
// Common rules of both kernels:
//   * LDS images are laid out so that every fragment read is bank-conflict-free
//     (scripts/lds_conflicts.py models the reads) AND every fragment address is a per-lane
//     base register plus a compile-time immediate.
//   * one barrier per frame: past it, every wave is done with the previous frame, whose
//     slot takes the DMA of frame + 2 at once.
//   * the weight-gradient waves issue all DMA (the data-gradient waves carry the dX
//     stores, which are issue-bound per instruction); dX goes straight from registers
//     to memory, 16 bytes per lane.
//   * fragment reads of step k+1 are issued between the MFMAs of step k
//     (sched_group_barrier pins the interleave).
// =====================================================================================

// conv2 backward LDS images (bank-conflict-free for every fragment read; MI355X_MICROARCH.md
// §LDS: a wave's ds_read_b128 is served in 16-lane groups, ds_read_b64_tr_b16 in 32-lane
// groups, each group conflict-free when its lanes cover 256 distinct bytes mod 256):
//   X (a1, 20x20x32): parity-class planes, pixel (iy, ix) -> plane 2(iy&1) + (ix&1), position
//     (iy>>1)*10 + (ix>>1), 64 B per pixel. The wgrad im2col read of 4 consecutive output
//     pixels then hits 4 consecutive positions (a 256-B run) and every tap is an immediate.
//   dY (da2, 9x9x64, zero border): 16-B channel chunk c of bordered pixel (Y, X) at unit
//     s + 128c + Z(c), s = 10Y + X, Z(c) = 8(c&1) + 4((c>>1)&1). Rows are 10 units apart, so
//     the right border (Y, 10) aliases (Y+1, 0) -- both zero. A class pixel ri of the dgrad
//     reads s = ri + 11 - 10kty - ktx, i.e. bank unit ri + const, and chunks c, c+1 sit 8
//     units apart: with lanes 8..15 of each 16-pixel tile swapped by 4 (sig below) the two
//     16-lane groups of a ds_read_b128 are conflict-free. The wgrad walks the reduction over
//     s = 11..106 (zero where dY is border), 4 consecutive s x chunk offsets {0, 8, 4, 12}.
// Both images arrive by LDS-DMA gathers whose per-lane source offsets sit in LDS tables.
namespace c2 {
constexpr int XB = 20 * 20 * 64;             // 25,600: a1 image (class planes)
constexpr int DYB = 16 * 1024;               // 1,019 used units of 16 B -> 16 KiB
constexpr int SLOT = XB + DYB;               // 41,984
[[maybe_unused]] constexpr int RING = 3;
constexpr int NX = XB / 1024, NDY = DYB / 1024;  // 25 + 16 pieces
static_assert(NX + NDY == 41, "c2_issue assigns 10 pieces to each of waves 0-3 + 1 to wave 0");
__host__ __device__ constexpr int zc(int c) { return 8 * (c & 1) + 4 * ((c >> 1) & 1); }
}  // namespace c2

__device__ __forceinline__ uint32_t c2_x_src(int u) {  // X image unit -> a1 byte offset
    const int P = u / 400, rem = u - 400 * P, pos = rem >> 2, c = rem & 3;
    const int py = pos / 10, px = pos - 10 * py;
    return (uint32_t)(((2 * py + (P >> 1)) * 20 + 2 * px + (P & 1)) * 64 + 16 * c);
}
__device__ __forceinline__ uint32_t c2_dy_src(int v) {  // dY image unit -> da2 byte offset
    const int c = v >> 7, k = (v & 127) - c2::zc(c), Y = k / 10, X = k - 10 * Y;
    const bool inside = k >= 0 && k <= 110 && Y >= 1 && Y <= 9 && X >= 1 && X <= 9;
    return inside ? (uint32_t)(((Y - 1) * 9 + X - 1) * 128 + 16 * c) : FI_OOB;
}

// 8 waves, two per SIMD: waves 0-3 compute the weight gradient (wave = kernel row ky),
// waves 4-7 the data gradient (wave = parity class), sharing one frame pipeline.
struct C2Ctx {
    const __bf16 *a1, *da2;
    __bf16* da1;
    int nframes;
};

// pieces j = w + 4i (< 41) of frame f, X 0..24 and dY 25..40, issued by the weight-gradient
// waves w = 0..3 only (ten each, an eleventh for wave 0): their MFMA work is the shorter one,
// and the data-gradient waves' 16-byte dX stores would otherwise sit in front of the DMA in
// their memory queue. All table reads first (one LDS round trip), base + immediate
// addressing, the X/dY switch a scalar select.
__device__ __forceinline__ void c2_issue(const C2Ctx& c, const uint32_t* tab, int f, uint32_t slot_lds, int w,
                                         int lane) {
    const fi_i32x4 xr = make_rsrc(c.a1 + (size_t)f * 12800, 25600);
    const fi_i32x4 dr = make_rsrc(c.da2 + (size_t)f * 5184, 10368);
    const uint32_t* tb = tab + 64 * w + lane;
    uint32_t o[11];
#pragma unroll
    for (int i = 0; i < 10; ++i) o[i] = tb[256 * i];
    if (w == 0) o[10] = tb[256 * 10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int j = w + 4 * i;
        blds16(j < c2::NX ? xr : dr, o[i], slot_lds + j * 1024);
    }
    if (w == 0) blds16(dr, o[10], slot_lds + 40 * 1024);
}

template <class Work>
__device__ __forceinline__ void c2_frames(const C2Ctx& c, char* smem, int nst, Work&& work) {
    const int lane = threadIdx.x & 63, w = wave_id(), tid = threadIdx.x;
    const uint32_t lds0 = lds_addr(smem);
    // per-unit source offsets of both gathers (FI_OOB for border / gap units)
    uint32_t* tab = (uint32_t*)(smem + c2::RING * c2::SLOT);
    for (int i = tid; i < c2::SLOT / 16; i += 512) tab[i] = i < c2::XB / 16 ? c2_x_src(i) : c2_dy_src(i - c2::XB / 16);
    __syncthreads();
    const int npw = w == 0 ? 11 : (w < 4 ? 10 : 0);  // pieces per wave
    const int nmine = c.nframes > (int)blockIdx.x ? (c.nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    int issued = 0, m0 = 0, m1 = 0;
    for (int i = 0; i < 2 && i < nmine; ++i) {
        if (w < 4) c2_issue(c, tab, blockIdx.x + i * gridDim.x, lds0 + i * c2::SLOT, w, lane);
        issued += npw;
        if (i == 0) m0 = issued; else m1 = issued;
    }
    for (int it = 0; it < nmine; ++it) {
        const int f = blockIdx.x + it * gridDim.x;
        wait_vmcnt(issued - m0);
        lds_barrier();  // frame it landed; frame it-1 consumed by every wave
        int m2 = 0;
        if (it + 2 < nmine) {
            if (w < 4) c2_issue(c, tab, f + 2 * gridDim.x, lds0 + ((it + 2) % 3) * c2::SLOT, w, lane);
            issued += npw;
            m2 = issued;
        }
        work(smem + (it % 3) * c2::SLOT, f);
        issued += nst;
        m0 = m1;
        m1 = m2;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(512, 2) void conv2_bwd_fr(const __bf16* __restrict__ a1,
                                                       const __bf16* __restrict__ da2,
                                                       const __bf16* __restrict__ w2d,  // [4][32][256]
                                                       __bf16* __restrict__ da1,
                                                       float* __restrict__ slab,     // [grid][512][64]
                                                       float* __restrict__ cs_slab,  // [grid][64]
                                                       int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c2::RING * c2::SLOT + c2::SLOT / 16 * 4];
    const int lane = threadIdx.x & 63;
    const int w = wave_id(), wr = w & 3;
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, h = lane >> 5, col = lane & 31;
    const C2Ctx ctx{a1, da2, da1, nframes};

    if (w < 4) {
        // ---------------- weight gradient: taps ky = wr, kx = 0..3, co halves ct. The reduction
        // runs over dY units s = 11 + mu (output pixel (oy, ox) = divmod(s - 11, 10); ox = 9 and
        // s >= 100 are zero border in dY, so whatever the A read there returns adds nothing).
        // A tap kx: class plane 2(wr&1) + (kx&1), position + (kx>>1) -> immediate 6400(kx&1) + 64(kx>>1).
        // lane bases for mu = 8(g>>1) + q; step ms and half hh add 16ms + 4hh (linear layouts:
        // every fragment address is one of two base registers plus an immediate)
        const int mu0 = 8 * (g >> 1) + q, c = 2 * (g & 1) + (p4 >> 1);
        const int ba0 = 64 * (200 * (wr & 1) + mu0 + 10 * (wr >> 1)) + 2 * (16 * (g & 1) + 4 * p4);
        const int bb0 = c2::XB + 16 * (11 + mu0 + 128 * c + c2::zc(c)) + 8 * (p4 & 1);
        f32x16 accw[4][2];
#pragma unroll
        for (int t = 0; t < 4; ++t) { accw[t][0] = f32x16{}; accw[t][1] = f32x16{}; }
        float bsum0 = 0.f, bsum1 = 0.f;
        c2_frames(ctx, smem, 0, [&](const char* X, int) {
            // software pipeline: the 6 fragments of step ms+1 (12 transposed reads) are issued
            // between the 8 MFMAs of step ms; sched_group_barrier pins that interleave
            bf16x8 fb[2][6];  // [0] b0, [1] b1, [2..5] A of kx = 0..3
            const char* XA = X + ba0;
            const char* XB_ = X + bb0;
            auto load = [&](int ms, bf16x8* d) {
                const int ob = 16 * 16 * ms, oa = 64 * 16 * ms;
                d[0] = tr2(XB_ + ob, XB_ + ob + 64);
                d[1] = tr2(XB_ + ob + 8192, XB_ + ob + 64 + 8192);  // chunk + 4
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int ao = oa + 6400 * (t & 1) + 64 * (t >> 1);
                    d[2 + t] = tr2(XA + ao, XA + ao + 256);
                }
            };
            load(0, fb[0]);
            __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
            for (int ms = 0; ms < 6; ++ms) {
                const bf16x8* cur = fb[ms & 1];
                if (ms + 1 < 6) load(ms + 1, fb[(ms + 1) & 1]);
                bsum0 = sum8_bf16(cur[0], bsum0);  // bias: column sums of dY (kept by wave 0)
                bsum1 = sum8_bf16(cur[1], bsum1);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    accw[t][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + t], cur[0], accw[t][0], 0, 0, 0);
                    accw[t][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + t], cur[1], accw[t][1], 0, 0, 0);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (ms + 1 < 6) {
                        if (k < 4) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                        else __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                }
            }
        });
        c2w_flush(accw, slab + (size_t)blockIdx.x * 512 * 64, wr, h, col, false);
        // lanes l and l+32 hold the same co (16*(g&1) + (l&15)), other m half; cs_slab has the
        // [grid][2][64] layout of conv21_bwd_fr's (row 1 zero), unless conv3_bwd fills it (FI_C2B_C3)
        if (!FI_C2B_C3 && wr == 0) {
            const float o0 = __shfl_xor(bsum0, 32, 64), o1 = __shfl_xor(bsum1, 32, 64);
            float* cb = cs_slab + (size_t)blockIdx.x * 128;
            if (lane < 32) {
                cb[lane] = bsum0 + o0;
                cb[32 + lane] = bsum1 + o1;
            } else {
                cb[64 + lane - 32] = 0.f;
                cb[96 + lane - 32] = 0.f;
            }
        }
    } else {
        // ---------------- data gradient, parity class (wr>>1, wr&1), transposed on 16x16x32:
        // D[ci][pixel] = W_cls^T dYcol^T with the class slice of W2 as the register-resident A
        // operand; 7 pixel tiles of 16 cover the class's 100 pixels. A row i of channel tile nt
        // is channel 8(i>>2) + 4nt + (i&3), so lane group g ends with channels 8g..8g+7 of its
        // pixel in acc[pt][0..1]: one 16-byte store of (a1 > 0) * dX per pixel tile.
        const int ty = wr >> 1, tx = wr & 1;
        bf16x8 bw[2][8];  // lane holds W[ci = 8(i>>2) + 4nt + (i&3), i = lane&15][k = 32ks + 8g..+8]
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const int i = lane & 15, ci = 8 * (i >> 2) + 4 * nt + (i & 3);
                bw[nt][ks] = *(const bf16x8*)(w2d + ((size_t)(wr * 32 + ci)) * 256 + 32 * ks + 8 * g);
            }
        // lane i of pixel tile pt holds class pixel ri = 16pt + sig(i), sig swapping lanes 8..15 by 4
        // dY unit of (iyq + 1, ixq + 1) in chunk g: tiles 0..5 are bd0 + 256pt, tile 6 is clamped;
        // tap (kty, ktx) adds 11 - 10kty - ktx units
        const int si = (lane & 15) ^ (((lane & 15) >> 1) & 4);
        const int bd0 = c2::XB + 16 * (si + 128 * g + c2::zc(g));
        const int bd6 = c2::XB + 16 * (min(96 + si, 99) + 128 * g + c2::zc(g));
        c2_frames(ctx, smem, 7, [&](const char* X, int f) {
            // pixel tile outer: each tile's 16 MFMAs (two accumulator chains; 16x16x32 chains
            // issue back to back) end in its own masked 16-byte store, so the dX stores spread
            // over the frame instead of queueing as a burst. The next tile's 8 fragments are
            // read between the current tile's MFMAs (sched_group_barrier pins the interleave).
            u32x4* dst = (u32x4*)(ctx.da1 + (size_t)f * 12800);
            bf16x8 fb[2][8];
            auto load = [&](int pt, bf16x8* d) {  // k = 64 tap + co: tap = ks>>1, co half = ks&1 (chunk + 4)
                const char* base = X + (pt < 6 ? bd0 + 256 * pt : bd6);
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) {
                    const int tap = ks >> 1, kty = tap >> 1, ktx = tap & 1;
                    d[ks] = *(const bf16x8*)(base + 16 * (11 - 10 * kty - ktx) + 8192 * (ks & 1));
                }
            };
            load(0, fb[0]);
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
            for (int pt = 0; pt < 7; ++pt) {
                const bf16x8* cur = fb[pt & 1];
                if (pt + 1 < 7) load(pt + 1, fb[(pt + 1) & 1]);
                f32x4 acc0 = f32x4{}, acc1 = f32x4{};
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[0][ks], cur[ks], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[1][ks], cur[ks], acc1, 0, 0, 0);
                }
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    if (pt + 1 < 7) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                // 7 stores per frame (nst above); tile 6 holds 4 pixels
                const int ri = pt * 16 + si;
                if (pt < 6 || ri < 100) {
                    const int iyq = ri / 10, ixq = ri - 10 * iyq;
                    const int pix = (2 * iyq + ty) * 20 + 2 * ixq + tx;
                    const s16x8 m = *(const s16x8*)(X + 64 * (100 * wr + ri) + 16 * g);
                    bf16x8 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        o[r] = m[r] > 0 ? (__bf16)acc0[r] : (__bf16)0.f;
                        o[4 + r] = m[4 + r] > 0 ? (__bf16)acc1[r] : (__bf16)0.f;
                    }
                    FI_ST16(__builtin_bit_cast(u32x4, o), dst + 4 * pix + g);
                }
            }
        });
    }
}

int conv2_bwd_fr_launch(const __bf16* a1, const __bf16* da2, const __bf16* w2d, __bf16* da1, float* slab,
                        float* cs_slab, int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv2_bwd_fr, dim3(grid), dim3(512), 0, s, a1, da2, w2d, da1,
                       slab, cs_slab, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// =====================================================================================
// Fused conv2 backward + conv1 weight gradient (frame-resident): da1 never touches HBM.
// Per frame, conv2's data gradient da1 = (a1 > 0) * dgrad(da2, W2) is written into an LDS
// tile [400 pixels][32 channels] (conv1_wgrad_fr's layout with the 16-B chunks of a row
// XOR-swizzled) and conv1's weight gradient reads it from there. HBM per frame: a1 25,600 + da2 10,368 + raw frame
// 28,224 = 64,192 B, against 61,568 + 53,824 B for conv2_bwd_fr + conv1_wgrad_fr.
// 8 waves, two per SIMD, two barriers per frame:
//   [B1] phase 1: waves 0-3 compute conv2's weight gradient exactly as conv2_bwd_fr (kernel
//        row ky = w, 128 accumulators), then convert the raw frame (held in their registers,
//        loaded one frame ahead; FI_C21_NRAW_A < 7 moves a share to waves 4-7, measured
//        slower: their loads in flight stall phase 2) into the bf16 pair-plane image I;
//        waves 4-7 compute conv2's data gradient (parity class) and write the masked da1
//        into the LDS tile D;
//   [B2] waves 0-3 queue the next frames' a1 / da2 DMA, all waves the next raw frame's
//        loads; phase 2: conv1's weight gradient on waves 4-7 (kernel rows 2wr, 2wr+1 over
//        the 25 16-pixel m-steps; both operands by transposed LDS reads).
// LDS: a1 class-plane image x2 (double-buffered: frame it+2 is DMA'd during frame it),
// bordered da2 image (single: frame it+1 DMA'd after B2), I, D, the DMA gather table:
//   2 x 25,600 + 16,384 + 56,576 + 25,600 + 10,496 = 160,256 B.
// Weight-gradient partials: conv2 [grid][512][64] (+ bias [grid][64]) as conv2_bwd_fr;
// conv1 [grid][256][32] (x 1/255) as conv1_wgrad_fr; conv1's bias partials come from the
// data-gradient epilogue, one per parity-class wave: [grid][4][32].
// =====================================================================================
namespace c21 {
constexpr int AXB = c2::XB;                              // 25,600
constexpr int DYB = c2::DYB;                             // 16,384
constexpr int O_AX = 0;                                  // 2 slots
constexpr int O_DY = 2 * AXB;
constexpr int O_IMG = O_DY + DYB;
constexpr int O_D = O_IMG + c1::IMG;
constexpr int O_TAB = O_D + c1::OUT;
constexpr int LDS = O_TAB + (c2::XB + c2::DYB) / 16 * 4;  // 160,256
#ifndef FI_C21_NRAW_A
#define FI_C21_NRAW_A 7
#endif
constexpr int NRAW_A = FI_C21_NRAW_A;  // 16-B raw-frame units per lane converted by waves 0-3
constexpr int NRAW_B = 7 - NRAW_A;     // ... by waves 4-7 (the rest of the 1,764)

static_assert(256 * (NRAW_A + NRAW_B) >= c1::FRAME_LOADS, "raw-frame split");
}  // namespace c21

template <bool KEEP_DA1>  // KEEP_DA1: also store da1 to HBM (parity checks); no branch in the hot loop
__global__ __launch_bounds__(512, 2) void conv21_bwd_fr(const __bf16* __restrict__ a1,
                                                        const __bf16* __restrict__ da2,
                                                        const __bf16* __restrict__ w2d,  // [4][32][256]
                                                        const uint8_t* __restrict__ frames,
                                                        __bf16* __restrict__ da1_out,  // optional (parity checks)
                                                        float* __restrict__ slab2,     // [grid][512][64]
                                                        float* __restrict__ cs2,       // [grid][2][64] (unless FI_C2B_C3)
                                                        float* __restrict__ slab1,     // [grid][SEGS][256][32]
                                                        float* __restrict__ cs1,       // [grid][4 waves][32]
                                                        int nframes, int a1_planar) {
    __shared__ __attribute__((aligned(16))) char smem[c21::LDS];
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int w = wave_id(), wr = w & 3;
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, h = lane >> 5, col = lane & 31;
    // waves 4-7 carry the critical path (conv2's data gradient, then conv1's weight gradient;
    // per-phase clocks: 6.3k + 2.7k per frame against waves 0-3's 1.5k + 1.8k + 3.8k parked at
    // the barriers): at s_setprio 1 their MFMAs and VALU win the SIMD's arbitration and waves
    // 0-3 fill the gaps (MI355X_MICROARCH.md, two waves per SIMD, item 4): 8.32 -> 7.89 ms.
    // The same for conv12_fwd / conv3_bwd (either half) measured time-neutral.
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
    const uint32_t lds0 = lds_addr(smem);
    uint32_t* tab = (uint32_t*)(smem + c21::O_TAB);
    // a1 planar (conv12_fwd_fr wrote it in this image's order): the a1 pieces are linear 1-KiB
    // runs; NHWC: 16-byte gathers at a 128-byte stride
    for (int i = tid; i < (c2::XB + c2::DYB) / 16; i += 512)
        tab[i] = i < c2::XB / 16 ? (a1_planar ? 16u * i : c2_x_src(i)) : c2_dy_src(i - c2::XB / 16);
    char* DY = smem + c21::O_DY;
    char* IMG = smem + c21::O_IMG;
    char* D = smem + c21::O_D;
    const int nmine = nframes > (int)blockIdx.x ? (nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    // The weight-gradient im2col reads of the last m-step run up to ~450 B past the end of an
    // a1 slot (those rows meet zero dY borders, so they add 0 * value): the bytes there must be
    // finite. Past slot 1 lies the da2 image; past slot 0 lies slot 1, which is zeroed here when
    // no frame will ever be DMA'd into it.
    if (nmine < 2 && tid < 64) ((u32x4*)(smem + c21::O_AX + c21::AXB))[tid] = u32x4{0, 0, 0, 0};
    __syncthreads();
    auto frame_of = [&](int k) { return (int)blockIdx.x + k * (int)gridDim.x; };

    // conv1 weight gradient (phase 2, waves 4-7): wave 4 + wr owns k-tiles (kernel rows) 2wr and
    // 2wr + 1 over the 25 m-steps of 16 pixels; A^T from the frame image and da1 from D, both
    // by transposed reads, every da1 fragment feeding two MFMAs (four k-tiles per wave over
    // half the m-steps measured slower: fewer registers left for reading ahead)
    // da1 tile D: row m (pixel) of 64 B, 16-B chunk c stored at slot c ^ ((m >> 1) & 3) -- the
    // data-gradient waves' writes (8 lanes on 8 class pixels two apart) then hit 4 slots instead
    // of one bank group; the transposed reads stay conflict-free and their swizzle is the same
    // for every m-step (m = 16 ms + m0: bits 1-2 of m come from m0)
    auto dsw = [](int m, int c) { return 64 * m + 16 * (c ^ ((m >> 1) & 3)); };
    const int dc = 2 * (g & 1) + (p4 >> 1);
    const int db0 = dsw(8 * (g >> 1) + q, dc) + 8 * (p4 & 1), db1 = dsw(8 * (g >> 1) + q + 4, dc) + 8 * (p4 & 1);
    f32x16 acc1[2] = {};  // this segment's frames (blocked accumulation, SEGS above)
    // conv1's bias gradient = column sums of da1: the B fragment of m-step ms holds 8 pixels of
    // channel lane & 31, so wave 4 + wr sums the fragments of m-steps ms = wr (mod 4) beside its
    // MFMAs (4 v_dot2 in a 64-cycle MFMA pair) instead of 16 VALU per tile in the phase-1 epilogue
    float bsum1 = 0.f;
    auto conv1_wgrad = [&](auto wrc) {  // wrc: wr as a compile-time constant (the bias split)
        // im2col offset of lane row m = 16ms + m0 (m0 = 8(g>>1) + q + 4hh < 16): output pixel
        // (oy, ox) = divmod(m, 20), input pixel (4oy + ky, 4ox + kx) with kx = 4(g&1) + p4, so
        // offset = base + 16 (m + 64 oy); with 16ms = 20a + b (compile time), oy = a + [m0 >= 20 - b]
        int ua[2], m0a[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int m0 = fi_opaque(8 * (g >> 1) + q + 4 * hh);
            const int kx = 4 * (g & 1) + p4;
            m0a[hh] = m0;
            ua[hh] = ((kx >> 1) & 1) * c1::PLANE + 16 * ((2 * wr) * 21 + (kx >> 2)) + 8 * (kx & 1) + 16 * m0;
        }
        auto aoff = [&](int ms, int hh) {
            const int a = 16 * ms / 20, b = 16 * ms - 20 * a;
            return ua[hh] + 16 * (16 * ms + 64 * a) + (m0a[hh] >= 20 - b ? 1024 : 0);
        };
        auto load = [&](int ms, bf16x8* d) {  // [0] da1, [1..2] A of the two k-tiles (m-step ms)
            d[0] = tr2(D + db0 + 1024 * ms, D + db1 + 1024 * ms);
            const int o0 = aoff(ms, 0), o1 = aoff(ms, 1);
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) d[1 + kt] = tr2(IMG + o0 + 336 * kt, IMG + o1 + 336 * kt);
        };
        constexpr int PD = 3;  // m-steps read ahead
        bf16x8 fb[PD + 1][3];
#pragma unroll
        for (int ms = 0; ms < PD; ++ms) load(ms, fb[ms]);
#pragma unroll
        for (int ms = 0; ms < 25; ++ms) {
            if (ms + PD < 25) load(ms + PD, fb[(ms + PD) % (PD + 1)]);
            const bf16x8* cur = fb[ms % (PD + 1)];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
                acc1[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[1 + kt], cur[0], acc1[kt], 0, 0, 0);
            if constexpr (FI_C1B_PH2) {
                if ((ms & 3) == decltype(wrc)::value) bsum1 = sum8_bf16(cur[0], bsum1);
            }
        }
    };

    if (w < 4) {
        // ---------------- conv2 weight gradient (as conv2_bwd_fr), raw-frame conversion,
        // all a1 / da2 DMA
        auto issue_ax = [&](int k, int slot) {  // pieces j = w + 4i < 25 of frame k's a1 image
            const fi_i32x4 xr = make_rsrc(a1 + (size_t)frame_of(k) * 12800, 25600);
            const uint32_t base = lds0 + c21::O_AX + slot * c21::AXB;
            uint32_t o[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) o[i] = tab[64 * min(w + 4 * i, c2::NX - 1) + lane];
            int n = 0;
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                const int j = w + 4 * i;
                if (j < c2::NX) {
                    blds16(xr, o[i], base + 1024 * j);
                    ++n;
                }
            }
            return n;
        };
        auto issue_dy = [&](int k) {  // pieces w + 4i of frame k's bordered da2 image
            const fi_i32x4 dr = make_rsrc(da2 + (size_t)frame_of(k) * 5184, 10368);
            uint32_t o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = tab[64 * (c2::NX + w + 4 * i) + lane];
#pragma unroll
            for (int i = 0; i < 4; ++i) blds16(dr, o[i], lds0 + c21::O_DY + 1024 * (w + 4 * i));
            return 4;
        };
        // raw frame units tid + 256i (< 256 NRAW_A) in registers, loaded one frame ahead (plain loads:
        // the compiler's own vmcnt waits cover them; they are issued after this wave's DMA)
        u32x4 rr[c21::NRAW_A];
        auto load_raw = [&](int k) {
            const u32x4* src = (const u32x4*)(frames + (size_t)frame_of(k) * 28224);
#pragma unroll
            for (int i = 0; i < c21::NRAW_A; ++i) {
                const int u = tid + 256 * i;
                rr[i] = (256 * (i + 1) <= c1::FRAME_LOADS || u < c1::FRAME_LOADS) ? src[u] : u32x4{0, 0, 0, 0};
            }
        };
        const int mu0 = 8 * (g >> 1) + q, c = 2 * (g & 1) + (p4 >> 1);
        const int ba0 = 64 * (200 * (wr & 1) + mu0 + 10 * (wr >> 1)) + 2 * (16 * (g & 1) + 4 * p4);
        const int bb0 = 16 * (11 + mu0 + 128 * c + c2::zc(c)) + 8 * (p4 & 1);
        f32x16 accw[4][2];
#pragma unroll
        for (int t = 0; t < 4; ++t) { accw[t][0] = f32x16{}; accw[t][1] = f32x16{}; }
        float bsum0 = 0.f, bsum1_ = 0.f;
        int issued = 0, m_dy = 0;
        if (nmine > 0) issued += issue_ax(0, 0);
        if (nmine > 1) issued += issue_ax(1, 1);
        if (nmine > 0) issued += issue_dy(0);
        m_dy = issued;
        if (nmine > 0) {
            load_raw(0);
            issued += c21::NRAW_A;
        }
        for (int it = 0; it < nmine; ++it) {
            wait_vmcnt(issued - m_dy);  // own pieces of da2(it) landed (a1(it) is older)
            lds_barrier();  // B1: frame it's images in LDS; frame it-1's D and image consumed
            {
                const char* XA = smem + c21::O_AX + (it & 1) * c21::AXB + ba0;
                const char* XB_ = DY + bb0;
                bf16x8 fb[2][6];  // [0] b0, [1] b1, [2..5] A of kx = 0..3
                auto load = [&](int ms, bf16x8* d) {
                    const int ob = 16 * 16 * ms, oa = 64 * 16 * ms;
                    d[0] = tr2(XB_ + ob, XB_ + ob + 64);
                    d[1] = tr2(XB_ + ob + 8192, XB_ + ob + 64 + 8192);  // chunk + 4
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int ao = oa + 6400 * (t & 1) + 64 * (t >> 1);
                        d[2 + t] = tr2(XA + ao, XA + ao + 256);
                    }
                };
                load(0, fb[0]);
                __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
                for (int ms = 0; ms < 6; ++ms) {
                    const bf16x8* cur = fb[ms & 1];
                    if (ms + 1 < 6) load(ms + 1, fb[(ms + 1) & 1]);
                    if constexpr (!FI_C2B_C3) {
                        bsum0 = sum8_bf16(cur[0], bsum0);
                        bsum1_ = sum8_bf16(cur[1], bsum1_);
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        accw[t][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + t], cur[0], accw[t][0], 0, 0, 0);
                        accw[t][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + t], cur[1], accw[t][1], 0, 0, 0);
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        if (ms + 1 < 6) {
                            if (k < 4) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                            else __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < c21::NRAW_A; ++i) {  // raw(it) -> bf16 pair-plane image (free since B1)
                const int u = tid + 256 * i;
                if (256 * (i + 1) <= c1::FRAME_LOADS || u < c1::FRAME_LOADS) {
                    bf16x8 lo, hi;
                    u8x16_to_bf16(rr[i], lo, hi);
                    *(bf16x8*)(IMG + 16 * u) = lo;
                    *(bf16x8*)(IMG + c1::PLANE + 16 * u) = hi;
                }
            }
            // raw(it + 1) goes out now, while this wave waits at B2 for the data-gradient
            // waves: in phase 2 its issue would queue behind the DMA (several thousand clocks
            // of issue stall per frame with both there)
            if (it + 1 < nmine) {
                load_raw(it + 1);
                issued += c21::NRAW_A;
            }
            lds_barrier();  // B2: D and the image complete; da2 image and a1 slot it&1 consumed
            if (it + 1 < nmine) {
                issued += issue_dy(it + 1);
                m_dy = issued;
            }
            if (it + 2 < nmine) issued += issue_ax(it + 2, it & 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        c2w_flush(accw, slab2 + (size_t)blockIdx.x * 512 * 64, wr, h, col, false);
        if constexpr (!FI_C2B_C3) {  // cs2[block][0][64] (row [1] zero: the layout conv3_bwd fills otherwise)
            if (wr == 0) {
                const float o0 = __shfl_xor(bsum0, 32, 64), o1 = __shfl_xor(bsum1_, 32, 64);
                float* cb = cs2 + (size_t)blockIdx.x * 128;
                if (lane < 32) {
                    cb[lane] = bsum0 + o0;
                    cb[32 + lane] = bsum1_ + o1;
                } else {
                    cb[64 + lane - 32] = 0.f;
                    cb[96 + lane - 32] = 0.f;
                }
            }
        }
    } else {
        // ---------------- conv2 data gradient -> D
        const int ty = wr >> 1, tx = wr & 1;
        bf16x8 bw[2][8];  // W2 class slice (conv2_bwd_fr)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const int i = lane & 15, ci = 8 * (i >> 2) + 4 * nt + (i & 3);
                bw[nt][ks] = *(const bf16x8*)(w2d + ((size_t)(wr * 32 + ci)) * 256 + 32 * ks + 8 * g);
            }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the weights are in before the frame loop
        const int t4 = tid - 256;
        u32x4 rr[c21::NRAW_B > 0 ? c21::NRAW_B : 1];  // raw units 256 NRAW_A + t4 + 256i, one frame ahead
        auto load_raw = [&](int k) {
            const u32x4* src = (const u32x4*)(frames + (size_t)frame_of(k) * 28224);
#pragma unroll
            for (int i = 0; i < c21::NRAW_B; ++i) {
                const int u = 256 * c21::NRAW_A + t4 + 256 * i;
                rr[i] = u < c1::FRAME_LOADS ? src[u] : u32x4{0, 0, 0, 0};
            }
        };
        if (nmine > 0) load_raw(0);
        const int si = (lane & 15) ^ (((lane & 15) >> 1) & 4);
        const int bd0 = 16 * (si + 128 * g + c2::zc(g));
        const int bd6 = 16 * (min(96 + si, 99) + 128 * g + c2::zc(g));
        float bs8[8] = {};  // !FI_C1B_PH2: conv1 bias partials, channels 8g + j of this lane's da1 pixels
        // conv1 segment slab out, rows k = 32(2wr + kt) + (r&3) + 8(r>>2) + 4(lane>>5) (x 1/255);
        // plain buffer stores, no drain: these waves issue no counted DMA
        int sg = 0;
        auto c1_flush = [&]() {
            const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
                slab1 + ((size_t)blockIdx.x * SEGS + sg) * 256 * 32 + 64 * wr * 32, 0, 64 * 32 * 4, 0x00020000);
            const int vo1 = fi_opaque((4 * h * 32 + col) * 4);
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) {
                    const float v = acc1[kt][rr] * (1.0f / 255.0f);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r1, vo1,
                                                          ((32 * kt + (rr & 3) + 8 * (rr >> 2)) * 32) * 4, 0);
                }
                acc1[kt] = f32x16{};
            }
            ++sg;
        };
        for (int it = 0; it < nmine; ++it) {
            const int f = frame_of(it);
            lds_barrier();  // B1
            {  // conv2 data gradient of class (ty, tx) -> D (and da1_out)
                const char* X = smem + c21::O_AX + (it & 1) * c21::AXB;
                u32x4* dst = KEEP_DA1 ? (u32x4*)(da1_out + (size_t)f * 12800) : nullptr;
                // step st = (pixel tile pt, k-step ks): dY fragment read PD steps ahead
                auto frag = [&](int st) {
                    const int pt = st >> 3, ks = st & 7, tap = ks >> 1, kty = tap >> 1, ktx = tap & 1;
                    return *(const bf16x8*)(DY + (pt < 6 ? bd0 + 256 * pt : bd6) + 16 * (11 - 10 * kty - ktx) +
                                            8192 * (ks & 1));
                };
                constexpr int PD = 6, NSTEP = 7 * 8;
                bf16x8 fb[PD + 1];
#pragma unroll
                for (int st = 0; st < PD; ++st) fb[st] = frag(st);
                __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
                // the (a1 > 0) mask of a tile is read when the tile starts, a tile's MFMAs
                // before its epilogue needs it
                auto mask_of = [&](int pt) {
                    return *(const s16x8*)(X + 64 * (100 * wr + min(pt * 16 + si, 99)) + 16 * g);
                };
                // tile pt's epilogue: mask by (a1 > 0), into D (and da1_out): the bf16 pairs and
                // the mask are handled per 32-bit word (3 packed ops per pair instead of two
                // compares, two selects and the repacking)
                auto epilogue = [&](int pt, const f32x4& e0, const f32x4& e1, const s16x8& m) {
                    const int ri = pt * 16 + si;
                    if (pt < 6 || ri < 100) {
                        const int iyq = ri / 10, ixq = ri - 10 * iyq;
                        const int pix = (2 * iyq + ty) * 20 + 2 * ixq + tx;
                        u32x4 ov;
                        if constexpr (FI_C21_PKMASK) {
                            const u32x4 mw = __builtin_bit_cast(u32x4, m);
                            ov = u32x4{relu_mask_pair(e0[0], e0[1], mw[0]), relu_mask_pair(e0[2], e0[3], mw[1]),
                                       relu_mask_pair(e1[0], e1[1], mw[2]), relu_mask_pair(e1[2], e1[3], mw[3])};
                        } else {
                            bf16x8 o;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                o[r] = m[r] > 0 ? (__bf16)e0[r] : (__bf16)0.f;
                                o[4 + r] = m[4 + r] > 0 ? (__bf16)e1[r] : (__bf16)0.f;
                            }
                            ov = __builtin_bit_cast(u32x4, o);
                        }
                        *(u32x4*)(D + dsw(pix, g)) = ov;
                        if constexpr (!FI_C1B_PH2) {
                            const bf16x8 o = __builtin_bit_cast(bf16x8, ov);
#pragma unroll
                            for (int j = 0; j < 8; ++j) bs8[j] += (float)o[j];
                        }
                        if constexpr (KEEP_DA1) FI_ST16(ov, dst + 4 * pix + g);
                    }
                };
                s16x8 mk = mask_of(0);
                f32x4 ac0 = f32x4{}, ac1 = f32x4{};
                // (a software-pipelined form -- tile pt-1's epilogue spread over tile pt's MFMAs --
                // measured slower: 6.2k -> 6.8k clocks per frame for this phase)
#pragma unroll
                for (int st = 0; st < NSTEP; ++st) {
                    const int pt = st >> 3, ks = st & 7;
                    if (st + PD < NSTEP) fb[(st + PD) % (PD + 1)] = frag(st + PD);
                    const bf16x8 b = fb[st % (PD + 1)];
                    ac0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[0][ks], b, ac0, 0, 0, 0);
                    ac1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[1][ks], b, ac1, 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    if (st + PD < NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    if (ks == 7) {
                        const s16x8 m = mk;
                        if (pt + 1 < 7) mk = mask_of(pt + 1);
                        epilogue(pt, ac0, ac1, m);
                        ac0 = f32x4{};
                        ac1 = f32x4{};
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < c21::NRAW_B; ++i) {  // raw(it), the last units -> image
                const int u = 256 * c21::NRAW_A + t4 + 256 * i;
                if (u < c1::FRAME_LOADS) {
                    bf16x8 lo, hi;
                    u8x16_to_bf16(rr[i], lo, hi);
                    *(bf16x8*)(IMG + 16 * u) = lo;
                    *(bf16x8*)(IMG + c1::PLANE + 16 * u) = hi;
                }
            }
            lds_barrier();  // B2: D and the image complete
            if (it + 1 < nmine) load_raw(it + 1);
            switch (wr) {  // the bias split is compile-time per wave (no branch in the m-step loop)
                case 0: conv1_wgrad(std::integral_constant<int, 0>{}); break;
                case 1: conv1_wgrad(std::integral_constant<int, 1>{}); break;
                case 2: conv1_wgrad(std::integral_constant<int, 2>{}); break;
                default: conv1_wgrad(std::integral_constant<int, 3>{}); break;
            }
            // a segment ends here (at most one per frame once nmine >= SEGS; with fewer frames than
            // SEGS, seg_last(0) is -1, so every frame lands in segment 0 and the trailing segments
            // are written as zero slabs after the loop). Marked unlikely: the block is placed out of the frame loop's code -- the
            // flush inlined in line cost conv21 0.45 ms though it runs 8 times per workgroup
            if (__builtin_expect(it == seg_last(sg, nmine), 0)) c1_flush();
        }
        while (sg < SEGS) c1_flush();  // the remaining segments (zero slabs unless nmine < SEGS)
        // conv1 bias partial of this wave: channel lane & 31, the two pixel halves of the B
        // fragments combined
        if constexpr (FI_C1B_PH2) {
            const float other = __shfl_xor(bsum1, 32, 64);
            if (lane < 32) cs1[((size_t)blockIdx.x * 4 + wr) * 32 + lane] = bsum1 + other;
        } else {  // sum over the 16 lanes of each channel group
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) bs8[j] += __shfl_xor(bs8[j], o, 64);
            if ((lane & 15) == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) cs1[((size_t)blockIdx.x * 4 + wr) * 32 + 8 * g + j] = bs8[j];
            }
        }
    }
}

int conv21_bwd_fr_launch(const __bf16* a1, const __bf16* da2, const __bf16* w2d, const uint8_t* frames,
                         __bf16* da1_out, float* slab2, float* cs2, float* slab1, float* cs1, int nframes,
                         int grid, hipStream_t s, int a1_planar) {
    if (da1_out)
        hipLaunchKernelGGL(conv21_bwd_fr<true>, dim3(grid), dim3(512), 0, s, a1, da2, w2d, frames, da1_out, slab2,
                           cs2, slab1, cs1, nframes, a1_planar);
    else
        hipLaunchKernelGGL(conv21_bwd_fr<false>, dim3(grid), dim3(512), 0, s, a1, da2, w2d, frames, da1_out, slab2,
                           cs2, slab1, cs1, nframes, a1_planar);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

// ------------------------------------------------------------------------------------
// conv3 backward (3x3 / stride 1, 9x9x64 -> 7x7x64): same structure as conv2's backward.
// LDS images (bank-conflict-free for every fragment read; checked by scripts/lds_model_c3):
//   X (a2): chunk planes, unit p + 96c + Z(c) for pixel p = 9y + x, 16-B channel chunk c.
//   dY (da3) and M (a3, its ReLU mask): bordered 11x11 (2-pixel border), unit
//     9Y + X + 128c + Z(c) -- rows 9 units apart, so right-border columns alias the next
//     row's left border (zeros either way). A dX pixel ri then reads dY unit
//     ri + 20 - 9ky - kx: bank unit ri + const, and with the tile lanes permuted as in
//     conv2 (sig) both 16-lane groups of a ds_read_b128 are conflict-free.
//   The weight-gradient reduction walks s = 20..83 (dY zero where it is border), A pixel
//     s - 20 + 9ky + kx: 4 consecutive s x chunk offsets {0, 8, 4, 12}.
// a3 (da3's ReLU mask) arrives beside da3 in the same byte order; the wave that DMAs and
// reshuffles da3 piece j applies the mask of piece j on the way.
// Waves 0-3: weight gradient (k-tiles kt = wr + 4i = (tap 2i + (wr>>1), channel half wr&1))
// and all DMA issue; waves 4-7: data gradient, transposed on 16x16x32 (wave = channel half
// wr&1 x pixel half wr>>1, W3 slice in registers), dX stored from registers.
// ------------------------------------------------------------------------------------
namespace c3 {
constexpr int XB = 12 * 1024;                // 768 units (8 chunk planes of 96)
constexpr int DYB = 16 * 1024;               // 1,009 used units -> 16 KiB
__host__ __device__ constexpr int zc(int c) { return 8 * (c & 1) + 4 * ((c >> 1) & 1); }
}  // namespace c3

struct C3Ctx {
    const __bf16 *a2, *da3, *a3;
    __bf16* da2;
    int nframes;
};

// Linear-DMA pipeline: every frame's a2, da3 and a3 arrive by LDS-DMA in their own byte order
// (1 KiB contiguous per wave instruction) into one of two staging buffers; the issuing wave
// then moves its own landed pieces into the frame's image slot (chunk-planar X, bordered dY),
// applying the a3 ReLU mask to da3 on the way, so the mask image needs no slot. The gathered
// DMA straight into the image layouts issued 16-byte pieces at a 128-byte
// stride: the same bytes, 8x the memory requests (timing with linear sources and wrong
// layouts: 4.29 -> 3.85 ms; the gathered form is no longer built).
// LDS: 2 image slots (X + dY, 28,672 B each; gap / border units zeroed once, never written),
// 2 staging buffers (a2 11 + da3 7 + a3 7 pieces of 1 KiB), destination tables: 110,624 B.
namespace c3 {
constexpr int SLOT2 = XB + DYB;                    // 28,672
constexpr int NPX = 11, NPD = 7;                   // 1-KiB pieces of a2, of da3 (= of a3)
constexpr int STGB = (NPX + 2 * NPD) * 1024;       // 25,600
constexpr int NUX = 10368 / 16, NUD = 6272 / 16;   // 16-B units of a2, of da3
constexpr int O_STG = 2 * SLOT2, O_TAB = O_STG + 2 * STGB;
constexpr int LDS = O_TAB + (NUX + NUD) * 2;       // 110,624
}  // namespace c3

// ISSUER: waves 0-3 (compile-time role, so the data-gradient waves carry none of the DMA /
// reshuffle code); wave w owns a2 pieces w + 4i (< 11) and da3 / a3 pieces w + 4i (< 7)
template <bool ISSUER, class Work>
__device__ __forceinline__ void c3_frames(const C3Ctx& c, char* smem, int nst, Work&& work) {
    const int lane = threadIdx.x & 63, w = wave_id(), tid = threadIdx.x;
    const uint32_t lds0 = lds_addr(smem);
    uint16_t* dstx = (uint16_t*)(smem + c3::O_TAB);
    uint16_t* dsty = dstx + c3::NUX;
    for (int i = tid; i < 2 * c3::SLOT2 / 16; i += 512) ((u32x4*)smem)[i] = u32x4{0, 0, 0, 0};
    for (int i = tid; i < c3::NUX; i += 512) {  // a2 unit (pixel p, chunk cc) -> X image unit
        const int p = i >> 3, cc = i & 7;
        dstx[i] = (uint16_t)(p + 96 * cc + c3::zc(cc));
    }
    for (int i = tid; i < c3::NUD; i += 512) {  // da3 unit (pixel (y, x), chunk cc) -> bordered dY unit
        const int q = i >> 3, cc = i & 7, y = q / 7, x = q - 7 * y;
        dsty[i] = (uint16_t)(9 * (y + 2) + (x + 2) + 128 * cc + c3::zc(cc));
    }
    __syncthreads();
    const int nmine = c.nframes > (int)blockIdx.x ? (c.nframes - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    auto issue = [&](int k, int sb) {  // frame k's pieces of this wave into staging sb
        const int f = blockIdx.x + k * gridDim.x;
        const fi_i32x4 xr = make_rsrc(c.a2 + (size_t)f * 5184, 10368);
        const fi_i32x4 dr = make_rsrc(c.da3 + (size_t)f * 3136, 6272);
        const fi_i32x4 mr = make_rsrc(c.a3 + (size_t)f * 3136, 6272);
        const uint32_t base = lds0 + c3::O_STG + sb * c3::STGB;
        int n = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int j = w + 4 * i;
            if (j < c3::NPX) {
                blds16(xr, 1024 * j + 16 * lane, base + 1024 * j);
                ++n;
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int j = w + 4 * i;
            if (j < c3::NPD) {
                blds16(dr, 1024 * j + 16 * lane, base + 1024 * (c3::NPX + j));
                blds16(mr, 1024 * j + 16 * lane, base + 1024 * (c3::NPX + c3::NPD + j));
                n += 2;
            }
        }
        return n;
    };
    const int sl = rs_lane(lane);  // lane order with bank-conflict-free write groups
    auto reshuffle = [&](int sb, int slot) {  // own landed pieces -> image slot (a2, then da3: reads, then writes)
        const char* st = smem + c3::O_STG + sb * c3::STGB;
        char* im = smem + slot * c3::SLOT2;
        {
            u32x4 xv[3];
            int xd[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int u = min(64 * (w + 4 * i) + sl, c3::NUX - 1);
                xv[i] = *(const u32x4*)(st + 16 * u);
                xd[i] = dstx[u];
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (64 * (w + 4 * i) + sl < c3::NUX) *(u32x4*)(im + 16 * xd[i]) = xv[i];
        }
        s16x8 dv[2], mv[2];
        int dd[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int u = min(64 * (w + 4 * i) + sl, c3::NUD - 1);
            dv[i] = *(const s16x8*)(st + 1024 * c3::NPX + 16 * u);
            mv[i] = *(const s16x8*)(st + 1024 * (c3::NPX + c3::NPD) + 16 * u);
            dd[i] = dsty[u];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (64 * (w + 4 * i) + sl < c3::NUD) {
                s16x8 v = dv[i];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = mv[i][q] > 0 ? v[q] : (short)0;
                *(s16x8*)(im + c3::XB + 16 * dd[i]) = v;
            }
    };
    // frame k: staging k % 2, image slot k & 1. mA / mB: this wave's issue count right after the
    // DMA of the next / next-but-one frame to reshuffle.
    int issued = 0, mA = 0, mB = 0;
    if constexpr (ISSUER) {
        int m0 = 0;
        if (nmine > 0) issued += issue(0, 0);
        m0 = issued;
        if (nmine > 1) issued += issue(1, 1);
        mA = issued;
        if (nmine > 0) {
            wait_vmcnt(issued - m0);
            reshuffle(0, 0);
        }
        if (nmine > 2) issued += issue(2, 0);
        mB = issued;
    }
    for (int it = 0; it < nmine; ++it) {
        const int f = blockIdx.x + it * gridDim.x;
        char* X = smem + (it & 1) * c3::SLOT2;
        lds_barrier();  // frame it in slot it&1; every wave done with frame it-1 (slot (it+1)&1)
        if (ISSUER && it + 1 < nmine) {
            wait_vmcnt(issued - mA);  // own pieces of frame it+1 landed
            reshuffle((it + 1) & 1, (it + 1) & 1);
            int mC = issued;
            if (it + 3 < nmine) {
                issued += issue(it + 3, (it + 1) & 1);  // into the staging buffer just emptied
                mC = issued;
            }
            mA = mB;
            mB = mC;
        }
        work(X, f);
        issued += nst;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// weight gradient of one wave, taps t = 2i + B (B = wr>>1), i < 5 - B
template <int B>
__device__ __forceinline__ void c3_wgrad(const C3Ctx& ctx, char* smem, float* slab, float* cs_slab, int wr) {
    constexpr int NKT = 5 - B;
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, h = lane >> 5;
    const int mu0 = 8 * (g >> 1) + q;
    const int ca = 4 * (wr & 1) + 2 * (g & 1) + (p4 >> 1), cb = 2 * (g & 1) + (p4 >> 1);
    const int ba0 = 16 * (mu0 + 96 * ca + c3::zc(ca)) + 8 * (p4 & 1);
    const int bb0 = c3::XB + 16 * (20 + mu0 + 128 * cb + c3::zc(cb)) + 8 * (p4 & 1);
    f32x16 accw[NKT][2];
#pragma unroll
    for (int i = 0; i < NKT; ++i) { accw[i][0] = f32x16{}; accw[i][1] = f32x16{}; }
    float bsum0 = 0.f, bsum1 = 0.f;
    c3_frames<true>(ctx, smem, 0, [&](const char* X, int) {
        const char* XA = X + ba0;
        const char* XB_ = X + bb0;
        bf16x8 fb[2][NKT + 2];  // [0] b0, [1] b1 (co halves), [2 + i] A of tap 2i + B
        auto load = [&](int ms, bf16x8* d) {
            const int o = 16 * 16 * ms;
            d[0] = tr2(XB_ + o, XB_ + o + 64);
            d[1] = tr2(XB_ + o + 8192, XB_ + o + 64 + 8192);  // chunk + 4
#pragma unroll
            for (int i = 0; i < NKT; ++i) {
                const int t = 2 * i + B, ky = t / 3, kx = t - 3 * ky;
                const int oa = o + 16 * (9 * ky + kx);
                d[2 + i] = tr2(XA + oa, XA + oa + 64);
            }
        };
        load(0, fb[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * NKT + 4, 0);
#pragma unroll
        for (int ms = 0; ms < 4; ++ms) {
            const bf16x8* cur = fb[ms & 1];
            if (ms + 1 < 4) load(ms + 1, fb[(ms + 1) & 1]);
            bsum0 = sum8_bf16(cur[0], bsum0);  // bias: column sums of dY (kept by wave 0)
            bsum1 = sum8_bf16(cur[1], bsum1);
#pragma unroll
            for (int i = 0; i < NKT; ++i) {
                accw[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + i], cur[0], accw[i][0], 0, 0, 0);
                accw[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[2 + i], cur[1], accw[i][1], 0, 0, 0);
            }
            // 2NKT MFMAs, 2NKT + 4 reads of the next step: pairs of reads between MFMAs
#pragma unroll
            for (int k = 0; k < 2 * NKT; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (ms + 1 < 4) {
                    if (k < NKT + 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    else __builtin_amdgcn_sched_group_barrier(0x100, 0, 0);
                }
            }
        }
    });
    float* out = slab + (size_t)blockIdx.x * 576 * 64;
#pragma unroll
    for (int i = 0; i < NKT; ++i) {
        const int kt = wr + 4 * i;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h;
                out[k * 64 + 32 * ct + (lane & 31)] = accw[i][ct][r];
            }
    }
    if (wr == 0) {  // lanes l and l+32 hold the same co, other m half
        const float o0 = __shfl_xor(bsum0, 32, 64), o1 = __shfl_xor(bsum1, 32, 64);
        if (lane < 32) {
            cs_slab[(size_t)blockIdx.x * 64 + lane] = bsum0 + o0;
            cs_slab[(size_t)blockIdx.x * 64 + 32 + lane] = bsum1 + o1;
        }
    }
}

__global__ __launch_bounds__(512, 2) void conv3_bwd_fr(const __bf16* __restrict__ a2,
                                                       const __bf16* __restrict__ da3,  // unmasked
                                                       const __bf16* __restrict__ a3,   // its mask
                                                       const __bf16* __restrict__ w3d,  // [64 ci][576]
                                                       __bf16* __restrict__ da2,
                                                       float* __restrict__ slab,     // [grid][576][64]
                                                       float* __restrict__ cs_slab,  // [grid][64]
                                                       float* __restrict__ cs2,      // [grid][2][64] conv2 bias partials
                                                       int nframes) {
    __shared__ __attribute__((aligned(16))) char smem[c3::LDS];
    const int lane = threadIdx.x & 63;
    const int w = wave_id(), wr = w & 3;
    const int g = lane >> 4;
    const C3Ctx ctx{a2, da3, a3, da2, nframes};

    if (w < 4) {
        if (wr >> 1) c3_wgrad<1>(ctx, smem, slab, cs_slab, wr);
        else c3_wgrad<0>(ctx, smem, slab, cs_slab, wr);
    } else {
        // data gradient: channel half chh = wr&1 (tiles ct = 0, 1 of 16 channels; row i of tile
        // ct is channel 32chh + 8(i>>2) + 4ct + (i&3), so lane group g ends with channels
        // 32chh + 8g..+8 of its pixel), three pixel tiles per wave ({1, 2, 5} for ph = wr>>1 = 0,
        // {0, 3, 4} for ph = 1), lane i of tile pt on pixel 16pt + sig(i)
        const int chh = wr & 1, ph = wr >> 1;
        s16x8 bw[2][18];  // lane holds W[ci(ct, lane&15)][k = 32ks + 8g..+8]
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int ks = 0; ks < 18; ++ks) {
                const int i = lane & 15, ci = 32 * chh + 8 * (i >> 2) + 4 * ct + (i & 3);
                bw[ct][ks] = *(const s16x8*)(w3d + (size_t)ci * 576 + 32 * ks + 8 * g);
            }
        const int si = (lane & 15) ^ (((lane & 15) >> 1) & 4);
        const int cg = g;  // dY chunk of k-step ks: g + 4(ks&1)
        // conv2's bias gradient is the column sum of da2 as stored (masked, bf16): summed here,
        // where the values are in registers anyway, instead of by conv21's weight-gradient waves
        // (48 v_dot2 per frame beside their MFMAs); channels 8c + j of this lane's pixels
        float bs8[8] = {};  // FI_C2B_C3 only
        // Tap skipping: dX pixel (iy, ix) meets dY row iy - ky, which exists only for
        // 0 <= iy - ky <= 6 (the zero border supplies the rest). Pixel tiles are 16 pixels of
        // the 9-wide image, so tile 0 (rows 0-1) never needs kernel row 2, tile 4 (rows 7-8)
        // never row 0 and tile 5 (pixel 80) only row 2: their all-zero k-steps are skipped
        // (the sums are unchanged bit for bit). Tiles {1, 2, 5} and {0, 3, 4} then carry 42
        // k-step x tile units each (84 MFMAs per wave instead of 108).
        auto work = [&](auto phc, const char* X, int f) {
            constexpr int PH = decltype(phc)::value;
            constexpr auto tile = [](int ti) { return PH == 0 ? (ti == 0 ? 1 : ti == 1 ? 2 : 5) : (ti == 0 ? 0 : ti == 1 ? 3 : 4); };
            constexpr auto active = [](int ks, int pt) {
                const int lo = pt == 4 ? 6 : (pt == 5 ? 12 : 0), hi = pt == 0 ? 12 : 18;
                return ks >= lo && ks < hi;
            };
            int bd[3];
#pragma unroll
            for (int ti = 0; ti < 3; ++ti) bd[ti] = c3::XB + 16 * (min(16 * tile(ti) + si, 80) + 128 * cg + c3::zc(cg));
            f32x4 acc[3][2];
#pragma unroll
            for (int ti = 0; ti < 3; ++ti) { acc[ti][0] = f32x4{}; acc[ti][1] = f32x4{}; }
            constexpr int PD = 3;  // k-steps of fragments read ahead
            bf16x8 fb[PD + 1][3];
            auto load = [&](int ks, bf16x8* d) {  // k = 64 tap + co: tap = ks>>1, co half = ks&1 (chunk + 4)
                const int tap = ks >> 1, ky = tap / 3, kx = tap - 3 * ky;
                const int off = 16 * (20 - 9 * ky - kx) + 8192 * (ks & 1);
#pragma unroll
                for (int ti = 0; ti < 3; ++ti)
                    if (active(ks, tile(ti))) d[ti] = *(const bf16x8*)(X + bd[ti] + off);
            };
#pragma unroll
            for (int ks = 0; ks < PD; ++ks) load(ks, fb[ks]);
#pragma unroll
            for (int ks = 0; ks < 18; ++ks) {
                const bf16x8* cur = fb[ks % (PD + 1)];
                if (ks + PD < 18) load(ks + PD, fb[(ks + PD) % (PD + 1)]);
#pragma unroll
                for (int ti = 0; ti < 3; ++ti) {
                    if (active(ks, tile(ti))) {
                        acc[ti][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bw[0][ks]),
                                                                            cur[ti], acc[ti][0], 0, 0, 0);
                        acc[ti][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bw[1][ks]),
                                                                            cur[ti], acc[ti][1], 0, 0, 0);
                    }
                }
            }
            u32x4* dst = (u32x4*)(ctx.da2 + (size_t)f * 5184);
            const int c = 4 * chh + g;
#pragma unroll
            for (int ti = 0; ti < 3; ++ti) {  // 3 stores per frame (nst above)
                const int ri = tile(ti) * 16 + si;
                if (ri < 81) {
                    const s16x8 m = *(const s16x8*)(X + 16 * (ri + 96 * c + c3::zc(c)));
                    bf16x8 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        o[r] = m[r] > 0 ? (__bf16)acc[ti][0][r] : (__bf16)0.f;
                        o[4 + r] = m[4 + r] > 0 ? (__bf16)acc[ti][1][r] : (__bf16)0.f;
                    }
                    FI_ST16(__builtin_bit_cast(u32x4, o), dst + 8 * ri + c);
                    if constexpr (FI_C2B_C3) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) bs8[j] += (float)o[j];
                    }
                }
            }
        };
        c3_frames<false>(ctx, smem, 3, [&](const char* X, int f) {
            if (ph) work(std::integral_constant<int, 1>{}, X, f);
            else work(std::integral_constant<int, 0>{}, X, f);
        });
        // sum over the 16 lanes (pixels) of each channel group; wave (chh, ph) owns channels
        // 32chh..+32 of its pixel tiles -> cs2[block][ph][64]
        if constexpr (FI_C2B_C3) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) bs8[j] += __shfl_xor(bs8[j], o, 64);
            if ((lane & 15) == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) cs2[((size_t)blockIdx.x * 2 + ph) * 64 + 8 * (4 * chh + g) + j] = bs8[j];
            }
        }
    }
}

int conv3_bwd_fr_launch(const __bf16* a2, const __bf16* da3, const __bf16* a3, const __bf16* w3d, __bf16* da2,
                        float* slab, float* cs_slab, float* cs2, int nframes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(conv3_bwd_fr, dim3(grid), dim3(512), 0, s, a2, da3, a3, w3d, da2,
                       slab, cs_slab, cs2, nframes);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

}  // namespace fi
