// fc_gemm.hip -- the Atari policy's fc layer (3136 -> 512, config #3) on hand-written bf16
// MFMA kernels for gfx950 (replaced the hipBLASLt GEMMs).
//
// No reference counterpart: the reference learner has no network (learner.h:32-49); the layer
// is SURVEY.md 8(a)'s "Policy network" row. R = (T+1)*B rows (frames):
//   forward  h[R][512]    = relu(a3[R][3136] . fcW[3136][512] + b)      (K = 3136)
//   dgrad    da3[R][3136] = dh[R][512] . fcW^T                           (K = 512)
//   wgrad    dW[3136][512] = a3^T . dh  (reduction over R, split into fp32 slabs)
//
// Two kernels, both 512 threads (8 waves), 16x16x32 bf16 MFMA, fp32 accumulation. Operands
// are staged by LDS-DMA (buffer_load_dwordx4 ... lds) into a ring of NS slots of BK k each;
// step i waits (counted vmcnt) for its own slot and leaves the next NS-2 slots in flight
// across the barrier, then issues step i+NS-1 into the slot step i-1 used (one barrier per
// step). The accumulator tile is C[x][y] with x on the MFMA's A side (rows = registers) and
// y on the B side (columns = lanes), so each lane holds 4 CONSECUTIVE x of one y: the
// output's contiguous dimension is x in all three GEMMs.
//  * fc_nt_kernel -- C[x][y] = sum_k X[x][k] Y[y][k], both operands k-contiguous rows (fwd:
//    X = W^T [512][3136], Y = a3; dgrad: X = W [3136][512], Y = dh). Persistent: each
//    workgroup walks output tiles lg, lg+G, ...; the ring runs on across tile boundaries (the
//    next tile's first steps land during the last MFMAs of the current one; the epilogue's
//    stores stay in flight, counted in the waits), which matters for dgrad's short K. LDS
//    image per operand and slot: [rows][BK] with 16-B chunks XOR-swizzled per row (swizzle
//    on the DMA source, the image stays lane-linear): conflict-free ds_read_b128 fragments.
//    Epilogue: pairs of x fragments are exchanged between lane groups by v_permlane16_swap
//    so every lane stores 8 consecutive bf16 (one 16-B buffer store per pair).
//  * fc_tn_kernel -- C[x][y] = sum_r X[r][x] Y[r][y] (wgrad: X = dh, Y = a3): both operands
//    are r-major, so the LDS image is [BK r][cols] and the fragments are read with the gfx950
//    transpose read ds_read_b64_tr_b16; 32-B granules XOR-swizzled per row (conflict-free
//    for the 512-B and 448-B rows used). One output tile x one R-slice per workgroup, fp32
//    slab per slice, reduced in a fixed order by reduce_slabs (deterministic).
// Operand rows past the end (ragged R) read as zero through the buffer descriptors' range;
// output rows past the end are dropped the same way (stores always issue, so the counted
// vmcnt waits stay exact).
#include <algorithm>

#include "fi_common.h"
#include "kernels.h"

namespace fi {
namespace fcg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int FCK = 3136, FCO = 512;

// LDS-DMA of 16 B per lane from a buffer descriptor built just before (s_nop 4: SGPRs fresh
// from v_readfirstlane feed the buffer instruction's descriptor)
__device__ __forceinline__ void dma16(fi_i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_nop 4\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_base)
        : "memory");
}

// the same with the non-temporal load policy (operands read once: not kept in the caches)
__device__ __forceinline__ void dma16_nt(fi_i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_nop 4\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_base)
        : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ int pack_bf16x2(float a, float b) {
    const bf16x4 v{(__bf16)a, (__bf16)b, (__bf16)0.f, (__bf16)0.f};
    return (int)(uint32_t)__builtin_bit_cast(uint64_t, v);
}

// (a = x-fragment f, b = fragment f+1; lane group G = lane >> 4 holds x 4G..4G+3 of each)
// -> 8 consecutive bf16 per lane at fragment-relative x offset xoff_pair(G)
__device__ __forceinline__ i32x4 pair_swap(i32x2 a, i32x2 b) {
    const auto r0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    return i32x4{(int)r0[0], (int)r1[0], (int)r0[1], (int)r1[1]};
}
__device__ __forceinline__ int xoff_pair(int G) { return (G & 1) * 16 + (G >> 1) * 8; }

// ---------------------------------------------------------------- epilogues (NT kernel)
// tile(y0, rows): the output descriptor of one tile (rows >= `rows` are dropped by its
// range). pair(o, lb, xf, y, G, v0, v1): fragments f, f+1 whose x base is xf (v_k[j] =
// C[xf + 16k + 4G + j][y]); single(o, lb, xf, y, G, v): an unpaired fragment. Exactly one
// buffer store per call. lb: the kernel's LDS float area (EpiFwd's bias).
struct OutTile {
    __amdgpu_buffer_rsrc_t r;
    int y0;
};
template <int LD>
struct EpiBf16Out {
    __bf16* out;
    __device__ OutTile tile(int y0, int rows) const {
        return OutTile{out_rsrc(out + (size_t)y0 * LD, (uint32_t)rows * LD * 2), y0};
    }
    __device__ static int off(const OutTile& o, int x, int y) { return ((y - o.y0) * LD + x) * 2; }
    template <int AUX>
    __device__ static void store_pair(const OutTile& o, int xf, int y, int G, i32x4 d) {
        __builtin_amdgcn_raw_buffer_store_b128(d, o.r, off(o, xf + xoff_pair(G), y), 0, AUX);
    }
    template <int AUX>
    __device__ static void store_single(const OutTile& o, int xf, int y, int G, i32x2 d) {
        __builtin_amdgcn_raw_buffer_store_b64(d, o.r, off(o, xf + 4 * G, y), 0, AUX);
    }
};
struct EpiFwd : EpiBf16Out<FCO> {  // h[y][x] = bf16(relu(v + b[x])); bias in LDS (no VMEM in the loop)
    const float* bias;  // [512], copied into LDS at kernel start
    static constexpr int kLdsFloats = FCO;
    __device__ void init(float* lds_f, int tid, int nthr) const {
        for (int i = tid; i < FCO; i += nthr) lds_f[i] = bias[i];
    }
    __device__ static i32x2 act(const float* lb, int x, f32x4 v) {
        const f32x4 b = *(const f32x4*)(lb + x);
        return i32x2{pack_bf16x2(fmaxf(v[0] + b[0], 0.f), fmaxf(v[1] + b[1], 0.f)),
                     pack_bf16x2(fmaxf(v[2] + b[2], 0.f), fmaxf(v[3] + b[3], 0.f))};
    }
    template <int AUX>
    __device__ static void pair(const OutTile& o, const float* lb, int xf, int y, int G, f32x4 v0, f32x4 v1) {
        store_pair<AUX>(o, xf, y, G, pair_swap(act(lb, xf + 4 * G, v0), act(lb, xf + 16 + 4 * G, v1)));
    }
    template <int AUX>
    __device__ static void single(const OutTile& o, const float* lb, int xf, int y, int G, f32x4 v) {
        store_single<AUX>(o, xf, y, G, act(lb, xf + 4 * G, v));
    }
};
struct EpiDgrad : EpiBf16Out<FCK> {  // da3[y][x] = bf16(v) (unmasked: conv3's backward applies the a3 mask)
    static constexpr int kLdsFloats = 0;
    __device__ void init(float*, int, int) const {}
    __device__ static i32x2 cvt(f32x4 v) { return i32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])}; }
    template <int AUX>
    __device__ static void pair(const OutTile& o, const float*, int xf, int y, int G, f32x4 v0, f32x4 v1) {
        store_pair<AUX>(o, xf, y, G, pair_swap(cvt(v0), cvt(v1)));
    }
    template <int AUX>
    __device__ static void single(const OutTile& o, const float*, int xf, int y, int G, f32x4 v) {
        store_single<AUX>(o, xf, y, G, cvt(v));
    }
};

// s_waitcnt vmcnt(n), n wave-uniform (rounds down: waits at least as long as asked)
__device__ __forceinline__ void vm_wait_rt(int n) { wait_vmcnt(n); }

// NT image swizzle: 16-B chunk c of row `row` in a [rows][BK] bf16 image
template <int BK>
__device__ __forceinline__ int nt_chunk(int c, int row) {
    if constexpr (BK == 64) return c ^ ((row >> 1) & 7);       // 128-B rows
    else return c ^ (3 * ((row >> 3) & 1));                     // 64-B rows
}

// ---------------------------------------------------------------- NT kernel
// OPT bits: 1 = s_setprio 1 around each MFMA cluster, 2 = nontemporal (streaming) output stores,
// 4 = accumulators in AGPRs (for 4-wave tiles of 128 x 128 per wave), 8 = non-temporal loads of
// the Y operand (the frame rows), 16 = the next step's DMA issued after the first sub-step's
// fragment reads (their LDS latency overlaps the issue), 32 = ... after the first sub-step's MFMAs,
// 64 = LDS-read prefetch across the barrier (BK 32, NS >= 4; see the branch below), 128 = tile
// rows dealt to XCDs in contiguous eighths (tile_of below), 4096 = one barrier per step, between
// its two halves (BK 64, NS 2; see the branch below)
template <int BX, int BY, int WX, int WY, int BK, int NS, class Epi, int OPT = 0>
__global__ __launch_bounds__(64 * WX * WY) void fc_nt_kernel(const __bf16* __restrict__ X, const __bf16* __restrict__ Y,
                                                    int NY, int K, int ntx, int ntiles, Epi epi) {
    constexpr int TX = BX / WX, TY = BY / WY, FX = TX / 16, FY = TY / 16;
    constexpr int RPP = 1024 / (BK * 2);                      // image rows per 1-KiB DMA piece
    constexpr int NW = WX * WY;                               // waves
    constexpr int PX = BX / RPP, P = (BX + BY) / RPP, PW = (P + NW - 1) / NW;
    constexpr int SLOT = (BX + BY) * BK * 2;
    constexpr int NST = FY * (FX / 2 + FX % 2);               // epilogue stores per wave
    constexpr int D = NS - 1;                                 // steps in flight ahead
    constexpr int AUX = (OPT & 2) ? 2 : 0;
    static_assert((NW == 8 || NW == 4) && FX * 16 == TX && FY * 16 == TY && (BK == 64 || BK == 32), "tile");
    static_assert(BX % RPP == 0 && BY % RPP == 0 && (D - 1) * PW + NST < 64, "ring");
    __shared__ __attribute__((aligned(16))) char lds[NS * SLOT + Epi::kLdsFloats * 4];
    if constexpr (OPT & 4) asm volatile("" ::"a"(0));  // AGPR-form MFMAs: accumulators in AGPRs
    const int lane = threadIdx.x & 63, w = wave_id(), G = lane >> 4;
    const int wx = w / WY, wy = w % WY;
    const int NG = gridDim.x, lg = xcd_remap(blockIdx.x, NG);
    const int nk = K / BK;
    // tile i of this workgroup. Default: lg + i NG (the XCD-contiguous lg of xcd_remap). OPT 128:
    // each XCD owns a contiguous eighth of the tile ROWS (ty) and its NG / 8 workgroups walk it
    // tile by tile, so the ntx tiles of a row -- which share its Y rows -- run on one XCD at
    // about the same time (with lg, a row's tiles straddle two XCDs at every 32-tile boundary)
    const bool xrow = (OPT & 128) && NG % 8 == 0;
    const int xcd = blockIdx.x % 8, jx = blockIdx.x / 8, ngx = NG / 8;
    const int nty_ = ntiles / ntx, r0x = xcd * nty_ / 8, r1x = (xcd + 1) * nty_ / 8;
    const int nmy = xrow ? ((r1x - r0x) * ntx - jx + ngx - 1) / ngx : (ntiles - 1 - lg) / NG + 1;
    auto tile_of = [&](int i) { return xrow ? r0x * ntx + jx + i * ngx : lg + i * NG; };
    const int total = max(nmy, 0) * nk;
    const uint32_t lbase = lds_addr(lds);
    const float* lb = (const float*)(lds + NS * SLOT);
    epi.init((float*)(lds + NS * SLOT), threadIdx.x, 64 * NW);

    int is_tile = 0, is_kt = 0;  // the next step to issue (tile index of this workgroup, k-step)
    auto issue = [&](int it) {   // this wave's 1-KiB pieces of step `it` into slot it % NS
        const int t = tile_of(is_tile);
        const int ty = t / ntx, tx = t - ty * ntx;
        const int x0 = tx * BX, y0 = ty * BY;
        const fi_i32x4 rx = make_rsrc(X + (size_t)x0 * K, (uint32_t)BX * K * 2);
        const fi_i32x4 ry = make_rsrc(Y + (size_t)y0 * K, (uint32_t)min(BY, NY - y0) * K * 2);
        const uint32_t sb = lbase + (uint32_t)(it % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            int pi = w + NW * i;
            if (pi >= P) pi -= NW;  // uneven piece count: a duplicate (same bytes, same place)
            const bool isx = pi < PX;
            const int prow = (isx ? pi : pi - PX) * RPP + lane / (BK / 8);
            const int ch = nt_chunk<BK>(lane % (BK / 8), prow);
            const uint32_t voff = (uint32_t)((prow * K + is_kt * BK + ch * 8) * 2), dst = sb + (uint32_t)pi * 1024u;
            if constexpr (OPT & 8) {
                if (isx) dma16(rx, voff, dst);
                else dma16_nt(ry, voff, dst);
            } else {
                dma16(isx ? rx : ry, voff, dst);
            }
        }
        if (++is_kt == nk) is_kt = 0, ++is_tile;
    };

    for (int d = 0; d < D && d < total; ++d) issue(d);
    if constexpr (OPT & 64) {
        // LDS-read prefetch across the barrier (BK = 32, NS >= 4): at barrier(it) step it + 1
        // has landed too, so its fragments are read while step it's MFMAs (fragments already in
        // registers) run -- the matrix pipe starts right after the barrier. Step it + D goes into
        // the slot of step it - 1, whose fragments were read before barrier(it - 1).
        static_assert(BK == 32 && NS >= 4, "prefetch ring");
        auto frags = [&](int step, bf16x8* fa, bf16x8* fb) {
            const char* sx = lds + (step % NS) * SLOT;
            const char* sy = sx + BX * BK * 2;
#pragma unroll
            for (int f = 0; f < FX; ++f) {
                const int row = wx * TX + f * 16 + (lane & 15);
                fa[f] = *(const bf16x8*)(sx + row * (BK * 2) + (nt_chunk<BK>(G, row) << 4));
            }
#pragma unroll
            for (int g = 0; g < FY; ++g) {
                const int row = wy * TY + g * 16 + (lane & 15);
                fb[g] = *(const bf16x8*)(sy + row * (BK * 2) + (nt_chunk<BK>(G, row) << 4));
            }
        };
        bf16x8 ca[FX], cb[FY];
        vm_wait_rt(min(D - 1, total - 1) * PW);
        lds_barrier();
        if (total > 0) frags(0, ca, cb);
        const int mytiles = total / nk;
        int it = 0, last_epi = -(1 << 20);
        for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
            f32x4 acc[FX][FY];
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int kt = 0; kt < nk; ++kt, ++it) {
                bf16x8 na[FX], nb[FY];
                if (it + 1 < total) {
                    // younger than step it + 1's pieces: steps it + 2 .. it + D - 1, and an
                    // epilogue issued after step it + 1's DMA (iteration >= it + 1 - D)
                    vm_wait_rt(max(0, min(D - 2, total - 2 - it)) * PW + (last_epi >= it + 1 - D ? NST : 0));
                    lds_barrier();
                    if (it + D < total) issue(it + D);
                    frags(it + 1, na, nb);
                }
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int f = 0; f < FX; ++f)
#pragma unroll
                    for (int g = 0; g < FY; ++g)
                        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[f], cb[g], acc[f][g], 0, 0, 0);
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
#pragma unroll
                for (int f = 0; f < FX; ++f) ca[f] = na[f];
#pragma unroll
                for (int g = 0; g < FY; ++g) cb[g] = nb[g];
            }
            const int t = tile_of(tile_it);
            const int ty = t / ntx, tx = t - ty * ntx;
            const int y0 = ty * BY;
            const OutTile ot = epi.tile(y0, min(BY, NY - y0));
            const int xw = tx * BX + wx * TX, yb = y0 + wy * TY + (lane & 15);
#pragma unroll
            for (int g = 0; g < FY; ++g) {
#pragma unroll
                for (int f = 0; f + 1 < FX; f += 2)
                    Epi::template pair<AUX>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f][g], acc[f + 1][g]);
                if constexpr (FX % 2)
                    Epi::template single<AUX>(ot, lb, xw + (FX - 1) * 16, yb + g * 16, G, acc[FX - 1][g]);
            }
            last_epi = it - 1;
        }
        return;
    }
    if constexpr (OPT & 4096) {
        // mid-step barrier (BK = 64, NS = 2): step it's second-half fragments are read into
        // registers BEFORE its first-half MFMAs, so at the one barrier per step (between the two
        // halves) every wave is done with slot it % 2; the barrier releases into step it + 2's DMA
        // (that slot), step it + 1's first-half reads, and step it's second-half MFMAs, whose
        // operands are already in registers -- the matrix pipe does not wait out the barrier and
        // the LDS latency behind it.
        static_assert(BK == 64 && NS == 2, "mid-step barrier ring");
        auto frags = [&](int step, int s, bf16x8* fa, bf16x8* fb) {
            const char* sx = lds + (step % NS) * SLOT;
            const char* sy = sx + BX * BK * 2;
            const int ch = s * 4 + G;
#pragma unroll
            for (int f = 0; f < FX; ++f) {
                const int row = wx * TX + f * 16 + (lane & 15);
                fa[f] = *(const bf16x8*)(sx + row * (BK * 2) + (nt_chunk<BK>(ch, row) << 4));
            }
#pragma unroll
            for (int g = 0; g < FY; ++g) {
                const int row = wy * TY + g * 16 + (lane & 15);
                fb[g] = *(const bf16x8*)(sy + row * (BK * 2) + (nt_chunk<BK>(ch, row) << 4));
            }
        };
        bf16x8 ca[FX], cb[FY];  // first-half fragments of the current step
        if (total > 0) {
            vm_wait_rt(0);
            lds_barrier();
            if (1 < total) issue(1);  // slot 1: untouched so far
            frags(0, 0, ca, cb);
        }
        const int mytiles = total / nk;
        int it = 0, last_epi = -(1 << 20);
        for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
            f32x4 acc[FX][FY];
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int kt = 0; kt < nk; ++kt, ++it) {
                bf16x8 ha[FX], hb[FY];  // second half of step it
                frags(it, 1, ha, hb);
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int f = 0; f < FX; ++f)
#pragma unroll
                    for (int g = 0; g < FY; ++g)
                        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[f], cb[g], acc[f][g], 0, 0, 0);
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
                if (it + 1 < total) {
                    // younger than step it + 1's pieces (issued right after barrier(it - 1)): the
                    // epilogue stores of a tile that ended at step it - 1
                    vm_wait_rt(last_epi == it - 1 ? NST : 0);
                    lds_barrier();
                    if (it + 2 < total) issue(it + 2);
                    frags(it + 1, 0, ca, cb);
                }
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int f = 0; f < FX; ++f)
#pragma unroll
                    for (int g = 0; g < FY; ++g)
                        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[f], hb[g], acc[f][g], 0, 0, 0);
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
            }
            const int t = tile_of(tile_it);
            const int ty = t / ntx, tx = t - ty * ntx;
            const int y0 = ty * BY;
            const OutTile ot = epi.tile(y0, min(BY, NY - y0));
            const int xw = tx * BX + wx * TX, yb = y0 + wy * TY + (lane & 15);
#pragma unroll
            for (int g = 0; g < FY; ++g) {
#pragma unroll
                for (int f = 0; f + 1 < FX; f += 2)
                    Epi::template pair<AUX>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f][g], acc[f + 1][g]);
                if constexpr (FX % 2)
                    Epi::template single<AUX>(ot, lb, xw + (FX - 1) * 16, yb + g * 16, G, acc[FX - 1][g]);
            }
            last_epi = it - 1;
        }
        return;
    }
    // tile-outer / k-inner: the accumulators are zeroed per tile outside the k loop (a reset
    // inside it would merge two definitions at the loop head: with AGPR accumulators the
    // compiler then copies every accumulator through VGPRs each step)
    const int mytiles = total / nk;
    int it = 0, last_epi = -(1 << 20);
    for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
        f32x4 acc[FX][FY];
#pragma unroll
        for (int f = 0; f < FX; ++f)
#pragma unroll
            for (int g = 0; g < FY; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt, ++it) {
            // younger than this step's loads: the steps issued after it (at most D-1), and the
            // last epilogue's stores if they were issued after this step's loads
            const int ahead = min(D - 1, total - 1 - it);
            vm_wait_rt(ahead * PW + (it - last_epi <= D ? NST : 0));
            lds_barrier();
            if constexpr (!(OPT & 48)) {
                if (it + D < total) issue(it + D);
            }
            const char* sx = lds + (it % NS) * SLOT;
            const char* sy = sx + BX * BK * 2;
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                const int ch = s * 4 + G;
                bf16x8 fa[FX], fb[FY];
#pragma unroll
                for (int f = 0; f < FX; ++f) {
                    const int row = wx * TX + f * 16 + (lane & 15);
                    fa[f] = *(const bf16x8*)(sx + row * (BK * 2) + (nt_chunk<BK>(ch, row) << 4));
                }
#pragma unroll
                for (int g = 0; g < FY; ++g) {
                    const int row = wy * TY + g * 16 + (lane & 15);
                    fb[g] = *(const bf16x8*)(sy + row * (BK * 2) + (nt_chunk<BK>(ch, row) << 4));
                }
                if constexpr ((OPT & 16) != 0) {
                    if (s == 0 && it + D < total) issue(it + D);
                }
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int f = 0; f < FX; ++f)
#pragma unroll
                    for (int g = 0; g < FY; ++g)
                        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[f], fb[g], acc[f][g], 0, 0, 0);
                if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
                if constexpr ((OPT & 32) != 0) {
                    if (s == 0 && it + D < total) issue(it + D);
                }
            }
        }
        const int t = tile_of(tile_it);
        const int ty = t / ntx, tx = t - ty * ntx;
        const int y0 = ty * BY;
        const OutTile ot = epi.tile(y0, min(BY, NY - y0));
        const int xw = tx * BX + wx * TX, yb = y0 + wy * TY + (lane & 15);
#pragma unroll
        for (int g = 0; g < FY; ++g) {
#pragma unroll
            for (int f = 0; f + 1 < FX; f += 2)
                Epi::template pair<AUX>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f][g], acc[f + 1][g]);
            if constexpr (FX % 2)
                Epi::template single<AUX>(ot, lb, xw + (FX - 1) * 16, yb + g * 16, G, acc[FX - 1][g]);
        }
        last_epi = it - 1;
    }
}

// ---------------------------------------------------------------- TN kernel
// 32-B granule swizzle of an r-major image row (pitch in bytes): distinct 8-bank windows for
// the 8 rows {q, 8 + q : q < 4} one 32-lane half of a ds_read_b64_tr_b16 touches
template <int PITCH>
__device__ __forceinline__ int tr_swz(int row) {
    static_assert(PITCH % 256 == 0 || PITCH == 448, "tr image pitch");
    if constexpr (PITCH % 256 == 0) return (row & 3) | (((row >> 3) & 1) << 2);
    else return (row >> 3) & 1;  // 448 B = 14 granules: rows q land on windows {0,6,4,2}
}

template <int PITCH>
__device__ __forceinline__ bf16x8 tr_frag16(const char* img, int s, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int ra = 32 * s + 8 * g + q, rb = ra + 4;
    const char* a = img + ra * PITCH + (((c0 >> 4) ^ tr_swz<PITCH>(ra)) << 5) + p * 8;
    const char* b = img + rb * PITCH + (((c0 >> 4) ^ tr_swz<PITCH>(rb)) << 5) + p * 8;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(b));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// slab[s][y][x] (row length NXT = all x) = sum over r in split s of X[r][x] Y[r][y]
template <int BX, int BY, int WX, int WY, int BK, int NS>
__global__ __launch_bounds__(512) void fc_tn_kernel(const __bf16* __restrict__ X, int NXT, const __bf16* __restrict__ Y,
                                                    int NYT, int R, int rps, float* __restrict__ slab) {
    constexpr int TX = BX / WX, TY = BY / WY, FX = TX / 16, FY = TY / 16;
    constexpr int PITX = BX * 2, PITY = BY * 2;       // image row bytes
    constexpr int UX = BX / 8, UY = BY / 8;           // 16-B units per image row
    constexpr int PX = BX * BK / 512, P = (BX + BY) * BK / 512, PW = (P + 7) / 8;
    constexpr int SLOT = (BX + BY) * BK * 2;
    constexpr int D = NS - 1;
    static_assert(WX * WY == 8 && FX * 16 == TX && FY * 16 == TY && (BK == 64 || BK == 32), "tile");
    static_assert(BX * BK % 512 == 0 && BY * BK % 512 == 0 && (D - 1) * PW < 64, "ring");
    __shared__ __attribute__((aligned(16))) char lds[NS * SLOT];
    const int lane = threadIdx.x & 63, w = wave_id();
    const int wx = w / WY, wy = w % WY;
    const int ntx = NXT / BX, nty = NYT / BY;
    // workgroup -> (R-slice, tile). Block b runs on XCD b % 8 (round-robin dispatch): whole
    // slices first, S / 8 of them per XCD, so the NT tiles of a slice share one XCD's L2 and the
    // slice's rows leave HBM once (with the slices laid contiguously over the XCDs, 9 slices on 8
    // XCDs straddled them: 1.47x the algorithmic traffic); the tiles of the S % 8 leftover slices
    // follow (XCD-contiguous when there is no whole slice per XCD, i.e. small R)
    const int NT = ntx * nty, per = (int)(gridDim.x / NT) / 8;
    const int b = blockIdx.x, j = b / 8;
    int sp, rem, tx, ty;
    if (j < per * NT) {
        sp = (b % 8) * per + j / NT;
        rem = j - (j / NT) * NT;
        tx = rem / nty, ty = rem - tx * nty;
    } else if (per > 0 && (int)gridDim.x == (8 * per + 1) * NT && ntx == 2 && nty == 14) {
        // one leftover slice of 2 x 14 tiles (the fc weight gradient at 9 slices): block b runs on
        // XCD x = b % 8 as its slot r = (b - 8 per NT) / 8. XCDs 0-3 take 2 x 2 tile blocks (ty 2x,
        // 2x+1, both tx), XCDs 4-7 1 x 3 blocks (one tx, three of ty 8..13), so each XCD reads few
        // of the slice's column blocks: 14.6 instead of 20 slice-units of HBM reads (dh column
        // half = 0.5, a3 column block = 0.43; once = 7)
        const int id = b - 8 * per * NT, x = id % 8, r = id / 8;
        sp = 8 * per;
        if (x < 4) tx = r & 1, ty = 2 * x + (r >> 1);
        else tx = (x - 4) >> 1, ty = 8 + 3 * ((x - 4) & 1) + r;
    } else {
        const int id = per > 0 ? b - 8 * per * NT : xcd_remap(b, gridDim.x);
        sp = 8 * per + id / NT;
        rem = id - (id / NT) * NT;
        tx = rem / nty, ty = rem - tx * nty;
    }
    const int x0 = tx * BX, y0 = ty * BY;
    const int rbeg = sp * rps, rend = min(R, rbeg + rps);
    const int nk = rend > rbeg ? (rend - rbeg + BK - 1) / BK : 0;
    const uint32_t lbase = lds_addr(lds);

    auto issue = [&](int kt) {
        const int r0 = rbeg + kt * BK, rows = min(BK, rend - r0);
        const fi_i32x4 rx = make_rsrc(X + (size_t)r0 * NXT + x0, (uint32_t)rows * NXT * 2);
        const fi_i32x4 ry = make_rsrc(Y + (size_t)r0 * NYT + y0, (uint32_t)rows * NYT * 2);
        const uint32_t sb = lbase + (uint32_t)(kt % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            int pi = w + 8 * i;
            if (pi >= P) pi -= 8;
            const bool isx = pi < PX;
            const int u = (isx ? pi : pi - PX) * 64 + lane;
            uint32_t voff;
            if (isx) {
                const int row = u / UX, uu = u - row * UX;
                voff = (uint32_t)(row * NXT * 2 + ((uu ^ (tr_swz<PITX>(row) << 1)) << 4));
            } else {
                const int row = u / UY, uu = u - row * UY;
                voff = (uint32_t)(row * NYT * 2 + ((uu ^ (tr_swz<PITY>(row) << 1)) << 4));
            }
            dma16(isx ? rx : ry, voff, sb + (uint32_t)pi * 1024u);
        }
    };

    f32x4 acc[FX][FY];
#pragma unroll
    for (int f = 0; f < FX; ++f)
#pragma unroll
        for (int g = 0; g < FY; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int d = 0; d < D && d < nk; ++d) issue(d);
    for (int kt = 0; kt < nk; ++kt) {
        vm_wait_rt(min(D - 1, nk - 1 - kt) * PW);
        lds_barrier();
        if (kt + D < nk) issue(kt + D);
        const char* sx = lds + (kt % NS) * SLOT;
        const char* sy = sx + BX * BK * 2;
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            bf16x8 fa[FX], fb[FY];
#pragma unroll
            for (int f = 0; f < FX; ++f) fa[f] = tr_frag16<PITX>(sx, s, wx * TX + f * 16, lane);
#pragma unroll
            for (int g = 0; g < FY; ++g) fb[g] = tr_frag16<PITY>(sy, s, wy * TY + g * 16, lane);
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[f], fb[g], acc[f][g], 0, 0, 0);
        }
    }
    float* out = slab + (size_t)sp * NXT * NYT;
    const int xb = x0 + wx * TX + 4 * (lane >> 4), yb = y0 + wy * TY + (lane & 15);
#pragma unroll
    for (int f = 0; f < FX; ++f)
#pragma unroll
        for (int g = 0; g < FY; ++g)
            __builtin_nontemporal_store(acc[f][g], (f32x4*)(out + (size_t)(yb + g * 16) * NXT + xb + f * 16));
}

}  // namespace fcg

#ifndef FI_FC_CONFIG_OVERRIDE
// (BX, BY, WX, WY, BK, NS[, OPT]) chosen with scripts/fc_bench.hip (interleaved A/B at R = 413,696)
// forward: 256 output columns x 256 rows, waves 4 (x) x 2 (y), 2 slots of k 64, one barrier per
// step between its two halves, non-temporal frame loads (round 4: 1.257 -> 1.17-1.20 ms)
#define FC_FW_CFG 256, 256, 4, 2, 64, 2, 8 | 4096
// dgrad: 3136 = 14 x 224 output columns, 256 rows, waves 1 x 8 (14 x 2 fragments per wave),
// s_setprio, non-temporal da3 stores (round 4: 1.652 -> 1.591 ms), tile rows dealt to XCDs in
// contiguous eighths so a row's 14 tiles share one XCD's L2 (round 5: 1.60-1.65 -> 1.56-1.60 ms
// alone, 1.69 -> 1.64 ms in the step; 4.47 -> 3.96 GB of HBM traffic per launch; with default
// stores 1.535-1.57 ms but 6.4 GB: the partial-line da3 writes are fetched first)
#define FC_DG_CFG 224, 256, 1, 8, 64, 2, 1 | 2 | 128
// wgrad: x = dh columns (2 x 256), y = a3 columns (14 x 224), waves 4 x 2
#define FC_WG_CFG 256, 224, 4, 2, 64, 2
#endif

using namespace fcg;

template <int BX, int BY, int WX, int WY, int BK, int NS, int OPT = 0>
static int fc_fwd_impl(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_fwd: rows must be positive");
    const int ntx = FCO / BX, nty = (rows + BY - 1) / BY, nt = ntx * nty;
    hipLaunchKernelGGL((fc_nt_kernel<BX, BY, WX, WY, BK, NS, EpiFwd, OPT>), dim3(std::min(nt, 256)), dim3(64 * WX * WY), 0, s, wT, a3,
                           rows, FCK, ntx, nt, EpiFwd{{h}, bias});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

template <int BX, int BY, int WX, int WY, int BK, int NS, int OPT = 0>
static int fc_dgrad_impl(const __bf16* dh, const __bf16* w, __bf16* da3, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_dgrad: rows must be positive");
    const int ntx = FCK / BX, nty = (rows + BY - 1) / BY, nt = ntx * nty;
    hipLaunchKernelGGL((fc_nt_kernel<BX, BY, WX, WY, BK, NS, EpiDgrad, OPT>), dim3(std::min(nt, 256)), dim3(64 * WX * WY), 0, s, w,
                           dh, rows, FCO, ntx, nt, EpiDgrad{{da3}});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

int fc_wgrad_splits(int rows) {
    // 28 output tiles; 9 R-slices -> 252 workgroups (one per CU); fewer for small R
    return std::max(1, std::min(9, (rows + 255) / 256));
}

template <int BX, int BY, int WX, int WY, int BK, int NS>
static int fc_wgrad_impl(const __bf16* a3, const __bf16* dh, float* slab, float* dw, int rows, hipStream_t s,
                         int S) {
    FI_REQUIRE(rows > 0, "fc_wgrad: rows must be positive");
    const int rps = ((rows + S - 1) / S + BK - 1) / BK * BK;
    const int nblk = S * (FCO / BX) * (FCK / BY);
    hipLaunchKernelGGL((fc_tn_kernel<BX, BY, WX, WY, BK, NS>), dim3(nblk), dim3(512), 0, s, dh, FCO, a3, FCK, rows, rps,
                       slab);
    FI_HIP_CHECK(hipGetLastError());
    return reduce_slabs(slab, S, (size_t)FCK * FCO, dw, s);
}

int fc_fwd_launch(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    return fc_fwd_impl<FC_FW_CFG>(a3, wT, bias, h, rows, s);
}
int fc_dgrad_launch(const __bf16* dh, const __bf16* w, __bf16* da3, int rows, hipStream_t s) {
    return fc_dgrad_impl<FC_DG_CFG>(dh, w, da3, rows, s);
}
int fc_wgrad_launch(const __bf16* a3, const __bf16* dh, float* slab, float* dw, int rows, hipStream_t s) {
    return fc_wgrad_impl<FC_WG_CFG>(a3, dh, slab, dw, rows, s, fc_wgrad_splits(rows));
}

}  // namespace fi
