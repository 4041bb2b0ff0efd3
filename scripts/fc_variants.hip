#include <tuple>
// fc_variants.hip -- bench-only fc GEMM variants measured against the shipped kernels in
// scripts/fc_bench.hip (included after freeimpala_amd/csrc/fc_gemm.hip; not part of the library).
// Round 4: the loader-wave NT kernel below measured 1.16 ms forward / 1.62-1.66 ms dgrad against
// 1.17-1.21 / 1.60 for the shipped 8-wave kernels and 0.99 / 1.35 for hipBLASLt
// (profiles/r04_fc_bench_variants.txt), so it stays here.
namespace fi {
namespace fcg {

// ---------------------------------------------------------------- NT kernel, loader waves
// The same GEMM as fc_nt_kernel with the roles split between the waves: NC = WX*WY compute
// waves (one per SIMD for NC = 4) only read fragments and issue MFMAs; NL loader waves (one
// per SIMD beside them) only issue the LDS-DMA and wait for it. An LDS-DMA piece blocks its
// issuing wave for ~60-180 cycles (MI355X_MICROARCH.md constants table); here that blocks a
// loader wave, never the matrix stream. The ring has NS = 3 slots of BK = 64 k; one barrier per
// step, placed between the step's two k-halves: the compute waves read step it's second half
// into registers before its first-half MFMAs, so at barrier(it) slot it % 3 is fully consumed
// and step it + 1 has landed (the loaders waited for it before arriving); after the barrier the
// loaders issue step it + 3 into the freed slot and the compute waves read step it + 1's first
// half while step it's second-half MFMAs (register operands) run. Loads run two steps ahead.
// OPT: 1 = loaders at s_setprio 2, 2 = nontemporal output stores, 8 = nt Y-operand loads.
template <int BX, int BY, int WX, int WY, int NL, int BK, int NS, class Epi, int OPT = 0>
__global__ __launch_bounds__(64 * (WX * WY + NL)) __attribute__((amdgpu_waves_per_eu(2))) void fc_ws_kernel(
    const __bf16* __restrict__ X, const __bf16* __restrict__ Y, int NY, int K, int ntx, int ntiles, Epi epi) {
    constexpr int TX = BX / WX, TY = BY / WY, FX = TX / 16, FY = TY / 16;
    constexpr int NC = WX * WY;
    constexpr int RPP = 1024 / (BK * 2);
    constexpr int PX = BX / RPP, P = (BX + BY) / RPP, PW = (P + NL - 1) / NL;  // pieces per loader
    constexpr int SLOT = (BX + BY) * BK * 2;
    constexpr int AUX = (OPT & 2) ? 2 : 0;
    static_assert(BK == 64 && NS == 3 && FX * 16 == TX && FY * 16 == TY, "ws tile");
    static_assert(BX % RPP == 0 && BY % RPP == 0 && 2 * PW < 64, "ws ring");
    __shared__ __attribute__((aligned(16))) char lds[NS * SLOT + Epi::kLdsFloats * 4];
    const int lane = threadIdx.x & 63, w = wave_id(), G = lane >> 4;
    const int NG = gridDim.x, lg = xcd_remap(blockIdx.x, NG);
    const int nk = K / BK;
    const int total = ((ntiles - 1 - lg) / NG + 1) * nk;
    const float* lb = (const float*)(lds + NS * SLOT);
    epi.init((float*)(lds + NS * SLOT), threadIdx.x, 64 * (NC + NL));

    if (w >= NC) {
        // ---- loader waves
        const int lw = w - NC;
        const uint32_t lbase = lds_addr(lds);
        int is_tile = 0, is_kt = 0;
        auto issue = [&](int it) {
            const int t = lg + is_tile * NG;
            const int ty = t / ntx, tx = t - ty * ntx;
            const int x0 = tx * BX, y0 = ty * BY;
            const fi_i32x4 rx = make_rsrc(X + (size_t)x0 * K, (uint32_t)BX * K * 2);
            const fi_i32x4 ry = make_rsrc(Y + (size_t)y0 * K, (uint32_t)min(BY, NY - y0) * K * 2);
            const uint32_t sb = lbase + (uint32_t)(it % NS) * SLOT;
#pragma unroll
            for (int i = 0; i < PW; ++i) {
                int pi = lw + NL * i;
                if (pi >= P) pi -= NL;  // uneven piece count: a duplicate (same bytes, same place)
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
        if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(2);
        for (int d = 0; d < NS && d < total; ++d) issue(d);
        if (total > 0) {
            vm_wait_rt(min(NS - 1, total - 1) * PW);  // step 0 landed
            lds_barrier();
        }
        for (int it = 0; it + 1 < total; ++it) {
            // step it + 1 landed: younger are step it + 2's pieces (issued after barrier(it - 1))
            vm_wait_rt(it + 2 < total ? PW : 0);
            lds_barrier();  // barrier(it): slot it % 3 consumed by every compute wave
            if (it + NS < total) issue(it + NS);
        }
        return;
    }

    // ---- compute waves
    const int wx = w / WY, wy = w % WY;
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
    bf16x8 ca[FX], cb[FY];
    if (total > 0) {
        lds_barrier();  // step 0 landed (and the epilogue's LDS constants written)
        frags(0, 0, ca, cb);
    }
    const int mytiles = total / nk;
    int it = 0;
    for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
        f32x4 acc[FX][FY];
#pragma unroll
        for (int f = 0; f < FX; ++f)
#pragma unroll
            for (int g = 0; g < FY; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt, ++it) {
            bf16x8 ha[FX], hb[FY];
            frags(it, 1, ha, hb);
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[f], cb[g], acc[f][g], 0, 0, 0);
            if (it + 1 < total) {
                lds_barrier();  // barrier(it)
                frags(it + 1, 0, ca, cb);
            }
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[f], hb[g], acc[f][g], 0, 0, 0);
        }
        const int t = lg + tile_it * NG;
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
    }
}


// ---------------------------------------------------------------- forward, one DMA block per step
// fc_nt_kernel<256, 256, 4, 2, 64, 2, Epi, 8 | 4096> (the shipped forward) with the step's 8 LDS-DMA
// pieces per wave issued from ONE asm block the way hipBLASLt's loop issues them: per-lane offsets
// computed once (constant across steps), the k advance in the instruction's soffset SGPR, M0
// advanced by one s_add per piece, one s_nop for the descriptor hazard per step instead of per piece.
#define FI_FC2_LOADS(NTY)                                                                         \
    "s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[mx]\n\ts_nop 0\n\t"                      \
    "buffer_load_dwordx4 %[v0], %[rx], %[ko] offen lds\n\ts_add_u32 m0, m0, 8192\n\t"            \
    "buffer_load_dwordx4 %[v1], %[rx], %[ko] offen lds\n\ts_add_u32 m0, m0, 8192\n\t"            \
    "buffer_load_dwordx4 %[v2], %[rx], %[ko] offen lds\n\ts_add_u32 m0, m0, 8192\n\t"            \
    "buffer_load_dwordx4 %[v3], %[rx], %[ko] offen lds\n\ts_mov_b32 m0, %[my]\n\ts_nop 0\n\t"    \
    "buffer_load_dwordx4 %[v4], %[ry], %[ko] offen " NTY " lds\n\ts_add_u32 m0, m0, 8192\n\t"    \
    "buffer_load_dwordx4 %[v5], %[ry], %[ko] offen " NTY " lds\n\ts_add_u32 m0, m0, 8192\n\t"    \
    "buffer_load_dwordx4 %[v6], %[ry], %[ko] offen " NTY " lds\n\ts_add_u32 m0, m0, 8192\n\t"    \
    "buffer_load_dwordx4 %[v7], %[ry], %[ko] offen " NTY " lds\n\ts_mov_b32 m0, %[keep]"

template <class Epi>
__global__ __launch_bounds__(512) void fc_nt2_kernel(const __bf16* __restrict__ X, const __bf16* __restrict__ Y,
                                                     int NY, int K, int ntx, int ntiles, Epi epi) {
    constexpr int BX = 256, BY = 256, WX = 4, WY = 2, BK = 64, NS = 2;
    constexpr int TX = BX / WX, TY = BY / WY, FX = TX / 16, FY = TY / 16;
    constexpr int RPP = 1024 / (BK * 2), NW = WX * WY, PX = BX / RPP, PW = (BX + BY) / RPP / NW;
    constexpr int SLOT = (BX + BY) * BK * 2;
    constexpr int NST = FY * (FX / 2 + FX % 2);
    static_assert(PW == 8 && PX == 4 * NW, "4 X pieces then 4 Y pieces per wave");
    __shared__ __attribute__((aligned(16))) char lds[NS * SLOT + Epi::kLdsFloats * 4];
    const int lane = threadIdx.x & 63, w = wave_id(), G = lane >> 4;
    const int wx = w / WY, wy = w % WY;
    const int NG = gridDim.x, lg = xcd_remap(blockIdx.x, NG);
    const int nk = K / BK;
    const int total = ((ntiles - 1 - lg) / NG + 1) * nk;
    const uint32_t lbase = lds_addr(lds);
    const float* lb = (const float*)(lds + NS * SLOT);
    epi.init((float*)(lds + NS * SLOT), threadIdx.x, 64 * NW);
    uint32_t vo[PW];  // piece i: X rows (w + 8i) * 8 + lane / 8 for i < 4, Y rows (w + 8(i - 4)) * 8 + ...
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int prow = (w + NW * (i & 3)) * RPP + lane / (BK / 8);
        vo[i] = (uint32_t)((prow * K + nt_chunk<BK>(lane % (BK / 8), prow) * 8) * 2);
    }
    int is_tile = 0, is_kt = 0;
    auto issue = [&](int it) {
        const int t = lg + is_tile * NG;
        const int ty = t / ntx, tx = t - ty * ntx;
        const fi_i32x4 rx = make_rsrc(X + (size_t)tx * BX * K, (uint32_t)BX * K * 2);
        const fi_i32x4 ry = make_rsrc(Y + (size_t)ty * BY * K, (uint32_t)min(BY, NY - ty * BY) * K * 2);
        const uint32_t mx = lbase + (uint32_t)(it % NS) * SLOT + (uint32_t)w * 1024u;
        const uint32_t my = mx + (uint32_t)PX * 1024u, ko = (uint32_t)(is_kt * BK * 2);
        uint32_t keep;
        asm volatile(FI_FC2_LOADS("nt")
                     : [keep] "=&s"(keep)
                     : [v0] "v"(vo[0]), [v1] "v"(vo[1]), [v2] "v"(vo[2]), [v3] "v"(vo[3]), [v4] "v"(vo[4]),
                       [v5] "v"(vo[5]), [v6] "v"(vo[6]), [v7] "v"(vo[7]), [rx] "s"(rx), [ry] "s"(ry), [ko] "s"(ko),
                       [mx] "s"(mx), [my] "s"(my)
                     : "memory");
        if (++is_kt == nk) is_kt = 0, ++is_tile;
    };
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
    if (total > 0) issue(0);
    bf16x8 ca[FX], cb[FY];
    if (total > 0) {
        vm_wait_rt(0);
        lds_barrier();
        if (1 < total) issue(1);
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
            bf16x8 ha[FX], hb[FY];
            frags(it, 1, ha, hb);
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[f], cb[g], acc[f][g], 0, 0, 0);
            if (it + 1 < total) {
                vm_wait_rt(last_epi == it - 1 ? NST : 0);
                lds_barrier();
                if (it + 2 < total) issue(it + 2);
                frags(it + 1, 0, ca, cb);
            }
#pragma unroll
            for (int f = 0; f < FX; ++f)
#pragma unroll
                for (int g = 0; g < FY; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[f], hb[g], acc[f][g], 0, 0, 0);
        }
        const int t = lg + tile_it * NG;
        const int ty = t / ntx, tx = t - ty * ntx;
        const int y0 = ty * BY;
        const OutTile ot = epi.tile(y0, min(BY, NY - y0));
        const int xw = tx * BX + wx * TX, yb = y0 + wy * TY + (lane & 15);
#pragma unroll
        for (int g = 0; g < FY; ++g) {
#pragma unroll
            for (int f = 0; f + 1 < FX; f += 2)
                Epi::template pair<0>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f][g], acc[f + 1][g]);
        }
        last_epi = it - 1;
    }
}
#undef FI_FC2_LOADS


// ---------------------------------------------------------------- forward, hand-placed half-steps
// 4 waves, 128 x 128 per wave (256 AGPR accumulators), 2 slots of k 64 (the same LDS images,
// swizzle and k order as fc_nt_kernel, so the output is bit-identical). Each k 64 step = two
// generated asm blocks (scripts/fc_asm_blocks.inc): block A = the first half's 64 MFMAs with the
// second half's 16 fragment reads between them; the one barrier; block B = the second half's 64
// MFMAs with the next step's first-half reads AND the step-after-next's 16 LDS-DMA pieces between
// them -- one read and one DMA piece per 4 MFMAs, the placement hipBLASLt's loop uses.
#include "fc_asm_blocks.inc"

template <class Epi, int ABL = 0>  // ABL: 1 = no vmcnt wait (timing only, wrong results); 2 = one W half per XCD (tile map)
__global__ __launch_bounds__(256) void fc_asm_kernel(const __bf16* __restrict__ X, const __bf16* __restrict__ Y, int NY,
                                                     int K, int ntx, int ntiles, Epi epi) {
    constexpr int BX = 256, BY = 256, BK = 64, NS = 2, SLOT = 65536, NST = 32;
    __shared__ __attribute__((aligned(16))) char lds[NS * SLOT + Epi::kLdsFloats * 4];
    const int lane = threadIdx.x & 63, w = wave_id(), G = lane >> 4;
    const int wx = w >> 1, wy = w & 1;
    const int NG = gridDim.x, lg = xcd_remap(blockIdx.x, NG);
    const int nk = K / BK;
    // tile of round i: default t = lg + i*NG (both W halves on every XCD); ABL 2 (grid 256, ntx 2):
    // XCD x = b % 8 keeps W half x & 1 and walks frame tiles i*128 + (x >> 1)*32 + b / 8
    const int b8 = blockIdx.x % 8, j8 = blockIdx.x / 8, nty = ntiles / ntx;
    auto tile = [&](int i, int& tx, int& ty) {
        if constexpr (ABL == 2) {
            tx = b8 & 1;
            ty = i * 128 + (b8 >> 1) * 32 + j8;
        } else {
            const int t = lg + i * NG;
            ty = t / ntx;
            tx = t - ty * ntx;
        }
    };
    const int first = (b8 >> 1) * 32 + j8;
    const int total = (ABL == 2 ? (first < nty ? (nty - first + 127) / 128 : 0) : (ntiles - 1 - lg) / NG + 1) * nk;
    const uint32_t lbase = lds_addr(lds);
    const float* lb = (const float*)(lds + NS * SLOT);
    epi.init((float*)(lds + NS * SLOT), threadIdx.x, 256);
    // per-lane DMA source offsets within a k-step (constant): piece j < 8 = X rows (w + 4j) * 8
    // + lane / 8, j >= 8 = Y rows (w + 4(j - 8)) * 8 + lane / 8; chunk swizzled as the images
    uint32_t vo[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int prow = (w + 4 * (j & 7)) * 8 + lane / 8;
        vo[j] = (uint32_t)((prow * K + nt_chunk<BK>(lane % 8, prow) * 8) * 2);
    }
    // fragment read bases (bytes in LDS) per slot s and k-half h: X rows wx*128 + (lane & 15)
    // (+16 f), Y rows wy*128 + (lane & 15) (+16 g); the row swizzle is the same for every f / g
    const int r15 = lane & 15, sw = (r15 >> 1) & 7;
    auto bxa = [&](int sl, int h) {
        return lbase + (uint32_t)(sl * SLOT + (wx * 128 + r15) * 128 + (((h * 4 + G) ^ sw) << 4));
    };
    auto bya = [&](int sl, int h) {
        return lbase + (uint32_t)(sl * SLOT + 32768 + (wy * 128 + r15) * 128 + (((h * 4 + G) ^ sw) << 4));
    };
    auto dma = [&](int j) {  // step j's 16 pieces into slot j % 2 (past the last step: 0-byte descriptors)
        const bool live = j < total;
        const int kt = j % nk;
        int tx, ty;
        tile(live ? j / nk : 0, tx, ty);
        const fi_i32x4 rx = make_rsrc(X + (size_t)tx * BX * K, live ? (uint32_t)BX * K * 2 : 0u);
        const fi_i32x4 ry = make_rsrc(Y + (size_t)ty * BY * K, live ? (uint32_t)min(BY, NY - ty * BY) * K * 2 : 0u);
        const uint32_t mx = lbase + (uint32_t)((j % NS) * SLOT + w * 1024);
        return std::make_tuple(rx, ry, (uint32_t)(kt * BK * 2), mx, mx + 32768u);
    };
    if (total <= 0) return;
    {
        auto [rx, ry, ko, mx, my] = dma(0);
        fc_asm_dma(vo, rx, ry, ko, mx, my);
    }
    if (total > 1) {
        auto [rx, ry, ko, mx, my] = dma(1);
        fc_asm_dma(vo, rx, ry, ko, mx, my);
        vm_wait_rt(16);
    } else {
        vm_wait_rt(0);
    }
    lds_barrier();
    bf16x8 P[16], Q[16];
    {
        const uint32_t bx = bxa(0, 0), by = bya(0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) P[j] = *(const bf16x8*)((const char*)lds + (bx - lbase) + j * 2048);
#pragma unroll
        for (int j = 0; j < 8; ++j) P[8 + j] = *(const bf16x8*)((const char*)lds + (by - lbase) + j * 2048);
    }
    const int mytiles = total / nk;
    int it = 0, last_epi = -(1 << 20);
    for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
        f32x4 acc[64];
#pragma unroll
        for (int i = 0; i < 64; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt, ++it) {
            // every step runs the same two blocks (a branch between block variants makes hipcc
            // copy the accumulators through VGPRs at the merge): past the end, the reads fetch
            // unused fragments and the DMA pieces carry 0-byte descriptors into a dead slot
            const int sl = it % NS, sn = (it + 1) % NS;
            fc_asm_mfma_reads(acc, P, Q, bxa(sl, 1), bya(sl, 1));
            if constexpr (ABL != 1) vm_wait_rt(last_epi == it - 1 ? NST : 0);
            lds_barrier();
            auto [rx, ry, ko, mx, my] = dma(it + 2);
            fc_asm_mfma_reads_dma(acc, Q, P, bxa(sn, 0), bya(sn, 0), vo, rx, ry, ko, mx, my);
        }
        int tx, ty;
        tile(tile_it, tx, ty);
        const int y0 = ty * BY;
        const OutTile ot = epi.tile(y0, min(BY, NY - y0));
        const int xw = tx * BX + wx * 128, yb = y0 + wy * 128 + (lane & 15);
#pragma unroll
        for (int g = 0; g < 8; ++g)
#pragma unroll
            for (int f = 0; f < 8; f += 2)
                Epi::template pair<0>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f * 8 + g], acc[(f + 1) * 8 + g]);
        last_epi = it - 1;
    }
}

// ---------------------------------------------------------------- forward, k-half-split ring
// fc_asm_kernel with each 64-KiB step slot split into two k-32 half-slots ([256 rows][32 k] X and
// Y images, 64-B rows, swizzle nt_chunk<32>), each freed by its own barrier (two per step) and
// refilled three half-steps ahead: block A(it) = the first half's MFMAs + the second half's
// reads + step it+2's FIRST half DMA; block B(it) = the second half's MFMAs + step it+1's first
// half reads + step it+2's SECOND half DMA. Every barrier waits with 16 pieces still in flight.
template <class Epi>
__global__ __launch_bounds__(256) void fc_asm2_kernel(const __bf16* __restrict__ X, const __bf16* __restrict__ Y, int NY,
                                                      int K, int ntx, int ntiles, Epi epi) {
    constexpr int BX = 256, BY = 256, BK = 64, HS = 32768, NST = 32;  // half-slot bytes
    __shared__ __attribute__((aligned(16))) char lds[4 * HS + Epi::kLdsFloats * 4];
    const int lane = threadIdx.x & 63, w = wave_id(), G = lane >> 4;
    const int wx = w >> 1, wy = w & 1;
    const int NG = gridDim.x, lg = xcd_remap(blockIdx.x, NG);
    const int nk = K / BK;
    const int total = ((ntiles - 1 - lg) / NG + 1) * nk;
    const uint32_t lbase = lds_addr(lds);
    const float* lb = (const float*)(lds + 4 * HS);
    epi.init((float*)(lds + 4 * HS), threadIdx.x, 256);
    // piece j < 4: X rows (w + 4j) * 16 + lane / 4; j >= 4: Y rows (w + 4(j - 4)) * 16 + lane / 4
    uint32_t vo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int prow = (w + 4 * (j & 3)) * 16 + lane / 4;
        vo[j] = (uint32_t)((prow * K + nt_chunk<32>(lane % 4, prow) * 8) * 2);
    }
    const int r15 = lane & 15, sw = nt_chunk<32>(G, r15);  // chunk position of k-group G
    auto bxa = [&](int hs) { return lbase + (uint32_t)(hs * HS + (wx * 128 + r15) * 64 + (sw << 4)); };
    auto bya = [&](int hs) { return lbase + (uint32_t)(hs * HS + 16384 + (wy * 128 + r15) * 64 + (sw << 4)); };
    auto dma = [&](int j, int h) {  // half h of step j into half-slot (j % 2) * 2 + h
        const bool live = j < total;
        const int t = live ? lg + (j / nk) * NG : lg, kt = j % nk;
        const int ty = t / ntx, tx = t - ty * ntx;
        const fi_i32x4 rx = make_rsrc(X + (size_t)tx * BX * K, live ? (uint32_t)BX * K * 2 : 0u);
        const fi_i32x4 ry = make_rsrc(Y + (size_t)ty * BY * K, live ? (uint32_t)min(BY, NY - ty * BY) * K * 2 : 0u);
        const uint32_t mx = lbase + (uint32_t)(((j % 2) * 2 + h) * HS + w * 1024);
        return std::make_tuple(rx, ry, (uint32_t)(kt * BK * 2 + h * 64), mx, mx + 16384u);
    };
    if (total <= 0) return;
    for (int j = 0; j < 2; ++j)
        for (int h = 0; h < 2; ++h) {
            auto [rx, ry, ko, mx, my] = dma(j, h);
            fc_asm2_dma(vo, rx, ry, ko, mx, my);
        }
    vm_wait_rt(24);  // step 0's first half landed
    lds_barrier();
    bf16x8 P[16], Q[16];
    {
        const uint32_t bx = bxa(0), by = bya(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) P[j] = *(const bf16x8*)((const char*)lds + (bx - lbase) + j * 1024);
#pragma unroll
        for (int j = 0; j < 8; ++j) P[8 + j] = *(const bf16x8*)((const char*)lds + (by - lbase) + j * 1024);
    }
    const int mytiles = total / nk;
    int it = 0, last_epi = -(1 << 20);
    for (int tile_it = 0; tile_it < mytiles; ++tile_it) {
        f32x4 acc[64];
#pragma unroll
        for (int i = 0; i < 64; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt, ++it) {
            const int sl = it % 2, sn = (it + 1) % 2;
            const int behind = 16 + (last_epi == it - 1 ? NST : 0);  // pieces (+ stores) newer than the one waited for
            vm_wait_rt(behind);  // step it's second half landed; everyone is done with half-slot sl*2
            lds_barrier();
            {
                auto [rx, ry, ko, mx, my] = dma(it + 2, 0);
                fc_asm2_mfma_reads_dma(acc, P, Q, bxa(sl * 2 + 1), bya(sl * 2 + 1), vo, rx, ry, ko, mx, my);
            }
            vm_wait_rt(behind);  // step it+1's first half landed; everyone is done with half-slot sl*2+1
            lds_barrier();
            {
                auto [rx, ry, ko, mx, my] = dma(it + 2, 1);
                fc_asm2_mfma_reads_dma(acc, Q, P, bxa(sn * 2), bya(sn * 2), vo, rx, ry, ko, mx, my);
            }
        }
        const int t = lg + tile_it * NG;
        const int ty = t / ntx, tx = t - ty * ntx;
        const int y0 = ty * BY;
        const OutTile ot = epi.tile(y0, min(BY, NY - y0));
        const int xw = tx * BX + wx * 128, yb = y0 + wy * 128 + (lane & 15);
#pragma unroll
        for (int g = 0; g < 8; ++g)
#pragma unroll
            for (int f = 0; f < 8; f += 2)
                Epi::template pair<0>(ot, lb, xw + f * 16, yb + g * 16, G, acc[f * 8 + g], acc[(f + 1) * 8 + g]);
        last_epi = it - 1;
    }
}
}  // namespace fcg

using namespace fcg;

template <int BX, int BY, int WX, int WY, int NL, int OPT = 0>
static int fc_fwd_ws_impl(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_fwd: rows must be positive");
    const int ntx = FCO / BX, nty = (rows + BY - 1) / BY, nt = ntx * nty;
    hipLaunchKernelGGL((fc_ws_kernel<BX, BY, WX, WY, NL, 64, 3, EpiFwd, OPT>), dim3(std::min(nt, 256)),
                       dim3(64 * (WX * WY + NL)), 0, s, wT, a3, rows, FCK, ntx, nt, EpiFwd{{h}, bias});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

template <int BX, int BY, int WX, int WY, int NL, int OPT = 0>
static int fc_dgrad_ws_impl(const __bf16* dh, const __bf16* w, __bf16* da3, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_dgrad: rows must be positive");
    const int ntx = FCK / BX, nty = (rows + BY - 1) / BY, nt = ntx * nty;
    hipLaunchKernelGGL((fc_ws_kernel<BX, BY, WX, WY, NL, 64, 3, EpiDgrad, OPT>), dim3(std::min(nt, 256)),
                       dim3(64 * (WX * WY + NL)), 0, s, w, dh, rows, FCO, ntx, nt, EpiDgrad{{da3}});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

static int fc_fwd2_impl(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_fwd: rows must be positive");
    const int ntx = FCO / 256, nty = (rows + 255) / 256, nt = ntx * nty;
    hipLaunchKernelGGL((fc_nt2_kernel<EpiFwd>), dim3(std::min(nt, 256)), dim3(512), 0, s, wT, a3, rows, FCK, ntx, nt,
                       EpiFwd{{h}, bias});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

template <int ABL = 0>
static int fc_fwd_asm_impl(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_fwd: rows must be positive");
    const int ntx = FCO / 256, nty = (rows + 255) / 256, nt = ntx * nty;
    hipLaunchKernelGGL((fc_asm_kernel<EpiFwd, ABL>), dim3(std::min(nt, 256)), dim3(256), 0, s, wT, a3, rows, FCK, ntx, nt,
                       EpiFwd{{h}, bias});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

static int fc_fwd_asm2_impl(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s) {
    FI_REQUIRE(rows > 0, "fc_fwd: rows must be positive");
    const int ntx = FCO / 256, nty = (rows + 255) / 256, nt = ntx * nty;
    hipLaunchKernelGGL((fc_asm2_kernel<EpiFwd>), dim3(std::min(nt, 256)), dim3(256), 0, s, wT, a3, rows, FCK, ntx, nt,
                       EpiFwd{{h}, bias});
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

}  // namespace fi
