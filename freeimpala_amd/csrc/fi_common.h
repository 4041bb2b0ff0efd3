// fi_common.h -- internal helpers shared by the HIP translation units of libfi_learner.so.
// gfx950 (CDNA4) only: wave64, raw s_barrier, LDS-DMA (global_load_lds_dwordx4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "fi_learner.h"

namespace fi {

// thread-local last-error string behind fi_last_error()
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define FI_HIP_CHECK(expr)                                                                  \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return ::fi::fail(FI_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define FI_REQUIRE(cond, msg)                                        \
    do {                                                             \
        if (!(cond)) return ::fi::fail(FI_ERR_INVALID, (msg));       \
    } while (0)

// propagate a non-OK status code
#define FI_TRY(x)                     \
    do {                              \
        int _rc = (x);                \
        if (_rc != FI_OK) return _rc; \
    } while (0)

constexpr int kWave = 64;

// ------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------

// Workgroup barrier that also makes this wave's LDS writes visible (lgkmcnt(0)) but does
// NOT drain vmcnt, so LDS-DMA / global loads stay in flight across it (guide section 5,
// "Pipelining across barriers"). The "memory" clobber stops hipcc moving LDS ops across.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 63]; rounds n DOWN to the
// nearest encoded step (a smaller n only waits longer, never shorter).
__device__ __forceinline__ void wait_vmcnt(int n) {
#define FI_VMW(N) \
    case N:       \
        asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
        break;
    switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
        FI_VMW(0) FI_VMW(1) FI_VMW(2) FI_VMW(3) FI_VMW(4) FI_VMW(5) FI_VMW(6) FI_VMW(7)
        FI_VMW(8) FI_VMW(9) FI_VMW(10) FI_VMW(11) FI_VMW(12) FI_VMW(13) FI_VMW(14) FI_VMW(15)
        FI_VMW(16) FI_VMW(17) FI_VMW(18) FI_VMW(19) FI_VMW(20) FI_VMW(21) FI_VMW(22) FI_VMW(23)
        FI_VMW(24) FI_VMW(25) FI_VMW(26) FI_VMW(27) FI_VMW(28) FI_VMW(29) FI_VMW(30) FI_VMW(31)
        FI_VMW(32) FI_VMW(33) FI_VMW(34) FI_VMW(35) FI_VMW(36) FI_VMW(37) FI_VMW(38) FI_VMW(39)
        FI_VMW(40) FI_VMW(41) FI_VMW(42) FI_VMW(43) FI_VMW(44) FI_VMW(45) FI_VMW(46) FI_VMW(47)
        FI_VMW(48) FI_VMW(49) FI_VMW(50) FI_VMW(51) FI_VMW(52) FI_VMW(53) FI_VMW(54) FI_VMW(55)
        FI_VMW(56) FI_VMW(57) FI_VMW(58) FI_VMW(59) FI_VMW(60) FI_VMW(61) FI_VMW(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
#undef FI_VMW
}

// One LDS-DMA piece: each lane copies 16 bytes from its own global address `gsrc` to LDS
// byte address (lds_base + 16 * lane), lds_base wave-uniform. Issued through inline asm so
// hipcc neither counts it nor inserts conservative vmcnt(0) waits for it: the caller owns
// the vmcnt bookkeeping (guide section 5.7 item 1, glds16 recipe).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_base)
        : "memory");
}

// 16-byte store of a frame-resident kernel's output (default cache policy; FI_NT_STORES: the
// non-temporal policy, A/B knob). Round 5: with non-temporal stores the lines that two waves of a
// workgroup fill in halves (a3, a2, da2: 64 B each) left the L2 as separate partial writes --
// conv12_fwd 27.6, conv3_fwd 7.65, conv3_bwd 15.0 GB per launch; with the default policy they merge
// in the L2: 26.6 / 6.89 / 13.7 GB (1.00x algorithmic), the step 0.07 ms shorter
// (profiles/r05_plain_stores_ab.txt)
#ifdef FI_NT_STORES
#define FI_ST16(v, p) __builtin_nontemporal_store((v), (p))
#else
#define FI_ST16(v, p) (*(p) = (v))
#endif

// Opaque copy: the compiler must assume x changed here, so values derived from it are
// recomputed after this point instead of being hoisted (and spilled) out of a loop.
__device__ __forceinline__ int fi_opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Raw buffer descriptor (stride 0, range-checked to `bytes`) from wave-uniform inputs.
typedef int fi_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ fi_i32x4 make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    fi_i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    r[2] = __builtin_amdgcn_readfirstlane(bytes);
    r[3] = 0x00020000;
    return r;
}

// LDS-DMA through a buffer descriptor: lane copies 16 B from byte offset `voff` of the
// buffer to LDS (lds_base + 16 * lane). Offsets past the descriptor's range read as zero,
// which the conv backward kernels use for zero borders (FI_OOB).
constexpr uint32_t FI_OOB = 0x80000000u;
__device__ __forceinline__ void blds16(fi_i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_base)
        : "memory");
}

// blds16 with the non-temporal cache policy: for single-use streams (the V-trace inputs) the
// line is not kept in the caches / Infinity Cache after it is read
__device__ __forceinline__ void blds16_nt(fi_i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_base)
        : "memory");
}

// the same with 4 bytes per lane: LDS (lds_base + 4 * lane)
__device__ __forceinline__ void blds4(fi_i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dword %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_base)
        : "memory");
}

template <typename T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(uintptr_t)p;
}

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// XCD-aware bijective remap (guide section 5, "XCD swizzle must be bijective"): blocks
// that share an XCD (same bid % 8) get consecutive logical ids.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace fi
