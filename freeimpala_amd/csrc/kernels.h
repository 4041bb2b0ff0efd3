// kernels.h -- internal launchers of libfi_learner.so (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_learner.h"

namespace fi {

// the heads' upstream gradient: virtual [rows][A+1] = dlogits (TB rows, then 0) | dvalue
struct HeadsGrad {
    const float* dlog;  // (TB, A)
    const float* dval;  // (rows)
    int rows;           // (T+1)*B
    int TB;             // T*B
    int A;
};

// vtrace.hip
size_t vtrace_workspace_bytes(int T, int B, int A);
int vtrace_launch(int variant, int T, int B, int A, const float* pi, const float* mu,
                  const int32_t* act, const float* rew, const float* disc, const float* val,
                  const fi_vtrace_hparams& hp, float* vs, float* adv, float* dlog, float* dval,
                  double* losses, void* ws, size_t ws_bytes, hipStream_t stream,
                  bool finalize = true, int* nblk_out = nullptr, int* bad = nullptr);
// bad: device counter of out-of-range actions (nullptr: a counter inside ws, zeroed here; with
// finalize the loss scalars become NaN when it is non-zero)
int vtrace_finalize_launch(void* ws, int nblk, double* losses, hipStream_t stream,
                           const int* bad = nullptr);
// per-workgroup loss partials [nblk][3] inside a vtrace workspace
const double* vtrace_partials(const void* ws);

// gemm_f32.hip (MLP, exact fp32)
int f32_linear_fwd(const float* X, int M, int K, const float* W, const float* bias, int N,
                   bool relu, float* Y, hipStream_t s);
int f32_heads_fwd(const float* X, int M, int K, const float* W, const float* bias, int A,
                  float* logits, float* values, hipStream_t s);
int f32_linear_dgrad(const float* dY, int M, int N, const float* W, int K, const float* act,
                     float* dX, hipStream_t s);
int f32_heads_dgrad(const HeadsGrad& g, const float* W, int K, const float* act, float* dX,
                    hipStream_t s);
int f32_linear_wgrad_partial(const float* X, int M, int I, const float* dY, int N, int splits,
                             float* slab, float* cs_slab, hipStream_t s);
int f32_heads_wgrad_partial(const float* X, int I, const HeadsGrad& g, int splits, float* slab,
                            float* cs_slab, hipStream_t s);
// heads weight gradient (slab [grid][H][A+1] + bias partials [grid][A+1]) and masked data
// gradient dz2 in one pass over h2 (H = 256, A = 18)
bool f32_heads_bwd_fused_supported(int H, int A);
constexpr int kHeadsFusedGrid = 512;
int f32_heads_bwd_fused(const HeadsGrad& g, const float* h2, const float* Wh, int H, float* dz2, float* slab,
                        float* cs_slab, int grid, hipStream_t s);

// misc.hip
int colsum_partial(const float* Y, int M, int N, int splits, float* slab, hipStream_t s);
int heads_colsum_partial(const HeadsGrad& g, int splits, float* slab, hipStream_t s);
// PyTorch-layout (W[N][K]) fp32 GEMMs on the same MFMA kernel (farmer.hip)
int f32_gemm_nt(const float* X, int ldx, int M, int K, const float* W, const float* bias, int N,
                bool relu, float* Y, hipStream_t s);
int f32_gemm_nn_dgrad(const float* dY, int M, int N, const float* W, int K, const float* act, float* dX,
                      hipStream_t s);
int f32_gemm_tn_wgrad(const float* dY, int M, int N, const float* X, int ldx, int K, int splits, float* slab,
                      hipStream_t s);
// fc_gemm.hip (the Atari fc layer, 3136 -> 512, rows = (T+1)*B)
int fc_fwd_launch(const __bf16* a3, const __bf16* wT, const float* bias, __bf16* h, int rows, hipStream_t s);
int fc_dgrad_launch(const __bf16* dh, const __bf16* w, __bf16* da3, int rows, hipStream_t s);  // da3 unmasked
int fc_wgrad_splits(int rows);  // R-slices (fp32 slabs of 3136 x 512) fc_wgrad_launch uses
int fc_wgrad_launch(const __bf16* a3, const __bf16* dh, float* slab, float* dw, int rows, hipStream_t s);
int reduce_slabs(float* slab, int splits, size_t count, float* out, hipStream_t s);  // slab is scratch (overwritten)
// squared L2 norm of g -> *out; optionally also sums vt_nblk V-trace loss partials [i][3]
// into vt_losses[0..2] in the same (final) launch; *nonfinite = 1 when the norm is NaN / Inf
int grad_sqnorm(const float* g, size_t n, double* part, int nblk, double* out, hipStream_t s,
                const double* vt_part = nullptr, int vt_nblk = 0, double* vt_losses = nullptr,
                int* nonfinite = nullptr);
int optimizer_step(int opt, float* p, const float* g, float* m, float* v, size_t n, float lr,
                   float b1, float b2, float eps, double bc1, double bc2, const double* sqnorm,
                   float max_norm, hipStream_t s, int* skip = nullptr);  // skip: int[4], see misc.hip
int to_bf16(const float* src, uint16_t* dst, size_t n, hipStream_t s);
int fill_hash_bf16(void* dst, size_t n, uint32_t seed, hipStream_t s);
int synth_launch(uint64_t seed, int T, int B, int B_glob, int b_off, int A, int D, float gamma,
                 float* obs, float* mu, int32_t* act, float* rew, float* disc, uint8_t* frames,
                 hipStream_t s);
// actions outside [0, A) are counted into *bad (nullable) and stored clamped
int ingest_launch(const void* rec, int T, int B, int A, int D, size_t entry_bytes, float* obs,
                  float* mu, int32_t* act, float* rew, float* disc, hipStream_t s, int* bad = nullptr);

}  // namespace fi
