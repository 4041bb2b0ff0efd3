/*
 * impala_oracle.c -- TEST INFRASTRUCTURE ONLY (the CPU oracle / CPU baseline).
 *
 * A plain-C restatement of the batched IMPALA learner step that freeimpala's
 * Learner::trainModel stands in for (reference: /root/reference/include/freeimpala/
 * learner.h:32-49 -- sleep + random bytes; the reference contains NO V-trace, loss or
 * network). The numerics therefore follow the IMPALA spec
 * (Espeholt et al. 2018, arXiv:1802.01561, section 4.1 eq. 1 and section 4.2) exactly
 * as restated in SURVEY.md section 8(a).
 *
 * Parity status: "parity unpinned by the reference" -- the reference has no golden
 * vectors / KATs for this path. This oracle is pinned
 * instead against (1) an independent PyTorch-autograd restatement whose outputs are
 * committed under tests/golden/ (tests/golden/make_golden.py), and (2) hand-derived
 * known-answer cases (tests/test_oracle.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library. The product (freeimpala_amd/, include/, cmd/) never links it.
 *
 * Conventions (shared with the HIP product, documented in DESIGN.md):
 *   - time-major tensors: logits (T,B,A), actions/rewards/discounts (T,B), values (T+1,B)
 *   - losses are SUMS over all T*B elements (not means), so a data-parallel
 *     sum-all-reduce of gradients equals the single-device gradient.
 *   - all reductions in double; outputs rounded to float once.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct orc_hparams {
    double rho_bar;        /* rho-bar: clip for the V-trace TD weights          */
    double c_bar;          /* c-bar: clip for the trace-cutting coefficients    */
    double pg_rho_bar;     /* clip for the policy-gradient importance weight    */
    double lambda_;        /* lambda multiplies c_t (IMPALA remark 2)           */
    double baseline_cost;  /* weight of 0.5 * sum (vs - V)^2                    */
    double entropy_cost;   /* weight of sum_a pi_a log pi_a  (negative entropy) */
} orc_hparams;

int orc_version(void) { return 3; }

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* log-softmax of one row of A logits, in double. lp[a] = z_a - logsumexp(z). */
static void log_softmax_row(const float* z, int A, double* lp) {
    double mx = -INFINITY;
    for (int a = 0; a < A; ++a) mx = z[a] > mx ? z[a] : mx;
    double s = 0.0;
    for (int a = 0; a < A; ++a) s += exp((double)z[a] - mx);
    double lse = mx + log(s);
    for (int a = 0; a < A; ++a) lp[a] = (double)z[a] - lse;
}

/*
 * V-trace targets + IMPALA loss + analytic gradients (SURVEY.md 8(a) rows "V-trace"
 * and "IMPALA loss + analytic grads").
 *
 *   log_rho_t = log pi(a_t|x_t) - log mu(a_t|x_t)
 *   rho_t     = min(rho_bar, exp(log_rho_t))
 *   c_t       = lambda * min(c_bar, exp(log_rho_t))
 *   delta_t   = rho_t * (r_t + gamma_t V_{t+1} - V_t)          (V_T = bootstrap)
 *   acc_T = 0;  acc_t = delta_t + gamma_t c_t acc_{t+1}           (reverse scan)
 *   vs_t      = V_t + acc_t                                     (vs_T := V_T)
 *   pg_adv_t  = min(pg_rho_bar, exp(log_rho_t)) (r_t + gamma_t vs_{t+1} - V_t)
 *   L = sum -pg_adv log pi(a_t) + bc * 0.5 sum (vs - V)^2 + ec * sum_a pi log pi
 *   dL/dz_a   = -pg_adv (1[a=a_t] - pi_a) + ec * pi_a (log pi_a - sum pi log pi)
 *   dL/dV_t   = bc (V_t - vs_t) for t < T, and 0 for the bootstrap row t = T.
 *
 * Outputs may be NULL (vs, pg_adv) when not wanted. losses[3] = {pg, baseline, entropy}
 * UNWEIGHTED sums (baseline already includes the 0.5); total = pg + bc*base + ec*ent.
 */
int orc_vtrace_loss(int T, int B, int A,
                    const float* pi_logits, const float* mu_logits,
                    const int32_t* actions, const float* rewards,
                    const float* discounts, const float* values,
                    const orc_hparams* hp,
                    float* vs_out, float* pg_adv_out,
                    float* dlogits, float* dvalue, double* losses) {
    if (T < 1 || B < 1 || A < 1 || A > 1024) return -1;
    double* part = (double*)calloc((size_t)B * 3, sizeof(double));
    if (!part) return -2;
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(|:bad)
    for (int b = 0; b < B; ++b) {
        double lpi[1024], lmu[1024];
        double acc_next = 0.0;                       /* acc_{t+1}, acc_T = 0 */
        double v_next = values[(size_t)T * B + b];   /* V_{t+1}, starts at bootstrap */
        double vs_next = v_next;                     /* vs_T = V_T */
        double pg = 0.0, base = 0.0, ent = 0.0;
        dvalue[(size_t)T * B + b] = 0.0f;
        for (int t = T - 1; t >= 0; --t) {
            size_t e = (size_t)t * B + b;
            const float* zp = pi_logits + e * A;
            const float* zm = mu_logits + e * A;
            int a_t = actions[e];
            if (a_t < 0 || a_t >= A) { bad = 1; a_t = 0; }
            log_softmax_row(zp, A, lpi);
            log_softmax_row(zm, A, lmu);
            double log_rho = lpi[a_t] - lmu[a_t];
            double ratio = exp(log_rho);
            double rho = ratio < hp->rho_bar ? ratio : hp->rho_bar;
            double c = hp->lambda_ * (ratio < hp->c_bar ? ratio : hp->c_bar);
            double pg_rho = ratio < hp->pg_rho_bar ? ratio : hp->pg_rho_bar;
            double r = rewards[e], g = discounts[e], v = values[e];
            double delta = rho * (r + g * v_next - v);
            double acc = delta + g * c * acc_next;
            double vs = v + acc;
            double adv = pg_rho * (r + g * vs_next - v);
            if (vs_out) vs_out[e] = (float)vs;
            if (pg_adv_out) pg_adv_out[e] = (float)adv;
            /* entropy term */
            double plogp = 0.0;
            for (int a = 0; a < A; ++a) plogp += exp(lpi[a]) * lpi[a];
            float* dz = dlogits + e * A;
            for (int a = 0; a < A; ++a) {
                double p = exp(lpi[a]);
                double d = -adv * ((a == a_t ? 1.0 : 0.0) - p)
                           + hp->entropy_cost * p * (lpi[a] - plogp);
                dz[a] = (float)d;
            }
            dvalue[e] = (float)(hp->baseline_cost * (v - vs));
            pg += -adv * lpi[a_t];
            base += 0.5 * acc * acc;
            ent += plogp;
            acc_next = acc; v_next = v; vs_next = vs;
        }
        part[(size_t)b * 3 + 0] = pg;
        part[(size_t)b * 3 + 1] = base;
        part[(size_t)b * 3 + 2] = ent;
    }
    double s0 = 0, s1 = 0, s2 = 0;
    for (int b = 0; b < B; ++b) { s0 += part[b * 3]; s1 += part[b * 3 + 1]; s2 += part[b * 3 + 2]; }
    losses[0] = s0; losses[1] = s1; losses[2] = s2;
    free(part);
    return bad ? -3 : 0;
}

/* ------------------------------------------------------------------------------------
 * Dense layers (row-major), double accumulation.
 *   Y[N][O] = X[N][I] W[I][O] + b[O]   (optional ReLU)
 * bf16_emul != 0: operands X and W are rounded to bf16 (RNE) before multiplying, the
 * way the product's bf16 MFMA path sees them; accumulation stays exact-ish (double).
 * ----------------------------------------------------------------------------------*/
static inline float bf16_round(float x) {
    uint32_t u; memcpy(&u, &x, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return x; /* inf/nan passthrough */
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    float y; memcpy(&y, &u, 4); return y;
}

float orc_bf16_round(float x) { return bf16_round(x); }

static inline float q(float x, int emul) { return emul ? bf16_round(x) : x; }

static void dense_fwd(int N, int I, int O, const float* X, const float* W, const float* bias,
                      int relu, int emul, float* Y) {
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) {
        double acc[4096];
        for (int o = 0; o < O; ++o) acc[o] = 0.0;
        for (int i = 0; i < I; ++i) {
            double x = q(X[(size_t)n * I + i], emul);
            if (x == 0.0) continue;
            const float* w = W + (size_t)i * O;
            for (int o = 0; o < O; ++o) acc[o] += x * (double)q(w[o], emul);
        }
        for (int o = 0; o < O; ++o) {
            double y = acc[o] + (bias ? bias[o] : 0.0);
            if (relu && y < 0) y = 0;
            Y[(size_t)n * O + o] = (float)y;
        }
    }
}

/* dX[N][I] = dY[N][O] W^T ; optionally multiplied by (Xact > 0) (ReLU'(pre) via post-act). */
static void dense_dgrad(int N, int I, int O, const float* dY, const float* W,
                        const float* mask_act, int emul, float* dX) {
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) {
        const float* dy = dY + (size_t)n * O;
        for (int i = 0; i < I; ++i) {
            double s = 0.0;
            const float* w = W + (size_t)i * O;
            for (int o = 0; o < O; ++o) s += (double)q(dy[o], emul) * (double)q(w[o], emul);
            if (mask_act && !(mask_act[(size_t)n * I + i] > 0.0f)) s = 0.0;
            dX[(size_t)n * I + i] = (float)s;
        }
    }
}

/* dW[I][O] = X^T dY ; db[O] = sum_n dY  (reduction over N, double, deterministic). */
static void dense_wgrad(int N, int I, int O, const float* X, const float* dY, int emul,
                        float* dW, float* db) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < I; ++i) {
        double acc[4096];
        for (int o = 0; o < O; ++o) acc[o] = 0.0;
        for (int n = 0; n < N; ++n) {
            double x = q(X[(size_t)n * I + i], emul);
            if (x == 0.0) continue;
            const float* dy = dY + (size_t)n * O;
            for (int o = 0; o < O; ++o) acc[o] += x * (double)q(dy[o], emul);
        }
        for (int o = 0; o < O; ++o) dW[(size_t)i * O + o] = (float)acc[o];
    }
    if (db) {
        for (int o = 0; o < O; ++o) {
            double s = 0.0;
            for (int n = 0; n < N; ++n) s += (double)dY[(size_t)n * O + o];
            db[o] = (float)s;
        }
    }
}

/* ------------------------------------------------------------------------------------
 * MLP policy (config #2): obs D -> H relu -> H relu -> (A logits | 1 value).
 * Flat parameter layout (fp32, little endian), identical to the product's blob:
 *   W1[D][H] b1[H] W2[H][H] b2[H] Wh[H][A+1] bh[A+1]
 * ----------------------------------------------------------------------------------*/
size_t orc_mlp_param_count(int D, int H, int A) {
    return (size_t)D * H + H + (size_t)H * H + H + (size_t)H * (A + 1) + (A + 1);
}

int orc_mlp_forward(int N, int D, int H, int A, const float* obs, const float* params,
                    float* h1, float* h2, float* out) {
    int O = A + 1;
    if (H > 4096 || O > 4096) return -1;
    const float* W1 = params;
    const float* b1 = W1 + (size_t)D * H;
    const float* W2 = b1 + H;
    const float* b2 = W2 + (size_t)H * H;
    const float* Wh = b2 + H;
    const float* bh = Wh + (size_t)H * O;
    dense_fwd(N, D, H, obs, W1, b1, 1, 0, h1);
    dense_fwd(N, H, H, h1, W2, b2, 1, 0, h2);
    dense_fwd(N, H, O, h2, Wh, bh, 0, 0, out);
    return 0;
}

/* dout[N][A+1] (dlogits | dvalue per row) -> grads (same layout as params). */
int orc_mlp_backward(int N, int D, int H, int A, const float* obs, const float* params,
                     const float* h1, const float* h2, const float* dout, float* grads) {
    int O = A + 1;
    if (H > 4096 || O > 4096) return -1;
    const float* W2 = params + (size_t)D * H + H;
    const float* Wh = W2 + (size_t)H * H + H;
    float* gW1 = grads;
    float* gb1 = gW1 + (size_t)D * H;
    float* gW2 = gb1 + H;
    float* gb2 = gW2 + (size_t)H * H;
    float* gWh = gb2 + H;
    float* gbh = gWh + (size_t)H * O;
    float* dz2 = (float*)malloc((size_t)N * H * sizeof(float));
    float* dz1 = (float*)malloc((size_t)N * H * sizeof(float));
    if (!dz1 || !dz2) { free(dz1); free(dz2); return -2; }
    dense_wgrad(N, H, O, h2, dout, 0, gWh, gbh);
    dense_dgrad(N, H, O, dout, Wh, h2, 0, dz2);
    dense_wgrad(N, H, H, h1, dz2, 0, gW2, gb2);
    dense_dgrad(N, H, H, dz2, W2, h1, 0, dz1);
    dense_wgrad(N, D, H, obs, dz1, 0, gW1, gb1);
    free(dz1); free(dz2);
    return 0;
}

/* ------------------------------------------------------------------------------------
 * Atari-shaped conv policy (config #3), NHWC, frames uint8 (84,84,4) scaled by 1/255:
 *   conv1 8x8/4 4->32 relu -> conv2 4x4/2 32->64 relu -> conv3 3x3/1 64->64 relu
 *   -> fc 3136->512 relu -> heads 512->(A logits | 1 value)
 * Parameter blob (fp32): c1W[8][8][4][32] c1b[32] c2W[4][4][32][64] c2b[64]
 *   c3W[3][3][64][64] c3b[64] fcW[3136][512] fcb[512] hW[512][A+1] hb[A+1]
 * bf16_emul != 0 rounds every GEMM operand (activations, weights, upstream grads) to
 * bf16 like the product's MFMA path; frames are integers (exact in bf16) and the 1/255
 * scale is applied to the fp32 accumulator.
 * ----------------------------------------------------------------------------------*/
#define AT_H 84
#define AT_C 4
size_t orc_atari_param_count(int A) {
    return 8 * 8 * 4 * 32 + 32 + 4 * 4 * 32 * 64 + 64 + 3 * 3 * 64 * 64 + 64 +
           (size_t)3136 * 512 + 512 + (size_t)512 * (A + 1) + (A + 1);
}

/* generic NHWC conv forward, input float (already scaled), double accumulation */
static void conv_fwd(int N, int IH, int IC, int K, int S, int OC, const float* X,
                     const float* W, const float* bias, float in_scale, int emul, float* Y) {
    int OH = (IH - K) / S + 1;
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) {
        double acc[64];
        for (int oy = 0; oy < OH; ++oy)
            for (int ox = 0; ox < OH; ++ox) {
                for (int o = 0; o < OC; ++o) acc[o] = 0.0;
                for (int ky = 0; ky < K; ++ky)
                    for (int kx = 0; kx < K; ++kx)
                        for (int c = 0; c < IC; ++c) {
                            double x = q(X[(((size_t)n * IH + oy * S + ky) * IH + ox * S + kx) * IC + c], emul);
                            if (x == 0.0) continue;
                            const float* w = W + (((size_t)ky * K + kx) * IC + c) * OC;
                            for (int o = 0; o < OC; ++o) acc[o] += x * (double)q(w[o], emul);
                        }
                float* y = Y + (((size_t)n * OH + oy) * OH + ox) * OC;
                for (int o = 0; o < OC; ++o) {
                    double v = acc[o] * in_scale + bias[o];
                    y[o] = (float)(v > 0 ? v : 0);
                }
            }
    }
}

/* dX (masked by X>0 when mask != 0) from dY; gather form */
static void conv_dgrad(int N, int IH, int IC, int K, int S, int OC, const float* dY,
                       const float* W, const float* Xact, int emul, float* dX) {
    int OH = (IH - K) / S + 1;
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n)
        for (int iy = 0; iy < IH; ++iy)
            for (int ix = 0; ix < IH; ++ix)
                for (int c = 0; c < IC; ++c) {
                    size_t xi = (((size_t)n * IH + iy) * IH + ix) * IC + c;
                    if (Xact && !(Xact[xi] > 0.0f)) { dX[xi] = 0.0f; continue; }
                    double s = 0.0;
                    for (int ky = 0; ky < K; ++ky) {
                        int ty = iy - ky;
                        if (ty < 0 || ty % S) continue;
                        int oy = ty / S;
                        if (oy >= OH) continue;
                        for (int kx = 0; kx < K; ++kx) {
                            int tx = ix - kx;
                            if (tx < 0 || tx % S) continue;
                            int ox = tx / S;
                            if (ox >= OH) continue;
                            const float* dy = dY + (((size_t)n * OH + oy) * OH + ox) * OC;
                            const float* w = W + (((size_t)ky * K + kx) * IC + c) * OC;
                            for (int o = 0; o < OC; ++o) s += (double)q(dy[o], emul) * (double)q(w[o], emul);
                        }
                    }
                    dX[xi] = (float)s;
                }
}

/* dW[ky][kx][c][o] = in_scale * sum_{n,oy,ox} X * dY ; db[o] = sum dY */
static void conv_wgrad(int N, int IH, int IC, int K, int S, int OC, const float* X,
                       const float* dY, float in_scale, int emul, float* dW, float* db) {
    int OH = (IH - K) / S + 1;
    int KK = K * K * IC;
#pragma omp parallel for schedule(static)
    for (int kk = 0; kk < KK; ++kk) {
        int ky = kk / (K * IC), kx = (kk / IC) % K, c = kk % IC;
        double acc[64];
        for (int o = 0; o < OC; ++o) acc[o] = 0.0;
        for (int n = 0; n < N; ++n)
            for (int oy = 0; oy < OH; ++oy)
                for (int ox = 0; ox < OH; ++ox) {
                    double x = q(X[(((size_t)n * IH + oy * S + ky) * IH + ox * S + kx) * IC + c], emul);
                    if (x == 0.0) continue;
                    const float* dy = dY + (((size_t)n * OH + oy) * OH + ox) * OC;
                    for (int o = 0; o < OC; ++o) acc[o] += x * (double)q(dy[o], emul);
                }
        for (int o = 0; o < OC; ++o) dW[(size_t)kk * OC + o] = (float)(acc[o] * in_scale);
    }
    for (int o = 0; o < OC; ++o) {
        double s = 0.0;
        for (size_t m = 0; m < (size_t)N * OH * OH; ++m) s += dY[m * OC + o];
        db[o] = (float)s;
    }
}

/* Checker for the full-depth weight-gradient test (tests/test_gpu_atari.py): fp64 sums of a
 * strided VALID conv's weight gradient straight from the GPU's own stored operands, for the
 * output channels cos[0..ncos):
 *   out[ky][kx][c][j] = sum_{n,oy,ox} X[n][oy*S+ky][ox*S+kx][c] * dY[n][oy][ox][cos[j]]
 * X: u8 (x_kind 0: raw frames, NHWC), bf16 NHWC (1), or bf16 in the stride-2 parity-plane order
 * [iy&1][ix&1][iy>>1][ix>>1][c] (2: conv21's a1 image order); dY: bf16 NHWC. No input scale.
 * Frames are split over the OpenMP threads; each thread's partial sums are added in thread
 * order (deterministic for a fixed thread count). Same arithmetic as conv_wgrad above, on the
 * stored bf16 values (no re-rounding needed: bf16 -> double is exact). */
static inline double bf16_bits_f64(uint16_t u) {
    union { uint32_t i; float f; } v;
    v.i = (uint32_t)u << 16;
    return (double)v.f;
}

int orc_conv_wgrad_f64(int N, int IH, int IC, int K, int S, int OC, const void* X, int x_kind,
                       const uint16_t* dY, int ncos, const int* cos, double* out) {
    if (N < 0 || IH < K || K < 1 || S < 1 || IC < 1 || OC < 1 || ncos < 1 || ncos > 64) return -1;
    if (x_kind == 2 && (IH & 1)) return -1;
    const int OH = (IH - K) / S + 1, KK = K * K * IC, HH = IH / 2;
    const size_t per = (size_t)KK * ncos;
    const int nt = orc_num_threads();
    double* part = (double*)calloc((size_t)nt * per, sizeof(double));
    if (!part) return -2;
#pragma omp parallel num_threads(nt)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        double* acc = part + (size_t)tid * per;
        double dy[64];
        double* xs = (double*)malloc(sizeof(double) * (size_t)KK);
#pragma omp for schedule(static)
        for (int n = 0; n < N; ++n) {
            for (int oy = 0; oy < OH; ++oy)
                for (int ox = 0; ox < OH; ++ox) {
                    const uint16_t* d = dY + (((size_t)n * OH + oy) * OH + ox) * OC;
                    int any = 0;
                    for (int j = 0; j < ncos; ++j) {
                        dy[j] = bf16_bits_f64(d[cos[j]]);
                        any |= dy[j] != 0.0;
                    }
                    if (!any) continue;
                    for (int ky = 0; ky < K; ++ky)
                        for (int kx = 0; kx < K; ++kx) {
                            const int iy = oy * S + ky, ix = ox * S + kx;
                            for (int c = 0; c < IC; ++c) {
                                size_t e;
                                if (x_kind == 2)
                                    e = ((((size_t)n * 4 + (iy & 1) * 2 + (ix & 1)) * HH + (iy >> 1)) * HH + (ix >> 1)) * IC + c;
                                else
                                    e = (((size_t)n * IH + iy) * IH + ix) * IC + c;
                                xs[(ky * K + kx) * IC + c] = x_kind == 0 ? (double)((const uint8_t*)X)[e]
                                                                         : bf16_bits_f64(((const uint16_t*)X)[e]);
                            }
                        }
                    if (ncos == 4) {  /* the test's case: a fixed-width inner loop the compiler vectorises */
                        for (int kk = 0; kk < KK; ++kk) {
                            const double x = xs[kk];
                            double* a = acc + (size_t)kk * 4;
                            for (int j = 0; j < 4; ++j) a[j] += x * dy[j];
                        }
                    } else {
                        for (int kk = 0; kk < KK; ++kk) {
                            const double x = xs[kk];
                            double* a = acc + (size_t)kk * ncos;
                            for (int j = 0; j < ncos; ++j) a[j] += x * dy[j];
                        }
                    }
                }
        }
        free(xs);
    }
    for (size_t i = 0; i < per; ++i) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += part[(size_t)t * per + i];
        out[i] = s;
    }
    free(part);
    return 0;
}

typedef struct orc_atari_acts {
    float* x0;  /* N*84*84*4 frames as float (unscaled integers)          */
    float* a1;  /* N*20*20*32 */
    float* a2;  /* N*9*9*64   */
    float* a3;  /* N*7*7*64 = N*3136 */
    float* h;   /* N*512      */
} orc_atari_acts;

static void atari_offsets(int A, size_t off[10]) {
    size_t o = 0;
    off[0] = o; o += 8 * 8 * 4 * 32;  off[1] = o; o += 32;
    off[2] = o; o += 4 * 4 * 32 * 64; off[3] = o; o += 64;
    off[4] = o; o += 3 * 3 * 64 * 64; off[5] = o; o += 64;
    off[6] = o; o += (size_t)3136 * 512; off[7] = o; o += 512;
    off[8] = o; o += (size_t)512 * (A + 1); off[9] = o;
}

int orc_atari_forward(int N, int A, const uint8_t* frames, const float* params, int emul,
                      float* a1, float* a2, float* a3, float* h, float* out) {
    size_t off[10]; atari_offsets(A, off);
    size_t nx = (size_t)N * AT_H * AT_H * AT_C;
    float* x0 = (float*)malloc(nx * sizeof(float));
    if (!x0) return -2;
    for (size_t i = 0; i < nx; ++i) x0[i] = (float)frames[i];
    conv_fwd(N, 84, 4, 8, 4, 32, x0, params + off[0], params + off[1], 1.0f / 255.0f, emul, a1);
    conv_fwd(N, 20, 32, 4, 2, 64, a1, params + off[2], params + off[3], 1.0f, emul, a2);
    conv_fwd(N, 9, 64, 3, 1, 64, a2, params + off[4], params + off[5], 1.0f, emul, a3);
    dense_fwd(N, 3136, 512, a3, params + off[6], params + off[7], 1, emul, h);
    dense_fwd(N, 512, A + 1, h, params + off[8], params + off[9], 0, emul, out);
    free(x0);
    return 0;
}

/* as orc_atari_backward, optionally returning the intermediate (masked) data gradients
 * dh (N,512), d3 (N,3136), d2 (N,81*64), d1 (N,400*32) -- any may be NULL */
int orc_atari_backward_ex(int N, int A, const uint8_t* frames, const float* params, int emul,
                          const float* a1, const float* a2, const float* a3, const float* h,
                          const float* dout, float* grads, float* dh_out, float* d3_out,
                          float* d2_out, float* d1_out);

int orc_atari_backward(int N, int A, const uint8_t* frames, const float* params, int emul,
                       const float* a1, const float* a2, const float* a3, const float* h,
                       const float* dout, float* grads) {
    return orc_atari_backward_ex(N, A, frames, params, emul, a1, a2, a3, h, dout, grads, NULL,
                                 NULL, NULL, NULL);
}

int orc_atari_backward_ex(int N, int A, const uint8_t* frames, const float* params, int emul,
                          const float* a1, const float* a2, const float* a3, const float* h,
                          const float* dout, float* grads, float* dh_out, float* d3_out,
                          float* d2_out, float* d1_out) {
    size_t off[10]; atari_offsets(A, off);
    int O = A + 1;
    size_t nx = (size_t)N * AT_H * AT_H * AT_C;
    float* x0 = (float*)malloc(nx * sizeof(float));
    float* dh = (float*)malloc((size_t)N * 512 * sizeof(float));
    float* d3 = (float*)malloc((size_t)N * 3136 * sizeof(float));
    float* d2 = (float*)malloc((size_t)N * 81 * 64 * sizeof(float));
    float* d1 = (float*)malloc((size_t)N * 400 * 32 * sizeof(float));
    if (!x0 || !dh || !d3 || !d2 || !d1) { free(x0); free(dh); free(d3); free(d2); free(d1); return -2; }
    for (size_t i = 0; i < nx; ++i) x0[i] = (float)frames[i];
    /* the device runs the heads backward in fp32 (packed VALU, K = A+1 is too thin for MFMA):
     * no operand rounding there, even in bf16-emulation mode (h is bf16-valued already) */
    dense_wgrad(N, 512, O, h, dout, 0, grads + off[8], grads + off[9]);
    dense_dgrad(N, 512, O, dout, params + off[8], h, 0, dh);
    dense_wgrad(N, 3136, 512, a3, dh, emul, grads + off[6], grads + off[7]);
    dense_dgrad(N, 3136, 512, dh, params + off[6], a3, emul, d3);
    conv_wgrad(N, 9, 64, 3, 1, 64, a2, d3, 1.0f, emul, grads + off[4], grads + off[5]);
    conv_dgrad(N, 9, 64, 3, 1, 64, d3, params + off[4], a2, emul, d2);
    conv_wgrad(N, 20, 32, 4, 2, 64, a1, d2, 1.0f, emul, grads + off[2], grads + off[3]);
    conv_dgrad(N, 20, 32, 4, 2, 64, d2, params + off[2], a1, emul, d1);
    conv_wgrad(N, 84, 4, 8, 4, 32, x0, d1, 1.0f / 255.0f, emul, grads + off[0], grads + off[1]);
    if (dh_out) memcpy(dh_out, dh, (size_t)N * 512 * sizeof(float));
    if (d3_out) memcpy(d3_out, d3, (size_t)N * 3136 * sizeof(float));
    if (d2_out) memcpy(d2_out, d2, (size_t)N * 81 * 64 * sizeof(float));
    if (d1_out) memcpy(d1_out, d1, (size_t)N * 400 * 32 * sizeof(float));
    free(x0); free(dh); free(d3); free(d2); free(d1);
    return 0;
}

/* ------------------------------------------------------------------------------------
 * Optimizers (flat fp32 buffers). Adam with bias correction (step counts from 1),
 * SGD, and global-norm clipping (returns the pre-clip norm; scale = min(1, max/(norm+1e-6))).
 * ----------------------------------------------------------------------------------*/
double orc_clip_grad_norm(size_t n, float* g, double max_norm) {
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) s += (double)g[i] * g[i];
    double norm = sqrt(s);
    if (max_norm > 0 && norm > max_norm) {
        float scale = (float)(max_norm / (norm + 1e-6));
        for (size_t i = 0; i < n; ++i) g[i] *= scale;
    }
    return norm;
}

void orc_adam(size_t n, float* p, const float* g, float* m, float* v, float lr, float b1,
              float b2, float eps, int step) {
    double bc1 = 1.0 - pow((double)b1, step);
    double bc2 = 1.0 - pow((double)b2, step);
    for (size_t i = 0; i < n; ++i) {
        float mi = b1 * m[i] + (1.0f - b1) * g[i];
        float vi = b2 * v[i] + (1.0f - b2) * g[i] * g[i];
        m[i] = mi; v[i] = vi;
        double mh = mi / bc1, vh = vi / bc2;
        p[i] = (float)(p[i] - lr * mh / (sqrt(vh) + eps));
    }
}

void orc_sgd(size_t n, float* p, const float* g, float lr) {
    for (size_t i = 0; i < n; ++i) p[i] -= lr * g[i];
}

/* ------------------------------------------------------------------------------------
 * Synthetic trajectories: Philox4x32-10, counter = (e_lo, e_hi,
 * stream, 0), key = (seed_lo, seed_hi). Element index e uses the GLOBAL batch column
 * so a shard's inputs do not depend on the GPU count.
 *   approx-normal  = (sum of four 24-bit uniforms - 2) * sqrt(3)  (Irwin-Hall, var 1)
 *   action         = ((u0 >> 8) * A) >> 24
 *   reward         = (u0 % 3) - 1
 *   done           = (u0 >> 8) < 167772   (p ~= 0.01); discount = done ? 0 : gamma
 *   frame byte j   = byte (j % 16) of the 4 outputs of counter e = pixel_block
 * All integer -> float steps are single IEEE ops, so the HIP generator matches bit-exactly.
 * ----------------------------------------------------------------------------------*/
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n1 = lo1, n2 = hi0 ^ c[3] ^ k1, n3 = lo0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

void orc_philox4(uint64_t seed, uint64_t e, uint32_t stream, uint32_t out[4]) {
    uint32_t c[4] = {(uint32_t)e, (uint32_t)(e >> 32), stream, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
}

static float approx_normal(const uint32_t u[4]) {
    uint32_t s = (u[0] >> 8) + (u[1] >> 8) + (u[2] >> 8) + (u[3] >> 8);
    float x = (float)((int32_t)s - (int32_t)(1u << 25));
    return x * 0x1.bb67aep-24f; /* fp32(sqrt(3)) * 2^-24 */
}

enum { ST_OBS = 0, ST_MU = 1, ST_ACT = 2, ST_REW = 3, ST_DONE = 4, ST_FRAME = 5 };

/* Fill one shard [b_off, b_off+B) of the global batch (B_glob columns). Any output may
 * be NULL. obs is (T+1,B,D); mu (T,B,A); act/rew/disc (T,B); frames (T+1,B,84*84*4). */
void orc_synth_batch(uint64_t seed, int T, int B, int B_glob, int b_off, int A, int D,
                     float gamma, float* obs, float* mu, int32_t* act, float* rew,
                     float* disc, uint8_t* frames) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t <= T; ++t) {
        uint32_t u[4];
        for (int b = 0; b < B; ++b) {
            uint64_t row = (uint64_t)t * B_glob + (uint64_t)(b_off + b);
            size_t lrow = (size_t)t * B + b;
            if (obs)
                for (int d = 0; d < D; ++d) {
                    orc_philox4(seed, row * D + d, ST_OBS, u);
                    obs[lrow * D + d] = approx_normal(u);
                }
            if (frames) {
                const int FB = 84 * 84 * 4;
                for (int qd = 0; qd < FB / 16; ++qd) {
                    orc_philox4(seed, row * (FB / 16) + qd, ST_FRAME, u);
                    memcpy(frames + lrow * FB + (size_t)qd * 16, u, 16);
                }
            }
            if (t == T) continue;
            if (mu)
                for (int a = 0; a < A; ++a) {
                    orc_philox4(seed, row * A + a, ST_MU, u);
                    mu[lrow * A + a] = approx_normal(u);
                }
            if (act) { orc_philox4(seed, row, ST_ACT, u); act[lrow] = (int32_t)(((uint64_t)(u[0] >> 8) * (uint32_t)A) >> 24); }
            if (rew) { orc_philox4(seed, row, ST_REW, u); rew[lrow] = (float)((int32_t)(u[0] % 3u) - 1); }
            if (disc) { orc_philox4(seed, row, ST_DONE, u); disc[lrow] = ((u[0] >> 8) < 167772u) ? 0.0f : gamma; }
        }
    }
}
