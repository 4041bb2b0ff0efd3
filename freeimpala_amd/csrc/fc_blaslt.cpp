// fc_blaslt.cpp -- the Atari policy's fully connected layer (3136 -> 512) on hipBLASLt.
//
// The fc layer is three plain bf16 GEMMs over R = (T+1)*B rows (no gathers, no fused
// masks of other tensors), which is what the library GEMM is for (hand-written MFMA kernels
// stay on the convolutions, the heads and the V-trace scan):
//   forward  h[R][512]    = relu(a3[R][3136] W[3136][512] + b)   (epilogue RELU_BIAS, bf16 out)
//   dgrad    da3[R][3136] = dh[R][512] W^T                      (bf16 out; the ReLU mask of
//                                                                 a3 is applied where conv3's
//                                                                 backward reads da3)
//   wgrad    dW[3136][512] = a3^T dh  (fp32 out, straight into the gradient blob)
// All row-major; hipBLASLt is column-major, so each call computes the transposed product.
// W is the bf16 copy of the fp32 master in the oracle's [3136][512] order.
// Algorithms: the heuristic's top 64 candidates (plus, at the bench shape, the fastest few of an
// exhaustive sweep, kSweepBest) are timed once at creation (16 missed a dgrad kernel 17 % faster),
// on operands filled
// with hashed bf16 values (the chip's clock under load depends on the data: candidates timed
// on zero-filled buffers ranked differently from the step), and the fastest kept. The choice is
// cached per GEMM shape for the life of the process, so every learner handle of one process
// runs the same algorithms and produces bit-identical results on identical inputs.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "fc_blaslt.h"
#include "fi_common.h"
#include "kernels.h"

namespace fi {

struct FcGemm {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
    hipblasLtMatmulAlgo_t algo{};
};

struct FcBlasLt {
    hipblasLtHandle_t h = nullptr;
    void* ws = nullptr;
    size_t wsb = 0;
    FcGemm g[5];  // 0 forward, 1 dgrad, 2 wgrad, 3 wgrad transposed (dW^T, then a transpose),
                  // 4 wgrad split over row blocks (a strided batch of partial dW, then a sum)
    int wgrad_mode = 0;      // 0 direct, 1 transposed, 2 split (the fastest at creation)
    float* dwT = nullptr;    // [512][3136] fp32 scratch of the transposed wgrad
    float* dwS = nullptr;    // [split][3136][512] fp32 partials of the split wgrad
    int split = 0;
    int rows = 0;
};

static std::string blt_err(const char* what, int st) { return std::string(what) + " failed: hipblasStatus " + std::to_string(st); }
#define BLT(x)                                                            \
    do {                                                                  \
        const int st_ = (int)(x);                                         \
        if (st_ != 0) { set_error(blt_err(#x, st_)); return FI_ERR_HIP; } \
    } while (0)

// shape -> hipBLASLt solution index of the timed winner (+ its time)
using GemmKey = std::tuple<int, int, int, bool, bool, int, int, int>;
#ifndef FI_BLT_CAND
#define FI_BLT_CAND 64
#endif
constexpr int kCand = FI_BLT_CAND;  // heuristic candidates timed at creation
static std::mutex g_algo_mu;
static std::map<GemmKey, std::pair<int, float>> g_algo_choice;  // -> (solution index, ms of 3 runs)
static std::map<int, int> g_wgrad_form;  // rows -> wgrad form (0 direct, 1 transposed, 2 + S split)

static void destroy_gemm(FcGemm& G) {
    if (G.la) hipblasLtMatrixLayoutDestroy(G.la);
    if (G.lb) hipblasLtMatrixLayoutDestroy(G.lb);
    if (G.ld) hipblasLtMatrixLayoutDestroy(G.ld);
    if (G.desc) hipblasLtMatmulDescDestroy(G.desc);
    G = FcGemm{};
}

// Extra candidates for the bench shape (R = 101 * 4096 rows), from an exhaustive sweep of every
// solution hipBLASLt 1.x of this image supports (scripts/blaslt_all.cpp: 1,242 forward and 2,050
// data-gradient solutions; the fastest ones are not in the heuristic's top 64). Solution indices
// are library-version specific: any that this library does not know or that does not support the
// problem is skipped, so the heuristic list alone remains the fallback.
static const std::map<std::tuple<int, int, int, bool, bool, int>, std::vector<int>> kSweepBest = {
    {{512, 101 * 4096, 3136, false, false, 1}, {436555, 437491, 436281, 436558, 436613, 436554}},
    {{3136, 101 * 4096, 512, true, false, 1}, {439401, 439365, 440236, 438309, 439398, 440239}},
};

static int make_gemm(FcBlasLt* F, FcGemm& G, int m, int n, int k, bool ta, bool tb, hipDataType dt_d,
                     hipblasLtEpilogue_t epi, const void* A, const void* B, void* D, hipStream_t s,
                     float* best_ms = nullptr, int batch = 1) {
    BLT(hipblasLtMatmulDescCreate(&G.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    const hipblasOperation_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    BLT(hipblasLtMatmulDescSetAttribute(G.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
    BLT(hipblasLtMatmulDescSetAttribute(G.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
    BLT(hipblasLtMatmulDescSetAttribute(G.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    if (epi == HIPBLASLT_EPILOGUE_RELU_BIAS) {
        const hipDataType bt = HIP_R_32F;
        BLT(hipblasLtMatmulDescSetAttribute(G.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
        const void* bias = D;  // any readable device buffer of >= m floats (timing only; set per call)
        BLT(hipblasLtMatmulDescSetAttribute(G.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    }
    BLT(hipblasLtMatrixLayoutCreate(&G.la, HIP_R_16BF, ta ? k : m, ta ? m : k, ta ? k : m));
    BLT(hipblasLtMatrixLayoutCreate(&G.lb, HIP_R_16BF, tb ? n : k, tb ? k : n, tb ? n : k));
    BLT(hipblasLtMatrixLayoutCreate(&G.ld, dt_d, m, n, m));
    if (batch > 1) {  // batch i = the i-th block of k (rows); D_i = its partial product
        const int32_t bc = batch;
        const int64_t sa = (int64_t)m * k, sb = (int64_t)n * k, sd = (int64_t)m * n;
        for (auto [L, st] : {std::make_pair(G.la, sa), std::make_pair(G.lb, sb), std::make_pair(G.ld, sd)}) {
            BLT(hipblasLtMatrixLayoutSetAttribute(L, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
            BLT(hipblasLtMatrixLayoutSetAttribute(L, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &st, sizeof(st)));
        }
    }
    hipblasLtMatmulPreference_t pref;
    BLT(hipblasLtMatmulPreferenceCreate(&pref));
    BLT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &F->wsb,
                                              sizeof(F->wsb)));
    std::vector<hipblasLtMatmulHeuristicResult_t> cands(kCand);
    int got = 0;
    const int st = (int)hipblasLtMatmulAlgoGetHeuristic(F->h, G.desc, G.la, G.lb, G.ld, G.ld, pref, kCand,
                                                        cands.data(), &got);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != 0 || got == 0) {
        set_error("hipBLASLt: no algorithm for the fc GEMM (m=" + std::to_string(m) + " n=" + std::to_string(n) +
                  " k=" + std::to_string(k) + ")");
        return FI_ERR_UNSUPPORTED;
    }
    cands.resize(got);
    const float alpha = 1.f, beta = 0.f;
    // solutions by index (the sweep table, or a cached winner): kept only if this library knows
    // them and they support this problem within the workspace
    auto add_by_index = [&](std::vector<int> idx) {
        std::vector<hipblasLtMatmulHeuristicResult_t> ex;
        const int rc = idx.empty() ? -1 : (int)hipblaslt_ext::getAlgosFromIndex(F->h, idx, ex);
        if (std::getenv("FI_VERBOSE"))
            std::fprintf(stderr, "[fc] %zu solutions by index: rc %d, %zu returned\n", idx.size(), rc, ex.size());
        if (rc != 0) return;
        for (auto& r : ex) {
            size_t need = 0;
            const int sup = (int)hipblaslt_ext::matmulIsAlgoSupported(F->h, G.desc, &alpha, G.la, G.lb, &beta, G.ld,
                                                                      G.ld, r.algo, need);
            if (std::getenv("FI_VERBOSE"))
                std::fprintf(stderr, "[fc]   solution %d: supported rc %d, workspace %zu\n",
                             hipblaslt_ext::getIndexFromAlgo(r.algo), sup, need);
            if (sup == 0 && need <= F->wsb) cands.push_back(r);
        }
    };
    auto find_index = [&](int idx) -> int {
        for (size_t a = 0; a < cands.size(); ++a)
            if (hipblaslt_ext::getIndexFromAlgo(cands[a].algo) == idx) return (int)a;
        return -1;
    };
    const GemmKey key{m, n, k, ta, tb, (int)dt_d, (int)epi, batch};
    {
        std::lock_guard<std::mutex> lk(g_algo_mu);
        auto it = g_algo_choice.find(key);
        if (it != g_algo_choice.end()) {  // same solution as every other handle of this process
            int a = find_index(it->second.first);
            if (a < 0) {
                add_by_index({it->second.first});
                a = find_index(it->second.first);
            }
            if (a >= 0) {
                G.algo = cands[a].algo;
                if (best_ms) *best_ms = it->second.second;
                return FI_OK;
            }
        }
    }
    if (std::getenv("FI_DETERMINISTIC")) {  // no timing: the heuristic's first solution, so every
        G.algo = cands[0].algo;             // process picks the same kernels (run-to-run bit-exact)
        if (best_ms) *best_ms = 0.f;
        return FI_OK;
    }
    auto tuned = kSweepBest.find({m, n, k, ta, tb, batch});
    if (tuned != kSweepBest.end() && !std::getenv("FI_BLT_NO_SWEEP")) add_by_index(tuned->second);
    // time the candidates once (the tensors hold hashed data at creation; only speed matters)
    hipEvent_t e0, e1;
    FI_HIP_CHECK(hipEventCreate(&e0));
    FI_HIP_CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    int bi = 0;
    for (size_t a = 0; a < cands.size(); ++a) {
        if (hipblasLtMatmul(F->h, G.desc, &alpha, A, G.la, B, G.lb, &beta, D, G.ld, D, G.ld, &cands[a].algo, F->ws,
                            F->wsb, s) != 0)
            continue;
        FI_HIP_CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < 3; ++i)
            BLT(hipblasLtMatmul(F->h, G.desc, &alpha, A, G.la, B, G.lb, &beta, D, G.ld, D, G.ld, &cands[a].algo,
                                F->ws, F->wsb, s));
        FI_HIP_CHECK(hipEventRecord(e1, s));
        FI_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        FI_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) { best = ms; bi = (int)a; }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (best >= 1e30f) {
        set_error("hipBLASLt: every fc GEMM candidate failed to launch");
        return FI_ERR_UNSUPPORTED;
    }
    if (std::getenv("FI_VERBOSE"))
        std::fprintf(stderr, "[fc] gemm m=%d n=%d k=%d batch=%d: %zu candidates (%d heuristic), best #%d %s %.3f ms/3\n",
                     m, n, k, batch, cands.size(), got, bi, bi >= got ? "(sweep)" : "(heuristic)", best);
    std::lock_guard<std::mutex> lk(g_algo_mu);
    // first timing wins for the whole process
    g_algo_choice.emplace(key, std::make_pair(hipblaslt_ext::getIndexFromAlgo(cands[bi].algo), best));
    const int want = g_algo_choice[key].first;
    int a = find_index(want);
    G.algo = cands[a >= 0 ? a : bi].algo;
    if (best_ms) *best_ms = g_algo_choice[key].second;
    return FI_OK;
}

// dW[3136][512] = transpose of dW^T[512][3136] (fp32, 32x32 tiles through LDS)
__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* __restrict__ src, int R, int C,
                                                            float* __restrict__ dst) {
    __shared__ float tile[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int i = ty; i < 32; i += 8)
        if (r0 + i < R && c0 + tx < C) tile[i][tx] = src[(size_t)(r0 + i) * C + c0 + tx];
    __syncthreads();
#pragma unroll
    for (int i = ty; i < 32; i += 8)
        if (c0 + i < C && r0 + tx < R) dst[(size_t)(c0 + i) * R + r0 + tx] = tile[tx][i];
}

static int transpose_f32(const float* src, int R, int C, float* dst, hipStream_t s) {
    hipLaunchKernelGGL(transpose_f32_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, s, src, R, C, dst);
    FI_HIP_CHECK(hipGetLastError());
    return FI_OK;
}

FcBlasLt* fc_blaslt_create(int rows, const void* a3, const void* w, const void* dh, void* h, void* da3,
                           float* dw, hipStream_t s) {
    FcBlasLt* F = new FcBlasLt();
    F->rows = rows;
    F->wsb = 64u << 20;
    int rc = FI_OK;
    if (hipblasLtCreate(&F->h) != 0) {
        set_error("hipblasLtCreate failed");
        rc = FI_ERR_HIP;
    }
    if (rc == FI_OK && hipMalloc(&F->ws, F->wsb) != hipSuccess) {
        set_error("hipBLASLt workspace allocation failed");
        rc = FI_ERR_OOM;
    }
    constexpr int K = 3136, N = 512;
    if (rc == FI_OK) {  // timing data (every buffer is overwritten by the step before it is read)
        rc = fill_hash_bf16((void*)a3, (size_t)rows * K, 1u, s);
        if (rc == FI_OK) rc = fill_hash_bf16((void*)dh, (size_t)rows * N, 2u, s);
        if (rc == FI_OK) rc = fill_hash_bf16((void*)w, (size_t)K * N, 3u, s);
    }
    // column-major views of the row-major products (see the header comment)
    if (rc == FI_OK) rc = make_gemm(F, F->g[0], N, rows, K, false, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_RELU_BIAS, w, a3, h, s);
    if (rc == FI_OK) rc = make_gemm(F, F->g[1], K, rows, N, true, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_DEFAULT, w, dh, da3, s);
    // wgrad forms: dW (column-major N x K) directly, dW^T (K x N) + a transpose, or S row blocks
    // as one strided-batched GEMM (S partial dW) summed by reduce_slabs in a fixed order
    // (S from FI_FC_SPLIT, or each of 8 / 16 / 32 / 64 that divides the rows)
    if (rc == FI_OK) rc = make_gemm(F, F->g[2], N, K, rows, false, true, HIP_R_32F, HIPBLASLT_EPILOGUE_DEFAULT, dh, a3, dw, s);
    if (rc == FI_OK && hipMalloc((void**)&F->dwT, (size_t)K * N * sizeof(float)) != hipSuccess) {
        set_error("fc: dW^T scratch allocation failed");
        rc = FI_ERR_OOM;
    }
    if (rc == FI_OK) rc = make_gemm(F, F->g[3], K, N, rows, false, true, HIP_R_32F, HIPBLASLT_EPILOGUE_DEFAULT, a3, dh, F->dwT, s);
    struct SplitForm {
        int S;
        FcGemm G;
        float* slab;
    };
    std::vector<SplitForm> splits;
    if (rc == FI_OK) {
        const char* e = std::getenv("FI_FC_SPLIT");
        const int fixed = e ? std::atoi(e) : 0;
        for (int S : {8, 16, 32, 64}) {
            if ((fixed > 0 && S != fixed) || rows % S || rows / S < 2048) continue;
            SplitForm sf{S, FcGemm{}, nullptr};
            if (hipMalloc((void**)&sf.slab, (size_t)S * K * N * sizeof(float)) != hipSuccess) break;
            if (make_gemm(F, sf.G, N, K, rows / S, false, true, HIP_R_32F, HIPBLASLT_EPILOGUE_DEFAULT, dh, a3, sf.slab,
                          s, nullptr, S) == FI_OK)
                splits.push_back(sf);
            else
                destroy_gemm(sf.G), (void)hipFree(sf.slab);
        }
    }
    // form 0 direct, 1 transposed, 2 + i split i: the process-wide choice for this row count
    // (every handle of the process then computes bit-identical gradients), else a tournament:
    // 2 rounds x 4 timed runs of each complete form (GEMM + transpose / partial sum), min kept
    int form = std::getenv("FI_DETERMINISTIC") ? 0 : -1;  // deterministic mode: dW directly
    if (rc == FI_OK && form < 0) {
        std::lock_guard<std::mutex> lk(g_algo_mu);
        auto it = g_wgrad_form.find(rows);
        if (it != g_wgrad_form.end()) {
            if (it->second < 2) form = it->second;
            for (size_t i = 0; i < splits.size(); ++i)
                if (it->second == 2 + splits[i].S) form = 2 + (int)i;
        }
    }
    auto run_form = [&](int f) -> int {
        const float alpha = 1.f, beta = 0.f;
        if (f == 0) { BLT(hipblasLtMatmul(F->h, F->g[2].desc, &alpha, dh, F->g[2].la, a3, F->g[2].lb, &beta, dw, F->g[2].ld, dw, F->g[2].ld, &F->g[2].algo, F->ws, F->wsb, s)); return FI_OK; }
        if (f == 1) {
            BLT(hipblasLtMatmul(F->h, F->g[3].desc, &alpha, a3, F->g[3].la, dh, F->g[3].lb, &beta, F->dwT, F->g[3].ld, F->dwT, F->g[3].ld, &F->g[3].algo, F->ws, F->wsb, s));
            return transpose_f32(F->dwT, 512, 3136, dw, s);
        }
        SplitForm& sf = splits[f - 2];
        BLT(hipblasLtMatmul(F->h, sf.G.desc, &alpha, dh, sf.G.la, a3, sf.G.lb, &beta, sf.slab, sf.G.ld, sf.slab, sf.G.ld, &sf.G.algo, F->ws, F->wsb, s));
        return reduce_slabs(sf.slab, sf.S, (size_t)K * N, dw, s);
    };
    if (rc == FI_OK && form < 0) {
        const int nf = 2 + (int)splits.size();
        std::vector<float> best(nf, 1e30f);
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) rc = FI_ERR_HIP;
        for (int round = 0; round < 2 && rc == FI_OK; ++round)
            for (int f = 0; f < nf && rc == FI_OK; ++f) {
                rc = run_form(f);  // warm
                if (rc == FI_OK && hipEventRecord(e0, s) != hipSuccess) rc = FI_ERR_HIP;
                for (int i = 0; i < 4 && rc == FI_OK; ++i) rc = run_form(f);
                float ms = 0.f;
                if (rc == FI_OK && (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                                    hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
                    rc = FI_ERR_HIP;
                if (rc == FI_OK) best[f] = std::min(best[f], ms / 4);
            }
        if (e0) hipEventDestroy(e0);
        if (e1) hipEventDestroy(e1);
        if (rc == FI_OK) {
            form = 0;
            for (int f = 1; f < nf; ++f)
                if (best[f] < best[form]) form = f;
            if (std::getenv("FI_VERBOSE")) {
                std::fprintf(stderr, "[fc] wgrad forms (ms/run): direct %.3f, transposed %.3f", best[0], best[1]);
                for (size_t i = 0; i < splits.size(); ++i) std::fprintf(stderr, ", split %d %.3f", splits[i].S, best[2 + i]);
                std::fprintf(stderr, " -> form %d\n", form);
            }
            std::lock_guard<std::mutex> lk(g_algo_mu);
            g_wgrad_form.emplace(rows, form < 2 ? form : 2 + splits[form - 2].S);  // first timing wins
        }
    }
    if (rc == FI_OK) {
        if (const char* e = std::getenv("FI_FC_WGRAD")) {  // experiment override: 0 / 1 / 2 (first split)
            const int m = std::atoi(e);
            if (m >= 0 && m <= 2 && (m != 2 || !splits.empty())) form = m;
        }
        F->wgrad_mode = form < 2 ? form : 2;
    }
    for (size_t i = 0; i < splits.size(); ++i) {  // keep the chosen split form only
        if (rc == FI_OK && form == 2 + (int)i) {
            F->g[4] = splits[i].G;
            F->dwS = splits[i].slab;
            F->split = splits[i].S;
        } else {
            destroy_gemm(splits[i].G);
            (void)hipFree(splits[i].slab);
        }
    }
    if (rc == FI_OK && hipStreamSynchronize(s) != hipSuccess) rc = FI_ERR_HIP;
    if (rc != FI_OK) {
        fc_blaslt_destroy(F);
        return nullptr;
    }
    return F;
}

void fc_blaslt_destroy(FcBlasLt* F) {
    if (!F) return;
    for (auto& G : F->g) destroy_gemm(G);
    if (F->ws) (void)hipFree(F->ws);
    if (F->dwT) (void)hipFree(F->dwT);
    if (F->dwS) (void)hipFree(F->dwS);
    if (F->h) hipblasLtDestroy(F->h);
    delete F;
}

static int run(FcBlasLt* F, FcGemm& G, const void* A, const void* B, void* D, hipStream_t s) {
    const float alpha = 1.f, beta = 0.f;
    BLT(hipblasLtMatmul(F->h, G.desc, &alpha, A, G.la, B, G.lb, &beta, D, G.ld, D, G.ld, &G.algo, F->ws, F->wsb, s));
    return FI_OK;
}

int fc_blaslt_forward(FcBlasLt* F, const void* a3, const void* w, const float* bias, void* h, hipStream_t s) {
    const void* b = bias;
    BLT(hipblasLtMatmulDescSetAttribute(F->g[0].desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &b, sizeof(b)));
    return run(F, F->g[0], w, a3, h, s);
}

int fc_blaslt_dgrad(FcBlasLt* F, const void* dh, const void* w, void* da3, hipStream_t s) {
    return run(F, F->g[1], w, dh, da3, s);
}

int fc_blaslt_wgrad(FcBlasLt* F, const void* a3, const void* dh, float* dw, hipStream_t s) {
    if (F->wgrad_mode == 1) {
        const int rc = run(F, F->g[3], a3, dh, F->dwT, s);
        return rc ? rc : transpose_f32(F->dwT, 512, 3136, dw, s);
    }
    if (F->wgrad_mode == 2) {
        const int rc = run(F, F->g[4], dh, a3, F->dwS, s);
        return rc ? rc : reduce_slabs(F->dwS, F->split, (size_t)3136 * 512, dw, s);
    }
    return run(F, F->g[2], dh, a3, dw, s);
}

}  // namespace fi
