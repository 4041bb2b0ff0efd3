// fc_blaslt.cpp -- the forward and data-gradient GEMMs of the Atari policy's fully connected
// layer (3136 -> 512) on hipBLASLt, the default for those two (fc_gemm.hip has hand-written
// kernels for all three; its weight gradient is the one the step uses, and FI_FC_OWN=1 takes
// its forward and data gradient too -- they run 20-25 % slower than these):
//   forward  h[R][512]    = relu(a3[R][3136] W[3136][512] + b)   (epilogue RELU_BIAS, bf16 out)
//   dgrad    da3[R][3136] = dh[R][512] W^T                      (bf16 out; the ReLU mask of
//                                                                 a3 is applied where conv3's
//                                                                 backward reads da3)
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
    FcGemm g[2];  // 0 forward, 1 dgrad
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
                     float* best_ms = nullptr) {
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
    const GemmKey key{m, n, k, ta, tb, (int)dt_d, (int)epi, 1};
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
    auto tuned = kSweepBest.find({m, n, k, ta, tb, 1});
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
        std::fprintf(stderr, "[fc] gemm m=%d n=%d k=%d: %zu candidates (%d heuristic), best #%d %s %.3f ms/3\n",
                     m, n, k, cands.size(), got, bi, bi >= got ? "(sweep)" : "(heuristic)", best);
    std::lock_guard<std::mutex> lk(g_algo_mu);
    // first timing wins for the whole process
    g_algo_choice.emplace(key, std::make_pair(hipblaslt_ext::getIndexFromAlgo(cands[bi].algo), best));
    const int want = g_algo_choice[key].first;
    int a = find_index(want);
    G.algo = cands[a >= 0 ? a : bi].algo;
    if (best_ms) *best_ms = g_algo_choice[key].second;
    return FI_OK;
}

FcBlasLt* fc_blaslt_create(int rows, const void* a3, const void* w, const void* dh, void* h, void* da3,
                           hipStream_t s) {
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
    if (rc == FI_OK) {  // timing data: the step overwrites a3 / h / da3 before reading them, and dh rows
        // T*B..N (never written by the step) get their zeros from atari_create, which runs after this call
        rc = fill_hash_bf16((void*)a3, (size_t)rows * K, 1u, s);
        if (rc == FI_OK) rc = fill_hash_bf16((void*)dh, (size_t)rows * N, 2u, s);
        if (rc == FI_OK) rc = fill_hash_bf16((void*)w, (size_t)K * N, 3u, s);
    }
    // column-major views of the row-major products (see the header comment)
    if (rc == FI_OK) rc = make_gemm(F, F->g[0], N, rows, K, false, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_RELU_BIAS, w, a3, h, s);
    if (rc == FI_OK) rc = make_gemm(F, F->g[1], K, rows, N, true, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_DEFAULT, w, dh, da3, s);
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

}  // namespace fi
