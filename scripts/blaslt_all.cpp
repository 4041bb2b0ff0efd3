// blaslt_all.cpp -- timing probe only (not product): every hipBLASLt algorithm that supports
// each fc-layer GEMM of the Atari step (R = 101*4096 rows, 3136 -> 512), against the
// heuristic's top 64. Prints the fastest few of each.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 scripts/blaslt_all.cpp -lhipblaslt -o build/blaslt_all
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                          \
    do {                                                                                               \
        auto e = (x);                                                                                  \
        if ((int)e != 0) { std::printf("err %d at %s:%d\n", (int)e, __FILE__, __LINE__); std::exit(1); } \
    } while (0)

struct Case {
    const char* name;
    int m, n, k;
    bool ta, tb;
    hipDataType dt;
    hipblasLtEpilogue_t epi;
    int batch;
};

int main(int argc, char** argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 101 * 4096;
    const int K = 3136, N = 512;
    hipblasLtHandle_t h;
    CK(hipblasLtCreate(&h));
    size_t wsb = 64u << 20;
    void *ws, *A, *B, *D, *bias;
    CK(hipMalloc(&ws, wsb));
    CK(hipMalloc(&A, (size_t)R * K * 2));
    CK(hipMalloc(&B, (size_t)R * K * 2));
    CK(hipMalloc(&D, (size_t)R * K * 4));
    CK(hipMalloc(&bias, 4096 * 4));
    CK(hipMemset(A, 0x3c, (size_t)R * K * 2));
    CK(hipMemset(B, 0x3b, (size_t)R * K * 2));
    CK(hipMemset(bias, 0, 4096 * 4));
    std::vector<Case> cases = {
        {"fwd", N, R, K, false, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_RELU_BIAS, 1},
        {"dgrad", K, R, N, true, false, HIP_R_16BF, HIPBLASLT_EPILOGUE_DEFAULT, 1},
        {"wgrad_split32", N, K, R / 32, false, true, HIP_R_32F, HIPBLASLT_EPILOGUE_DEFAULT, 32},
    };
    for (const Case& c : cases) {
        hipblasLtMatmulDesc_t desc;
        CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
        hipblasOperation_t opa = c.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = c.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &c.epi, sizeof(c.epi)));
        if (c.epi == HIPBLASLT_EPILOGUE_RELU_BIAS) {
            const hipDataType bt = HIP_R_32F;
            CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
            CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
        }
        hipblasLtMatrixLayout_t la, lb, ld;
        CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, c.ta ? c.k : c.m, c.ta ? c.m : c.k, c.ta ? c.k : c.m));
        CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, c.tb ? c.n : c.k, c.tb ? c.k : c.n, c.tb ? c.n : c.k));
        CK(hipblasLtMatrixLayoutCreate(&ld, c.dt, c.m, c.n, c.m));
        if (c.batch > 1) {
            const int32_t bc = c.batch;
            const int64_t sa = (int64_t)c.m * c.k, sb = (int64_t)c.n * c.k, sd = (int64_t)c.m * c.n;
            for (auto [l, s] : {std::pair{la, sa}, std::pair{lb, sb}, std::pair{ld, sd}}) {
                CK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
                CK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &s, sizeof(s)));
            }
        }
        // heuristic top 64
        hipblasLtMatmulPreference_t pref;
        CK(hipblasLtMatmulPreferenceCreate(&pref));
        CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
        std::vector<hipblasLtMatmulHeuristicResult_t> heur(64);
        int got = 0;
        CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 64, heur.data(), &got));
        heur.resize(got);
        std::vector<int> hidx;
        for (auto& r : heur) hidx.push_back(hipblaslt_ext::getIndexFromAlgo(r.algo));
        std::vector<hipblasLtMatmulHeuristicResult_t> all;
        CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opa, opb, HIP_R_16BF, HIP_R_16BF,
                                      c.dt, c.dt, HIPBLAS_COMPUTE_32F, all));
        const float alpha = 1.f, beta = 0.f;
        std::vector<std::pair<float, int>> times;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        int nsup = 0;
        for (size_t a = 0; a < all.size(); ++a) {
            size_t need = 0;
            if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &alpha, la, lb, &beta, ld, ld, all[a].algo, need) != 0) continue;
            if (need > wsb) continue;
            ++nsup;
            if (hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &all[a].algo, ws, wsb, 0) != 0) continue;
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 2; ++i)
                CK(hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &all[a].algo, ws, wsb, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            times.push_back({ms / 2, hipblaslt_ext::getIndexFromAlgo(all[a].algo)});
        }
        std::sort(times.begin(), times.end());
        float hbest = 1e30f;
        for (auto& t : times)
            if (std::find(hidx.begin(), hidx.end(), t.second) != hidx.end()) { hbest = t.first; break; }
        std::printf("%s: %zu algos, %d supported, heuristic-best %.3f ms; fastest:", c.name, all.size(), nsup, hbest);
        for (size_t i = 0; i < times.size() && i < 6; ++i) {
            const bool inh = std::find(hidx.begin(), hidx.end(), times[i].second) != hidx.end();
            std::printf(" %.3f(%d%s)", times[i].first, times[i].second, inh ? "*" : "");
        }
        std::printf("\n");
        std::fflush(stdout);
    }
    return 0;
}
