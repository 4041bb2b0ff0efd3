// blaslt_probe.cpp -- timing probe only (not product): hipBLASLt bf16 GEMMs at the fc-layer
// shapes of the Atari policy step (R = 101*4096 rows, 3136 -> 512): every heuristic candidate
// (up to 16), and the weight gradient split into a strided batch over row chunks.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/blaslt_probe.cpp -lhipblaslt -o build/blaslt_probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        auto e = (x);                                                                \
        if ((int)e != 0) { std::printf("err %d at %s:%d\n", (int)e, __FILE__, __LINE__); std::exit(1); } \
    } while (0)

// column-major D[m x n] = op(A)[m x k] * op(B)[k x n], batch of `batch` with strides sa/sb/sd
static double run(hipblasLtHandle_t h, int m, int n, int k, bool ta, bool tb, hipDataType dt_d, const void* A,
                  const void* B, void* D, void* ws, size_t wsb, int iters, int batch = 1, long long sa = 0,
                  long long sb = 0, long long sd = 0) {
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
    hipblasLtMatrixLayout_t la, lb, ld;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ta ? k : m, ta ? m : k, ta ? k : m));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, tb ? n : k, tb ? k : n, tb ? n : k));
    CK(hipblasLtMatrixLayoutCreate(&ld, dt_d, m, n, m));
    if (batch > 1) {
        for (auto [l, s] : {std::pair{la, sa}, std::pair{lb, sb}, std::pair{ld, sd}}) {
            CK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &batch, sizeof(batch)));
            CK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &s, sizeof(s)));
        }
    }
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t res[16];
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 16, res, &got));
    if (!got) { std::printf("no algo\n"); return 0; }
    float alpha = 1.f, beta = 0.f;
    double best = 1e30;
    int bi = -1;
    for (int a = 0; a < got; ++a) {
        if (hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[a].algo, ws, wsb, 0) != 0) continue;
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i)
            CK(hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[a].algo, ws, wsb, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms / iters < best) { best = ms / iters; bi = a; }
    }
    std::printf("   (%d candidates, best #%d)\n", got, bi);
    return best;
}

__global__ void fill(uint16_t* d, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
        x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
        const float v = (float)(x >> 8) * (1.0f / 8388608.0f) - 1.0f;
        d[i] = __builtin_bit_cast(uint16_t, (__bf16)v);
    }
}

int main(int argc, char** argv) {
    const bool rnd = argc > 1;
    const long R = 101L * 4096, K = 3136, N = 512;
    void *a3, *w, *h, *dh, *da3, *dw, *ws;
    const size_t wsb = 256 << 20;
    CK(hipMalloc(&a3, R * K * 2));
    CK(hipMalloc(&da3, R * K * 2));
    CK(hipMalloc(&h, R * N * 2));
    CK(hipMalloc(&dh, R * N * 2));
    CK(hipMalloc(&w, K * N * 2));
    CK(hipMalloc(&dw, 32 * K * N * 4));
    CK(hipMalloc(&ws, wsb));
    if (rnd) {  // hashed values in [-1, 1)
        fill<<<2048, 256>>>((uint16_t*)a3, R * K, 1);
        fill<<<2048, 256>>>((uint16_t*)dh, R * N, 2);
        fill<<<2048, 256>>>((uint16_t*)w, K * N, 3);
        CK(hipDeviceSynchronize());
    } else {
        CK(hipMemset(a3, 0x3c, R * K * 2));
        CK(hipMemset(dh, 0x3c, R * N * 2));
        CK(hipMemset(w, 0x3c, K * N * 2));
    }
    std::printf("operands: %s\n", rnd ? "hashed random" : "constant 0x3c3c");
    hipblasLtHandle_t hd;
    CK(hipblasLtCreate(&hd));
    const double fl = 2.0 * R * K * N;
    double t = run(hd, N, R, K, false, false, HIP_R_16BF, w, a3, h, ws, wsb, 5);
    std::printf("fc_fwd   %.3f ms  %.0f TF/s\n", t, fl / t / 1e9);
    t = run(hd, K, R, N, true, false, HIP_R_16BF, w, dh, da3, ws, wsb, 5);
    std::printf("fc_dgrad %.3f ms  %.0f TF/s\n", t, fl / t / 1e9);
    t = run(hd, N, K, R, false, true, HIP_R_32F, dh, a3, dw, ws, wsb, 5);
    std::printf("fc_wgrad %.3f ms  %.0f TF/s\n", t, fl / t / 1e9);
    for (int b : {4, 8, 16, 32}) {  // row chunks: dW_b^T[N x K] = dh_b^T a3_b, then a sum of b partials
        const long rc = R / b;
        t = run(hd, N, K, rc, false, true, HIP_R_32F, dh, a3, dw, ws, wsb, 5, b, rc * N, rc * K, (long long)N * K);
        std::printf("fc_wgrad batch %2d x %ld rows  %.3f ms  %.0f TF/s (+ sum of partials)\n", b, rc, t, fl / t / 1e9);
    }
    // dgrad as the transposed product: da3^T? same; try bf16 B stored transposed (dh^T layout) not available
    return 0;
}
