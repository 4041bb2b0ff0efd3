// fc_bench.hip -- A/B timing of fc_gemm.hip tile / ring configurations in ONE process
// (interleaved rounds, HIP events), at the bench shape R = 413,696 (T=100, B=4096), random
// bf16 operands. Every variant's output is compared bit for bit with the first variant of its
// GEMM (same k order per output element, so the results must be identical).
// Build: scripts/build_fc_bench.sh; run: build/fc_bench [rounds]
#define FI_FC_CONFIG_OVERRIDE
#define FC_FW_CFG 256, 256, 4, 2, 64, 2, 8 | 4096
#define FC_DG_CFG 224, 256, 1, 8, 64, 2, 1 | 2 | 128
#define FC_WG_CFG 256, 224, 4, 2, 64, 2
#include "../freeimpala_amd/csrc/fc_gemm.hip"

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace fi;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

struct Variant {
    std::string name;
    std::function<int(hipStream_t)> run;
    double flops;
    void* out;
    size_t out_bytes;
    int group;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int R = argc > 2 ? atoi(argv[2]) : 413696;
    const int reps = 10;
    const char* only = argc > 3 ? argv[3] : nullptr;  // run only variants whose name contains this
    hipStream_t s;
    CK(hipStreamCreate(&s));
    __bf16 *a3, *wT, *w, *dh, *h[2], *da3[2];
    float *bias, *slab, *dw[2];
    CK(hipMalloc(&a3, (size_t)R * FCK * 2));
    CK(hipMalloc(&dh, (size_t)R * FCO * 2));
    CK(hipMalloc(&wT, (size_t)FCK * FCO * 2));
    CK(hipMalloc(&w, (size_t)FCK * FCO * 2));
    CK(hipMalloc(&bias, FCO * 4));
    for (int i = 0; i < 2; ++i) {
        CK(hipMalloc(&h[i], (size_t)R * FCO * 2));
        CK(hipMalloc(&da3[i], (size_t)R * FCK * 2));
        CK(hipMalloc(&dw[i], (size_t)FCK * FCO * 4));
    }
    CK(hipMalloc(&slab, (size_t)20 * FCK * FCO * 4));
    fill_hash_bf16(a3, (size_t)R * FCK, 1, s);
    fill_hash_bf16(dh, (size_t)R * FCO, 2, s);
    fill_hash_bf16(wT, (size_t)FCK * FCO, 3, s);
    fill_hash_bf16(w, (size_t)FCK * FCO, 4, s);
    CK(hipMemsetAsync(bias, 0, FCO * 4, s));
    const double fl = 2.0 * R * FCK * FCO;
    std::vector<Variant> vs;
    // outputs: first variant of a group writes buffer 0, the others buffer 1
    auto add = [&](const char* nm, int group, std::function<int(hipStream_t, int)> f, void* o0, void* o1, size_t bytes) {
        if (only && !strstr(nm, only)) return;
        const bool first = std::none_of(vs.begin(), vs.end(), [&](const Variant& v) { return v.group == group; });
        void* o = first ? o0 : o1;
        const int which = first ? 0 : 1;
        vs.push_back({nm, [f, which](hipStream_t st) { return f(st, which); }, fl, o, bytes, group});
    };
#define FWDV(nm, ...) add("fwd  " nm, 0, [&](hipStream_t st, int k) { return fc_fwd_impl<__VA_ARGS__>(a3, wT, bias, h[k], R, st); }, h[0], h[1], (size_t)R * FCO * 2)
#define DGV(nm, ...) add("dgrd " nm, 1, [&](hipStream_t st, int k) { return fc_dgrad_impl<__VA_ARGS__>(dh, w, da3[k], R, st); }, da3[0], da3[1], (size_t)R * FCK * 2)
#define WGV(nm, S, ...) add("wgrd " nm, 2, [&](hipStream_t st, int k) { return fc_wgrad_impl<__VA_ARGS__>(a3, dh, slab, dw[k], R, st, S); }, dw[0], dw[1], (size_t)FCK * FCO * 4)
    // the shipped configurations first (fc_gemm.hip FC_*_CFG), then alternatives
    FWDV("256x256 w4x2 bk64 ns2 ntY midbar", 256, 256, 4, 2, 64, 2, 8 | 4096);
    DGV("224x256 w1x8 bk64 ns2 prio ntst xrow", 224, 256, 1, 8, 64, 2, 1 | 2 | 128);
    DGV("224x256 w1x8 bk64 ns2 prio ntst", 224, 256, 1, 8, 64, 2, 1 | 2);
    DGV("224x256 w1x8 bk64 ns2 prio xrow", 224, 256, 1, 8, 64, 2, 1 | 128);
    DGV("224x256 w1x8 bk64 ns2 prio", 224, 256, 1, 8, 64, 2, 1);
    DGV("448x128 w4x2 bk64 ns2 prio xrow", 448, 128, 4, 2, 64, 2, 1 | 128);
    DGV("448x128 w4x2 bk64 ns2 prio ntst xrow", 448, 128, 4, 2, 64, 2, 1 | 2 | 128);
    WGV("256x224 w4x2 bk64 ns2", 9, 256, 224, 4, 2, 64, 2);
    std::vector<std::vector<float>> ms(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) {  // warm-up + correctness
        if (v.run(s) != FI_OK) { fprintf(stderr, "%s: %s\n", v.name.c_str(), fi_last_error()); return 1; }
    }
    CK(hipStreamSynchronize(s));
    // bit-exact comparison with the group's first variant (runs in creation order above, so
    // buffer 1 holds the LAST variant of each group: compare each one right after running it)
    for (size_t i = 0; i < vs.size(); ++i) {
        if (vs[i].out == nullptr) continue;
        bool first = true;
        for (size_t j = 0; j < i; ++j) first = first && vs[j].group != vs[i].group;
        if (first) continue;
        size_t g0 = 0;
        while (vs[g0].group != vs[i].group) ++g0;
        CK(vs[i].run(s) == FI_OK ? hipSuccess : hipErrorUnknown);
        CK(hipStreamSynchronize(s));
        const size_t n = vs[i].out_bytes;
        const size_t cmp = std::min(n, (size_t)64 << 20);
        std::vector<char> a(cmp), b(cmp);
        for (int part = 0; part < 2; ++part) {
            const size_t off = part ? n - cmp : 0;
            CK(hipMemcpy(a.data(), (char*)vs[g0].out + off, cmp, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), (char*)vs[i].out + off, cmp, hipMemcpyDeviceToHost));
            if (memcmp(a.data(), b.data(), cmp) != 0) {
                size_t k = 0;
                while (a[k] == b[k]) ++k;
                printf("MISMATCH %s vs %s (part %d, first byte %zu)\n", vs[i].name.c_str(), vs[g0].name.c_str(), part, off + k);
            }
        }
    }
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) vs[i].run(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / reps);
        }
        printf("round %d done\n", r);
        fflush(stdout);
    }
    for (size_t i = 0; i < vs.size(); ++i) {
        std::vector<float> v = ms[i];
        std::sort(v.begin(), v.end());
        printf("%-34s median %.4f ms  min %.4f ms  %.3f PF/s\n", vs[i].name.c_str(), v[v.size() / 2], v[0],
               vs[i].flops / (v[v.size() / 2] * 1e-3) / 1e15);
    }
    return 0;
}
