// learner.cpp -- fi_learner: one device learner per player, behind the C ABI of
// include/fi_learner.h. Replaces the body of Learner::trainModel
// (reference include/freeimpala/learner.h:32-49): ingest -> policy forward -> V-trace +
// loss + analytic grads -> policy backward -> [RCCL all-reduce over xGMI] -> optimizer ->
// new parameter version (published through ModelManager::updateModel by the C++ caller,
// reference data_structures.h:441-451).
//
// Everything runs on one HIP stream per handle; no global mutable state, so handles of
// different players may step concurrently from different threads (reference learner.h:
// 158-163 runs one worker thread per player).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "atari.h"
#include "fi_common.h"
#include "kernels.h"

namespace fi {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace fi

using namespace fi;

struct fi_learner {
    fi_learner_config cfg{};
    int dev = 0;
    hipStream_t stream = nullptr;
    int T = 0, B = 0, A = 0, D = 0, H = 0;
    int rows = 0, TB = 0;
    size_t nparams = 0;
    // parameters / optimizer
    float* params = nullptr;
    float* grads = nullptr;
    float* opt_m = nullptr;
    float* opt_v = nullptr;
    // batch (time-major SoA)
    float* obs = nullptr;
    uint8_t* frames = nullptr;
    float* mu = nullptr;
    int32_t* act = nullptr;
    float* rew = nullptr;
    float* disc = nullptr;
    // network / loss tensors
    float* h1 = nullptr;  // MLP
    float* h2 = nullptr;
    float* dz1 = nullptr;
    float* dz2 = nullptr;
    float* logits = nullptr;
    float* values = nullptr;
    float* vs = nullptr;
    float* pg_adv = nullptr;
    float* dlogits = nullptr;
    float* dvalue = nullptr;
    double* small = nullptr;  // [0..2] losses, [3] grad sqnorm, [8..] sqnorm partials
    int* bad = nullptr;       // actions outside [0, A) in the current step's batch
    void* vt_ws = nullptr;
    size_t vt_ws_bytes = 0;
    float* slab = nullptr;
    size_t slab_floats = 0;
    int splits = 1;
    AtariNet* atari = nullptr;
    // host entry staging, double-buffered on both sides of PCIe: the host copy of batch k+1
    // into pinned2[s] and its H2D into rec_slot[s] (on copy_stream) overlap the device step
    // of batch k (fi_learner_step_async). h2d_done[s] marks the end of the H2D that reads
    // pinned2[s] / writes rec_slot[s]; ingest_done[s] the end of the ingest kernel that reads
    // rec_slot[s].
    char* pinned2[2] = {nullptr, nullptr};
    char* rec_slot[2] = {nullptr, nullptr};
    hipEvent_t h2d_done[2] = {nullptr, nullptr};
    hipEvent_t ingest_done[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr;
    int stage = 0;
    int cur = 0;             // slot the next run_step ingests from
    int acquired = -1;       // slot handed out by acquire_slot and not yet submitted
    bool in_flight = false;  // an async step was enqueued and not yet waited for
    size_t rec_bytes = 0;
    size_t rec_entry_bytes = 0;
    // data parallel
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    // bucketed gradient all-reduce: buckets start on comm_stream as the backward finalises
    // them (reverse layer order); the optimizer waits for the last one (comm_done)
    hipStream_t comm_stream = nullptr;
    std::vector<hipEvent_t> bucket_ev;
    hipEvent_t comm_done = nullptr;
    hipEvent_t bad_ready = nullptr;  // orders the reject-flag all-reduce when no bucket ran
    int buckets = 0;  // buckets issued in the last step (introspection)
    // bookkeeping
    uint64_t version = 0;
    int step_count = 0;
    bool profiling = false;
    hipEvent_t ev[FI_PHASE_COUNT + 1] = {};
    hipEvent_t ev_a = nullptr, ev_b = nullptr;
    double phase_sum[FI_PHASE_COUNT] = {};
    int phase_steps = 0;
    // per-launch tags (profiling mode): event pairs consumed in launch order each step
    std::vector<hipEvent_t> tag_ev;
    std::vector<const char*> tag_name;
    int tag_used = 0;
    std::vector<std::pair<std::string, std::pair<double, int>>> tag_sum;
    std::vector<void*> allocs;
};

static constexpr int kSqParts = 512;

static int dalloc(fi_learner* l, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(FI_ERR_OOM, std::string("hipMalloc(") + std::to_string(bytes) + "): " +
                                    hipGetErrorString(e));
    }
    l->allocs.push_back(*p);
    return FI_OK;
}

template <typename T>
static int dalloc_n(fi_learner* l, T** p, size_t n) {
    return dalloc(l, (void**)p, n * sizeof(T));
}

// ------------------------------------------------------------------ parameters
static uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Glorot-uniform weights (U(-l, l), l = sqrt(6/(fan_in+fan_out))), zero biases.
static void glorot(std::vector<float>& p, size_t off, size_t n, int fan_in, int fan_out,
                   uint64_t& st) {
    const double lim = std::sqrt(6.0 / (double)(fan_in + fan_out));
    for (size_t i = 0; i < n; ++i) {
        const double u = (double)(splitmix64(st) >> 11) * (1.0 / 9007199254740992.0);
        p[off + i] = (float)((2.0 * u - 1.0) * lim);
    }
}

static void init_mlp_params(const fi_learner* l, std::vector<float>& p) {
    const int D = l->D, H = l->H, O = l->A + 1;
    p.assign(l->nparams, 0.f);
    uint64_t st = l->cfg.seed;
    size_t o = 0;
    glorot(p, o, (size_t)D * H, D, H, st); o += (size_t)D * H + H;
    glorot(p, o, (size_t)H * H, H, H, st); o += (size_t)H * H + H;
    glorot(p, o, (size_t)H * O, H, O, st);
}

// ------------------------------------------------------------------ lifecycle
extern "C" int fi_abi_version(void) { return FI_ABI_VERSION; }
extern "C" const char* fi_last_error(void) { return fi::g_err.c_str(); }

extern "C" void fi_learner_config_init(fi_learner_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->struct_size = sizeof(*c);
    c->arch = FI_ARCH_MLP;
    c->seq_len = 100;
    c->batch = 32;
    c->num_actions = 18;
    c->obs_dim = 128;
    c->hidden = 256;
    c->optimizer = FI_OPT_ADAM;
    c->publish_dtype = FI_PUBLISH_FP32;
    c->device = 0;
    c->gamma = 0.99f;
    c->hp = fi_vtrace_hparams{1.f, 1.f, 1.f, 1.f, 0.5f, 0.01f};
    c->lr = 5e-4f;
    c->beta1 = 0.9f;
    c->beta2 = 0.999f;
    c->eps = 1e-8f;
    c->max_grad_norm = 40.f;
    c->seed = 1;
}

static void destroy(fi_learner* l) {
    if (!l) return;
    if (l->stream) hipStreamSynchronize(l->stream);
    if (l->copy_stream) hipStreamSynchronize(l->copy_stream);
    if (l->comm) ncclCommDestroy(l->comm);
    for (hipEvent_t e : l->bucket_ev) hipEventDestroy(e);
    if (l->comm_done) hipEventDestroy(l->comm_done);
    if (l->bad_ready) hipEventDestroy(l->bad_ready);
    if (l->comm_stream) hipStreamDestroy(l->comm_stream);
    atari_destroy(l->atari);
    for (void* p : l->allocs) hipFree(p);
    for (int i = 0; i < 2; ++i) {
        if (l->pinned2[i]) hipHostFree(l->pinned2[i]);
        if (l->h2d_done[i]) hipEventDestroy(l->h2d_done[i]);
        if (l->ingest_done[i]) hipEventDestroy(l->ingest_done[i]);
    }
    for (auto& e : l->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : l->tag_ev)
        if (e) hipEventDestroy(e);
    if (l->ev_a) hipEventDestroy(l->ev_a);
    if (l->ev_b) hipEventDestroy(l->ev_b);
    if (l->stream) hipStreamDestroy(l->stream);
    if (l->copy_stream) hipStreamDestroy(l->copy_stream);
    delete l;
}

extern "C" void fi_learner_destroy(fi_learner* l) {
    if (!l) return;
    hipSetDevice(l->dev);
    destroy(l);
}

static int create(const fi_learner_config* cfg, fi_learner** out) {
    FI_REQUIRE(cfg && out, "create: null argument");
    FI_REQUIRE(cfg->struct_size == sizeof(fi_learner_config), "create: struct_size mismatch");
    FI_REQUIRE(cfg->seq_len >= 1 && cfg->batch >= 1, "create: T and B must be >= 1");
    FI_REQUIRE(cfg->num_actions >= 2 && cfg->num_actions <= 64, "create: 2 <= A <= 64");
    FI_REQUIRE(cfg->arch == FI_ARCH_MLP || cfg->arch == FI_ARCH_ATARI, "create: unknown arch");
    FI_REQUIRE(cfg->optimizer == FI_OPT_ADAM || cfg->optimizer == FI_OPT_SGD, "create: optimizer");
    if (cfg->arch == FI_ARCH_MLP)
        FI_REQUIRE(cfg->obs_dim >= 1 && cfg->obs_dim <= 128 && cfg->hidden >= 1 && cfg->hidden <= 4096,
                   "create: MLP needs 1 <= obs_dim <= 128 (record schema), hidden <= 4096");
    int ndev = 0;
    FI_HIP_CHECK(hipGetDeviceCount(&ndev));
    FI_REQUIRE(cfg->device >= 0 && cfg->device < ndev, "create: no such HIP device");
    FI_HIP_CHECK(hipSetDevice(cfg->device));

    fi_learner* l = new (std::nothrow) fi_learner();
    FI_REQUIRE(l, "create: out of host memory");
    *out = nullptr;
    struct Guard {
        fi_learner* l;
        bool ok = false;
        ~Guard() { if (!ok) destroy(l); }
    } guard{l};

    l->cfg = *cfg;
    l->dev = cfg->device;
    l->T = cfg->seq_len;
    l->B = cfg->batch;
    l->A = cfg->num_actions;
    l->D = cfg->obs_dim;
    l->H = cfg->hidden;
    l->rows = (l->T + 1) * l->B;
    l->TB = l->T * l->B;
    FI_HIP_CHECK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
    for (auto& e : l->ev) FI_HIP_CHECK(hipEventCreate(&e));
    FI_HIP_CHECK(hipEventCreate(&l->ev_a));
    FI_HIP_CHECK(hipEventCreate(&l->ev_b));

    const size_t rows = l->rows, TB = l->TB;
    const int A = l->A;
    std::vector<float> init;
    if (cfg->arch == FI_ARCH_MLP) {
        const int D = l->D, H = l->H, O = A + 1;
        l->nparams = (size_t)D * H + H + (size_t)H * H + H + (size_t)H * O + O;
        init_mlp_params(l, init);
        FI_TRY(dalloc_n(l, &l->obs, rows * D));
        FI_TRY(dalloc_n(l, &l->h1, rows * H));
        FI_TRY(dalloc_n(l, &l->h2, rows * H));
        FI_TRY(dalloc_n(l, &l->dz1, rows * H));
        FI_TRY(dalloc_n(l, &l->dz2, rows * H));
        // weight-gradient R-slices: 384 at R = 413,696 gives the K = 128 layer 1,536 workgroups
        // (6 per CU, the kernel's occupancy) -- with 128 its 512 workgroups left the CUs
        // latency-bound (wgrad_l1 0.44 -> 0.29 ms, wgrad_l2 0.60 -> 0.54 ms; 512 slices measured
        // slower: the slab sums grow)
        l->splits = (int)std::min<size_t>(384, std::max<size_t>(1, rows / 1024));
        const size_t big = std::max<size_t>((size_t)D * H, (size_t)H * H);
        l->slab_floats = (size_t)l->splits * (big + 4096);  // wgrad slabs | bias colsum slabs
        FI_TRY(dalloc_n(l, &l->slab, l->slab_floats));
    } else {
        l->atari = atari_create(l->B, l->T, A);
        FI_REQUIRE(l->atari, "create: Atari net allocation failed: " + std::string(fi_last_error()));
        l->nparams = atari_param_count(A);
        atari_init_params(A, cfg->seed, init);
        FI_TRY(dalloc_n(l, &l->frames, rows * AtariNet::kFrameBytes));
    }
    FI_TRY(dalloc_n(l, &l->params, l->nparams));
    FI_TRY(dalloc_n(l, &l->grads, l->nparams));
    FI_TRY(dalloc_n(l, &l->opt_m, l->nparams));
    FI_TRY(dalloc_n(l, &l->opt_v, l->nparams));
    FI_TRY(dalloc_n(l, &l->mu, TB * A));
    FI_TRY(dalloc_n(l, &l->act, TB));
    FI_TRY(dalloc_n(l, &l->rew, TB));
    FI_TRY(dalloc_n(l, &l->disc, TB));
    FI_TRY(dalloc_n(l, &l->logits, rows * A));
    FI_TRY(dalloc_n(l, &l->values, rows));
    FI_TRY(dalloc_n(l, &l->vs, TB));
    FI_TRY(dalloc_n(l, &l->pg_adv, TB));
    FI_TRY(dalloc_n(l, &l->dlogits, TB * A));
    FI_TRY(dalloc_n(l, &l->dvalue, rows));
    FI_TRY(dalloc_n(l, &l->small, 8 + kSqParts));
    FI_TRY(dalloc_n(l, &l->bad, 64));
    FI_HIP_CHECK(hipMemsetAsync(l->bad, 0, 64 * sizeof(int), l->stream));
    l->vt_ws_bytes = vtrace_workspace_bytes(l->T, l->B, A);
    FI_TRY(dalloc(l, &l->vt_ws, l->vt_ws_bytes));

    FI_HIP_CHECK(hipMemcpyAsync(l->params, init.data(), l->nparams * sizeof(float),
                                hipMemcpyHostToDevice, l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->opt_m, 0, l->nparams * sizeof(float), l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->opt_v, 0, l->nparams * sizeof(float), l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->grads, 0, l->nparams * sizeof(float), l->stream));
    // a defined (all-zero) batch until the first synth/step
    if (l->obs) FI_HIP_CHECK(hipMemsetAsync(l->obs, 0, rows * l->D * sizeof(float), l->stream));
    if (l->frames) FI_HIP_CHECK(hipMemsetAsync(l->frames, 0, rows * AtariNet::kFrameBytes, l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->mu, 0, TB * A * sizeof(float), l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->act, 0, TB * sizeof(int32_t), l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->rew, 0, TB * sizeof(float), l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->disc, 0, TB * sizeof(float), l->stream));
    if (l->atari) FI_TRY(atari_sync_weights(l->atari, l->params, l->stream));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    guard.ok = true;
    *out = l;
    return FI_OK;
}

extern "C" int fi_learner_create(const fi_learner_config* cfg, fi_learner** out) {
    try {
        return create(cfg, out);
    } catch (const std::exception& e) {
        return fail(FI_ERR_OOM, std::string("create: ") + e.what());
    }
}

extern "C" size_t fi_learner_param_count(const fi_learner* l) { return l ? l->nparams : 0; }
extern "C" size_t fi_learner_param_bytes(const fi_learner* l) {
    if (!l) return 0;
    return l->nparams * (l->cfg.publish_dtype == FI_PUBLISH_BF16 ? 2 : 4);
}
extern "C" size_t fi_learner_entry_bytes(const fi_learner* l) {
    return l ? (size_t)(l->T + 1) * FI_RECORD_BYTES : 0;
}
extern "C" void* fi_learner_stream(fi_learner* l) { return l ? (void*)l->stream : nullptr; }
extern "C" int fi_learner_sync(fi_learner* l) {
    FI_REQUIRE(l, "sync: null");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    return FI_OK;
}

// ------------------------------------------------------------------ the step
static void mark(fi_learner* l, int phase) {
    if (l->profiling) hipEventRecord(l->ev[phase], l->stream);
}

// RAII launch tag: records an event pair around the launches in its scope when profiling.
struct Tag {
    fi_learner* l;
    int idx = -1;
    Tag(fi_learner* l_, const char* name) : l(l_) {
        if (!l->profiling) return;
        if ((size_t)(2 * l->tag_used + 2) > l->tag_ev.size()) {
            hipEvent_t a = nullptr, b = nullptr;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
            l->tag_ev.push_back(a);
            l->tag_ev.push_back(b);
            l->tag_name.push_back(nullptr);
        }
        idx = l->tag_used++;
        l->tag_name[idx] = name;
        (void)hipEventRecord(l->tag_ev[2 * idx], l->stream);
    }
    ~Tag() {
        if (idx >= 0) (void)hipEventRecord(l->tag_ev[2 * idx + 1], l->stream);
    }
};

// the same events, driven from inside the Atari net's launch sequence
struct LearnerTagger : KernelTagger {
    fi_learner* l;
    std::vector<Tag*> open;
    explicit LearnerTagger(fi_learner* l_) : l(l_) {}
    void begin(const char* name) override { open.push_back(new Tag(l, name)); }
    void end() override {
        delete open.back();
        open.pop_back();
    }
    ~LearnerTagger() override {
        for (Tag* t : open) delete t;
    }
};

static void collect_tags(fi_learner* l) {
    for (int i = 0; i < l->tag_used; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, l->tag_ev[2 * i], l->tag_ev[2 * i + 1]) != hipSuccess) continue;
        bool found = false;
        for (auto& e : l->tag_sum)
            if (e.first == l->tag_name[i]) {
                e.second.first += ms;
                e.second.second += 1;
                found = true;
                break;
            }
        if (!found) l->tag_sum.push_back({l->tag_name[i], {ms, 1}});
    }
    l->tag_used = 0;
}

// Gradient buckets in reverse layer order: once the backward has enqueued
// the final write of grads[off, off+n), an event on the compute stream gates that bucket's
// in-place ncclAllReduce(sum) on comm_stream, so the reduction of the fc/heads gradients
// (95 % of the Atari net's bytes) overlaps the conv backward. Every rank issues the same
// buckets in the same order. Without a communicator the hook does nothing.
struct BucketAllReduce : GradReadyHook {
    fi_learner* l;
    int n = 0;
    explicit BucketAllReduce(fi_learner* l_) : l(l_) {}
    int ready(size_t off, size_t count) override {
        if (!l->comm || count == 0) return FI_OK;
        if ((size_t)n >= l->bucket_ev.size()) {
            hipEvent_t e;
            FI_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            l->bucket_ev.push_back(e);
        }
        FI_HIP_CHECK(hipEventRecord(l->bucket_ev[n], l->stream));
        FI_HIP_CHECK(hipStreamWaitEvent(l->comm_stream, l->bucket_ev[n], 0));
        ++n;
        ncclResult_t r = ncclAllReduce(l->grads + off, l->grads + off, count, ncclFloat, ncclSum,
                                       l->comm, l->comm_stream);
        if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        return FI_OK;
    }
    // The reject decision is agreed before anything is applied: after the last bucket the
    // int counter of out-of-range actions (written by ingest and the V-trace kernel, both
    // ordered before the first bucket's event) is summed over the ranks on the same stream,
    // so the optimizer of EVERY replica sees the group's count and all of them skip the
    // update together -- a shard's gradient from clamped actions is in the summed gradient,
    // and no replica may apply it (reference log-and-skip: data_structures.h:420-421,
    // agent.h:88-91). The compute stream then waits for every bucket before the optimizer
    // reads the gradients.
    int join() {
        l->buckets = n;
        if (!l->comm) return FI_OK;
        if (n == 0) {  // a backward without buckets still has to agree on the reject flag
            FI_HIP_CHECK(hipEventRecord(l->bad_ready, l->stream));
            FI_HIP_CHECK(hipStreamWaitEvent(l->comm_stream, l->bad_ready, 0));
        }
        ncclResult_t r = ncclAllReduce(l->bad, l->bad, 1, ncclInt32, ncclSum, l->comm, l->comm_stream);
        if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclAllReduce(reject flag): ") + ncclGetErrorString(r));
        FI_HIP_CHECK(hipEventRecord(l->comm_done, l->comm_stream));
        FI_HIP_CHECK(hipStreamWaitEvent(l->stream, l->comm_done, 0));
        return FI_OK;
    }
};

static int mlp_forward(fi_learner* l) {
    const int D = l->D, H = l->H, A = l->A;
    const float* W1 = l->params;
    const float* b1 = W1 + (size_t)D * H;
    const float* W2 = b1 + H;
    const float* b2 = W2 + (size_t)H * H;
    const float* Wh = b2 + H;
    const float* bh = Wh + (size_t)H * (A + 1);
    { Tag t(l, "mlp_fwd_l1"); FI_TRY(f32_linear_fwd(l->obs, l->rows, D, W1, b1, H, true, l->h1, l->stream)); }
    { Tag t(l, "mlp_fwd_l2"); FI_TRY(f32_linear_fwd(l->h1, l->rows, H, W2, b2, H, true, l->h2, l->stream)); }
    { Tag t(l, "mlp_fwd_heads"); FI_TRY(f32_heads_fwd(l->h2, l->rows, H, Wh, bh, A, l->logits, l->values, l->stream)); }
    return FI_OK;
}

static int wgrad(fi_learner* l, const char* tag, const float* X, int I, const float* dY, int N,
                 float* gW, float* gb) {
    float* cs = l->slab + l->slab_floats - (size_t)l->splits * 4096;
    { Tag t(l, tag); FI_TRY(f32_linear_wgrad_partial(X, l->rows, I, dY, N, l->splits, l->slab, cs, l->stream)); }
    { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(l->slab, l->splits, (size_t)I * N, gW, l->stream)); }
    { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(cs, l->splits, (size_t)N, gb, l->stream)); }
    return FI_OK;
}

static int mlp_backward(fi_learner* l, GradReadyHook* gr) {
    const int D = l->D, H = l->H, A = l->A, O = A + 1;
    const float* W2 = l->params + (size_t)D * H + H;
    const float* Wh = W2 + (size_t)H * H + H;
    float* gW1 = l->grads;
    float* gb1 = gW1 + (size_t)D * H;
    float* gW2 = gb1 + H;
    float* gb2 = gW2 + (size_t)H * H;
    float* gWh = gb2 + H;
    float* gbh = gWh + (size_t)H * O;
    HeadsGrad g{l->dlogits, l->dvalue, l->rows, l->TB, A};
    float* cs = l->slab + l->slab_floats - (size_t)l->splits * 4096;
    if (f32_heads_bwd_fused_supported(H, A) && (size_t)kHeadsFusedGrid * (H * O + O) <= l->slab_floats) {
        // both heads gradients in one pass over h2 (weight-gradient slabs, then dz2)
        float* hcs = l->slab + (size_t)kHeadsFusedGrid * H * O;
        { Tag t(l, "mlp_heads_bwd"); FI_TRY(f32_heads_bwd_fused(g, l->h2, Wh, H, l->dz2, l->slab, hcs, kHeadsFusedGrid, l->stream)); }
        { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(l->slab, kHeadsFusedGrid, (size_t)H * O, gWh, l->stream)); }
        { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(hcs, kHeadsFusedGrid, (size_t)O, gbh, l->stream)); }
        FI_TRY(gr->ready((size_t)(gWh - l->grads), (size_t)H * O + O));
    } else {
        { Tag t(l, "mlp_wgrad_heads"); FI_TRY(f32_heads_wgrad_partial(l->h2, H, g, l->splits, l->slab, cs, l->stream)); }
        { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(l->slab, l->splits, (size_t)H * O, gWh, l->stream)); }
        { Tag t(l, "reduce_slabs"); FI_TRY(reduce_slabs(cs, l->splits, (size_t)O, gbh, l->stream)); }
        FI_TRY(gr->ready((size_t)(gWh - l->grads), (size_t)H * O + O));
        { Tag t(l, "mlp_dgrad_heads"); FI_TRY(f32_heads_dgrad(g, Wh, H, l->h2, l->dz2, l->stream)); }
    }
    FI_TRY(wgrad(l, "mlp_wgrad_l2", l->h1, H, l->dz2, H, gW2, gb2));
    FI_TRY(gr->ready((size_t)(gW2 - l->grads), (size_t)H * H + H));
    { Tag t(l, "mlp_dgrad_l2"); FI_TRY(f32_linear_dgrad(l->dz2, l->rows, H, W2, H, l->h1, l->dz1, l->stream)); }
    FI_TRY(wgrad(l, "mlp_wgrad_l1", l->obs, D, l->dz1, H, gW1, gb1));
    FI_TRY(gr->ready(0, (size_t)D * H + H));
    return FI_OK;
}

// A batch with actions outside [0, A) (a corrupt record, or actors configured with another
// --num-actions) is rejected: the optimizer kernels see the device counter and leave the
// parameters and moments untouched, and the step reports FI_ERR_INVALID once it has
// completed (the oracle rejects the same batch, oracle/impala_oracle.c). Called after the
// stream has been synchronised.
// The flag words l->bad (csrc/misc.hip, skip_update): [0] out-of-range actions of the current
// step (all-reduced), [1] its gradient norm was NaN / Inf (taken from the all-reduced gradient,
// so every replica sees the same value), [2] updates skipped since the last check, [3] their
// reasons (1 = actions, 2 = non-finite). Every replica skips the same updates. A synchronous
// step checks its own; fi_learner_wait checks every step enqueued since the last check, so a
// skipped step behind others still in flight is reported, and the version counts applied
// updates only (an enqueued step behind a skipped one keeps the Adam step number it was given).
static int check_rejected(fi_learner* l) {
    int bad[4] = {0, 0, 0, 0};
    FI_HIP_CHECK(hipMemcpy(bad, l->bad, sizeof(bad), hipMemcpyDeviceToHost));
    const int skipped = bad[2], why = bad[3];
    if (skipped == 0) return FI_OK;
    FI_HIP_CHECK(hipMemsetAsync(l->bad + 2, 0, 2 * sizeof(int), l->stream));  // ordered before the next step
    l->step_count -= skipped;
    l->version -= (uint64_t)skipped;
    const std::string n = skipped > 1 ? std::to_string(skipped) + " of the enqueued updates skipped" : "update skipped";
    if (!(why & 1))
        return fail(FI_ERR_NONFINITE, "step: the gradient norm is not finite (NaN / Inf in the batch's losses or "
                                      "gradients); " + n + ", parameters unchanged");
    const std::string acts = bad[0] > 0 ? std::to_string(bad[0]) + " action(s)" : "action(s)";
    if (l->comm && l->nranks > 1)
        return fail(FI_ERR_INVALID, "step: " + acts + " outside [0, " + std::to_string(l->A) +
                                        ") in the data-parallel group's batch (all-reduced reject flag); batch "
                                        "rejected on every replica, " + n + ", parameters unchanged");
    return fail(FI_ERR_INVALID, "step: " + acts + " outside [0, " + std::to_string(l->A) + ") in the batch; batch "
                                "rejected, " + n + ", parameters unchanged");
}

static void fill_stats(fi_learner* l, fi_step_stats* out) {
    double h[4];
    if (hipMemcpy(h, l->small, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        for (double& x : h) x = std::nan("");
    const fi_vtrace_hparams& hp = l->cfg.hp;
    out->pg_loss = h[0];
    out->baseline_loss = h[1];
    out->entropy_loss = h[2];
    out->total_loss = h[0] + hp.baseline_cost * h[1] + hp.entropy_cost * h[2];
    out->grad_norm = std::sqrt(h[3]);
    out->version = l->version;
    out->step_ms = 0.f;
}

static int run_step(fi_learner* l, bool have_host_batch, fi_step_stats* out) {
    const bool sync = out != nullptr || l->profiling;
    l->tag_used = 0;
    if (out) FI_HIP_CHECK(hipEventRecord(l->ev_a, l->stream));
    mark(l, FI_PHASE_INGEST);
    FI_HIP_CHECK(hipMemsetAsync(l->bad, 0, sizeof(int), l->stream));
    if (have_host_batch) {
        const int s = l->cur;
        FI_HIP_CHECK(hipStreamWaitEvent(l->stream, l->h2d_done[s], 0));
        {
            Tag t(l, "ingest");
            FI_TRY(ingest_launch(l->rec_slot[s], l->T, l->B, l->A, l->D, l->rec_entry_bytes,
                                 l->cfg.arch == FI_ARCH_MLP ? l->obs : nullptr, l->mu, l->act,
                                 l->rew, l->disc, l->stream, l->bad));
        }
        FI_HIP_CHECK(hipEventRecord(l->ingest_done[s], l->stream));
    }
    mark(l, FI_PHASE_FORWARD);
    if (l->cfg.arch == FI_ARCH_MLP) FI_TRY(mlp_forward(l));
    else {
        LearnerTagger tg(l);
        FI_TRY(atari_forward(l->atari, l->frames, l->logits, l->values, l->stream, l->profiling ? &tg : nullptr));
    }
    mark(l, FI_PHASE_VTRACE);
    int vt_nblk = 0;
    {
        // scan + loss + gradients; the loss partials are summed by the gradient-norm kernel
        Tag t(l, "vtrace");
        FI_TRY(vtrace_launch(0, l->T, l->B, l->A, l->logits, l->mu, l->act, l->rew, l->disc,
                             l->values, l->cfg.hp, l->vs, l->pg_adv, l->dlogits, l->dvalue,
                             l->small, l->vt_ws, l->vt_ws_bytes, l->stream, false, &vt_nblk,
                             l->bad));
    }
    mark(l, FI_PHASE_BACKWARD);
    BucketAllReduce bar(l);
    if (l->cfg.arch == FI_ARCH_MLP) FI_TRY(mlp_backward(l, &bar));
    else {
        LearnerTagger tg(l);
        FI_TRY(atari_backward(l->atari, l->frames, l->dlogits, l->dvalue, l->grads, l->stream,
                              l->profiling ? &tg : nullptr, &bar));
    }
    // the "allreduce" phase is the exposed tail: the wait for the buckets still in flight
    // when the backward has finished
    mark(l, FI_PHASE_ALLREDUCE);
    {
        Tag t(l, "allreduce_wait");
        FI_TRY(bar.join());
    }
    mark(l, FI_PHASE_OPTIMIZER);
    {
        Tag t(l, "grad_norm");  // + the V-trace loss sums (losses land in small[0..2])
        FI_TRY(grad_sqnorm(l->grads, l->nparams, l->small + 8, kSqParts, l->small + 3, l->stream,
                           vtrace_partials(l->vt_ws), vt_nblk, l->small, l->bad + 1));
    }
    const int step = l->step_count + 1;
    const double bc1 = 1.0 - std::pow((double)l->cfg.beta1, step);
    const double bc2 = 1.0 - std::pow((double)l->cfg.beta2, step);
    {
        Tag t(l, "optimizer");
        FI_TRY(optimizer_step(l->cfg.optimizer, l->params, l->grads, l->opt_m, l->opt_v, l->nparams,
                              l->cfg.lr, l->cfg.beta1, l->cfg.beta2, l->cfg.eps, bc1, bc2,
                              l->small + 3, l->cfg.max_grad_norm, l->stream, l->bad));
    }
    if (l->atari) {
        Tag t(l, "weights_bf16");
        FI_TRY(atari_sync_weights(l->atari, l->params, l->stream));
    }
    mark(l, FI_PHASE_COUNT);
    if (out) FI_HIP_CHECK(hipEventRecord(l->ev_b, l->stream));
    l->step_count = step;
    l->version++;
    if (sync) {
        FI_HIP_CHECK(hipStreamSynchronize(l->stream));
        if (l->profiling) {
            for (int p = 0; p < FI_PHASE_COUNT; ++p) {
                float ms = 0.f;
                FI_HIP_CHECK(hipEventElapsedTime(&ms, l->ev[p], l->ev[p + 1]));
                l->phase_sum[p] += ms;
            }
            l->phase_steps++;
            collect_tags(l);
        }
    }
    if (out) {
        FI_TRY(check_rejected(l));
        fill_stats(l, out);
        float ms = 0.f;
        FI_HIP_CHECK(hipEventElapsedTime(&ms, l->ev_a, l->ev_b));
        out->step_ms = ms;
    }
    return FI_OK;
}

extern "C" int fi_learner_step_resident(fi_learner* l, fi_step_stats* out) {
    FI_REQUIRE(l, "step: null learner");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    try {
        return run_step(l, false, out);
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("step: ") + e.what());
    }
}

static void parallel_copy(char* dst, const void* const* entries, size_t n, size_t entry_bytes,
                          size_t stride) {
    const size_t total = n * entry_bytes;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>({n, (size_t)std::min(hw, 16u), 1 + total / (64u << 20)});
    auto work = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) std::memcpy(dst + i * stride, entries[i], entry_bytes);
    };
    if (nt <= 1) {
        work(0, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + nt - 1) / nt;
    for (size_t t = 0; t < nt; ++t) {
        const size_t lo = t * per, hi = std::min(n, lo + per);
        if (lo < hi) th.emplace_back(work, lo, hi);
    }
    for (auto& t : th) t.join();
}

// Host staging, double-buffered: acquire_slot() hands out the next pinned buffer once the
// H2D that last read it is done; submit_slot() enqueues its H2D on the copy stream (after the
// ingest that last read the device slot) and makes it the batch the next run_step ingests.
static int ensure_staging(fi_learner* l) {
    FI_REQUIRE(l->cfg.arch == FI_ARCH_MLP,
               "step: host trajectory records carry <=128-float observations (MLP); the Atari "
               "config is device-synthetic (fi_learner_synth_batch + fi_learner_step_resident)");
    const size_t need = (size_t)(l->T + 1) * FI_RECORD_BYTES;
    const size_t bytes = (size_t)l->B * need;
    if (bytes <= l->rec_bytes) return FI_OK;
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    if (l->copy_stream) FI_HIP_CHECK(hipStreamSynchronize(l->copy_stream));
    else FI_HIP_CHECK(hipStreamCreateWithFlags(&l->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        if (l->pinned2[i]) hipHostFree(l->pinned2[i]);
        l->pinned2[i] = nullptr;
        if (l->rec_slot[i]) {
            hipFree(l->rec_slot[i]);
            l->allocs.erase(std::find(l->allocs.begin(), l->allocs.end(), (void*)l->rec_slot[i]));
        }
        l->rec_slot[i] = nullptr;
    }
    l->rec_bytes = 0;
    for (int i = 0; i < 2; ++i) {
        FI_HIP_CHECK(hipHostMalloc((void**)&l->pinned2[i], bytes, hipHostMallocDefault));
        FI_TRY(dalloc(l, (void**)&l->rec_slot[i], bytes));
        if (!l->h2d_done[i]) FI_HIP_CHECK(hipEventCreateWithFlags(&l->h2d_done[i], hipEventDisableTiming));
        if (!l->ingest_done[i]) FI_HIP_CHECK(hipEventCreateWithFlags(&l->ingest_done[i], hipEventDisableTiming));
        FI_HIP_CHECK(hipEventRecord(l->h2d_done[i], l->copy_stream));
        FI_HIP_CHECK(hipEventRecord(l->ingest_done[i], l->stream));
    }
    l->rec_bytes = bytes;
    l->rec_entry_bytes = need;
    return FI_OK;
}

static bool stage_timing() {
    static const bool on = std::getenv("FI_STAGE_TIMING") != nullptr;
    return on;
}

static int acquire_slot(fi_learner* l, int* slot) {
    FI_TRY(ensure_staging(l));
    if (l->acquired < 0) {
        const auto t0 = std::chrono::steady_clock::now();
        // pinned2[s] is free once the H2D that read it (two steps ago) is done
        FI_HIP_CHECK(hipEventSynchronize(l->h2d_done[l->stage]));
        l->acquired = l->stage;
        l->stage ^= 1;
        if (stage_timing())
            std::fprintf(stderr, "[fi stage] slot %d wait %.3f ms\n", l->acquired,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    *slot = l->acquired;
    return FI_OK;
}

static int submit_slot(fi_learner* l) {
    FI_REQUIRE(l->acquired >= 0, "step_staged: no staging slot acquired (fi_learner_acquire_staging)");
    const int s = l->acquired;
    // the device slot is rewritten after the ingest kernel of two steps ago has read it; the
    // copy runs on its own stream, beside the device step of the previous batch
    FI_HIP_CHECK(hipStreamWaitEvent(l->copy_stream, l->ingest_done[s], 0));
    FI_HIP_CHECK(hipMemcpyAsync(l->rec_slot[s], l->pinned2[s], l->rec_bytes, hipMemcpyHostToDevice,
                                l->copy_stream));
    FI_HIP_CHECK(hipEventRecord(l->h2d_done[s], l->copy_stream));
    l->cur = s;
    l->acquired = -1;
    return FI_OK;
}

// stage M host entries (only their first T+1 records) through the next pinned buffer; returns
// once the host copy is done (the entries may then be freed)
static int stage_entries(fi_learner* l, const void* const* entries, size_t n_entries, size_t entry_bytes) {
    FI_REQUIRE(l && entries, "step: null argument");
    FI_REQUIRE(n_entries == (size_t)l->B, "step: n_entries must equal the configured batch");
    const size_t need = (size_t)(l->T + 1) * FI_RECORD_BYTES;
    FI_REQUIRE(entry_bytes >= need, "step: entry_bytes < (T+1)*1024");
    for (size_t i = 0; i < n_entries; ++i) FI_REQUIRE(entries[i], "step: null entry");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    int s = 0;
    FI_TRY(acquire_slot(l, &s));
    const auto t0 = std::chrono::steady_clock::now();
    parallel_copy(l->pinned2[s], entries, n_entries, need, need);
    if (stage_timing()) {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "[fi stage] slot %d copy %.3f ms (%.1f GB/s)\n", s, ms, l->rec_bytes / 1e6 / ms);
    }
    return submit_slot(l);
}

// a synchronous step: returns when the device step has completed, statistics or not
static int step_and_wait(fi_learner* l, fi_step_stats* out) {
    l->in_flight = false;
    FI_TRY(run_step(l, true, out));
    if (!out) {
        FI_HIP_CHECK(hipStreamSynchronize(l->stream));
        FI_TRY(check_rejected(l));
    }
    return FI_OK;
}

extern "C" int fi_learner_step(fi_learner* l, const void* const* entries, size_t n_entries,
                               size_t entry_bytes, fi_step_stats* out) {
    try {
        FI_TRY(stage_entries(l, entries, n_entries, entry_bytes));
        return step_and_wait(l, out);
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("step: ") + e.what());
    }
}

extern "C" int fi_learner_step_async(fi_learner* l, const void* const* entries, size_t n_entries,
                                     size_t entry_bytes) {
    try {
        FI_TRY(stage_entries(l, entries, n_entries, entry_bytes));
        FI_TRY(run_step(l, true, nullptr));  // enqueued only (no stats requested: no sync)
        l->in_flight = true;
        return FI_OK;
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("step_async: ") + e.what());
    }
}

extern "C" int fi_learner_acquire_staging(fi_learner* l, void** dst, size_t* entry_stride) {
    FI_REQUIRE(l && dst, "acquire_staging: null argument");
    try {
        FI_HIP_CHECK(hipSetDevice(l->dev));
        int s = 0;
        FI_TRY(acquire_slot(l, &s));
        *dst = l->pinned2[s];
        if (entry_stride) *entry_stride = l->rec_entry_bytes;
        return FI_OK;
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("acquire_staging: ") + e.what());
    }
}

extern "C" int fi_learner_step_staged(fi_learner* l, fi_step_stats* out) {
    FI_REQUIRE(l, "step_staged: null learner");
    try {
        FI_HIP_CHECK(hipSetDevice(l->dev));
        FI_TRY(submit_slot(l));
        return step_and_wait(l, out);
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("step_staged: ") + e.what());
    }
}

extern "C" int fi_learner_step_staged_async(fi_learner* l) {
    FI_REQUIRE(l, "step_staged_async: null learner");
    try {
        FI_HIP_CHECK(hipSetDevice(l->dev));
        FI_TRY(submit_slot(l));
        FI_TRY(run_step(l, true, nullptr));
        l->in_flight = true;
        return FI_OK;
    } catch (const std::exception& e) {
        return fail(FI_ERR_STATE, std::string("step_staged_async: ") + e.what());
    }
}

extern "C" int fi_learner_wait(fi_learner* l, fi_step_stats* out) {
    FI_REQUIRE(l, "wait: null learner");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    const bool was_in_flight = l->in_flight;
    l->in_flight = false;
    if (was_in_flight) FI_TRY(check_rejected(l));
    if (out) fill_stats(l, out);  // step_ms = 0: not timed on the asynchronous path
    return FI_OK;
}

extern "C" int fi_learner_synth_batch(fi_learner* l, uint64_t seed, int32_t b_global,
                                      int32_t b_offset) {
    FI_REQUIRE(l, "synth: null learner");
    if (b_global <= 0) b_global = l->B;
    FI_REQUIRE(b_offset >= 0 && b_offset + l->B <= b_global, "synth: shard outside global batch");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    FI_TRY(synth_launch(seed, l->T, l->B, b_global, b_offset, l->A, l->D, l->cfg.gamma, l->obs, l->mu,
                        l->act, l->rew, l->disc, l->frames, l->stream));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    return FI_OK;
}

// ------------------------------------------------------------------ params
extern "C" int fi_learner_get_params_fp32(fi_learner* l, float* dst, size_t count) {
    FI_REQUIRE(l && dst && count == l->nparams, "get_params_fp32: bad arguments");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    FI_HIP_CHECK(hipMemcpyAsync(dst, l->params, count * sizeof(float), hipMemcpyDeviceToHost,
                                l->stream));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    return FI_OK;
}

static uint16_t f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

extern "C" int fi_learner_get_params(fi_learner* l, void* dst, size_t bytes, uint64_t* version) {
    FI_REQUIRE(l && dst, "get_params: null argument");
    FI_REQUIRE(bytes == fi_learner_param_bytes(l), "get_params: bytes != fi_learner_param_bytes");
    if (l->cfg.publish_dtype == FI_PUBLISH_FP32) {
        FI_TRY(fi_learner_get_params_fp32(l, (float*)dst, l->nparams));
    } else {
        std::vector<float> tmp(l->nparams);
        FI_TRY(fi_learner_get_params_fp32(l, tmp.data(), l->nparams));
        uint16_t* o = (uint16_t*)dst;
        for (size_t i = 0; i < l->nparams; ++i) o[i] = f2bf(tmp[i]);
    }
    if (version) {
        // updates skipped by steps not yet checked (asynchronous submission, reported by the
        // next fi_learner_wait) are not counted, so the published version never goes back
        int pending = 0;
        FI_HIP_CHECK(hipMemcpy(&pending, l->bad + 2, sizeof(int), hipMemcpyDeviceToHost));
        *version = l->version - (uint64_t)pending;
    }
    return FI_OK;
}

extern "C" int fi_learner_set_params(fi_learner* l, const void* src, size_t bytes,
                                     uint64_t version) {
    FI_REQUIRE(l && src, "set_params: null argument");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    std::vector<float> tmp;
    const float* p;
    if (bytes == l->nparams * 4) {
        p = (const float*)src;
    } else if (bytes == l->nparams * 2) {
        tmp.resize(l->nparams);
        const uint16_t* s = (const uint16_t*)src;
        for (size_t i = 0; i < l->nparams; ++i) {
            uint32_t u = (uint32_t)s[i] << 16;
            std::memcpy(&tmp[i], &u, 4);
        }
        p = tmp.data();
    } else {
        return fail(FI_ERR_INVALID, "set_params: size is neither fp32 nor bf16 blob");
    }
    FI_HIP_CHECK(hipMemcpyAsync(l->params, p, l->nparams * 4, hipMemcpyHostToDevice, l->stream));
    if (l->atari) FI_TRY(atari_sync_weights(l->atari, l->params, l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->bad + 2, 0, 2 * sizeof(int), l->stream));  // a new version line
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    l->version = version;
    return FI_OK;
}

// ------------------------------------------------------------------ checkpoint / resume
// State blob: header {magic, abi, arch, nparams, step_count, version} then fp32 params, Adam
// m, Adam v (little endian). Together with the published Model blob this lets a restarted
// learner continue bit-identically.
namespace {
struct StateHeader {
    uint32_t magic, abi;
    int32_t arch, step_count;
    uint64_t nparams, version;
};
constexpr uint32_t kStateMagic = 0x46495354u;  // "FIST"
}  // namespace

extern "C" size_t fi_learner_state_bytes(const fi_learner* l) {
    return l ? sizeof(StateHeader) + 3 * l->nparams * sizeof(float) : 0;
}

extern "C" int fi_learner_save_state(fi_learner* l, void* dst, size_t bytes) {
    FI_REQUIRE(l && dst, "save_state: null argument");
    FI_REQUIRE(bytes == fi_learner_state_bytes(l), "save_state: bytes != fi_learner_state_bytes");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    StateHeader h{kStateMagic, FI_ABI_VERSION, l->cfg.arch, l->step_count, l->nparams, l->version};
    char* o = (char*)dst;
    std::memcpy(o, &h, sizeof(h));
    float* f = (float*)(o + sizeof(h));
    FI_HIP_CHECK(hipMemcpyAsync(f, l->params, l->nparams * 4, hipMemcpyDeviceToHost, l->stream));
    FI_HIP_CHECK(hipMemcpyAsync(f + l->nparams, l->opt_m, l->nparams * 4, hipMemcpyDeviceToHost, l->stream));
    FI_HIP_CHECK(hipMemcpyAsync(f + 2 * l->nparams, l->opt_v, l->nparams * 4, hipMemcpyDeviceToHost, l->stream));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    return FI_OK;
}

extern "C" int fi_learner_load_state(fi_learner* l, const void* src, size_t bytes) {
    FI_REQUIRE(l && src, "load_state: null argument");
    FI_REQUIRE(bytes == fi_learner_state_bytes(l), "load_state: bytes != fi_learner_state_bytes");
    StateHeader h;
    std::memcpy(&h, src, sizeof(h));
    FI_REQUIRE(h.magic == kStateMagic && h.abi == FI_ABI_VERSION, "load_state: not a learner state blob");
    FI_REQUIRE(h.arch == l->cfg.arch && h.nparams == l->nparams, "load_state: state of a different network");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    const float* f = (const float*)((const char*)src + sizeof(h));
    FI_HIP_CHECK(hipMemcpyAsync(l->params, f, l->nparams * 4, hipMemcpyHostToDevice, l->stream));
    FI_HIP_CHECK(hipMemcpyAsync(l->opt_m, f + l->nparams, l->nparams * 4, hipMemcpyHostToDevice, l->stream));
    FI_HIP_CHECK(hipMemcpyAsync(l->opt_v, f + 2 * l->nparams, l->nparams * 4, hipMemcpyHostToDevice, l->stream));
    if (l->atari) FI_TRY(atari_sync_weights(l->atari, l->params, l->stream));
    FI_HIP_CHECK(hipMemsetAsync(l->bad + 2, 0, 2 * sizeof(int), l->stream));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    l->step_count = h.step_count;
    l->version = h.version;
    return FI_OK;
}

// ------------------------------------------------------------------ data parallel
static int ensure_comm_stream(fi_learner* l) {
    if (!l->comm_stream) FI_HIP_CHECK(hipStreamCreateWithFlags(&l->comm_stream, hipStreamNonBlocking));
    if (!l->comm_done) FI_HIP_CHECK(hipEventCreateWithFlags(&l->comm_done, hipEventDisableTiming));
    if (!l->bad_ready) FI_HIP_CHECK(hipEventCreateWithFlags(&l->bad_ready, hipEventDisableTiming));
    return FI_OK;
}

extern "C" int fi_comm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int fi_comm_get_unique_id(void* dst, size_t bytes) {
    FI_REQUIRE(dst && bytes >= sizeof(ncclUniqueId), "comm_get_unique_id: buffer too small");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(dst, &id, sizeof(id));
    return FI_OK;
}

extern "C" int fi_learner_attach_comm(fi_learner* l, const void* uid, size_t bytes, int rank,
                                      int nranks) {
    FI_REQUIRE(l && uid && bytes >= sizeof(ncclUniqueId), "attach_comm: bad arguments");
    FI_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "attach_comm: bad rank");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    if (l->comm) {
        ncclCommDestroy(l->comm);
        l->comm = nullptr;
    }
    // one rank: no communicator (the sum over one rank is the identity), unless FI_COMM_SINGLE
    // asks for one -- the tests use it to run the in-step all-reduce path on a single GPU
    if (nranks == 1 && !std::getenv("FI_COMM_SINGLE")) return FI_OK;
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    FI_TRY(ensure_comm_stream(l));
    ncclResult_t r = ncclCommInitRank(&l->comm, nranks, id, rank);
    if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    l->rank = rank;
    l->nranks = nranks;
    return FI_OK;
}

// One process driving several devices (one handle per device, e.g. the threaded
// cmd/freeimpala with --devices 0,1,...): the per-device ncclCommInitRank calls are one group,
// so a single thread can attach them all (called one by one, the first would block waiting
// for its peers). Handle i becomes rank i of n.
extern "C" int fi_comm_init_all(fi_learner* const* handles, int n) {
    FI_REQUIRE(handles && n >= 1, "comm_init_all: bad arguments");
    for (int i = 0; i < n; ++i) {
        FI_REQUIRE(handles[i], "comm_init_all: null handle");
        for (int j = 0; j < i; ++j)
            FI_REQUIRE(handles[j]->dev != handles[i]->dev, "comm_init_all: two handles on one device");
    }
    if (n == 1 && !std::getenv("FI_COMM_SINGLE")) return FI_OK;
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    for (int i = 0; i < n; ++i) {
        fi_learner* l = handles[i];
        FI_HIP_CHECK(hipSetDevice(l->dev));
        if (l->comm) {
            ncclCommDestroy(l->comm);
            l->comm = nullptr;
        }
        FI_TRY(ensure_comm_stream(l));
    }
    r = ncclGroupStart();
    if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclGroupStart: ") + ncclGetErrorString(r));
    for (int i = 0; i < n; ++i) {
        FI_HIP_CHECK(hipSetDevice(handles[i]->dev));
        r = ncclCommInitRank(&handles[i]->comm, n, id, i);
        if (r != ncclSuccess) {
            ncclGroupEnd();
            return fail(FI_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclGroupEnd: ") + ncclGetErrorString(r));
    for (int i = 0; i < n; ++i) {
        handles[i]->rank = i;
        handles[i]->nranks = n;
    }
    return FI_OK;
}

// what RCCL reports for the handle's communicator (1 / 0 / 0 without one)
extern "C" int fi_learner_comm_info(fi_learner* l, int* nranks, int* rank, int* buckets) {
    FI_REQUIRE(l, "comm_info: null learner");
    int n = 1, r = 0;
    if (l->comm) {
        ncclResult_t e = ncclCommCount(l->comm, &n);
        if (e == ncclSuccess) e = ncclCommUserRank(l->comm, &r);
        if (e != ncclSuccess) return fail(FI_ERR_COMM, std::string("ncclCommCount: ") + ncclGetErrorString(e));
    }
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    if (buckets) *buckets = l->comm ? l->buckets : 0;
    return FI_OK;
}

// ------------------------------------------------------------------ introspection
extern "C" int fi_learner_read_tensor(fi_learner* l, const char* name, void* dst, size_t bytes) {
    FI_REQUIRE(l && name && dst, "read_tensor: null argument");
    void* p = nullptr;
    size_t have = 0;
    FI_TRY(fi_learner_tensor(l, name, &p, &have));
    FI_REQUIRE(bytes <= have, std::string("read_tensor: ") + name + " holds " + std::to_string(have) + " bytes");
    FI_HIP_CHECK(hipSetDevice(l->dev));
    FI_HIP_CHECK(hipStreamSynchronize(l->stream));
    FI_HIP_CHECK(hipMemcpy(dst, p, bytes, hipMemcpyDeviceToHost));
    return FI_OK;
}

extern "C" int fi_learner_tensor(fi_learner* l, const char* name, void** ptr, size_t* bytes) {
    FI_REQUIRE(l && name && ptr && bytes, "tensor: null argument");
    const size_t rows = l->rows, TB = l->TB, A = l->A;
    struct E {
        const char* n;
        void* p;
        size_t b;
    };
    std::vector<E> t = {
        {"params", l->params, l->nparams * 4},  {"grads", l->grads, l->nparams * 4},
        {"adam_m", l->opt_m, l->nparams * 4},   {"adam_v", l->opt_v, l->nparams * 4},
        {"obs", l->obs, l->obs ? rows * l->D * 4 : 0},
        {"frames", l->frames, l->frames ? rows * AtariNet::kFrameBytes : 0},
        {"mu", l->mu, TB * A * 4},               {"actions", l->act, TB * 4},
        {"rewards", l->rew, TB * 4},             {"discounts", l->disc, TB * 4},
        {"logits", l->logits, rows * A * 4},     {"values", l->values, rows * 4},
        {"vs", l->vs, TB * 4},                   {"pg_adv", l->pg_adv, TB * 4},
        {"dlogits", l->dlogits, TB * A * 4},     {"dvalue", l->dvalue, rows * 4},
        {"losses", l->small, 3 * 8},             {"h1", l->h1, l->h1 ? rows * l->H * 4 : 0},
        {"h2", l->h2, l->h2 ? rows * l->H * 4 : 0},
    };
    for (auto& e : t)
        if (std::strcmp(e.n, name) == 0) {
            *ptr = e.p;
            *bytes = e.b;
            return e.p ? FI_OK : fail(FI_ERR_INVALID, std::string("tensor: not present: ") + name);
        }
    if (l->atari) {
        void* p = nullptr;
        size_t b = 0;
        if (atari_tensor(l->atari, name, &p, &b)) {
            *ptr = p;
            *bytes = b;
            return FI_OK;
        }
    }
    return fail(FI_ERR_INVALID, std::string("tensor: unknown name: ") + name);
}

extern "C" int fi_learner_set_profiling(fi_learner* l, int on) {
    FI_REQUIRE(l, "set_profiling: null");
    l->profiling = on != 0;
    for (double& s : l->phase_sum) s = 0.0;
    l->phase_steps = 0;
    l->tag_sum.clear();
    l->tag_used = 0;
    return FI_OK;
}

extern "C" int fi_learner_phase_times(fi_learner* l, float* ms, int n, int* n_steps) {
    FI_REQUIRE(l && ms && n >= 1, "phase_times: bad arguments");
    for (int p = 0; p < n && p < FI_PHASE_COUNT; ++p)
        ms[p] = l->phase_steps ? (float)(l->phase_sum[p] / l->phase_steps) : 0.f;
    if (n_steps) *n_steps = l->phase_steps;
    return FI_OK;
}

// Mean device ms per launch of every tagged kernel site seen while profiling.
// names: '\n'-separated, written into names_buf; returns the number of entries (<= max).
extern "C" int fi_learner_kernel_times(fi_learner* l, char* names_buf, size_t buflen, float* ms,
                                       int* counts, int max) {
    FI_REQUIRE(l && names_buf && buflen > 0 && ms && counts && max >= 1, "kernel_times: args");
    std::string all;
    int n = 0;
    for (auto& e : l->tag_sum) {
        if (n >= max) break;
        ms[n] = (float)(e.second.first / std::max(1, e.second.second));
        counts[n] = e.second.second;
        all += e.first;
        all += '\n';
        ++n;
    }
    std::strncpy(names_buf, all.c_str(), buflen - 1);
    names_buf[buflen - 1] = 0;
    return n;
}
