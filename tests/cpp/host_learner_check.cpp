// host_learner_check.cpp -- exercises the C++ host side (include/freeimpala_amd/
// device_learner.hpp) the way the reference's Learner would drive it.
//
//   host_learner_check cpu
//       flag parsing (reference cmd/freeimpala flags + learner flags), error behaviour,
//       and that constructing a DeviceLearner without a usable GPU fails loudly.
//   host_learner_check gpu OUT_DIR
//       two players, one std::thread each (reference learner.h:158-163), both stepping the
//       same SharedBuffer-shaped batch (M entries of S*1024 bytes, DESIGN.md section 3
//       record schema) from the same parameters; checks the two results are identical,
//       then writes the batch, the parameters and the step statistics to OUT_DIR so that
//       tests/test_host_cpp.py can compare them with the CPU oracle.
//   host_learner_check pipeline
//       one player at B = 1344, T = 100 (139 MB per batch: the library copies it with its
//       parallel staging threads), three asynchronous steps back to back (pinned double
//       buffering, H2D on the copy stream beside the previous step) against the same three
//       steps taken synchronously on a twin handle: identical parameters. Built under
//       ThreadSanitizer with the library's host side instrumented (tests/cpp/tsan.mk).
//   host_learner_check worker_fail DIR
//       freeimpala_amd::Learner whose staging acquisition fails (a test subclass): the worker
//       must stop, report workerFailed(), and drain its buffer so an actor blocked in write() on
//       the full buffer returns instead of hanging.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "freeimpala_amd/device_learner.hpp"
#include "freeimpala_amd/learner.hpp"

using freeimpala_amd::DeviceLearner;
using freeimpala_amd::LearnerConfig;

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c);  \
            return 1;                                                             \
        }                                                                         \
    } while (0)

static int cpu_mode() {
    const char* argv[] = {"freeimpala", "-p", "2", "-M", "64", "--seq-length", "20", "-S", "24",
                          "--learner-arch", "mlp", "--lr", "0.001", "--devices", "0,1",
                          "--agents", "4", "--publish", "bf16"};
    const LearnerConfig c = LearnerConfig::from_args(sizeof(argv) / sizeof(argv[0]), argv);
    CHECK(c.players == 2 && c.batch_size == 64 && c.seq_length == 20 && c.entry_size == 24);
    CHECK(c.entry_records() == 24 && c.devices.size() == 2 && c.devices[1] == 1);
    CHECK(std::fabs(c.lr - 0.001f) < 1e-9f && c.publish == "bf16");
    const fi_learner_config k = c.abi_config(1);
    CHECK(k.struct_size == sizeof(fi_learner_config) && k.batch == 64 && k.seq_len == 20);
    CHECK(k.device == 1 && k.publish_dtype == FI_PUBLISH_BF16 && k.seed == c.seed + 1);

    bool threw = false;
    try {
        const char* bad[] = {"x", "--seq-length", "10", "-S", "5"};  // entries too short
        LearnerConfig::from_args(5, bad);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
    threw = false;
    try {
        const char* bad[] = {"x", "--batch-size", "12x"};
        LearnerConfig::from_args(3, bad);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);

    // no GPU in this container: construction must fail loudly, never fall back to the CPU
    threw = false;
    try {
        LearnerConfig one;
        one.batch_size = 16;
        one.seq_length = 4;
        DeviceLearner L(one);
    } catch (const std::runtime_error& e) {
        threw = std::string(e.what()).find("fi_learner_create") != std::string::npos;
        std::printf("expected failure: %s\n", e.what());
    }
    CHECK(threw);
    std::printf("OK cpu\n");
    return 0;
}

// deterministic host-side batch in the record schema (obs@0, mu@512, act@768, rew@772,
// disc@776); any generator works: the oracle reads back the same bytes.
static std::vector<std::vector<char>> make_batch(size_t M, size_t S, int T, int A, int D) {
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto next = [&x]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return x;
    };
    auto unif = [&]() { return (float)((next() >> 40) * (1.0 / 16777216.0)) * 2.f - 1.f; };
    std::vector<std::vector<char>> batch(M, std::vector<char>(S * FI_RECORD_BYTES, 0));
    for (size_t b = 0; b < M; ++b) {
        for (int t = 0; t <= T; ++t) {
            char* rec = batch[b].data() + (size_t)t * FI_RECORD_BYTES;
            for (int i = 0; i < D; ++i) {
                const float v = 1.5f * unif();
                std::memcpy(rec + 4 * i, &v, 4);
            }
            for (int i = 0; i < A; ++i) {
                const float v = 2.f * unif();
                std::memcpy(rec + 512 + 4 * i, &v, 4);
            }
            const int32_t act = (int32_t)(next() % (uint64_t)A);
            const float rew = (float)((int)(next() % 3) - 1);
            const float disc = (next() % 100) == 0 ? 0.f : 0.99f;
            std::memcpy(rec + 768, &act, 4);
            std::memcpy(rec + 772, &rew, 4);
            std::memcpy(rec + 776, &disc, 4);
        }
    }
    return batch;
}

static int gpu_mode(const std::string& out) {
    LearnerConfig c;
    c.players = 2;
    c.batch_size = 32;
    c.seq_length = 8;
    c.entry_size = 10;  // one spare record per entry, like --entry-size > T+1
    c.optimizer = "sgd";
    c.lr = 1e-3f;
    c.max_grad_norm = 0.f;
    DeviceLearner L(c);
    CHECK(L.entry_bytes() == (c.seq_length + 1) * FI_RECORD_BYTES);
    const int T = (int)c.seq_length, A = c.num_actions, D = c.obs_dim;
    const auto batch = make_batch(c.batch_size, c.entry_records(), T, A, D);

    // same starting parameters for both players (publish -> resume path)
    std::vector<char> p0;
    uint64_t v0 = 0;
    CHECK(L.publish(0, p0, v0));
    CHECK(p0.size() == L.param_bytes());
    CHECK(L.load(1, p0, v0));

    bool ok0 = false, ok1 = false;
    std::thread t0([&] { ok0 = L.step(0, batch); });
    std::thread t1([&] { ok1 = L.step(1, batch); });
    t0.join();
    t1.join();
    if (!ok0 || !ok1) std::fprintf(stderr, "step failed: %s | %s\n", L.last_error(0).c_str(), L.last_error(1).c_str());
    CHECK(ok0 && ok1);
    const fi_step_stats s0 = L.last_stats(0);  // copies: player 0 steps again below
    const fi_step_stats s1 = L.last_stats(1);
    CHECK(s0.total_loss == s1.total_loss && s0.grad_norm == s1.grad_norm);
    CHECK(s0.version == v0 + 1 && s1.version == v0 + 1);
    std::vector<char> p1a, p1b;
    uint64_t va = 0, vb = 0;
    CHECK(L.publish(0, p1a, va) && L.publish(1, p1b, vb));
    CHECK(va == v0 + 1 && p1a == p1b && p1a != p0);

    // error path: wrong batch size is reported, not thrown, and the handle stays usable
    std::vector<std::vector<char>> short_batch(batch.begin(), batch.begin() + 5);
    CHECK(!L.step(0, short_batch));
    CHECK(!L.last_error(0).empty());
    CHECK(L.step(0, batch));

    // zero-copy staging (SharedBuffer::readBatchInto): a drained buffer submits nothing; then
    // player 1 takes its second step from the staging buffer and must match player 0's second
    // step (which went through the entry-pointer path) bit for bit
    CHECK(!L.step_staged(1, [](char*, size_t, size_t) { return false; }));
    uint64_t vd = 0;
    std::vector<char> pd;
    CHECK(L.publish(1, pd, vd) && vd == v0 + 1);
    CHECK(L.step_staged(1, [&](char* dst, size_t stride, size_t n) {
        if (n != batch.size() || stride > batch[0].size()) return false;
        for (size_t i = 0; i < n; ++i) std::memcpy(dst + i * stride, batch[i].data(), stride);
        return true;
    }));
    std::vector<char> p2a, p2b;
    CHECK(L.publish(0, p2a, va) && L.publish(1, p2b, vb));
    CHECK(va == v0 + 2 && vb == v0 + 2 && p2a == p2b);

    std::vector<char> flat;
    for (const auto& e : batch) flat.insert(flat.end(), e.begin(), e.end());
    std::ofstream(out + "/batch.bin", std::ios::binary).write(flat.data(), (std::streamsize)flat.size());
    std::ofstream(out + "/params0.bin", std::ios::binary).write(p0.data(), (std::streamsize)p0.size());
    std::ofstream(out + "/params1.bin", std::ios::binary).write(p1a.data(), (std::streamsize)p1a.size());
    std::ofstream js(out + "/stats.json");
    char buf[512];
    std::snprintf(buf, sizeof(buf),
                  "{\"T\": %d, \"B\": %zu, \"S\": %zu, \"A\": %d, \"D\": %d, \"lr\": %.9g, "
                  "\"pg_loss\": %.17g, \"baseline_loss\": %.17g, \"entropy_loss\": %.17g, "
                  "\"total_loss\": %.17g, \"grad_norm\": %.17g, \"version\": %llu}\n",
                  T, c.batch_size, c.entry_records(), A, D, (double)c.lr, s0.pg_loss, s0.baseline_loss,
                  s0.entropy_loss, s0.total_loss, s0.grad_norm, (unsigned long long)s0.version);
    js << buf;
    std::printf("OK gpu total_loss=%.9g\n", s0.total_loss);
    return 0;
}

static int pipeline_mode() {
    LearnerConfig c;
    c.players = 2;  // player 0 asynchronous, player 1 its synchronous twin
    c.batch_size = 1344;  // 139 MB per batch: 3 staging copy threads (one per 64 MiB, csrc/learner.cpp)
    c.seq_length = 100;
    c.entry_size = 101;
    c.optimizer = "adam";
    DeviceLearner L(c);
    const int T = (int)c.seq_length, A = c.num_actions, D = c.obs_dim;
    std::vector<std::vector<std::vector<char>>> batches;
    for (int k = 0; k < 3; ++k) {
        auto b = make_batch(c.batch_size, c.entry_records(), T, A, D);
        for (auto& e : b) e[772] ^= (char)k;  // distinct rewards per batch
        batches.push_back(std::move(b));
    }
    std::vector<char> p0;
    uint64_t v0 = 0;
    CHECK(L.publish(0, p0, v0) && L.load(1, p0, v0));
    std::atomic<bool> twin_ok{true};
    std::thread twin([&] {
        for (const auto& b : batches)
            if (!L.step(1, b)) twin_ok = false;
    });
    for (const auto& b : batches) CHECK(L.step_async(0, b));
    CHECK(L.wait(0));
    twin.join();
    CHECK(twin_ok.load());
    std::vector<char> pa, pb;
    uint64_t va = 0, vb = 0;
    CHECK(L.publish(0, pa, va) && L.publish(1, pb, vb));
    CHECK(va == v0 + 3 && vb == v0 + 3 && pa == pb && pa != p0);
    std::printf("OK pipeline\n");
    return 0;
}

struct FailingLearner : freeimpala_amd::Learner {
    using freeimpala_amd::Learner::Learner;
    std::atomic<int> calls{0};
    int acquireStaging(fi_learner*, void**, size_t*) override {
        ++calls;
        return FI_ERR_STATE;
    }
};

static int worker_fail_mode(const std::string& dir) {
    LearnerConfig c;
    c.seq_length = 8;
    constexpr size_t CAP = 4, S = 9, M = 2, WRITES = 3 * CAP;
    FailingLearner L(1, CAP, S, M, 0, 0, dir, "", 100, c);
    L.start();
    auto buf = L.getSharedBuffers()[0];
    std::atomic<int> written{0}, refused{0};
    std::atomic<bool> done{false};
    std::thread agent([&] {  // more entries than the buffer holds: blocks once it is full
        const std::vector<char> e(S * FI_RECORD_BYTES, 1);
        for (size_t i = 0; i < WRITES; ++i) (buf->write(e) ? written : refused)++;
        done = true;
    });
    for (int i = 0; i < 3000 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (!done) {
        std::fprintf(stderr, "actor still blocked in write() after the worker failed\n");
        std::_Exit(1);  // the blocked thread cannot be joined
    }
    agent.join();
    CHECK(L.workerFailed() && L.iterations(0) == 0 && L.calls.load() == 1);
    CHECK(refused.load() > 0 && (size_t)(written.load() + refused.load()) == WRITES);
    L.stop();
    std::printf("OK worker_fail written=%d refused=%d\n", written.load(), refused.load());
    return 0;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        if (mode == "cpu") return cpu_mode();
        if (mode == "gpu" && argc > 2) return gpu_mode(argv[2]);
        if (mode == "pipeline") return pipeline_mode();
        if (mode == "worker_fail" && argc > 2) return worker_fail_mode(argv[2]);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "unexpected exception: %s\n", e.what());
        return 1;
    }
    std::fprintf(stderr, "usage: host_learner_check cpu | gpu OUT_DIR | pipeline | worker_fail DIR\n");
    return 2;
}
