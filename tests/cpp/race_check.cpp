// race_check.cpp -- concurrency stress of the host side around the learner step, built under
// ThreadSanitizer (and separately under AddressSanitizer + UBSan) by tests/test_sanitizers.py.
// the reference has no sanitizer runs and latent races (global rand() from
// many threads, ModelManager::getModel reading a shared_ptr unlocked, data_structures.h:433-437,
// saveModel reading unlocked state, :395,402); the restated classes here must be race-free.
//   * SharedBuffer (reference data_structures.h:160-307): writers and try_writers against
//     readBatch / readBatchInto readers, then setDraining; every entry consumed once and intact,
//     FIFO order per writer;
//   * Model / ModelManager (:43-157, :310-481): one publisher against readers copying the model
//     (no torn copy: every blob byte equals its version's pattern), version polling, waits, and
//     concurrent checkpoint saves of one player;
//   * MetricsTracker (metrics_tracker.h): scoped timers, counters and agent iterations from many
//     threads while the --metrics-file CSV is written;
//   * SimLearner (learner.h:32-197, config #1's learner): worker threads, checkpoint threads,
//     actor threads writing entries and syncing the published model, stop().
// No GPU: nothing here calls the C ABI. Prints "OK race" and exits 0 when every check holds.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <thread>
#include <vector>

#include "freeimpala_amd/metrics.hpp"
#include "freeimpala_amd/replay.hpp"
#include "freeimpala_amd/sim_learner.hpp"

using namespace freeimpala_amd;

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c);  \
            return 1;                                                             \
        }                                                                         \
    } while (0)

// entry of writer w, sequence s: header (w, s), then a pattern derived from both
static std::vector<char> tagged(size_t bytes, uint32_t w, uint32_t s) {
    std::vector<char> e(bytes);
    std::memcpy(e.data(), &w, 4);
    std::memcpy(e.data() + 4, &s, 4);
    for (size_t i = 8; i < bytes; ++i) e[i] = (char)(w * 31 + s * 7 + i);
    return e;
}
static bool intact(const char* e, size_t bytes, uint32_t* w, uint32_t* s) {
    std::memcpy(w, e, 4);
    std::memcpy(s, e + 4, 4);
    for (size_t i = 8; i < bytes; ++i)
        if (e[i] != (char)(*w * 31 + *s * 7 + i)) return false;
    return true;
}

static int buffer_stress() {
    constexpr int W = 6, PER = 300, M = 4;
    SharedBuffer sb(1, 16);  // 1 KiB entries, capacity 16
    std::vector<std::thread> ws;
    std::atomic<int> written{0};
    for (int w = 0; w < W; ++w)
        ws.emplace_back([&, w] {
            for (int s = 0; s < PER; ++s) {
                const auto e = tagged(1024, (uint32_t)w, (uint32_t)s);
                bool ok = (w & 1) ? sb.write(e) : false;
                while (!ok) {  // even writers retry try_write (mpi_async_pool-style producers); a
                    ok = sb.try_write(e);  // short sleep, not a yield: under TSAN a yield spin can
                    if (!ok) std::this_thread::sleep_for(std::chrono::microseconds(20));  // starve the lock holder
                }
                written.fetch_add(1);
            }
        });
    std::vector<std::vector<int>> seen(2, std::vector<int>(W * PER, 0));
    std::vector<std::vector<int>> last(2, std::vector<int>(W, -1));
    std::atomic<bool> bad{false};
    std::vector<std::thread> rs;
    for (int r = 0; r < 2; ++r)
        rs.emplace_back([&, r] {
            std::vector<char> dst(M * 1024);
            for (;;) {
                std::vector<std::vector<char>> batch;
                if (r == 0) {
                    batch = sb.readBatch(M);
                    if (batch.empty()) return;
                } else {
                    if (!sb.readBatchInto(M, dst.data(), 1024)) return;
                    for (int i = 0; i < M; ++i) batch.emplace_back(dst.begin() + i * 1024, dst.begin() + (i + 1) * 1024);
                }
                for (const auto& e : batch) {
                    uint32_t w, s;
                    if (!intact(e.data(), 1024, &w, &s) || w >= (uint32_t)W || s >= (uint32_t)PER) {
                        bad = true;
                        continue;
                    }
                    // FIFO per writer: a reader sees a writer's entries in increasing order
                    if ((int)s <= last[r][w]) bad = true;
                    last[r][w] = (int)s;
                    seen[r][w * PER + s]++;
                }
            }
        });
    for (auto& t : ws) t.join();
    while (sb.getFilledCount() >= (size_t)M) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    const size_t left = sb.getFilledCount();
    sb.setDraining();
    for (auto& t : rs) t.join();
    CHECK(!bad.load() && written.load() == W * PER);
    int once = 0, twice = 0;
    for (int i = 0; i < W * PER; ++i) {
        const int n = seen[0][i] + seen[1][i];
        once += n == 1;
        twice += n > 1;
    }
    CHECK(twice == 0 && (size_t)once + left == (size_t)(W * PER) && left < (size_t)M);
    return 0;
}

static int model_stress(const std::string& dir) {
    constexpr int VERSIONS = 400, READERS = 4;
    constexpr size_t BYTES = 4096;
    std::filesystem::remove_all(dir);
    ModelManager mm(2, BYTES, dir);
    std::atomic<bool> done{false}, bad{false};
    // a new Model holds random bytes at version 1 (the reference's constructor, data_structures.h:
    // 52-59, bumps the version when it fills them): the publisher's versions start at 2
    std::thread pub([&] {
        for (int v = 2; v <= VERSIONS + 1; ++v) {
            auto m = mm.getModel(1)->createCopy();
            m->update(std::vector<char>(BYTES, (char)v), (uint64_t)v);
            mm.updateModel(1, m);
        }
        done = true;
    });
    std::vector<std::thread> rs;
    for (int r = 0; r < READERS; ++r)
        rs.emplace_back([&, r] {
            uint64_t prev = 0;
            while (!done.load()) {
                const uint64_t lv = mm.getLatestVersion(1);
                if (lv < prev) bad = true;  // versions never go back
                prev = lv;
                const auto c = mm.getModel(1)->createCopy();  // the actors' model sync (agent.h:154-181)
                const auto d = c->getData();
                const uint64_t v = c->getVersion();
                for (char b : d)
                    if (v >= 2 && b != (char)v) {  // a torn copy: bytes of another version
                        bad = true;
                        break;
                    }
                if (r == 0) mm.waitForModelUpdate(1, lv, 1);
            }
        });
    // checkpoints of player 1 while it is being published: two savers numbering from the counter
    std::thread s1([&] {
        for (int i = 0; i < 20; ++i) mm.saveModel(1);
    });
    std::thread s2([&] {
        for (int i = 0; i < 20; ++i) mm.saveModel(1);
    });
    pub.join();
    for (auto& t : rs) t.join();
    s1.join();
    s2.join();
    CHECK(!bad.load() && mm.getLatestVersion(1) == (uint64_t)VERSIONS + 1);
    // 40 saves, 40 distinct numbered files (no counter value handed out twice)
    int files = 0;
    for (const auto& e : std::filesystem::directory_iterator(dir)) {
        const auto n = e.path().filename().string();
        files += n.rfind("model_1_", 0) == 0 && n.find("latest") == std::string::npos && n.size() > 12 &&
                 n.substr(n.size() - 4) == ".bin";
    }
    CHECK(files == 40);
    return 0;
}

static int metrics_stress(const std::string& dir) {
    auto m = MetricsTracker::getInstance();
    m->start();
    const uint64_t u0 = m->getTotalLearnerModelUpdates(), t0 = m->getTotalDataTransfers();
    std::vector<std::thread> ts;
    const uint64_t i0 = m->getTotalIterations();
    for (int i = 0; i < 8; ++i)
        ts.emplace_back([&, i] {
            for (int k = 0; k < 500; ++k) {
                m->startAgentIteration((size_t)i);  // per-thread start time (agent.h:236, :290)
                {
                    auto timer = m->createTrainingTimer();
                    m->recordLearnerModelUpdate();
                    m->recordDataTransfer();
                    m->recordAgentModelSync();
                    m->recordLearnerEnvSteps(100, 0.01);
                }
                { auto s = m->createSimulationTimer(); }
                { auto x = m->createTransferTimer(); }
                { auto y = m->createSyncTimer(); }
                m->endAgentIteration((size_t)i);
            }
        });
    // the --metrics-file writer reading every counter while they move
    std::thread writer([&] {
        for (int k = 0; k < 20; ++k) m->saveMetricsToCSV(dir + "/metrics.csv");
    });
    for (auto& t : ts) t.join();
    writer.join();
    m->stop();
    CHECK(m->getTotalLearnerModelUpdates() - u0 == 4000 && m->getTotalDataTransfers() - t0 == 4000);
    CHECK(m->getTotalIterations() - i0 == 4000);
    return 0;
}

static int sim_learner_stress(const std::string& dir) {
    // config #1's shape, shortened: 2 players, 4 actor threads, M = 4, S = 3 elements, no sleeps
    constexpr size_t P = 2, A = 4, ITERS = 24, M = 4, S = 3;
    std::filesystem::remove_all(dir);
    const size_t T = A * ITERS / M;  // floor(A * iterations / M) learner iterations per player
    SimLearner<SharedBuffer, ModelManager, MetricsTracker> L(P, 8, S, M, 0, 5, dir, "", T);
    L.start();
    auto bufs = L.getSharedBuffers();
    auto mm = L.getModelManager();
    std::atomic<bool> bad{false};
    std::vector<std::thread> actors;
    for (size_t a = 0; a < A; ++a)
        actors.emplace_back([&, a] {
            uint64_t seen = 0;
            for (size_t it = 0; it < ITERS; ++it) {
                for (size_t p = 0; p < P; ++p)
                    if (!bufs[p]->write(tagged(S * 1024, (uint32_t)a, (uint32_t)it))) bad = true;
                for (size_t p = 0; p < P; ++p) {  // model sync (agent.h:154-181)
                    const uint64_t v = mm->getLatestVersion(p);
                    if (v > seen) {
                        const auto c = mm->getModel(p)->createCopy();
                        if (c->getData().size() != SimLearner<SharedBuffer, ModelManager, MetricsTracker>::kModelBytes) bad = true;
                        seen = v;
                    }
                }
            }
        });
    for (auto& t : actors) t.join();
    for (int i = 0; i < 2000 && (L.iterations(0) < T || L.iterations(1) < T); ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
    L.stop();
    CHECK(!bad.load() && L.iterations(0) == T && L.iterations(1) == T);
    for (size_t p = 0; p < P; ++p)
        CHECK(std::filesystem::exists(ModelManager::iter_path(dir, p, T)) &&
              std::filesystem::exists(ModelManager::latest_path(dir, p)));
    return 0;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp/fi_race_check";
    if (buffer_stress() || model_stress(dir + "/models") || (std::filesystem::create_directories(dir), metrics_stress(dir)) || sim_learner_stress(dir + "/sim")) return 1;
    std::printf("OK race\n");
    return 0;
}
