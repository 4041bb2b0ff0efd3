// mpi_pool_check -- CPU check of include/freeimpala_amd/mpi_pool.hpp under mpiexec (no GPU):
// rank 0 runs LearnerEndpoint over freeimpala_amd SharedBuffers + ModelManager with a consumer
// thread per player standing in for the learner worker (readBatch(M), then publish a new Model
// version whose bytes encode the version); ranks > 0 run ActorClient like agent.h's MPI paths.
// Checks: every (actor, iteration, player) entry arrives exactly once, intact, in its player's
// buffer; the endpoint's counters; actors only ever see newer versions, each with the bytes of
// that version and the publisher's blob size. Prints "OK mpi_pool" on rank 0; any failure
// exits non-zero (mpiexec then fails).
#include <mpi.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "freeimpala_amd/mpi_pool.hpp"
#include "freeimpala_amd/replay.hpp"

using namespace freeimpala_amd;

namespace {

constexpr size_t P = 2, S = 3, CAP = 4, M = 2, ITERS = 6, BLOB = 4096;

#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "rank check failed: %s (line %d)\n", #c, __LINE__); \
            std::exit(3);                                                             \
        }                                                                             \
    } while (0)

struct Header {
    uint32_t rank, iter, player, magic;
};

void fill_entry(std::vector<char>& e, uint32_t rank, uint32_t it, uint32_t p) {
    Header h{rank, it, p, 0xF1A5u};
    std::memcpy(e.data(), &h, sizeof h);
    for (size_t i = sizeof h; i < e.size(); ++i) e[i] = (char)((rank * 131 + it * 17 + p * 7 + i) & 0xff);
}
bool entry_ok(const std::vector<char>& e, Header& h) {
    std::memcpy(&h, e.data(), sizeof h);
    if (h.magic != 0xF1A5u) return false;
    for (size_t i = sizeof h; i < e.size(); ++i)
        if (e[i] != (char)((h.rank * 131 + h.iter * 17 + h.player * 7 + i) & 0xff)) return false;
    return true;
}

int learner(int world, const std::string& dir) {
    std::vector<std::shared_ptr<SharedBuffer>> bufs;
    for (size_t p = 0; p < P; ++p) bufs.push_back(std::make_shared<SharedBuffer>(S, CAP));
    auto models = std::make_shared<ModelManager>(P, BLOB, dir);
    for (size_t p = 0; p < P; ++p)  // version 1 (a new Model's): bytes 1, like every later version
        models->updateModel(p, Model::fromData(ModelManager::latest_path(dir, p), std::vector<char>(BLOB, 1), 1));
    const size_t total = (size_t)(world - 1) * ITERS;  // entries per player
    CHECK(total % M == 0);
    std::vector<std::set<std::tuple<uint32_t, uint32_t>>> seen(P);
    std::atomic<int> bad{0};
    std::vector<std::thread> workers;
    for (size_t p = 0; p < P; ++p)
        workers.emplace_back([&, p] {
            for (size_t b = 0; b < total / M; ++b) {
                auto batch = bufs[p]->readBatch(M);
                if (batch.size() != M) {
                    ++bad;
                    return;
                }
                for (auto& e : batch) {
                    Header h;
                    if (e.size() != S * ELEMENT_SIZE || !entry_ok(e, h) || h.player != p ||
                        !seen[p].insert({h.rank, h.iter}).second)
                        ++bad;
                }
                const uint64_t v = b + 2;  // publish: blob bytes = v
                auto m = models->getModel(p)->createCopy();
                m->update(std::vector<char>(BLOB, (char)(v & 0xff)), v);
                models->updateModel(p, m);
            }
        });
    mpi::LearnerEndpoint<SharedBuffer, ModelManager> ep(bufs, models, S * ELEMENT_SIZE, 3, 8);
    const mpi::EndpointStats st = ep.run();
    for (auto& t : workers) t.join();
    CHECK(bad.load() == 0);
    for (size_t p = 0; p < P; ++p) CHECK(seen[p].size() == total);
    CHECK(st.trajectories == total * P);
    CHECK(st.trajectory_bytes == total * P * S * ELEMENT_SIZE);
    CHECK(st.version_requests == total * P);
    CHECK(st.weights_replies >= 1 && st.weights_replies <= total * P);
    CHECK(st.bad_messages == 0 && st.dropped_entries == 0);
    std::printf("OK mpi_pool actors=%d trajectories=%llu weights_replies=%llu\n", world - 1,
                (unsigned long long)st.trajectories, (unsigned long long)st.weights_replies);
    return 0;
}

int actor(int rank) {
    mpi::ActorClient c(0);
    std::vector<char> e(S * ELEMENT_SIZE);
    std::vector<uint64_t> have(P, 0);
    std::vector<std::vector<char>> blob(P);
    for (uint32_t it = 0; it < ITERS; ++it) {
        for (uint32_t p = 0; p < P; ++p) {
            fill_entry(e, (uint32_t)rank, it, p);
            CHECK(c.send_trajectory(p, e.data(), e.size()));
        }
        for (size_t p = 0; p < P; ++p) {
            const uint64_t before = have[p];
            if (c.sync_model(p, have[p], blob[p])) {
                CHECK(have[p] > before);
                CHECK(blob[p].size() == BLOB);
                for (char x : blob[p]) CHECK(x == (char)(have[p] & 0xff));
            } else {
                CHECK(have[p] == before);
            }
        }
    }
    c.terminate();
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    int provided = 0;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    CHECK(provided >= MPI_THREAD_MULTIPLE);
    int rank = 0, world = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    CHECK(world >= 2);
    const std::string dir = argc > 1 ? argv[1] : "/tmp/mpi_pool_check";
    const int rc = rank == 0 ? learner(world, dir) : actor(rank);
    MPI_Finalize();
    return rc;
}
