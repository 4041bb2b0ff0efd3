// reference_mpi_check -- INTEGRATION.md section 3b compiled for real: the rank-0 patch of
// freeimpala_mpi_async_pool (`freeimpala_amd::mpi::LearnerEndpoint<SharedBuffer, ModelManager>`,
// replacing mpi_receiver_posted + the processor threads, reference
// cmd/freeimpala_mpi_async_pool/main.cpp:243-357, 399-428) instantiated on the reference's OWN
// SharedBuffer / ModelManager / Model (/root/reference/include/freeimpala/data_structures.h,
// global namespace), run under mpiexec. Built in the build container only (the reference tree is
// read in place, never copied; the binary travels to the GPU box):
//
//   g++ -std=c++17 -O2 -I/root/reference/include -Itests/cpp/stubs -Iinclude -include optional
//       -I/opt/conda/include tests/cpp/reference_mpi_check.cpp -lfi_learner /opt/conda/lib/libmpi.so
//
// Modes (argv[1]); every failure exits non-zero on the rank that saw it, so mpiexec fails:
//
//   protocol <dir> <slots> <processors>
//       rank 0: the endpoint + a stand-in learner thread per player (reference readBatch(M), then a
//       new Model version whose bytes encode the version, published with Model::update +
//       ModelManager::updateModel, learner.h:40-48). Ranks > 0: the actor side written with the
//       raw MPI calls of agent.h:85-151 (MPI_CHAR entry on tag 100 + p; MPI_UNSIGNED player on
//       200 / 210; MPI_UNSIGNED_LONG_LONG reply on 201; the 211 reply received into an
//       8 + 6 MiB buffer as the reference actors allocate it, mpi_async_pool/main.cpp:443).
//       Checks: every (actor, iteration, player) entry reaches its player's buffer once and
//       intact; with one slot and one processor in the exact order the actor sent it (FIFO end
//       to end); 201 carries the latest version and 211 exactly `u64 version || blob` of a
//       published version; after the last TAG_TERMINATE the endpoint returns, setDraining makes
//       the stand-in's readBatch return {} with the < M leftover entries still in the buffer
//       (data_structures.h:273-280, learner.h:79-84); the endpoint's counters.
//   agents <dir>
//       ranks > 0 run the reference's own Agent (agent.h, compiled with USE_MPI) exactly as
//       mpi_async_pool/main.cpp:437-460 does (dummy buffers, a 6 MiB dummy ModelManager, then
//       TAG_TERMINATE); rank 0 as in `protocol`. Checks the counts and sizes the endpoint saw.
//   learner <dir>
//       GPU: rank 0 is the INTEGRATION.md section 2 alias `BasicLearner<SharedBuffer, ModelManager,
//       MetricsTracker>` on the reference classes plus the endpoint (the whole patched rank 0);
//       actors as in `protocol` but writing record-schema entries. Checks the learner iteration
//       count floor(A * iterations / M) (main.cpp:178), the published version, and that every
//       weights reply is `u64 version || param blob`.
#include "freeimpala/data_structures.h"
#include "freeimpala/metrics_tracker.h"
#define USE_MPI 1
#include "freeimpala/agent.h"
#include "freeimpala_amd/learner.hpp"
#include "freeimpala_amd/mpi_pool.hpp"
using Learner = freeimpala_amd::BasicLearner<SharedBuffer, ModelManager, MetricsTracker>;

#include <mpi.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace {

#define CHECK(c)                                                                              \
    do {                                                                                      \
        if (!(c)) {                                                                           \
            std::fprintf(stderr, "reference_mpi_check: check failed: %s (line %d)\n", #c, __LINE__); \
            std::exit(3);                                                                     \
        }                                                                                     \
    } while (0)

constexpr size_t ACTOR_RECV_MODEL = 6 * 1024 * 1024;  // mpi_async_pool/main.cpp:443

struct Header {
    uint32_t rank, iter, player, magic;
};
void fill_entry(std::vector<char>& e, uint32_t rank, uint32_t it, uint32_t p) {
    Header h{rank, it, p, 0xF1A5u};
    std::memcpy(e.data(), &h, sizeof h);
    for (size_t i = sizeof h; i < e.size(); ++i) e[i] = (char)((rank * 131 + it * 17 + p * 7 + i) & 0xff);
}
bool entry_ok(const std::vector<char>& e, Header& h) {
    if (e.size() < sizeof h) return false;
    std::memcpy(&h, e.data(), sizeof h);
    if (h.magic != 0xF1A5u) return false;
    for (size_t i = sizeof h; i < e.size(); ++i)
        if (e[i] != (char)((h.rank * 131 + h.iter * 17 + h.player * 7 + i) & 0xff)) return false;
    return true;
}

// record schema: obs [0,512) | mu logits [512,768) | action 768 |
// reward 772 | discount 776; T + 1 records per entry
void fill_records(std::vector<char>& e, uint32_t rank, uint32_t it, int A) {
    std::mt19937 rng(97u * rank + 7919u * it + 1u);
    std::normal_distribution<float> nrm(0.f, 1.f);
    std::fill(e.begin(), e.end(), 0);
    for (size_t off = 0; off + ELEMENT_SIZE <= e.size(); off += ELEMENT_SIZE) {
        char* r = e.data() + off;
        float obs[128], mu[64] = {};
        for (float& x : obs) x = nrm(rng);
        for (int a = 0; a < A; ++a) mu[a] = nrm(rng);
        const int32_t action = (int32_t)(rng() % (unsigned)A);
        const float reward = (float)((int)(rng() % 3) - 1), discount = (rng() % 100) ? 0.99f : 0.f;
        std::memcpy(r, obs, sizeof obs);
        std::memcpy(r + 512, mu, sizeof mu);
        std::memcpy(r + 768, &action, 4);
        std::memcpy(r + 772, &reward, 4);
        std::memcpy(r + 776, &discount, 4);
    }
}

// agent.h:112-151 with the reference's datatypes; returns the weights reply's byte count (0 when
// the learner's version was not newer)
size_t sync_like_agent(uint32_t p, uint64_t& have, std::vector<uint8_t>& reply) {
    CHECK(MPI_Send(&p, 1, MPI_UNSIGNED, 0, MessageTag::TAG_VERSION_REQ, MPI_COMM_WORLD) == MPI_SUCCESS);
    uint64_t latest = 0;
    MPI_Recv(&latest, 1, MPI_UNSIGNED_LONG_LONG, 0, MessageTag::TAG_VERSION_RES, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    CHECK(latest >= have);  // versions never go backwards
    if (latest == have) return 0;
    CHECK(MPI_Send(&p, 1, MPI_UNSIGNED, 0, MessageTag::TAG_WEIGHTS_REQ, MPI_COMM_WORLD) == MPI_SUCCESS);
    reply.assign(sizeof(uint64_t) + ACTOR_RECV_MODEL, 0);
    MPI_Status st;
    MPI_Recv(reply.data(), (int)reply.size(), MPI_BYTE, 0, MessageTag::TAG_WEIGHTS_RES, MPI_COMM_WORLD, &st);
    int n = 0;
    MPI_Get_count(&st, MPI_BYTE, &n);
    CHECK(n > (int)sizeof(uint64_t));
    uint64_t v = 0;
    std::memcpy(&v, reply.data(), sizeof v);
    CHECK(v >= latest);  // the weights of the version announced, or a newer one
    have = v;
    return (size_t)n;
}

// ---------------------------------------------------------------------------------------------
// protocol / agents: the stand-in learner on rank 0

struct StandIn {
    size_t P, M, blob;
    std::vector<std::shared_ptr<SharedBuffer>> bufs;
    std::shared_ptr<ModelManager> models;
    std::vector<std::vector<Header>> consumed;  // per player, in readBatch order
    std::atomic<int> bad{0};
    std::vector<std::thread> threads;

    StandIn(size_t P_, size_t S, size_t cap, size_t M_, size_t blob_, const std::string& dir)
        : P(P_), M(M_), blob(blob_), consumed(P_) {
        for (size_t p = 0; p < P; ++p) bufs.push_back(std::make_shared<SharedBuffer>(S, cap));
        models = std::make_shared<ModelManager>(P, blob, dir);
        for (size_t p = 0; p < P; ++p) publish(p, 1);
    }
    void publish(size_t p, uint64_t v) {  // learner.h:40-48 on the reference Model / ModelManager
        auto m = models->getModel(p)->createCopy();
        m->update(std::vector<char>(blob, (char)(v & 0xff)), v);
        models->updateModel(p, m);
    }
    void start(bool check_content) {
        for (size_t p = 0; p < P; ++p)
            threads.emplace_back([this, p, check_content] {
                for (uint64_t b = 0;; ++b) {
                    auto batch = bufs[p]->readBatch(M);
                    if (batch.empty()) return;  // draining with < M entries (learner.h:79-84)
                    if (batch.size() != M) ++bad;
                    for (auto& e : batch) {
                        Header h{};
                        if (check_content && (!entry_ok(e, h) || h.player != p)) ++bad;
                        consumed[p].push_back(h);
                    }
                    publish(p, b + 2);
                }
            });
    }
    void drain_and_join() {
        for (auto& b : bufs) b->setDraining();
        for (auto& t : threads) t.join();
    }
};

int rank0_standin(const std::string& mode, int world, const std::string& dir, int slots, int procs) {
    const bool agents = mode == "agents";
    const size_t P = agents ? 1 : 2, S = 3, M = 3, ITERS = agents ? 4 : 5, BLOB = 4096;
    const size_t actors = (size_t)world - 1, per_player = actors * ITERS;
    StandIn s(P, S, per_player + M, M, BLOB, dir);
    s.start(!agents);
    freeimpala_amd::mpi::LearnerEndpoint<SharedBuffer, ModelManager> ep(s.bufs, s.models, S * ELEMENT_SIZE, procs,
                                                                         slots);
    const auto st = ep.run();
    // every message is in the buffers now; what is left (< M per player) stays there
    for (size_t p = 0; p < P; ++p) {
        for (int i = 0; i < 2000 && s.bufs[p]->getFilledCount() >= M; ++i)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        CHECK(s.bufs[p]->getFilledCount() == per_player % M);
    }
    s.drain_and_join();
    CHECK(s.bad.load() == 0);
    for (size_t p = 0; p < P; ++p) {
        CHECK(s.consumed[p].size() == per_player / M * M);
        CHECK(s.bufs[p]->getFilledCount() == per_player % M);  // drained readBatch took nothing
        if (agents) continue;
        std::set<std::tuple<uint32_t, uint32_t>> seen;
        std::map<uint32_t, uint32_t> next_iter;  // per actor rank
        for (const Header& h : s.consumed[p]) {
            CHECK(seen.insert({h.rank, h.iter}).second);
            if (slots == 1 && procs == 1) {  // one receive and one processor: FIFO end to end
                CHECK(h.iter == next_iter[h.rank]);
                ++next_iter[h.rank];
            }
        }
    }
    CHECK(st.trajectories == per_player * P);
    CHECK(st.trajectory_bytes == per_player * P * S * ELEMENT_SIZE);
    CHECK(st.version_requests == per_player * P);
    CHECK(st.weights_replies >= 1 && st.weights_bytes == st.weights_replies * (8 + BLOB));
    CHECK(st.bad_messages == 0 && st.dropped_entries == 0);
    std::printf("OK reference_mpi %s actors=%zu slots=%d processors=%d trajectories=%llu weights_replies=%llu "
                "left_in_buffer=%zu\n",
                mode.c_str(), actors, slots, procs, (unsigned long long)st.trajectories,
                (unsigned long long)st.weights_replies, per_player % M);
    return 0;
}

int actor_protocol(int rank) {
    const size_t P = 2, S = 3, ITERS = 5, BLOB = 4096;
    std::vector<char> e(S * ELEMENT_SIZE);
    std::vector<uint64_t> have(P, 0);
    std::vector<uint8_t> reply;
    for (uint32_t it = 0; it < ITERS; ++it) {
        for (uint32_t p = 0; p < P; ++p) {  // agent.h:85-90
            fill_entry(e, (uint32_t)rank, it, p);
            CHECK(MPI_Send(e.data(), (int)e.size(), MPI_CHAR, 0, MessageTag::TAG_TRAJECTORY_BASE + (int)p,
                           MPI_COMM_WORLD) == MPI_SUCCESS);
        }
        for (uint32_t p = 0; p < P; ++p) {
            const size_t n = sync_like_agent(p, have[p], reply);
            if (!n) continue;
            CHECK(n == 8 + BLOB);  // u64 version || blob, nothing else
            for (size_t i = 8; i < n; ++i) CHECK(reply[i] == (uint8_t)(have[p] & 0xff));
        }
    }
    MPI_Send(nullptr, 0, MPI_CHAR, 0, MessageTag::TAG_TERMINATE, MPI_COMM_WORLD);  // main.cpp:458
    return 0;
}

// mpi_async_pool/main.cpp:437-460, verbatim in behaviour: the reference Agent on this rank
int actor_reference_agent(int rank, const std::string& dir) {
    const size_t P = 1, S = 3, ITERS = 4;
    std::vector<std::shared_ptr<SharedBuffer>> dummy;
    auto dummy_model_mgr = std::make_shared<ModelManager>(P, ACTOR_RECV_MODEL, dir + "/actor" + std::to_string(rank));
    {
        Agent agent((size_t)rank - 1, P, S, /*game_steps*/ S, /*agent_time*/ 0, ITERS, dummy, dummy_model_mgr);
        agent.run();
    }
    CHECK(MPI_Send(nullptr, 0, MPI_CHAR, 0, MessageTag::TAG_TERMINATE, MPI_COMM_WORLD) == MPI_SUCCESS);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// learner: the patched rank 0 of freeimpala_mpi_async_pool on the GPU

constexpr size_t LT = 8, LS = LT + 1, LM = 4, LITERS = 6;

int rank0_learner(int world, const std::string& dir) {
    freeimpala_amd::LearnerConfig lc;
    lc.seq_length = LT;
    lc.arch = "mlp";
    lc.optimizer = "adam";
    lc.lr = 1e-3f;
    const size_t actors = (size_t)world - 1, total = actors * LITERS;
    const size_t expected = total / LM;  // main.cpp:178 (integer division first)
    std::unique_ptr<Learner> learner;
    try {
        learner = std::make_unique<Learner>(1, total + LM, LS, LM, 0, 0, dir, "", expected, lc);
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "reference_mpi_check: no device: %s\n", ex.what());
        MPI_Abort(MPI_COMM_WORLD, 4);
    }
    auto mm = learner->getModelManager();
    const uint64_t v0 = mm->getLatestVersion(0);
    const size_t param_bytes = learner->param_bytes();
    learner->start();
    freeimpala_amd::mpi::LearnerEndpoint<SharedBuffer, ModelManager> endpoint(learner->getSharedBuffers(), mm,
                                                                              LS * ELEMENT_SIZE);
    const auto st = endpoint.run();
    for (int i = 0; i < 6000 && learner->iterations(0) < expected; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    CHECK(learner->iterations(0) == expected);
    learner->stop();
    CHECK(mm->getLatestVersion(0) == v0 + expected);
    CHECK(mm->getModel(0)->getData().size() == param_bytes);
    CHECK(st.trajectories == total && st.trajectory_bytes == total * LS * ELEMENT_SIZE);
    CHECK(st.version_requests >= total);
    CHECK(st.weights_replies >= actors && st.weights_bytes == st.weights_replies * (8 + param_bytes));
    CHECK(st.bad_messages == 0 && st.dropped_entries == 0);
    std::printf("OK reference_mpi learner actors=%zu iterations=%zu version=%llu param_bytes=%zu weights_replies=%llu\n",
                actors, expected, (unsigned long long)mm->getLatestVersion(0), param_bytes,
                (unsigned long long)st.weights_replies);
    return 0;
}

int actor_learner(int rank, int world) {
    const size_t LWORLD_ACTORS = (size_t)world - 1;
    const int A = freeimpala_amd::LearnerConfig().num_actions;
    std::vector<char> e(LS * ELEMENT_SIZE);
    uint64_t have = 0;
    size_t blob_bytes = 0;
    std::vector<uint8_t> reply;
    for (uint32_t it = 0; it < LITERS; ++it) {
        fill_records(e, (uint32_t)rank, it, A);
        CHECK(MPI_Send(e.data(), (int)e.size(), MPI_CHAR, 0, MessageTag::TAG_TRAJECTORY_BASE, MPI_COMM_WORLD) ==
              MPI_SUCCESS);
        const size_t n = sync_like_agent(0, have, reply);
        if (!n) continue;
        if (blob_bytes) CHECK(n == blob_bytes);  // every version has the same blob size
        blob_bytes = n;
    }
    // the learner's steps can outlast the actors' sends: poll until the last version of the run
    // is published, then take its weights, so the 211 path always carries trained parameters
    const uint64_t last = (uint64_t)(LITERS * (LWORLD_ACTORS)) / LM;
    for (int i = 0; i < 3000 && have < last; ++i) {
        const size_t n = sync_like_agent(0, have, reply);
        if (n) {
            if (blob_bytes) CHECK(n == blob_bytes);
            blob_bytes = n;
        }
        if (have < last) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    CHECK(have >= last && blob_bytes > 8);
    MPI_Send(nullptr, 0, MPI_CHAR, 0, MessageTag::TAG_TERMINATE, MPI_COMM_WORLD);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    int provided = 0;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    CHECK(provided >= MPI_THREAD_MULTIPLE);  // mpi_async_pool/main.cpp:361-365
    int rank = 0, world = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    CHECK(world >= 2);
    const std::string mode = argc > 1 ? argv[1] : "protocol";
    const std::string dir = argc > 2 ? argv[2] : "/tmp/reference_mpi_check";
    const int slots = argc > 3 ? std::atoi(argv[3]) : 128, procs = argc > 4 ? std::atoi(argv[4]) : 8;
    int rc = 0;
    if (mode == "protocol") {
        rc = rank == 0 ? rank0_standin(mode, world, dir, slots, procs) : actor_protocol(rank);
    } else if (mode == "agents") {
        rc = rank == 0 ? rank0_standin(mode, world, dir, slots, procs) : actor_reference_agent(rank, dir);
    } else if (mode == "learner") {
        rc = rank == 0 ? rank0_learner(world, dir) : actor_learner(rank, world);
    } else {
        std::fprintf(stderr, "reference_mpi_check: unknown mode %s\n", mode.c_str());
        rc = 2;
    }
    MPI_Finalize();
    return rc;
}
