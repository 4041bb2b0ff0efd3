// fi_freeimpala -- cmd/freeimpala with the learner step on the MI355X.
//
// The reference binary (cmd/freeimpala/main.cpp) wires agents (producer threads) to the
// Learner through per-player SharedBuffers and a ModelManager; this one runs the same
// program shape on freeimpala_amd::Learner (include/freeimpala_amd/learner.hpp):
//   * the reference's flags, names, short forms and defaults (main.cpp:38-121), parsed
//     strictly (an unknown flag is an error, main.cpp:131-137), plus the learner flags of
//     add_learner_arguments (--seq-length, --learner-arch, --lr, --devices, ...);
//   * the same validation (main.cpp:164-176) and learner iteration count
//     floor(agents * iterations / batch_size) (main.cpp:179);
//   * agents are synthetic actors: each game writes per-step 1 KiB records in the learner's
//     record schema at the reference's producer offsets -- step s goes to
//     player s % P at byte (s / P) * 1024 (agent.h:48-73) -- then writes one entry per player
//     into that player's SharedBuffer (agent.h:78-104), and syncs the published model when its
//     version moved (agent.h:151-178); the record's flags word carries the policy version;
//   * cleanup as main.cpp:233-262: join agents, stop the learner (drain + final save), print
//     the metrics (one JSON line here).
// --dump-dir D (verification only) also writes every batch the learner consumed and every
// parameter version it published, so a test can replay the run through the CPU oracle.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "freeimpala_amd/flags.hpp"
#include "freeimpala_amd/learner.hpp"

using namespace freeimpala_amd;

namespace {

std::string g_dump_dir;

void dump(const std::string& name, const char* p, size_t n) {
    std::ofstream f(g_dump_dir + "/" + name, std::ios::binary);
    f.write(p, (std::streamsize)n);
}

// SharedBuffer that also records each batch it hands to the learner (--dump-dir only)
class DumpingBuffer : public SharedBuffer {
public:
    using SharedBuffer::SharedBuffer;
    bool readBatchInto(size_t M, char* dst, size_t stride) {
        if (!SharedBuffer::readBatchInto(M, dst, stride)) return false;
        if (!g_dump_dir.empty()) dump("batch_" + std::to_string(id_) + "_" + std::to_string(n_++) + ".bin", dst, M * stride);
        return true;
    }
    void setId(size_t id) { id_ = id; }

private:
    size_t id_ = 0, n_ = 0;
};

// ModelManager that also records each published version (--dump-dir only)
class DumpingManager : public ModelManager {
public:
    using ModelManager::ModelManager;
    void updateModel(size_t p, const std::shared_ptr<Model>& m) {
        if (!g_dump_dir.empty()) {
            const auto d = m->getData();
            dump("params_" + std::to_string(p) + "_" + std::to_string(m->getVersion()) + ".bin", d.data(), d.size());
        }
        ModelManager::updateModel(p, m);
    }
};

using CliLearner = BasicLearner<DumpingBuffer, DumpingManager, MetricsTracker>;

struct Params {
    size_t num_players, total_iterations, entry_size, buffer_capacity, batch_size, learner_time,
        checkpoint_freq, num_agents, game_steps, agent_time;
    std::string checkpoint_location, starting_model, metrics_file, log_level, broker;
    unsigned seed;
};

void setup_parser(ArgumentParser& program) {
    program.add_description("Parallel consumer-producer system for game simulation (MI355X learner)");
    program.add_argument("--broker").help("MQTT Broker").default_value(std::string("tcp://localhost:1883"));
    program.add_argument("-p", "--players").help("Number of players").default_value(2).scan<'i', int>();
    program.add_argument("-T", "--iterations").help("Total number of iterations").default_value(100).scan<'i', int>();
    program.add_argument("-S", "--entry-size").help("Size of each buffer entry (in 1024-byte elements)")
        .default_value(100).scan<'i', int>();
    program.add_argument("-B", "--buffer-capacity").help("Capacity of each shared buffer").default_value(10).scan<'i', int>();
    program.add_argument("-M", "--batch-size").help("Number of entries to process in each batch")
        .default_value(5).scan<'i', int>();
    program.add_argument("--learner-time").help("Simulated training time (accepted; the device step replaces it)")
        .default_value(500).scan<'i', int>();
    program.add_argument("-c", "--checkpoint-freq").help("Checkpoint frequency (in iterations)").default_value(10).scan<'i', int>();
    program.add_argument("-l", "--checkpoint-location").help("Location to store and load checkpoint files")
        .default_value(std::string("/tmp/freeimpala_checkpoints"));
    program.add_argument("-m", "--starting-model").help("Starting model location").default_value(std::string(""));
    program.add_argument("-a", "--agents").help("Number of agent processes").default_value(4).scan<'i', int>();
    program.add_argument("--game-steps").help("Number of steps in each game simulation").default_value(100).scan<'i', int>();
    program.add_argument("--agent-time").help("Simulated game play time for agents (in ms)").default_value(200).scan<'i', int>();
    program.add_argument("--metrics-file").help("File to save performance metrics (JSON)").default_value(std::string(""));
    program.add_argument("--seed").help("Seed for random number generation")
        .default_value(static_cast<unsigned>(std::time(nullptr))).scan<'u', unsigned>();
    program.add_argument("--log-level").help("Set the logging level").default_value(std::string("info"))
        .choices("trace", "debug", "info", "warn", "error", "critical", "off");
    add_learner_arguments(program);
    program.add_argument("--dump-dir").help("(verification) write consumed batches and published versions here")
        .default_value(std::string(""));
}

// One synthetic actor (agent.h:11-260 with the learner's record schema instead of rand() bytes).
class SyntheticAgent {
public:
    SyntheticAgent(size_t id, const Params& P, const LearnerConfig& lc, std::vector<std::shared_ptr<DumpingBuffer>> bufs,
                   std::shared_ptr<DumpingManager> models)
        : id_(id), P_(P), lc_(lc), bufs_(std::move(bufs)), models_(std::move(models)),
          versions_(P.num_players, 0), rng_(((uint64_t)P.seed << 20) ^ (0x9E3779B97F4A7C15ull * (id + 1))) {
        for (size_t p = 0; p < P.num_players; ++p) versions_[p] = models_->getLatestVersion(p);
    }

    void run() {
        auto metrics = MetricsTracker::getInstance();
        const size_t entry_bytes = P_.entry_size * ELEMENT_SIZE;
        std::vector<std::vector<char>> entries(P_.num_players, std::vector<char>(entry_bytes, 0));
        for (size_t it = 0; it < P_.total_iterations; ++it) {
            if (P_.agent_time) std::this_thread::sleep_for(std::chrono::milliseconds(P_.agent_time));
            for (auto& e : entries) std::fill(e.begin(), e.end(), 0);
            for (size_t s = 0; s < P_.game_steps; ++s) {
                const size_t p = s % P_.num_players;
                const size_t off = (s / P_.num_players) * ELEMENT_SIZE;
                if (off + ELEMENT_SIZE <= entry_bytes) write_record(entries[p].data() + off, (uint32_t)versions_[p]);
            }
            for (size_t p = 0; p < P_.num_players; ++p) {
                if (bufs_[p]->write(entries[p])) metrics->recordDataTransfer();
                else std::fprintf(stderr, "[agent %zu] failed to write data for player %zu\n", id_, p);
                const uint64_t latest = models_->getLatestVersion(p);
                if (latest > versions_[p]) {
                    local_ = models_->getModel(p)->getData();  // the actor's copy of the policy
                    versions_[p] = latest;
                    metrics->recordAgentModelSync();
                }
            }
        }
    }

private:
    // record schema: obs[0,512) | mu logits [512,768) | action 768 | reward 772 | discount 776 |
    // flags 780 (here: the policy version the actor held)
    void write_record(char* r, uint32_t version) {
        std::normal_distribution<float> nrm(0.f, 1.f);
        std::uniform_real_distribution<float> uni(0.f, 1.f);
        float obs[128] = {}, mu[64] = {};
        for (int d = 0; d < lc_.obs_dim; ++d) obs[d] = nrm(rng_);
        const int A = lc_.num_actions;
        double mx = -1e30, z = 0.0;
        for (int a = 0; a < A; ++a) mx = std::max(mx, (double)(mu[a] = nrm(rng_)));
        for (int a = 0; a < A; ++a) z += std::exp(mu[a] - mx);
        double u = uni(rng_) * z, c = 0.0;
        int32_t action = A - 1;
        for (int a = 0; a < A; ++a) {
            c += std::exp(mu[a] - mx);
            if (u < c) {
                action = a;
                break;
            }
        }
        const float reward = (float)((int)(rng_() % 3) - 1);
        const float discount = uni(rng_) < 0.01f ? 0.f : lc_.gamma;
        std::memcpy(r, obs, sizeof obs);
        std::memcpy(r + 512, mu, sizeof mu);
        std::memcpy(r + 768, &action, 4);
        std::memcpy(r + 772, &reward, 4);
        std::memcpy(r + 776, &discount, 4);
        std::memcpy(r + 780, &version, 4);
    }

    size_t id_;
    Params P_;
    LearnerConfig lc_;
    std::vector<std::shared_ptr<DumpingBuffer>> bufs_;
    std::shared_ptr<DumpingManager> models_;
    std::vector<uint64_t> versions_;
    std::vector<char> local_;
    std::mt19937_64 rng_;
};

}  // namespace

int main(int argc, char** argv) {
    ArgumentParser program("fi_freeimpala");
    setup_parser(program);
    Params P{};
    LearnerConfig lc;
    try {
        program.parse_args(argc, argv);
        P.num_players = program.get<int>("--players");
        P.total_iterations = program.get<int>("--iterations");
        P.entry_size = program.get<int>("--entry-size");
        P.buffer_capacity = program.get<int>("--buffer-capacity");
        P.batch_size = program.get<int>("--batch-size");
        P.learner_time = program.get<int>("--learner-time");
        P.checkpoint_freq = program.get<int>("--checkpoint-freq");
        P.checkpoint_location = program.get<std::string>("--checkpoint-location");
        P.starting_model = program.get<std::string>("--starting-model");
        P.num_agents = program.get<int>("--agents");
        P.game_steps = program.get<int>("--game-steps");
        P.agent_time = program.get<int>("--agent-time");
        P.metrics_file = program.get<std::string>("--metrics-file");
        P.seed = program.get<unsigned>("--seed");
        P.log_level = program.get<std::string>("--log-level");
        P.broker = program.get<std::string>("--broker");
        g_dump_dir = program.get<std::string>("--dump-dir");
        lc = LearnerConfig::from_parser(program);
        if (!program.is_used("--seq-length")) {  // default T: what an entry / a game holds
            const size_t per_player = (P.game_steps + P.num_players - 1) / std::max<size_t>(1, P.num_players);
            lc.seq_length = std::max<size_t>(1, std::min<size_t>({lc.seq_length, P.entry_size, per_player}) - 1);
        }
    } catch (const std::exception& e) {
        const std::string msg = e.what();
        if (msg.rfind("Usage:", 0) == 0) {  // -h / --help
            std::cout << msg;
            return 0;
        }
        std::cerr << e.what() << "\n" << program;
        return 1;
    }
    // main.cpp:164-176, plus what the record schema needs
    if (P.batch_size > P.buffer_capacity) {
        std::cerr << "Batch size must be less than buffer capacity\n";
        return 1;
    }
    if (P.game_steps > P.entry_size) {
        std::cerr << "Game steps must be less than or equal to entry size\n";
        return 1;
    }
    if ((P.game_steps + P.num_players - 1) / P.num_players < lc.seq_length + 1) {
        std::cerr << "Each player needs seq_length + 1 = " << lc.seq_length + 1 << " records per game: raise "
                  << "--game-steps (" << P.game_steps << ") or lower --seq-length\n";
        return 1;
    }
    if (!g_dump_dir.empty()) std::filesystem::create_directories(g_dump_dir);

    auto metrics = MetricsTracker::getInstance();
    metrics->start();
    const size_t learner_iterations = (P.num_agents * P.total_iterations) / P.batch_size;  // main.cpp:179
    std::unique_ptr<CliLearner> learner;
    try {
        learner = std::make_unique<CliLearner>(P.num_players, P.buffer_capacity, P.entry_size, P.batch_size,
                                               P.learner_time, P.checkpoint_freq, P.checkpoint_location,
                                               P.starting_model, learner_iterations, lc);
    } catch (const std::exception& e) {
        std::cerr << "learner: " << e.what() << "\n";
        return 2;
    }
    auto bufs = learner->getSharedBuffers();
    for (size_t p = 0; p < bufs.size(); ++p) bufs[p]->setId(p);
    learner->start();

    std::vector<std::unique_ptr<SyntheticAgent>> agents;
    std::vector<std::thread> threads;
    for (size_t a = 0; a < P.num_agents; ++a) {
        agents.push_back(std::make_unique<SyntheticAgent>(a, P, learner->config(), bufs, learner->getModelManager()));
        threads.emplace_back([ag = agents.back().get()] { ag->run(); });
    }
    for (auto& t : threads) t.join();
    // the agents are done and every entry is written: each player's buffer holds
    // A * iterations entries, so its worker completes floor(A * iterations / M) iterations and
    // then stops by itself (learner.h:75); wait for that before stop() drains (the reference
    // stops right away, main.cpp:241-242, which makes its iteration count timing-dependent)
    const auto t_wait = std::chrono::steady_clock::now();
    for (size_t p = 0; p < P.num_players; ++p)
        while (learner->iterations(p) < learner_iterations &&
               std::chrono::steady_clock::now() - t_wait < std::chrono::minutes(10))
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
    learner->stop();
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    metrics->stop();

    std::string iters = "[";
    for (size_t p = 0; p < P.num_players; ++p) iters += (p ? ", " : "") + std::to_string(learner->iterations(p));
    iters += "]";
    const std::string line = "{\"learner_iterations\": " + iters + ", \"expected_iterations\": " +
                             std::to_string(learner_iterations) + ", \"param_bytes\": " +
                             std::to_string(learner->device().param_bytes()) + ", \"metrics\": " +
                             metrics->summaryJson() + "}";
    std::cout << line << std::endl;
    if (!P.metrics_file.empty()) {
        std::ofstream f(P.metrics_file);
        f << line << "\n";
    }
    return 0;
}
