// cli_common.hpp -- what the cmd/freeimpala-shaped binaries share (tools/fi_freeimpala.cpp,
// tools/fi_freeimpala_mpi.cpp): the reference's flags and validation, the learner flags, the
// synthetic actors' record writer and the --dump-dir verification hooks.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "freeimpala_amd/flags.hpp"
#include "freeimpala_amd/learner.hpp"
#include "freeimpala_amd/sim_learner.hpp"

namespace fi_cli {

using namespace freeimpala_amd;

inline std::string g_dump_dir;

inline void dump(const std::string& name, const char* p, size_t n) {
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

// --dump-dir: after every step of player p also write the step's loss statistics
// (stats_<p>_<k>.json) and, per named tensor, <name>_<p>_<k>.bin: the gradient ("grads", fp32,
// all-reduced, before clipping) and -- where the network has them (MLP) -- the hidden
// activations and the V-trace output gradients ("h1", "h2", "dlogits", "dvalue"), so a test can
// check every stage of each step against the CPU oracle directly
inline void install_dump_observer(CliLearner& l, size_t players) {
    if (g_dump_dir.empty()) return;
    auto count = std::make_shared<std::vector<size_t>>(players, 0);
    l.setStepObserver([count](size_t p, const fi_step_stats& st, fi_learner* h) {
        const size_t k = (*count)[p]++;  // one worker thread per player
        const std::string sfx = "_" + std::to_string(p) + "_" + std::to_string(k);
        for (const char* name : {"grads", "h1", "h2", "dlogits", "dvalue"}) {
            void* dev = nullptr;
            size_t bytes = 0;
            if (fi_learner_tensor(h, name, &dev, &bytes) != FI_OK || !dev || !bytes) continue;
            std::vector<char> host(bytes);
            if (fi_learner_read_tensor(h, name, host.data(), bytes) == FI_OK) dump(name + sfx + ".bin", host.data(), bytes);
        }
        char js[384];
        const int n = std::snprintf(js, sizeof js,
                                    "{\"pg_loss\": %.17g, \"baseline_loss\": %.17g, \"entropy_loss\": %.17g, "
                                    "\"total_loss\": %.17g, \"grad_norm\": %.17g, \"version\": %llu}",
                                    st.pg_loss, st.baseline_loss, st.entropy_loss, st.total_loss, st.grad_norm,
                                    (unsigned long long)st.version);
        dump("stats" + sfx + ".json", js, (size_t)n);
    });
}

// --learner sim: the reference's placeholder step (sleep + random bytes, learner.h:32-49)
using CliSimLearner = SimLearner<DumpingBuffer, DumpingManager, MetricsTracker>;

struct Params {
    size_t num_players, total_iterations, entry_size, buffer_capacity, batch_size, learner_time,
        checkpoint_freq, num_agents, game_steps, agent_time;
    std::string checkpoint_location, starting_model, metrics_file, log_level, broker;
    unsigned seed;
};

// the reference's flags, names, short forms and defaults (cmd/freeimpala/main.cpp:38-121,
// mpi_async_pool/main.cpp:40-119), plus the learner flags of add_learner_arguments
inline void setup_parser(ArgumentParser& program, const std::string& description, bool broker) {
    program.add_description(description);
    if (broker) program.add_argument("--broker").help("MQTT Broker").default_value(std::string("tcp://localhost:1883"));
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
    program.add_argument("--metrics-file").help("File to save performance metrics (CSV)").default_value(std::string(""));
    program.add_argument("--seed").help("Seed for random number generation")
        .default_value(static_cast<unsigned>(std::time(nullptr))).scan<'u', unsigned>();
    program.add_argument("--log-level").help("Set the logging level").default_value(std::string("info"))
        .choices("trace", "debug", "info", "warn", "error", "critical", "off");
    add_learner_arguments(program);
    program.add_argument("--dump-dir").help("(verification) write consumed batches and published versions here")
        .default_value(std::string(""));
}

// Parses and validates (main.cpp:123-176, plus what the record schema needs). Returns -1 to
// go on, else the process exit code (0 after --help).
inline int parse(ArgumentParser& program, int argc, char** argv, Params& P, LearnerConfig& lc, bool broker) {
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
        if (broker) P.broker = program.get<std::string>("--broker");
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
    return -1;
}

// One synthetic actor's game (agent.h:34-73 with the learner's record schema instead of
// rand() bytes): step s goes to player s % P at byte (s / P) * 1024 of that player's entry.
class GameWriter {
public:
    GameWriter(size_t actor_id, const Params& P, const LearnerConfig& lc)
        : P_(P), lc_(lc), rng_(((uint64_t)P.seed << 20) ^ (0x9E3779B97F4A7C15ull * (actor_id + 1))),
          entries_(P.num_players, std::vector<char>(P.entry_size * ELEMENT_SIZE, 0)) {}

    // versions[p]: the policy version the actor holds for player p (goes into the flags word)
    std::vector<std::vector<char>>& play(const std::vector<uint64_t>& versions) {
        const size_t entry_bytes = P_.entry_size * ELEMENT_SIZE;
        for (auto& e : entries_) std::fill(e.begin(), e.end(), 0);
        for (size_t s = 0; s < P_.game_steps; ++s) {
            const size_t p = s % P_.num_players;
            const size_t off = (s / P_.num_players) * ELEMENT_SIZE;
            if (off + ELEMENT_SIZE <= entry_bytes) write_record(entries_[p].data() + off, (uint32_t)versions[p]);
        }
        return entries_;
    }

private:
    // record schema: obs[0,512) | mu logits [512,768) | action 768 |
    // reward 772 | discount 776 | flags 780 (here: the policy version the actor held)
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

    Params P_;
    LearnerConfig lc_;
    std::mt19937_64 rng_;
    std::vector<std::vector<char>> entries_;
};

// the reference's metrics summary, then the run's closing JSON line on stdout (the last line);
// --metrics-file gets the reference's CSV
// (MetricsTracker::saveMetricsToCSV, cmd/freeimpala/main.cpp:254-257)
inline void report(const Params& P, const std::string& line) {
    MetricsTracker::getInstance()->printMetricsSummary();  // main.cpp:252
    std::cout << line << std::endl;
    if (!P.metrics_file.empty()) MetricsTracker::getInstance()->saveMetricsToCSV(P.metrics_file);
}

template <class L>
std::string iterations_json(const L& l, size_t players) {
    std::string s = "[";
    for (size_t p = 0; p < players; ++p) s += (p ? ", " : "") + std::to_string(l.iterations(p));
    return s + "]";
}

}  // namespace fi_cli
