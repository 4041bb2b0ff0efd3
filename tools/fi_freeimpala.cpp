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
#include <chrono>
#include <cstdio>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "cli_common.hpp"

using namespace freeimpala_amd;
using namespace fi_cli;

namespace {

// One synthetic actor thread (agent.h:11-260): play a game, write one entry per player into
// that player's SharedBuffer (agent.h:78-104), sync the published model when its version moved
// (agent.h:151-178).
class SyntheticAgent {
public:
    SyntheticAgent(size_t id, const Params& P, const LearnerConfig& lc, std::vector<std::shared_ptr<DumpingBuffer>> bufs,
                   std::shared_ptr<DumpingManager> models)
        : id_(id), P_(P), game_(id, P, lc), bufs_(std::move(bufs)), models_(std::move(models)),
          versions_(P.num_players, 0) {
        for (size_t p = 0; p < P.num_players; ++p) versions_[p] = models_->getLatestVersion(p);
    }

    // the reference agent's loop and its metric hooks (agent.h:34-98, 154-181, 236-290): a timed
    // simulation, a timed transfer per player, a timed model sync, one timed iteration
    void run() {
        auto metrics = MetricsTracker::getInstance();
        for (size_t it = 0; it < P_.total_iterations; ++it) {
            metrics->startAgentIteration(id_);
            std::vector<std::vector<char>>* entries = nullptr;
            {
                auto timer = metrics->createSimulationTimer();
                if (P_.agent_time) std::this_thread::sleep_for(std::chrono::milliseconds(P_.agent_time));
                entries = &game_.play(versions_);
            }
            for (size_t p = 0; p < P_.num_players; ++p) {
                auto timer = metrics->createTransferTimer();
                if (bufs_[p]->write((*entries)[p])) metrics->recordDataTransfer();
                else std::fprintf(stderr, "[agent %zu] failed to write data for player %zu\n", id_, p);
            }
            {
                auto timer = metrics->createSyncTimer();
                for (size_t p = 0; p < P_.num_players; ++p) {
                    const uint64_t latest = models_->getLatestVersion(p);
                    if (latest > versions_[p]) {
                        local_ = models_->getModel(p)->getData();  // the actor's copy of the policy
                        versions_[p] = latest;
                        metrics->recordAgentModelSync();
                    }
                }
            }
            metrics->endAgentIteration(id_);
        }
    }

private:
    size_t id_;
    Params P_;
    GameWriter game_;
    std::vector<std::shared_ptr<DumpingBuffer>> bufs_;
    std::shared_ptr<DumpingManager> models_;
    std::vector<uint64_t> versions_;
    std::vector<char> local_;
};

}  // namespace

template <class L>
int run(const Params& P, const LearnerConfig& lc, const std::string& kind) {
    auto metrics = MetricsTracker::getInstance();
    metrics->start();
    const size_t learner_iterations = (P.num_agents * P.total_iterations) / P.batch_size;  // main.cpp:179
    std::unique_ptr<L> learner;
    try {
        learner = std::make_unique<L>(P.num_players, P.buffer_capacity, P.entry_size, P.batch_size, P.learner_time,
                                      P.checkpoint_freq, P.checkpoint_location, P.starting_model, learner_iterations,
                                      lc);
    } catch (const std::exception& e) {
        std::cerr << "learner: " << e.what() << "\n";
        return 2;
    }
    auto bufs = learner->getSharedBuffers();
    for (size_t p = 0; p < bufs.size(); ++p) bufs[p]->setId(p);
    if constexpr (std::is_same_v<L, CliLearner>) install_dump_observer(*learner, P.num_players);
    const auto t0 = std::chrono::steady_clock::now();
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
        while (learner->iterations(p) < learner_iterations && !learner->workerFailed() &&
               std::chrono::steady_clock::now() - t_wait < std::chrono::minutes(10))
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    learner->stop();
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    metrics->stop();

    // learner env-steps/s over the whole run: T x M per learner iteration (the BASELINE metric's
    // unit; sleep-bound with --learner sim, as the reference's own config #1 is)
    size_t iters = 0;
    for (size_t p = 0; p < P.num_players; ++p) iters += learner->iterations(p);
    const double env_steps = (double)iters * (double)learner->config().seq_length * (double)P.batch_size;
    char buf[160];
    std::snprintf(buf, sizeof buf, ", \"wall_seconds\": %.4f, \"learner_env_steps_per_s\": %.1f", wall,
                  wall > 0 ? env_steps / wall : 0.0);
    report(P, "{\"learner\": \"" + kind + "\", \"learner_iterations\": " + iterations_json(*learner, P.num_players) +
                  ", \"expected_iterations\": " + std::to_string(learner_iterations) + ", \"param_bytes\": " +
                  std::to_string(learner->param_bytes()) + buf + ", \"metrics\": " + metrics->summaryJson() + "}");
    if (learner->workerFailed()) {  // a worker stopped on a device failure: the run is incomplete
        std::cerr << "learner: a worker stopped on a device failure\n";
        return 5;
    }
    return 0;
}

int main(int argc, char** argv) {
    ArgumentParser program("fi_freeimpala");
    setup_parser(program, "Parallel consumer-producer system for game simulation (MI355X learner)", true);
    program.add_argument("--learner")
        .help("device: the MI355X learner step; sim: the reference's placeholder step (sleep --learner-time, "
              "then random model bytes; learner.h:32-49), no GPU")
        .default_value(std::string("device"))
        .choices("device", "sim");
    Params P{};
    LearnerConfig lc;
    if (const int rc = parse(program, argc, argv, P, lc, true); rc >= 0) return rc;
    const std::string kind = program.get<std::string>("--learner");
    return kind == "sim" ? run<CliSimLearner>(P, lc, kind) : run<CliLearner>(P, lc, kind);
}
