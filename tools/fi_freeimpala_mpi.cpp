// fi_freeimpala_mpi -- freeimpala_mpi_async_pool with the learner step on the MI355X.
//
// Same process layout as the reference (cmd/freeimpala_mpi_async_pool/main.cpp:361-460):
//   rank 0      the learner: freeimpala_amd::Learner (device step, SharedBuffers, ModelManager)
//               fed by mpi::LearnerEndpoint -- posted MPI_Irecv slots drained by MPI_Waitany,
//               processor threads writing trajectories into the buffers and answering version /
//               weights requests (include/freeimpala_amd/mpi_pool.hpp);
//   ranks 1..N  one actor each (--agents is overridden by world_size - 1, main.cpp:377): play
//               a game, send each player's entry with tag 100 + p, then per player ask for the
//               latest version (tag 200 -> 201) and, when it moved, for the weights
//               (tag 210 -> 211, `u64 version || blob`), agent.h:76-151; TAG_TERMINATE when done.
// The reference flags and validation, the learner flags (--seq-length, --learner-arch, --lr,
// --devices, ...) and the learner iteration count floor(agents * iterations / M)
// (main.cpp:167-170) as in tools/fi_freeimpala.cpp. Actors write the learner's 1 KiB record
// schema instead of rand() bytes. Only rank 0 touches a GPU.
// Rank 0 prints one JSON line: learner iterations, the endpoint's message counts, the
// end-to-end env-steps/s (T * M per learner step over the wall time from the first posted
// receive to the last learner step) and the metrics summary.
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "cli_common.hpp"
#include "freeimpala_amd/mpi_pool.hpp"

using namespace freeimpala_amd;
using namespace fi_cli;

namespace {

int run_actor(int rank, const Params& P, const LearnerConfig& lc) {
    mpi::ActorClient client(0);
    GameWriter game((size_t)rank - 1, P, lc);
    std::vector<uint64_t> versions(P.num_players, 0);
    std::vector<std::vector<char>> local(P.num_players);  // the actor's copy of each policy
    uint64_t sent = 0, syncs = 0;
    for (size_t it = 0; it < P.total_iterations; ++it) {
        if (P.agent_time) std::this_thread::sleep_for(std::chrono::milliseconds(P.agent_time));
        auto& entries = game.play(versions);
        for (size_t p = 0; p < P.num_players; ++p) {
            if (client.send_trajectory(p, entries[p].data(), entries[p].size())) ++sent;
            else std::fprintf(stderr, "[actor %d] MPI_Send(trajectory) failed for player %zu\n", rank, p);
        }
        for (size_t p = 0; p < P.num_players; ++p)
            if (client.sync_model(p, versions[p], local[p])) ++syncs;
    }
    client.terminate();
    if (P.log_level == "debug" || P.log_level == "trace")
        std::fprintf(stderr, "[actor %d] sent %llu entries, %llu model syncs, last versions %llu\n", rank,
                     (unsigned long long)sent, (unsigned long long)syncs, (unsigned long long)versions[0]);
    return 0;
}

int run_learner(int world, const Params& P, const LearnerConfig& lc) {
    auto metrics = MetricsTracker::getInstance();
    metrics->start();
    const size_t learner_iterations = (P.num_agents * P.total_iterations) / P.batch_size;  // main.cpp:167-170
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
    install_dump_observer(*learner, P.num_players);
    learner->start();

    const auto t0 = std::chrono::steady_clock::now();
    mpi::LearnerEndpoint<DumpingBuffer, DumpingManager> endpoint(bufs, learner->getModelManager(),
                                                                 P.entry_size * ELEMENT_SIZE);
    const mpi::EndpointStats es = endpoint.run();
    // every actor is done and every entry written: wait for the workers to consume them
    // (floor(A * iterations / M) steps per player), then stop (drain + final save)
    for (size_t p = 0; p < P.num_players; ++p)
        while (learner->iterations(p) < learner_iterations && !learner->workerFailed() &&
               std::chrono::steady_clock::now() - t0 < std::chrono::minutes(10))
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    learner->stop();
    metrics->stop();

    uint64_t steps = 0;
    for (size_t p = 0; p < P.num_players; ++p) steps += learner->iterations(p);
    const double env_steps = (double)steps * (double)learner->config().seq_length * (double)P.batch_size;
    char buf[768];
    std::snprintf(buf, sizeof buf,
                  "{\"actors\": %d, \"trajectories\": %llu, \"trajectory_bytes\": %llu, \"version_requests\": %llu, "
                  "\"weights_replies\": %llu, \"weights_bytes\": %llu, \"bad_messages\": %llu, \"late_messages\": %llu, "
                  "\"receive_seconds\": %.4f, \"wall_seconds\": %.4f, \"e2e_env_steps_per_s\": %.1f, "
                  "\"receive_GBps\": %.4f}",
                  world - 1, (unsigned long long)es.trajectories, (unsigned long long)es.trajectory_bytes,
                  (unsigned long long)es.version_requests, (unsigned long long)es.weights_replies,
                  (unsigned long long)es.weights_bytes, (unsigned long long)es.bad_messages,
                  (unsigned long long)es.late_messages, es.seconds, wall,
                  wall > 0 ? env_steps / wall : 0.0, es.seconds > 0 ? es.trajectory_bytes / es.seconds / 1e9 : 0.0);
    report(P, "{\"learner_iterations\": " + iterations_json(*learner, P.num_players) +
                  ", \"expected_iterations\": " + std::to_string(learner_iterations) + ", \"param_bytes\": " +
                  std::to_string(learner->device().param_bytes()) + ", \"mpi\": " + buf +
                  ", \"metrics\": " + metrics->summaryJson() + "}");
    if (learner->workerFailed()) {  // a worker stopped on a device failure: the run is incomplete
        std::cerr << "learner: a worker stopped on a device failure\n";
        return 5;
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    int provided = 0;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    if (provided < MPI_THREAD_MULTIPLE) {
        std::fprintf(stderr, "MPI library does not provide MPI_THREAD_MULTIPLE\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    int rank = 0, world = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);

    ArgumentParser program("fi_freeimpala_mpi");
    setup_parser(program, "freeimpala_mpi_async_pool: MPI actor ranks feeding the MI355X learner on rank 0", false);
    Params P{};
    LearnerConfig lc;
    if (const int rc = parse(program, argc, argv, P, lc, false); rc >= 0) {
        MPI_Finalize();
        return rc;
    }
    if (rank != 0) g_dump_dir.clear();
    P.num_agents = (size_t)(world - 1);  // main.cpp:377
    if (world < 2) {
        if (rank == 0) std::fprintf(stderr, "fi_freeimpala_mpi needs at least one actor rank (mpiexec -n >= 2)\n");
        MPI_Finalize();
        return 1;
    }
    int rc;
    if (rank == 0) {
        rc = run_learner(world, P, lc);
        if (rc != 0) MPI_Abort(MPI_COMM_WORLD, rc);  // actors would wait for replies forever
    } else {
        rc = run_actor(rank, P, lc);
    }
    MPI_Finalize();
    return rc;
}
