// metrics.hpp -- the learner's counters of freeimpala's MetricsTracker, natively.
//
// Reference include/freeimpala/metrics_tracker.h: a process-wide singleton; counters only count
// between start() and stop(); scoped timers add their elapsed ns to the simulation / training /
// transfer / sync times (:126-177); recordLearnerModelUpdate() counts published models
// (:109-112); per-agent iteration times (:92-107); rates and the time distribution (:205-254);
// saveMetricsToCSV writes the reference's "Metric,Value" file (:265-329), which cmd/freeimpala
// writes for --metrics-file (main.cpp:254-257). The learner step also reports what the device
// did: env-steps trained (T x B per step), device milliseconds and rejected batches, appended
// as rows of their own so the file states env-steps/s next to the reference's counters.
// printMetricsSummary is the reference's end-of-run report (:332-382) with a learner section.
// An agent iteration's start time is per thread, as in the reference (:388); unlike the
// reference, the execution time stops at stop().
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace freeimpala_amd {

class MetricsTracker {
public:
    using Clock = std::chrono::steady_clock;

    static std::shared_ptr<MetricsTracker> getInstance() {
        static std::shared_ptr<MetricsTracker> inst(new MetricsTracker());
        return inst;
    }

    void start() {
        t0_ = Clock::now();
        running_.store(true);
    }
    void stop() {
        if (running_.exchange(false)) t1_ = Clock::now();
    }
    bool isRunning() const { return running_.load(); }

    class ScopedTimer {
    public:
        explicit ScopedTimer(std::function<void(uint64_t)> cb) : start_(Clock::now()), cb_(std::move(cb)) {}
        ScopedTimer(ScopedTimer&& o) noexcept : start_(o.start_), cb_(std::move(o.cb_)) { o.cb_ = nullptr; }
        ScopedTimer(const ScopedTimer&) = delete;
        ~ScopedTimer() {
            if (cb_) cb_((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - start_).count());
        }

    private:
        Clock::time_point start_;
        std::function<void(uint64_t)> cb_;
    };

    ScopedTimer createTrainingTimer() {
        return ScopedTimer([this](uint64_t ns) { recordTrainingTime(ns); });
    }
    ScopedTimer createSimulationTimer() {
        return ScopedTimer([this](uint64_t ns) { recordSimulationTime(ns); });
    }
    ScopedTimer createTransferTimer() {
        return ScopedTimer([this](uint64_t ns) { recordTransferTime(ns); });
    }
    ScopedTimer createSyncTimer() {
        return ScopedTimer([this](uint64_t ns) { recordSyncTime(ns); });
    }
    void recordTrainingTime(uint64_t ns) {
        if (running_.load()) training_ns_ += ns;
    }
    void recordSimulationTime(uint64_t ns) {
        if (running_.load()) simulation_ns_ += ns;
    }
    void recordTransferTime(uint64_t ns) {
        if (running_.load()) transfer_ns_ += ns;
    }
    void recordSyncTime(uint64_t ns) {
        if (running_.load()) sync_ns_ += ns;
    }
    // one agent iteration (agent.h:236, :290): the start time is the calling thread's own (:388)
    void startAgentIteration(size_t) {
        if (running_.load()) iter_start() = Clock::now();
    }
    void endAgentIteration(size_t agent_id) {
        if (!running_.load()) return;
        const uint64_t ns =
            (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - iter_start()).count();
        std::lock_guard<std::mutex> lk(mu_);
        AgentTimes& a = agents_[agent_id];
        a.total += ns;
        a.count++;
        a.min = std::min(a.min, ns);
        a.max = std::max(a.max, ns);
        iterations_++;
    }
    void recordLearnerModelUpdate() {
        if (running_.load()) model_updates_++;
    }
    void recordDataTransfer() {
        if (running_.load()) data_transfers_++;
    }
    void recordAgentModelSync() {
        if (running_.load()) agent_syncs_++;
    }
    // device learner: env-steps (T x B) trained by one step and its device time
    void recordLearnerEnvSteps(uint64_t env_steps, double device_ms) {
        if (!running_.load()) return;
        env_steps_ += env_steps;
        std::lock_guard<std::mutex> lk(mu_);
        device_ms_ += device_ms;
    }
    void recordLearnerRejectedBatch() {
        if (running_.load()) rejected_++;
    }

    uint64_t getTotalLearnerModelUpdates() const { return model_updates_.load(); }
    uint64_t getTotalDataTransfers() const { return data_transfers_.load(); }
    uint64_t getTotalAgentModelSyncs() const { return agent_syncs_.load(); }
    uint64_t getTotalTrainingTime() const { return training_ns_.load(); }
    uint64_t getTotalLearnerEnvSteps() const { return env_steps_.load(); }
    uint64_t getTotalRejectedBatches() const { return rejected_.load(); }
    double getTotalDeviceMs() const {
        std::lock_guard<std::mutex> lk(mu_);
        return device_ms_;
    }
    double getElapsedSeconds() const {
        const auto end = running_.load() ? Clock::now() : t1_;
        return std::chrono::duration<double>(end - t0_).count();
    }
    uint64_t getTotalExecutionTime() const { return (uint64_t)(getElapsedSeconds() * 1e9); }
    uint64_t getTotalIterations() const { return iterations_.load(); }
    uint64_t getTotalSimulationTime() const { return simulation_ns_.load(); }
    uint64_t getTotalTransferTime() const { return transfer_ns_.load(); }
    uint64_t getTotalSyncTime() const { return sync_ns_.load(); }
    double getIterationsPerSecond() const { return per_second(getTotalIterations()); }
    double getLearnerUpdatesPerSecond() const { return per_second(getTotalLearnerModelUpdates()); }
    double getAgentSyncsPerSecond() const { return per_second(getTotalAgentModelSyncs()); }
    double getDataTransfersPerSecond() const { return per_second(getTotalDataTransfers()); }
    double getLearnerEnvStepsPerSecond() const { return per_second(getTotalLearnerEnvSteps()); }
    // shares of the four timed activities, in percent (metrics_tracker.h:235-254)
    std::map<std::string, double> getTimeDistribution() const {
        const double sim = (double)getTotalSimulationTime(), tr = (double)getTotalTrainingTime(),
                     xf = (double)getTotalTransferTime(), sy = (double)getTotalSyncTime();
        const double tot = sim + tr + xf + sy;
        auto pct = [tot](double v) { return tot > 0 ? 100.0 * v / tot : 0.0; };
        return {{"simulation", pct(sim)}, {"training", pct(tr)}, {"transfer", pct(xf)}, {"sync", pct(sy)}};
    }

    // the reference's --metrics-file (metrics_tracker.h:265-329), then the device learner's rows
    bool saveMetricsToCSV(const std::string& filename) const {
        std::ofstream f(filename);
        if (!f) {
            std::fprintf(stderr, "Could not open file for writing: %s\n", filename.c_str());
            return false;
        }
        f << "Metric,Value\n";
        f << "TotalExecutionTime_ns," << getTotalExecutionTime() << "\n";
        f << "TotalSimulationTime_ns," << getTotalSimulationTime() << "\n";
        f << "TotalTrainingTime_ns," << getTotalTrainingTime() << "\n";
        f << "TotalTransferTime_ns," << getTotalTransferTime() << "\n";
        f << "TotalSyncTime_ns," << getTotalSyncTime() << "\n";
        f << "TotalIterations," << getTotalIterations() << "\n";
        f << "TotalLearnerModelUpdates," << getTotalLearnerModelUpdates() << "\n";
        f << "TotalAgentModelSyncs," << getTotalAgentModelSyncs() << "\n";
        f << "TotalDataTransfers," << getTotalDataTransfers() << "\n";
        f << "IterationsPerSecond," << getIterationsPerSecond() << "\n";
        f << "LearnerUpdatesPerSecond," << getLearnerUpdatesPerSecond() << "\n";
        f << "AgentSyncsPerSecond," << getAgentSyncsPerSecond() << "\n";
        f << "DataTransfersPerSecond," << getDataTransfersPerSecond() << "\n";
        for (const auto& [key, value] : getTimeDistribution()) f << "TimePercentage_" << key << "," << value << "\n";
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (const auto& [id, a] : agents_) {
                if (a.count == 0) continue;
                f << "Agent_" << id << "_TotalTime_ns," << a.total << "\n";
                f << "Agent_" << id << "_AvgIterationTime_ns," << (double)a.total / (double)a.count << "\n";
                f << "Agent_" << id << "_MinIterationTime_ns," << a.min << "\n";
                f << "Agent_" << id << "_MaxIterationTime_ns," << a.max << "\n";
            }
        }
        f << "TotalLearnerEnvSteps," << getTotalLearnerEnvSteps() << "\n";
        f << "LearnerEnvStepsPerSecond," << getLearnerEnvStepsPerSecond() << "\n";
        f << "TotalDeviceTime_ms," << getTotalDeviceMs() << "\n";
        f << "TotalRejectedBatches," << getTotalRejectedBatches() << "\n";
        return (bool)f;
    }

    // the reference's end-of-run report (metrics_tracker.h:332-382), then the device learner's
    void printMetricsSummary() const {
        std::string o = "\n===== Performance Metrics Summary =====\n";
        char b[160];
        auto line = [&](const char* fmt, double v) {
            std::snprintf(b, sizeof b, fmt, v);
            o += b;
        };
        line("Total Execution Time: %.3f seconds\n", getTotalExecutionTime() / 1e9);
        o += "\n--- Throughput Metrics ---\n";
        line("Iterations Per Second: %.2f\n", getIterationsPerSecond());
        line("Learner Model Updates Per Second: %.2f\n", getLearnerUpdatesPerSecond());
        line("Agent Model Syncs Per Second: %.2f\n", getAgentSyncsPerSecond());
        line("Data Transfers Per Second: %.2f\n", getDataTransfersPerSecond());
        o += "\n--- Time Distribution ---\n";
        for (const auto& [key, value] : getTimeDistribution()) {
            std::snprintf(b, sizeof b, "%s: %.1f%%\n", key.c_str(), value);
            o += b;
        }
        o += "\n--- Total Counts ---\n";
        o += "Total Iterations: " + std::to_string(getTotalIterations()) + "\n";
        o += "Total Learner Model Updates: " + std::to_string(getTotalLearnerModelUpdates()) + "\n";
        o += "Total Agent Model Syncs: " + std::to_string(getTotalAgentModelSyncs()) + "\n";
        o += "Total Data Transfers: " + std::to_string(getTotalDataTransfers()) + "\n";
        o += "\n--- Per-Agent Metrics ---\n";
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (const auto& [id, a] : agents_) {
                if (a.count == 0) continue;
                std::snprintf(b, sizeof b, "Agent %zu Avg Iteration Time: %.3f ms\n", id,
                              (double)a.total / (double)a.count / 1e6);
                o += b;
            }
        }
        o += "\n--- Device Learner ---\n";
        o += "Total Learner Env-Steps: " + std::to_string(getTotalLearnerEnvSteps()) + "\n";
        line("Learner Env-Steps Per Second: %.1f\n", getLearnerEnvStepsPerSecond());
        line("Device Time: %.3f ms\n", getTotalDeviceMs());
        o += "Rejected Batches: " + std::to_string(getTotalRejectedBatches()) + "\n";
        o += "=====================================\n";
        std::fputs(o.c_str(), stdout);
        std::fflush(stdout);
    }

    // one JSON object with every counter (the CLI prints it as its summary line)
    std::string summaryJson() const {
        char buf[512];
        const double s = getElapsedSeconds();
        const double tr = getTotalTrainingTime() * 1e-9;
        std::snprintf(buf, sizeof buf,
                      "{\"elapsed_s\": %.4f, \"learner_model_updates\": %llu, \"data_transfers\": %llu, "
                      "\"agent_model_syncs\": %llu, \"training_s\": %.4f, \"learner_env_steps\": %llu, "
                      "\"device_ms\": %.3f, \"rejected_batches\": %llu, \"env_steps_per_s_wall\": %.1f, "
                      "\"env_steps_per_s_training\": %.1f}",
                      s, (unsigned long long)getTotalLearnerModelUpdates(),
                      (unsigned long long)getTotalDataTransfers(), (unsigned long long)getTotalAgentModelSyncs(),
                      tr, (unsigned long long)getTotalLearnerEnvSteps(), getTotalDeviceMs(),
                      (unsigned long long)getTotalRejectedBatches(),
                      s > 0 ? getTotalLearnerEnvSteps() / s : 0.0, tr > 0 ? getTotalLearnerEnvSteps() / tr : 0.0);
        return buf;
    }

private:
    MetricsTracker() = default;
    struct AgentTimes {
        uint64_t total = 0, count = 0, min = std::numeric_limits<uint64_t>::max(), max = 0;
    };
    static Clock::time_point& iter_start() {
        thread_local Clock::time_point t{};
        return t;
    }
    double per_second(uint64_t n) const {
        const double s = getElapsedSeconds();
        return s > 0 ? (double)n / s : 0.0;
    }
    std::atomic<bool> running_{false};
    Clock::time_point t0_{}, t1_{};
    std::atomic<uint64_t> training_ns_{0}, simulation_ns_{0}, transfer_ns_{0}, sync_ns_{0}, model_updates_{0},
        data_transfers_{0}, agent_syncs_{0}, env_steps_{0}, rejected_{0}, iterations_{0};
    mutable std::mutex mu_;
    double device_ms_ = 0.0;
    std::map<size_t, AgentTimes> agents_;
};

}  // namespace freeimpala_amd
