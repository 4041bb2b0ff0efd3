// metrics.hpp -- the learner's counters of freeimpala's MetricsTracker, natively.
//
// Reference include/freeimpala/metrics_tracker.h: a process-wide singleton; counters only count
// between start() and stop(); createTrainingTimer() returns a scoped timer whose destructor
// adds the elapsed ns to the training time (:131-134, :146-169); recordLearnerModelUpdate()
// counts published models (:109-112). The learner step also reports what the device did:
// env-steps trained (T x B per step) and device milliseconds, so the summary can state
// env-steps/s next to the reference's counters.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <mutex>
#include <string>

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
    void recordTrainingTime(uint64_t ns) {
        if (running_.load()) training_ns_ += ns;
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
    std::atomic<bool> running_{false};
    Clock::time_point t0_{}, t1_{};
    std::atomic<uint64_t> training_ns_{0}, model_updates_{0}, data_transfers_{0}, agent_syncs_{0},
        env_steps_{0}, rejected_{0};
    mutable std::mutex mu_;
    double device_ms_ = 0.0;
};

}  // namespace freeimpala_amd
