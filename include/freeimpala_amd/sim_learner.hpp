// sim_learner.hpp -- the reference's placeholder learner (`--learner sim`), restated so BASELINE
// config #1 ("reference learner, no GPU") runs in the same binary as the device learner.
//
// Behaviour of reference include/freeimpala/learner.h, member by member:
//   * constructor (learner.h:100-140): ModelManager(p, 1 MiB, l) (:123-127), loadModels(m) when a
//     starting model is given (:130-132), one SharedBuffer(S, B) per player (:135-139);
//   * trainModel (:32-49): inside MetricsTracker::createTrainingTimer(), sleep r ms, copy the
//     player's model, refill the copy with random bytes (Model::generateRandomData, which also
//     bumps the version, data_structures.h:121-127), ModelManager::updateModel,
//     recordLearnerModelUpdate;
//   * workerThread (:72-97): readBatch(M); empty -> exit when stopping, else retry; train;
//     ++iteration; checkpoint every c iterations on a separate thread; stop at T;
//   * checkpointModel (:52-69), stop (:166-197): ModelManager::saveModel / saveAllModels(T).
// No device and no arithmetic on the batch (not the CPU checker either): the reference's timing
// model of a learner (the batch is read and dropped), kept for the behavioural baseline.
// Same surface as BasicLearner where the CLI uses it: start / stop / getSharedBuffers /
// getModelManager / iterations / config / param_bytes.
#pragma once

#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "freeimpala_amd/device_learner.hpp"  // LearnerConfig only (no device is touched)

namespace freeimpala_amd {

template <class Buffer, class Manager, class Metrics>
class SimLearner {
public:
    static constexpr size_t kModelBytes = 1 * 1024 * 1024;  // learner.h:125

    SimLearner(size_t p, size_t B, size_t S, size_t M, size_t r, size_t c, const std::string& l,
               const std::string& m, size_t T, LearnerConfig lc = LearnerConfig())
        : num_players_(p), batch_size_(M), train_time_ms_(r), checkpoint_frequency_(c),
          total_iterations_(T), iterations_(p) {
        lc.players = p;
        lc.batch_size = M;
        lc.entry_size = S;
        cfg_ = lc;
        model_manager_ = std::make_shared<Manager>(num_players_, kModelBytes, l);
        if (!m.empty()) model_manager_->loadModels(m);
        for (size_t q = 0; q < num_players_; ++q) shared_buffers_.push_back(std::make_shared<Buffer>(S, B));
    }
    ~SimLearner() {
        stop();
        std::lock_guard<std::mutex> lk(checkpoint_mutex_);
        for (auto& t : checkpoint_threads_)
            if (t.joinable()) t.join();
        checkpoint_threads_.clear();
    }
    SimLearner(const SimLearner&) = delete;
    SimLearner& operator=(const SimLearner&) = delete;

    void start() {
        for (size_t q = 0; q < num_players_; ++q) worker_threads_.emplace_back([this, q] { workerThread(q); });
    }

    void stop() {
        should_stop_.store(true);
        for (auto& b : shared_buffers_) b->setDraining();
        for (auto& t : worker_threads_)
            if (t.joinable()) t.join();
        worker_threads_.clear();
        if (!final_saved_.exchange(true)) model_manager_->saveAllModels(total_iterations_);
        std::lock_guard<std::mutex> lk(checkpoint_mutex_);
        for (auto& t : checkpoint_threads_)
            if (t.joinable()) t.join();
        checkpoint_threads_.clear();
    }

    std::vector<std::shared_ptr<Buffer>> getSharedBuffers() { return shared_buffers_; }
    std::shared_ptr<Manager> getModelManager() { return model_manager_; }
    size_t iterations(size_t p) const { return iterations_.at(p).load(); }
    bool workerFailed() const { return false; }  // no device: nothing fails
    const LearnerConfig& config() const { return cfg_; }
    size_t param_bytes() const { return kModelBytes; }

private:
    void trainModel(size_t p, const std::vector<std::vector<char>>& /*batch*/) {
        auto metrics = Metrics::getInstance();
        auto timer = metrics->createTrainingTimer();
        std::this_thread::sleep_for(std::chrono::milliseconds(train_time_ms_));
        auto next = model_manager_->getModel(p)->createCopy();
        next->generateRandomData();
        model_manager_->updateModel(p, next);
        metrics->recordLearnerModelUpdate();
    }

    void checkpointModel(size_t p, uint64_t it) {
        std::lock_guard<std::mutex> lk(checkpoint_mutex_);
        for (auto i = checkpoint_threads_.begin(); i != checkpoint_threads_.end();) {
            if (i->joinable()) {
                i->join();
                i = checkpoint_threads_.erase(i);
            } else {
                ++i;
            }
        }
        checkpoint_threads_.emplace_back([this, p, it] { model_manager_->saveModel(p, it); });
    }

    void workerThread(size_t p) {
        size_t n = 0;
        while (!should_stop_.load() && n < total_iterations_) {
            auto batch = shared_buffers_[p]->readBatch(batch_size_);
            if (batch.empty()) {
                if (should_stop_.load()) break;
                continue;
            }
            trainModel(p, batch);
            ++n;
            iterations_[p].store(n);
            if (checkpoint_frequency_ > 0 && n % checkpoint_frequency_ == 0) checkpointModel(p, n);
        }
    }

    size_t num_players_, batch_size_, train_time_ms_, checkpoint_frequency_, total_iterations_;
    LearnerConfig cfg_;
    std::vector<std::shared_ptr<Buffer>> shared_buffers_;
    std::shared_ptr<Manager> model_manager_;
    std::vector<std::thread> worker_threads_, checkpoint_threads_;
    std::atomic<bool> should_stop_{false}, final_saved_{false};
    std::mutex checkpoint_mutex_;
    std::vector<std::atomic<size_t>> iterations_;
};

}  // namespace freeimpala_amd
