// learner.hpp -- freeimpala's Learner with the step on the MI355X (drop-in for
// reference include/freeimpala/learner.h).
//
// Same surface as the reference class (learner.h:7-208):
//   Learner(p, B, S, M, r, c, l, m, T)   players, buffer capacity, entry size (elements), batch
//                                        size, learner time (ms), checkpoint frequency,
//                                        checkpoint location, starting model, total iterations
//                                        (+ an optional LearnerConfig: T, arch, lr, devices ...)
//   start() / stop() / getSharedBuffers() / getModelManager()
// plus the public step the north star asks for:
//   bool step(size_t player_index, const std::vector<std::vector<char>>& batch)
// with the parameters of the reference's private trainModel (learner.h:32-49). The worker
// loop keeps the reference's rules (learner.h:72-97): readBatch(M); an empty batch means
// "draining -> exit" or "spurious wake-up -> retry"; step; ++iteration; checkpoint every c
// iterations on a separate thread; stop at T iterations. stop() drains the buffers, joins the
// workers and saves every model as iteration T (learner.h:166-197).
//
// What changes inside:
//   * the step runs on the device (DeviceLearner over libfi_learner.so), and the published
//     Model blob holds the real parameters (fp32, or bf16 with --publish bf16) with the
//     learner's version -- ModelManager is sized from the parameter blob, not 1 MiB
//     (learner.h:123-127);
//   * when the buffer type offers readBatchInto (freeimpala_amd::SharedBuffer), the worker
//     copies the batch once, straight into the learner's pinned staging buffer; with the
//     reference SharedBuffer it uses readBatch + step() (the same result bit for bit);
//   * checkpoints keep the reference file format (<dir>/model_<p>_<iter>.bin and _latest.bin,
//     `u64 version || blob`) and add the optimizer state beside each file
//     (model_<p>_<iter>.state, model_<p>_latest.state: params + Adam moments + counters);
//     --starting-model resumes from the .state next to the loaded model file when it exists,
//     else from the model blob's weights;
//   * MetricsTracker: createTrainingTimer around the step and recordLearnerModelUpdate after
//     the publication (learner.h:33-48), plus env-steps (T x B per step) and device time when
//     the tracker has recordLearnerEnvSteps.
// Template over the buffer / model-manager / metrics types so the same code runs on the
// reference's own classes and on freeimpala_amd's (replay.hpp,
// metrics.hpp; `freeimpala_amd::Learner`). Construction throws std::runtime_error when the HIP
// library or device is unusable: there is no CPU fallback.
#pragma once

#include <atomic>
#include <cstring>
#include <cstdio>
#include <filesystem>
#include <functional>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "freeimpala_amd/device_learner.hpp"
#include "freeimpala_amd/metrics.hpp"
#include "freeimpala_amd/replay.hpp"

namespace freeimpala_amd {

namespace detail {
template <class B, class = void>
struct has_read_batch_into : std::false_type {};
template <class B>
struct has_read_batch_into<B, std::void_t<decltype(std::declval<B&>().readBatchInto(size_t{}, (char*)nullptr, size_t{}))>>
    : std::true_type {};
template <class M, class = void>
struct has_env_steps : std::false_type {};
template <class M>
struct has_env_steps<M, std::void_t<decltype(std::declval<M&>().recordLearnerEnvSteps(uint64_t{}, 0.0))>>
    : std::true_type {};
template <class M, class = void>
struct has_rejected : std::false_type {};
template <class M>
struct has_rejected<M, std::void_t<decltype(std::declval<M&>().recordLearnerRejectedBatch())>> : std::true_type {};

inline bool write_file_atomic(const std::string& path, const std::vector<char>& bytes) {
    const std::string tmp = path + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
        if (!f) return false;
        f.write(bytes.data(), (std::streamsize)bytes.size());
        if (!f) return false;
    }
    std::error_code ec;
    std::filesystem::rename(tmp, path, ec);
    return !ec;
}
inline bool read_file(const std::string& path, std::vector<char>& out) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return false;
    out.resize((size_t)f.tellg());
    f.seekg(0);
    f.read(out.data(), (std::streamsize)out.size());
    return (bool)f;
}
struct ModelSnapshot {
    uint64_t version;
    std::vector<char> blob;
};
inline std::string state_path_for(const std::string& model_file) {
    std::filesystem::path p(model_file);
    p.replace_extension(".state");
    return p.string();
}
}  // namespace detail

template <class Buffer, class Manager, class Metrics>
class BasicLearner {
public:
    BasicLearner(size_t p, size_t B, size_t S, size_t M, size_t r, size_t c, const std::string& l,
                 const std::string& m, size_t T, LearnerConfig lc = LearnerConfig())
        : num_players_(p), buffer_capacity_(B), entry_size_(S), batch_size_(M), train_time_ms_(r),
          checkpoint_frequency_(c), checkpoint_location_(l), starting_model_(m), total_iterations_(T),
          iterations_(p) {
        lc.players = p;
        lc.batch_size = M;
        lc.entry_size = S;
        if (lc.seq_length + 1 > S) {
            log("warn", "entry size " + std::to_string(S) + " holds at most " + std::to_string(S ? S - 1 : 0) +
                            " steps + bootstrap: seq_length lowered from " + std::to_string(lc.seq_length));
            lc.seq_length = S > 1 ? S - 1 : 1;
        }
        cfg_ = lc;
        device_ = std::make_unique<DeviceLearner>(cfg_);
        model_manager_ = std::make_shared<Manager>(num_players_, device_->param_bytes(), checkpoint_location_);
        for (size_t q = 0; q < num_players_; ++q) publish(q, /*count=*/false);  // actors start from the init weights
        if (!starting_model_.empty()) {
            model_manager_->loadModels(starting_model_);
            for (size_t q = 0; q < num_players_; ++q) resume(q);
        }
        for (size_t q = 0; q < num_players_; ++q)
            shared_buffers_.push_back(std::make_shared<Buffer>(entry_size_, buffer_capacity_));
    }

    virtual ~BasicLearner() { stop(); }
    BasicLearner(const BasicLearner&) = delete;
    BasicLearner& operator=(const BasicLearner&) = delete;

    void start() {
        for (size_t q = 0; q < num_players_; ++q) worker_threads_.emplace_back([this, q] { workerThread(q); });
    }

    void stop() {
        should_stop_.store(true);
        for (auto& b : shared_buffers_) b->setDraining();
        for (auto& t : worker_threads_)
            if (t.joinable()) t.join();
        worker_threads_.clear();
        std::lock_guard<std::mutex> lk(checkpoint_mutex_);
        for (auto& t : checkpoint_threads_)  // before the final save: both write the _latest files
            if (t.joinable()) t.join();
        checkpoint_threads_.clear();
        if (!final_saved_.exchange(true)) {
            log("info", "Performing final model save before exit");
            // workers are joined: the device state and the published model are read from this
            // thread (learner.h:186-196 saveAllModels(T), written from the same snapshot)
            for (size_t q = 0; q < num_players_; ++q) {
                std::vector<char> st;
                const bool have = save_state_sidecars(q, total_iterations_, &st);
                write_checkpoint(q, total_iterations_, snapshot(q), have ? &st : nullptr);
            }
        }
    }

    std::vector<std::shared_ptr<Buffer>> getSharedBuffers() { return shared_buffers_; }
    std::shared_ptr<Manager> getModelManager() { return model_manager_; }

    // Learner::step(player_index, batch): trainModel's parameters (learner.h:32), the device
    // step, then the new Model published through ModelManager::updateModel. false (logged,
    // nothing published) on a rejected batch or a device error.
    bool step(size_t player_index, const std::vector<std::vector<char>>& batch) {
        auto metrics = Metrics::getInstance();
        bool ok;
        {
            auto timer = metrics->createTrainingTimer();
            ok = device_->step(player_index, batch);
            if (ok) publish(player_index, true);
        }
        if (ok && observer_) observer_(player_index, device_->last_stats(player_index), device_->handle(player_index));
        if (!ok) rejected(player_index, device_->last_error(player_index));
        return ok;
    }

    // Verification hook: called on player p's worker thread after every successful step with
    // the step's statistics and the player's (first-shard) handle, before the next batch is
    // read -- the handle's tensors (e.g. "grads") still hold that step's values. Set before
    // start().
    using StepObserver = std::function<void(size_t, const fi_step_stats&, fi_learner*)>;
    void setStepObserver(StepObserver f) { observer_ = std::move(f); }

    // iterations completed by player p's worker
    size_t iterations(size_t p) const { return iterations_.at(p).load(); }
    DeviceLearner& device() { return *device_; }
    size_t param_bytes() const { return device_->param_bytes(); }
    const LearnerConfig& config() const { return cfg_; }
    size_t learnerTimeMs() const { return train_time_ms_; }  // accepted; the device step replaces the sleep
    // A worker ended on a device failure. Its buffer is then draining: blocked readers and (on
    // buffer types whose write honours draining, freeimpala_amd::SharedBuffer) blocked writers
    // return, so callers poll this flag instead of waiting for iterations that never come.
    bool workerFailed() const { return worker_failed_.load(); }

protected:
    // fi_learner_acquire_staging for the zero-copy worker path; virtual so a test can make it fail
    virtual int acquireStaging(fi_learner* h, void** dst, size_t* stride) {
        return fi_learner_acquire_staging(h, dst, stride);
    }

private:
    void workerThread(size_t player_index) {
        size_t iteration_count = 0;
        while (!should_stop_.load() && iteration_count < total_iterations_) {
            bool got = false;
            if constexpr (detail::has_read_batch_into<Buffer>::value) {
                if (device_->shards(player_index) == 1) {
                    const int r = step_zero_copy(player_index);
                    if (r < 0) break;  // the staging buffer is unusable: this worker stops (logged)
                    got = r > 0;
                } else {  // --data-parallel: readBatch, then the shards step concurrently
                    auto batch = shared_buffers_[player_index]->readBatch(batch_size_);
                    got = !batch.empty();
                    if (got) step(player_index, batch);
                }
            } else {
                auto batch = shared_buffers_[player_index]->readBatch(batch_size_);
                got = !batch.empty();
                if (got) step(player_index, batch);
            }
            if (!got) {  // draining with < M entries, or a spurious wake-up (learner.h:79-84)
                if (should_stop_.load()) break;
                continue;
            }
            ++iteration_count;
            iterations_[player_index].store(iteration_count);
            if (checkpoint_frequency_ > 0 && iteration_count % checkpoint_frequency_ == 0)
                checkpointModel(player_index, iteration_count);
        }
    }

    // readBatchInto the pinned staging buffer, then the step. Returns 1 when a batch was read
    // (stepped or rejected), 0 when none was (draining / spurious wake-up), -1 when the staging
    // buffer cannot be acquired: a device-side failure that retrying would only repeat, so the
    // worker ends (logged once) instead of spinning on it.
    int step_zero_copy(size_t p) {
        fi_learner* h = device_->handle(p);
        void* dst = nullptr;
        size_t stride = 0;
        if (acquireStaging(h, &dst, &stride) != FI_OK) {
            log("error", "player " + std::to_string(p) + ": acquire_staging failed, worker stops: " +
                             fi_last_error());
            worker_failed_.store(true);
            shared_buffers_[p]->setDraining();  // wake this player's readers and writers
            return -1;
        }
        if (!shared_buffers_[p]->readBatchInto(batch_size_, static_cast<char*>(dst), stride)) return 0;
        auto metrics = Metrics::getInstance();
        bool ok;
        fi_step_stats st{};
        {
            auto timer = metrics->createTrainingTimer();
            ok = fi_learner_step_staged(h, &st) == FI_OK;
            if (ok) publish(p, true, &st);
        }
        if (ok && observer_) observer_(p, st, h);
        if (!ok) rejected(p, fi_last_error());
        return 1;
    }

    void rejected(size_t p, const std::string& why) {
        auto metrics = Metrics::getInstance();
        if constexpr (detail::has_rejected<std::remove_reference_t<decltype(*metrics)>>::value)
            metrics->recordLearnerRejectedBatch();
        log("error", "learner step failed for player " + std::to_string(p) + ": " + why);
    }

    void publish(size_t p, bool count, const fi_step_stats* st = nullptr) {
        std::vector<char> blob;
        uint64_t version = 0;
        if (!device_->publish(p, blob, version)) {
            log("error", "publish failed for player " + std::to_string(p) + ": " + device_->last_error(p));
            return;
        }
        auto model = model_manager_->getModel(p)->createCopy();
        model->update(blob, version);
        model_manager_->updateModel(p, model);
        if (!count) return;
        auto metrics = Metrics::getInstance();
        metrics->recordLearnerModelUpdate();
        if constexpr (detail::has_env_steps<std::remove_reference_t<decltype(*metrics)>>::value) {
            const fi_step_stats& s = st ? *st : device_->last_stats(p);
            metrics->recordLearnerEnvSteps((uint64_t)cfg_.seq_length * cfg_.batch_size, s.step_ms);
        }
    }

    // --starting-model: optimizer state from the .state beside the loaded model file when it
    // exists, else the model blob's weights (a blob of another size is left alone)
    void resume(size_t p) {
        auto model = model_manager_->getModel(p);
        const std::string file = model->getFilePath();
        std::error_code ec;
        if (!std::filesystem::exists(file, ec)) return;
        std::vector<char> st;
        if (detail::read_file(detail::state_path_for(file), st)) {
            if (device_->load_state(p, st)) {
                log("info", "player " + std::to_string(p) + ": resumed learner state from " +
                                detail::state_path_for(file));
                publish(p, false);
                return;
            }
            log("warn", "player " + std::to_string(p) + ": ignoring " + detail::state_path_for(file) + ": " +
                            device_->last_error(p));
        }
        const std::vector<char> blob = model->getData();
        if (blob.size() == device_->param_bytes() && device_->load(p, blob, model->getVersion()))
            log("info", "player " + std::to_string(p) + ": resumed weights from " + file);
        else
            log("warn", "player " + std::to_string(p) + ": " + file + " does not hold this network's weights");
        publish(p, false);
    }

    bool save_state_sidecars(size_t p, uint64_t iteration, std::vector<char>* keep = nullptr) {
        std::vector<char> st;
        if (!device_->save_state(p, st)) {
            log("error", "save_state failed for player " + std::to_string(p) + ": " + device_->last_error(p));
            return false;
        }
        if (keep) {
            *keep = std::move(st);
            return true;
        }
        write_sidecars(p, iteration, st);
        return true;
    }
    void write_sidecars(size_t p, uint64_t iteration, const std::vector<char>& st) const {
        std::error_code ec;
        std::filesystem::create_directories(checkpoint_location_, ec);
        const std::string base = checkpoint_location_ + "/model_" + std::to_string(p) + "_";
        detail::write_file_atomic(base + std::to_string(iteration) + ".state", st);
        detail::write_file_atomic(base + "latest.state", st);
    }

    // The published model of player p (what actors see), copied under the Model's own lock.
    // On the worker thread that owns the device handle it is exactly the device state the
    // optimizer-state blob is read from, so the pair written below belongs to one iteration.
    std::shared_ptr<const detail::ModelSnapshot> snapshot(size_t p) {
        auto m = model_manager_->getModel(p)->createCopy();
        return std::make_shared<const detail::ModelSnapshot>(detail::ModelSnapshot{m->getVersion(), m->getData()});
    }

    // <dir>/model_<p>_<iter>.bin and model_<p>_latest.bin in the reference file format
    // (`u64 version || blob`, data_structures.h:105-110), plus the .state sidecars. Written
    // here from the snapshot instead of through Manager::saveModel: the reference's saveModel
    // re-creates the copy as a fresh Model before saving (data_structures.h:409-410), whose
    // constructor fills it with rand() bytes, so its checkpoint files never hold the trained
    // weights; and a saveModel on the checkpoint thread would read whatever version is current
    // then, not the one the optimizer state belongs to.
    void write_checkpoint(size_t p, uint64_t it, const std::shared_ptr<const detail::ModelSnapshot>& snap,
                          const std::vector<char>* state) const {
        std::vector<char> file(sizeof(uint64_t) + snap->blob.size());
        std::memcpy(file.data(), &snap->version, sizeof(uint64_t));
        std::memcpy(file.data() + sizeof(uint64_t), snap->blob.data(), snap->blob.size());
        std::error_code ec;
        std::filesystem::create_directories(checkpoint_location_, ec);
        const std::string base = checkpoint_location_ + "/model_" + std::to_string(p) + "_";
        if (!detail::write_file_atomic(base + std::to_string(it) + ".bin", file) ||
            !detail::write_file_atomic(base + "latest.bin", file)) {
            log("error", "Failed to save checkpoint for player " + std::to_string(p));
            return;
        }
        log("info", "Saved checkpoint for player " + std::to_string(p) + " at iteration " + std::to_string(it) +
                        " to " + base + std::to_string(it) + ".bin (version " + std::to_string(snap->version) + ")");
        if (state) write_sidecars(p, it, *state);
    }

    // learner.h:52-69: earlier checkpoint threads are joined, then a new one writes this
    // player's checkpoint. The model snapshot and the optimizer state are both taken here, on
    // the worker thread, so the .bin and the .state of one checkpoint hold the same iteration.
    void checkpointModel(size_t p, uint64_t it) {
        auto st = std::make_shared<std::vector<char>>();
        const bool have = save_state_sidecars(p, it, st.get());
        auto snap = snapshot(p);
        std::lock_guard<std::mutex> lk(checkpoint_mutex_);
        for (auto i = checkpoint_threads_.begin(); i != checkpoint_threads_.end();) {
            if (i->joinable()) {
                i->join();
                i = checkpoint_threads_.erase(i);
            } else {
                ++i;
            }
        }
        checkpoint_threads_.emplace_back(
            [this, p, it, st, have, snap] { write_checkpoint(p, it, snap, have ? st.get() : nullptr); });
    }

    static void log(const char* level, const std::string& m) {
        std::fprintf(stderr, "[learner] [%s] %s\n", level, m.c_str());
    }

    size_t num_players_, buffer_capacity_, entry_size_, batch_size_, train_time_ms_, checkpoint_frequency_;
    std::string checkpoint_location_, starting_model_;
    size_t total_iterations_;
    LearnerConfig cfg_;
    std::unique_ptr<DeviceLearner> device_;
    std::vector<std::shared_ptr<Buffer>> shared_buffers_;
    std::shared_ptr<Manager> model_manager_;
    std::vector<std::thread> worker_threads_, checkpoint_threads_;
    std::atomic<bool> should_stop_{false}, final_saved_{false}, worker_failed_{false};
    std::mutex checkpoint_mutex_;
    std::vector<std::atomic<size_t>> iterations_;
    StepObserver observer_;
};

// freeimpala_amd's own buffer / model store / metrics (replay.hpp, metrics.hpp)
using Learner = BasicLearner<SharedBuffer, ModelManager, MetricsTracker>;

}  // namespace freeimpala_amd
