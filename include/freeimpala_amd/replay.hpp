// replay.hpp -- the learner-side replay buffer and model store of freeimpala, natively, with
// the reference's class names, method signatures and semantics, plus the zero-copy read the
// device learner needs.
//
//   SharedBuffer  reference include/freeimpala/data_structures.h:191-307
//     ring of `capacity` entries of entry_size * ELEMENT_SIZE bytes; write blocks while full,
//     try_write never blocks; readBatch(M) waits for M entries (or draining), returns {} when
//     draining with fewer than M, else pops M entries FIFO (copies, :267-300).
//     NEW readBatchInto(M, dst, stride): the same wait / drain / FIFO rules, but the M entries
//     are copied once, straight into `dst` (the learner's pinned staging buffer), instead of
//     into M fresh vectors -- SURVEY.md 8(f) rank 1.
//     Storage is one contiguous slab (capacity * entry bytes) rather than a vector per entry.
//   Model         data_structures.h:43-157: bytes + version + file path; file format
//                 `u64 version (little endian) || blob` (:72-77, :105-110).
//   ModelManager  data_structures.h:310-481: one Model per player, updateModel swaps the
//                 pointer and wakes waiters, checkpoints as <dir>/model_<p>_<iter>.bin plus
//                 <dir>/model_<p>_latest.bin, loadModels(dir) takes _latest or else the highest
//                 numbered checkpoint (:337-385).
// Header-only, C++17, no dependencies beyond the standard library.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <string>
#include <vector>

namespace freeimpala_amd {

// Size of one per-step record / buffer element (reference data_structures.h:35).
constexpr size_t ELEMENT_SIZE = 1024;

// MPI message tags of the freeimpala_mpi_* binaries (reference data_structures.h:21-32).
enum MessageTag : int {
    TAG_TRAJECTORY_BASE = 100,  // + player index; payload: one buffer entry
    TAG_VERSION_REQ = 200,      // uint32 player index
    TAG_WEIGHTS_REQ = 210,      // uint32 player index
    TAG_VERSION_RES = 201,      // uint64 latest version
    TAG_WEIGHTS_RES = 211,      // uint64 version || weights blob
    TAG_TERMINATE = 999
};

inline void log_line(const char* level, const std::string& msg) {
    std::fprintf(stderr, "[freeimpala_amd] [%s] %s\n", level, msg.c_str());
}

class SharedBuffer {
public:
    SharedBuffer(size_t entry_size, size_t buffer_capacity)
        : entry_bytes_(entry_size * ELEMENT_SIZE),
          capacity_(buffer_capacity),
          slab_(entry_bytes_ * buffer_capacity, 0),
          filled_(buffer_capacity, 0) {}

    // Wake every blocked reader and writer; readers then get {} / false unless a full batch
    // is still there (reference data_structures.h:212-216).
    void setDraining() {
        draining_.store(true);
        not_empty_.notify_all();
        not_full_.notify_all();
    }

    // Blocking enqueue; false when the data is larger than an entry, or when the buffer is
    // full and draining. The reference's write waits for space even while draining
    // (data_structures.h:223), so a writer on a full buffer whose reader has stopped blocks
    // forever; here setDraining releases it (a learner worker that fails drains its buffer).
    bool write(const std::vector<char>& data) { return write(data.data(), data.size()); }
    bool write(const char* data, size_t n) {
        std::unique_lock<std::mutex> lk(mu_);
        not_full_.wait(lk, [this] { return count_ < capacity_ || draining_.load(); });
        if (count_ >= capacity_) return false;
        return push_locked(lk, data, n);
    }

    // Non-blocking enqueue: false if the lock is busy or the buffer is full.
    bool try_write(const std::vector<char>& data) {
        std::unique_lock<std::mutex> lk(mu_, std::try_to_lock);
        if (!lk.owns_lock() || count_ >= capacity_) return false;
        return push_locked(lk, data.data(), data.size());
    }

    std::vector<std::vector<char>> readBatch(size_t batch_size) {
        std::unique_lock<std::mutex> lk(mu_);
        if (!wait_batch(lk, batch_size)) return {};
        std::vector<std::vector<char>> batch;
        batch.reserve(batch_size);
        for (size_t i = 0; i < batch_size; ++i) {
            const char* src = slab_.data() + read_index_ * entry_bytes_;
            batch.emplace_back(src, src + entry_bytes_);
            pop_locked();
        }
        lk.unlock();
        not_full_.notify_all();
        return batch;
    }

    // Zero-copy form of readBatch: entry i's first `stride` bytes go to dst + i * stride
    // (stride <= entry bytes). Returns false exactly when readBatch would return {}.
    bool readBatchInto(size_t batch_size, char* dst, size_t stride) {
        if (stride > entry_bytes_) return false;
        std::unique_lock<std::mutex> lk(mu_);
        if (!wait_batch(lk, batch_size)) return false;
        for (size_t i = 0; i < batch_size; ++i) {
            std::memcpy(dst + i * stride, slab_.data() + read_index_ * entry_bytes_, stride);
            pop_locked();
        }
        lk.unlock();
        not_full_.notify_all();
        return true;
    }

    size_t getFilledCount() {
        std::lock_guard<std::mutex> lk(mu_);
        return count_;
    }
    size_t entryBytes() const { return entry_bytes_; }
    size_t capacity() const { return capacity_; }

private:
    bool push_locked(std::unique_lock<std::mutex>& lk, const char* data, size_t n) {
        if (n > entry_bytes_) return false;
        std::memcpy(slab_.data() + write_index_ * entry_bytes_, data, n);
        filled_[write_index_] = 1;
        write_index_ = (write_index_ + 1) % capacity_;
        ++count_;
        lk.unlock();
        not_empty_.notify_one();
        return true;
    }
    // waits for a full batch or draining; false = no batch (draining with fewer than M)
    bool wait_batch(std::unique_lock<std::mutex>& lk, size_t batch_size) {
        not_empty_.wait(lk, [&] { return count_ >= batch_size || draining_.load(); });
        return !(draining_.load() && count_ < batch_size);
    }
    void pop_locked() {
        filled_[read_index_] = 0;
        read_index_ = (read_index_ + 1) % capacity_;
        --count_;
    }

    const size_t entry_bytes_;
    const size_t capacity_;
    std::vector<char> slab_;
    std::vector<uint8_t> filled_;
    std::mutex mu_;
    std::condition_variable not_full_, not_empty_;
    size_t write_index_ = 0, read_index_ = 0, count_ = 0;
    std::atomic<bool> draining_{false};
};

class Model {
public:
    // The reference fills a new model with random bytes (data_structures.h:52-59); the device
    // learner overwrites it with its initial parameters before any actor reads it.
    Model(size_t size_bytes, const std::string& path) : data_(size_bytes, 0), filepath_(path) {
        generateRandomData();
    }

    // `u64 version || blob`; false if the file is missing or shorter than the blob
    bool loadFromDisk() {
        std::ifstream f(filepath_, std::ios::binary);
        if (!f) return false;
        uint64_t v = 0;
        f.read(reinterpret_cast<char*>(&v), sizeof(v));
        std::vector<char> d(data_.size());
        f.read(d.data(), (std::streamsize)d.size());
        if (!f) return false;
        std::lock_guard<std::mutex> lk(mu_);
        data_.swap(d);
        version_.store(v);
        return true;
    }

    bool saveToDisk() {
        if (filepath_.empty()) {
            log_line("error", "Cannot save model with empty filepath");
            return false;
        }
        const auto dir = std::filesystem::path(filepath_).parent_path();
        std::error_code ec;
        if (!dir.empty()) std::filesystem::create_directories(dir, ec);
        // write-then-rename, so a reader (or a crash) never sees a half-written checkpoint
        const std::string tmp = filepath_ + ".tmp";
        {
            std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
            if (!f) {
                log_line("info", "Could not open file for writing: " + tmp);
                return false;
            }
            const uint64_t v = version_.load();
            std::lock_guard<std::mutex> lk(mu_);
            f.write(reinterpret_cast<const char*>(&v), sizeof(v));
            f.write(data_.data(), (std::streamsize)data_.size());
            if (!f) return false;
        }
        std::filesystem::rename(tmp, filepath_, ec);
        return !ec;
    }

    std::string getFilePath() const { return filepath_; }

    void generateRandomData() {
        std::lock_guard<std::mutex> lk(mu_);
        std::mt19937 rng((uint32_t)std::chrono::steady_clock::now().time_since_epoch().count());
        for (auto& c : data_) c = (char)(rng() & 0xff);
        version_++;
    }

    uint64_t getVersion() const { return version_.load(); }

    std::vector<char> getData() const {
        std::lock_guard<std::mutex> lk(mu_);
        return data_;
    }

    // Same rule as the reference (data_structures.h:141-147): a blob of another size is ignored.
    void update(const std::vector<char>& new_data, std::optional<uint64_t> new_version = std::nullopt) {
        std::lock_guard<std::mutex> lk(mu_);
        if (new_data.size() != data_.size()) return;
        data_ = new_data;
        version_ = new_version.has_value() ? *new_version : version_.load() + 1;
    }

    // a model holding `data` at `version` (no random fill)
    static std::shared_ptr<Model> fromData(const std::string& path, std::vector<char> data, uint64_t version) {
        auto m = std::make_shared<Model>(0, path);
        m->data_ = std::move(data);
        m->version_.store(version);
        return m;
    }

    std::shared_ptr<Model> createCopy() const {
        auto c = std::make_shared<Model>(0, filepath_);
        std::lock_guard<std::mutex> lk(mu_);
        c->data_ = data_;
        c->version_.store(version_.load());
        return c;
    }

private:
    std::vector<char> data_;
    std::atomic<uint64_t> version_{0};
    std::string filepath_;
    mutable std::mutex mu_;
};

class ModelManager {
public:
    ModelManager(size_t num_players, size_t model_size, const std::string& directory)
        : models_(num_players), mu_(num_players), updated_(num_players), latest_(num_players),
          dir_(directory), ckpt_counter_(num_players) {
        for (size_t p = 0; p < num_players; ++p) {
            models_[p] = std::make_shared<Model>(model_size, latest_path(dir_, p));
            latest_[p].store(models_[p]->getVersion());
        }
    }

    static std::string latest_path(const std::string& dir, size_t p) {
        return dir + "/model_" + std::to_string(p) + "_latest.bin";
    }
    static std::string iter_path(const std::string& dir, size_t p, uint64_t iter) {
        return dir + "/model_" + std::to_string(p) + "_" + std::to_string(iter) + ".bin";
    }

    // --starting-model: model_<p>_latest.bin, or the highest numbered model_<p>_<n>.bin when
    // there is no _latest file (then checkpoints continue from n + 1).
    void loadModels(const std::string& model_path) {
        if (model_path.empty()) return;
        namespace fs = std::filesystem;
        for (size_t p = 0; p < models_.size(); ++p) {
            std::string path = latest_path(model_path, p);
            std::error_code ec;
            if (fs::exists(model_path, ec) && !fs::exists(path, ec)) {
                const std::string prefix = "model_" + std::to_string(p) + "_";
                uint64_t best = 0;
                std::string best_file;
                for (const auto& e : fs::directory_iterator(model_path, ec)) {
                    const std::string name = e.path().filename().string();
                    if (name.rfind(prefix, 0) != 0) continue;
                    const size_t end = name.find(".bin");
                    if (end == std::string::npos || end + 4 != name.size()) continue;
                    const std::string num = name.substr(prefix.size(), end - prefix.size());
                    if (num.empty() || num.find_first_not_of("0123456789") != std::string::npos) continue;
                    const uint64_t n = std::stoull(num);
                    if (n > best) {
                        best = n;
                        best_file = e.path().string();
                    }
                }
                if (!best_file.empty()) {
                    path = best_file;
                    ckpt_counter_[p] = best + 1;
                    log_line("info", "Found highest checkpoint for player " + std::to_string(p) + ": " + path);
                }
            }
            auto m = std::make_shared<Model>(models_[p]->getData().size(), path);
            if (m->loadFromDisk()) {
                std::lock_guard<std::mutex> lk(mu_[p]);
                models_[p] = m;
                latest_[p].store(m->getVersion());
                log_line("info", "Loaded model " + std::to_string(p) + " from disk, version: " +
                                     std::to_string(m->getVersion()));
            }
        }
    }

    // Checkpoint: <dir>/model_<p>_<iter>.bin (iter 0: the next internal counter) and
    // <dir>/model_<p>_latest.bin, both `u64 version || blob`. Returns the versioned path
    // ("" on failure).
    // Thread-safe where the reference is not (data_structures.h:395,402 read models[p] and the
    // checkpoint counter unlocked): the model is read under the player's lock (getModel) and the
    // counter is atomic, so checkpoint threads may save while the worker publishes
    // (tests/cpp/race_check.cpp under ThreadSanitizer).
    std::string saveModel(size_t player_index, uint64_t current_iteration = 0) {
        const auto cur = getModel(player_index);
        if (!cur) {
            log_line("error", "Invalid model index or null model: " + std::to_string(player_index));
            return "";
        }
        const auto snap = cur->createCopy();
        const uint64_t it = current_iteration > 0 ? current_iteration : ckpt_counter_[player_index].fetch_add(1);
        const std::string vpath = iter_path(dir_, player_index, it);
        const std::vector<char> blob = snap->getData();
        if (!Model::fromData(vpath, blob, snap->getVersion())->saveToDisk()) {
            log_line("error", "Failed to save checkpoint for player " + std::to_string(player_index));
            return "";
        }
        Model::fromData(latest_path(dir_, player_index), blob, snap->getVersion())->saveToDisk();
        log_line("info", "Saved checkpoint for player " + std::to_string(player_index) + " at iteration " +
                             std::to_string(it) + " to " + vpath);
        return vpath;
    }

    void saveAllModels(uint64_t current_iteration = 0) {
        for (size_t p = 0; p < models_.size(); ++p) saveModel(p, current_iteration);
    }

    std::shared_ptr<Model> getModel(size_t player_index) {
        if (player_index >= models_.size()) return nullptr;
        std::lock_guard<std::mutex> lk(mu_[player_index]);
        return models_[player_index];
    }

    void updateModel(size_t player_index, const std::shared_ptr<Model>& new_model) {
        if (player_index >= models_.size()) return;
        {
            std::lock_guard<std::mutex> lk(mu_[player_index]);
            models_[player_index] = new_model;
            latest_[player_index].store(new_model->getVersion());
        }
        updated_[player_index].notify_all();
    }

    bool waitForModelUpdate(size_t player_index, uint64_t current_version, int timeout_ms) {
        if (player_index >= models_.size()) return false;
        std::unique_lock<std::mutex> lk(mu_[player_index]);
        return updated_[player_index].wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] {
            return latest_[player_index].load() > current_version;
        });
    }

    uint64_t getLatestVersion(size_t player_index) {
        return player_index < latest_.size() ? latest_[player_index].load() : 0;
    }
    size_t numPlayers() const { return models_.size(); }
    const std::string& directory() const { return dir_; }

private:
    std::vector<std::shared_ptr<Model>> models_;
    std::vector<std::mutex> mu_;
    std::vector<std::condition_variable> updated_;
    std::vector<std::atomic<uint64_t>> latest_;
    std::string dir_;
    std::vector<std::atomic<uint64_t>> ckpt_counter_;
};

}  // namespace freeimpala_amd
