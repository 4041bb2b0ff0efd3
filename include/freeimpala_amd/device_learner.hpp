// device_learner.hpp -- C++ host side of the MI355X learner step, above the C ABI.
//
// What the reference's Learner needs to move its step on-device, with the reference's
// own vocabulary and signatures:
//   * LearnerConfig::from_args   -- the learner flags of cmd/freeimpala (reference
//     cmd/freeimpala/main.cpp: --players, --batch-size, --seq-length, --entry-size) plus
//     the device-learner hyper-parameters (--learner-arch, --num-actions, --lr, ...).
//   * DeviceLearner::step(player_index, batch) -- same parameters as
//     Learner::trainModel (reference include/freeimpala/learner.h:32) and the same
//     `batch` that SharedBuffer::readBatch returns (data_structures.h:267-300):
//     M entries of S * ELEMENT_SIZE bytes, record schema in DESIGN.md section 3.
//   * DeviceLearner::publish(player_index, blob, version) -- the bytes and version that go
//     into Model::update / ModelManager::updateModel (data_structures.h:141-148, 441-451);
//     blob size == param_bytes() is the ModelManager model_size.
// One fi_learner handle per player (the reference runs one worker thread per player,
// learner.h:158-163): handles own their HIP stream and device memory, so different
// players may call step() concurrently from their own threads. Failures never throw
// across step(): it returns false and last_error() holds the message, matching the
// reference's log-and-continue style (data_structures.h:420-421). Construction throws
// std::runtime_error when the HIP library or device is unusable -- there is no CPU
// fallback.
#pragma once

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fi_learner.h"

namespace freeimpala_amd {

struct LearnerConfig {
    size_t players = 1;        // --players
    size_t batch_size = 32;    // --batch-size (M entries per step)
    size_t seq_length = 100;   // --seq-length (T); entries carry T+1 records
    size_t entry_size = 0;     // --entry-size in ELEMENT_SIZE units (0: T+1)
    std::string arch = "mlp";  // --learner-arch mlp|atari
    int num_actions = 18;      // --num-actions
    int obs_dim = 128;         // --obs-dim
    int hidden = 256;          // --hidden
    std::string optimizer = "adam";  // --optimizer adam|sgd
    std::string publish = "fp32";    // --publish fp32|bf16
    float lr = 5e-4f;          // --lr  (reference README.md:112 default)
    float max_grad_norm = 40.f;      // --max-grad-norm
    float gamma = 0.99f;       // --gamma (synthetic generator only)
    fi_vtrace_hparams hp{1.f, 1.f, 1.f, 1.f, 0.5f, 0.01f};
    std::vector<int> devices{0};     // --devices 0,1,... (player p -> devices[p % n])
    size_t data_parallel = 1;  // --data-parallel G: each player's batch split over G devices
                               // (shard g of player p on devices[(p G + g) % n]; RCCL all-reduce)
    uint64_t seed = 42;        // --seed (parameter init)

    size_t entry_records() const { return entry_size ? entry_size : seq_length + 1; }

    // Parses the flags above from argv (unknown flags are ignored so the reference's own
    // parser can own the rest of the command line). Throws std::invalid_argument on a
    // malformed value.
    static LearnerConfig from_args(int argc, const char* const* argv) {
        return from_args(argc, argv, LearnerConfig());
    }
    static LearnerConfig from_args(int argc, const char* const* argv, LearnerConfig c) {
        auto num = [](const std::string& f, const char* v) -> double {
            char* end = nullptr;
            const double x = std::strtod(v, &end);
            if (!v[0] || (end && *end)) throw std::invalid_argument("bad value for " + f + ": " + v);
            return x;
        };
        for (int i = 1; i + 1 < argc; ++i) {
            const std::string f = argv[i];
            const char* v = argv[i + 1];
            bool used = true;
            if (f == "--players" || f == "-p") c.players = (size_t)num(f, v);
            else if (f == "--batch-size" || f == "-M") c.batch_size = (size_t)num(f, v);
            else if (f == "--seq-length") c.seq_length = (size_t)num(f, v);
            else if (f == "--entry-size" || f == "-S") c.entry_size = (size_t)num(f, v);
            else if (f == "--learner-arch") c.arch = v;
            else if (f == "--num-actions") c.num_actions = (int)num(f, v);
            else if (f == "--obs-dim") c.obs_dim = (int)num(f, v);
            else if (f == "--hidden") c.hidden = (int)num(f, v);
            else if (f == "--optimizer") c.optimizer = v;
            else if (f == "--publish") c.publish = v;
            else if (f == "--lr") c.lr = (float)num(f, v);
            else if (f == "--max-grad-norm") c.max_grad_norm = (float)num(f, v);
            else if (f == "--gamma") c.gamma = (float)num(f, v);
            else if (f == "--seed") c.seed = (uint64_t)num(f, v);
            else if (f == "--data-parallel") c.data_parallel = (size_t)num(f, v);
            else if (f == "--devices") {
                c.devices.clear();
                std::string s = v;
                size_t p = 0;
                while (p <= s.size()) {
                    const size_t q = s.find(',', p);
                    const std::string tok = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
                    if (!tok.empty()) c.devices.push_back((int)num(f, tok.c_str()));
                    if (q == std::string::npos) break;
                    p = q + 1;
                }
                if (c.devices.empty()) throw std::invalid_argument("--devices: empty list");
            } else used = false;
            if (used) ++i;
        }
        if (c.players == 0 || c.batch_size == 0 || c.seq_length == 0)
            throw std::invalid_argument("--players, --batch-size and --seq-length must be > 0");
        if (c.entry_records() < c.seq_length + 1)
            throw std::invalid_argument("--entry-size must hold seq_length + 1 records");
        if (c.arch != "mlp" && c.arch != "atari") throw std::invalid_argument("--learner-arch: mlp|atari");
        if (c.optimizer != "adam" && c.optimizer != "sgd") throw std::invalid_argument("--optimizer: adam|sgd");
        if (c.publish != "fp32" && c.publish != "bf16") throw std::invalid_argument("--publish: fp32|bf16");
        if (c.data_parallel == 0 || c.batch_size % c.data_parallel != 0)
            throw std::invalid_argument("--data-parallel must divide --batch-size");
        return c;
    }

    // Learner flags through a strict parser (freeimpala_amd::ArgumentParser or the argparse
    // library of the reference binaries): the reference's own -p/--players, -M/--batch-size and
    // -S/--entry-size (registered by its setupArgumentParser, cmd/freeimpala/main.cpp:45-72)
    // plus the flags add_learner_arguments() registers. Throws std::invalid_argument.
    // (two overloads, not a defaulted `LearnerConfig()` argument: clang rejects a default
    // argument that needs the class's member initializers inside the class definition)
    template <class Parser>
    static LearnerConfig from_parser(const Parser& program) {
        return from_parser(program, LearnerConfig());
    }
    template <class Parser>
    static LearnerConfig from_parser(const Parser& program, LearnerConfig c) {
        auto num = [](const std::string& f, const std::string& v) -> double {
            char* end = nullptr;
            const double x = std::strtod(v.c_str(), &end);
            if (v.empty() || (end && *end)) throw std::invalid_argument("bad value for " + f + ": " + v);
            return x;
        };
        auto str = [&](const char* f) { return program.template get<std::string>(f); };
        c.players = (size_t)program.template get<int>("--players");
        c.batch_size = (size_t)program.template get<int>("--batch-size");
        c.entry_size = (size_t)program.template get<int>("--entry-size");
        c.seq_length = (size_t)num("--seq-length", str("--seq-length"));
        c.arch = str("--learner-arch");
        c.num_actions = (int)num("--num-actions", str("--num-actions"));
        c.obs_dim = (int)num("--obs-dim", str("--obs-dim"));
        c.hidden = (int)num("--hidden", str("--hidden"));
        c.optimizer = str("--optimizer");
        c.publish = str("--publish");
        c.lr = (float)num("--lr", str("--lr"));
        c.max_grad_norm = (float)num("--max-grad-norm", str("--max-grad-norm"));
        c.gamma = (float)num("--gamma", str("--gamma"));
        c.seed = (uint64_t)num("--learner-seed", str("--learner-seed"));
        c.data_parallel = (size_t)num("--data-parallel", str("--data-parallel"));
        const char* argv[] = {"", "--devices", nullptr};
        const std::string dev = str("--devices");
        argv[2] = dev.c_str();
        // (validation as from_args; an entry size too small for seq_length + 1 records is left
        // to the Learner, which lowers seq_length with a warning)
        LearnerConfig v = c;
        v.entry_size = 0;
        c.devices = from_args(3, argv, v).devices;
        return c;
    }

    // The C-ABI configuration of player p's handle (shard g of it under --data-parallel: the
    // same seed, so every replica starts from the same parameters).
    fi_learner_config abi_config(size_t p, size_t g = 0) const {
        fi_learner_config k;
        fi_learner_config_init(&k);
        k.arch = arch == "atari" ? FI_ARCH_ATARI : FI_ARCH_MLP;
        k.seq_len = (int32_t)seq_length;
        k.batch = (int32_t)(batch_size / data_parallel);
        k.num_actions = num_actions;
        k.obs_dim = obs_dim;
        k.hidden = hidden;
        k.optimizer = optimizer == "sgd" ? FI_OPT_SGD : FI_OPT_ADAM;
        k.publish_dtype = publish == "bf16" ? FI_PUBLISH_BF16 : FI_PUBLISH_FP32;
        k.device = devices[(p * data_parallel + g) % devices.size()];
        k.gamma = gamma;
        k.hp = hp;
        k.lr = lr;
        k.max_grad_norm = max_grad_norm;
        k.seed = seed + p;
        return k;
    }
};

// Registers the device-learner flags with a strict parser (string-valued, so the same calls
// work on argparse::ArgumentParser); values are checked by LearnerConfig::from_parser. --seed
// stays the reference's own (rand() seeding, main.cpp:111-114): parameter init is
// --learner-seed.
template <class Parser>
void add_learner_arguments(Parser& program) {
    const LearnerConfig d;
    program.add_argument("--seq-length").help("Trajectory length T (entries carry T+1 records)")
        .default_value(std::to_string(d.seq_length));
    program.add_argument("--learner-arch").help("Policy network: mlp | atari").default_value(d.arch);
    program.add_argument("--num-actions").help("Number of actions A").default_value(std::to_string(d.num_actions));
    program.add_argument("--obs-dim").help("MLP observation width (<= 128)").default_value(std::to_string(d.obs_dim));
    program.add_argument("--hidden").help("MLP hidden width").default_value(std::to_string(d.hidden));
    program.add_argument("--optimizer").help("adam | sgd").default_value(d.optimizer);
    program.add_argument("--publish").help("Published weights dtype: fp32 | bf16").default_value(d.publish);
    program.add_argument("--lr").help("Learning rate").default_value(std::string("0.0005"));
    program.add_argument("--max-grad-norm").help("Global-norm gradient clip (<= 0: off)")
        .default_value(std::string("40"));
    program.add_argument("--gamma").help("Discount of the synthetic trajectories").default_value(std::string("0.99"));
    program.add_argument("--learner-seed").help("Parameter-initialisation seed").default_value(std::to_string(d.seed));
    program.add_argument("--devices").help("HIP devices, comma separated (player p -> devices[p % n])")
        .default_value(std::string("0"));
    program.add_argument("--data-parallel").help("Devices per player: the batch is split over them, RCCL all-reduce")
        .default_value(std::string("1"));
}

class DeviceLearner {
public:
    explicit DeviceLearner(const LearnerConfig& cfg) : cfg_(cfg), stats_(cfg.players), err_(cfg.players) {
        if (fi_abi_version() != FI_ABI_VERSION)
            throw std::runtime_error("libfi_learner ABI version mismatch");
        const size_t G = cfg.data_parallel ? cfg.data_parallel : 1;
        handles_.resize(cfg.players, nullptr);
        shards_.assign(cfg.players, std::vector<fi_learner*>(G, nullptr));
        for (size_t p = 0; p < cfg.players; ++p) {
            for (size_t g = 0; g < G; ++g) {
                const fi_learner_config k = cfg.abi_config(p, g);
                if (fi_learner_create(&k, &shards_[p][g]) != FI_OK) {
                    const std::string msg = std::string("fi_learner_create(player ") + std::to_string(p) +
                                            ", shard " + std::to_string(g) + "): " + fi_last_error();
                    release();
                    throw std::runtime_error(msg);
                }
            }
            handles_[p] = shards_[p][0];
            // one RCCL communicator per player over its G devices: the in-step all-reduce sums
            // the shards' gradients, every replica applies the same update
            if (G > 1 && fi_comm_init_all(shards_[p].data(), (int)G) != FI_OK) {
                const std::string msg = std::string("fi_comm_init_all(player ") + std::to_string(p) + "): " + fi_last_error();
                release();
                throw std::runtime_error(msg);
            }
        }
    }
    ~DeviceLearner() { release(); }
    DeviceLearner(const DeviceLearner&) = delete;
    DeviceLearner& operator=(const DeviceLearner&) = delete;

    // Learner::step(player_index, batch): the body of Learner::trainModel on the device.
    bool step(size_t player_index, const std::vector<std::vector<char>>& batch) {
        if (player_index >= handles_.size()) return fail(0, "player_index out of range");
        if (batch.empty()) return fail(player_index, "empty batch");
        const size_t eb = batch[0].size();
        std::vector<const void*> ptrs(batch.size());
        for (size_t i = 0; i < batch.size(); ++i) {
            if (batch[i].size() != eb) return fail(player_index, "entries of different sizes");
            ptrs[i] = batch[i].data();
        }
        if (shards_[player_index].size() > 1) return step_sharded(player_index, ptrs, eb);
        fi_step_stats st{};
        if (fi_learner_step(handles_[player_index], ptrs.data(), ptrs.size(), eb, &st) != FI_OK)
            return fail(player_index, fi_last_error());
        stats_[player_index] = st;
        return true;
    }

    // Asynchronous step: returns once the batch is copied into pinned memory (the caller may
    // drop it and block in readBatch for the next one); wait() completes it.
    bool step_async(size_t player_index, const std::vector<std::vector<char>>& batch) {
        if (player_index >= handles_.size()) return fail(0, "player_index out of range");
        if (shards_[player_index].size() > 1) return fail(player_index, "step_async: not with --data-parallel > 1");
        if (batch.empty()) return fail(player_index, "empty batch");
        const size_t eb = batch[0].size();
        std::vector<const void*> ptrs(batch.size());
        for (size_t i = 0; i < batch.size(); ++i) {
            if (batch[i].size() != eb) return fail(player_index, "entries of different sizes");
            ptrs[i] = batch[i].data();
        }
        if (fi_learner_step_async(handles_[player_index], ptrs.data(), ptrs.size(), eb) != FI_OK)
            return fail(player_index, fi_last_error());
        return true;
    }
    // Zero-copy step: fill(dst, entry_stride, n) writes n entries straight into the pinned
    // staging buffer (SharedBuffer::readBatchInto, under the buffer's own mutex) and returns
    // false when there is no batch (draining, data_structures.h:278-280): then nothing is
    // submitted and the same buffer is handed out next time. async as in step_async.
    template <class Fill>
    bool step_staged(size_t player_index, Fill&& fill, bool async = false) {
        if (player_index >= handles_.size()) return fail(0, "player_index out of range");
        if (shards_[player_index].size() > 1) return fail(player_index, "step_staged: not with --data-parallel > 1");
        fi_learner* h = handles_[player_index];
        void* dst = nullptr;
        size_t stride = 0;
        if (fi_learner_acquire_staging(h, &dst, &stride) != FI_OK) return fail(player_index, fi_last_error());
        if (!fill(static_cast<char*>(dst), stride, cfg_.batch_size)) return false;
        if (async) {
            if (fi_learner_step_staged_async(h) != FI_OK) return fail(player_index, fi_last_error());
            return true;
        }
        fi_step_stats st{};
        if (fi_learner_step_staged(h, &st) != FI_OK) return fail(player_index, fi_last_error());
        stats_[player_index] = st;
        return true;
    }

    bool wait(size_t p) {
        if (p >= handles_.size()) return fail(0, "player_index out of range");
        fi_step_stats st{};
        if (fi_learner_wait(handles_[p], &st) != FI_OK) return fail(p, fi_last_error());
        stats_[p] = st;
        return true;
    }

    // Full learner state (params + Adam moments + counters) for checkpoint / resume.
    bool save_state(size_t p, std::vector<char>& blob) {
        if (p >= handles_.size()) return fail(0, "player_index out of range");
        blob.resize(fi_learner_state_bytes(handles_[p]));
        if (fi_learner_save_state(handles_[p], blob.data(), blob.size()) != FI_OK) return fail(p, fi_last_error());
        return true;
    }
    bool load_state(size_t p, const std::vector<char>& blob) {
        if (p >= handles_.size()) return fail(0, "player_index out of range");
        for (fi_learner* h : shards_[p])
            if (fi_learner_load_state(h, blob.data(), blob.size()) != FI_OK) return fail(p, fi_last_error());
        return true;
    }

    // Parameters of player p as the published Model blob (fp32 or bf16, little endian,
    // DESIGN.md section 3 order); resizes `blob` to param_bytes().
    bool publish(size_t p, std::vector<char>& blob, uint64_t& version) {
        if (p >= handles_.size()) return fail(0, "player_index out of range");
        blob.resize(param_bytes());
        if (fi_learner_get_params(handles_[p], blob.data(), blob.size(), &version) != FI_OK)
            return fail(p, fi_last_error());
        return true;
    }
    // --starting-model resume (Model::loadFromDisk bytes + version).
    bool load(size_t p, const std::vector<char>& blob, uint64_t version) {
        if (p >= handles_.size()) return fail(0, "player_index out of range");
        for (fi_learner* h : shards_[p])
            if (fi_learner_set_params(h, blob.data(), blob.size(), version) != FI_OK) return fail(p, fi_last_error());
        return true;
    }

    size_t param_bytes() const { return fi_learner_param_bytes(handles_[0]); }
    size_t param_count() const { return fi_learner_param_count(handles_[0]); }
    size_t entry_bytes() const { return fi_learner_entry_bytes(handles_[0]); }
    size_t players() const { return handles_.size(); }
    const fi_step_stats& last_stats(size_t p) const { return stats_.at(p); }
    std::string last_error(size_t p = 0) const {
        std::lock_guard<std::mutex> g(mu_);
        return err_.at(p);
    }
    fi_learner* handle(size_t p) { return handles_.at(p); }
    size_t shards(size_t p = 0) const { return shards_.at(p).size(); }
    const LearnerConfig& config() const { return cfg_; }

private:
    // --data-parallel: contiguous shards of the M entries, one per device, stepped
    // concurrently (the in-step all-reduce needs every rank); loss sums added over the shards
    bool step_sharded(size_t p, const std::vector<const void*>& ptrs, size_t eb) {
        const size_t G = shards_[p].size();
        if (ptrs.size() % G != 0) return fail(p, "batch not divisible by --data-parallel");
        const size_t per = ptrs.size() / G;
        std::vector<fi_step_stats> st(G);
        std::vector<int> rc(G, FI_OK);
        std::vector<std::string> why(G);
        auto run = [&](size_t g) {
            rc[g] = fi_learner_step(shards_[p][g], ptrs.data() + g * per, per, eb, &st[g]);
            if (rc[g] != FI_OK) why[g] = fi_last_error();  // thread-local: read on the same thread
        };
        std::vector<std::thread> th;
        for (size_t g = 1; g < G; ++g) th.emplace_back(run, g);
        run(0);
        for (auto& t : th) t.join();
        // A rejected batch (an out-of-range action in any shard) fails on EVERY shard: the
        // reject counter is all-reduced with the gradient before the optimizer, so all
        // replicas skip the update together and stay identical; one rejection is reported.
        for (size_t g = 0; g < G; ++g)
            if (rc[g] != FI_OK) return fail(p, "shard " + std::to_string(g) + ": " + why[g]);
        fi_step_stats sum = st[0];
        for (size_t g = 1; g < G; ++g) {
            sum.pg_loss += st[g].pg_loss;
            sum.baseline_loss += st[g].baseline_loss;
            sum.entropy_loss += st[g].entropy_loss;
            sum.total_loss += st[g].total_loss;
            sum.step_ms = std::max(sum.step_ms, st[g].step_ms);
        }
        stats_[p] = sum;
        return true;
    }

    bool fail(size_t p, const std::string& m) {
        std::lock_guard<std::mutex> g(mu_);
        err_.at(p < err_.size() ? p : 0) = m;
        return false;
    }
    void release() {
        for (auto& v : shards_)
            for (auto& h : v) {
                if (h) fi_learner_destroy(h);
                h = nullptr;
            }
        for (auto& h : handles_) h = nullptr;
    }

    LearnerConfig cfg_;
    std::vector<fi_learner*> handles_;               // per player: shard 0 (publishes, checkpoints)
    std::vector<std::vector<fi_learner*>> shards_;  // per player: its G data-parallel replicas
    std::vector<fi_step_stats> stats_;
    mutable std::mutex mu_;
    std::vector<std::string> err_;
};

}  // namespace freeimpala_amd
