// mpi_pool.hpp -- MPI feeding of the device learner: the learner-side receiver of
// freeimpala_mpi_async_pool and the actor-side wire protocol, on the reference's tags and
// payloads so actor ranks and the rank-0 learner interoperate unchanged.
//
// Wire protocol (reference data_structures.h:21-32, agent.h:76-151,
// cmd/freeimpala_mpi_async_pool/main.cpp:243-357), all on MPI_COMM_WORLD, learner = rank 0:
//   actor -> learner  tag 100 + p   one buffer entry for player p (S * 1024 bytes)
//                     tag 200       u32 player   version request
//                     tag 210       u32 player   weights request
//                     tag 999       (empty)      this actor is done
//   learner -> actor  tag 201       u64 latest version
//                     tag 211       u64 version || weights blob (<= 6 MiB for the reference
//                                   actors' receive buffer, mpi_async_pool/main.cpp:350)
//
// LearnerEndpoint (rank 0) keeps the reference's shape -- a ring of posted MPI_Irecv slots
// drained with MPI_Waitany on the calling thread, a pool of processor threads that write
// trajectories into the per-player SharedBuffers (blocking when full: back-pressure on the
// actors) and answer version / weights requests -- with three changes for a learner that
// consumes ~0.4 GB of trajectories per step:
//   * slots are sized for the largest message rank 0 RECEIVES (an entry), not for the weights
//     it only sends (the reference sizes all 128 slots by max(entry, 8 + model));
//   * a received slot is handed to the processor by moving its vector (a recycled one is
//     re-posted), so an entry is copied once, into the SharedBuffer, instead of twice;
//   * the `version || blob` reply is serialised once per published version and shared by
//     every request for it, instead of createCopy + a fresh buffer per request.
// ActorClient (ranks > 0) implements agent.h's transfer / model-sync exchanges; a request and
// its reply are serialised per actor, so several player threads of one actor cannot take each
// other's replies (the reference's per-player threads share tags 201/211).
#pragma once

#include <mpi.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "freeimpala_amd/replay.hpp"

namespace freeimpala_amd {
namespace mpi {

namespace detail {
// Buffer::write(const char*, size_t) (freeimpala_amd::SharedBuffer) is used when the buffer type
// has it; the reference SharedBuffer only has write(const std::vector<char>&)
// (data_structures.h:219), which gets the received vector trimmed to the message size.
template <class B, class = void>
struct has_write_ptr : std::false_type {};
template <class B>
struct has_write_ptr<B, std::void_t<decltype(std::declval<B&>().write((const char*)nullptr, size_t{}))>>
    : std::true_type {};
}  // namespace detail

struct EndpointStats {
    uint64_t trajectories = 0, trajectory_bytes = 0, version_requests = 0, weights_replies = 0,
             weights_bytes = 0, bad_messages = 0, dropped_entries = 0,
             late_messages = 0;  // completed receives found in the slots after the last terminate
    double seconds = 0.0;  // from the first slot posted to the last actor's TAG_TERMINATE
};

template <class Buffer, class Manager>
class LearnerEndpoint {
public:
    // max_entry_bytes: the largest trajectory message (S * ELEMENT_SIZE).
    LearnerEndpoint(std::vector<std::shared_ptr<Buffer>> buffers, std::shared_ptr<Manager> models,
                    size_t max_entry_bytes, int processors = 8, int slots = 128, MPI_Comm comm = MPI_COMM_WORLD)
        : bufs_(std::move(buffers)), models_(std::move(models)), comm_(comm),
          slot_bytes_(std::max<size_t>(max_entry_bytes, 8)), n_proc_(std::max(1, processors)),
          n_slots_(std::max(1, slots)), cache_(bufs_.size()) {}

    // Runs the receiver on the calling thread until every other rank has sent TAG_TERMINATE,
    // then lets the processors finish the queued messages and joins them.
    EndpointStats run() {
        int world = 1;
        MPI_Comm_size(comm_, &world);
        MPI_Comm_set_errhandler(comm_, MPI_ERRORS_RETURN);
        std::vector<std::thread> procs;
        for (int i = 0; i < n_proc_; ++i) procs.emplace_back([this] { processor(); });

        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::vector<char>> bufs(n_slots_);
        std::vector<MPI_Request> reqs(n_slots_, MPI_REQUEST_NULL);
        for (int i = 0; i < n_slots_; ++i) post(bufs[i], reqs[i]);
        int done = 0;
        while (done < world - 1) {
            int idx = MPI_UNDEFINED;
            MPI_Status st;
            if (MPI_Waitany(n_slots_, reqs.data(), &idx, &st) != MPI_SUCCESS || idx == MPI_UNDEFINED) {
                bump(&EndpointStats::bad_messages);
                if (idx == MPI_UNDEFINED) break;  // every slot inactive: nothing can arrive any more
                post(bufs[idx], reqs[idx]);
                continue;
            }
            if (st.MPI_TAG == TAG_TERMINATE) {
                ++done;
            } else {
                int n = 0;
                MPI_Get_count(&st, MPI_BYTE, &n);
                Msg m{st.MPI_TAG, st.MPI_SOURCE, (size_t)n, std::move(bufs[idx])};
                enqueue(std::move(m));
            }
            post(bufs[idx], reqs[idx]);
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        // Drain the posted slots. MPI_Waitany hands back an arbitrary completed request, so
        // the last TAG_TERMINATE may have been picked while other slots already held
        // trajectories that arrived before it: a slot whose receive completed (or completes
        // while being cancelled) is enqueued like any other message, never thrown away.
        for (int i = 0; i < n_slots_; ++i) {
            MPI_Request& r = reqs[i];
            if (r == MPI_REQUEST_NULL) continue;
            MPI_Status st;
            int flag = 0;
            MPI_Test(&r, &flag, &st);
            if (!flag) {
                MPI_Cancel(&r);
                MPI_Wait(&r, &st);
                int cancelled = 0;
                MPI_Test_cancelled(&st, &cancelled);
                if (cancelled) continue;
            }
            if (st.MPI_TAG == TAG_TERMINATE) {  // a surplus terminate: counted, not fatal
                bump(&EndpointStats::late_messages);
                continue;
            }
            int n = 0;
            MPI_Get_count(&st, MPI_BYTE, &n);
            bump(&EndpointStats::late_messages);
            enqueue(Msg{st.MPI_TAG, st.MPI_SOURCE, (size_t)n, std::move(bufs[i])});
        }
        {
            std::lock_guard<std::mutex> lk(qmu_);
            stopping_ = true;
        }
        qcv_.notify_all();
        for (auto& t : procs) t.join();
        std::lock_guard<std::mutex> lk(smu_);
        stats_.seconds = secs;
        return stats_;
    }

private:
    struct Msg {
        int tag, source;
        size_t bytes;
        std::vector<char> data;
    };

    void post(std::vector<char>& b, MPI_Request& r) {
        if (b.size() != slot_bytes_) {
            std::lock_guard<std::mutex> lk(pool_mu_);
            if (!pool_.empty()) {
                b = std::move(pool_.back());
                pool_.pop_back();
            } else {
                b.assign(slot_bytes_, 0);
            }
        }
        MPI_Irecv(b.data(), (int)b.size(), MPI_BYTE, MPI_ANY_SOURCE, MPI_ANY_TAG, comm_, &r);
    }
    void recycle(std::vector<char>&& b) {
        b.resize(slot_bytes_);  // a vector trimmed for Buffer::write regrows within its capacity
        std::lock_guard<std::mutex> lk(pool_mu_);
        if (pool_.size() < (size_t)n_slots_) pool_.push_back(std::move(b));
    }
    bool write_entry(Buffer& buf, Msg& m) {
        if constexpr (detail::has_write_ptr<Buffer>::value) {
            return buf.write(m.data.data(), m.bytes);
        } else {  // the reference's write(const std::vector<char>&): exactly the received bytes
            m.data.resize(m.bytes);
            return buf.write(static_cast<const std::vector<char>&>(m.data));
        }
    }
    void enqueue(Msg&& m) {
        {
            std::lock_guard<std::mutex> lk(qmu_);
            q_.push_back(std::move(m));
        }
        qcv_.notify_one();
    }
    void bump(uint64_t EndpointStats::*f, uint64_t by = 1) {
        std::lock_guard<std::mutex> lk(smu_);
        stats_.*f += by;
    }

    void processor() {
        for (;;) {
            Msg m;
            {
                std::unique_lock<std::mutex> lk(qmu_);
                qcv_.wait(lk, [this] { return !q_.empty() || stopping_; });
                if (q_.empty()) return;
                m = std::move(q_.front());
                q_.pop_front();
            }
            handle(m);
            recycle(std::move(m.data));
        }
    }

    // mpi_async_pool/main.cpp:247-303
    void handle(Msg& m) {
        if (m.tag == TAG_VERSION_REQ || m.tag == TAG_WEIGHTS_REQ) {
            uint32_t p = 0;
            if (m.bytes < sizeof p) return bump(&EndpointStats::bad_messages);
            std::memcpy(&p, m.data.data(), sizeof p);
            if (p >= bufs_.size()) return bump(&EndpointStats::bad_messages);
            if (m.tag == TAG_VERSION_REQ) {
                uint64_t v = models_->getLatestVersion(p);
                if (MPI_Send(&v, 1, MPI_UINT64_T, m.source, TAG_VERSION_RES, comm_) != MPI_SUCCESS)
                    log_line("error", "MPI_Send(version_res) failed");
                bump(&EndpointStats::version_requests);
            } else {
                auto w = weights(p);
                if (MPI_Send(w->data(), (int)w->size(), MPI_BYTE, m.source, TAG_WEIGHTS_RES, comm_) != MPI_SUCCESS)
                    log_line("error", "MPI_Send(weights_res) failed");
                std::lock_guard<std::mutex> lk(smu_);
                ++stats_.weights_replies;
                stats_.weights_bytes += w->size();
            }
            return;
        }
        const int p = m.tag - TAG_TRAJECTORY_BASE;
        if (m.tag < TAG_TRAJECTORY_BASE || p >= (int)bufs_.size() || m.tag >= TAG_VERSION_REQ) {
            log_line("error", "unexpected tag " + std::to_string(m.tag) + " from rank " + std::to_string(m.source));
            return bump(&EndpointStats::bad_messages);
        }
        // blocks while the buffer is full (the reference's write, mpi_async_pool/main.cpp:260)
        if (!write_entry(*bufs_[p], m)) return bump(&EndpointStats::dropped_entries);
        std::lock_guard<std::mutex> lk(smu_);
        ++stats_.trajectories;
        stats_.trajectory_bytes += m.bytes;
    }

    // `u64 version || blob` of player p's latest model, built once per version
    std::shared_ptr<const std::vector<char>> weights(size_t p) {
        std::lock_guard<std::mutex> lk(cache_mu_);
        auto model = models_->getModel(p);
        const uint64_t v = model->getVersion();
        auto& c = cache_[p];
        if (!c.blob || c.version != v) {
            const std::vector<char> d = model->getData();
            auto out = std::make_shared<std::vector<char>>(sizeof(uint64_t) + d.size());
            std::memcpy(out->data(), &v, sizeof v);
            std::memcpy(out->data() + sizeof v, d.data(), d.size());
            c.blob = std::move(out);
            c.version = v;
        }
        return c.blob;
    }

    struct Cached {
        uint64_t version = 0;
        std::shared_ptr<const std::vector<char>> blob;
    };

    std::vector<std::shared_ptr<Buffer>> bufs_;
    std::shared_ptr<Manager> models_;
    MPI_Comm comm_;
    size_t slot_bytes_;
    int n_proc_, n_slots_;
    std::mutex qmu_, smu_, pool_mu_, cache_mu_;
    std::condition_variable qcv_;
    std::deque<Msg> q_;
    bool stopping_ = false;
    std::vector<std::vector<char>> pool_;
    std::vector<Cached> cache_;
    EndpointStats stats_;
};

// The actor side of agent.h's USE_MPI paths.
class ActorClient {
public:
    explicit ActorClient(int learner_rank = 0, MPI_Comm comm = MPI_COMM_WORLD) : dst_(learner_rank), comm_(comm) {}

    // agent.h:82-90: the whole entry, tag TRAJECTORY_BASE + p
    bool send_trajectory(size_t p, const char* data, size_t n) {
        return MPI_Send(data, (int)n, MPI_CHAR, dst_, TAG_TRAJECTORY_BASE + (int)p, comm_) == MPI_SUCCESS;
    }

    // agent.h:108-151: ask for the latest version; when it is newer than `have`, ask for the
    // weights and take `u64 version || blob`. Returns true when `blob` / `have` were updated.
    bool sync_model(size_t p, uint64_t& have, std::vector<char>& blob) {
        std::lock_guard<std::mutex> lk(mu_);
        const uint32_t p32 = (uint32_t)p;
        uint64_t latest = 0;
        if (MPI_Send(&p32, 1, MPI_UINT32_T, dst_, TAG_VERSION_REQ, comm_) != MPI_SUCCESS) return false;
        MPI_Recv(&latest, 1, MPI_UINT64_T, dst_, TAG_VERSION_RES, comm_, MPI_STATUS_IGNORE);
        if (latest <= have) return false;
        if (MPI_Send(&p32, 1, MPI_UINT32_T, dst_, TAG_WEIGHTS_REQ, comm_) != MPI_SUCCESS) return false;
        MPI_Status st;
        MPI_Probe(dst_, TAG_WEIGHTS_RES, comm_, &st);
        int n = 0;
        MPI_Get_count(&st, MPI_BYTE, &n);
        std::vector<char> buf((size_t)std::max(n, 0));
        MPI_Recv(buf.data(), n, MPI_BYTE, dst_, TAG_WEIGHTS_RES, comm_, MPI_STATUS_IGNORE);
        if (buf.size() < sizeof(uint64_t)) return false;
        uint64_t v = 0;
        std::memcpy(&v, buf.data(), sizeof v);
        blob.assign(buf.begin() + sizeof v, buf.end());
        have = v;
        return true;
    }

    // mpi_async_pool/main.cpp:457-460
    void terminate() { MPI_Send(nullptr, 0, MPI_CHAR, dst_, TAG_TERMINATE, comm_); }

private:
    int dst_;
    MPI_Comm comm_;
    std::mutex mu_;
};

}  // namespace mpi
}  // namespace freeimpala_amd
