// reference_binding.cpp -- INTEGRATION.md section 2, compiled for real: the reference's own
// SharedBuffer / ModelManager / MetricsTracker (/root/reference/include/freeimpala/
// data_structures.h:43-481, metrics_tracker.h:21-385, global namespace) under
// freeimpala_amd::BasicLearner, exactly the three-line alias the patch puts in place of
// include/freeimpala/learner.h. Built by tests/test_reference_binding.py in the build container
// only (the reference tree is never copied; the GPU box runs the binary built here):
//
//   g++ -std=c++17 -I/root/reference/include -Itests/cpp/stubs -Iinclude -include optional
//       tests/cpp/reference_binding.cpp -Lfreeimpala_amd/lib -lfi_learner -pthread   (Makefile)
//
// (`-include optional`: data_structures.h:141 uses std::optional without including it;
// tests/cpp/stubs/spdlog/spdlog.h stands in for the FetchContent'd spdlog.)
//
//   reference_binding nodevice      construct the Learner as setupLearner does
//                                   (cmd/freeimpala/main.cpp:174-197); exit 3 with the loud
//                                   "no device" error when no GPU is usable, 0 if one is
//   reference_binding run <dir>     on the GPU: the same record-schema entries are written
//                                   through the reference SharedBuffer::write into the alias
//                                   Learner and through freeimpala_amd::SharedBuffer into
//                                   freeimpala_amd::Learner; both run ITERS steps (start(),
//                                   worker loop, stop()); exit 0 iff every published version
//                                   and the final parameter blobs are bit-identical and the
//                                   reference-format checkpoint files hold the published model
#include "freeimpala/data_structures.h"
#include "freeimpala/metrics_tracker.h"
#include "freeimpala_amd/learner.hpp"  // no name clashes: everything lives in namespace freeimpala_amd
using Learner = freeimpala_amd::BasicLearner<SharedBuffer, ModelManager, MetricsTracker>;

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

// metrics_tracker.h declares these statics and defines them at its end (:385-387) -- nothing to add

namespace {

constexpr size_t P = 1, CAP = 16, T = 8, S = T + 1, M = 4, ITERS = 3, CKPT = 2;

freeimpala_amd::LearnerConfig config() {
    freeimpala_amd::LearnerConfig lc;
    lc.seq_length = T;
    lc.arch = "mlp";
    lc.optimizer = "adam";
    lc.lr = 1e-3f;
    return lc;
}

// record schema, deterministic per (entry, step)
std::vector<char> make_entry(size_t e, int A) {
    std::vector<char> buf(S * ELEMENT_SIZE, 0);
    std::mt19937 rng(1234u + 7919u * (unsigned)e);
    std::normal_distribution<float> nrm(0.f, 1.f);
    for (size_t s = 0; s < S; ++s) {
        char* r = buf.data() + s * ELEMENT_SIZE;
        float obs[128], mu[64] = {};
        for (float& x : obs) x = nrm(rng);
        for (int a = 0; a < A; ++a) mu[a] = nrm(rng);
        const int32_t action = (int32_t)(rng() % (unsigned)A);
        const float reward = (float)((int)(rng() % 3) - 1), discount = (rng() % 100) ? 0.99f : 0.f;
        std::memcpy(r, obs, sizeof obs);
        std::memcpy(r + 512, mu, sizeof mu);
        std::memcpy(r + 768, &action, 4);
        std::memcpy(r + 772, &reward, 4);
        std::memcpy(r + 776, &discount, 4);
    }
    return buf;
}

template <class L>
bool wait_iterations(const L& l, size_t n) {
    for (int i = 0; i < 6000 && l.iterations(0) < n; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    return l.iterations(0) >= n;
}

bool read_file(const std::string& path, std::vector<char>& out) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return false;
    out.resize((size_t)f.tellg());
    f.seekg(0);
    f.read(out.data(), (std::streamsize)out.size());
    return (bool)f;
}

int fail(const std::string& m) {
    std::fprintf(stderr, "reference_binding: FAIL: %s\n", m.c_str());
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "nodevice";
    const std::string dir = argc > 2 ? argv[2] : "/tmp/fi_reference_binding";
    const auto lc = config();
    if (mode == "nodevice") {
        try {
            Learner learner(P, CAP, S, M, /*learner_time*/ 0, CKPT, dir + "/ref", "", ITERS, lc);
            std::printf("reference_binding: device learner constructed on the reference classes (%zu param bytes)\n",
                        learner.device().param_bytes());
            return 0;
        } catch (const std::exception& e) {
            std::printf("reference_binding: no device: %s\n", e.what());
            return 3;
        }
    }
    if (mode != "run") return fail("unknown mode " + mode);

    // the same entries for both learners, M per step
    std::vector<std::vector<char>> entries;
    for (size_t e = 0; e < M * ITERS; ++e) entries.push_back(make_entry(e, lc.num_actions));

    // 1) the alias: reference SharedBuffer::write (data_structures.h:219-241), reference
    //    ModelManager / Model for publication, reference MetricsTracker singleton
    std::vector<std::vector<char>> ref_versions;
    uint64_t ref_version = 0;
    {
        Learner learner(P, CAP, S, M, 0, CKPT, dir + "/ref", "", ITERS, lc);
        auto mm = learner.getModelManager();
        learner.start();
        auto buf = learner.getSharedBuffers()[0];
        for (size_t it = 0; it < ITERS; ++it) {
            for (size_t j = 0; j < M; ++j)
                if (!buf->write(entries[it * M + j])) return fail("SharedBuffer::write refused an entry");
            if (!wait_iterations(learner, it + 1)) return fail("alias learner stalled");
            ref_versions.push_back(mm->getModel(0)->getData());
        }
        learner.stop();
        ref_version = mm->getLatestVersion(0);
        if (MetricsTracker::getInstance()->getLearnerUpdatesPerSecond() <= 0.0)
            return fail("reference MetricsTracker saw no recordLearnerModelUpdate");
    }

    // 2) freeimpala_amd's own classes (zero-copy readBatchInto path), same entries
    std::vector<std::vector<char>> own_versions;
    {
        freeimpala_amd::Learner learner(P, CAP, S, M, 0, CKPT, dir + "/own", "", ITERS, lc);
        auto mm = learner.getModelManager();
        learner.start();
        auto buf = learner.getSharedBuffers()[0];
        for (size_t it = 0; it < ITERS; ++it) {
            for (size_t j = 0; j < M; ++j)
                if (!buf->write(entries[it * M + j])) return fail("freeimpala_amd::SharedBuffer::write refused");
            if (!wait_iterations(learner, it + 1)) return fail("own learner stalled");
            own_versions.push_back(mm->getModel(0)->getData());
        }
        learner.stop();
        if (mm->getLatestVersion(0) != ref_version) return fail("published versions differ");
    }
    for (size_t it = 0; it < ITERS; ++it)
        if (ref_versions[it] != own_versions[it]) return fail("published blob differs at step " + std::to_string(it + 1));

    // 3) checkpoints written through the alias: reference file format, trained weights
    std::vector<char> f;
    if (!read_file(dir + "/ref/model_0_" + std::to_string(CKPT) + ".bin", f) || f.size() != 8 + ref_versions[0].size())
        return fail("missing / wrong-size model_0_" + std::to_string(CKPT) + ".bin");
    if (std::memcmp(f.data() + 8, ref_versions[CKPT - 1].data(), ref_versions[0].size()) != 0)
        return fail("model_0_" + std::to_string(CKPT) + ".bin does not hold the published weights of that iteration");
    if (!read_file(dir + "/ref/model_0_latest.bin", f) ||
        std::memcmp(f.data() + 8, ref_versions.back().data(), ref_versions.back().size()) != 0)
        return fail("model_0_latest.bin does not hold the final weights");
    uint64_t v = 0;
    std::memcpy(&v, f.data(), 8);
    if (v != ref_version) return fail("model_0_latest.bin version " + std::to_string(v));

    // 4) --starting-model on the alias: resumes from the .state next to model_0_latest.bin
    {
        Learner learner(P, CAP, S, M, 0, 0, dir + "/ref2", dir + "/ref", ITERS, lc);
        if (learner.getModelManager()->getLatestVersion(0) != ref_version)
            return fail("resume did not pick up version " + std::to_string(ref_version));
        if (learner.getModelManager()->getModel(0)->getData() != ref_versions.back())
            return fail("resume did not restore the final weights");
        learner.stop();
    }
    std::printf("reference_binding: ok (%zu steps, version %llu, %zu-byte blobs identical on both class sets)\n",
                ITERS, (unsigned long long)ref_version, ref_versions[0].size());
    return 0;
}
