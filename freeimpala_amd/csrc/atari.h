// atari.h -- Atari-shaped conv policy (config #3): bf16 MFMA implicit-GEMM convs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fi {

// partial conv1 weight-gradient slabs per workgroup of the fused conv2 backward + conv1 weight
// gradient (blocked fp32 accumulation over the workgroup's frames, atari_fr.hip): the kernel
// writes this many slabs per workgroup, atari.hip sizes the slab region and reduces that many
constexpr int kC1Segs = 8;

// per-launch timing hook (implemented by the learner's profiling events)
struct KernelTagger {
    virtual void begin(const char* name) = 0;
    virtual void end() = 0;
    virtual ~KernelTagger() {}
};
struct TagScope {
    KernelTagger* t;
    TagScope(KernelTagger* t_, const char* name) : t(t_) {
        if (t) t->begin(name);
    }
    ~TagScope() {
        if (t) t->end();
    }
};

// gradient-ready hook: the backward pass calls ready(off, n) once grads[off, off+n) hold
// their final values for this step (enqueued on the stream), latest layers first; the
// learner starts that bucket's all-reduce on its comm stream while the backward continues
struct GradReadyHook {
    virtual int ready(size_t off, size_t n) = 0;
    virtual ~GradReadyHook() {}
};

struct AtariNet {
    static constexpr size_t kFrameBytes = 84 * 84 * 4;
    int B = 0, T = 0, A = 0, N = 0;  // N = (T+1)*B frames
    void* impl = nullptr;
};

size_t atari_param_count(int A);
void atari_init_params(int A, uint64_t seed, std::vector<float>& p);
AtariNet* atari_create(int B, int T, int A);
void atari_destroy(AtariNet* n);
int atari_sync_weights(AtariNet* n, const float* params, hipStream_t s);
int atari_forward(AtariNet* n, const uint8_t* frames, float* logits, float* values, hipStream_t s,
                  KernelTagger* tg = nullptr);
int atari_backward(AtariNet* n, const uint8_t* frames, const float* dlogits, const float* dvalue,
                   float* grads, hipStream_t s, KernelTagger* tg = nullptr, GradReadyHook* gr = nullptr);
bool atari_tensor(AtariNet* n, const char* name, void** p, size_t* bytes);

}  // namespace fi
