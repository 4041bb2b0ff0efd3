// atari.h -- Atari-shaped conv policy (config #3): bf16 MFMA implicit-GEMM convs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fi {

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
int atari_forward(AtariNet* n, const uint8_t* frames, float* logits, float* values, hipStream_t s);
int atari_backward(AtariNet* n, const uint8_t* frames, const float* dlogits, const float* dvalue,
                   float* grads, hipStream_t s);
bool atari_tensor(AtariNet* n, const char* name, void** p, size_t* bytes);

}  // namespace fi
