// atari.hip -- placeholder until the bf16 conv path lands (returns FI_ERR_UNSUPPORTED).
#include "atari.h"
#include "fi_common.h"

namespace fi {
size_t atari_param_count(int A) {
    return 8 * 8 * 4 * 32 + 32 + 4 * 4 * 32 * 64 + 64 + 3 * 3 * 64 * 64 + 64 + (size_t)3136 * 512 +
           512 + (size_t)512 * (A + 1) + (A + 1);
}
void atari_init_params(int A, uint64_t, std::vector<float>& p) { p.assign(atari_param_count(A), 0.f); }
AtariNet* atari_create(int, int, int) {
    set_error("Atari conv policy not built yet");
    return nullptr;
}
void atari_destroy(AtariNet* n) { delete n; }
int atari_sync_weights(AtariNet*, const float*, hipStream_t) { return fail(FI_ERR_UNSUPPORTED, "atari"); }
int atari_forward(AtariNet*, const uint8_t*, float*, float*, hipStream_t) { return fail(FI_ERR_UNSUPPORTED, "atari"); }
int atari_backward(AtariNet*, const uint8_t*, const float*, const float*, float*, hipStream_t) {
    return fail(FI_ERR_UNSUPPORTED, "atari");
}
bool atari_tensor(AtariNet*, const char*, void**, size_t*) { return false; }
}  // namespace fi
