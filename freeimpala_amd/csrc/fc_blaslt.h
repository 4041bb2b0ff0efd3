// fc_blaslt.h -- the Atari policy's fc forward / data-gradient GEMMs on hipBLASLt (see fc_blaslt.cpp).
#pragma once

#include <hip/hip_runtime.h>

namespace fi {

struct FcBlasLt;
// rows = (T+1)*B; the buffers are the layer's tensors (used to time the algorithm candidates)
FcBlasLt* fc_blaslt_create(int rows, const void* a3, const void* w, const void* dh, void* h, void* da3,
                           hipStream_t s);
void fc_blaslt_destroy(FcBlasLt* F);
int fc_blaslt_forward(FcBlasLt* F, const void* a3, const void* w, const float* bias, void* h, hipStream_t s);
int fc_blaslt_dgrad(FcBlasLt* F, const void* dh, const void* w, void* da3, hipStream_t s);

}  // namespace fi
