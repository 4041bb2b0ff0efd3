/* fi_farmer.h -- C ABI of the MI355X FarmerLstm train step (libfi_learner.so).
 *
 * Replaces the reference's only neural-network step: FarmerLstmModel (LSTM 162 -> 128 over T
 * steps, the last step's h concatenated with x[484], 5 x (Linear 512 + ReLU), Linear 512 -> 1)
 * and its supervised train step (zero_grad -> forward -> criterion -> backward -> optimizer.step):
 *   /root/reference/scripts/gpu_benchmark.py:11-44   FarmerLstmModel.forward (return_value=True)
 *   /root/reference/scripts/gpu_benchmark.py:46-66   get_loss_function / get_optimizer
 *   /root/reference/scripts/gpu_benchmark.py:99-125  run_single_training_iteration
 *   /root/reference/cmd/libtorch_bench/main.cpp:14-42, 94-135  the same model and train_step
 * (the policy torso the reference defines). Plain C types only; status
 * codes as fi_learner.h (FI_OK / FI_ERR_*), message in fi_last_error().
 *
 * Parameters: ONE fp32 blob in the model's state_dict order and PyTorch layouts
 *   lstm.weight_ih_l0 [512][162] | lstm.weight_hh_l0 [512][128] | lstm.bias_ih_l0 [512] |
 *   lstm.bias_hh_l0 [512] | dense1.weight [512][612] dense1.bias [512] | dense2..5 [512][512]
 *   + [512] | dense6.weight [1][512] dense6.bias [1]   (1,514,497 floats; gates i, f, g, o)
 * so a torch state_dict flattened in order loads unchanged.
 * Inputs (batch_first, fp32, as generate_synthetic_data, gpu_benchmark.py:86-97):
 *   z [B][T][162], x [B][484], targets [B][1].
 */
#ifndef FI_FARMER_H
#define FI_FARMER_H

#include <stddef.h>
#include <stdint.h>

#include "fi_learner.h"

#ifdef __cplusplus
extern "C" {
#endif

enum fi_farmer_loss { FI_LOSS_MSE = 0, FI_LOSS_MAE = 1, FI_LOSS_HUBER = 2 };          /* gpu_benchmark.py:46-55 */
enum fi_farmer_opt { FI_FOPT_ADAM = 0, FI_FOPT_SGD = 1, FI_FOPT_ADAMW = 2 };          /* gpu_benchmark.py:57-66 */

typedef struct fi_farmer_config {
    int batch;          /* B (--batch-size, default 32)                                    */
    int seq_len;        /* T (--seq-length, default 10)                                    */
    int loss;           /* fi_farmer_loss (--loss-function, default mse)                    */
    int optimizer;      /* fi_farmer_opt (--optimizer, default adam)                        */
    float lr;           /* --learning-rate, default 1e-3                                    */
    float beta1, beta2, eps;  /* torch defaults 0.9, 0.999, 1e-8                            */
    float weight_decay; /* torch defaults: 0 (adam), 0.01 (adamw); ignored by sgd           */
    int device;         /* HIP device ordinal                                               */
} fi_farmer_config;

typedef struct fi_farmer fi_farmer;

typedef struct fi_farmer_stats {
    double loss;        /* criterion(values, targets) of this step (before the update)     */
    float step_ms;      /* device time of the step (HIP events)                            */
    uint64_t step;      /* optimizer steps taken so far                                    */
} fi_farmer_stats;

size_t fi_farmer_param_count(void); /* 1,514,497 */
void fi_farmer_config_init(fi_farmer_config* cfg);
int fi_farmer_create(const fi_farmer_config* cfg, fi_farmer** out);
void fi_farmer_destroy(fi_farmer* f);
/* parameters (host fp32, state_dict order); set also resets the optimizer state */
int fi_farmer_set_params(fi_farmer* f, const float* host, size_t n);
int fi_farmer_get_params(fi_farmer* f, float* host, size_t n);
/* gradients of the last train step (host fp32, same order) */
int fi_farmer_get_grads(fi_farmer* f, float* host, size_t n);
/* one train step. inputs_on_device != 0: z / x / targets are device pointers (resident
 * batch, no copy); else host pointers, copied in on the handle's stream. values (nullable,
 * host, B floats) receives the forward output the loss was taken on. */
int fi_farmer_train_step(fi_farmer* f, const float* z, const float* x, const float* targets,
                         int inputs_on_device, float* values, fi_farmer_stats* out);
/* forward only (FarmerLstmModel.forward(z, x, return_value=True)): values [B] on the host */
int fi_farmer_forward(fi_farmer* f, const float* z, const float* x, int inputs_on_device,
                      float* values);
/* introspection: device pointer / bytes of "params", "grads", "values", "z", "x",
 * "targets" (the handle's resident input buffers), "gates", "h_last", "act1".."act5" (the
 * dense layers' ReLU outputs [B][512]) */
int fi_farmer_tensor(fi_farmer* f, const char* name, void** dev_ptr, size_t* bytes);
void* fi_farmer_stream(fi_farmer* f);
/* Profiling (bench / roofline): with profiling on, every later train step records HIP events
 * around the two recurrence kernels; fi_farmer_recurrence_ms returns their mean device ms
 * per step so far (forward LSTM, BPTT) and the step count, and resets the sums.          */
int fi_farmer_set_profiling(fi_farmer* f, int on);
int fi_farmer_recurrence_ms(fi_farmer* f, float* fwd_ms, float* bwd_ms, int* steps);

#ifdef __cplusplus
}
#endif
#endif
