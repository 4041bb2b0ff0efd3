/*
 * fi_learner.h -- the drop-in C ABI of the MI355X learner step (libfi_learner.so).
 *
 * It replaces the body of freeimpala's learner step:
 *   reference  include/freeimpala/learner.h:32-49   Learner::trainModel(player, batch)
 *              (sleep(train_time_ms) + createCopy + generateRandomData + updateModel)
 * which is reached from Learner::workerThread (learner.h:72-97) with the output of
 *   reference  include/freeimpala/data_structures.h:267-300   SharedBuffer::readBatch(M)
 * and whose result is published through
 *   reference  include/freeimpala/data_structures.h:441-451   ModelManager::updateModel
 *
 * Plain C types only (no torch, no HIP types): host pointers in, status codes out, no
 * exceptions across the boundary, one handle per player (independent streams, no global
 * mutable state). 0 = success, negative = failure; fi_last_error() is thread-local.
 * The C++ Learner (include/freeimpala/learner.h) and any FFI (ctypes stub in
 * INTEGRATION.md) bind exactly these symbols.
 */
#ifndef FI_LEARNER_H_
#define FI_LEARNER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FI_ABI_VERSION 1
#define FI_RECORD_BYTES 1024 /* == ELEMENT_SIZE, reference data_structures.h:35 */

enum fi_status {
    FI_OK = 0,
    FI_ERR_INVALID = -1,     /* bad argument / shape                                */
    FI_ERR_HIP = -2,         /* HIP runtime error (message in fi_last_error)         */
    FI_ERR_OOM = -3,         /* device or pinned allocation failed                   */
    FI_ERR_STATE = -4,       /* call not valid in the current state                  */
    FI_ERR_COMM = -5,        /* RCCL failure                                         */
    FI_ERR_UNSUPPORTED = -6, /* configuration not built                              */
    FI_ERR_NONFINITE = -7    /* NaN / Inf in the (all-reduced) gradient: update skipped */
};

enum fi_arch { FI_ARCH_MLP = 0, FI_ARCH_ATARI = 1 };
enum fi_optimizer { FI_OPT_ADAM = 0, FI_OPT_SGD = 1 };
enum fi_publish { FI_PUBLISH_FP32 = 0, FI_PUBLISH_BF16 = 1 };

/* V-trace / IMPALA loss hyper-parameters (IMPALA defaults). */
typedef struct fi_vtrace_hparams {
    float rho_bar;       /* 1.0  */
    float c_bar;         /* 1.0  */
    float pg_rho_bar;    /* 1.0  */
    float lambda_;       /* 1.0  */
    float baseline_cost; /* 0.5  */
    float entropy_cost;  /* 0.01 */
} fi_vtrace_hparams;

typedef struct fi_learner_config {
    uint32_t struct_size;     /* = sizeof(fi_learner_config)                         */
    int32_t arch;             /* fi_arch                                              */
    int32_t seq_len;          /* T  (--seq-length)                                    */
    int32_t batch;            /* B  per device (--batch-size / number of GPUs)        */
    int32_t num_actions;      /* A: 2..64 (MLP), 2..18 (Atari: the ALE action sets)   */
    int32_t obs_dim;          /* MLP observation width (128)                          */
    int32_t hidden;           /* MLP hidden width (256)                               */
    int32_t optimizer;        /* fi_optimizer                                         */
    int32_t publish_dtype;    /* fi_publish                                           */
    int32_t device;           /* HIP device ordinal                                   */
    float gamma;              /* discount used by the synthetic generator only       */
    fi_vtrace_hparams hp;
    float lr, beta1, beta2, eps;
    float max_grad_norm;      /* global-norm clip, <= 0 disables                      */
    uint64_t seed;            /* parameter-initialisation seed                        */
} fi_learner_config;

typedef struct fi_step_stats {
    double pg_loss;       /* sum over T*B of -pg_adv * log pi(a_t)                       */
    double baseline_loss; /* 0.5 * sum (vs - V)^2   (unweighted)                         */
    double entropy_loss;  /* sum pi log pi          (unweighted)                         */
    double total_loss;    /* pg + baseline_cost*baseline + entropy_cost*entropy           */
    double grad_norm;     /* global L2 norm of the (all-reduced) gradient before clipping */
    uint64_t version;     /* parameter version after the step                             */
    float step_ms;        /* device time of the step (HIP events on the learner stream)  */
} fi_step_stats;

typedef struct fi_learner fi_learner;

/* ---- lifecycle ------------------------------------------------------------------- */
void fi_learner_config_init(fi_learner_config* cfg);
int fi_learner_create(const fi_learner_config* cfg, fi_learner** out);
void fi_learner_destroy(fi_learner* l);
const char* fi_last_error(void);
int fi_abi_version(void);

/* ---- sizes ------------------------------------------------------------------------ */
size_t fi_learner_param_count(const fi_learner* l);  /* fp32 parameters              */
size_t fi_learner_param_bytes(const fi_learner* l);  /* published blob (fp32|bf16)   */
size_t fi_learner_entry_bytes(const fi_learner* l);  /* minimum (T+1)*1024 per entry */

/* ---- the learner step ---------------------------------------------------------------
 * fi_learner_step: Learner::step(player, batch) body. entries[i] points at one
 * SharedBuffer entry (host memory, borrowed for the call only; entry_bytes >= (T+1)*1024,
 * record schema in DESIGN.md section 3). n_entries must equal cfg.batch. The call stages
 * the batch (pinned copy + async H2D), runs ingest -> policy fwd -> V-trace/loss -> bwd
 * -> [RCCL all-reduce] -> optimizer, and returns when the step has completed.
 * fi_learner_step_resident: same step on the batch already resident in HBM (filled by
 * fi_learner_synth_batch or a previous fi_learner_step).                                */
int fi_learner_step(fi_learner* l, const void* const* entries, size_t n_entries,
                    size_t entry_bytes, fi_step_stats* out);
int fi_learner_step_resident(fi_learner* l, fi_step_stats* out);
/* Asynchronous form: copies the entries into one of two pinned
 * buffers, enqueues the H2D copy and the whole step, and returns -- the caller may free the
 * entries and read the next batch while the device works. fi_learner_wait blocks until the
 * last enqueued step is done and reports its statistics (step_ms = 0), and fails with
 * FI_ERR_INVALID / FI_ERR_NONFINITE when any update enqueued since the last check was
 * skipped (the device counts them; the version counts applied updates only). Publication
 * calls (fi_learner_get_params*) also see the completed step.                            */
int fi_learner_step_async(fi_learner* l, const void* const* entries, size_t n_entries,
                          size_t entry_bytes);
int fi_learner_wait(fi_learner* l, fi_step_stats* out);
/* Zero-copy staging (a SharedBuffer::readBatchInto(pinned dst)
 * replacing readBatch's per-entry vector copies, data_structures.h:286-293).
 * fi_learner_acquire_staging returns the next of the two pinned staging buffers, once the
 * H2D that last read it has completed: cfg.batch entries, entry i at dst + i*entry_stride,
 * entry_stride = fi_learner_entry_bytes(). The caller copies the first entry_stride bytes of
 * each entry there (e.g. under the SharedBuffer mutex) and submits the buffer with
 * fi_learner_step_staged (returns when the step is done) or fi_learner_step_staged_async
 * (returns once enqueued; fi_learner_wait as above). The H2D runs on a copy stream beside
 * the previous device step. Acquiring again before submitting returns the same buffer;
 * submitting without an acquired buffer is FI_ERR_INVALID. MLP configuration only.       */
int fi_learner_acquire_staging(fi_learner* l, void** dst, size_t* entry_stride);
int fi_learner_step_staged(fi_learner* l, fi_step_stats* out);
int fi_learner_step_staged_async(fi_learner* l);
int fi_learner_synth_batch(fi_learner* l, uint64_t seed, int32_t b_global, int32_t b_offset);

/* ---- parameter publication / resume (ModelManager::updateModel, Model::loadFromDisk) - */
int fi_learner_get_params(fi_learner* l, void* dst, size_t bytes, uint64_t* version);
int fi_learner_get_params_fp32(fi_learner* l, float* dst, size_t count);
int fi_learner_set_params(fi_learner* l, const void* src, size_t bytes, uint64_t version);
/* Checkpoint / resume of the full learner state (params, Adam m and v, step count, version):
 * Learner::checkpointModel / --starting-model with optimizer state. */
size_t fi_learner_state_bytes(const fi_learner* l);
int fi_learner_save_state(fi_learner* l, void* dst, size_t bytes);
int fi_learner_load_state(fi_learner* l, const void* src, size_t bytes);

/* ---- data parallel (RCCL over xGMI) ------------------------------------------------ */
int fi_comm_unique_id_bytes(void);
int fi_comm_get_unique_id(void* dst, size_t bytes);
int fi_learner_attach_comm(fi_learner* l, const void* unique_id, size_t bytes, int rank,
                           int nranks);
/* One process, several devices: handle i (each on its own device) becomes rank i of n; the
 * per-device communicator inits run as one RCCL group, so one thread can call this (the
 * one-rank-per-process form above blocks until every peer has joined).                    */
int fi_comm_init_all(fi_learner* const* handles, int n);
/* The handle's communicator as RCCL reports it (ncclCommCount / ncclCommUserRank; 1 / 0
 * without one) and the gradient buckets its last step all-reduced (reverse layer order,
 * overlapped with the backward on a second stream).                                        */
int fi_learner_comm_info(fi_learner* l, int* nranks, int* rank, int* buckets);

/* ---- introspection for tests / bench ------------------------------------------------
 * fi_learner_tensor: device pointer + bytes of a named internal tensor ("params", "grads",
 * "obs", "frames", "mu", "actions", "rewards", "discounts", "logits", "values", "vs",
 * "pg_adv", "dlogits", "dvalue", "h1", "h2", "a1", "a2", "a3", "h").
 * fi_learner_set_profiling(1) records HIP events around every phase of later steps;
 * fi_learner_phase_times returns the mean device ms of each phase (see fi_phase).       */
enum fi_phase {
    FI_PHASE_INGEST = 0, FI_PHASE_FORWARD = 1, FI_PHASE_VTRACE = 2, FI_PHASE_BACKWARD = 3,
    FI_PHASE_ALLREDUCE = 4, FI_PHASE_OPTIMIZER = 5, FI_PHASE_COUNT = 6
};
int fi_learner_tensor(fi_learner* l, const char* name, void** dev_ptr, size_t* bytes);
/* fi_learner_read_tensor: waits for the handle's stream, then copies the first `bytes` bytes
 * of a named tensor into host memory (for hosts that do not link HIP: verification dumps,
 * e.g. the CLI's --dump-dir gradients). FI_ERR_INVALID when bytes exceeds the tensor.      */
int fi_learner_read_tensor(fi_learner* l, const char* name, void* host_dst, size_t bytes);
int fi_learner_set_profiling(fi_learner* l, int on);
int fi_learner_phase_times(fi_learner* l, float* ms, int n, int* n_steps);
int fi_learner_kernel_times(fi_learner* l, char* names_buf, size_t buflen, float* ms,
                            int* counts, int max);
void* fi_learner_stream(fi_learner* l);
int fi_learner_sync(fi_learner* l);

/* ---- standalone kernels on device pointers (stream: hipStream_t or NULL) -----------
 * Layouts: pi/mu/dlogits (T,B,A) fp32; actions (T,B) int32; rewards/discounts/vs/pg_adv
 * (T,B) fp32; values/dvalue (T+1,B) fp32; losses_dev: 3 doubles {pg, baseline, entropy}.
 * workspace: fi_vtrace_workspace_bytes() bytes of device scratch (one per stream in flight).
 * losses_dev may be NULL: the loss sums are then not finalised (one kernel launch only).     */
size_t fi_vtrace_workspace_bytes(int T, int B, int A);
int fi_vtrace_loss_fp32(int T, int B, int A, const float* pi_logits, const float* mu_logits,
                        const int32_t* actions, const float* rewards, const float* discounts,
                        const float* values, const fi_vtrace_hparams* hp, float* vs,
                        float* pg_adv, float* dlogits, float* dvalue, double* losses_dev,
                        void* workspace, size_t workspace_bytes, void* stream);
/* variant: 0 = auto, 1 = LDS-staged scan kernel, 2 = one-column-per-lane kernel        */
int fi_vtrace_loss_fp32_variant(int variant, int T, int B, int A, const float* pi_logits,
                                const float* mu_logits, const int32_t* actions,
                                const float* rewards, const float* discounts,
                                const float* values, const fi_vtrace_hparams* hp, float* vs,
                                float* pg_adv, float* dlogits, float* dvalue,
                                double* losses_dev, void* workspace, size_t workspace_bytes,
                                void* stream);
/* Repack B host-layout entries already copied to the device ((B, S*1024) bytes) into the
 * time-major SoA tensors (record schema: DESIGN.md section 3).                            */
int fi_ingest_records(const void* records_dev, int T, int B, int A, int D,
                      size_t entry_bytes, float* obs, float* mu, int32_t* actions,
                      float* rewards, float* discounts, void* stream);
/* Device synthetic trajectories (Philox4x32-10; bit-identical to the oracle's generator) */
int fi_synth_trajectories(uint64_t seed, int T, int B, int B_glob, int b_off, int A, int D,
                          float gamma, float* obs, float* mu, int32_t* actions,
                          float* rewards, float* discounts, uint8_t* frames, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FI_LEARNER_H_ */
