/*
 * ecnf.h — C-ABI of libecnf_hip.so, the MI355X (gfx950) equivariant-CNF sample / log_prob path.
 *
 * The reference (Kalyan0821/ecnf-baseline-neurips-2023) is pure JAX; its "plugin/operator API" for this
 * path is the FlowMatchingCNF bundle and the three solver entry points.  Each function below replaces one
 * of them (file:line in the reference snapshot):
 *
 *   ecnf_create / ecnf_destroy   <- build_cnf(...) + cnf.init params   ecnf/cnf/build_cnf.py:34-102
 *                                   (the handle owns the device copy of the flat params blob)
 *   ecnf_vector_field            <- cnf.apply(params, x, t, features)  ecnf/cnf/core.py:7-19,45;
 *                                   FlatEgnn.__call__ build_cnf.py:68-93; EGNN egnn.py:130-190
 *   ecnf_vf_jvp                  <- jax.vjp(cnf.apply) + vmap(vjp_fn)  ecnf/cnf/sample_and_log_prob.py:64-66,75-77
 *                                   (forward-mode tangents J @ u instead of reverse-mode u^T J)
 *   ecnf_integrate               <- diffrax.diffeqsolve(ODETerm, Dopri5, [PIDController])
 *                                   sample_and_log_prob.py:28-38 (sample_cnf), :81-94 (get_log_prob),
 *                                   :135-149 (sample_and_log_prob_cnf)
 *   ecnf_base_sample             <- cnf.sample_base (distrax Transformed._sample_n)
 *                                   zero_com_base.py:16-19,88-93 + build_cnf.py:46-61
 *   ecnf_base_log_prob           <- cnf.log_prob_base  zero_com_base.py:21-24,64-84 + build_cnf.py:50-57
 *   ecnf_target_log_prob         <- target log_prob_fn (-energy) of LJ13 / DW4   
 *                                   ecnf/targets/target_energy/leonard_jones.py:10-35, double_well.py:9-28
 *   ecnf_lse_partials            <- the log-sum-exp reductions behind forward / reverse ESS  (section 8f, rank 2)
 *                                   ecnf/utils/evaluation.py:10-22, setup_training.py:182
 *   ecnf_last_error              <- the chex / diffrax exceptions (trace-time asserts, max_steps)
 *
 * Conventions
 *   - every array argument is a DEVICE pointer (hipMalloc'd or a torch tensor's data_ptr()), fp32 / int32,
 *     contiguous row-major; x is flat [batch, n_nodes*dim] exactly like the reference's flat events.
 *   - `stream` is a hipStream_t (NULL = default stream).  Calls are stream-ordered and asynchronous,
 *     except ecnf_create/ecnf_destroy which synchronise.
 *   - return value: ECNF_OK or an ECNF_E_* code; ecnf_last_error() gives a thread-local message.
 *   - one handle per device; a handle is not re-entrant, distinct handles may be used from distinct threads.
 */
#ifndef ECNF_H_
#define ECNF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECNF_ABI_VERSION 3

enum ecnf_status {
  ECNF_OK = 0,
  ECNF_E_INVALID = 1,      /* bad argument / shape (the reference's chex.assert_* failures) */
  ECNF_E_UNSUPPORTED = 2,  /* a configuration this build has no kernel for */
  ECNF_E_HIP = 3,          /* a HIP runtime error (message in ecnf_last_error) */
  ECNF_E_MAX_STEPS = 4,    /* reported per molecule through ecnf_integrate's `status` output */
  ECNF_E_NONFINITE = 5     /* per molecule: the final state (positions or log-density) is not finite, e.g. an
                              activation beyond the fp16 range (|a| >= 65504) of the split GEMMs; rerun those
                              molecules with ECNF_PREC_FP32 (ecnf_amd does this automatically) */
};

/* GEMM arithmetic of a handle's kernels (ecnf_set_precision):
 *   ECNF_PREC_SPLIT_F16  (default) fp32 operands split into two fp16 pieces, three cross terms on the 16-bit
 *                        matrix cores with fp32 accumulation (fp32-class accuracy; activations must stay below
 *                        65504 in magnitude, else the molecule reports ECNF_E_NONFINITE)
 *   ECNF_PREC_FP32       every GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32): the strict-fp32 path */
enum ecnf_precision { ECNF_PREC_SPLIT_F16 = 0, ECNF_PREC_FP32 = 1 };

enum ecnf_solver { ECNF_SOLVER_EULER = 0, ECNF_SOLVER_DOPRI5 = 1 };
enum ecnf_divergence { ECNF_DIV_NONE = 0, ECNF_DIV_HUTCHINSON = 1, ECNF_DIV_EXACT = 2 };

/* Model hyper-parameters: the `flow:` block of examples/config/{dw4,lj13,aldp,qm9}.yaml and the
 * build_cnf(...) arguments (build_cnf.py:34-44).  mlp_units is (mlp_width,) * mlp_depth. */
typedef struct ecnf_cfg {
  int32_t n_nodes;             /* n_frames (N), 2 .. 64                          */
  int32_t dim;                 /* spatial dim (D): 2 or 3                        */
  int32_t n_features;          /* nn.Embed vocabulary                            */
  int32_t hidden;              /* n_invariant_feat_hidden (H): multiple of 32    */
  int32_t time_embedding_dim;  /* T: even, 4 <= T <= 16                          */
  int32_t mlp_width;           /* M: 64, 128 or 256                              */
  int32_t mlp_depth;           /* L = len(mlp_units): 2..4                       */
  int32_t n_blocks;            /* n_blocks_egnn (K): 1..10                       */
  float base_scale;            /* ScalarAffine scale of the base (build_cnf.py:46) */
  float normalization_constant;/* EGCL C (egnn.py:127), 1.0 in the reference     */
} ecnf_cfg;

/* Options of one ODE solve (diffeqsolve arguments).  t0 < t1 samples (0 -> 1); t0 > t1 is the
 * density direction of get_log_prob (1 -> 0).  dt0 > 0 selects ConstantStepSize; dt0 <= 0 selects
 * PIDController(rtol, atol, dtmin) with Hairer's initial step (dt0=None in the reference). */
typedef struct ecnf_solve_opts {
  int32_t solver;      /* ecnf_solver                       */
  int32_t divergence;  /* ecnf_divergence: d logp / dt term */
  float t0, t1;
  float dt0;           /* > 0: fixed step; <= 0: adaptive   */
  float rtol, atol, dtmin;
  int32_t max_steps;   /* diffrax default 4096              */
} ecnf_solve_opts;

typedef struct ecnf_handle ecnf_handle;

/* Number of fp32 params the flat blob must hold for `cfg` (the jax ravel_pytree order of the flax
 * params tree: EGNN_0/{k}/{Dense_0,Dense_1,phi_e,phi_h,phi_x_torso}, EGNN_0/Dense_k, final_scaling,
 * Embed_0/embedding, sorted keys, bias before kernel). */
int ecnf_param_count(const ecnf_cfg* cfg, size_t* n_floats);

/* Upload `params` (HOST pointer, n_floats fp32) to `device`, repack them into MFMA fragment order and
 * return a handle.  Synchronous. */
int ecnf_create(const ecnf_cfg* cfg, const float* params, size_t n_floats, int device, ecnf_handle** out);
int ecnf_destroy(ecnf_handle* h);

/* v[b] = apply(params, x[b], t[b], feat[b])   (x, v: [batch, N*D]; t: [batch]; feat: [batch, N]). */
int ecnf_vector_field(ecnf_handle* h, const float* x, const float* t, const int32_t* feat, float* v,
                      int32_t batch, void* stream);

/* Forward-mode Jacobian-vector products: tan_out[b, k] = (d apply / d x)(x[b]) @ tan_in[b, k] for
 * k < n_tangents (tan_in/tan_out: [batch, n_tangents, N*D]); v as in ecnf_vector_field (may be NULL). */
int ecnf_vf_jvp(ecnf_handle* h, const float* x, const float* t, const int32_t* feat, const float* tan_in,
                int32_t n_tangents, float* v, float* tan_out, int32_t batch, void* stream);

/* Solve the ODE for every molecule of the batch in ONE launch (each workgroup integrates its molecules
 * end to end; adaptive steps are per molecule, as under jax.vmap).
 *   y0   [batch, N*D]  initial positions (at t0)
 *   eps  [batch, N*D]  Hutchinson probe (required for ECNF_DIV_HUTCHINSON, else ignored / NULL)
 *   y1   [batch, N*D]  positions at t1
 *   dlogp[batch]       l(t1) with dl/dt = div v, l(t0) = 0 (NULL allowed when divergence == NONE)
 *   nfe  [batch]       vector-field evaluations spent on the molecule (NULL allowed)
 *   status [batch]     ECNF_OK, ECNF_E_MAX_STEPS or ECNF_E_NONFINITE per molecule (NULL allowed) */
int ecnf_integrate(ecnf_handle* h, const ecnf_solve_opts* opts, const float* y0, const int32_t* feat,
                   const float* eps, float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch,
                   void* stream);

/* Device workspace of a solve.  The exact trace (ECNF_DIV_EXACT) runs N*D - D JVP passes per evaluation whose
 * primal is the same; with a workspace, the first pass caches the primal edge aggregates of the blocks whose edge
 * tangents are sparse (blocks 1 and K) and the later passes skip those primal tiles.  Results are bitwise equal with
 * and without a workspace; only the time differs (LJ13 B = 1024 Euler-100 log_prob: ~1.35 s vs ~1.75 s).
 * Adaptive (Dopri5 + PID) solves of 2 .. 2^20 molecules also use it, after the exact trace's cache, for the re-deal
 * scratch: when the batch needs more workgroups than the device has CUs, a first launch runs every molecule for a
 * few steps and stores its solver state, and a second launch resumes the unfinished molecules longest estimated
 * remainder first, so the slow molecules do not start late in dispatch order (ALDP B = 512 PID log_prob: ~43 ms vs
 * ~53 ms).  Where the shape has a tangent team kernel (ALDP's M = 64 network, one molecule per workgroup), the second
 * launch of a Hutchinson solve also runs its longest-estimate eighth of the molecules (at most 64) as teams of two
 * workgroups (ecnf_set_team below), stops every molecule at a step boundary once at most 64 are unfinished, and a
 * third launch resumes those as teams of four (~36 ms).  Bitwise the same results; a workspace too small for both
 * regions runs the solve in one launch.
 *   ecnf_integrate_workspace_size  bytes a call with these options and batch needs (0: none is used)
 *   ecnf_integrate_ws              ecnf_integrate with a CALLER-owned device workspace (NULL: none); the workspace is
 *                                  used stream-ordered on `stream` only, so concurrent calls with distinct
 *                                  workspaces are independent.  A non-NULL workspace below the size is ECNF_E_INVALID.
 *   ecnf_reserve_workspace         allocate (synchronously, outside the solve calls) a handle-owned arena that
 *                                  ecnf_integrate uses when it is large enough; calls on different streams that share
 *                                  it are ordered by an event (no host synchronisation).
 * The solve calls themselves never allocate or free device memory. */
int ecnf_integrate_workspace_size(ecnf_handle* h, const ecnf_solve_opts* opts, int32_t batch, size_t* bytes);
int ecnf_integrate_ws(ecnf_handle* h, const ecnf_solve_opts* opts, const float* y0, const int32_t* feat,
                      const float* eps, float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch,
                      void* workspace, size_t workspace_bytes, void* stream);
int ecnf_reserve_workspace(ecnf_handle* h, size_t bytes);
/* Diagnostic: how a solve with these options and batch is launched when given a workspace of
 * ecnf_integrate_workspace_size bytes -- the workgroups of its (first) launch and the number of launches (2: the
 * chunked, re-dealt adaptive solve above; 3: the same with tail teams and the stop-and-team launch; 1: one launch). */
int ecnf_integrate_plan(ecnf_handle* h, const ecnf_solve_opts* opts, int32_t batch, int32_t* workgroups,
                        int32_t* launches);

/* A/B diagnostics of the exact trace (not needed in production; results: SPARSE and DEFAULT are bitwise equal, ALL_DUAL
 * agrees to fp32 rounding):  DEFAULT  sparse blocks 1 and K + the primal cache when a workspace is available;
 * ALL_DUAL every edge tile carries a tangent;  SPARSE  sparse blocks without the cache. */
enum ecnf_exact_form { ECNF_EXACT_FORM_DEFAULT = 0, ECNF_EXACT_FORM_ALL_DUAL = 1, ECNF_EXACT_FORM_SPARSE = 2 };
int ecnf_set_exact_form(ecnf_handle* h, int32_t form);

/* Team (latency) mode of the primal solves (DIV_NONE: sample_cnf), for batches far below the CU count -- the
 * reference's one-molecule-per-call sampling timer (examples/load_checkpoint_measure_sampling_time.py:101-119):
 * G workgroups integrate one molecule together, its edge tiles dealt over them, the edge aggregates exchanged through
 * global memory after every block's edge phase (a cooperative launch of batch x G workgroups).  Results are bitwise
 * those of the batch path.  mode: 0 auto (G = ceil(edge tiles / waves) when M = 256, batch x G <= CUs and
 * batch <= 32), 1 off (also turns off the re-dealt solves' tail teams), G >= 2 forced (batch <= 64, capped by the
 * handle's buffers).  Hutchinson tangent solves (get_log_prob / sample_and_log_prob_cnf with approx=True) of ALDP's
 * M = 64 network have a team kernel too (the tangent message and shift rows are exchanged as well), used when forced
 * and for the re-dealt solves' tail teams; the exact trace always takes the batch path.  ecnf_team_workgroups reports
 * the G a solve of `batch` molecules would use (1: the batch path; with_tangent: a Hutchinson solve).  A team whose
 * exchange times out (a member not co-resident) reports status ECNF_E_HIP for its molecule. */
int ecnf_set_team(ecnf_handle* h, int32_t mode);
int ecnf_team_workgroups(ecnf_handle* h, int32_t with_tangent, int32_t batch, int32_t* G);

/* x0 = base_scale * (z - mean_nodes(z)) for a standard-normal draw z [batch, N*D]. */
int ecnf_base_sample(ecnf_handle* h, const float* z, float* x0, int32_t batch, void* stream);

/* log_prob_base(y) [batch] of the scaled zero-CoM Gaussian. */
int ecnf_base_log_prob(ecnf_handle* h, const float* y, float* log_p, int32_t batch, void* stream);

/* Select the GEMM arithmetic (ecnf_precision) of every later call on this handle; ecnf_get_precision reads it. */
int ecnf_set_precision(ecnf_handle* h, int32_t precision);
int ecnf_get_precision(ecnf_handle* h, int32_t* precision);

/* Molecules processed by one workgroup for this handle (diagnostic; kernels pick it from the LDS budget). */
int ecnf_molecules_per_workgroup(ecnf_handle* h, int32_t with_tangent, int32_t* mpw);

/* Arithmetic of the edge-MLP chain GEMMs (the bulk of the FLOPs) in this handle's kernels at its current precision
 * (diagnostic):
 *   ECNF_CHAIN_FP32_MFMA   v_mfma_f32_32x32x2_f32, fp32 operands
 *   ECNF_CHAIN_SPLIT_BF16  (reserved: the round-1 three-piece bf16 form, no longer built)
 *   ECNF_CHAIN_SPLIT_F16   fp32 operands split into two fp16 pieces (RNE; node-GEMM weights scaled by a power of two
 *                          per matrix), the three cross terms above 2^-21 of the product on v_mfma_f32_32x32x16_f16,
 *                          fp32 accumulation */
#define ECNF_CHAIN_FP32_MFMA 0
#define ECNF_CHAIN_SPLIT_BF16 1
#define ECNF_CHAIN_SPLIT_F16 2
int ecnf_chain_arithmetic(ecnf_handle* h, int32_t with_tangent, int32_t* mode);

/* ---- targets and eval reductions (no handle needed) ---- */
enum ecnf_target_kind { ECNF_TARGET_LJ = 0, ECNF_TARGET_DW = 1 };

/* Target energy parameters.  LJ (leonard_jones.py:10-27): epsilon, tau, r (a scalar, or the reference's per-node
 * array `r: chex.Array` as r_nodes, a DEVICE float[n_nodes]; pair (receiver i, sender j) uses r_i,
 * leonard_jones.py:14-16,20), harmonic_coef.  DW (double_well.py:9-19): a, b, c, d0, tau.  Defaults are the
 * reference's keyword defaults (LJ: 1, 1, 1, 0.5; DW: 0, -4, 0.9, 4, 1). */
typedef struct ecnf_target {
  int32_t kind;      /* ecnf_target_kind */
  int32_t n_nodes;
  int32_t dim;
  float epsilon, tau, r, harmonic_coef;  /* LJ */
  float a, b, c, d0;                     /* DW (tau shared) */
  const float* r_nodes;                  /* LJ: per-node r (device, n_nodes floats) or NULL for the scalar r */
} ecnf_target;

/* log_p[i] = -energy(x[i]) for x [batch, n_nodes*dim] (log_prob_fn of the target).  Pair distances use
 * safe_norm (1 for coincident atoms) and the ordered-pair sum of the reference (each pair counted twice). */
int ecnf_target_log_prob(const ecnf_target* t, const float* x, float* log_p, int32_t batch, void* stream);

/* One workgroup reduces v[0..n) (entries with mask[i] <= 0 skipped when mask != NULL) to log-sum-exp partials
 * for the scales s = +1, -1, +2:  out[2k] = max_i s v_i,  out[2k+1] = sum_i exp(s v_i - out[2k]),  out[6] = count.
 * out is a DEVICE float[7].  Ranks combine partials with one MAX and one SUM all-reduce (ecnf_amd.distributed). */
int ecnf_lse_partials(const float* v, const float* mask, int32_t n, float* out, void* stream);

/* ---- flow-matching training --------------------------------------------------
 *   ecnf_fm_loss_grad   <- jax.grad(flow_matching_loss_fn)     ecnf/cnf/loss.py:10-32, cnf/gradient_step.py:30-36
 *   ecnf_adam_update    <- optax.adam update + apply_updates (+ EMA)   gradient_step.py:38-51, setup_training.py:100-109
 *   ecnf_update_params  <- the new state.params in cnf.apply (re-packs a sampling handle's weights)
 * Parameters, gradients and Adam moments are DEVICE flat fp32 blobs in the ravel_pytree order (ecnf_param_count).
 * Every dense layer runs on the fp32 matrix cores (v_mfma_f32_32x32x2_f32); the step is deterministic. */
typedef struct ecnf_trainer ecnf_trainer;

/* Workspace for batches of up to max_batch molecules (activations kept for the backward pass). */
int ecnf_trainer_create(const ecnf_cfg* cfg, int32_t max_batch, int device, ecnf_trainer** out);
int ecnf_trainer_destroy(ecnf_trainer* tr);

/* Diagnostic: shrink the partial arena of the step's deferred split reductions to `floats` (clamped to
 * [the embedding partials' minimum, the allocated size]; 0 restores the allocated size) and return the size in use
 * through `used` (may be NULL).  A small arena makes the step flush mid-way and choose fewer K-splits; the
 * gradient agrees with the default arena to fp32 rounding (tests/test_gpu_train.py). */
int ecnf_trainer_set_reduction_arena(ecnf_trainer* tr, size_t floats, size_t* used);

/* loss[0] = mean((v(x_t, t) - u_t)^2) over batch x N*D with x_t = (1 - (1 - sigma_min) t) x0 + t x1,
 * u_t = x1 - (1 - sigma_min) x0 (core.py:35-39); grad = d loss / d params.  x1 (data), x0 (base sample):
 * [batch, N*D]; t: [batch]; feat: [batch, N] (ids must lie in [0, n_features)); loss: DEVICE float[1]. */
int ecnf_fm_loss_grad(ecnf_trainer* tr, const float* params, const float* x1, const float* x0, const float* t,
                      const int32_t* feat, float sigma_min, int32_t batch, float* loss, float* grad, void* stream);

/* optax.adam(lr, b1, b2, eps, eps_root) at step `count` (1 for the first update: the bias corrections use
 * 1 - b^count) applied in place: params += -lr mu_hat / (sqrt(nu_hat + eps_root) + eps); ema (optional, may be
 * NULL) = ema * ema_beta + (1 - ema_beta) * params.  norms (optional): DEVICE float[2] = (|grad|, |update|), the
 * optax.global_norm values of gradient_step.py:41-44. */
typedef struct ecnf_adam_opts {
  float lr, b1, b2, eps, eps_root;
  int32_t count;
  float ema_beta;
} ecnf_adam_opts;
int ecnf_adam_update(ecnf_trainer* tr, const float* grad, float* params, float* mu, float* nu, float* ema, size_t n,
                     const ecnf_adam_opts* opts, float* norms, void* stream);

/* Replace a handle's weights with the blob `params` (on_device: a DEVICE pointer, else host).  Synchronous. */
int ecnf_update_params(ecnf_handle* h, const float* params, int32_t on_device);

/* Layout of the ABI structs as this library was compiled: out[0] = sizeof, out[1 + i] = offsetof field i (declaration
 * order) for which = 0 ecnf_cfg, 1 ecnf_solve_opts, 2 ecnf_target, 3 ecnf_adam_opts.  Writes min(cap, 1 + fields)
 * values and returns the number of fields (-1 for an unknown `which`).  Bindings (ctypes, cgo, ...) check their struct
 * mirrors against it. */
int ecnf_struct_layout(int32_t which, size_t* out, int32_t cap);

/* Thread-local description of the last error ("" when none). */
const char* ecnf_last_error(void);

int ecnf_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ECNF_H_ */
