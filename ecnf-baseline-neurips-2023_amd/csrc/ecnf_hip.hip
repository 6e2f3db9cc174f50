// ecnf_hip.hip — libecnf_hip.so: the equivariant-CNF sample / log_prob path on MI355X (gfx950).
//
// Kernels: ecnf_kernels.hpp (integrate_kernel, vf_kernel); here the base-distribution kernels
//   base kernels     zero-CoM Gaussian projection and log-density    <- distrax Transformed(FlatZeroCoMGaussian)
// Host
//   parameter walk of the flat (ravel_pytree-ordered) blob, repacking into MFMA fragment order, C-ABI.
// Build: one translation unit (every shape instantiated here), or with -DECNF_SPLIT_TU, where the shapes are
// compiled in parallel as ecnf_part.hip units (__graft_entry__.build()) and only declared here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ecnf.h"
#include "ecnf_kernels.hpp"

namespace ecnf {

// every shape in both GEMM arithmetics (P = 0 split fp16, P = 1 strict fp32)
#define ECNF_INST_PRIMAL(m, l, d) \
  ECNF_INST_SHAPE(ECNF_INST_KW, m, l, d, 0, 0) ECNF_INST_SHAPE(ECNF_INST_KW, m, l, d, 0, 1)
#define ECNF_INST_BOTH(m, l, d) \
  ECNF_INST_PRIMAL(m, l, d) ECNF_INST_SHAPE(ECNF_INST_KW, m, l, d, 1, 0) ECNF_INST_SHAPE(ECNF_INST_KW, m, l, d, 1, 1)
#define ECNF_INST_WIDE(m, l, d) ECNF_INST_BOTH(m, l, d)
#ifdef ECNF_SPLIT_TU
#define ECNF_INST_KW extern template
#else
#define ECNF_INST_KW template
#endif
ECNF_SHAPES(ECNF_INST_BOTH)
ECNF_SHAPES_WIDE_TAN(ECNF_INST_WIDE)
#undef ECNF_INST_KW

// x0 = s * (z - mean_nodes z)   (zero_com_base.py:88-93, build_cnf.py:46)
__global__ void base_sample_kernel(const float* __restrict__ z, float* x0, int B, int N, int D, float scale) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;   // (b, d)
  if (idx >= B * D) return;
  const int bb = idx / D, d = idx - bb * D;
  const float* zb = z + (size_t)bb * N * D;
  float acc = 0.f;
  for (int i = 0; i < N; ++i) acc += zb[i * D + d];
  const float mean = acc / (float)N;
  for (int i = 0; i < N; ++i) x0[(size_t)bb * N * D + i * D + d] = scale * (zb[i * D + d] - mean);
}

// log N_{(N-1)D}(remove_mean(y / s)) - (N-1) D log s   (zero_com_base.py:64-84, build_cnf.py:50-57)
__global__ void base_log_prob_kernel(const float* __restrict__ y, float* out, int B, int N, int D, float scale) {
  const int bb = blockIdx.x * blockDim.x + threadIdx.x;
  if (bb >= B) return;
  const float* yb = y + (size_t)bb * N * D;
  const float inv = 1.0f / scale;
  float mean[3] = {0.f, 0.f, 0.f};
  for (int i = 0; i < N; ++i)
    for (int d = 0; d < D; ++d) mean[d] += yb[i * D + d] * inv;
  for (int d = 0; d < D; ++d) mean[d] /= (float)N;
  float r2 = 0.f;
  for (int i = 0; i < N; ++i)
    for (int d = 0; d < D; ++d) {
      const float u = yb[i * D + d] * inv - mean[d];
      r2 += u * u;
    }
  const int dof = (N - 1) * D;
  const float log_norm = -0.5f * (float)dof * logf(2.0f * 3.14159265358979f);
  const float ildj = -(float)(N * D) * logf(scale) * (float)(N - 1) / (float)N;
  out[bb] = -0.5f * r2 + log_norm + ildj;
}

// -log_p = energy of the LJ / DW targets (leonard_jones.py:10-27, double_well.py:9-19), one thread per molecule.
// The reference sums f(d) over the N(N-1) ordered pairs; each unordered pair is visited once here and both orders
// are added (LJ: with the receiver's r, a per-node array when r_nodes != NULL).
__global__ void target_log_prob_kernel(ecnf_target t, const float* __restrict__ x, float* log_p, int B) {
  const int bb = blockIdx.x * blockDim.x + threadIdx.x;
  if (bb >= B) return;
  const int N = t.n_nodes, D = t.dim;
  const float* xb = x + (size_t)bb * N * D;
  float pair = 0.f;
  for (int i = 0; i < N; ++i)
    for (int j = i + 1; j < N; ++j) {
      float x2 = 0.f;
      for (int d = 0; d < D; ++d) {
        const float v = xb[j * D + d] - xb[i * D + d];
        x2 += v * v;
      }
      const float dist = sqrtf(x2 == 0.f ? 1.0f : x2);   // safe_norm (numerical.py:7-10)
      if (t.kind == ECNF_TARGET_LJ) {
        // ordered pairs (receiver i, sender j) and (j, i) use the receiver's r (leonard_jones.py:20)
        const float ri = t.r_nodes ? t.r_nodes[i] : t.r, rj = t.r_nodes ? t.r_nodes[j] : t.r;
        const float qi = ri / dist, qi2 = qi * qi, qi6 = qi2 * qi2 * qi2;
        const float qj = rj / dist, qj2 = qj * qj, qj6 = qj2 * qj2 * qj2;
        pair += (qi6 * qi6 - 2.0f * qi6) + (qj6 * qj6 - 2.0f * qj6);
      } else {
        const float u = dist - t.d0, u2 = u * u;
        pair += 2.0f * (t.a * u + t.b * u2 + t.c * u2 * u2);
      }
    }
  float e;
  if (t.kind == ECNF_TARGET_LJ) {
    float com[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < N; ++i)
      for (int d = 0; d < D; ++d) com[d] += xb[i * D + d];
    for (int d = 0; d < D; ++d) com[d] /= (float)N;
    float h = 0.f;
    for (int i = 0; i < N; ++i)
      for (int d = 0; d < D; ++d) {
        const float v = xb[i * D + d] - com[d];
        h += v * v;
      }
    e = t.epsilon / (2.0f * t.tau) * pair + t.harmonic_coef * h;
  } else {
    e = pair / t.tau / 2.0f;
  }
  log_p[bb] = -e;
}

// log-sum-exp partials (max, sum exp(s v - max)) for s = +1, -1, +2 and the count, one workgroup: online
// rescaling per thread, then a tree over the workgroup in LDS
constexpr int kLseThreads = 1024;
// v = -inf has zero weight (exp(-inf) = 0, as jax.nn.logsumexp gives it) and is skipped; equal maxima (+inf) add
// their counts instead of exp(inf - inf) = NaN.  A NaN value makes the partial NaN.
__device__ __forceinline__ void lse_push(float& m, float& s, float v) {
  if (v == -INFINITY) return;
  if (v > m) {
    s = (m == -INFINITY ? 0.0f : s * __expf(m - v)) + 1.0f;
    m = v;
  } else {
    s += (v == m) ? 1.0f : __expf(v - m);
  }
}
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 > m) {
    s = (m == -INFINITY ? 0.0f : s * __expf(m - m2)) + s2;
    m = m2;
  } else if (m2 > -INFINITY) {
    s += (m2 == m) ? s2 : s2 * __expf(m2 - m);
  } else if (m2 != m2) {
    m = m2;
    s = m2;
  }
}
__global__ __launch_bounds__(kLseThreads) void lse_partials_kernel(const float* __restrict__ v,
                                                                   const float* __restrict__ mask, int n, float* out) {
  __shared__ float red[7][kLseThreads];
  float m[3] = {-INFINITY, -INFINITY, -INFINITY}, sm[3] = {0.f, 0.f, 0.f}, cnt = 0.f;
  const float sc[3] = {1.0f, -1.0f, 2.0f};
  for (int i = threadIdx.x; i < n; i += kLseThreads) {
    if (mask && !(mask[i] > 0.f)) continue;
    cnt += 1.0f;
    for (int k = 0; k < 3; ++k) lse_push(m[k], sm[k], sc[k] * v[i]);
  }
  const int tid = threadIdx.x;
  for (int k = 0; k < 3; ++k) {
    red[2 * k][tid] = m[k];
    red[2 * k + 1][tid] = sm[k];
  }
  red[6][tid] = cnt;
  __syncthreads();
  for (int w = kLseThreads / 2; w > 0; w >>= 1) {
    if (tid < w) {
      for (int k = 0; k < 3; ++k) {
        float mm = red[2 * k][tid], ss = red[2 * k + 1][tid];
        lse_merge(mm, ss, red[2 * k][tid + w], red[2 * k + 1][tid + w]);
        red[2 * k][tid] = mm;
        red[2 * k + 1][tid] = ss;
      }
      red[6][tid] += red[6][tid + w];
    }
    __syncthreads();
  }
  if (tid < 7) out[tid] = red[tid][0];
}

// Re-deal of a chunked adaptive solve (integrate_impl): the molecules still unfinished after the first chunk
// (SolverState kSsActive), ordered by their estimated remaining steps (tau1 - tau) / dt, longest first (ties in batch
// order), into order[0 .. *nslots).  The next launch resumes them in that order: with more workgroups than CUs, the
// workgroups start in dispatch order as CUs free up, and a long solve dealt late finishes late (ALDP B = 512 PID
// log_prob: 55.5 ms in batch order, 37.9 ms with the molecules sorted by their step counts; the slowest molecule alone
// 36.8 ms).  One workgroup, bitonic sort of (key, index): in LDS up to kRedealLds molecules, beyond that in the
// workspace (gkey / gidx, next power of two entries; one workgroup's global accesses are ordered by its barriers).
constexpr int kRedealLds = 4096;
constexpr int kRedealMax = 1 << 20;
constexpr int kRedealThreads = 1024;
__host__ __device__ inline int pow2_at_least(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}
// step controls of a re-dealt solve's first launch (sched_floats).  ALDP B = 512 PID log_prob (tools/diag/
// redeal_keys.py, sched_check.py): after 2 / 4 / 8 steps the (tau1 - tau) / dt order ranks the remaining NFE at
// Spearman 0.29 / 0.53 / 0.82 and the launch takes 51.8 / 44.3 / 43.9 ms (one launch: 55.3); at 8 the second launch's
// makespan equals that of the true remaining-NFE order, the rest is the first launch's two rounds of 512 workgroups
constexpr int kChunkSteps = 8;

// Tail teams (ALDP's tangent kernels, team_shape with NT = 1): the re-dealt launch runs its K longest-estimate slots as
// teams of kTailG workgroups (egnn_eval.hpp team_exchange; results bitwise the batch path's), an evaluation 1.24 times
// faster at 2 CUs (tools/team_tangent_probe.py: ALDP 107 us per evaluation alone, G = 2 / 3 / 4: 86 / 85 / 75 us).
// K = the longest eighth of the unfinished slots, at most kmax (the exchange buffers; at most half the CUs in teams).
// Chosen by measurement against the alternatives (tools/diag/tail_sim.py, profiles/round6/aldp_tail/): ALDP B = 512
// PID Hutchinson log_prob from base draws 42.6 -> 37.7 ms (G = 4 with a makespan model choosing K = 26: 39.3 ms; G = 4,
// K = 32: 39.7 ms); from real frames, whose long solves the 8-step estimate ranks worse, 49.8 -> 50.4 ms.
constexpr int kTailG = 2;
// Stop-and-team: the tail-team launch stops every molecule at its next step boundary once at most kStopLeft of its
// slots are unfinished, and a third launch resumes the survivors as teams of kStopG (every CU in a team)
#ifdef ECNF_STOP_G   // (experiment builds)
constexpr int kStopG = ECNF_STOP_G;
#else
constexpr int kStopG = 4;
#endif

__global__ __launch_bounds__(kRedealThreads) void redeal_kernel(const float* __restrict__ state, int stride, int ND,
                                                                int B, float tau1, int* order, int* nslots, float* gkey,
                                                                int* gidx, int* nteam, int kmax, int team_all) {
  __shared__ float lkey[kRedealLds];
  __shared__ int lidx[kRedealLds];
  const int tid = threadIdx.x;
  const int n2 = pow2_at_least(B);
  float* key = n2 <= kRedealLds ? lkey : gkey;
  int* idx = n2 <= kRedealLds ? lidx : gidx;
  for (int i = tid; i < n2; i += kRedealThreads) {
    float k = -INFINITY;   // finished molecules and padding sort last
    if (i < B) {
      const float* S = state + (size_t)i * stride + 2 * ND;
      if (__builtin_bit_cast(int, S[kSsActive])) {
        const float r = (tau1 - S[kSsTau]) / S[kSsDt];
        k = r >= 0.f ? fminf(r, 3.0e38f) : (r < 0.f ? 0.f : 3.0e38f);   // a NaN estimate (non-finite step) first
      }
    }
    key[i] = k;
    idx[i] = i;
  }
  __syncthreads();
  // bitonic sort into "before" order: larger key first, then smaller index (a strict total order)
  for (int size = 2; size <= n2; size <<= 1)
    for (int half = size >> 1; half > 0; half >>= 1) {
      for (int i = tid; i < n2; i += kRedealThreads) {
        const int j = i ^ half;
        if (j > i) {
          const float ki = key[i], kj = key[j];
          const int ii = idx[i], ij = idx[j];
          const bool j_before = kj > ki || (kj == ki && ij < ii);
          if (((i & size) == 0) == j_before) {
            key[i] = kj;
            key[j] = ki;
            idx[i] = ij;
            idx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < B; i += kRedealThreads) {
    if (!(key[i] > -INFINITY)) continue;
    order[i] = idx[i];
    if (i + 1 == B || !(key[i + 1] > -INFINITY)) *nslots = i + 1;
  }
  if (tid == 0 && !(key[0] > -INFINITY)) *nslots = 0;
  if (!nteam) return;
  __syncthreads();
#ifndef ECNF_TAIL_DIV   // (experiment builds may override)
#define ECNF_TAIL_DIV 8
#endif
  if (tid == 0) *nteam = min(kmax, team_all ? *nslots : (*nslots + ECNF_TAIL_DIV - 1) / ECNF_TAIL_DIV);
}

}  // namespace ecnf

// =====================================================================================================
// host side
// =====================================================================================================
using namespace ecnf;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

}  // namespace

// shared with the training translation unit (ecnf_train.hip): sets the thread-local ecnf_last_error() text
namespace ecnf {
int set_error(int code, const char* msg) {
  g_err = msg;
  return code;
}
}  // namespace ecnf

namespace {

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(ECNF_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// edge slots per receiver (Net::SR): the receiver runs packed back to back while a run fits one 32-edge tile
// (N <= 33: a run touches at most two tiles); beyond that every run is padded to two whole tiles
constexpr int kMaxNodes = 64;
int edge_slots_per_receiver(int n_nodes) { return n_nodes - 1 <= 32 ? n_nodes - 1 : 64; }

int check_cfg(const ecnf_cfg* c) {
  if (!c) return fail(ECNF_E_INVALID, "cfg is NULL");
  if (c->n_nodes < 2 || c->n_nodes > kMaxNodes)
    return fail(ECNF_E_UNSUPPORTED, "n_nodes must be in [2, 64] (a receiver's N-1 edges must fit two 32-edge tiles)");
  if (c->dim != 2 && c->dim != 3) return fail(ECNF_E_UNSUPPORTED, "dim must be 2 or 3");
  if (c->n_features < 1) return fail(ECNF_E_INVALID, "n_features must be >= 1");
  if (c->hidden < 32 || c->hidden % 32) return fail(ECNF_E_UNSUPPORTED, "hidden must be a multiple of 32");
  if (c->time_embedding_dim < 4 || c->time_embedding_dim > 2 * kMaxHalfT || c->time_embedding_dim % 2)
    return fail(ECNF_E_UNSUPPORTED, "time_embedding_dim must be even and in [4, 16]");
  if (c->mlp_width != 64 && c->mlp_width != 128 && c->mlp_width != 256)
    return fail(ECNF_E_UNSUPPORTED, "mlp_width must be 64, 128 or 256");
  if (c->mlp_depth < 2 || c->mlp_depth > 4) return fail(ECNF_E_UNSUPPORTED, "mlp_depth must be in [2, 4]");
  if (c->n_blocks < 1 || c->n_blocks > kMaxBlocks) return fail(ECNF_E_UNSUPPORTED, "n_blocks must be in [1, 10]");
  if (!(c->base_scale > 0.f)) return fail(ECNF_E_INVALID, "base_scale must be > 0");
  return ECNF_OK;
}

size_t param_count(const ecnf_cfg& c) {
  const size_t H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width, L = c.mlp_depth, K = c.n_blocks;
  size_t per_block = 2 * (1 + M);                                 // Dense_0, Dense_1
  per_block += (2 * H + 1) * M + M + (L - 1) * (M * M + M);      // phi_e
  per_block += (M + H) * M + M + (L - 1) * (M * M + M) + M * H + H;  // phi_h
  per_block += L * (M * M + M);                                   // phi_x_torso
  per_block += (H + T) * H + H;                                   // EGNN_0/Dense_k
  return K * per_block + 1 + (size_t)c.n_features * H;
}

}  // namespace

static_assert(sizeof(Net) <= 4096, "Net is passed by value as a kernel argument");

struct ecnf_handle {
  ecnf_cfg cfg;
  int device;
  float* dbuf;
  int prec;            // ecnf_precision of later calls
  Net net[4];          // [2 P + NT], at the LDS-optimal molecules per workgroup (choose_mpw)
  size_t lds[4];       // dynamic LDS bytes per workgroup [2 P + NT]
  int ncu;             // compute units of the device (batch-aware workgroup sizing, net_for_batch)
  int exact_form;      // ecnf_exact_form (A/B diagnostics; ECNF_EXACT_FORM_DEFAULT in the product)
  bool split_ok;       // the split-fp16 kernels can represent the weights (else the handle is strict fp32 only)
  // ecnf_reserve_workspace: the arena ecnf_integrate uses for the exact trace's primal-aggregate cache
  // (SolveP::pcache); never (re)allocated inside a solve call.  Calls on different streams are ordered by arena_ev.
  float* arena;
  size_t arena_bytes;
  std::mutex arena_mu;
  hipEvent_t arena_ev;
  bool arena_used;
  hipStream_t arena_stream;
  // team (latency) mode of the primal kernels (egnn_eval.hpp team_exchange): exchange slots and the per-molecule
  // arrival counters / timeout flags for up to team_cap molecules of team_gcap workgroups, allocated at create only
  // for shapes with a team kernel (team_shape) whose weights the split kernels represent; shared by every
  // ecnf_integrate on the handle (ordered across streams by team_ev under team_mu)
  std::atomic<int> team_mode;   // ecnf_set_team: 0 auto, 1 off, G >= 2 forced; read once per solve (team_size)
  int team_cap, team_gcap, team_slot;
  // atomic: team_size reads it without team_mu while ecnf_update_params may publish new buffers under it (team_sync
  // is only read with team_mu held: the G > 1 dispatch in integrate_impl)
  std::atomic<float*> team_buf{nullptr};
  unsigned* team_sync;  // [team_cap] counters, then [team_cap] timeout flags (one 16-B-padded block, zeroed per launch)
  std::mutex team_mu;
  hipEvent_t team_ev;
  bool team_used;
  hipStream_t team_stream;
};

namespace {

struct Packer {
  std::vector<float> buf;
  size_t put(const float* src, size_t n) {
    size_t off = (buf.size() + 15) & ~size_t(15);   // 64-byte alignment
    buf.resize(off + n, 0.f);
    if (src) std::memcpy(buf.data() + off, src, n * sizeof(float));
    return off;
  }
};

// the power-of-two scale s of a split weight matrix (chain_split.hpp): max |w s| in [2^12, 2^13) for fp16 pieces
static float split_scale(const float* W, size_t n, size_t ld = 0, size_t cols = 0) {
  float mx = 0.f;
  for (size_t i = 0; i < n; ++i) {
    const float a = std::fabs(ld ? W[(i / cols) * ld + (i % cols)] : W[i]);
    if (a > mx) mx = a;
  }
  if (!(mx > 0.f) || !std::isfinite(mx)) return 1.0f;
  const int e = std::max(-100, std::min(100, 12 - std::ilogb(mx)));
  return std::ldexp(1.0f, e);
}

// w s = piece0 + ... by successive RNE; stores 16-bit element j of a lane's 8-element fragment, pieces
// piece_stride u32 apart
static inline void put_split(uint32_t* frag_p0, size_t piece_stride, int j, float w, float scale) {
  uint16_t piece[kPieces];
  const float ws = w * scale;   // exact (power of two, no overflow by construction)
  const _Float16 h0 = (_Float16)ws;
  const _Float16 h1 = (_Float16)(ws - (float)h0);
  std::memcpy(&piece[0], &h0, 2);
  std::memcpy(&piece[1], &h1, 2);
  for (int p = 0; p < kPieces; ++p) {
    uint32_t& word = frag_p0[p * piece_stride + (j >> 1)];
    word = (j & 1) ? ((word & 0x0000ffffu) | ((uint32_t)piece[p] << 16)) : ((word & 0xffff0000u) | piece[p]);
  }
}

// split fragments of a node GEMM W [K][NOUT] (row-major, node_task_split): [out block b][k-step s][piece]
// [lane l][8 x 16 bit], element j = W[16 s + 8 (l >> 5) + j][32 b + (l & 31)], zero for k >= K
static void pack_split_node(const float* W, int K, int NOUT, float scale, uint32_t* dst) {
  const int nks = (K + 15) / 16;
  for (int b = 0; b < NOUT / 32; ++b)
    for (int ks = 0; ks < nks; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * ks + 8 * (l >> 5) + j;
          const float w = k < K ? W[(size_t)k * NOUT + 32 * b + (l & 31)] : 0.f;
          put_split(dst + (((size_t)b * nks + ks) * kPieces * 64 + l) * 4, 64 * 4, j, w, scale);
        }
}

// split fragments of one [M][M] chain layer (chain_split.hpp): group g = (jb * NF + fb) * 2 + u, piece p,
// lane l = (c, h), element j = W[32 fb + f(8u + j, h)][32 jb + c], f(r, h) = (r & 3) + 8 (r >> 2) + 4 h
static void pack_split_layer(const float* W, int M, float scale, uint32_t* dst) {
  const int NF = M / 32;
  for (int jb = 0; jb < NF; ++jb)
    for (int fb = 0; fb < NF; ++fb)
      for (int u = 0; u < 2; ++u) {
        const int g = (jb * NF + fb) * 2 + u;
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int r = 8 * u + j, h = l >> 5;
            const int in = 32 * fb + (r & 3) + 8 * (r >> 2) + 4 * h, out = 32 * jb + (l & 31);
            put_split(dst + ((size_t)g * kPieces * 64 + l) * 4, 64 * 4, j, W[(size_t)in * M + out], scale);
          }
      }
}

// the divergence kernels' exact chain weights (chain_split WP = 3): w s = h0 + h1 + h2 in fp16 pieces, exact for every
// weight within 2^-5 of the layer's largest (the differences are exact in fp32; below that h2 is an fp16 subnormal,
// |error| <= 2^-25 in scaled units, i.e. <= 2^-37 of the largest weight).  Layout as pack_split_layer with 3 pieces:
// [group][piece][lane][4 u32]
static void pack_split_layer3(const float* W, int M, float scale, uint32_t* dst) {
  const int NF = M / 32;
  for (int jb = 0; jb < NF; ++jb)
    for (int fb = 0; fb < NF; ++fb)
      for (int u = 0; u < 2; ++u) {
        const int g = (jb * NF + fb) * 2 + u;
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int r = 8 * u + j, h = l >> 5;
            const int in = 32 * fb + (r & 3) + 8 * (r >> 2) + 4 * h, out = 32 * jb + (l & 31);
            const float ws = W[(size_t)in * M + out] * scale;
            const _Float16 h0 = (_Float16)ws;
            const float r1 = ws - (float)h0;
            const _Float16 h1 = (_Float16)r1;
            const _Float16 h2 = (_Float16)(r1 - (float)h1);
            const _Float16 hp[3] = {h0, h1, h2};
            for (int p = 0; p < 3; ++p) {
              uint16_t bits;
              std::memcpy(&bits, &hp[p], 2);
              uint32_t& word = dst[(((size_t)g * 3 + p) * 64 + l) * 4 + (j >> 1)];
              word = (j & 1) ? ((word & 0x0000ffffu) | ((uint32_t)bits << 16)) : ((word & 0xffff0000u) | bits);
            }
          }
      }
}

struct HostBlock {
  const float *xb, *xk, *gb, *gk;
  const float *eb[4], *ek[4];
  const float *hb[5], *hk[5];
  const float *tb[4], *tk[4];
  const float *nb, *nk;
};

// team mode (team_size): molecules per launch, and the bytes of the counter / timeout block (16-B multiple)
constexpr int kTeamCap = 64;      // molecules with team buffers (forced team mode, the re-dealt solve's tail teams)
constexpr int kTeamAutoMax = 32;  // auto team mode up to this batch (include/ecnf.h ecnf_set_team)
constexpr size_t kTeamSyncBytes = 2 * kTeamCap * sizeof(unsigned);

// waves per workgroup of the primal kernels (Geo<NF, 0, P>::NW)
int primal_waves(const ecnf_cfg& c) { return c.mlp_width <= 128 ? 8 : 4; }

// Geo<NF, NT, P>::kSplit: the split primal kernels (16-B node-row strides, stored segment parts)
bool split_primal(const ecnf_cfg& c, int NT, int P) {
  return kSplitChain && P == 0 && !NT && c.mlp_width <= 32 * kSplitMaxNF;
}

// Geo<NF, 1, P, BN>::kWideT / kWideT32: the tangent kernels in the wide form at either precision (per-edge phi_e.0,
// no P rows in LDS, in-place phi_h): every M = 256 tangent kernel, and the M = 128 ones (Geo BN, Net::wide) for
// molecules of 34 .. 64 atoms, whose primal + tangent P rows do not fit the LDS
bool wide_tangent(const ecnf_cfg& c, int NT, int P) {
  (void)P;
  return NT && (c.mlp_width == 256 || (c.mlp_width == 128 && c.n_nodes > 33));
}

// Geo<NF, NT, P>::kSplitN: split node GEMMs, i.e. 16-B node-row strides (split primal kernels and, with
// kSplitTanNode, the split tangent kernels)
bool vec_layout(const ecnf_cfg& c, int NT, int P) {
  return split_primal(c, NT, P) || (kSplitTanNode && kSplitTanChain && P == 0 && NT && c.mlp_width <= 128) ||
         (P == 0 && wide_tangent(c, NT, P));
}

// dynamic LDS bytes of one workgroup holding m molecules (RP padded node rows)
size_t lds_bytes(const ecnf_cfg& c, int NT, int P, int m, int RP) {
  const int N = c.n_nodes, D = c.dim, H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width;
  const bool vec = vec_layout(c, NT, P), wide = wide_tangent(c, NT, P);
  const int floats = (NT ? lds_eval_floats<1>(N, D, H, T, M, c.mlp_depth, m, RP, vec, wide)
                         : lds_eval_floats<0>(N, D, H, T, M, c.mlp_depth, m, RP, vec)) +
                     solver_lds_floats(m, N * D);
  return (size_t)floats * 4;
}

// the Net fields that depend on the molecules per workgroup: MPW, RP, and the split primal kernels' stored
// segment parts (cross rows overlaying hin; the receiver segments a tile boundary splits)
void set_mpw(Net& n, const ecnf_cfg& c, int NT, int P, int mpw, int rp) {
  const int M = c.mlp_width, H = c.hidden, T = c.time_embedding_dim;
  n.MPW = mpw;
  n.RP = rp;
  n.wide = wide_tangent(c, NT, P) && M == 128 ? 1 : 0;
  const bool vec = split_primal(c, NT, P);
  n.cross = vec && n.SR == c.n_nodes - 1 &&
            (size_t)mpw * (n.EP / 32) * ld_node(M, 1, true) <= (size_t)rp * ld_node(H + T, 1, true) &&
            n.EP / 32 <= kMaxTilesPerMol;
  n.ncross = 0;
  const int nn1 = c.n_nodes - 1;
  for (int t = 1; n.cross && t < n.EP / 32; ++t)
    if (32 * t < n.E && (32 * t) % nn1 != 0) {
      n.xs_i[n.ncross] = (unsigned char)((32 * t) / nn1);
      n.xs_t[n.ncross] = (unsigned char)t;
      ++n.ncross;
    }
}

// static LDS of the integrate kernels beside the dynamic carve-up (ecnf_kernels.hpp solver_sizes), reserved when a
// configuration is sized against the CU's 160 KiB
constexpr size_t kStaticLdsBytes = 64;

int choose_mpw(const ecnf_cfg& c, int NT, int P, int* mpw_out, size_t* lds_out, int* rp_out) {
  const int N = c.n_nodes, D = c.dim, H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width;
  const int E = N * (N - 1), SR = edge_slots_per_receiver(N);
  double best = -1;
  int best_m = 0;
  size_t best_lds = 0;
  int best_rp = 0;
  for (int m = 1; m <= 32; ++m) {
    const int RP = 32 * ((m * N + 31) / 32);
    const bool vec = vec_layout(c, NT, P), wide = wide_tangent(c, NT, P);
    // in-place phi_h (node_gemm_inplace): one (output block pair, 32-row tile) task per wave of the 4-wave kernels
    if (wide && (M / 64) * (RP / 32) > 4) break;
    const int floats = (NT ? lds_eval_floats<1>(N, D, H, T, M, c.mlp_depth, m, RP, vec, wide)
                           : lds_eval_floats<0>(N, D, H, T, M, c.mlp_depth, m, RP, vec)) +
                       solver_lds_floats(m, N * D);
    const size_t bytes = (size_t)floats * 4;
    if (bytes + kStaticLdsBytes > 160 * 1024) break;
    const int EP = 32 * ((N * SR + 31) / 32);
    const int tiles = m * EP / 32;
    const double eff = (double)tiles / (kSimds * ((tiles + kSimds - 1) / kSimds)) * (double)(m * E) / (tiles * 32.0);
    if (eff > best + 1e-9) {
      best = eff;
      best_m = m;
      best_lds = bytes;
      best_rp = RP;
    }
  }
  if (!best_m) return fail(ECNF_E_UNSUPPORTED, "configuration does not fit the 160 KiB LDS of one CU");
  *mpw_out = best_m;
  *lds_out = best_lds;
  *rp_out = best_rp;
  return ECNF_OK;
}

// a kernel is compiled for (cfg, NT, P); P < 0: either precision
bool shape_supported(const ecnf_cfg& c, int NT, int P = -1) {
  (void)NT;   // every compiled shape has tangent kernels at both precisions
  (void)P;
  const int M = c.mlp_width, L = c.mlp_depth, D = c.dim;
#define X(m, l, d) \
  if (M == m && L == l && D == d) return true;
  ECNF_SHAPES(X)
#undef X
#define X(m, l, d) \
  if (M == m && L == l && D == d) return true;
  ECNF_SHAPES_WIDE_TAN(X)
#undef X
  return false;
}


// Batch-aware workgroup sizing: the handle's MPW maximises the tile balance of one workgroup, but a batch that
// fills fewer workgroups than the device has CUs (ALDP B = 512 at MPW = 4: 128 workgroups on 256 CUs) leaves CUs
// idle.  Pick m <= MPW minimising (workgroup rounds) x (per-workgroup time), with the time of one workgroup taken as
// its edge tiles per SIMD plus ~0.6 tile-equivalents of node-GEMM work per 32 node rows (LJ13 stamps: node phases ~
// 18 % beside 5 tiles per SIMD at 2 row tiles); ties keep the larger m.  A molecule's arithmetic does not depend
// on m (every molecule owns its edge tiles and node rows), so results are bitwise independent of the choice.
// Adaptive solves: a workgroup runs until its slowest molecule is done, and workgroups of unequal length balance
// over the CUs as they retire, so the model charges (workgroups / CUs) continuous rounds, plus a per-workgroup
// penalty per extra molecule for the expected max of m step counts (0: measured on ALDP B = 512 PID, penalty
// 0 / 0.15 / 0.3 -> sample 3.23 / 3.73 / 3.70 ms, Hutchinson log_prob 57.9 / 58.0 / 58.1 ms,
// profiles/round2/mpw_ab.log).
// (Round 5: the M = 64 tangent kernels run one molecule per workgroup anyway (MPW = 1, LDS); their tail is the
// dispatch order of the workgroups beyond the CU count, which the re-dealt solve addresses, redeal_kernel.)
constexpr double adaptive_penalty() { return 0.0; }

Net net_for_batch(const ecnf_handle* h, int ix, int B, size_t* lds, bool adaptive = false) {
  Net n = h->net[ix];
  *lds = h->lds[ix];
  const int mpw_max = n.MPW;
  if (mpw_max <= 1 || B <= 0) return n;
  const ecnf_cfg& c = h->cfg;
  const int NT = ix & 1, P = ix >> 1;
  const int tiles_mol = n.EP / 32;
  double best = 1e300;
  int best_m = mpw_max;
  for (int m = mpw_max; m >= 1; --m) {
    const int RP = 32 * ((m * c.n_nodes + 31) / 32);
    const long wgs = (B + m - 1) / m;
    const double rounds = adaptive ? std::max(1.0, (double)wgs / h->ncu) : (double)((wgs + h->ncu - 1) / h->ncu);
    const double t_wg = ((double)((m * tiles_mol + kSimds - 1) / kSimds) + 0.6 * (RP / 32)) *
                        (adaptive ? 1.0 + adaptive_penalty() * (m - 1) : 1.0);
    const double cost = rounds * t_wg;
    if (cost < best - 1e-9) {
      best = cost;
      best_m = m;
    }
  }
  if (best_m != mpw_max) {
    const int RP = 32 * ((best_m * c.n_nodes + 31) / 32);
    set_mpw(n, c, NT, P, best_m, RP);
    *lds = lds_bytes(c, NT, P, best_m, RP);
    n.lds_floats = (int)(*lds / 4);
  }
  return n;
}

// Team (latency) mode: G workgroups per molecule (egnn_eval.hpp team_exchange) for the primal kernels when the batch
// leaves most CUs idle.  Auto: one edge-tile round per block (G = ceil(tiles per molecule / waves)) where a round is
// long against the ~5 us exchange (M = 256: QM9's 36-60 us rounds), B G <= CUs (one member per CU is always
// co-resident) and B <= team_cap.  ecnf_set_team forces G (>= 2) or turns it off (1).
// floats of the column-split mode's LDS layer image (egnn_eval.hpp edge_tile_cols: NF blocks x 2 k-steps x 2 pieces
// x 64 lanes x 16 B, the same bytes as the fp32 image NF x 4 x 64 x 16 B)
int cols_image_floats(const ecnf_cfg& c) { return (c.mlp_width / 32) * 2 * 2 * 64 * 4; }

// Column-split team mode (egnn_eval.hpp edge_tile_cols, M = 256 split primal kernels): G = tiles per molecule, each
// member runs one tile with its 4 waves split by output block.  Auto mode prefers it when B G <= CUs and the layer
// image fits the LDS beside the MPW = 1 carve-up.
bool cols_fits(const ecnf_handle* h, int NT, int B) {
  const ecnf_cfg& c = h->cfg;
  if (NT != 0 || h->prec != 0 || !cols_shape(c.mlp_width, NT, c.mlp_depth, c.dim, 0)) return false;
  const int tpm = h->net[0].EP / 32, RP = 32 * ((c.n_nodes + 31) / 32);
  if (tpm > h->team_gcap || (long)B * tpm > h->ncu) return false;
  return lds_bytes(c, 0, 0, 1, RP) + (size_t)cols_image_floats(c) * 4 + kStaticLdsBytes <= 160 * 1024;
}

// mode: the handle's team_mode, read ONCE by the caller (a concurrent ecnf_set_team cannot split one solve's decision).
// Tangent solves run in team mode only when forced (mode >= 2), for the Hutchinson divergence (the exact trace's
// sparse blocks are not exchanged) on the tangent team shape (team_shape: ALDP's M = 64 kernel, one molecule per
// workgroup); the re-dealt adaptive log_prob teams its tail on its own (team_tail).
int team_size(const ecnf_handle* h, int NT, int B, int* cols, int mode, int div = ECNF_DIV_HUTCHINSON) {
  const ecnf_cfg& c = h->cfg;
  if (cols) *cols = 0;
  if (B < 1 || B > (mode >= 2 ? h->team_cap : kTeamAutoMax) || mode == 1 || !h->team_buf.load() ||
      !team_shape(c.mlp_width, NT, c.mlp_depth, c.dim, h->prec))
    return 1;
  if (NT && (mode < 2 || div != ECNF_DIV_HUTCHINSON)) return 1;
  const int tpm = h->net[0].EP / 32;
  int G;
  if (mode >= 2) {
    G = std::min(std::min(mode, h->team_gcap), tpm);
  } else {
    if (h->cfg.mlp_width < 256) return 1;
    if (cols_fits(h, NT, B)) {
      if (cols) *cols = 1;
      return tpm;
    }
    G = std::min((tpm + primal_waves(h->cfg) - 1) / primal_waves(h->cfg), h->team_gcap);
  }
  if (G < 2 || (long)B * G > h->ncu) return 1;
  return G;
}

// Does a re-dealt solve on this handle run its longest slots as tail teams (redeal_kernel, kTailG)?  Hutchinson solves
// of a shape with a tangent team kernel (team_shape), one molecule per workgroup, split precision, team buffers present.
bool tail_teams(const ecnf_handle* h, int NT, int div, int mpw) {
  const ecnf_cfg& c = h->cfg;
  return NT == 1 && div == ECNF_DIV_HUTCHINSON && mpw == 1 && h->prec == 0 && h->team_buf.load() &&
         h->team_mode.load() != 1 && kTailG <= h->team_gcap && kStopG <= h->team_gcap &&
         team_shape(c.mlp_width, 1, c.mlp_depth, c.dim, 0);
}

// G, cols: team_size's decision for this solve (G = 1: the batch path)
hipError_t dispatch_integrate(const ecnf_handle* h, int NT, const SolveP& sp_in, int G, int cols, const float* y0,
                              const int32_t* feat, const float* eps, float* y1, float* dlogp, int32_t* nfe,
                              int32_t* status, int B, hipStream_t stream, float* sched = nullptr) {
  const int M = h->cfg.mlp_width, L = h->cfg.mlp_depth, D = h->cfg.dim, P = h->prec, ix = 2 * P + NT;
  size_t lds = 0;
  SolveP sp = sp_in;
  Net net;
  if (G > 1) {
    net = h->net[ix];
    const int RP = 32 * ((h->cfg.n_nodes + 31) / 32);
    set_mpw(net, h->cfg, NT, P, 1, RP);
    lds = lds_bytes(h->cfg, NT, P, 1, RP);
    if (cols) {   // the layer image sits before the solver state (carve_lds)
      net.xs_floats = cols_image_floats(h->cfg);
      lds += (size_t)net.xs_floats * 4;
    }
    net.lds_floats = (int)(lds / 4);
    sp.team.G = G;
    sp.team.cols = cols;
    sp.team.nteam = nullptr;
    sp.team.slot = h->team_slot;
    sp.team.buf = h->team_buf.load();
    sp.team.ctr = h->team_sync;
    sp.team.timeout = reinterpret_cast<int*>(h->team_sync + kTeamCap);
    hipError_t e = hipMemsetAsync(h->team_sync, 0, kTeamSyncBytes, stream);
    if (e != hipSuccess) return e;
  } else {
    sp.team = TeamP{};
    net = net_for_batch(h, ix, B, &lds, sp.adaptive != 0);
  }
  auto launch = [&](const SolveP& spl) -> hipError_t {
#define ECNF_CALL(m, l, d, nt, p) \
  launch_integrate<m / 32, nt, l, d, p>(net, lds, spl, y0, feat, eps, y1, dlogp, nfe, status, B, stream)
#define X(m, l, d)                                                                                           \
  if (M == m && L == l && D == d)                                                                            \
    return NT ? (P ? ECNF_CALL(m, l, d, 1, 1) : ECNF_CALL(m, l, d, 1, 0)) : (P ? ECNF_CALL(m, l, d, 0, 1) : ECNF_CALL(m, l, d, 0, 0));
  ECNF_SHAPES(X)
#undef X
#define X(m, l, d)                                                                                            \
  if (M == m && L == l && D == d)                                                                             \
    return NT ? (P ? ECNF_CALL(m, l, d, 1, 1) : ECNF_CALL(m, l, d, 1, 0)) : (P ? ECNF_CALL(m, l, d, 0, 1) : ECNF_CALL(m, l, d, 0, 0));
  ECNF_SHAPES_WIDE_TAN(X)
#undef X
#undef ECNF_CALL
    return hipErrorInvalidValue;
  };
  const int grid = (B + net.MPW - 1) / net.MPW;
  if (!(sched && G == 1 && sp.adaptive && grid > h->ncu && chunkable(M / 32, NT, P))) return launch(sp);
  // chunked, re-dealt solve (sched_floats, redeal_kernel)
  const int ND = h->cfg.n_nodes * h->cfg.dim, stride = solver_state_stride(ND);
  int* order = reinterpret_cast<int*>(sched + (size_t)B * stride);
  int* nslots = order + align4(B);
  float* gkey = reinterpret_cast<float*>(nslots + 4);   // the sort's scratch beyond kRedealLds molecules
  int* gidx = reinterpret_cast<int*>(gkey + pow2_at_least(B));
  SolveP s1 = sp;
  s1.state = sched;
  s1.state_stride = stride;
  s1.chunk_steps = kChunkSteps;
  hipError_t e = launch(s1);
  if (e != hipSuccess) return e;
  // tail teams (kTailG workgroups for the longest slots) where the shape has a tangent team kernel and the batch runs
  // one molecule per workgroup; the caller holds team_mu (integrate_impl) and the team buffers are this solve's
  const bool tail = tail_teams(h, NT, sp.div, net.MPW);
#ifdef ECNF_TAIL_KMAX   // (experiment builds)
  const int kmax = tail ? ECNF_TAIL_KMAX : 0;
#else
  const int kmax = tail ? std::min(h->team_cap, h->ncu / (2 * kTailG)) : 0;
#endif
  int* nteam = tail ? nslots + 1 : nullptr;
  hipLaunchKernelGGL(redeal_kernel, dim3(1), dim3(kRedealThreads), 0, stream, sched, stride, ND, B, sp.tau1, order,
                     nslots, gkey, gidx, nteam, kmax, 0);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  SolveP s2 = sp;
  s2.state = sched;
  s2.state_stride = stride;
  s2.resume = 1;
  s2.order = order;
  s2.nslots = nslots;
  if (tail) {
    s2.team.G = kTailG;
    s2.team.cols = 0;
    s2.team.slot = h->team_slot;
    s2.team.buf = h->team_buf.load();
    s2.team.ctr = h->team_sync;
    s2.team.timeout = reinterpret_cast<int*>(h->team_sync + kTeamCap);
    s2.team.nteam = nteam;
    s2.team.nteam_max = kmax;
    // stop-and-team: the molecules still unfinished once at most kstop are left go on in a third launch, all of
    // them teams of kStopG
#ifdef ECNF_STOP_LEFT   // (experiment builds)
    const int kstop = ECNF_STOP_LEFT;
#else
    const int kstop = std::min(h->team_cap, h->ncu / kStopG);
#endif
    s2.team.fin = nslots + 2;
    s2.team.nsl = nslots;
    s2.team.stop_left = kstop;
    e = hipMemsetAsync(h->team_sync, 0, kTeamSyncBytes, stream);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(s2.team.fin, 0, sizeof(int), stream);
    if (e != hipSuccess) return e;
    e = launch(s2);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(redeal_kernel, dim3(1), dim3(kRedealThreads), 0, stream, sched, stride, ND, B, sp.tau1, order,
                       nslots, gkey, gidx, nteam, kstop, 1);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    SolveP s3 = s2;
    s3.team.G = kStopG;
    s3.team.nteam_max = kstop;
    s3.team.fin = nullptr;
    e = hipMemsetAsync(h->team_sync, 0, kTeamSyncBytes, stream);
    if (e != hipSuccess) return e;
    return launch(s3);
  }
  return launch(s2);
}

hipError_t dispatch_vf(const ecnf_handle* h, int NT, const float* x, const float* t, const int32_t* feat,
                       const float* tan_in, int ntan, float* v, float* tan_out, int B, hipStream_t stream) {
  const int M = h->cfg.mlp_width, L = h->cfg.mlp_depth, D = h->cfg.dim, P = h->prec, ix = 2 * P + NT;
  size_t lds = 0;
  const Net net = net_for_batch(h, ix, B, &lds);
#define ECNF_CALL(m, l, d, nt, p) \
  launch_vf<m / 32, nt, l, d, p>(net, lds, x, t, feat, tan_in, ntan, v, tan_out, B, stream)
#define X(m, l, d)                                                                                           \
  if (M == m && L == l && D == d)                                                                            \
    return NT ? (P ? ECNF_CALL(m, l, d, 1, 1) : ECNF_CALL(m, l, d, 1, 0)) : (P ? ECNF_CALL(m, l, d, 0, 1) : ECNF_CALL(m, l, d, 0, 0));
  ECNF_SHAPES(X)
#undef X
#define X(m, l, d)                                                                                            \
  if (M == m && L == l && D == d)                                                                             \
    return NT ? (P ? ECNF_CALL(m, l, d, 1, 1) : ECNF_CALL(m, l, d, 1, 0)) : (P ? ECNF_CALL(m, l, d, 0, 1) : ECNF_CALL(m, l, d, 0, 0));
  ECNF_SHAPES_WIDE_TAN(X)
#undef X
#undef ECNF_CALL
  return hipErrorInvalidValue;
}

// Does an exact-trace solve on this handle run the sparse blocks 1 and K (egnn_eval sparse_a)?  Only the kernels that
// compile them (egnn_eval kSparseX: the M <= 128 split tangent kernels except the L = 2 shapes (128, *, *) and
// (*, 2, 2)), and only where a molecule has >= 3 edge tiles per dual tile (LJ13: 5 vs 1, ALDP: 15 vs 2; not DW4).
bool exact_sparse(const ecnf_handle* h, int divergence) {
  const ecnf_cfg& c = h->cfg;
  if (divergence != ECNF_DIV_EXACT || h->prec != ECNF_PREC_SPLIT_F16 || c.mlp_width > 128) return false;
  if (edge_slots_per_receiver(c.n_nodes) != c.n_nodes - 1) return false;   // receiver-tiled (N > 33): all-dual form
  if (c.mlp_depth == 2 && (c.mlp_width == 128 || c.dim == 2)) return false;
  const int nn1 = c.n_nodes - 1, tpm = (c.n_nodes * nn1 + 31) / 32, ndt = (2 * nn1 + 31) / 32;
  return tpm >= 3 * ndt;
}

// why a handle has no tangent (divergence / JVP) kernel: the shape is not compiled for it at this precision, or its
// node rows (doubled by the tangent rows) do not fit the LDS of one CU (mlp_width 128 beyond 33 atoms, 256 beyond 32)
std::string no_tangent_msg(const ecnf_cfg& c, int prec) {
  const int P = prec == ECNF_PREC_FP32 ? 1 : 0;
  if (!shape_supported(c, 1, P))
    return "no tangent kernel for mlp_width=" + std::to_string(c.mlp_width) + ", mlp_depth=" + std::to_string(c.mlp_depth) +
           " at this precision";
  return "the tangent kernel's LDS does not fit one CU for n_nodes=" + std::to_string(c.n_nodes) +
         ", mlp_width=" + std::to_string(c.mlp_width);
}

// floats of one molecule slot of the primal-aggregate cache: block 1's message sums [N][M] and the shift sums of
// blocks 1 and K [2][N][D] (egnn_eval, pcache)
size_t pcache_stride(const ecnf_handle* h) {
  const ecnf_cfg& c = h->cfg;
  return (size_t)c.n_nodes * c.mlp_width + 2 * (size_t)c.n_nodes * c.dim;
}

// slots of a batch: the grid covers ceil(B / m) m <= B + MPW - 1 molecule slots (m <= MPW, net_for_batch)
size_t pcache_floats(const ecnf_handle* h, int batch) {
  return (size_t)(batch + h->net[2 * h->prec + 1].MPW) * pcache_stride(h);
}

// Chunked, re-dealt adaptive solves (redeal_kernel): the first launch runs every molecule for kChunkSteps step
// controls and stores its solver state; the second resumes the unfinished ones, longest estimated remainder first.
// Results are bitwise those of one launch (a molecule's arithmetic does not depend on its slot or workgroup, and the
// state crosses the launches exactly).  Taken when the grid has more workgroups than the device has CUs and the
// caller's workspace (or the handle's arena) holds the scratch below.
// floats of the re-deal scratch of a solve (0: never re-dealt): [B][solver_state_stride] states, the slot order and
// the slot count; it follows the exact trace's pcache in the workspace
size_t sched_floats(const ecnf_handle* h, const ecnf_solve_opts* o, int batch) {
  if (o->solver != ECNF_SOLVER_DOPRI5 || o->dt0 > 0.f || batch < 2 || batch > kRedealMax) return 0;
  const int ND = h->cfg.n_nodes * h->cfg.dim, n2 = pow2_at_least(batch);
  return (size_t)batch * solver_state_stride(ND) + align4(batch) + 4 + (n2 > kRedealLds ? 2 * (size_t)n2 : 0);
}

int integrate_impl(ecnf_handle* h, const ecnf_solve_opts* o, const float* y0, const int32_t* feat, const float* eps,
                   float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch, float* ws, size_t ws_bytes,
                   hipStream_t stream, bool arena);

}  // namespace

// =====================================================================================================
// C-ABI
// =====================================================================================================
extern "C" {

int ecnf_abi_version(void) { return ECNF_ABI_VERSION; }

#ifdef ECNF_DEVICE_CHECKS
// device-checked diagnostic build only: OR of the failed-check bits of every kernel since the last reset
int ecnf_debug_checks(uint32_t* flags, int reset) {
  if (!flags) return fail(ECNF_E_INVALID, "NULL argument");
  HIP_TRY(hipDeviceSynchronize());
  unsigned w[64];
  HIP_TRY(hipMemcpyFromSymbol(w, HIP_SYMBOL(g_checks), sizeof(w)));
  unsigned acc = 0;
  for (unsigned v : w) acc |= v;
  *flags = acc;
  if (reset) {
    unsigned z[64] = {0};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_checks), z, sizeof(z)));
  }
  return ECNF_OK;
}
#endif

#ifdef ECNF_STAMPS
// diagnostic build only: copy (and optionally reset) the accumulated phase cycles
int ecnf_debug_stamps(unsigned long long* out, int n, int reset) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * std::min(n, 32)));
  if (reset) {
    unsigned long long z[32] = {0};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
  }
  return ECNF_OK;
}
#endif

const char* ecnf_last_error(void) { return g_err.c_str(); }

int ecnf_struct_layout(int32_t which, size_t* out, int32_t cap) {
#define L_(T, f) offsetof(T, f)
  size_t v[16];
  int n = 0;
  switch (which) {
    case 0: {
      const size_t o[] = {sizeof(ecnf_cfg), L_(ecnf_cfg, n_nodes), L_(ecnf_cfg, dim), L_(ecnf_cfg, n_features),
                          L_(ecnf_cfg, hidden), L_(ecnf_cfg, time_embedding_dim), L_(ecnf_cfg, mlp_width),
                          L_(ecnf_cfg, mlp_depth), L_(ecnf_cfg, n_blocks), L_(ecnf_cfg, base_scale),
                          L_(ecnf_cfg, normalization_constant)};
      n = sizeof(o) / sizeof(o[0]);
      std::memcpy(v, o, sizeof(o));
      break;
    }
    case 1: {
      const size_t o[] = {sizeof(ecnf_solve_opts), L_(ecnf_solve_opts, solver), L_(ecnf_solve_opts, divergence),
                          L_(ecnf_solve_opts, t0), L_(ecnf_solve_opts, t1), L_(ecnf_solve_opts, dt0),
                          L_(ecnf_solve_opts, rtol), L_(ecnf_solve_opts, atol), L_(ecnf_solve_opts, dtmin),
                          L_(ecnf_solve_opts, max_steps)};
      n = sizeof(o) / sizeof(o[0]);
      std::memcpy(v, o, sizeof(o));
      break;
    }
    case 2: {
      const size_t o[] = {sizeof(ecnf_target), L_(ecnf_target, kind), L_(ecnf_target, n_nodes), L_(ecnf_target, dim),
                          L_(ecnf_target, epsilon), L_(ecnf_target, tau), L_(ecnf_target, r),
                          L_(ecnf_target, harmonic_coef), L_(ecnf_target, a), L_(ecnf_target, b), L_(ecnf_target, c),
                          L_(ecnf_target, d0), L_(ecnf_target, r_nodes)};
      n = sizeof(o) / sizeof(o[0]);
      std::memcpy(v, o, sizeof(o));
      break;
    }
    case 3: {
      const size_t o[] = {sizeof(ecnf_adam_opts), L_(ecnf_adam_opts, lr), L_(ecnf_adam_opts, b1),
                          L_(ecnf_adam_opts, b2), L_(ecnf_adam_opts, eps), L_(ecnf_adam_opts, eps_root),
                          L_(ecnf_adam_opts, count), L_(ecnf_adam_opts, ema_beta)};
      n = sizeof(o) / sizeof(o[0]);
      std::memcpy(v, o, sizeof(o));
      break;
    }
    default:
      return -1;
  }
#undef L_
  for (int i = 0; i < n && i < cap; ++i)
    if (out) out[i] = v[i];
  return n - 1;
}

int ecnf_param_count(const ecnf_cfg* cfg, size_t* n_floats) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!n_floats) return fail(ECNF_E_INVALID, "n_floats is NULL");
  *n_floats = param_count(*cfg);
  g_err.clear();
  return ECNF_OK;
}

int ecnf_create(const ecnf_cfg* cfg, const float* params, size_t n_floats, int device, ecnf_handle** out) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!params || !out) return fail(ECNF_E_INVALID, "params/out is NULL");
  const ecnf_cfg c = *cfg;
  if (n_floats != param_count(c))
    return fail(ECNF_E_INVALID, "params blob has " + std::to_string(n_floats) + " floats, expected " +
                                    std::to_string(param_count(c)));
  if (!shape_supported(c, 0))
    return fail(ECNF_E_UNSUPPORTED, "no kernel compiled for mlp_width=" + std::to_string(c.mlp_width) +
                                        " mlp_depth=" + std::to_string(c.mlp_depth) + " dim=" + std::to_string(c.dim));
  const int H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width, L = c.mlp_depth, K = c.n_blocks;
  const int NF = M / 32;

  // ---- walk the ravel_pytree-ordered blob ----
  std::vector<HostBlock> hb(K);
  const float* p = params;
  auto take = [&](size_t n) {
    const float* q = p;
    p += n;
    return q;
  };
  for (int k = 0; k < K; ++k) {   // EGNN_0/{k} in sorted order (K <= 10 so lexicographic == numeric)
    HostBlock& b = hb[k];
    b.xb = take(1); b.xk = take(M);
    b.gb = take(1); b.gk = take(M);
    for (int l = 0; l < L; ++l) { b.eb[l] = take(M); b.ek[l] = take((size_t)(l == 0 ? 2 * H + 1 : M) * M); }
    for (int l = 0; l <= L; ++l) {
      const int out_f = l == L ? H : M, in_f = l == 0 ? M + H : M;
      b.hb[l] = take(out_f); b.hk[l] = take((size_t)in_f * out_f);
    }
    for (int l = 0; l < L; ++l) { b.tb[l] = take(M); b.tk[l] = take((size_t)M * M); }
  }
  for (int k = 0; k < K; ++k) { hb[k].nb = take(H); hb[k].nk = take((size_t)(H + T) * H); }
  const float fs = *take(1);
  const float* emb = take((size_t)c.n_features * H);
  if ((size_t)(p - params) != n_floats) return fail(ECNF_E_INVALID, "internal: param walk size mismatch");

  // ---- repack ----
  Packer pk;
  bool split_ok = true;   // every edge-chain weight fits the unscaled fp16 split (|w| < 2^15)
  struct Off {
    size_t Wn, bn, Wp, bp, wd, We, Ws, be, wx, wg, Wh[kMaxPhiH], bh[kMaxPhiH], Wn_s, Wp_s, Wh_s[kMaxPhiH];
    size_t bp_u, wd_u, be_u, wg_u, wx_u, Wh_sn0, W1_s, Ws3;
    float bx, bg, hinv_n0, w1inv;
    float cinv[2 * 4 - 1], ninv, pinv, hinv[kMaxPhiH];
  };
  // packs W [K][NOUT] as split node fragments; returns the offset, *inv = 1 / its scale
  auto put_split_node = [&](const float* W, int K, int NOUT, float* inv) {
    std::vector<uint32_t> v((size_t)(NOUT / 32) * ((K + 15) / 16) * kPieces * 64 * 4, 0u);
    const float sc = split_scale(W, (size_t)K * NOUT);
    *inv = 1.0f / sc;
    pack_split_node(W, K, NOUT, sc, v.data());
    return pk.put(reinterpret_cast<const float*>(v.data()), v.size());
  };
  std::vector<Off> off(K);
  for (int k = 0; k < K; ++k) {
    const HostBlock& b = hb[k];
    Off& o = off[k];
    o.Wn = pk.put(b.nk, (size_t)(H + T) * H);
    o.bn = pk.put(b.nb, H);
    std::vector<float> wp((size_t)H * 2 * M), bp(2 * M, 0.f), wd(M);
    for (int r = 0; r < H; ++r)
      for (int j = 0; j < M; ++j) {
        wp[(size_t)r * 2 * M + j] = b.ek[0][(size_t)r * M + j];             // sender rows 0..H-1
        wp[(size_t)r * 2 * M + M + j] = b.ek[0][(size_t)(H + r) * M + j];   // receiver rows H..2H-1
      }
    for (int j = 0; j < M; ++j) { bp[M + j] = b.eb[0][j]; wd[j] = b.ek[0][(size_t)2 * H * M + j]; }
    o.Wp = pk.put(wp.data(), wp.size());
    o.Wn_s = put_split_node(b.nk, H + T, H, &o.ninv);
    // log2-domain copies for the split kernels (chain_split.hpp, silu_u)
    constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.69314718055994531f;
    auto scaled = [](const float* v, size_t n, float f) {
      std::vector<float> r(v, v + n);
      for (auto& x : r) x *= f;
      return r;
    };
    const std::vector<float> wp_u = scaled(wp.data(), wp.size(), kNegLog2e);
    o.Wp_s = put_split_node(wp_u.data(), H, 2 * M, &o.pinv);
    // the M = 256 tangent kernels' per-edge phi_e.0: [h_s | h_r | |r|^2] rows 0 .. 2H of the kernel, x -log2(e)
    o.W1_s = put_split_node(scaled(b.ek[0], (size_t)(2 * H + 1) * M, kNegLog2e).data(), 2 * H + 1, M, &o.w1inv);
    o.bp_u = pk.put(scaled(bp.data(), bp.size(), kNegLog2e).data(), bp.size());
    o.wd_u = pk.put(scaled(wd.data(), wd.size(), kNegLog2e).data(), wd.size());
    o.bp = pk.put(bp.data(), bp.size());
    o.wd = pk.put(wd.data(), wd.size());
    // chain: phi_e.1..L-1, phi_x.0..L-1, each [M][M] -> fragment order
    const int nchain = 2 * L - 1;
    std::vector<float> we((size_t)nchain * M * M), be((size_t)nchain * M);
    for (int cl = 0; cl < nchain; ++cl) {
      const float* W = cl < L - 1 ? b.ek[cl + 1] : b.tk[cl - (L - 1)];
      const float* bb = cl < L - 1 ? b.eb[cl + 1] : b.tb[cl - (L - 1)];
      float* dst = we.data() + (size_t)cl * M * M;
      for (int jb = 0; jb < NF; ++jb)
        for (int fb = 0; fb < NF; ++fb)
          for (int q = 0; q < 4; ++q)
            for (int l = 0; l < 64; ++l)
              for (int e = 0; e < 4; ++e) {
                const int krow = fb * 32 + e + 8 * q + 4 * (l >> 5);
                const int col = jb * 32 + (l & 31);
                dst[((((size_t)jb * NF + fb) * 4 + q) * 64 + l) * 4 + e] = W[(size_t)krow * M + col];
              }
      std::memcpy(be.data() + (size_t)cl * M, bb, M * sizeof(float));
    }
    o.We = pk.put(we.data(), we.size());
    // the same chain as split fragments: [layer][2 NF^2 groups][kPieces][64 lanes][4 u32]
    const size_t split_layer = (size_t)2 * NF * NF * kGroupU32;
    std::vector<uint32_t> ws((size_t)nchain * split_layer, 0u);
    for (int cl = 0; cl < 2 * 4 - 1; ++cl) o.cinv[cl] = 1.0f;
    for (int cl = 0; cl < nchain; ++cl) {
      const float* W = cl < L - 1 ? b.ek[cl + 1] : b.tk[cl - (L - 1)];
      // unscaled pieces: the chain adds the bias through the accumulator (chain_split.hpp); fp16 piece 0 must not
      // overflow: such a network runs on the strict-fp32 kernels only (split_ok = false, see below)
      float mx = 0.f;
      for (size_t i = 0; i < (size_t)M * M; ++i) mx = std::max(mx, std::fabs(W[i]));
      if (!(mx < 32768.f)) split_ok = false;
      o.cinv[cl] = 1.0f / split_scale(W, (size_t)M * M);   // the 3-piece chain's scale (Ws3); the 2-piece set is unscaled
      pack_split_layer(W, M, 1.0f, ws.data() + cl * split_layer);
    }
    o.Ws = pk.put(reinterpret_cast<const float*>(ws.data()), ws.size());
    {   // the divergence kernels' exact 3-piece chain (scaled per layer)
      const size_t layer3 = (size_t)2 * NF * NF * 3 * 256;
      std::vector<uint32_t> ws3((size_t)nchain * layer3, 0u);
      for (int cl = 0; cl < nchain; ++cl) {
        const float* W = cl < L - 1 ? b.ek[cl + 1] : b.tk[cl - (L - 1)];
        pack_split_layer3(W, M, 1.0f / o.cinv[cl], ws3.data() + cl * layer3);
      }
      o.Ws3 = pk.put(reinterpret_cast<const float*>(ws3.data()), ws3.size());
    }
    o.be = pk.put(be.data(), be.size());
    o.be_u = pk.put(scaled(be.data(), be.size(), kNegLog2e).data(), be.size());
    o.wx = pk.put(b.xk, M);
    o.wg = pk.put(b.gk, M);
    o.wx_u = pk.put(scaled(b.xk, M, kNegLn2).data(), M);
    o.wg_u = pk.put(scaled(b.gk, M, kNegLn2).data(), M);
    o.bx = *b.xb;
    o.bg = *b.gb;
    for (int l = 0; l <= L; ++l) {
      const int out_f = l == L ? H : M, in_f = l == 0 ? M + H : M;
      o.Wh[l] = pk.put(b.hk[l], (size_t)in_f * out_f);
      if (l == 0) {
        // the split kernels' aggregated messages arrive unscaled and in the log2 domain: fold -ln2 / sqrt(N-1)
        // (egnn.py:104) into the message rows 0..M-1 of phi_h.0 (the node update then only combines segment parts)
        std::vector<float> w0(b.hk[0], b.hk[0] + (size_t)in_f * out_f);
        const float f = kNegLn2 / std::sqrt((float)(c.n_nodes - 1));
        for (size_t i = 0; i < (size_t)M * out_f; ++i) w0[i] *= f;
        o.Wh_s[l] = put_split_node(w0.data(), in_f, out_f, &o.hinv[l]);
        o.Wh_sn0 = put_split_node(b.hk[0], in_f, out_f, &o.hinv_n0);   // natural domain (tangent kernels)
      } else {
        o.Wh_s[l] = put_split_node(b.hk[l], in_f, out_f, &o.hinv[l]);
      }
      o.bh[l] = pk.put(b.hb[l], out_f);
    }
  }
  const size_t off_emb = pk.put(emb, (size_t)c.n_features * H);

  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(ECNF_E_INVALID, "device index out of range");
  HIP_TRY(hipSetDevice(device));
  float* dbuf = nullptr;
  HIP_TRY(hipMalloc(&dbuf, pk.buf.size() * sizeof(float)));
  HIP_TRY(hipMemcpy(dbuf, pk.buf.data(), pk.buf.size() * sizeof(float), hipMemcpyHostToDevice));

  ecnf_handle* h = new ecnf_handle();
  h->cfg = c;
  h->device = device;
  h->dbuf = dbuf;
  // a network the split kernels cannot represent runs on the strict-fp32 kernels (ecnf_get_precision reports it)
  h->split_ok = split_ok;
  h->prec = split_ok ? ECNF_PREC_SPLIT_F16 : ECNF_PREC_FP32;
  {
    hipDeviceProp_t prop;
    h->ncu = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  for (int ix = 0; ix < 4; ++ix) {
    const int NT = ix & 1, P = ix >> 1;
    Net& n = h->net[ix];
    std::memset(&n, 0, sizeof(Net));
    n.N = c.n_nodes; n.D = c.dim; n.H = H; n.T = T; n.M = M; n.L = L; n.K = K; n.nfeat = c.n_features;
    n.E = c.n_nodes * (c.n_nodes - 1);
    n.SR = edge_slots_per_receiver(c.n_nodes);
    n.EP = 32 * ((c.n_nodes * n.SR + 31) / 32);
    n.ND = c.n_nodes * c.dim;
    n.C = c.normalization_constant;
    n.fs = fs;
    n.nn1 = (float)(c.n_nodes - 1);
    n.sqrt_nn1 = std::sqrt((float)(c.n_nodes - 1));
    const int half = T / 2;
    const float ex = std::log(10000.0f) / (float)(half - 1);
    for (int k = 0; k < half; ++k) n.freqs[k] = std::exp((float)k * -ex);
    n.emb = dbuf + off_emb;
    for (int k = 0; k < K; ++k) {
      BlockW& w = n.blk[k];
      const Off& o = off[k];
      w.Wn = dbuf + o.Wn; w.bn = dbuf + o.bn; w.Wp = dbuf + o.Wp; w.bp = dbuf + o.bp; w.wd = dbuf + o.wd;
      w.We = dbuf + o.We; w.Ws = reinterpret_cast<const unsigned*>(dbuf + o.Ws); w.be = dbuf + o.be; w.wx = dbuf + o.wx; w.wg = dbuf + o.wg; w.bx = o.bx; w.bg = o.bg;
      for (int l = 0; l <= L; ++l) {
        w.Wh[l] = dbuf + o.Wh[l];
        w.bh[l] = dbuf + o.bh[l];
        w.Wh_s[l] = reinterpret_cast<const unsigned*>(dbuf + o.Wh_s[l]);
      }
      w.Wn_s = reinterpret_cast<const unsigned*>(dbuf + o.Wn_s);
      w.bp_u = dbuf + o.bp_u; w.wd_u = dbuf + o.wd_u; w.be_u = dbuf + o.be_u; w.wg_u = dbuf + o.wg_u;
      w.wx_u = dbuf + o.wx_u;
      for (int cl = 0; cl < 2 * 4 - 1; ++cl) w.cinv[cl] = o.cinv[cl];
      w.ninv = o.ninv;
      w.pinv = o.pinv;
      for (int l = 0; l <= L; ++l) w.hinv[l] = o.hinv[l];
      w.Wp_s = reinterpret_cast<const unsigned*>(dbuf + o.Wp_s);
      w.Wh_sn0 = reinterpret_cast<const unsigned*>(dbuf + o.Wh_sn0);
      w.hinv_n0 = o.hinv_n0;
      w.W1_s = reinterpret_cast<const unsigned*>(dbuf + o.W1_s);
      w.w1inv = o.w1inv;
      w.Ws3 = reinterpret_cast<const unsigned*>(dbuf + o.Ws3);
    }
    int mpw = 0, rp = 0;
    size_t lds = 0;
    if (shape_supported(c, NT, P) && choose_mpw(c, NT, P, &mpw, &lds, &rp) == ECNF_OK) {
      set_mpw(n, c, NT, P, mpw, rp);
      n.lds_floats = (int)(lds / 4);
      h->lds[ix] = lds;
      // block-1 pair tiles (egnn_eval.hpp PairPlan13): one node feature (every atom's block-1 h is the same), 13 atoms,
      // the M = 128 split primal kernels (8 waves, each with a 1024-float slice of the >= 32 x 260-float P rows) and
      // split tangent kernels (4 waves; 64 P rows)
      n.pairs = (P == 0 && c.n_features == 1 && c.n_nodes == 13 && c.mlp_width == 128 &&
                 (NT == 0 ? split_primal(c, 0, 0) && primal_waves(c) * 1024 <= 32 * 260 : !wide_tangent(c, 1, 0)))
                    ? 1 : 0;
    } else {
      n.MPW = 0;
      h->lds[ix] = 0;
    }
  }
  if (h->net[0].MPW == 0 || h->net[2].MPW == 0) {
    hipFree(dbuf);
    delete h;
    return fail(ECNF_E_UNSUPPORTED, "configuration does not fit the LDS budget");
  }
  {
    // team-mode buffers (team_size): up to kTeamCap molecules of up to team_gcap workgroups each, only where a team
    // kernel exists (the split primal kernels of the BASELINE shapes) and the split kernels can run this parameter
    // set (team_size returns 1 without them)
    const Net& n = h->net[0];
    const int tpm = n.EP / 32;
    h->team_cap = kTeamCap;
    // (M = 256: room for the column-split mode's G = tiles per molecule)
    h->team_gcap = c.mlp_width == 256 ? tpm : std::min(tpm, std::max(4, (tpm + primal_waves(c) - 1) / primal_waves(c)));
    // (the tangent team kernels also exchange the tangent message and shift rows: egnn_eval.hpp team_exchange)
    const bool tan_team = team_shape(c.mlp_width, 1, c.mlp_depth, c.dim, 0);
    // (+ 4 floats: member 0's stop verdict, egnn_eval.hpp team_exchange)
    h->team_slot = (tan_team ? 2 : 1) * (c.n_nodes * M + ((c.n_nodes * c.dim + 3) & ~3)) + tpm * M + 4;
    const size_t nb = (size_t)h->team_cap * 2 * h->team_gcap * h->team_slot * sizeof(float);
    const bool want = h->split_ok && (team_shape(c.mlp_width, 0, c.mlp_depth, c.dim, 0) || tan_team);
    float* tb = nullptr;
    const bool ok_buf = !want || hipMalloc(&tb, nb) == hipSuccess;
    h->team_buf.store(tb);
    if (want && (!ok_buf || hipMalloc(&h->team_sync, kTeamSyncBytes) != hipSuccess)) {
      if (tb) hipFree(tb);
      hipFree(dbuf);
      delete h;
      return fail(ECNF_E_HIP, "team-mode exchange buffers: out of device memory");
    }
  }
  *out = h;
  g_err.clear();
  return ECNF_OK;
}

int ecnf_update_params(ecnf_handle* h, const float* params, int32_t on_device) {
  if (!h || !params) return fail(ECNF_E_INVALID, "NULL argument");
  const size_t n = param_count(h->cfg);
  std::vector<float> host;
  const float* src = params;
  HIP_TRY(hipSetDevice(h->device));
  if (on_device) {
    host.resize(n);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(host.data(), params, n * sizeof(float), hipMemcpyDeviceToHost));
    src = host.data();
  }
  // pack into a fresh handle, then take over its weight buffer and kernel arguments
  ecnf_handle* t = nullptr;
  const int rc = ecnf_create(&h->cfg, src, n, h->device, &t);
  if (rc) return rc;
  HIP_TRY(hipDeviceSynchronize());   // no launch on h's old weights is in flight
  std::swap(h->dbuf, t->dbuf);
  for (int i = 0; i < 4; ++i) {
    h->net[i] = t->net[i];
    h->lds[i] = t->lds[i];
  }
  h->split_ok = t->split_ok;
  if (!h->split_ok) h->prec = ECNF_PREC_FP32;
  if (!h->team_buf.load() && t->team_buf.load()) {   // the new weights admit the split team kernels the old ones did not
    std::lock_guard<std::mutex> tl(h->team_mu);
    std::swap(h->team_sync, t->team_sync);
    t->team_buf.store(h->team_buf.exchange(t->team_buf.load()));   // team_sync first: team_size keys on team_buf
  }
  return ecnf_destroy(t);
}

int ecnf_destroy(ecnf_handle* h) {
  if (!h) return ECNF_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipFree(h->dbuf));
  if (h->arena) HIP_TRY(hipFree(h->arena));
  if (h->arena_ev) HIP_TRY(hipEventDestroy(h->arena_ev));
  if (h->team_buf.load()) HIP_TRY(hipFree(h->team_buf.load()));
  if (h->team_sync) HIP_TRY(hipFree(h->team_sync));
  if (h->team_ev) HIP_TRY(hipEventDestroy(h->team_ev));
  delete h;
  return ECNF_OK;
}

int ecnf_molecules_per_workgroup(ecnf_handle* h, int32_t with_tangent, int32_t* mpw) {
  if (!h || !mpw) return fail(ECNF_E_INVALID, "NULL argument");
  *mpw = h->net[2 * h->prec + (with_tangent ? 1 : 0)].MPW;
  return ECNF_OK;
}

int ecnf_set_precision(ecnf_handle* h, int32_t precision) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (precision != ECNF_PREC_SPLIT_F16 && precision != ECNF_PREC_FP32) return fail(ECNF_E_INVALID, "unknown precision");
  if (precision == ECNF_PREC_SPLIT_F16 && !h->split_ok)
    return fail(ECNF_E_UNSUPPORTED, "edge-MLP weights >= 2^15 in magnitude: this handle runs the strict-fp32 kernels only");
  h->prec = precision;
  return ECNF_OK;
}

int ecnf_get_precision(ecnf_handle* h, int32_t* precision) {
  if (!h || !precision) return fail(ECNF_E_INVALID, "NULL argument");
  *precision = h->prec;
  return ECNF_OK;
}

int ecnf_chain_arithmetic(ecnf_handle* h, int32_t with_tangent, int32_t* mode) {
  if (!h || !mode) return fail(ECNF_E_INVALID, "NULL argument");
  const bool split = split_primal(h->cfg, with_tangent ? 1 : 0, h->prec) ||
                     (kSplitTanChain && h->prec == ECNF_PREC_SPLIT_F16 && with_tangent && h->cfg.mlp_width <= 128) ||
                     (kSplitTanChain && h->prec == ECNF_PREC_SPLIT_F16 && wide_tangent(h->cfg, with_tangent ? 1 : 0, h->prec));
  *mode = split ? ECNF_CHAIN_SPLIT_F16 : ECNF_CHAIN_FP32_MFMA;
  return ECNF_OK;
}

int ecnf_vector_field(ecnf_handle* h, const float* x, const float* t, const int32_t* feat, float* v, int32_t batch,
                      void* stream) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (batch < 0) return fail(ECNF_E_INVALID, "batch < 0");
  if (batch == 0) return ECNF_OK;
  if (!x || !t || !feat || !v) return fail(ECNF_E_INVALID, "NULL argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(dispatch_vf(h, 0, x, t, feat, nullptr, 0, v, nullptr, batch, (hipStream_t)stream));
  g_err.clear();
  return ECNF_OK;
}

int ecnf_vf_jvp(ecnf_handle* h, const float* x, const float* t, const int32_t* feat, const float* tan_in,
                int32_t n_tangents, float* v, float* tan_out, int32_t batch, void* stream) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (batch < 0 || n_tangents < 1) return fail(ECNF_E_INVALID, "batch < 0 or n_tangents < 1");
  if (batch > 0 && (!x || !t || !feat || !tan_in || !tan_out)) return fail(ECNF_E_INVALID, "NULL argument");
  if (h->net[2 * h->prec + 1].MPW == 0)
    return fail(ECNF_E_UNSUPPORTED, no_tangent_msg(h->cfg, h->prec));
  if (batch == 0) return ECNF_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(dispatch_vf(h, 1, x, t, feat, tan_in, n_tangents, v, tan_out, batch, (hipStream_t)stream));
  g_err.clear();
  return ECNF_OK;
}

int ecnf_integrate_workspace_size(ecnf_handle* h, const ecnf_solve_opts* o, int32_t batch, size_t* bytes) {
  if (!h || !o || !bytes) return fail(ECNF_E_INVALID, "NULL argument");
  if (batch < 0) return fail(ECNF_E_INVALID, "batch < 0");
  *bytes = ((exact_sparse(h, o->divergence) ? pcache_floats(h, batch) : 0) + sched_floats(h, o, batch)) * sizeof(float);
  return ECNF_OK;
}

int ecnf_integrate_plan(ecnf_handle* h, const ecnf_solve_opts* o, int32_t batch, int32_t* workgroups,
                        int32_t* launches) {
  if (!h || !o || !workgroups || !launches) return fail(ECNF_E_INVALID, "NULL argument");
  if (batch < 1) return fail(ECNF_E_INVALID, "batch < 1");
  if (o->divergence < ECNF_DIV_NONE || o->divergence > ECNF_DIV_EXACT) return fail(ECNF_E_INVALID, "unknown divergence");
  const int NT = o->divergence == ECNF_DIV_NONE ? 0 : 1, ix = 2 * h->prec + NT;
  if (NT && h->net[ix].MPW == 0) return fail(ECNF_E_UNSUPPORTED, no_tangent_msg(h->cfg, h->prec));
  const bool adaptive = !(o->dt0 > 0.f);
  const int G = team_size(h, NT, batch, nullptr, h->team_mode.load(), o->divergence);
  if (G > 1) {
    *workgroups = batch * G;
    *launches = 1;
    return ECNF_OK;
  }
  // dispatch_integrate's decision, with a workspace of ecnf_integrate_workspace_size bytes
  size_t lds = 0;
  const Net net = net_for_batch(h, ix, batch, &lds, adaptive);
  const int grid = (batch + net.MPW - 1) / net.MPW;
  *workgroups = grid;
  *launches = (sched_floats(h, o, batch) > 0 && adaptive && grid > h->ncu &&
               chunkable(h->cfg.mlp_width / 32, NT, h->prec)) ? 2 : 1;
  // (the re-dealt solve with tail teams adds the stop-and-team launch)
  if (*launches == 2 && tail_teams(h, NT, o->divergence, net.MPW)) *launches = 3;
  return ECNF_OK;
}

int ecnf_reserve_workspace(ecnf_handle* h, size_t bytes) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  std::lock_guard<std::mutex> lk(h->arena_mu);
  if (bytes <= h->arena_bytes) return ECNF_OK;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());   // no call is using the old arena
  if (h->arena) HIP_TRY(hipFree(h->arena));
  h->arena = nullptr;
  h->arena_bytes = 0;
  HIP_TRY(hipMalloc(&h->arena, bytes));
  h->arena_bytes = bytes;
  return ECNF_OK;
}

int ecnf_set_exact_form(ecnf_handle* h, int32_t form) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (form < ECNF_EXACT_FORM_DEFAULT || form > ECNF_EXACT_FORM_SPARSE) return fail(ECNF_E_INVALID, "unknown exact form");
  h->exact_form = form;
  return ECNF_OK;
}

int ecnf_set_team(ecnf_handle* h, int32_t mode) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (mode < 0) return fail(ECNF_E_INVALID, "team mode must be 0 (auto), 1 (off) or >= 2 workgroups per molecule");
  h->team_mode = mode;
  return ECNF_OK;
}

int ecnf_team_workgroups(ecnf_handle* h, int32_t with_tangent, int32_t batch, int32_t* G) {
  if (!h || !G) return fail(ECNF_E_INVALID, "NULL argument");
  *G = team_size(h, with_tangent ? 1 : 0, batch, nullptr, h->team_mode.load(), ECNF_DIV_HUTCHINSON);
  return ECNF_OK;
}

int ecnf_integrate_ws(ecnf_handle* h, const ecnf_solve_opts* o, const float* y0, const int32_t* feat, const float* eps,
                      float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch, void* workspace,
                      size_t workspace_bytes, void* stream) {
  if (!h || !o) return fail(ECNF_E_INVALID, "NULL handle/options");
  if (batch < 0) return fail(ECNF_E_INVALID, "batch < 0");
  if (workspace && batch > 0 && exact_sparse(h, o->divergence) &&
      workspace_bytes < pcache_floats(h, batch) * sizeof(float))
    return fail(ECNF_E_INVALID, "workspace smaller than ecnf_integrate_workspace_size");
  return integrate_impl(h, o, y0, feat, eps, y1, dlogp, nfe, status, batch, (float*)workspace, workspace_bytes,
                        (hipStream_t)stream, false);
}

int ecnf_integrate(ecnf_handle* h, const ecnf_solve_opts* o, const float* y0, const int32_t* feat, const float* eps,
                   float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch, void* stream) {
  if (!h || !o) return fail(ECNF_E_INVALID, "NULL handle/options");
  if (batch < 0) return fail(ECNF_E_INVALID, "batch < 0");
  // the handle's arena (ecnf_reserve_workspace) when it is large enough, else the uncached form (same results);
  // integrate_impl reads the arena under its mutex
  return integrate_impl(h, o, y0, feat, eps, y1, dlogp, nfe, status, batch, nullptr, 0, (hipStream_t)stream, true);
}

}  // extern "C"

namespace {

int integrate_impl(ecnf_handle* h, const ecnf_solve_opts* o, const float* y0, const int32_t* feat, const float* eps,
                   float* y1, float* dlogp, int32_t* nfe, int32_t* status, int32_t batch, float* ws, size_t ws_bytes,
                   hipStream_t stream, bool arena) {
  if (batch > 0 && (!y0 || !feat || !y1)) return fail(ECNF_E_INVALID, "NULL argument");
  if (o->solver != ECNF_SOLVER_EULER && o->solver != ECNF_SOLVER_DOPRI5) return fail(ECNF_E_INVALID, "unknown solver");
  if (o->divergence < ECNF_DIV_NONE || o->divergence > ECNF_DIV_EXACT) return fail(ECNF_E_INVALID, "unknown divergence");
  if (batch > 0 && o->divergence == ECNF_DIV_HUTCHINSON && !eps)
    return fail(ECNF_E_INVALID, "Hutchinson divergence needs eps");
  if (batch > 0 && o->divergence != ECNF_DIV_NONE && !dlogp)
    return fail(ECNF_E_INVALID, "divergence requested but dlogp is NULL");
  if (o->t0 == o->t1) return fail(ECNF_E_INVALID, "t0 == t1");
  const bool adaptive = !(o->dt0 > 0.f);
  if (adaptive && o->solver == ECNF_SOLVER_EULER) return fail(ECNF_E_INVALID, "Euler has no error estimate: give dt0 > 0");
  if (adaptive && !(o->rtol > 0.f && o->atol > 0.f)) return fail(ECNF_E_INVALID, "adaptive stepping needs rtol, atol > 0");
  if (o->max_steps < 1) return fail(ECNF_E_INVALID, "max_steps < 1");
  const int NT = o->divergence == ECNF_DIV_NONE ? 0 : 1;
  if (NT && h->net[2 * h->prec + 1].MPW == 0)
    return fail(ECNF_E_UNSUPPORTED, no_tangent_msg(h->cfg, h->prec));
  if (batch == 0) return ECNF_OK;
  SolveP sp;
  sp.solver = o->solver;
  sp.div = o->divergence;
  sp.adaptive = adaptive ? 1 : 0;
  sp.max_steps = o->max_steps;
  sp.dirf = o->t1 > o->t0 ? 1.0f : -1.0f;
  sp.tau0 = sp.dirf * o->t0;
  sp.tau1 = sp.dirf * o->t1;
  sp.dt0 = adaptive ? 0.f : std::fabs(o->dt0);
  sp.rtol = o->rtol;
  sp.atol = o->atol;
  sp.dtmin = o->dtmin;
  // exact trace: the sparse blocks 1 and K (egnn_eval sparse_a) where they pay (exact_sparse), and their primal
  // aggregates cached over the JVP passes of an evaluation when a workspace of pcache_floats is given: the caller's
  // (ecnf_integrate_ws) or the handle's arena (ecnf_integrate).  The three forms give bitwise equal results between
  // the sparse and the cached form; ecnf_set_exact_form selects the others for A/B runs only.
  sp.sparse1 = exact_sparse(h, o->divergence) && h->exact_form != ECNF_EXACT_FORM_ALL_DUAL ? 1 : 0;
  sp.pcache = nullptr;
  sp.pcache_slots = 0;
  sp.team = TeamP{};   // dispatch_integrate sets it (team_size)
  sp.order = nullptr;
  sp.nslots = nullptr;
  sp.state = nullptr;
  sp.state_stride = 0;
  sp.chunk_steps = 0;
  sp.resume = 0;
  // team mode decided once for this solve: one read of the handle's mode (ecnf_set_team may run concurrently)
  int cols = 0;
  const int G = team_size(h, NT, batch, &cols, h->team_mode.load(), o->divergence);
  const size_t need = sp.sparse1 ? pcache_floats(h, batch) : 0;
  const size_t need_s = G == 1 ? sched_floats(h, o, batch) : 0;
  // the arena pointer and size are read under arena_mu, and the lock is held through the dispatch that uses them:
  // an ecnf_reserve_workspace on another thread cannot free the arena between the read and the launch
  std::unique_lock<std::mutex> lk(h->arena_mu, std::defer_lock);
  if (arena && (need || need_s)) {
    lk.lock();
    ws = h->arena;
    ws_bytes = h->arena_bytes;
  }
  const bool cached = sp.sparse1 && h->exact_form == ECNF_EXACT_FORM_DEFAULT && ws && ws_bytes >= need * sizeof(float);
  if (cached) {
    sp.pcache = ws;
    sp.pcache_slots = (int)(need / pcache_stride(h));
  }
  // the re-deal scratch follows the pcache region (a workspace too small for both runs the solve in one launch)
  float* sched = need_s && ws && ws_bytes >= (need + need_s) * sizeof(float) ? ws + need : nullptr;
  HIP_TRY(hipSetDevice(h->device));
  // a re-dealt solve with tail teams uses the handle's team buffers: ordered like the team-mode solves (team_mu, team_ev)
  std::unique_lock<std::mutex> tlk(h->team_mu, std::defer_lock);
  if (sched && tail_teams(h, NT, o->divergence, h->net[2 * h->prec + NT].MPW)) {
    tlk.lock();
    if (!h->team_ev) HIP_TRY(hipEventCreateWithFlags(&h->team_ev, hipEventDisableTiming));
    if (h->team_used && h->team_stream != stream) HIP_TRY(hipStreamWaitEvent(stream, h->team_ev, 0));
  }
  auto team_done = [&]() -> hipError_t {
    if (!tlk.owns_lock()) return hipSuccess;
    const hipError_t e = hipEventRecord(h->team_ev, stream);
    h->team_used = true;
    h->team_stream = stream;
    return e;
  };
  if ((cached || sched) && arena) {
    // the arena is shared by every ecnf_integrate call on the handle: calls on different streams are ordered
    // through an event (no host synchronisation), and the bookkeeping is guarded for calls from several threads
    // (arena_mu, held since the arena was read)
    if (!h->arena_ev) HIP_TRY(hipEventCreateWithFlags(&h->arena_ev, hipEventDisableTiming));
    if (h->arena_used && h->arena_stream != stream) HIP_TRY(hipStreamWaitEvent(stream, h->arena_ev, 0));
    HIP_TRY(dispatch_integrate(h, NT, sp, G, cols, y0, feat, eps, y1, dlogp, nfe, status, batch, stream, sched));
    HIP_TRY(team_done());
    HIP_TRY(hipEventRecord(h->arena_ev, stream));
    h->arena_used = true;
    h->arena_stream = stream;
  } else if (G > 1) {
    // team mode: the exchange slots and counters are shared by every solve on the handle (ordered as the arena)
    std::lock_guard<std::mutex> tl(h->team_mu);
    if (!h->team_ev) HIP_TRY(hipEventCreateWithFlags(&h->team_ev, hipEventDisableTiming));
    if (h->team_used && h->team_stream != stream) HIP_TRY(hipStreamWaitEvent(stream, h->team_ev, 0));
    HIP_TRY(dispatch_integrate(h, NT, sp, G, cols, y0, feat, eps, y1, dlogp, nfe, status, batch, stream));
    HIP_TRY(hipEventRecord(h->team_ev, stream));
    h->team_used = true;
    h->team_stream = stream;
  } else {
    HIP_TRY(dispatch_integrate(h, NT, sp, G, cols, y0, feat, eps, y1, dlogp, nfe, status, batch, stream, sched));
    HIP_TRY(team_done());
  }
  g_err.clear();
  return ECNF_OK;
}

}  // namespace

extern "C" {

int ecnf_base_sample(ecnf_handle* h, const float* z, float* x0, int32_t batch, void* stream) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (batch <= 0) return batch == 0 ? ECNF_OK : fail(ECNF_E_INVALID, "batch < 0");
  if (!z || !x0) return fail(ECNF_E_INVALID, "NULL argument");
  HIP_TRY(hipSetDevice(h->device));
  const int n = batch * h->cfg.dim;
  hipLaunchKernelGGL(base_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, z, x0, batch,
                     h->cfg.n_nodes, h->cfg.dim, h->cfg.base_scale);
  HIP_TRY(hipGetLastError());
  return ECNF_OK;
}

int ecnf_base_log_prob(ecnf_handle* h, const float* y, float* log_p, int32_t batch, void* stream) {
  if (!h) return fail(ECNF_E_INVALID, "NULL handle");
  if (batch <= 0) return batch == 0 ? ECNF_OK : fail(ECNF_E_INVALID, "batch < 0");
  if (!y || !log_p) return fail(ECNF_E_INVALID, "NULL argument");
  HIP_TRY(hipSetDevice(h->device));
  hipLaunchKernelGGL(base_log_prob_kernel, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, y, log_p,
                     batch, h->cfg.n_nodes, h->cfg.dim, h->cfg.base_scale);
  HIP_TRY(hipGetLastError());
  return ECNF_OK;
}

int ecnf_target_log_prob(const ecnf_target* t, const float* x, float* log_p, int32_t batch, void* stream) {
  if (!t) return fail(ECNF_E_INVALID, "target is NULL");
  if (t->kind != ECNF_TARGET_LJ && t->kind != ECNF_TARGET_DW) return fail(ECNF_E_INVALID, "unknown target kind");
  if (t->n_nodes < 2 || t->dim < 1 || t->dim > 3) return fail(ECNF_E_INVALID, "target needs n_nodes >= 2, 1 <= dim <= 3");
  if (!(t->tau > 0.f)) return fail(ECNF_E_INVALID, "target tau must be > 0");
  if (batch < 0) return fail(ECNF_E_INVALID, "batch < 0");
  if (batch == 0) return ECNF_OK;
  if (!x || !log_p) return fail(ECNF_E_INVALID, "NULL argument");
  hipLaunchKernelGGL(target_log_prob_kernel, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, *t, x, log_p,
                     batch);
  HIP_TRY(hipGetLastError());
  return ECNF_OK;
}

int ecnf_lse_partials(const float* v, const float* mask, int32_t n, float* out, void* stream) {
  if (n < 0) return fail(ECNF_E_INVALID, "n < 0");
  if (!out || (n > 0 && !v)) return fail(ECNF_E_INVALID, "NULL argument");
  hipLaunchKernelGGL(lse_partials_kernel, dim3(1), dim3(kLseThreads), 0, (hipStream_t)stream, v, mask, n, out);
  HIP_TRY(hipGetLastError());
  return ECNF_OK;
}

}  // extern "C"
