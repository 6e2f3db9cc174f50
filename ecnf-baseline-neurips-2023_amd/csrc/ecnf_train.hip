// ecnf_train.hip — the flow-matching training step of the EGNN vector field on MI355X (gfx950).
//
// Restates, with reverse-mode derivatives written out by hand (no autodiff framework):
//   flow_matching_loss_fn      ecnf/cnf/loss.py:10-32        loss = mean((v(x_t, t) - u_t)^2),
//                              ecnf/cnf/core.py:35-39        x_t = (1 - (1 - sigma) t) x0 + t x1, u_t = x1 - (1 - sigma) x0
//   jax.grad(loss, params)     ecnf/cnf/gradient_step.py:30-36
//   optax.adam + apply_updates ecnf/cnf/gradient_step.py:38-40, setup_training.py:100-109 (+ EMA :43-47)
// through FlatEgnn (build_cnf.py:68-93), EGNN.call_single (egnn.py:144-190), EGCL (egnn.py:49-114) and MLP
// (mlp.py:7-19).
//
// Design.  Training batches are small (lj13.yaml: 64 molecules, 9984 edges), so the step is a stream of layered
// kernels over HBM-resident activations rather than one fused kernel: every dense layer is a strict-fp32 GEMM on
// v_mfma_f32_32x32x2_f32 (gemm_kernel: 64x64 tiles, 4 waves of 32x32, LDS-staged 16-deep k tiles) with a fused
// epilogue (bias, residual, SiLU / SiLU' ), weight gradients are split-K GEMMs reduced in a fixed order, and the
// graph operations (edge gathers, receiver / sender segment sums, shifts, gate) are one thread per output element
// summing a fixed edge order.  Every gradient entry is written exactly once: the step is deterministic (bitwise
// run-to-run) and allocation-free after ecnf_trainer_create.
//
// Activations saved per block k for the backward pass (B molecules, BN = B N node rows, BE = B N (N-1) edge rows):
//   hin [BN][H+T], h1 [BN][H], xc [BN][D] (per block input), P_s / P_r [BN][M], r [BE][D], len [BE],
//   z_e / a_e [L][BE][M] (phi_e), z_x / a_x [L][BE][M] (phi_x torso), px [BE], g [BE], hcat [BN][M+H],
//   z_h / a_h [L+1][BN][M|H] (phi_h)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ecnf.h"

namespace ecnf {
int set_error(int code, const char* msg);   // ecnf_hip.hip
}

namespace ecnf_train {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + __expf(-z)); }
__device__ __forceinline__ float silu(float z) { return z * sigm(z); }
__device__ __forceinline__ float dsilu(float z) {
  const float s = sigm(z);
  return s * (1.0f + z * (1.0f - s));
}

// ---------------------------------------------------------------------------------------------------------------
// GEMM: C[M][N] = alpha op(A)[M][K] op(B)[K][N] (+ bias[N]) (+ R) (+ C if accumulate), then optionally
// z *= silu'(Zs) (the backward of a SiLU layer) and Aout = silu(z) (the forward one, C keeps the pre-activation).
// TA: A stored [K][M] (lda over m); TB: B stored [N][K].  ksplit > 1: block z sums its k-range into the partial
// C + z * split_stride (no epilogue), combined by reduce_batched in split order.  colsum (weight gradients, TA && !TB):
// the column sums of B over the block's k-range (the bias gradient sum_k dZ[k][n]), written by the first m-tile's
// wave 0 into colsum[n] (ksplit == 1) or colsum_part[z][n].
//
// 64x64 tile per 256-thread workgroup (4 waves of 32x32 on v_mfma_f32_32x32x2_f32), 32-deep k tiles double-buffered
// in LDS with the next tile's global loads in flight (registers) while the current one is multiplied.  Both operands
// are staged k-contiguous ([m][k], [n][k], row stride 33): the MFMA operand reads (32 rows x 2 k per wave) and the
// stores of either source layout touch distinct banks.
// ---------------------------------------------------------------------------------------------------------------
struct GemmArgs {
  int M, N, K;
  const float* A; long lda;
  const float* B; long ldb;
  float* C; long ldc;
  float alpha;
  const float* bias;
  const float* R; long ldr;
  const float* Zs; long ldz;
  float* Aout; long ldo;
  int accumulate;
  int ksplit; long split_stride;
  float* colsum; float* colsum_part;
  int sqA;   // A's elements enter squared (|r|^2 from the edge lengths)
};

constexpr int GT = 64, GK = 32, GS = GK + 1, GE = GT * GK / 256;   // GE: elements per thread per operand tile

template <bool TA, bool TB, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  // VA / VB (host-checked for the whole launch): the operand's rows are 16-B aligned, its tiles whole (the m / n
  // extent a multiple of 64, K a multiple of 32), so it is loaded as float4s; otherwise as clamped scalars (every lane
  // loads a valid address, out-of-range elements are zeroed afterwards: no divergent branches around the loads, so
  // the next tile's loads stay in flight across the MFMAs)
  __shared__ float As[2][GT * GS];
  __shared__ float Bs[2][GT * GS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  int kb = 0, ke = g.K;
  if (g.ksplit > 1) {
    const int kc = (((g.K + g.ksplit - 1) / g.ksplit) + GK - 1) / GK * GK;
    kb = blockIdx.z * kc;
    ke = min(g.K, kb + kc);
  }
  // scalar element e of this thread: (row within the tile, k within the tile), source-coalesced
  auto a_idx = [&](int e, int& mm, int& kk) {
    const int i = tid + 256 * e;
    if (TA) { mm = i % GT; kk = i / GT; } else { kk = i % GK; mm = i / GK; }
  };
  auto b_idx = [&](int e, int& nn, int& kk) {
    const int i = tid + 256 * e;
    if (TB) { kk = i % GK; nn = i / GK; } else { nn = i % GT; kk = i / GT; }
  };
  float ra[GE], rb[GE];
  auto load = [&](int k0) {
    if (VA) {
#pragma unroll
      for (int e = 0; e < GE / 4; ++e) {
        const int q = tid + 256 * e;
        const float4 v = TA ? *reinterpret_cast<const float4*>(g.A + (long)(k0 + q / 16) * g.lda + m0 + 4 * (q % 16))
                            : *reinterpret_cast<const float4*>(g.A + (long)(m0 + q / 8) * g.lda + k0 + 4 * (q % 8));
        ra[4 * e] = v.x; ra[4 * e + 1] = v.y; ra[4 * e + 2] = v.z; ra[4 * e + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < GE; ++e) {
        int mm, kk;
        a_idx(e, mm, kk);
        const int gm = min(m0 + mm, g.M - 1), gk = min(k0 + kk, ke - 1);
        ra[e] = TA ? g.A[(long)gk * g.lda + gm] : g.A[(long)gm * g.lda + gk];
      }
    }
    if (VB) {
#pragma unroll
      for (int e = 0; e < GE / 4; ++e) {
        const int q = tid + 256 * e;
        const float4 v = TB ? *reinterpret_cast<const float4*>(g.B + (long)(n0 + q / 8) * g.ldb + k0 + 4 * (q % 8))
                            : *reinterpret_cast<const float4*>(g.B + (long)(k0 + q / 16) * g.ldb + n0 + 4 * (q % 16));
        rb[4 * e] = v.x; rb[4 * e + 1] = v.y; rb[4 * e + 2] = v.z; rb[4 * e + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < GE; ++e) {
        int nn, kk;
        b_idx(e, nn, kk);
        const int gn = min(n0 + nn, g.N - 1), gk = min(k0 + kk, ke - 1);
        rb[e] = TB ? g.B[(long)gn * g.ldb + gk] : g.B[(long)gk * g.ldb + gn];
      }
    }
  };
  auto store = [&](int buf, int k0) {
    if (VA) {
#pragma unroll
      for (int e = 0; e < GE / 4; ++e) {
        const int q = tid + 256 * e;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (TA) As[buf][(4 * (q % 16) + j) * GS + q / 16] = ra[4 * e + j];
          else As[buf][(q / 8) * GS + 4 * (q % 8) + j] = ra[4 * e + j];
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < GE; ++e) {
        int mm, kk;
        a_idx(e, mm, kk);
        const float v = g.sqA ? ra[e] * ra[e] : ra[e];
        As[buf][mm * GS + kk] = (m0 + mm < g.M && k0 + kk < ke) ? v : 0.f;
      }
    }
    if (VB) {
#pragma unroll
      for (int e = 0; e < GE / 4; ++e) {
        const int q = tid + 256 * e;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (TB) Bs[buf][(q / 8) * GS + 4 * (q % 8) + j] = rb[4 * e + j];
          else Bs[buf][(4 * (q % 16) + j) * GS + q / 16] = rb[4 * e + j];
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < GE; ++e) {
        int nn, kk;
        b_idx(e, nn, kk);
        Bs[buf][nn * GS + kk] = (n0 + nn < g.N && k0 + kk < ke) ? rb[e] : 0.f;
      }
    }
  };
  const bool do_colsum = g.colsum && blockIdx.y == 0 && tid < GT;
  float csum = 0.f;
  f32x16 acc = {};
  if (kb < ke) {
    load(kb);
    store(0, kb);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += GK) {
    const bool more = k0 + GK < ke;
    if (more) load(k0 + GK);
    const float* Ab = &As[buf][(wm + (lane & 31)) * GS + (lane >> 5)];
    const float* Bb = &Bs[buf][(wn + (lane & 31)) * GS + (lane >> 5)];
    float av[GK / 2], bv[GK / 2];
#pragma unroll
    for (int kk = 0; kk < GK / 2; ++kk) {
      av[kk] = Ab[2 * kk];
      bv[kk] = Bb[2 * kk];
    }
#pragma unroll
    for (int kk = 0; kk < GK / 2; ++kk) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk], bv[kk], acc, 0, 0, 0);
    if (do_colsum) {
#pragma unroll 8
      for (int kk = 0; kk < GK; ++kk) csum += Bs[buf][tid * GS + kk];
    }
    if (more) store(buf ^ 1, k0 + GK);
    __syncthreads();
    buf ^= 1;
  }
  if (do_colsum && n0 + tid < g.N) {
    if (g.ksplit > 1) g.colsum_part[(long)blockIdx.z * g.N + n0 + tid] = csum;
    else g.colsum[n0 + tid] = csum;
  }
  // epilogue: every operand of the 16 rows is loaded (clamped addresses) before any store, so the loads overlap
  // (C may alias nothing the epilogue reads except itself under `accumulate`)
  const int col = n0 + wn + (lane & 31);
  if (col >= g.N) return;
  int rows[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) rows[r] = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
  float z[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = g.alpha * acc[r];
  if (g.ksplit > 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (rows[r] < g.M) g.C[blockIdx.z * g.split_stride + (long)rows[r] * g.ldc + col] = z[r];
    return;
  }
  auto ld16 = [&](const float* p, long ld, float* out) {
#pragma unroll
    for (int r = 0; r < 16; ++r) out[r] = p[(long)min(rows[r], g.M - 1) * ld + col];
  };
  if (g.bias) {
    const float b = g.bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] += b;
  }
  float t[16];
  if (g.R) {
    ld16(g.R, g.ldr, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] += t[r];
  }
  if (g.accumulate) {
    ld16(g.C, g.ldc, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] += t[r];
  }
  if (g.Zs) {
    ld16(g.Zs, g.ldz, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] *= dsilu(t[r]);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (rows[r] < g.M) g.C[(long)rows[r] * g.ldc + col] = z[r];
  if (g.Aout) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (rows[r] < g.M) g.Aout[(long)rows[r] * g.ldo + col] = silu(z[r]);
  }
}

// Deferred split reductions: dst[i] = sum_s P[s][i] (s in order) for up to kRedMax (P, S, n, dst) entries in one
// launch.  Nothing in the step reads a gradient before the step ends, so the weight-gradient GEMMs' partials stay in
// a partial arena and are reduced together (one launch per arena fill instead of one per GEMM).  Entry e owns blocks
// [first[e], first[e + 1]) of 256 outputs each.
constexpr int kRedMax = 64;
struct RedEntry {
  const float* P;
  float* dst;
  int S, n, first;
};
struct RedBatch {
  int count;
  RedEntry e[kRedMax];
};

__global__ void reduce_batched(RedBatch rb) {
  int k = 0;
  while (k + 1 < rb.count && (int)blockIdx.x >= rb.e[k + 1].first) ++k;
  const RedEntry& r = rb.e[k];
  const long i = (long)((int)blockIdx.x - r.first) * blockDim.x + threadIdx.x;
  if (i >= r.n) return;
  float acc = 0.f;
#pragma unroll 4
  for (int q = 0; q < r.S; ++q) acc += r.P[(long)q * r.n + i];
  r.dst[i] = acc;
}

// ---------------------------------------------------------------------------------------------------------------
// model geometry: molecule b, receiver i, slot j -> edge row b E + i (N-1) + j, sender (i + 1 + j) mod N
// (graph.py:6-14); node row b N + i
// ---------------------------------------------------------------------------------------------------------------
struct Geom {
  int B, N, D, H, T, M, L, K, E, nfeat;
  float C, sigma;
};

__device__ __forceinline__ int sender_of(int i, int j, int N) {
  int s = i + 1 + j;
  return s >= N ? s - N : s;
}
// edge slot of (receiver i, sender s != i)
__device__ __forceinline__ int slot_of(int i, int s, int N) {
  int j = s - i - 1;
  return j < 0 ? j + N : j;
}

struct Freqs {
  float f[8];   // exp(-k ln(1e4) / (T/2 - 1)) in fp32 (build_cnf.py:23-27)
};

// x_t, u_t (core.py:35-39), input mean, centred positions (egnn.py:160), time embedding (build_cnf.py:18-32).  One
// 64-thread block per molecule: coordinates one per thread, the per-dimension means summed over the nodes in order
// (N * D <= kMaxND)
constexpr int kMaxND = 256;
__global__ void k_prologue(Geom G, const float* __restrict__ x1, const float* __restrict__ x0,
                           const float* __restrict__ t, Freqs freqs, float* ut, float* mean, float* xc0,
                           float* temb) {
  __shared__ float xs[kMaxND];
  __shared__ float mu[3];
  const int b = blockIdx.x, ND = G.N * G.D;
  const float tb = t[b];
  for (int k = threadIdx.x; k < ND; k += blockDim.x) {
    const long o = (long)b * ND + k;
    xs[k] = (1.0f - (1.0f - G.sigma) * tb) * x0[o] + tb * x1[o];
    ut[o] = x1[o] - (1.0f - G.sigma) * x0[o];
  }
  __syncthreads();
  if ((int)threadIdx.x < G.D) {
    const int d = threadIdx.x;
    float a = 0.f;
    for (int i = 0; i < G.N; ++i) a += xs[i * G.D + d];
    a /= (float)G.N;
    mu[d] = a;
    mean[b * G.D + d] = a;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < ND; k += blockDim.x) xc0[(long)b * ND + k] = xs[k] - mu[k % G.D];
  const int half = G.T / 2;
  const float ts = tb * 1000.0f;
  for (int k = threadIdx.x; k < G.T; k += blockDim.x) {
    const float arg = ts * freqs.f[k < half ? k : k - half];
    temb[b * G.T + k] = k < half ? sinf(arg) : cosf(arg);
  }
}

// hin = [h | temb] (h: embedding rows for block 0, else the previous block's output).  An embedding id outside
// [0, n_features) (device-resident features are not checked on the host: no sync on the call path) is never used as
// an index: its row becomes NaN, so the loss and the gradient are NaN instead of silently reading past the params
// (nn.Embed would fail on it); k_embed_bwd matches no vocabulary row for it.
__global__ void k_hin(Geom G, const float* __restrict__ h, long ldh, const int32_t* __restrict__ feat,
                      const float* __restrict__ emb, const float* __restrict__ temb, float* hin) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int W = G.H + G.T;
  if (idx >= (long)G.B * G.N * W) return;
  const long row = idx / W;
  const int c = (int)(idx - row * W);
  float v;
  if (c < G.H) {
    if (feat) {
      const int f = feat[row];
      v = (f >= 0 && f < G.nfeat) ? emb[(long)f * G.H + c] : __builtin_nanf("");
    } else {
      v = h[row * ldh + c];
    }
  } else {
    v = temb[(row / G.N) * G.T + (c - G.H)];
  }
  hin[idx] = v;
}

// r_ij = x_i - x_j, |r| = safe_norm (egnn.py:73-74, numerical.py:7-10)
__global__ void k_edge_geom(Geom G, const float* __restrict__ xc, float* r, float* len) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)G.B * G.E) return;
  const int b = (int)(e / G.E), el = (int)(e - (long)b * G.E), i = el / (G.N - 1), j = el - i * (G.N - 1);
  const int s = sender_of(i, j, G.N);
  float x2 = 0.f;
  for (int d = 0; d < G.D; ++d) {
    const float v = xc[((long)b * G.N + i) * G.D + d] - xc[((long)b * G.N + s) * G.D + d];
    r[e * G.D + d] = v;
    x2 += v * v;
  }
  len[e] = sqrtf(x2 == 0.f ? 1.0f : x2);
}

// phi_e layer 1 from the per-node halves: z = P_s[s] + P_r[r] + |r|^2 w_d + b; a = silu(z)  (egnn.py:76,79)
__global__ void k_layer1(Geom G, const float* __restrict__ Ps, const float* __restrict__ Pr,
                         const float* __restrict__ len, const float* __restrict__ wd, const float* __restrict__ bias,
                         float* Z, float* A) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)G.B * G.E * G.M) return;
  const long e = idx / G.M;
  const int c = (int)(idx - e * G.M);
  const int b = (int)(e / G.E), el = (int)(e - (long)b * G.E), i = el / (G.N - 1), j = el - i * (G.N - 1);
  const int s = sender_of(i, j, G.N);
  const float l = len[e];
  const float z = Ps[((long)b * G.N + s) * G.M + c] + Pr[((long)b * G.N + i) * G.M + c] + (l * l) * wd[c] + bias[c];
  Z[idx] = z;
  A[idx] = silu(z);
}

// per edge: px = a_x . w_x + b_x (egnn.py:83-85); gate g = sigmoid(m . w_g + b_g) (egnn.py:99-101).  64 threads
// per edge (4 edges per 256-thread block)
__global__ void k_edge_dots(Geom G, const float* __restrict__ ax, const float* __restrict__ wx,
                            const float* __restrict__ bx, const float* __restrict__ m, const float* __restrict__ wg,
                            const float* __restrict__ bg, float* px, float* gate) {
  const long e = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= (long)G.B * G.E) return;
  float sx = 0.f, sg = 0.f;
  for (int c = lane; c < G.M; c += 64) {
    sx += ax[e * G.M + c] * wx[c];
    if (gate) sg += m[e * G.M + c] * wg[c];
  }
  for (int o = 32; o > 0; o >>= 1) {
    sx += __shfl_xor(sx, o);
    sg += __shfl_xor(sg, o);
  }
  if (lane == 0) {
    px[e] = sx + bx[0];
    if (gate) gate[e] = sigm(sg + bg[0]);
  }
}

// receiver segment sums (e3nn scatter_sum): x_out = x_in + sum_j px r / (C + |r|) / (N - 1) (egnn.py:87-95,113);
// hcat = [sum_j g m / sqrt(N - 1) | h1] (egnn.py:102-105).  One thread per output element, j in order.
__global__ void k_node_shift(Geom G, const float* __restrict__ xin, const float* __restrict__ px,
                             const float* __restrict__ r, const float* __restrict__ len, float* xout) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)G.B * G.N * G.D) return;
  const long row = idx / G.D;
  const int d = (int)(idx - row * G.D);
  const long e0 = row * (G.N - 1);   // b E + i (N - 1) == (b N + i)(N - 1)
  float acc = 0.f;
  for (int j = 0; j < G.N - 1; ++j) {
    const long e = e0 + j;
    acc += px[e] * r[e * G.D + d] / (G.C + len[e]);
  }
  xout[idx] = xin[idx] + acc / (float)(G.N - 1);
}

__global__ void k_node_agg(Geom G, const float* __restrict__ m, const float* __restrict__ gate,
                           const float* __restrict__ h1, float* hcat) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int W = G.M + G.H;
  if (idx >= (long)G.B * G.N * W) return;
  const long row = idx / W;
  const int c = (int)(idx - row * W);
  if (c >= G.M) {
    hcat[idx] = h1[row * G.H + (c - G.M)];
    return;
  }
  const long e0 = row * (G.N - 1);
  float acc = 0.f;
  for (int j = 0; j < G.N - 1; ++j) acc += m[(e0 + j) * G.M + c] * gate[e0 + j];
  hcat[idx] = acc / sqrtf((float)(G.N - 1));
}

// v = ((x_K - x_c0) - mean) fs (egnn.py:183-188), per-molecule partial loss sum((v - u)^2) and d fs, and
// d loss / d x_K = 2 (v - u) fs / (B N D).  One 64-thread block per molecule; the two sums in coordinate order
__global__ void k_output(Geom G, const float* __restrict__ xK, const float* __restrict__ xc0,
                         const float* __restrict__ mean, const float* __restrict__ ut, const float* __restrict__ fs_p,
                         float* dxK, float* part_loss, float* part_dfs) {
  __shared__ float sq[kMaxND], sf[kMaxND];
  const int b = blockIdx.x, ND = G.N * G.D;
  const float fs = fs_p[0];
  const float sc = 2.0f / ((float)G.B * (float)ND);
  for (int k = threadIdx.x; k < ND; k += blockDim.x) {
    const long o = (long)b * ND + k;
    const float pre = (xK[o] - xc0[o]) - mean[b * G.D + (k % G.D)];
    const float diff = pre * fs - ut[o];
    sq[k] = diff * diff;
    sf[k] = sc * diff * pre;
    dxK[o] = sc * diff * fs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
    for (int k = 0; k < ND; ++k) {
      a += sq[k];
      c += sf[k];
    }
    part_loss[b] = a;
    part_dfs[b] = c;
  }
}

__global__ void k_finish_loss(int B, float inv_count, const float* __restrict__ part_loss,
                              const float* __restrict__ part_dfs, float* loss, float* dfs) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float a = 0.f, f = 0.f;
  for (int b = 0; b < B; ++b) {
    a += part_loss[b];
    f += part_dfs[b];
  }
  *loss = a * inv_count;
  *dfs = f;
}

// ---- backward ----

// out[r][c] = X[r][c] (+ Y[r][c])
__global__ void k_copy_add(long rows, int cols, const float* __restrict__ X, long ldx, const float* __restrict__ Y,
                           long ldy, float* out, long ldo) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const long r = idx / cols;
  const int c = (int)(idx - r * cols);
  out[r * ldo + c] = X[r * ldx + c] + (Y ? Y[r * ldy + c] : 0.0f);
}

// gate / aggregation backward (egnn.py:99-104): dm_i = dhcat[:, :M] of the receiver; per edge
// dgm = dm_i / sqrt(N-1); de = (m . dgm) g (1 - g); dm = g dgm + de w_g.  64 threads per edge.
__global__ void k_gate_bwd(Geom G, const float* __restrict__ m, const float* __restrict__ gate,
                           const float* __restrict__ dhcat, const float* __restrict__ wg, float* dm, float* de_out) {
  const long e = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= (long)G.B * G.E) return;
  const long row = e / (G.N - 1);
  const float is = 1.0f / sqrtf((float)(G.N - 1));
  const float* dmi = dhcat + row * (G.M + G.H);
  float dg = 0.f;
  for (int c = lane; c < G.M; c += 64) dg += m[e * G.M + c] * (dmi[c] * is);
  for (int o = 32; o > 0; o >>= 1) dg += __shfl_xor(dg, o);
  const float gv = gate[e];
  const float de = dg * gv * (1.0f - gv);
  for (int c = lane; c < G.M; c += 64) dm[e * G.M + c] = gv * (dmi[c] * is) + de * wg[c];
  if (lane == 0) de_out[e] = de;
}

// shift backward (egnn.py:87-95): with dD = d x_out[receiver] / (N - 1), den = C + |r|:
//   dpx = dD . r / den;  dr = px dD / den - px (r . dD) / den^2 * d|r|/dr  (d|r|/dr = r / |r|, 0 for safe_norm's 1)
// fused with the phi_x torso's last layer: dZ[e][c] = dpx w_x[c] silu'(Z[e][c]) (the Dense(1) output's input).
// One thread per (edge, column); column 0 also writes dpx and dr
__global__ void k_shift_bwd(Geom G, const float* __restrict__ dxout, const float* __restrict__ px,
                            const float* __restrict__ r, const float* __restrict__ len, const float* __restrict__ wx,
                            const float* __restrict__ Z, float* dpx, float* dr, float* dZ) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)G.B * G.E * G.M) return;
  const long e = idx / G.M;
  const int c = (int)(idx - e * G.M);
  const long row = e / (G.N - 1);
  const float l = len[e], den = G.C + l;
  float x2 = 0.f, rd = 0.f, dD[3];
  for (int d = 0; d < G.D; ++d) {
    dD[d] = dxout[row * G.D + d] / (float)(G.N - 1);
    const float rv = r[e * G.D + d];
    x2 += rv * rv;
    rd += rv * dD[d];
  }
  const float dp = rd / den;
  dZ[idx] = dp * wx[c] * dsilu(Z[idx]);
  if (c == 0) {
    const float p = px[e];
    dpx[e] = dp;
    const float dl = x2 == 0.f ? 0.f : -p * rd / (den * den) / l;
    for (int d = 0; d < G.D; ++d) dr[e * G.D + d] = p * dD[d] / den + dl * r[e * G.D + d];
  }
}

// layer-1 backward, node side: dP_r[i] = sum over the receiver's edges of dz1, dP_s[j] = sum over the sender's
__global__ void k_layer1_node_bwd(Geom G, const float* __restrict__ dz1, float* dPs, float* dPr) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)G.B * G.N * G.M) return;
  const long row = idx / G.M;
  const int c = (int)(idx - row * G.M);
  const int b = (int)(row / G.N), n = (int)(row - (long)b * G.N);
  const long eb = (long)b * G.E;
  float ar = 0.f, as = 0.f;
  for (int j = 0; j < G.N - 1; ++j) ar += dz1[(eb + n * (G.N - 1) + j) * G.M + c];
  for (int i = 0; i < G.N; ++i) {
    if (i == n) continue;
    as += dz1[(eb + i * (G.N - 1) + slot_of(i, n, G.N)) * G.M + c];
  }
  dPr[idx] = ar;
  dPs[idx] = as;
}

// layer-1 backward, edge side: d|r|^2 = dz1 . w_d -> dr += 2 d|r|^2 r (0 for safe_norm's constant branch)
__global__ void k_layer1_edge_bwd(Geom G, const float* __restrict__ dz1, const float* __restrict__ wd,
                                  const float* __restrict__ r, float* dr) {
  const long e = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= (long)G.B * G.E) return;
  float s = 0.f;
  for (int c = lane; c < G.M; c += 64) s += dz1[e * G.M + c] * wd[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) {
    float x2 = 0.f;
    for (int d = 0; d < G.D; ++d) x2 += r[e * G.D + d] * r[e * G.D + d];
    if (x2 != 0.f)
      for (int d = 0; d < G.D; ++d) dr[e * G.D + d] += 2.0f * s * r[e * G.D + d];
  }
}

// positions backward through r_ij = x_i - x_j: dx_in[i] = dx_out[i] + sum_{e: recv i} dr - sum_{e: send i} dr
__global__ void k_dx_bwd(Geom G, const float* __restrict__ dxout, const float* __restrict__ dr, float* dxin) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)G.B * G.N * G.D) return;
  const long row = idx / G.D;
  const int d = (int)(idx - row * G.D);
  const int b = (int)(row / G.N), n = (int)(row - (long)b * G.N);
  const long eb = (long)b * G.E;
  float a = 0.f;
  for (int j = 0; j < G.N - 1; ++j) a += dr[(eb + n * (G.N - 1) + j) * G.D + d];
  float s = 0.f;
  for (int i = 0; i < G.N; ++i) {
    if (i == n) continue;
    s += dr[(eb + i * (G.N - 1) + slot_of(i, n, G.N)) * G.D + d];
  }
  dxin[idx] = dxout[idx] + a - s;
}

// embedding gradient: dEmb[f][c] = sum over node rows with feature f of dhin[row][c].  Partial sums over chunks of
// 64 rows (256 threads = 4 row lanes x 64 columns; grid.x = n_features x column blocks, grid.y = row chunks), each
// chunk's 4 lanes combined in order; the chunks are summed in order by reduce_batched: part[chunk][f H + c]
__global__ void k_embed_bwd(Geom G, const float* __restrict__ dhin, long ld, const int32_t* __restrict__ feat,
                            float* part) {
  __shared__ float red[4][64];
  const int hc = (G.H + 63) / 64;
  const int f = blockIdx.x / hc, c = (blockIdx.x % hc) * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const long BN = (long)G.B * G.N, r0 = (long)blockIdx.y * 64;
  float a = 0.f;
  if (c < G.H)
    for (int j = 0; j < 16; ++j) {
      const long row = r0 + rl + 4 * j;
      if (row < BN && feat[row] == f) a += dhin[row * ld + c];
    }
  red[rl][threadIdx.x & 63] = a;
  __syncthreads();
  if (rl == 0 && c < G.H) {
    const int q = threadIdx.x;
    part[(long)blockIdx.y * G.nfeat * G.H + (long)f * G.H + c] = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
  }
}

// ---- Adam (optax.scale_by_adam + scale(-lr)) and EMA, with the global norms of the gradient and the update ----
__global__ void k_adam(long n, const float* __restrict__ grad, float* params, float* mu, float* nu, float* ema,
                       float lr, float b1, float b2, float eps, float eps_root, float bc1, float bc2, float ema_beta,
                       float* part) {
  __shared__ float red[2][256];
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float gg = 0.f, uu = 0.f;
  if (i < n) {
    const float gv = grad[i];
    const float m = b1 * mu[i] + (1.0f - b1) * gv;
    const float v = b2 * nu[i] + (1.0f - b2) * gv * gv;
    mu[i] = m;
    nu[i] = v;
    const float mh = m / bc1, vh = v / bc2;
    const float u = -lr * (mh / (sqrtf(vh + eps_root) + eps));
    const float p = params[i] + u;
    params[i] = p;
    if (ema) ema[i] = ema[i] * ema_beta + (1.0f - ema_beta) * p;
    gg = gv * gv;
    uu = u * u;
  }
  red[0][threadIdx.x] = gg;
  red[1][threadIdx.x] = uu;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0];
    part[2 * blockIdx.x + 1] = red[1][0];
  }
}

// global norms from the Adam blocks' partials: one 256-thread block, strided partial sums then a fixed-order tree
__global__ void k_norms(int nb, const float* __restrict__ part, float* norms) {
  __shared__ float red[2][256];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    norms[0] = sqrtf(red[0][0]);
    norms[1] = sqrtf(red[1][0]);
  }
}

}  // namespace ecnf_train

using namespace ecnf_train;

// ---------------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------------
namespace {

// offsets (floats) of every parameter in the flat ravel_pytree blob (flax paths sorted at every level, bias before
// kernel): EGNN_0/{k}/{Dense_0, Dense_1, phi_e/Dense_l, phi_h/Dense_l, phi_x_torso/Dense_l}, EGNN_0/Dense_k,
// EGNN_0/final_scaling, Embed_0/embedding (the same walk as ecnf_create)
struct BlockOff {
  long xb, xk, gb, gk, eb[4], ek[4], hb[5], hk[5], tb[4], tk[4], nb, nk;
};
struct ParamOff {
  std::vector<BlockOff> blk;
  long fs, emb, total;
};

ParamOff param_offsets(const ecnf_cfg& c) {
  const long H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width, L = c.mlp_depth, K = c.n_blocks;
  ParamOff o;
  o.blk.resize(K);
  long p = 0;
  auto take = [&](long n) {
    const long q = p;
    p += n;
    return q;
  };
  for (int k = 0; k < K; ++k) {
    BlockOff& b = o.blk[k];
    b.xb = take(1); b.xk = take(M);
    b.gb = take(1); b.gk = take(M);
    for (int l = 0; l < L; ++l) { b.eb[l] = take(M); b.ek[l] = take((l == 0 ? 2 * H + 1 : M) * M); }
    for (int l = 0; l <= L; ++l) {
      const long out_f = l == L ? H : M, in_f = l == 0 ? M + H : M;
      b.hb[l] = take(out_f); b.hk[l] = take(in_f * out_f);
    }
    for (int l = 0; l < L; ++l) { b.tb[l] = take(M); b.tk[l] = take(M * M); }
  }
  for (int k = 0; k < K; ++k) { o.blk[k].nb = take(H); o.blk[k].nk = take((H + T) * H); }
  o.fs = take(1);
  o.emb = take((long)c.n_features * H);
  o.total = p;
  return o;
}

int fail(int code, const std::string& msg) { return ecnf::set_error(code, msg.c_str()); }

#define TR_TRY(expr)                                                                                          \
  do {                                                                                                        \
    hipError_t e_ = (expr);                                                                                   \
    if (e_ != hipSuccess) return fail(ECNF_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
  } while (0)

}  // namespace

struct ecnf_trainer {
  ecnf_cfg cfg;
  int device;
  int max_batch;
  ParamOff off;
  float freqs[8];
  float* arena;
  size_t arena_floats;
  // views into the arena (sized for max_batch)
  float *ut, *mean, *temb, *part_loss, *part_dfs, *dxa, *dxb, *norm_part;
  std::vector<float*> xc, hin, h1, Ps, Pr, r, len, px, gate, hcat;   // [K] (xc: [K + 1])
  std::vector<float*> ze, ae, zx, ax, zh, ah;                        // [K * L], [K * (L + 1)]
  float *dA, *dB, *dm_gate, *de, *dpx, *dr, *dPs, *dPr, *dhcat, *dh1, *dhin, *dhA, *dhB, *dhn, *red;
  size_t red_floats;   // partial arena of the deferred split reductions (in use)
  size_t red_capacity; // allocated floats of red
  size_t red_min;      // the embedding gradient's row-chunk partials
};

namespace {

struct Launcher {
  hipStream_t s;
  const ecnf_trainer* tr;
  hipError_t err = hipSuccess;

  void check() {
    if (err == hipSuccess) err = hipGetLastError();
  }
  static unsigned nblk(long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

  // C = op(A) op(B) (+ bias) (+ R) (+ C) (* silu'(Zs)); Aout = silu(C)
  void gemm(bool ta, bool tb, int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C,
            long ldc, const float* bias = nullptr, const float* R = nullptr, long ldr = 0, const float* Zs = nullptr,
            long ldz = 0, float* Aout = nullptr, long ldo = 0, int accumulate = 0) {
    GemmArgs g{M, N, K, A, lda, B, ldb, C, ldc, 1.0f, bias, R, ldr, Zs, ldz, Aout, ldo, accumulate, 1, 0,
               nullptr, nullptr, 0};
    dim3 grid(nblk(N, GT), nblk(M, GT), 1);
    launch(ta, tb, g, grid);
  }
  // deferred split reductions (reduce_batched)
  std::vector<RedEntry> pending;
  size_t red_used = 0;   // floats of tr->red in use by pending partials

  // every caller asks for at most tr->red_floats (gemm_wgrad sizes S to it; the embedding partials are part of the
  // arena's minimum), so after a flush the request fits
  float* red_alloc(size_t floats) {
    if (red_used + floats > tr->red_floats) flush();
    float* p = tr->red + red_used;
    red_used += (floats + 63) & ~size_t(63);
    return p;
  }
  void defer(const float* P, int S, long n, float* dst) {
    pending.push_back(RedEntry{P, dst, S, (int)n, 0});
  }
  void flush() {
    for (size_t b = 0; b < pending.size(); b += kRedMax) {
      RedBatch rb{};
      rb.count = (int)std::min<size_t>(kRedMax, pending.size() - b);
      int blocks = 0;
      for (int k = 0; k < rb.count; ++k) {
        rb.e[k] = pending[b + k];
        rb.e[k].first = blocks;
        blocks += (int)nblk(rb.e[k].n);
      }
      hipLaunchKernelGGL(reduce_batched, dim3((unsigned)blocks), dim3(256), 0, s, rb);
      check();
    }
    pending.clear();
    red_used = 0;
  }

  // weight gradient dW[M][N] = A^T dZ over K rows and the bias gradient db[N] = sum_k dZ[k] (db may be NULL),
  // split over the K dimension into >= ~384 workgroups of >= 128 rows; the partials are reduced (in split order) by
  // the next flush().  sqA: A's entries enter squared.  ldw == N for every weight block of the flat blob.
  void gemm_wgrad(int M, int N, int K, const float* A, long lda, const float* dZ, long ldz, float* dW, long ldw,
                  float* db = nullptr, int sqA = 0) {
    const long n = (long)M * N;
    const long tiles = (long)nblk(M, GT) * nblk(N, GT);
    int S = (int)std::min<long>({128, std::max<long>(1, (384 + tiles - 1) / tiles), std::max<long>(1, K / 128)});
    while (S > 1 && (size_t)S * (n + N + 128) > tr->red_floats) --S;
    if (S == 1) {
      GemmArgs g{M, N, K, A, lda, dZ, ldz, dW, ldw, 1.0f, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, 0, 1, 0,
                 db, nullptr, sqA};
      launch(true, false, g, dim3(nblk(N, GT), nblk(M, GT), 1));
      return;
    }
    // P and Pb come from ONE reservation: a flush between two separate calls would reset the arena while P is not
    // yet deferred, and Pb (or a later partial) could then land on P's region before P is reduced
    const size_t np = ((size_t)S * n + 63) & ~size_t(63);
    float* P = red_alloc(np + (db ? (size_t)S * N : 0));
    float* Pb = db ? P + np : nullptr;
    GemmArgs g{M, N, K, A, lda, dZ, ldz, P, N, 1.0f, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, 0, S, n,
               db, Pb, sqA};
    launch(true, false, g, dim3(nblk(N, GT), nblk(M, GT), S));
    defer(P, S, n, dW);
    if (db) defer(Pb, S, N, db);
  }
  template <bool TA, bool TB>
  void launch_t(const GemmArgs& g, dim3 grid) {
    auto aligned = [](const float* p, long ld) {
      return ((reinterpret_cast<uintptr_t>(p) | (uintptr_t)(ld * 4)) & 15) == 0;
    };
    const bool kw = g.K % GK == 0;
    const bool va = kw && g.M % GT == 0 && aligned(g.A, g.lda) && !g.sqA;
    const bool vb = kw && g.N % GT == 0 && aligned(g.B, g.ldb);
    if (va && vb) hipLaunchKernelGGL((gemm_kernel<TA, TB, true, true>), grid, dim3(256), 0, s, g);
    else if (va) hipLaunchKernelGGL((gemm_kernel<TA, TB, true, false>), grid, dim3(256), 0, s, g);
    else if (vb) hipLaunchKernelGGL((gemm_kernel<TA, TB, false, true>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_kernel<TA, TB, false, false>), grid, dim3(256), 0, s, g);
  }
  void launch(bool ta, bool tb, const GemmArgs& g, dim3 grid) {
    if (g.M <= 0 || g.N <= 0) return;
    if (ta && tb) launch_t<true, true>(g, grid);
    else if (ta) launch_t<true, false>(g, grid);
    else if (tb) launch_t<false, true>(g, grid);
    else launch_t<false, false>(g, grid);
    check();
  }
};

}  // namespace

extern "C" {

int ecnf_trainer_create(const ecnf_cfg* cfg, int32_t max_batch, int device, ecnf_trainer** out) {
  size_t n = 0;
  int rc = ecnf_param_count(cfg, &n);   // validates the config
  if (rc) return rc;
  if (!out) return fail(ECNF_E_INVALID, "out is NULL");
  if (max_batch < 1) return fail(ECNF_E_INVALID, "max_batch must be >= 1");
  if (cfg->n_nodes * cfg->dim > kMaxND) return fail(ECNF_E_UNSUPPORTED, "training needs n_nodes * dim <= 256");
  const ecnf_cfg c = *cfg;
  const long B = max_batch, N = c.n_nodes, D = c.dim, H = c.hidden, T = c.time_embedding_dim, M = c.mlp_width,
             L = c.mlp_depth, K = c.n_blocks;
  const long E = N * (N - 1), BN = B * N, BE = B * E;
  ecnf_trainer* tr = new ecnf_trainer();
  tr->cfg = c;
  tr->device = device;
  tr->max_batch = max_batch;
  tr->off = param_offsets(c);
  const int half = (int)T / 2;
  const float ex = std::log(10000.0f) / (float)(half - 1);
  for (int k = 0; k < 8; ++k) tr->freqs[k] = k < half ? std::exp((float)k * -ex) : 0.f;
  // arena layout
  std::vector<std::pair<float**, long>> plan;
  auto add = [&](float** p, long nf) { plan.push_back({p, (nf + 63) & ~63L}); };
  add(&tr->ut, B * N * D); add(&tr->mean, B * D); add(&tr->temb, B * T);
  add(&tr->part_loss, B); add(&tr->part_dfs, B); add(&tr->dxa, BN * D); add(&tr->dxb, BN * D);
  add(&tr->norm_part, 2 * ((n + 255) / 256) + 64);
  tr->xc.resize(K + 1); tr->hin.resize(K); tr->h1.resize(K); tr->Ps.resize(K); tr->Pr.resize(K); tr->r.resize(K);
  tr->len.resize(K); tr->px.resize(K); tr->gate.resize(K); tr->hcat.resize(K);
  tr->ze.resize(K * L); tr->ae.resize(K * L); tr->zx.resize(K * L); tr->ax.resize(K * L);
  tr->zh.resize(K * (L + 1)); tr->ah.resize(K * (L + 1));
  for (long k = 0; k <= K; ++k) add(&tr->xc[k], BN * D);
  for (long k = 0; k < K; ++k) {
    add(&tr->hin[k], BN * (H + T)); add(&tr->h1[k], BN * H); add(&tr->Ps[k], BN * M); add(&tr->Pr[k], BN * M);
    add(&tr->r[k], BE * D); add(&tr->len[k], BE); add(&tr->px[k], BE); add(&tr->gate[k], BE);
    add(&tr->hcat[k], BN * (M + H));
    for (long l = 0; l < L; ++l) {
      add(&tr->ze[k * L + l], BE * M); add(&tr->ae[k * L + l], BE * M);
      add(&tr->zx[k * L + l], BE * M); add(&tr->ax[k * L + l], BE * M);
    }
    for (long l = 0; l <= L; ++l) {
      add(&tr->zh[k * (L + 1) + l], BN * std::max(M, H)); add(&tr->ah[k * (L + 1) + l], BN * M);
    }
  }
  add(&tr->dA, BE * M); add(&tr->dB, BE * M); add(&tr->dm_gate, BE * M); add(&tr->de, BE); add(&tr->dpx, BE);
  add(&tr->dr, BE * D); add(&tr->dPs, BN * M); add(&tr->dPr, BN * M); add(&tr->dhcat, BN * (M + H));
  add(&tr->dh1, BN * H); add(&tr->dhin, BN * (H + T)); add(&tr->dhA, BN * M); add(&tr->dhB, BN * M);
  add(&tr->dhn, BN * H);
  // partial arena of the deferred split reductions: at least 128 splits of the largest weight block and its bias
  // ((M + H) x M, (H + T) x H) and the embedding gradient's row-chunk partials; 32 M floats (128 MiB) when larger,
  // which holds a whole LJ13 step's partials in about two flushes
  tr->red_floats = (size_t)std::max<long>({128 * (std::max((M + H) * M, (H + T) * H) + std::max(M + H, H + T) + 256),
                                           ((BN + 63) / 64) * (long)c.n_features * H + 64, 32L << 20});
  add(&tr->red, (long)tr->red_floats);
  tr->red_capacity = tr->red_floats;
  tr->red_min = (size_t)(((BN + 63) / 64) * (long)c.n_features * H + 64);
  size_t total = 0;
  for (auto& q : plan) total += (size_t)q.second;
  tr->arena_floats = total;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || device < 0 || device >= ndev) {
    delete tr;
    return e != hipSuccess ? fail(ECNF_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e))
                           : fail(ECNF_E_INVALID, "device index out of range");
  }
  if ((e = hipSetDevice(device)) != hipSuccess || (e = hipMalloc(&tr->arena, total * sizeof(float))) != hipSuccess) {
    delete tr;
    return fail(ECNF_E_HIP, std::string("trainer allocation: ") + hipGetErrorString(e));
  }
  float* p = tr->arena;
  for (auto& q : plan) {
    *q.first = p;
    p += q.second;
  }
  *out = tr;
  return ECNF_OK;
}

int ecnf_trainer_destroy(ecnf_trainer* tr) {
  if (!tr) return ECNF_OK;
  TR_TRY(hipSetDevice(tr->device));
  TR_TRY(hipDeviceSynchronize());
  TR_TRY(hipFree(tr->arena));
  delete tr;
  return ECNF_OK;
}

int ecnf_trainer_set_reduction_arena(ecnf_trainer* tr, size_t floats, size_t* used) {
  if (!tr) return fail(ECNF_E_INVALID, "NULL trainer");
  tr->red_floats = floats == 0 ? tr->red_capacity : std::min(tr->red_capacity, std::max(tr->red_min, floats));
  if (used) *used = tr->red_floats;
  return ECNF_OK;
}

int ecnf_fm_loss_grad(ecnf_trainer* tr, const float* params, const float* x1, const float* x0, const float* t,
                      const int32_t* feat, float sigma_min, int32_t batch, float* loss, float* grad, void* stream) {
  if (!tr) return fail(ECNF_E_INVALID, "NULL trainer");
  if (batch < 1 || batch > tr->max_batch) return fail(ECNF_E_INVALID, "batch must be in [1, max_batch]");
  if (!params || !x1 || !x0 || !t || !feat || !loss || !grad) return fail(ECNF_E_INVALID, "NULL argument");
  const ecnf_cfg& c = tr->cfg;
  Geom G{batch, c.n_nodes, c.dim, c.hidden, c.time_embedding_dim, c.mlp_width, c.mlp_depth, c.n_blocks,
         c.n_nodes * (c.n_nodes - 1), c.n_features, c.normalization_constant, sigma_min};
  const long B = batch, N = G.N, D = G.D, H = G.H, T = G.T, M = G.M, L = G.L, K = G.K;
  const long BN = B * N, BE = B * G.E, ND = N * D;
  const ParamOff& o = tr->off;
  const float* P = params;
  float* dP = grad;
  TR_TRY(hipSetDevice(tr->device));
  hipStream_t s = (hipStream_t)stream;
  Launcher Lc{s, tr};
  auto nb = [](long n) { return Launcher::nblk(n); };
  TR_TRY(hipMemsetAsync(grad, 0, (size_t)o.total * sizeof(float), s));
  Freqs fq;
  std::memcpy(fq.f, tr->freqs, sizeof(fq.f));

  // ------------------------------------------------------------------ forward
  hipLaunchKernelGGL(k_prologue, dim3((unsigned)B), dim3(64), 0, s, G, x1, x0, t, fq, tr->ut, tr->mean, tr->xc[0],
                     tr->temb);
  Lc.check();
  for (long k = 0; k < K; ++k) {
    const BlockOff& bo = o.blk[k];
    // hin = [h | temb]; h1 = hin Wn + bn  (egnn.py:166-167)
    if (k == 0)
      hipLaunchKernelGGL(k_hin, dim3(nb(BN * (H + T))), dim3(256), 0, s, G, (const float*)nullptr, 0L, feat,
                         P + o.emb, (const float*)tr->temb, tr->hin[0]);
    else
      hipLaunchKernelGGL(k_hin, dim3(nb(BN * (H + T))), dim3(256), 0, s, G, (const float*)tr->zh[(k - 1) * (L + 1) + L],
                         H, (const int32_t*)nullptr, (const float*)nullptr, (const float*)tr->temb, tr->hin[k]);
    Lc.check();
    Lc.gemm(false, false, (int)BN, (int)H, (int)(H + T), tr->hin[k], H + T, P + bo.nk, H, tr->h1[k], H, P + bo.nb);
    // per-node halves of phi_e layer 1: P_s = h1 W[0:H], P_r = h1 W[H:2H]
    Lc.gemm(false, false, (int)BN, (int)M, (int)H, tr->h1[k], H, P + bo.ek[0], M, tr->Ps[k], M);
    Lc.gemm(false, false, (int)BN, (int)M, (int)H, tr->h1[k], H, P + bo.ek[0] + H * M, M, tr->Pr[k], M);
    hipLaunchKernelGGL(k_edge_geom, dim3(nb(BE)), dim3(256), 0, s, G, (const float*)tr->xc[k], tr->r[k], tr->len[k]);
    Lc.check();
    hipLaunchKernelGGL(k_layer1, dim3(nb(BE * M)), dim3(256), 0, s, G, (const float*)tr->Ps[k],
                       (const float*)tr->Pr[k], (const float*)tr->len[k], P + bo.ek[0] + 2 * H * M, P + bo.eb[0],
                       tr->ze[k * L], tr->ae[k * L]);
    Lc.check();
    for (long l = 1; l < L; ++l)   // phi_e layers 2..L (egnn.py:79, SiLU after every layer)
      Lc.gemm(false, false, (int)BE, (int)M, (int)M, tr->ae[k * L + l - 1], M, P + bo.ek[l], M, tr->ze[k * L + l], M,
              P + bo.eb[l], nullptr, 0, nullptr, 0, tr->ae[k * L + l], M);
    const float* m = tr->ae[k * L + L - 1];
    for (long l = 0; l < L; ++l)   // phi_x torso (egnn.py:82)
      Lc.gemm(false, false, (int)BE, (int)M, (int)M, l == 0 ? m : tr->ax[k * L + l - 1], M, P + bo.tk[l], M,
              tr->zx[k * L + l], M, P + bo.tb[l], nullptr, 0, nullptr, 0, tr->ax[k * L + l], M);
    // px and the gate (the gate only feeds h: skipped in the last block, whose h nothing reads)
    const bool need_h = k + 1 < K;
    hipLaunchKernelGGL(k_edge_dots, dim3((unsigned)((BE + 3) / 4)), dim3(256), 0, s, G,
                       (const float*)tr->ax[k * L + L - 1], P + bo.xk, P + bo.xb, m, P + bo.gk, P + bo.gb, tr->px[k],
                       need_h ? tr->gate[k] : (float*)nullptr);
    Lc.check();
    hipLaunchKernelGGL(k_node_shift, dim3(nb(BN * D)), dim3(256), 0, s, G, (const float*)tr->xc[k],
                       (const float*)tr->px[k], (const float*)tr->r[k], (const float*)tr->len[k], tr->xc[k + 1]);
    Lc.check();
    if (need_h) {
      hipLaunchKernelGGL(k_node_agg, dim3(nb(BN * (M + H))), dim3(256), 0, s, G, m, (const float*)tr->gate[k],
                         (const float*)tr->h1[k], tr->hcat[k]);
      Lc.check();
      // phi_h = MLP((M,) * L + (H,)) on [m_i | h1], residual h1 (egnn.py:105-111)
      for (long l = 0; l <= L; ++l) {
        const int in_f = (int)(l == 0 ? M + H : M), out_f = (int)(l == L ? H : M);
        const float* X = l == 0 ? tr->hcat[k] : tr->ah[k * (L + 1) + l - 1];
        Lc.gemm(false, false, (int)BN, out_f, in_f, X, in_f, P + bo.hk[l], out_f, tr->zh[k * (L + 1) + l], out_f,
                P + bo.hb[l], l == L ? tr->h1[k] : nullptr, H, nullptr, 0,
                l == L ? nullptr : tr->ah[k * (L + 1) + l], out_f);
      }
    }
  }
  hipLaunchKernelGGL(k_output, dim3((unsigned)B), dim3(64), 0, s, G, (const float*)tr->xc[K], (const float*)tr->xc[0],
                     (const float*)tr->mean, (const float*)tr->ut, P + o.fs, tr->dxa, tr->part_loss, tr->part_dfs);
  Lc.check();
  hipLaunchKernelGGL(k_finish_loss, dim3(1), dim3(64), 0, s, (int)B, 1.0f / (float)(B * ND),
                     (const float*)tr->part_loss, (const float*)tr->part_dfs, loss, dP + o.fs);
  Lc.check();

  // ------------------------------------------------------------------ backward
  float* dx = tr->dxa;      // d loss / d x_{k+1}
  float* dxn = tr->dxb;
  const float* dh_next = nullptr;   // d loss / d h_new of block k (nullptr: zero, the last block)
  for (long k = K - 1; k >= 0; --k) {
    const BlockOff& bo = o.blk[k];
    const bool need_h = k + 1 < K;
    const float* m = tr->ae[k * L + L - 1];
    // dh1 starts from the residual of phi_h (h_new = phi_h(hcat) + h1)
    if (need_h) {
      // phi_h backward: dZ_L = dh_new (no final activation)
      const float* dZ = dh_next;
      float* bufs[2] = {tr->dhA, tr->dhB};
      for (long l = L; l >= 0; --l) {
        const int in_f = (int)(l == 0 ? M + H : M), out_f = (int)(l == L ? H : M);
        const float* X = l == 0 ? tr->hcat[k] : tr->ah[k * (L + 1) + l - 1];
        Lc.gemm_wgrad(in_f, out_f, (int)BN, X, in_f, dZ, out_f, dP + bo.hk[l], out_f, dP + bo.hb[l]);
        if (l > 0) {
          float* dZp = bufs[l & 1];
          Lc.gemm(false, true, (int)BN, (int)M, out_f, dZ, out_f, P + bo.hk[l], out_f, dZp, M, nullptr, nullptr, 0,
                  tr->zh[k * (L + 1) + l - 1], M);
          dZ = dZp;
        } else {
          Lc.gemm(false, true, (int)BN, (int)(M + H), (int)M, dZ, M, P + bo.hk[0], M, tr->dhcat, M + H);
        }
      }
      // dh1 = dh_new (the residual) + dhcat[:, M:] (phi_h's input h1)
      hipLaunchKernelGGL(k_copy_add, dim3(nb(BN * H)), dim3(256), 0, s, BN, (int)H, dh_next, H,
                         (const float*)(tr->dhcat + M), M + H, tr->dh1, H);
      Lc.check();
    }
    // shifts: dpx, dr (egnn.py:87-95) and the phi_x torso's last dZ = dpx w_x silu'(z)
    hipLaunchKernelGGL(k_shift_bwd, dim3(nb(BE * M)), dim3(256), 0, s, G, (const float*)dx, (const float*)tr->px[k],
                       (const float*)tr->r[k], (const float*)tr->len[k], P + bo.xk,
                       (const float*)tr->zx[k * L + L - 1], tr->dpx, tr->dr, tr->dA);
    Lc.check();
    // phi_x output Dense(1): dw_x = a_x[L-1]^T dpx, db_x = sum dpx
    Lc.gemm_wgrad((int)M, 1, (int)BE, tr->ax[k * L + L - 1], M, tr->dpx, 1, dP + bo.xk, 1, dP + bo.xb);
    // gate path (egnn.py:99-104) into dm_gate, its weights
    if (need_h) {
      hipLaunchKernelGGL(k_gate_bwd, dim3((unsigned)((BE + 3) / 4)), dim3(256), 0, s, G, m,
                         (const float*)tr->gate[k], (const float*)tr->dhcat, P + bo.gk, tr->dm_gate, tr->de);
      Lc.check();
      Lc.gemm_wgrad((int)M, 1, (int)BE, m, M, tr->de, 1, dP + bo.gk, 1, dP + bo.gb);
    }
    // phi_x torso backward: layers L-1 .. 0; the input of layer 0 is m
    float* dZ = tr->dA;
    float* other = tr->dB;
    for (long l = L - 1; l >= 0; --l) {
      const float* X = l == 0 ? m : tr->ax[k * L + l - 1];
      Lc.gemm_wgrad((int)M, (int)M, (int)BE, X, M, dZ, M, dP + bo.tk[l], M, dP + bo.tb[l]);
      if (l > 0) {
        Lc.gemm(false, true, (int)BE, (int)M, (int)M, dZ, M, P + bo.tk[l], M, other, M, nullptr, nullptr, 0,
                tr->zx[k * L + l - 1], M);
      } else {
        // d m = dZ_0 W_0^T (+ the gate path), times silu'(z_e[L-1]): the phi_e output layer's dZ
        Lc.gemm(false, true, (int)BE, (int)M, (int)M, dZ, M, P + bo.tk[0], M, other, M, nullptr,
                need_h ? tr->dm_gate : nullptr, M, tr->ze[k * L + L - 1], M);
      }
      std::swap(dZ, other);
    }
    // phi_e backward: layers L-1 .. 1 (layer 0 is the factorised layer 1)
    for (long l = L - 1; l >= 1; --l) {
      Lc.gemm_wgrad((int)M, (int)M, (int)BE, tr->ae[k * L + l - 1], M, dZ, M, dP + bo.ek[l], M, dP + bo.eb[l]);
      Lc.gemm(false, true, (int)BE, (int)M, (int)M, dZ, M, P + bo.ek[l], M, other, M, nullptr, nullptr, 0,
              tr->ze[k * L + l - 1], M);
      std::swap(dZ, other);
    }
    // layer 1: dz1 = dZ.  dw_d = |r|^2 . dz1, db, node halves, |r|^2 -> dr
    {
      // dw_d = (|r|^2)^T dz1 (the lengths squared as they are loaded)
      Lc.gemm_wgrad(1, (int)M, (int)BE, tr->len[k], 1, dZ, M, dP + bo.ek[0] + 2 * H * M, M, dP + bo.eb[0], 1);
      hipLaunchKernelGGL(k_layer1_node_bwd, dim3(nb(BN * M)), dim3(256), 0, s, G, (const float*)dZ, tr->dPs,
                         tr->dPr);
      Lc.check();
      hipLaunchKernelGGL(k_layer1_edge_bwd, dim3((unsigned)((BE + 3) / 4)), dim3(256), 0, s, G, (const float*)dZ,
                         P + bo.ek[0] + 2 * H * M, (const float*)tr->r[k], tr->dr);
      Lc.check();
      Lc.gemm_wgrad((int)H, (int)M, (int)BN, tr->h1[k], H, tr->dPs, M, dP + bo.ek[0], M);
      Lc.gemm_wgrad((int)H, (int)M, (int)BN, tr->h1[k], H, tr->dPr, M, dP + bo.ek[0] + H * M, M);
      // dh1 (+)= dP_s W_s^T + dP_r W_r^T
      Lc.gemm(false, true, (int)BN, (int)H, (int)M, tr->dPs, M, P + bo.ek[0], M, tr->dh1, H, nullptr, nullptr, 0,
              nullptr, 0, nullptr, 0, need_h ? 1 : 0);
      Lc.gemm(false, true, (int)BN, (int)H, (int)M, tr->dPr, M, P + bo.ek[0] + H * M, M, tr->dh1, H, nullptr, nullptr,
              0, nullptr, 0, nullptr, 0, 1);
    }
    // positions: dx_k = dx_{k+1} + receiver sums - sender sums of dr
    hipLaunchKernelGGL(k_dx_bwd, dim3(nb(BN * D)), dim3(256), 0, s, G, (const float*)dx, (const float*)tr->dr, dxn);
    Lc.check();
    std::swap(dx, dxn);
    // node Dense: dWn = hin^T dh1, dbn, dhin = dh1 Wn^T
    Lc.gemm_wgrad((int)(H + T), (int)H, (int)BN, tr->hin[k], H + T, tr->dh1, H, dP + bo.nk, H, dP + bo.nb);
    Lc.gemm(false, true, (int)BN, (int)(H + T), (int)H, tr->dh1, H, P + bo.nk, H, tr->dhin, H + T);
    dh_next = nullptr;
    if (k > 0) {
      // the previous block's h_new gradient: dhin[:, :H] (the temb columns carry no parameters), compacted
      hipLaunchKernelGGL(k_copy_add, dim3(nb(BN * H)), dim3(256), 0, s, BN, (int)H, (const float*)tr->dhin, H + T,
                         (const float*)nullptr, 0L, tr->dhn, H);
      Lc.check();
      dh_next = tr->dhn;
    }
  }
  {
    const unsigned chunks = (unsigned)((BN + 63) / 64), hc = (unsigned)((H + 63) / 64);
    const long ne = (long)G.nfeat * H;
    float* part = Lc.red_alloc((size_t)chunks * ne);
    hipLaunchKernelGGL(k_embed_bwd, dim3((unsigned)G.nfeat * hc, chunks), dim3(256), 0, s, G, (const float*)tr->dhin,
                       H + T, feat, part);
    Lc.check();
    Lc.defer(part, (int)chunks, ne, dP + o.emb);
  }
  Lc.flush();
  if (Lc.err != hipSuccess) return fail(ECNF_E_HIP, std::string("training step launch: ") + hipGetErrorString(Lc.err));
  return ECNF_OK;
}

int ecnf_adam_update(ecnf_trainer* tr, const float* grad, float* params, float* mu, float* nu, float* ema, size_t n,
                     const ecnf_adam_opts* o, float* norms, void* stream) {
  if (!tr || !o) return fail(ECNF_E_INVALID, "NULL trainer/options");
  if ((long)n != tr->off.total) return fail(ECNF_E_INVALID, "n must be the trainer's parameter count");
  if (!grad || !params || !mu || !nu) return fail(ECNF_E_INVALID, "NULL argument");
  if (o->count < 1) return fail(ECNF_E_INVALID, "count (the step number after this update) must be >= 1");
  TR_TRY(hipSetDevice(tr->device));
  hipStream_t s = (hipStream_t)stream;
  const unsigned nbk = (unsigned)((n + 255) / 256);
  const float bc1 = 1.0f - std::pow(o->b1, (float)o->count), bc2 = 1.0f - std::pow(o->b2, (float)o->count);
  hipLaunchKernelGGL(k_adam, dim3(nbk), dim3(256), 0, s, (long)n, grad, params, mu, nu, ema, o->lr, o->b1, o->b2,
                     o->eps, o->eps_root, bc1, bc2, o->ema_beta, tr->norm_part);
  TR_TRY(hipGetLastError());
  if (norms) {
    hipLaunchKernelGGL(k_norms, dim3(1), dim3(256), 0, s, (int)nbk, (const float*)tr->norm_part, norms);
    TR_TRY(hipGetLastError());
  }
  return ECNF_OK;
}

}  // extern "C"
