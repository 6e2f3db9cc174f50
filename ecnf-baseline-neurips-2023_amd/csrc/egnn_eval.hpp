// egnn_eval.hpp — one EGNN vector-field evaluation for the MPW molecules of a workgroup (gfx950 / CDNA4).
//
// Restates FlatEgnn.__call__ (ecnf/cnf/build_cnf.py:68-93), EGNN.call_single (ecnf/nets/egnn.py:144-190)
// and EGCL.__call__ (ecnf/nets/egnn.py:49-114) of the reference, with forward-mode tangents (NT = 1) for the
// divergence terms of ecnf/cnf/sample_and_log_prob.py:57-78.
//
// Layout (per workgroup = Geo<NF, NT>::NW waves, MPW molecules):
//   * node rows: molecule m, atom i -> row n = m*N + i, padded to RP = 32*ceil(MPW*N/32); tangent row of n is
//     RP + n.  All node state lives in LDS as [row][feature] with odd leading dimensions (conflict-free
//     column reads by 32 lanes).
//   * node GEMMs (Dense layers on node rows) run on v_mfma_f32_32x32x2_f32 in transposed form
//     Y^T[j][n] = sum_k W[k][j] X^T[k][n]: A = weights (global, L2-resident), B = node rows (LDS), one output
//     32x32 tile per (32-output block, 32-node tile); the tangent tile shares every A fragment.
//   * edge MLPs: edge e (receiver-major, graph.py:6-14) of a molecule sits on MFMA column (lane & 31) of a
//     32-edge tile; a molecule owns EP = 32*ceil(N*SR/32) edge slots starting on a tile boundary (SR = N-1 slots
//     per receiver for N <= 33; for 33 < N <= 64 every receiver run is padded to SR = 64 slots, two whole tiles).  A whole tile's activation is 16*M/32 registers per lane
//     and the MFMA accumulator of layer l IS the B operand of layer l+1 (register r of output block fb is the
//     k-step (fb, r)), so phi_e layers 2..L and all phi_x layers chain with zero LDS traffic; weights are
//     pre-packed on the host into lane order (one dwordx4 per lane = 4 A fragments).
//   * phi_e layer 1 is factorised: [h_s | h_r | d^2] W = (h W_s)[s] + (h W_r + b)[r] + d^2 w_d; the per-node
//     halves are one node GEMM into LDS and are gathered per edge.
//   * segment sums (e3nn.scatter_sum over the contiguous receiver runs) are segmented prefix scans in DPP
//     (row_shr / row_bcast:15) inside each 32-edge tile followed by one LDS add per (segment, tile); a node's
//     edges touch at most two tiles (N-1 <= 32 packed, or SR = 64 receiver-tiled) and 0 + a + b == 0 + b + a, so the
//     result is run-to-run deterministic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace ecnf {

constexpr int kSimds = 4;   // SIMDs per CU
// Edge-chain arithmetic: the primal and tangent kernels of the default precision run their chains on the 16-bit
// matrix cores with fp32-accurate operand splitting (chain_split.hpp); the strict-fp32 kernels (P = 1) on
// v_mfma_f32_32x32x2_f32.
constexpr bool kSplitChain = true;
// Waves per workgroup.  Split primal kernels: 8 waves = 2 per SIMD (<= 256 registers each): one wave's VALU and
// LDS phases (activations, gate / aggregation scans, layer-1 gathers) overlap the other wave's MFMA chain
// (measured 31.5 -> 28.6 ms at LJ13 over 4 waves with 512 registers).  fp32-MFMA chain, primal, M <= 128: 8 waves.
// Tangent kernels and the split M = 256 chain (QM9: 3 x 128 registers of split input / output / accumulators per
// tile) need up to 512 registers: 4 waves, 1 per SIMD (QM9 B = 2048 Euler-100: fp32 MFMA 7203 ms -> split 2271 ms).
constexpr bool kSplitTanChain = kSplitChain;
constexpr int kSplitMaxNF = 8;   // split chain up to M = 32 kSplitMaxNF
// k-steps of node-GEMM A fragments in flight (node_task_split; Geo::kNodePFA).  Measured: depth 2 / 4 / 6 of the M = 256
// kernels 311 / 314 / 322 us per QM9 cols evaluation (profiles/round4/r4w); LJ13 2 / 4 / 6 within noise (r4k)
constexpr int kNodePFADefault = 2;
// Tangent kernels' node GEMMs (node Dense, the phi_e.0 halves, phi_h) on the split path (M <= 128)
constexpr bool kSplitTanNode = true;
// P: GEMM arithmetic of the kernel.  P = 0 (ECNF_PREC_SPLIT_F16, the default) as described above; P = 1
// (ECNF_PREC_FP32, ecnf_set_precision) every GEMM on v_mfma_f32_32x32x2_f32 with fp32 operands: the strict-fp32
// comparator and the fallback for molecules whose activations leave the fp16 range (ECNF_E_NONFINITE).
// BN ("big N"): the M = 128 tangent kernels in the wide form (kWideT / kWideT32: per-edge phi_e.0, no P rows) for
// molecules of 34 .. 64 atoms, whose P rows (primal + tangent) do not fit the LDS beside the rest.
template <int NF, int NT, int P = 0, bool BN = false>
struct Geo {
  static_assert(!BN || (NT == 1 && NF == 4), "the big-N form is an M = 128 tangent kernel");
  static constexpr bool kSplit = kSplitChain && P == 0 && NT == 0 && NF <= kSplitMaxNF;
  // tangent kernels: the edge chains run split (chain_split_tangent); node GEMMs, layer 1 and the tail stay fp32
  static constexpr bool kSplitT = kSplitTanChain && P == 0 && NT == 1 && NF <= 4 && !BN;
  // node GEMMs on the split path with 16-B node-row strides: the split primal kernels and (kSplitTanNode) the
  // M <= 128 tangent kernels (log2-domain P via the primal Wp_s; tangent rows share every A fragment).  (The padded
  // 16-B strides fit ALDP's M = 64 tangent kernel at 2 molecules per workgroup only since the x_c0 copy left LDS
  // and vecs is sized by L: before, split node GEMMs dropped it to 1, 55.9 -> 62.0 ms.)
  // M = 256 tangent kernels (QM9), and the big-N M = 128 ones: per-edge phi_e.0 (no P buffer), sequential primal /
  // tangent split chains (chain_dual_seq), phi_h in place on macc
  static constexpr bool kWideT = kSplitTanChain && P == 0 && NT == 1 && (NF == 8 || BN);
  // M = 256 strict-fp32 tangent kernels (P = 1): kWideT's structure on v_mfma_f32_32x32x2_f32 (per-edge phi_e.0
  // from the fp32 kernel rows, sequential primal / tangent chain passes, in-place phi_h): the fallback for QM9
  // divergence solves whose activations leave the fp16 range and for checkpoints with edge weights >= 2^15
  static constexpr bool kWideT32 = P == 1 && NT == 1 && (NF == 8 || BN);
  static constexpr bool kNoP = kWideT || kWideT32;   // no per-node phi_e.0 halves (P rows) in LDS
  static constexpr bool kSplitN = kSplit || (kSplitTanNode && kSplitT) || kWideT;
  // M <= 128 split tangent kernels: P (primal and tangent rows) in the log2 domain (the primal kernels' -log2(e)
  // fragments), phi_e.0's SiLU and its tangent evaluated there and split straight into the chain's input buffers
  static constexpr bool kL2T = kSplitT && kSplitN;
  // M <= 128 primal kernels: 8 waves (2 per SIMD, 256 registers: one wave's VALU / LDS phases beside the other's chain,
  // 31.5 -> 28.6 ms at LJ13 over 4 waves with 512 registers; two 4-wave workgroups per CU measured 29.4 ms).
  // M = 64 tangent kernels (ALDP): 8 waves too, so one wave's VALU phases (layer-1 assembly, gate / aggregation
  // scans, shifts: twice the VALU per MFMA of M = 128) overlap the other's chain (ALDP B = 512 PID Hutchinson log_prob
  // 61.8 -> 50.2 ms, outputs bitwise equal).  The M = 128 tangent kernels (1.2 KB per lane of spills at 256
  // registers) and the M = 256 kernels (968 B per lane at 2 waves per SIMD; QM9 2162 -> 3423 ms) run 4 waves.
  static constexpr int NW = (NT == 0 && NF <= 4) ? 8 : (NT == 1 && P == 0 && NF <= 2 ? 8 : 4);
  static constexpr int NTHR = 64 * NW;
  // minimum waves per SIMD the register allocation must allow (the 8-wave tangent kernels: 256 registers)
  static constexpr int WPE = (NT == 1 && NW == 8) ? 2 : 1;
  // k-steps of node-GEMM A fragments in flight (node_task_split)
  static constexpr int kNodePFA = kNodePFADefault;
};
// waves of the column-split team kernel (M = 256 split primal): 8, one output block of each chain layer per wave, two
// waves per SIMD to hide the fragment stream (QM9 B = 1 Euler-20: 456 -> 311 us per evaluation, bitwise equal;
// profiles/round4/r4q).  The batch-path and tile-dealt M = 256 kernels stay at 4 waves: at 8 they spill 828 B per
// lane (2283 -> 2587 us per evaluation).
constexpr int kColsNW = 8;
// waves / threads per workgroup of a kernel: Geo's, or kColsNW for the column-split team kernel
template <int NF, int NT, int P, bool COLS>
constexpr int kernel_waves() { return COLS ? kColsNW : Geo<NF, NT, P>::NW; }
template <int NF, int NT, int P, bool COLS>
constexpr int kernel_threads() { return 64 * kernel_waves<NF, NT, P, COLS>(); }
constexpr int kMaxBlocks = 10;
constexpr int kMaxPhiH = 5;     // L + 1 <= 5
constexpr int kMaxHalfT = 8;    // T <= 16
constexpr int kMaxTilesPerMol = 32;   // EP / 32 for N <= 33

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// compile-time loop: f(std::integral_constant<int, i>) for i = 0..N-1, always fully expanded (a long unrolled
// loop that the optimiser only partially unrolls turns ring-buffer register indices dynamic -> scratch)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// global (address space 1) views of the weight buffers: global_load_* with counted vmcnt waits instead of flat
// loads, which hipcc must fence with vmcnt(0) lgkmcnt(0)
#define ECNF_GLOBAL __attribute__((address_space(1)))
typedef const ECNF_GLOBAL float* gfloat_p;
typedef const ECNF_GLOBAL f32x4* gf32x4_p;
__device__ __forceinline__ gfloat_p gptr(const float* p) { return (gfloat_p)(p); }
__device__ __forceinline__ gf32x4_p gptr4(const float* p) { return (gf32x4_p)(p); }

struct BlockW {
  const float* Wn;  const float* bn;    // node Dense [(H+T)][H], [H]           (egnn.py:166-167)
  const float* Wp;  const float* bp;    // [H][2M] = [W_send | W_recv] of phi_e.0, bias [2M] = [0 | b]
  const float* wd;                      // [M]  phi_e.0 kernel row 2H (the |r|^2 feature)
  const float* We;  const float* be;    // packed chain weights: phi_e.1..L-1 then phi_x.0..L-1, biases [(2L-1)][M]
  const unsigned* Ws;                   // the same chain as split-bf16 fragments (chain_split.hpp)
  const float* wx;  const float* wg;    // [M] phi_x output Dense(1) kernel, [M] gate Dense(1) kernel
  float bx, bg;                         // their biases
  const float* Wh[kMaxPhiH]; const float* bh[kMaxPhiH];  // phi_h layers, row-major [in][out]
  // split node GEMM fragments [out block][16-deep k-step][piece][lane] (node_task_split)
  const unsigned* Wn_s; const unsigned* Wp_s; const unsigned* Wh_s[kMaxPhiH];
  // log2-domain copies for the split kernels (chain_split.hpp, silu_u): -log2(e) x {phi_e.0 Wp (in Wp_s), bp, w_d,
  // chain biases}, -ln 2 x {w_g, w_x}
  const float* bp_u; const float* wd_u; const float* be_u; const float* wg_u; const float* wx_u;
  // 1 / the power-of-two scale of each split weight matrix (chain_split.hpp): chain layers, Wn, Wp, phi_h
  float cinv[2 * 4 - 1];
  float ninv, pinv, hinv[kMaxPhiH];
  // natural-domain split fragments of phi_h.0 for the tangent kernels (the primal copy above carries the message
  // scale -ln2 / sqrt(N-1)), with its 1 / scale
  const unsigned* Wh_sn0;
  float hinv_n0;
  // M = 256 tangent kernels: phi_e.0 kernel [(2H+1)][M] x -log2(e) as split node fragments (edge_layer1_dual)
  const unsigned* W1_s;
  float w1inv;
  // the divergence kernels' chain: every chain layer scaled by a power of two and split into THREE fp16 pieces that
  // hold the fp32 weight exactly (chain_split WP = 3); 1 / the scales are cinv (the 2-piece chain Ws is unscaled and
  // ignores them with ECNF_CHAIN_BIAS_INIT, and uses the same scales without it)
  const unsigned* Ws3;
};

struct Net {
  int N, D, H, T, M, L, K, nfeat;
  int E;          // N (N - 1)
  int SR;         // edge slots per receiver: N - 1 (receiver runs packed back to back, N <= 33), or 64 (N > 33:
                  // receiver-tiled, every run starts on a tile boundary and spans exactly two tiles)
  int EP;         // edge slots per molecule (N SR) padded to a multiple of 32 (every molecule starts on a tile boundary)
  int MPW;        // molecules per workgroup
  int lds_floats; // dynamic LDS of one workgroup (device-checked build: ECNF_DCHECK bit 0)
  int xs_floats;  // column-split team mode (edge_tile_cols): floats of the layer-exchange image (0 otherwise)
  int RP;         // padded primal node rows
  int ND;         // N * D
  float C;        // EGCL normalization constant
  float fs;       // EGNN final_scaling
  float nn1;      // avg_num_neighbours = N - 1
  float sqrt_nn1; // sqrt(N - 1) in fp32
  int cross;      // split kernels: message segment parts are stored, not atomically added (Lds::cross)
  int wide;       // M = 128 tangent kernels in the wide form (Geo BN: per-edge phi_e.0, no P rows; 34 .. 64 atoms)
  int ncross;     // receiver segments per molecule that cross a tile boundary (split kernels with cross)
  int pairs;      // block-1 pair tiles (PairPlan13: one node feature, N = 13, the M = 128 split primal kernels)
  unsigned char xs_i[kMaxTilesPerMol];   // ... their receiver atom i
  unsigned char xs_t[kMaxTilesPerMol];   // ... and the molecule tile that holds their continuation part
  float freqs[kMaxHalfT];
  const float* emb;
  BlockW blk[kMaxBlocks];
};

// ---------------------------------------------------------------------------------------------------
// diagnostic phase stamps (separate build, -DECNF_STAMPS): thread 0 of every workgroup adds the shader-clock
// cycles of each barrier-delimited phase into LDS slots; the kernel flushes them to g_stamps at exit.
// Never compiled into the product library.
// ---------------------------------------------------------------------------------------------------
enum StampSlot {
  kStPrologue = 0, kStNodeDense, kStPGemm, kStEdge, kStNodeUpd, kStPhiH, kStEpilogue, kStSolver,
  kStEdgeChainE, kStEdgeTail, kStEdgeLayer1, kStEdgeAgg, kStEdgePhiXIn, kStEdgePhiX, kStTeam, kStCount
};
#ifdef ECNF_STAMPS
__device__ unsigned long long g_stamps[32];
#define ECNF_STAMP_DECL unsigned long long* stamps;
#define STAMP(s, slot)                                                    \
  do {                                                                    \
    if (threadIdx.x == 0) {                                               \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
      (s).stamps[slot] += t_ - (s).stamps[31];                            \
      (s).stamps[31] = t_;                                                \
    }                                                                     \
  } while (0)
#define STAMP_LANE0(s, slot, t0)                                          \
  do {                                                                    \
    if (threadIdx.x == 0) {                                               \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
      (s).stamps[slot] += t_ - (t0);                                      \
      (t0) = t_;                                                          \
    }                                                                     \
  } while (0)
#else
#define ECNF_STAMP_DECL
#define STAMP(s, slot) do {} while (0)
#define STAMP_LANE0(s, slot, t0) do {} while (0)
#endif

// ---------------------------------------------------------------------------------------------------
// device-side bounds checks (separate diagnostic build, -DECNF_DEVICE_CHECKS): a failed check
// ORs its bit into g_checks (one word per lane, vector atomics) and the kernel carries on; ecnf_debug_checks() reads
// and clears the words.  Never compiled into the product library.
//   bit 0  LDS carve-up + solver state past the launch's dynamic LDS      bit 1  edge receiver / sender row out of range
//   bit 2  edge tile past the workgroup's tiles                           bit 3  node-GEMM row tile past RP
//   bit 4  stored segment part (cross row) out of range                    bit 5  molecule slot past the workgroup
//   bit 6  exact-trace primal-cache slot past the caller's workspace (SolveP::pcache_slots)
// ---------------------------------------------------------------------------------------------------
#ifdef ECNF_DEVICE_CHECKS
__device__ unsigned g_checks[64];
#define ECNF_DCHECK(cond, bit)                                                                           \
  do {                                                                                                   \
    if (!(cond)) __hip_atomic_fetch_or(&g_checks[threadIdx.x & 63], 1u << (bit), __ATOMIC_RELAXED,       \
                                       __HIP_MEMORY_SCOPE_AGENT);                                        \
  } while (0)
#else
#define ECNF_DCHECK(cond, bit) do {} while (0)
#endif

// ---------------------------------------------------------------------------------------------------
// LDS carve-up
// ---------------------------------------------------------------------------------------------------
struct Lds {
  float* hin;  int ld_hin;   // [R][H+T]  h (cols 0..H-1) | time embedding (cols H..H+T-1)
  float* hb;   int ld_hb;    // [R][H]    h after the per-block Dense (residual source)
  float* P;    int ld_P;     // [R][2M]   per-node phi_e.0 halves; reused as phi_h ping-pong
  float* macc; int ld_m;     // [R][M]    message aggregate
  float* xc;                 // [R][D]    centred positions, updated per block
  float* dxacc;              // [R][D]    shift aggregate
  float* mean;               // [2][MPW][D] input mean (primal, tangent)
  float* temb;               // [MPW][T]
  float* vecs;               // [(2L-1) + 3][M] this block's chain biases, w_d, w_g, w_x (staged once per block)
  int*   feat;               // [MPW][N]
  float* cross;              // [MPW][EP/32][ld_m] continuation parts of receiver segments that cross a tile
                             // boundary (aliases hin, which is dead during the edge phase; split kernels)
  float* tail;               // first free float (solver state follows)
  ECNF_STAMP_DECL
};

__host__ __device__ inline int align4(int n) { return (n + 3) & ~3; }

// Leading dimensions of the node-row buffers.  fp32 node GEMMs (VEC = false) read one column per lane: odd
// strides, conflict-free.  Split node GEMMs and the phi_e layer-1 gathers (VEC = true) read / write 16 B per lane
// (ds_read_b128 / ds_write_b128): strides that are multiples of 4 floats with an odd multiple, so 16 consecutive
// rows cover all 64 banks.
__host__ __device__ inline int ld_node(int k, int odd_pad, bool vec) {
  if (!vec) return k + odd_pad;
  const int a = align4(k);
  return ((a >> 2) & 1) ? a : a + 4;
}

template <int NT>
__host__ __device__ inline int lds_eval_floats(int N, int D, int H, int T, int M, int L, int MPW, int RP, bool vec,
                                               bool noP = false) {
  const int R = RP * (1 + NT);
  int n = 0;
  n += align4(R * ld_node(H + T, 1, vec));
  n += align4(R * ld_node(H, 1, vec));
  if (!noP) n += align4(R * ld_node(2 * M, 3, vec));
  n += align4(R * ld_node(M, 1, vec));
  n += 2 * align4(R * D);
  n += align4(2 * MPW * D);
  n += align4(MPW * T);
  n += align4((2 * L + 2) * M);   // vecs: 2L - 1 chain biases, w_d, w_g, w_x
  n += align4(MPW * N);
#ifdef ECNF_STAMPS
  n += 64;   // 32 x u64 stamp slots
#endif
  return n;
}

template <int NT, bool VEC, bool NOP = false>
__device__ inline Lds carve_lds(const Net& net, float* base) {
  Lds s;
  const int R = net.RP * (1 + NT);
  float* p = base;
  s.hin = p;  s.ld_hin = ld_node(net.H + net.T, 1, VEC); p += align4(R * s.ld_hin);
  s.hb = p;   s.ld_hb = ld_node(net.H, 1, VEC);          p += align4(R * s.ld_hb);
  s.P = NOP ? nullptr : p;
  s.ld_P = ld_node(2 * net.M, 3, VEC);
  if (!NOP) p += align4(R * s.ld_P);
  s.macc = p; s.ld_m = ld_node(net.M, 1, VEC);           p += align4(R * s.ld_m);
  s.xc = p;    p += align4(R * net.D);
  s.dxacc = p; p += align4(R * net.D);
  s.mean = p;  p += align4(2 * net.MPW * net.D);
  s.temb = p;  p += align4(net.MPW * net.T);
  s.vecs = p;  p += align4((2 * net.L + 2) * net.M);
  s.feat = reinterpret_cast<int*>(p); p += align4(net.MPW * net.N);
  p += net.xs_floats;   // column-split team mode's layer image (lds_xs), 0 floats otherwise
#ifdef ECNF_STAMPS
  s.stamps = reinterpret_cast<unsigned long long*>(p); p += 64;
#endif
  s.cross = s.hin;
  s.tail = p;
  return s;
}

// ---------------------------------------------------------------------------------------------------
// scalar helpers
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

// y = silu(p); dy = silu'(p) * dp
template <int NT>
__device__ __forceinline__ void silu_dual(float p, float dp, float& y, float& dy) {
  const float s = sigmoidf_(p);
  y = p * s;
  if constexpr (NT) dy = s * (1.0f + p * (1.0f - s)) * dp;
}

// Returns `p` as a wave-uniform (SGPR) value the optimiser cannot see through: keeps per-tile weight loads inside
// the tile loop (no LICM of a layer's weights into registers) and their addresses scalar.
template <typename T>
__device__ __forceinline__ const T* launder_uniform(const T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  return reinterpret_cast<const T*>(((uint64_t)hi << 32) | lo);
}

// threadIdx.x through an empty asm: per-thread indices and LDS addresses derived from it are recomputed where they
// are used (a few VALU) instead of being hoisted out of the solver loop and kept live across the edge phase, whose
// tiles need every register (hoisted, they spill to scratch)
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// a wave-uniform int through an empty asm: sizes used as divisors in per-evaluation loops (i / ND, i % ND) are seen
// afresh at each use site, so the compiler does not hoist their division constants out of the solver loop and keep
// them live (in VGPRs, which then spill) across every evaluation
__device__ __forceinline__ int opaque_u(int v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}

__device__ __forceinline__ f32x4 ldg4(const float* p, int idx4) { return gptr4(p)[idx4]; }

__device__ __forceinline__ f32x16 mfma32(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// accumulator row of register r for lane half kk (C/D map of the 32x32 f32 MFMA)
__device__ __forceinline__ int acc_row(int r, int kk) { return (r & 3) + 8 * (r >> 2) + 4 * kk; }

__device__ __forceinline__ void init_bias(f32x16& acc, const float* __restrict__ bias, int jb, int kk) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 b = bias ? gptr4(bias + jb * 32 + 8 * q + 4 * kk)[0] : f32x4{0.f, 0.f, 0.f, 0.f};
    acc[4 * q + 0] = b[0];
    acc[4 * q + 1] = b[1];
    acc[4 * q + 2] = b[2];
    acc[4 * q + 3] = b[3];
  }
}

#include "chain_split.hpp"

// ---------------------------------------------------------------------------------------------------
// node GEMM k-loop over one source: acc[a] += sum_k W[k][(jb + a)*32 + i] X[n][k] for k in [0, K), NA output
// blocks sharing every B fragment.  A (global) and B (LDS) fragments are software-pipelined one chunk of CH
// k-steps ahead, so neither the L2 nor the LDS latency sits between dependent MFMAs.
// ---------------------------------------------------------------------------------------------------
template <int NT, int NA>
__device__ __forceinline__ void node_kloop(f32x16 (&acc)[NA], f32x16 (&accT)[NA], gfloat_p wcol, int ldw,
                                           const float* xr, const float* xrT, int K) {
  constexpr int CH = 8;
  const int nks = K >> 1;              // k-steps of 2
  const int nch = nks / CH;
  float an[NA][CH], bn[CH], btn[CH];
  if (nch > 0) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
#pragma unroll
      for (int a = 0; a < NA; ++a) an[a][j] = wcol[(2 * j) * ldw + 32 * a];
      bn[j] = xr[2 * j];
      if constexpr (NT) btn[j] = xrT[2 * j];
    }
  }
  for (int c = 0; c < nch; ++c) {
    float ac[NA][CH], bc[CH], btc[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
#pragma unroll
      for (int a = 0; a < NA; ++a) ac[a][j] = an[a][j];
      bc[j] = bn[j];
      if constexpr (NT) btc[j] = btn[j];
    }
    if (c + 1 < nch) {
      const int k0 = 2 * CH * (c + 1);
#pragma unroll
      for (int j = 0; j < CH; ++j) {
#pragma unroll
        for (int a = 0; a < NA; ++a) an[a][j] = wcol[(k0 + 2 * j) * ldw + 32 * a];
        bn[j] = xr[k0 + 2 * j];
        if constexpr (NT) btn[j] = xrT[k0 + 2 * j];
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        acc[a] = mfma32(ac[a][j], bc[j], acc[a]);
        if constexpr (NT) accT[a] = mfma32(ac[a][j], btc[j], accT[a]);
      }
    }
  }
  for (int k = 2 * CH * nch; k < K; k += 2) {
    const float b = xr[k];
    const float bt = NT ? xrT[k] : 0.f;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const float w = wcol[k * ldw + 32 * a];
      acc[a] = mfma32(w, b, acc[a]);
      if constexpr (NT) accT[a] = mfma32(w, bt, accT[a]);
    }
  }
}

// bias/act/residual epilogue of a node GEMM task: Y[n][j] (and the tangent row RP + n)
template <int NT, int NA>
__device__ __forceinline__ void node_epilogue(const f32x16 (&acc)[NA], const f32x16 (&accT)[NA], bool act,
                                              const float* resid, int ldr, float* Y, int ldy, int RP, int nvalid,
                                              int jb, int n, int kk) {
  if (n < nvalid) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = (jb + a) * 32 + acc_row(r, kk);
        float y = acc[a][r], yT = 0.f;
        if (act) {
          silu_dual<NT>(acc[a][r], NT ? accT[a][r] : 0.f, y, yT);
        } else if constexpr (NT) {
          yT = accT[a][r];
        }
        if (resid) {
          y += resid[n * ldr + j];
          if constexpr (NT) yT += resid[(RP + n) * ldr + j];
        }
        Y[n * ldy + j] = y;
        if constexpr (NT) Y[(RP + n) * ldy + j] = yT;
      }
  }
}

template <int NT, int NA>
__device__ __forceinline__ void node_task(const float* X1, int ldx1, int K1, const float* X2, int ldx2, int K2,
                                          const float* __restrict__ W, int ldw, const float* __restrict__ bias,
                                          bool act, const float* resid, int ldr, float* Y, int ldy, int RP,
                                          int nvalid, int jb, int ct, int lane) {
  const int kk = lane >> 5, li = lane & 31;
  const int n = ct * 32 + li;
  f32x16 acc[NA], accT[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    init_bias(acc[a], bias, jb + a, kk);
#pragma unroll
    for (int r = 0; r < 16; ++r) accT[a][r] = 0.f;
  }
  const gfloat_p wcol = gptr(W) + kk * ldw + jb * 32 + li;
  node_kloop<NT, NA>(acc, accT, wcol, ldw, X1 + n * ldx1 + kk, X1 + (RP + n) * ldx1 + kk, K1);
  if (K2 > 0)
    node_kloop<NT, NA>(acc, accT, wcol + K1 * ldw, ldw, X2 + n * ldx2 + kk, X2 + (RP + n) * ldx2 + kk, K2);
  node_epilogue<NT, NA>(acc, accT, act, resid, ldr, Y, ldy, RP, nvalid, jb, n, kk);
}

// split node GEMM task: acc[a] = b + sum_k W[k][(jb + a) * 32 + i] X[n][k], the fp32 operands split into two fp16
// pieces (three cross terms, chain_split.hpp).  A: host-packed fragments, K zero-padded to a multiple of 16, fetched
// by buffer loads PFA k-steps ahead; B: the lane's node row, 8 consecutive features from LDS (16-B row strides),
// split in registers; NA output blocks share every B split.  NT = 1 (the divergence kernels): the tangent row RP + n
// shares every A fragment and gets no bias, act'(pre) * (X_T W) (as node_task).
// INPLACE (Y may alias X1): every wave of the workgroup calls it once (active = false: no task) and the outputs are
// written after a barrier that follows every wave's k-loop.

template <int NA, int NT = 0, bool INPLACE = false, int PFA = kNodePFADefault>
__device__ __forceinline__ void node_task_split(const float* X1, int ldx1, int K1, const float* X2, int ldx2, int K2,
                                                const unsigned* __restrict__ Wpk, float winv,
                                                const float* __restrict__ bias, bool act, const float* resid, int ldr, float* Y, int ldy, int RP,
                                                int nvalid, int jb, int ct, int lane, bool active = true) {
  // PFA: k-steps of A fragments in flight ahead of the MFMAs
  jb = __builtin_amdgcn_readfirstlane(jb);   // uniform: buffer-load offsets in SGPRs (no waterfall loops)
  ct = __builtin_amdgcn_readfirstlane(ct);
  const int kk = lane >> 5, li = lane & 31;
  const int n = ct * 32 + li;
  ECNF_DCHECK(!active || ct * 32 < RP, 3);
  const int nks1 = (K1 + 15) >> 4, nks = nks1 + ((K2 + 15) >> 4);
  // biases are added in the epilogue: their load latency hides behind the k-loop
  f32x4 bq[NA][4];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      bq[a][q] = bias ? gptr4(bias + (jb + a) * 32 + 8 * q + 4 * kk)[0] : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x16 acc[NA], accT[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    acc[a] = f32x16{};
    if constexpr (NT) accT[a] = f32x16{};
  }
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(Wpk), (short)0,
                                                                         0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  // B: 8 consecutive features of node row `row` for k-step ks
  auto bload = [&](int ks, int row, float (&v)[8]) {
    const bool first = ks < nks1;
    const float* src = first ? X1 + row * ldx1 : X2 + row * ldx2;
    const int c0 = 16 * (first ? ks : ks - nks1) + 8 * kk;
    const int K = first ? K1 : K2;
    if (c0 + 8 <= K) {   // 16-B aligned (ld_node with VEC): two ds_read_b128
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src + c0);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + c0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = lo[j];
        v[4 + j] = hi[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (c0 + j < K) ? src[c0 + j] : 0.f;
    }
  };
  auto aload = [&](int ks, u32x4 (&w)[NA][kPieces]) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int p = 0; p < kPieces; ++p) w[a][p] = wload(rsrc, voff, (((jb + a) * nks + ks) * kPieces + p) * kPieceBytes);
  };
  auto bsplit = [&](const float (&v)[8], u32x4 (&B)[kPieces]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned pc[kPieces];
      split_pair(v[2 * e], v[2 * e + 1], pc);
#pragma unroll
      for (int p = 0; p < kPieces; ++p) B[p][e] = pc[p];
    }
  };
  // A fragments: a ring of S = PFA + 1 k-step slots; the load of k-step ks + PFA is issued (clamped to the last
  // k-step, so the main loop has no branches) before the MFMAs of k-step ks and pinned there by a sched_barrier,
  // so PFA k-steps of MFMAs cover its latency
  constexpr int S = PFA + 1;
  float bv[8], bvT[8];
  u32x4 wa[S][NA][kPieces];
  if (active) {
  bload(0, n, bv);
  if constexpr (NT) bload(0, RP + n, bvT);
  static_for<PFA>([&](auto Ic) { aload(min((int)decltype(Ic)::value, nks - 1), wa[decltype(Ic)::value]); });
  auto kstep = [&](int ks, auto Ic) {
    constexpr int i = decltype(Ic)::value;
    aload(min(ks + PFA, nks - 1), wa[(i + PFA) % S]);
    u32x4 B[kPieces], BT[kPieces];
    bsplit(bv, B);
    if constexpr (NT) bsplit(bvT, BT);
    bload(min(ks + 1, nks - 1), n, bv);
    if constexpr (NT) bload(min(ks + 1, nks - 1), RP + n, bvT);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      static_for<kTerms>([&](auto Tc) {
        constexpr int t = decltype(Tc)::value;
        acc[a] = mfma_split(wa[i][a][term_w(t)], B[term_x(t)], acc[a]);
        if constexpr (NT) accT[a] = mfma_split(wa[i][a][term_w(t)], BT[term_x(t)], accT[a]);
      });
    __builtin_amdgcn_sched_barrier(0);
  };
  int ks = 0;
  for (; ks + S <= nks; ks += S) static_for<S>([&](auto Ic) { kstep(ks + decltype(Ic)::value, Ic); });
  static_for<S>([&](auto Ic) {
    if (ks + (int)decltype(Ic)::value < nks) kstep(ks + decltype(Ic)::value, Ic);
  });
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[a][r] = fmaf(acc[a][r], winv, bq[a][r >> 2][r & 3]);
      if constexpr (NT) accT[a][r] *= winv;
    }
  }  // active
  if constexpr (INPLACE) __syncthreads();
  // epilogue with 16-B LDS accesses: registers 4q..4q+3 are 4 consecutive output features
  if (active && n < nvalid) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = (jb + a) * 32 + 8 * q + 4 * kk;
        f32x4 y, yT;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = acc[a][4 * q + e];
          if constexpr (NT) {
            if (act) {
              float ye, yte;
              silu_dual<NT>(t, accT[a][4 * q + e], ye, yte);
              y[e] = ye;
              yT[e] = yte;
            } else {
              y[e] = t;
              yT[e] = accT[a][4 * q + e];
            }
          } else {
            y[e] = act ? t * sigmoidf_(t) : t;
          }
        }
        if (resid) {
          y += *reinterpret_cast<const f32x4*>(resid + n * ldr + j);
          if constexpr (NT) yT += *reinterpret_cast<const f32x4*>(resid + (RP + n) * ldr + j);
        }
        *reinterpret_cast<f32x4*>(Y + n * ldy + j) = y;
        if constexpr (NT) *reinterpret_cast<f32x4*>(Y + (RP + n) * ldy + j) = yT;
      }
  }
}

// ---------------------------------------------------------------------------------------------------
// node GEMM: Y[n][0:NOUT] = act([X1 | X2][n] W + b) (+ resid[n]); tangent rows RP+n share the A fragments
// and get no bias, act'(pre) * (X_T W).  Output blocks are paired (shared B reads, two independent MFMA
// chains) whenever the pairs still give every wave a task.
// ---------------------------------------------------------------------------------------------------
// split node GEMM task deal: two output blocks per task (sharing the B split) when the pairs still give every wave a
// task (pairing at half / a quarter of the waves measured within noise, profiles/round3/ab)
template <int NW>
__device__ __forceinline__ bool node_paired(int njb, int nct) {
  return (njb % 2) == 0 && (njb / 2) * nct >= NW;
}

template <int NT, int NW, bool SPLIT, int PFA = kNodePFADefault>
__device__ __forceinline__ void node_gemm(const float* X1, int ldx1, int K1, const float* X2, int ldx2, int K2,
                                          const float* __restrict__ W, const unsigned* __restrict__ Ws, float winv,
                                          int ldw, const float* __restrict__ bias, int NOUT, bool act, const float* resid,
                                          int ldr, float* Y, int ldy, int RP, int nvalid, int wave, int lane) {
  const int njb = NOUT >> 5, nct = RP >> 5;
  if constexpr (SPLIT) {
    if (node_paired<NW>(njb, nct)) {   // two output blocks per task share the B split
      const int npair = njb / 2;
      for (int task = wave; task < npair * nct; task += NW)
        node_task_split<2, NT, false, PFA>(X1, ldx1, K1, X2, ldx2, K2, Ws, winv, bias, act, resid, ldr, Y, ldy, RP,
                                           nvalid, 2 * (task % npair), task / npair, lane);
    } else {
      for (int task = wave; task < njb * nct; task += NW)
        node_task_split<1, NT, false, PFA>(X1, ldx1, K1, X2, ldx2, K2, Ws, winv, bias, act, resid, ldr, Y, ldy, RP,
                                           nvalid, task % njb, task / njb, lane);
    }
    return;
  }
  // the fp32 node GEMMs (strict-fp32 kernels): one output block per task (pairing measured slower for phi_h, r01)
  for (int task = wave; task < njb * nct; task += NW)
    node_task<NT, 1>(X1, ldx1, K1, X2, ldx2, K2, W, ldw, bias, act, resid, ldr, Y, ldy, RP, nvalid, task % njb,
                     task / njb, lane);
}

// in-place split node GEMM (Y aliases X1; the wide tangent kernels' phi_h on macc): one (output block pair, 32-row
// tile) task per wave at most (the host admits these kernels only where (NOUT / 64) (RP / 32) <= NW: M = 256 at one
// row tile, M = 128 at two)
template <int NT, int NW>
__device__ __forceinline__ void node_gemm_inplace(const float* X1, int ldx1, int K1, const float* X2, int ldx2, int K2,
                                                  const unsigned* __restrict__ Ws, float winv,
                                                  const float* __restrict__ bias, int NOUT, bool act, float* Y, int ldy,
                                                  int RP, int nvalid, int wave, int lane) {
  const int npair = NOUT >> 6, ntask = npair * (RP >> 5);
  const bool active = wave < ntask;
  ECNF_DCHECK(ntask <= NW, 3);
  node_task_split<2, NT, true>(X1, ldx1, K1, X2, ldx2, K2, Ws, winv, bias, act, nullptr, 0, Y, ldy, RP, nvalid,
                               active ? 2 * (wave % npair) : 0, active ? wave / npair : 0, lane, active);
}

// the same in strict fp32 (the M = 256 fp32 tangent kernels, Geo::kWideT32): node_task's k-loop and epilogue on
// v_mfma_f32_32x32x2_f32 with the epilogue behind a barrier every wave of the workgroup reaches
template <int NT, int NW>
__device__ __forceinline__ void node_gemm_inplace_f32(const float* X1, int ldx1, int K1, const float* X2, int ldx2,
                                                      int K2, const float* __restrict__ W, int ldw,
                                                      const float* __restrict__ bias, int NOUT, bool act, float* Y,
                                                      int ldy, int RP, int nvalid, int wave, int lane) {
  const int npair = NOUT >> 6, ntask = npair * (RP >> 5);
  const bool active = wave < ntask;
  const int jb = active ? 2 * (wave % npair) : 0, ct = active ? wave / npair : 0;
  const int kk = lane >> 5, li = lane & 31, n = ct * 32 + li;
  ECNF_DCHECK(ntask <= NW, 3);
  f32x16 acc[2], accT[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    init_bias(acc[a], bias, jb + a, kk);
#pragma unroll
    for (int r = 0; r < 16; ++r) accT[a][r] = 0.f;
  }
  if (active) {
    const gfloat_p wcol = gptr(W) + kk * ldw + jb * 32 + li;
    node_kloop<NT, 2>(acc, accT, wcol, ldw, X1 + n * ldx1 + kk, X1 + (RP + n) * ldx1 + kk, K1);
    if (K2 > 0)
      node_kloop<NT, 2>(acc, accT, wcol + K1 * ldw, ldw, X2 + n * ldx2 + kk, X2 + (RP + n) * ldx2 + kk, K2);
  }
  __syncthreads();
  if (active) node_epilogue<NT, 2>(acc, accT, act, nullptr, 0, Y, ldy, RP, nvalid, jb, n, kk);
}

// ---------------------------------------------------------------------------------------------------
// edge-MLP chain layer: b = silu(a W + bias), all in registers (a, b: NF blocks of 32 rows x 32 edges).
// The A fragments of one (output block jb, input block fb) group are 4 dwordx4 per lane (16 MFMAs); groups are
// software-pipelined PF groups ahead so the L2 latency hides behind MFMAs (counted vmcnt, no vmcnt(0) stalls).
// ---------------------------------------------------------------------------------------------------
// One software pipeline over NL consecutive chain layers (phi_e 2..L, or phi_x 1..L), IN PLACE:
// X <- silu(X W_l + b_l) for l = 0..NL-1, one 32-edge tile in registers.
//
// Group (l, g = fb * NF + jb) is 16 MFMAs that accumulate input block fb of X into output block jb; the NF output
// blocks of a layer accumulate side by side, so a wave holds 16 NF activation + 16 NF accumulator registers.
// The SiLU epilogue is NOT a burst at the layer end: an fp32 32x32x2 MFMA keeps the SIMD busy for 64 cycles but
// holds its vector issue for only a few of them, so independent VALU placed between the wave's own MFMAs is
// almost free (MI355X_MICROARCH.md, "vector-instruction ISSUE cost").  Output block j < NF-1 is final after group
// (NF-1, j) and is activated (X[j] <- silu(acc[j] + b), in place: X[j] was last read by group (j, *)) one
// element per MFMA slot during the next group; block NF-1 is activated during the first NF-1 groups of the next
// layer, before group (0, NF-1) re-zeroes its accumulator and long before group (NF-1, *) reads it.  Only the
// last layer's block NF-1 is left for a short tail.  sched_barriers pin this order and the weight prefetch
// (PF groups ahead, contiguous across layers).
template <int NF>
struct ChainPlan {
  // SiLU work of group g (0..NF*NF-1) of a layer l: {block, layer offset (0 = this layer, -1 = previous), first
  // element, end element}; block -1 = none
  struct Task { int j, dl, e0, e1; };
  static constexpr Task task(int g, bool has_prev) {
    if (g >= (NF - 1) * NF + 1) return Task{g - (NF - 1) * NF - 1, 0, 0, 16};
    if (has_prev && g <= NF - 2) return Task{NF - 1, -1, (16 * g) / (NF - 1), (16 * (g + 1)) / (NF - 1)};
    return Task{-1, 0, 0, 0};
  }
  // MFMA slot (1..15) after which element k of n is activated
  static constexpr int slot(int k, int n) { return 1 + (k * 15) / (n > 0 ? n : 1); }
};

template <int NT>
__device__ __forceinline__ void chain_act(f32x16& x, f32x16& xt, const f32x16& a, const f32x16& at, int r, float b) {
  float y, yT = 0.f;
  silu_dual<NT>(a[r] + b, NT ? at[r] : 0.f, y, yT);
  x[r] = y;
  if constexpr (NT) xt[r] = yT;
}

template <int NF, int NT, int NL>
__device__ __forceinline__ void chain_segment(f32x16 (&X)[NF], f32x16 (&XT)[NF], const float* __restrict__ Wpk,
                                              const float* __restrict__ bias /* LDS, [NL][M] */, int lane) {
  constexpr int GL = NF * NF;             // groups per layer, g = fb * NF + jb
  constexpr int G = NL * GL;
  constexpr int M = NF * 32;
  constexpr int PF = 2;                   // groups in flight ahead of the MFMAs
  using Plan = ChainPlan<NF>;
  const int kk = lane >> 5;
  const gf32x4_p wp = gptr4(Wpk) + lane;
  // group (l, jb, fb) sits at wp[((l * NF * NF + jb * NF + fb) * 4 + q) * 64]
  auto gidx = [](int gg) constexpr {
    const int l = gg / GL, g = gg % GL, fb = g / NF, jb = g % NF;
    return (l * NF * NF + jb * NF + fb) * 4;
  };
  f32x4 wbuf[PF + 1][4];
#pragma unroll
  for (int gg = 0; gg < PF && gg < G; ++gg)
#pragma unroll
    for (int q = 0; q < 4; ++q) wbuf[gg][q] = wp[(gidx(gg) + q) * 64];
  f32x16 acc[NF], accT[NF];
  f32x4 bb[4];                            // bias of the block being activated
  static_for<G>([&](auto GGc) {
    constexpr int gg = decltype(GGc)::value;
    constexpr int l = gg / GL, g = gg % GL, fb = g / NF, jb = g % NF;
    constexpr typename Plan::Task tk = Plan::task(g, l > 0);
    if constexpr (gg + PF < G) {
#pragma unroll
      for (int q = 0; q < 4; ++q) wbuf[(gg + PF) % (PF + 1)][q] = wp[(gidx(gg + PF) + q) * 64];
    }
    if constexpr (tk.j >= 0 && tk.e0 == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bb[q] = *reinterpret_cast<const f32x4*>(bias + (l + tk.dl) * M + tk.j * 32 + 8 * q + 4 * kk);
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<16>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value, q = i >> 2, e = i & 3;
      const float w = wbuf[gg % (PF + 1)][q][e];
      if constexpr (fb == 0 && i == 0) {
        const f32x16 z = {};
        acc[jb] = mfma32(w, X[fb][i], z);
        if constexpr (NT) accT[jb] = mfma32(w, XT[fb][i], z);
      } else {
        acc[jb] = mfma32(w, X[fb][i], acc[jb]);
        if constexpr (NT) accT[jb] = mfma32(w, XT[fb][i], accT[jb]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (tk.j >= 0) {
        constexpr int n = tk.e1 - tk.e0;
        static_for<16>([&](auto Kc) {
          constexpr int k = decltype(Kc)::value;
          if constexpr (k < n && Plan::slot(k, n) == i) {
            constexpr int r = tk.e0 + k;
            chain_act<NT>(X[tk.j], XT[tk.j], acc[tk.j], accT[tk.j], r, bb[r >> 2][r & 3]);
          }
        });
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  });
  // tail: the last layer's block NF-1
#pragma unroll
  for (int q = 0; q < 4; ++q) bb[q] = *reinterpret_cast<const f32x4*>(bias + (NL - 1) * M + (NF - 1) * 32 + 8 * q + 4 * kk);
#pragma unroll
  for (int r = 0; r < 16; ++r) chain_act<NT>(X[NF - 1], XT[NF - 1], acc[NF - 1], accT[NF - 1], r, bb[r >> 2][r & 3]);
}

// Segmented (by receiver row) inclusive PREFIX sum over the 32 edge lanes of each half-wave, in DPP:
// row_shr:1,2,4,8 inside each 16-lane row, then row_bcast:15 carries lane 15's running sum into lanes 16..31
// (rows 1 and 3 only, so the two half-waves — same edges, different feature rows — never mix).  Each step is
// v += ok_step * dpp(v): one fused v_fmac_f32_dpp per value, no LDS traffic and no waits.  Segments are contiguous
// lane runs, so "same segment as the source lane" is the Hillis-Steele condition; the tail lane of a segment
// ends holding the segment's sum inside this tile.
struct SegScan {
  float okf[5];
  bool tail;
  template <int CTRL, int ROWMASK>
  __device__ __forceinline__ static int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xF, true);
  }
  __device__ __forceinline__ void init(int seg, int li) {
    const int sp = seg + 1;   // 0 marks "no source lane" (bound_ctrl / masked rows read 0)
    int src;
    src = dpp_i<0x111, 0xF>(sp); okf[0] = (sp != 0 && src == sp) ? 1.f : 0.f;   // row_shr:1
    src = dpp_i<0x112, 0xF>(sp); okf[1] = (sp != 0 && src == sp) ? 1.f : 0.f;   // row_shr:2
    src = dpp_i<0x114, 0xF>(sp); okf[2] = (sp != 0 && src == sp) ? 1.f : 0.f;   // row_shr:4
    src = dpp_i<0x118, 0xF>(sp); okf[3] = (sp != 0 && src == sp) ? 1.f : 0.f;   // row_shr:8
    src = dpp_i<0x142, 0xA>(sp); okf[4] = (sp != 0 && src == sp) ? 1.f : 0.f;   // row_bcast:15 -> rows 1, 3
    const int nxt = __shfl_down(seg, 1, 32);
    tail = (li == 31) || (nxt != seg);
  }
  // one fused v_fmac_f32_dpp per value and step (v += ok * v[lane - shift]).  The __builtin_amdgcn_update_dpp form
  // compiles to v_mov_b32_dpp + v_fmac_f32 + s_nop 0 per value (the DPP read of a just-written temp needs wait
  // states), 3 issue slots instead of 1.  Wait states for the fused form (the compiler's hazard recognizer does not look inside
  // inline asm): a value is re-read through DPP NV - 1 >= 2 instructions after its last write inside the scan, and
  // the s_nop 4 in front covers VALU writes of v (2 wait states) and an EXEC write just before the scan (5; e.g. the
  // end of the tangent kernels' `if (writer)` stores).  row_bcast:15 writes rows 1 and 3 only; rows 0 and 2 keep v.
  // The consumers' wait states after the asm are checked on the built kernels (tools/isa_hazards.py,
  // tests/test_isa_hazards.py).
  template <int NV>
  __device__ __forceinline__ void sum_many(float (&v)[NV]) const {
    static_assert(NV >= 3, "DPP wait states assume >= 3 interleaved values");
    // the scheduler must not sink the producers of v below the s_nop (volatile asm only orders asm statements)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4");
#define ECNF_DPP_STEP(K, CTRL)                                                                          \
    _Pragma("unroll") for (int i = 0; i < NV; ++i)                                                      \
      asm volatile("v_fmac_f32_dpp %0, %0, %1 " CTRL " bank_mask:0xf bound_ctrl:1" : "+v"(v[i]) : "v"(okf[K]));
    ECNF_DPP_STEP(0, "row_shr:1 row_mask:0xf")
    ECNF_DPP_STEP(1, "row_shr:2 row_mask:0xf")
    ECNF_DPP_STEP(2, "row_shr:4 row_mask:0xf")
    ECNF_DPP_STEP(3, "row_shr:8 row_mask:0xf")
    ECNF_DPP_STEP(4, "row_bcast:15 row_mask:0xa")
#undef ECNF_DPP_STEP
    __builtin_amdgcn_sched_barrier(0);
  }
};

__device__ __forceinline__ void lds_add(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// m_i += the lane's 16 segment sums of block fb into macc row `row` (the message aggregation's LDS atomics).  The row
// goes through an empty asm, so the compiler does not precompute (and spill) the 16 lane addresses per block.
//  * M = 64 and 256 (NF 2, 8): an opaque integer row offset -> ds_add_f32 with the 16 offsets in the instruction
//    (interleaved A/B, profiles/round5/ab/ds_vs_flat/: ALDP B = 512 PID Hutchinson 24.2 -> 23.4 ms, QM9 B = 512
//    Euler-20 Hutchinson 297.5 -> 296.3 ms, QM9 B = 2048 Euler-20 sample 438.6 -> 435.7 ms);
//  * M = 128 (NF 4): an opaque row pointer -> flat_atomic_add_f32 on the LDS aperture.  The ds form is equally fast
//    there (LJ13 Hutchinson 63.6 ms both), and in the (128, 2, 3) tangent vf_kernel it leads the compiler into a
//    miscompile: five register copies placed before an EXEC restore where EXEC is 0 (DESIGN 5.4;
//    tests/test_isa_hazards.py checks every shipped kernel for that pattern).
template <int NF>
__device__ __forceinline__ void agg_rows(const Lds& s, int row, int kk, int fb, const float (&v)[16]) {
  if constexpr (NF != 4) {
    int mo = row * s.ld_m + 4 * kk;
    asm volatile("" : "+v"(mo));
#pragma unroll
    for (int r16 = 0; r16 < 16; ++r16) lds_add(s.macc + mo + fb * 32 + acc_row(r16, 0), v[r16]);
  } else {
    float* mrow = s.macc + row * s.ld_m + 4 * kk;
    asm volatile("" : "+v"(mrow));
#pragma unroll
    for (int r16 = 0; r16 < 16; ++r16) lds_add(mrow + fb * 32 + acc_row(r16, 0), v[r16]);
  }
}

// d = w . x (and dT = w . xT) over the lane's NF x 16 feature registers, w an LDS vector in accumulator row order
// (rows acc_row(r, kk), 16-B reads); the caller adds the other lane half.  Four partial sums, and the weight reads
// issued one group of 4 ahead behind scheduling fences: the one-accumulator form compiled to 4 NF rounds of
// read -> s_waitcnt lgkmcnt(0) -> 4 dependent FMAs, exposing the LDS latency and the FMA chain 4 NF times per tile.
template <int NF, int NT>
__device__ __forceinline__ void lds_dot(const float* __restrict__ w, const f32x16 (&x)[NF], const f32x16 (&xt)[NF],
                                        int kk, float& d, float& dT) {
  // (2 reads per group in the M = 256 tangent kernels, whose 512-register waves have no 32 registers to spare)
  constexpr int NQ = 4 * NF, GQ = (NT && NF >= 8) ? 2 : 4, NG = NQ / GQ;
  auto rd = [&](int q) { return *reinterpret_cast<const f32x4*>(w + (q >> 2) * 32 + 8 * (q & 3) + 4 * kk); };
  f32x4 wb[2][GQ];
  float p[4] = {0.f, 0.f, 0.f, 0.f}, pt[4] = {0.f, 0.f, 0.f, 0.f};
  static_for<GQ>([&](auto Ic) { wb[0][decltype(Ic)::value] = rd(decltype(Ic)::value); });
  static_for<NG>([&](auto Gc) {
    constexpr int g = decltype(Gc)::value;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (g + 1 < NG)
      static_for<GQ>([&](auto Ic) { wb[(g + 1) & 1][decltype(Ic)::value] = rd((g + 1) * GQ + decltype(Ic)::value); });
    static_for<GQ>([&](auto Ic) {
      constexpr int q = g * GQ + decltype(Ic)::value, fb = q >> 2, qq = q & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        p[e] = fmaf(wb[g & 1][decltype(Ic)::value][e], x[fb][4 * qq + e], p[e]);
        if constexpr (NT) pt[e] = fmaf(wb[g & 1][decltype(Ic)::value][e], xt[fb][4 * qq + e], pt[e]);
      }
    });
  });
  __builtin_amdgcn_sched_barrier(0);
  d = (p[0] + p[1]) + (p[2] + p[3]);
  dT = NT ? (pt[0] + pt[1]) + (pt[2] + pt[3]) : 0.f;
}

// ---------------------------------------------------------------------------------------------------
// Block-1 pair tiles (single-feature molecules of 13 atoms, e.g. LJ13; the M = 128 split primal kernels).  With one
// node feature every atom enters block 1 with the same h (the embedding of that feature and the time, egnn.py:162-167),
// so phi_e's input [h_s, h_r, |r|^2] (egnn.py:76) is symmetric: m_ij = m_ji BITWISE (|r_ji| = |r_ij| exactly and the
// per-node phi_e.0 halves P_s, P_r are equal rows), and so are the gate and phi_x (egnn.py:82-101).  Block 1 then runs
// the chains once per unordered pair, 78 pairs in 3 tiles instead of 156 edges in 5, and adds each pair's gated
// message to both atoms and its shift with opposite signs (r_ji = -r_ij).  Tiles over the groups A = {0..3},
// B = {4..7}, C = {8..12}: tile 0 = the pairs inside A u B (28), tile 1 = A x C and inside C (30), tile 2 = B x C (20),
// so every atom sits in exactly two tiles and gets two atomic contributions per block (0 + a + b, exact in either
// order, as the receiver segments' two parts: run-to-run deterministic and independent of the molecules per
// workgroup).  Inside a tile an atom's pairs sit on several lanes: the wave transposes its gated messages through a
// 1024-float slice of the P rows (dead once layer 1 read its per-molecule rows, copied before the edge phase) and sums
// each atom's pairs in a fixed order.
// ---------------------------------------------------------------------------------------------------
#ifndef ECNF_PAIR_NODE_FENCE   // (experiment builds may override)
#define ECNF_PAIR_NODE_FENCE 0
#endif
struct PairPlan13 {
  static constexpr int kN = 13, kTiles = 3, kMaxNodes = 9, kMaxDeg = 8;
  struct Tile {
    int np;                      // pairs (lanes np .. 31 are padding)
    unsigned char a[32], b[32];  // pair (a, b), a < b: r = x_a - x_b; +m, +shift to a and +m, -shift to b
    int nn;                      // atoms touched
    unsigned char node[kMaxNodes], deg[kMaxNodes], lane[kMaxNodes][kMaxDeg], role[kMaxNodes][kMaxDeg];
  };
  static constexpr Tile make(int t) {
    Tile x{};
    auto add = [&](int a, int b) {
      x.a[x.np] = (unsigned char)a;
      x.b[x.np] = (unsigned char)b;
      ++x.np;
    };
    if (t == 0) {
      for (int a = 0; a < 8; ++a)
        for (int b = a + 1; b < 8; ++b) add(a, b);
    } else if (t == 1) {
      for (int a = 0; a < 4; ++a)
        for (int b = 8; b < 13; ++b) add(a, b);
      for (int a = 8; a < 13; ++a)
        for (int b = a + 1; b < 13; ++b) add(a, b);
    } else {
      for (int a = 4; a < 8; ++a)
        for (int b = 8; b < 13; ++b) add(a, b);
    }
    for (int n = 0; n < kN; ++n) {
      int d = 0;
      for (int p = 0; p < x.np; ++p)
        if (x.a[p] == n || x.b[p] == n) {
          x.lane[x.nn][d] = (unsigned char)p;
          x.role[x.nn][d] = x.b[p] == n ? 1 : 0;
          ++d;
        }
      if (d) {
        x.node[x.nn] = (unsigned char)n;
        x.deg[x.nn] = (unsigned char)d;
        ++x.nn;
      }
    }
    return x;
  }
  // the two tiles that hold atom n's pairs (team_exchange's owners)
  __host__ __device__ __forceinline__ static constexpr int tile_lo(int n) { return n < 8 ? 0 : 1; }
  __host__ __device__ __forceinline__ static constexpr int tile_hi(int n) { return n < 4 ? 1 : 2; }
  // lane word w (lanes 8w .. 8w+7) of tile t: bytes a | b << 4, 0xFF on padding lanes
  static constexpr unsigned long long word(int t, int w) {
    const Tile x = make(t);
    unsigned long long v = 0;
    for (int e = 0; e < 8; ++e) {
      const int p = 8 * w + e;
      const unsigned long long byte = p < x.np ? (unsigned long long)(x.a[p] | (x.b[p] << 4)) : 0xFFull;
      v |= byte << (8 * e);
    }
    return v;
  }
};
// every unordered pair in exactly one tile, every atom in exactly the two tiles tile_lo / tile_hi name, and each
// atom's slot listing all of its pairs in that tile with the right role
constexpr bool pair_plan13_valid() {
  int seen[13][13] = {};
  int tiles_of[13] = {};
  for (int t = 0; t < PairPlan13::kTiles; ++t) {
    const PairPlan13::Tile x = PairPlan13::make(t);
    if (x.np > 30 || x.nn > PairPlan13::kMaxNodes) return false;   // (two halves of 15 transposition rows)
    for (int p = 0; p < x.np; ++p) {
      if (!(x.a[p] < x.b[p] && x.b[p] < 13)) return false;
      ++seen[x.a[p]][x.b[p]];
    }
    for (int sl = 0; sl < x.nn; ++sl) {
      const int n = x.node[sl];
      if (!(PairPlan13::tile_lo(n) == t || PairPlan13::tile_hi(n) == t)) return false;
      ++tiles_of[n];
      int deg = 0;
      for (int p = 0; p < x.np; ++p) deg += (x.a[p] == n || x.b[p] == n) ? 1 : 0;
      if (deg != x.deg[sl] || deg > PairPlan13::kMaxDeg) return false;
      for (int q = 0; q < deg; ++q) {
        const int p = x.lane[sl][q];
        if (!((x.role[sl][q] == 0 && x.a[p] == n) || (x.role[sl][q] == 1 && x.b[p] == n))) return false;
      }
    }
  }
  for (int a = 0; a < 13; ++a) {
    if (tiles_of[a] != 2 || PairPlan13::tile_lo(a) == PairPlan13::tile_hi(a)) return false;
    for (int b = a + 1; b < 13; ++b)
      if (seen[a][b] != 1) return false;
  }
  return true;
}
static_assert(pair_plan13_valid(), "pair tiles of a 13-atom molecule");

// this lane's pair code (a | b << 4, 0xFF: padding) in pair tile tp (wave-uniform)
__device__ __forceinline__ unsigned pair13_code(int tp, int li) {
  // (the words as constants: PairPlan13::word called with a runtime tile compiled to real function calls)
  unsigned long long w[4];
  static_for<4>([&](auto Wc) {
    constexpr int q = decltype(Wc)::value;
    constexpr unsigned long long w0 = PairPlan13::word(0, q), w1 = PairPlan13::word(1, q), w2 = PairPlan13::word(2, q);
    w[q] = tp == 0 ? w0 : tp == 1 ? w1 : w2;
  });
  const int h = li >> 3;
  const unsigned long long v = h == 0 ? w[0] : h == 1 ? w[1] : h == 2 ? w[2] : w[3];
  return (unsigned)(v >> (8 * (li & 7))) & 0xFFu;
}

// per-pair context of a block-1 pair tile, passed by value (sb == nullptr: the receiver-segment path; a pointer to a
// local context kept it in scratch, and its LDS pointers became flat ones)
struct PairCtx {
  int mol;     // molecule slot in the workgroup
  int tp;      // pair tile of the molecule (0 .. 2)
  float* sb;   // this wave's 1024-float transposition slice (16-B aligned)
  int rp;      // tangent row offset RP (the divergence kernels' tangent aggregates and shifts)
};

// m_i += sum over atom i's pairs of m e (egnn.py:102-104) for pair tile TP: per pass two 32-feature blocks, the tile's
// pairs in two halves of 15 LDS rows of 64 features (+4 padding), then lane c sums feature c over each atom's pairs
// (fixed order) and adds it to macc
// (val(fb, r): the value of accumulator register r of block fb; row0: 0, or RP for the tangent aggregates)
template <int TP, int NF, typename Val>
__device__ __forceinline__ void pair_agg_tile(const Lds& s, Val&& val, int mol, int row0, float* sb, int lane) {
  constexpr PairPlan13::Tile T = PairPlan13::make(TP);
  const int kk = lane >> 5, li = lane & 31;
  float* mrows = s.macc + (row0 + mol * PairPlan13::kN) * s.ld_m + lane;
  static_for<NF / 2>([&](auto Pc) {
    constexpr int pass = decltype(Pc)::value;
    float acc[T.nn];
    static_for<2>([&](auto Hc) {
      constexpr int h = decltype(Hc)::value;
      // this half's pairs (15: 1020 floats) as rows of 68 floats (16-B chunks; 4-bank row shift: conflict-free column
      // reads at immediate offsets.  An XOR-swizzled 64-float form needed 2-3 address VALU per read and 32 more registers)
      if (li >= 15 * h && li < 15 * h + 15) {
        const int p = li - 15 * h;
        static_for<2>([&](auto Fc) {
          constexpr int fbl = decltype(Fc)::value, fb = 2 * pass + fbl;
          static_for<4>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value;
            const int c16 = fbl * 8 + 2 * q + kk;
            *reinterpret_cast<f32x4*>(sb + p * 68 + (c16 << 2)) =
                f32x4{val(fb, 4 * q), val(fb, 4 * q + 1), val(fb, 4 * q + 2), val(fb, 4 * q + 3)};
          });
        });
      }
      // the wave's own LDS traffic runs in order; keep the compiler from moving the column reads above the stores (or
      // the next half's stores above these reads).  (A scheduling fence per atom: 23.49 against 23.34 ms without;
      // reading each pair row once into registers first: equal time)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      static_for<T.nn>([&](auto Sc) {
        constexpr int sl = decltype(Sc)::value;
        float v;
        if constexpr (h == 0) v = 0.f;
        else v = acc[sl];
        static_for<T.deg[sl]>([&](auto Qc) {
          constexpr int p = T.lane[sl][decltype(Qc)::value];
          if constexpr (p / 15 == h) v += sb[(p - 15 * h) * 68 + lane];
        });
        acc[sl] = v;
#if ECNF_PAIR_NODE_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
      });
      asm volatile("" ::: "memory");
    });
    static_for<T.nn>([&](auto Sc) {
      constexpr int sl = decltype(Sc)::value;
      lds_add(mrows + T.node[sl] * s.ld_m + pass * 64, acc[sl]);
    });
  });
}

// shift_i += sum over atom i's pairs of +-phi_x r / (C + |r|) (egnn.py:87-94) for pair tile TP, and the tangent shifts
// (V = D or 2 D values per pair: the tangent of shift_ji = -shift_ij is -dshift_ij): rows of 16 floats [+v | -v],
// lanes d < V sum each atom's pairs (fixed order) into dxacc (tangent values into the rows RP + n)
template <int TP, int V, int D>
__device__ __forceinline__ void pair_shift_tile(const Lds& s, const float (&sh)[V], int mol, int rp, float* sb, int lane) {
  static_assert(V <= 8 && (V == D || V == 2 * D), "primal, or primal + tangent shifts");
  constexpr PairPlan13::Tile T = PairPlan13::make(TP);
  const int kk = lane >> 5, li = lane & 31;
  if (kk == 0) {
    f32x4 pv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, nv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int d = 0; d < V; ++d) {
      pv[d >> 2][d & 3] = sh[d];
      nv[d >> 2][d & 3] = -sh[d];
    }
    static_for<(V + 3) / 4>([&](auto Hc) {
      constexpr int hh = decltype(Hc)::value;
      *reinterpret_cast<f32x4*>(sb + li * 16 + 4 * hh) = pv[hh];
      *reinterpret_cast<f32x4*>(sb + li * 16 + 8 + 4 * hh) = nv[hh];
    });
  }
  asm volatile("" ::: "memory");
  if (lane < V) {
    const int row = lane < D ? mol * PairPlan13::kN : rp + mol * PairPlan13::kN, d = lane < D ? lane : lane - D;
    static_for<T.nn>([&](auto Sc) {
      constexpr int sl = decltype(Sc)::value;
      float v = 0.f;
      static_for<T.deg[sl]>([&](auto Qc) {
        constexpr int q = decltype(Qc)::value;
        v += sb[T.lane[sl][q] * 16 + T.role[sl][q] * 8 + lane];
      });
      lds_add(&s.dxacc[(row + T.node[sl]) * D + d], v);
    });
  }
  asm volatile("" ::: "memory");
}

// m e to both atoms of each pair (primal rows), and for NT = 1 its tangent gT m + g mT (rows RP + n)
template <int NF, int NT>
__device__ __forceinline__ void pair_agg(const Lds& s, const f32x16 (&m)[NF], const f32x16 (&mT)[NF], float g, float gT,
                                         const PairCtx& pc, int lane) {
  auto prim = [&](int fb, int r) { return m[fb][r] * g; };
  auto tang = [&](int fb, int r) { return gT * m[fb][r] + g * mT[fb][r]; };
  auto one = [&](auto Tc) {
    constexpr int TP = decltype(Tc)::value;
    pair_agg_tile<TP, NF>(s, prim, pc.mol, 0, pc.sb, lane);
    if constexpr (NT) pair_agg_tile<TP, NF>(s, tang, pc.mol, pc.rp, pc.sb, lane);
  };
  if (pc.tp == 0) one(std::integral_constant<int, 0>{});
  else if (pc.tp == 1) one(std::integral_constant<int, 1>{});
  else one(std::integral_constant<int, 2>{});
}

template <int V, int D>
__device__ __forceinline__ void pair_shift(const Lds& s, const float (&sh)[V], const PairCtx& pc, int lane) {
  if (pc.tp == 0) pair_shift_tile<0, V, D>(s, sh, pc.mol, pc.rp, pc.sb, lane);
  else if (pc.tp == 1) pair_shift_tile<1, V, D>(s, sh, pc.mol, pc.rp, pc.sb, lane);
  else pair_shift_tile<2, V, D>(s, sh, pc.mol, pc.rp, pc.sb, lane);
}

// phi_x output Dense(1) (egnn.py:83-85), shifts_ij = phi_x * r_ij / (C + |r_ij|) and their segment sum
// (egnn.py:87-94)
template <int NF, int NT, int L, int D>
__device__ __forceinline__ void edge_shift(const Net& net, const BlockW& bw, const Lds& s, const f32x16 (&px)[NF],
                                           const f32x16 (&pxT)[NF], bool writer, const SegScan& sc, int rr,
                                           const float (&r)[D], const float (&dr)[D], float length, float dlength,
                                           int lane, bool pw = true) {
  const int kk = lane >> 5;
  float phx, phxT;
  lds_dot<NF, NT>(s.vecs + (2 * L + 1) * (NF * 32), px, pxT, kk, phx, phxT);
  phx += __shfl_xor(phx, 32);
  if constexpr (NT) phxT += __shfl_xor(phxT, 32);
  phx += bw.bx;
  // full-precision divisions, as the oracle: a reciprocal-multiply form (1 division instead of 2D) moved the DW4
  // exact-trace PID solves outside their fp32-oracle envelope (tests/test_gpu_eval_modes.py; profiles/round5/dw4_envelope) and
  // saved no measurable time
  const float den = net.C + length;
  const int RP = net.RP;
  float sh[2 * D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    sh[d] = (phx * r[d]) / den;
    sh[D + d] = NT ? (phxT * r[d] + phx * dr[d]) / den - (phx * r[d]) * dlength / (den * den) : 0.f;
  }
  sc.sum_many<2 * D>(sh);
  if (writer && kk == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (pw) lds_add(&s.dxacc[rr * D + d], sh[d]);
      if constexpr (NT) lds_add(&s.dxacc[(RP + rr) * D + d], sh[D + d]);
    }
  }
}

// gate, message aggregation, phi_x torso + output, shifts (egnn.py:81-104); `m` holds the messages.
// pw = false: the tile's primal outputs are computed (the tangents need them) but not stored (exact-trace block-1
// dual tiles, whose edges' primal contributions come from the primal tiles)
template <int NF, int NT, int L, int D, typename PhiX>
__device__ __forceinline__ void edge_tail(const Net& net, const BlockW& bw, const Lds& s, f32x16 (&X)[NF],
                                          f32x16 (&XT)[NF], bool valid, int rr, float* agg_dst,
                                          const float (&r)[D], const float (&dr)[D], float length, float dlength,
                                          int lane, bool agg, PhiX&& phi_x, bool pw = true) {
  f32x16(&m)[NF] = X;
  f32x16(&mT)[NF] = XT;
  const int kk = lane >> 5, li = lane & 31;
  SegScan sc;
  sc.init(valid ? rr : -1, li);
  const bool writer = valid && sc.tail;
  const int RP = net.RP;
  // the gate and the message aggregate only feed phi_h, i.e. h, which the last block's caller never reads (v depends
  // on x alone, egnn.py:176-188): agg == false skips them (wave-uniform)
  if (agg) {
  // gate e_ij = sigmoid(m_ij . w_g + b_g)  (egnn.py:99-101)
  float part, partT;
  lds_dot<NF, NT>(s.vecs + (2 * L) * (NF * 32), m, mT, kk, part, partT);
  part += __shfl_xor(part, 32);
  if constexpr (NT) partT += __shfl_xor(partT, 32);
  const float g = sigmoidf_(part + bw.bg);
  const float gT = NT ? g * (1.0f - g) * partT : 0.f;

  // m_i = scatter_sum(m_ij * e_ij) (the / sqrt(N-1) happens in the node update)   (egnn.py:102-104)
#pragma unroll
  for (int fb = 0; fb < NF; ++fb) {
    float v[16];
#pragma unroll
    for (int r16 = 0; r16 < 16; ++r16) v[r16] = m[fb][r16] * g;
    sc.sum_many<16>(v);
    if (writer && pw) {
      if (agg_dst) {
        // the segment part's sums as 4 x 16-B stores into its own row (no atomics; combined in the node update)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(agg_dst + fb * 32 + 8 * q + 4 * kk) =
              f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      } else {
        agg_rows<NF>(s, rr, kk, fb, v);
      }
    }
    if constexpr (NT) {
#pragma unroll
      for (int r16 = 0; r16 < 16; ++r16) v[r16] = gT * m[fb][r16] + g * mT[fb][r16];
      sc.sum_many<16>(v);
      if (writer) {
        agg_rows<NF>(s, RP + rr, kk, fb, v);
      }
    }
  }
  }  // agg

  // phi_x torso (egnn.py:82) then its Dense(1) and the shifts
  phi_x(X, XT);
  edge_shift<NF, NT, L, D>(net, bw, s, X, XT, writer, sc, rr, r, dr, length, dlength, lane, pw);
}


// edge_shift with block-1 pair tiles (pc.sb != nullptr; the M = 128 split primal kernels only, so no other kernel's
// code changes: a pair context threaded through edge_shift / edge_tail crashed the compiler on the M = 256 strict-fp32
// tangent vf_kernel, AMDGPU Rewrite AGPR-Copy-MFMA).  phi_x output Dense(1) (egnn.py:83-85), shifts_ij = phi_x * r_ij / (C + |r_ij|) and their segment sum
// (egnn.py:87-94)
template <int NF, int NT, int L, int D>
__device__ __forceinline__ void edge_shift_pc(const Net& net, const BlockW& bw, const Lds& s, const f32x16 (&px)[NF],
                                           const f32x16 (&pxT)[NF], bool writer, const SegScan& sc, int rr,
                                           const float (&r)[D], const float (&dr)[D], float length, float dlength,
                                           int lane, bool pw, const PairCtx& pc) {
  const int kk = lane >> 5;
  float phx, phxT;
  lds_dot<NF, NT>(s.vecs + (2 * L + 1) * (NF * 32), px, pxT, kk, phx, phxT);
  phx += __shfl_xor(phx, 32);
  if constexpr (NT) phxT += __shfl_xor(phxT, 32);
  phx += bw.bx;
  // full-precision divisions, as the oracle: a reciprocal-multiply form (1 division instead of 2D) moved the DW4
  // exact-trace PID solves outside their fp32-oracle envelope (tests/test_gpu_eval_modes.py; profiles/round5/dw4_envelope) and
  // saved no measurable time
  const float den = net.C + length;
  const int RP = net.RP;
  float sh[2 * D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    sh[d] = (phx * r[d]) / den;
    sh[D + d] = NT ? (phxT * r[d] + phx * dr[d]) / den - (phx * r[d]) * dlength / (den * den) : 0.f;
  }
  if (pc.sb) {   // block-1 pair tile: +shift (and its tangent) to atom a, -shift to atom b
    float sv[(1 + NT) * D];
#pragma unroll
    for (int d = 0; d < (1 + NT) * D; ++d) sv[d] = sh[d];
    pair_shift<(1 + NT) * D, D>(s, sv, pc, lane);
    return;
  }
  sc.sum_many<2 * D>(sh);
  if (writer && kk == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (pw) lds_add(&s.dxacc[rr * D + d], sh[d]);
      if constexpr (NT) lds_add(&s.dxacc[(RP + rr) * D + d], sh[D + d]);
    }
  }
}

// edge_tail with block-1 pair tiles (edge_shift_pc).  Gate, message aggregation, phi_x torso + output, shifts.
// pw = false: the tile's primal outputs are computed (the tangents need them) but not stored (exact-trace block-1
// dual tiles, whose edges' primal contributions come from the primal tiles)
template <int NF, int NT, int L, int D, typename PhiX>
__device__ __forceinline__ void edge_tail_pc(const Net& net, const BlockW& bw, const Lds& s, f32x16 (&X)[NF],
                                          f32x16 (&XT)[NF], bool valid, int rr, float* agg_dst,
                                          const float (&r)[D], const float (&dr)[D], float length, float dlength,
                                          int lane, bool agg, PhiX&& phi_x, bool pw, const PairCtx& pc) {
  f32x16(&m)[NF] = X;
  f32x16(&mT)[NF] = XT;
  const int kk = lane >> 5, li = lane & 31;
  SegScan sc;
  sc.init(valid ? rr : -1, li);
  const bool writer = valid && sc.tail;
  const int RP = net.RP;
  // the gate and the message aggregate only feed phi_h, i.e. h, which the last block's caller never reads (v depends
  // on x alone, egnn.py:176-188): agg == false skips them (wave-uniform)
  if (agg) {
  // gate e_ij = sigmoid(m_ij . w_g + b_g)  (egnn.py:99-101)
  float part, partT;
  lds_dot<NF, NT>(s.vecs + (2 * L) * (NF * 32), m, mT, kk, part, partT);
  part += __shfl_xor(part, 32);
  if constexpr (NT) partT += __shfl_xor(partT, 32);
  const float g = sigmoidf_(part + bw.bg);
  const float gT = NT ? g * (1.0f - g) * partT : 0.f;

  // m_i = scatter_sum(m_ij * e_ij) (the / sqrt(N-1) happens in the node update)   (egnn.py:102-104)
  if (pc.sb) {   // block-1 pair tile: each pair's m e to both of its atoms
    pair_agg<NF, NT>(s, m, mT, g, gT, pc, lane);
  } else {
#pragma unroll
  for (int fb = 0; fb < NF; ++fb) {
    float v[16];
#pragma unroll
    for (int r16 = 0; r16 < 16; ++r16) v[r16] = m[fb][r16] * g;
    sc.sum_many<16>(v);
    if (writer && pw) {
      if (agg_dst) {
        // the segment part's sums as 4 x 16-B stores into its own row (no atomics; combined in the node update)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(agg_dst + fb * 32 + 8 * q + 4 * kk) =
              f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      } else {
        agg_rows<NF>(s, rr, kk, fb, v);
      }
    }
    if constexpr (NT) {
#pragma unroll
      for (int r16 = 0; r16 < 16; ++r16) v[r16] = gT * m[fb][r16] + g * mT[fb][r16];
      sc.sum_many<16>(v);
      if (writer) {
        agg_rows<NF>(s, RP + rr, kk, fb, v);
      }
    }
  }
  }  // !pc.sb
  }  // agg

  // phi_x torso (egnn.py:82) then its Dense(1) and the shifts
  phi_x(X, XT);
  edge_shift_pc<NF, NT, L, D>(net, bw, s, X, XT, writer, sc, rr, r, dr, length, dlength, lane, pw, pc);
}


// M = 256 tangent kernels: phi_e.0 on the edge itself, [h_s | h_r | |r|^2] W1 + b1 (egnn.py:76-79; no per-node P
// halves, whose primal + tangent rows would need 132 KB of LDS), as split MFMAs with the node-GEMM fragment layout
// (host-packed -log2(e) W1, K = 2H + 1 zero-padded to 16-deep k-steps): B = 8 consecutive input features of the
// lane's edge, gathered from the hb rows (16-B reads), primal and tangent sharing every A fragment.  Output: the
// log2-domain activation y' = silu_u(u) and its tangent (chain_dual_seq's input form).
template <int NF>
__device__ __forceinline__ void edge_layer1_dual(const Net& net, const BlockW& bw, const Lds& s, int rr, int rs,
                                                 float len2, float dlen2, f32x16 (&X)[NF], f32x16 (&XT)[NF],
                                                 int lane) {
  const int kk = lane >> 5, H = net.H, RP = net.RP;
  const int K = 2 * H + 1, nks = (K + 15) >> 4;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(launder_uniform(bw.W1_s)),
                                                                         (short)0, 0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  auto feat8 = [&](int ks, bool tan, float (&v)[8]) {
    const int c0 = 16 * ks + 8 * kk;
    if (c0 + 8 <= 2 * H) {   // h_s or h_r: 8 consecutive features of one hb row (H is a multiple of 32)
      const int row = (c0 < H ? rs : rr) + (tan ? RP : 0);
      const float* src = s.hb + row * s.ld_hb + (c0 < H ? c0 : c0 - H);
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = lo[j];
        v[4 + j] = hi[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (c0 + j == 2 * H) ? (tan ? dlen2 : len2) : 0.f;
    }
  };
#pragma unroll
  for (int jb = 0; jb < NF; ++jb) {
    X[jb] = f32x16{};
    XT[jb] = f32x16{};
  }
  for (int ks = 0; ks < nks; ++ks) {
    float v[8], vt[8];
    feat8(ks, false, v);
    feat8(ks, true, vt);
    u32x4 B[kPieces], BT[kPieces];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned pc[kPieces], pt[kPieces];
      split_pair(v[2 * e], v[2 * e + 1], pc);
      split_pair(vt[2 * e], vt[2 * e + 1], pt);
#pragma unroll
      for (int p = 0; p < kPieces; ++p) {
        B[p][e] = pc[p];
        BT[p][e] = pt[p];
      }
    }
    static_for<NF>([&](auto Jc) {
      constexpr int jb = decltype(Jc)::value;
      u32x4 A[kPieces];
#pragma unroll
      for (int p = 0; p < kPieces; ++p) A[p] = wload(rsrc, voff, ((jb * nks + ks) * kPieces + p) * kPieceBytes);
      static_for<kTerms>([&](auto Tc) {
        constexpr int t = decltype(Tc)::value;
        X[jb] = mfma_split(A[term_w(t)], B[term_x(t)], X[jb]);
        XT[jb] = mfma_split(A[term_w(t)], BT[term_x(t)], XT[jb]);
      });
    });
  }
  // u = acc / s - log2(e) b1, the log2-domain SiLU and its tangent
  constexpr float kNegLn2 = -0.69314718055994531f;
  const float winv = bw.w1inv;
#pragma unroll
  for (int jb = 0; jb < NF; ++jb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b4 = gptr4(bw.bp_u + net.M + jb * 32 + 8 * q + 4 * kk)[0];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * q + e;
        const float u = fmaf(X[jb][r], winv, b4[e]);
        const float du = XT[jb][r] * winv;
        const float rr = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
        const float y = u * rr;
        X[jb][r] = y;
        XT[jb][r] = rr * du * fmaf(u - y, kNegLn2, 1.0f);
      }
    }
}

// ---------------------------------------------------------------------------------------------------
// M = 256 strict-fp32 tangent kernels (Geo::kWideT32): the kWideT edge path on v_mfma_f32_32x32x2_f32.
// ---------------------------------------------------------------------------------------------------
// phi_e.0 per edge in fp32: [h_s | h_r | |r|^2] W1 + b1 (egnn.py:76-79), natural-domain SiLU and its tangent.  A =
// the fp32 kernel rows read in place from the node-GEMM copy Wp = [W_send | W_recv] ([H][2M]) and w_d, B = feature
// k0 + kk of the lane's edge from the hb rows (tangent rows RP + n); primal and tangent share every A value.
template <int NF>
__device__ __forceinline__ void edge_layer1_dual_f32(const Net& net, const BlockW& bw, const Lds& s, int rr, int rs,
                                                     float len2, float dlen2, f32x16 (&X)[NF], f32x16 (&XT)[NF],
                                                     int lane) {
  const int kk = lane >> 5, li = lane & 31, H = net.H, RP = net.RP, M = NF * 32;
#pragma unroll
  for (int jb = 0; jb < NF; ++jb) {
    X[jb] = f32x16{};
    XT[jb] = f32x16{};
  }
  const gfloat_p wp = gptr(launder_uniform(bw.Wp));
  // k-steps of 2 over h_s (columns 0 .. M-1 of Wp) and h_r (columns M .. 2M-1): lane half kk holds feature k0 + kk
  for (int part = 0; part < 2; ++part) {
    const float* hrow = s.hb + (part ? rr : rs) * s.ld_hb + kk;
    const float* hrowT = s.hb + (RP + (part ? rr : rs)) * s.ld_hb + kk;
    const gfloat_p wcol = wp + kk * 2 * M + part * M + li;
    for (int k0 = 0; k0 < H; k0 += 2) {
      const float b = hrow[k0], bt = hrowT[k0];
      static_for<NF>([&](auto Jc) {
        constexpr int jb = decltype(Jc)::value;
        const float a = wcol[k0 * 2 * M + jb * 32];
        X[jb] = mfma32(a, b, X[jb]);
        XT[jb] = mfma32(a, bt, XT[jb]);
      });
    }
  }
  {  // the |r|^2 row (k = 2H on lane half 0; half 1 holds the zero padding k = 2H + 1)
    const float b = kk ? 0.f : len2, bt = kk ? 0.f : dlen2;
    const gfloat_p wd = gptr(launder_uniform(bw.wd)) + li;
    static_for<NF>([&](auto Jc) {
      constexpr int jb = decltype(Jc)::value;
      const float a = kk ? 0.f : wd[jb * 32];
      X[jb] = mfma32(a, b, X[jb]);
      XT[jb] = mfma32(a, bt, XT[jb]);
    });
  }
#pragma unroll
  for (int jb = 0; jb < NF; ++jb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b4 = gptr4(bw.bp + M + jb * 32 + 8 * q + 4 * kk)[0];   // bias [0 | b1]
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * q + e;
        float y, yT;
        silu_dual<1>(X[jb][r] + b4[e], XT[jb][r], y, yT);
        X[jb][r] = y;
        XT[jb][r] = yT;
      }
    }
}

// one fp32 pass of a chain layer: acc[jb] = sum over fb of W[l][jb][fb] X[fb] (16 k-steps of 2 per 32-row input
// block), the fp32 fragments of chain_segment ([layer][jb][fb][q][lane][4]) streamed PF groups ahead
template <int NF>
__device__ __forceinline__ void dual_pass_f32(const f32x16 (&X)[NF], f32x16 (&acc)[NF], gf32x4_p wl) {
  constexpr int G = NF * NF, PF = 2;
  f32x4 wbuf[PF + 1][4];
  static_for<PF>([&](auto Gc) {
    constexpr int gg = decltype(Gc)::value;
#pragma unroll
    for (int q = 0; q < 4; ++q) wbuf[gg][q] = wl[(gg * 4 + q) * 64];
  });
  static_for<G>([&](auto Gc) {
    constexpr int gg = decltype(Gc)::value;
    constexpr int jb = gg / NF, fb = gg % NF;   // group (jb, fb) sits at wl[((jb * NF + fb) * 4 + q) * 64]
    if constexpr (gg + PF < G) {
#pragma unroll
      for (int q = 0; q < 4; ++q) wbuf[(gg + PF) % (PF + 1)][q] = wl[((gg + PF) * 4 + q) * 64];
    }
    if constexpr (fb == 0) acc[jb] = f32x16{};
    static_for<16>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value;
      acc[jb] = mfma32(wbuf[gg % (PF + 1)][i >> 2][i & 3], X[fb][i], acc[jb]);
    });
    __builtin_amdgcn_sched_barrier(0);
  });
}

// NL chain layers X <- silu(X W + b) with forward-mode tangents, the primal and the tangent in sequential passes
// over the same fp32 fragments (as chain_dual_seq): at most X, XT and one accumulator set (3 x 128 registers) live.
// bias: the natural-domain chain biases staged in LDS ([NL][M]).
template <int NF, int NL>
__device__ __forceinline__ void chain_dual_seq_f32(f32x16 (&X)[NF], f32x16 (&XT)[NF], const float* __restrict__ Wpk,
                                                   const float* __restrict__ bias, int lane) {
  constexpr int M = NF * 32;
  const int kk = lane >> 5;
  for (int l = 0; l < NL; ++l) {
    // the layer's fragments through launder_uniform once per pass: the tangent pass must load them again (plain
    // loads of one address would be merged with the primal pass's, keeping 1024 weight values live across it)
    const size_t loff = (size_t)l * NF * NF * 4 * 64 + lane;
    f32x16 acc[NF];
    dual_pass_f32<NF>(X, acc, gptr4(launder_uniform(Wpk)) + loff);    // acc = W X
    __builtin_amdgcn_sched_barrier(0);
    dual_pass_f32<NF>(XT, X, gptr4(launder_uniform(Wpk)) + loff);     // X (dead after the primal pass) <- W X_T
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int fb = 0; fb < NF; ++fb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + l * M + fb * 32 + 8 * q + 4 * kk);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * q + e;
          float y, yT;
          silu_dual<1>(acc[fb][r] + b4[e], X[fb][r], y, yT);
          X[fb][r] = y;
          XT[fb][r] = yT;
        }
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// one 32-edge tile through phi_e / gate / phi_x  (egnn.py:72-95)
// a >= 0 (split tangent kernels only, exact trace, egnn_eval sparse_a): `tile` is a molecule and the tile is dual
// tile `part` of 2(N - 1) edges of that molecule, in receiver-major order, storing tangent outputs only.
//   amode 1 (block 1): the edges at atom a (receivers i < a with sender a, receiver a with its N - 1 senders in
//                      graph.py order, receivers i > a with sender a)
//   amode 2 (last block): the edges INTO atoms 0 and a (receiver 0's N - 1 edges, then receiver a's; a >= 1)
// WPP: weight pieces of the primal split chain (kSplit branch): 2 in the primal kernels, 3 (exact weights, as the
// dual tiles' primal) for the exact trace's primal-only tiles inside the divergence kernels
template <int NF, int NT, int L, int D, int P, int WPP = kPieces, bool BN = false>
__device__ __forceinline__ void edge_tile(const Net& net, const BlockW& bw, const Lds& s, int tile, int lane, bool agg,
                                          int a = -1, int part = 0, int amode = 1, float* psb = nullptr) {
  const int kk = lane >> 5, li = lane & 31;
  const int N = net.N, nn1 = N - 1, RP = net.RP, M = NF * 32;
  int mol, i, sd;
  bool valid;
  PairCtx pctx{0, 0, psb, net.RP};
  if (psb) {
    // block-1 pair tile (PairPlan13): tile = 3 molecule + pair tile; lane = pair (a, b), r = x_a - x_b
    mol = tile / PairPlan13::kTiles;
    pctx.mol = mol;
    pctx.tp = tile - PairPlan13::kTiles * mol;
    const unsigned code = pair13_code(pctx.tp, li);
    valid = (mol < net.MPW) && code != 0xFFu;
    i = valid ? (int)(code & 15u) : 0;
    sd = valid ? (int)(code >> 4) : 1;
  } else if (a < 0) {
    // each molecule owns EP = 32*ceil(E/32) edge slots, so its tiles (and every rounding inside them) do not
    // depend on which slot of the workgroup, i.e. which batch position, it occupies
    mol = (tile * 32) / net.EP;
    const int e_in = tile * 32 + li - mol * net.EP;
    const int i0 = e_in / net.SR, j0 = e_in - i0 * net.SR;   // receiver, slot (receiver-tiled: j0 >= N - 1 is padding)
    valid = (mol < net.MPW) && (i0 < N) && (j0 < nn1);
    i = valid ? i0 : 0;
    sd = i + 1 + (valid ? j0 : 0);
    if (sd >= N) sd -= N;
  } else {
    ECNF_DCHECK((Geo<NF, NT, P, BN>::kL2T && tile < net.MPW && a < N), 6);
    mol = tile;
    const int q = part * 32 + li;
    valid = q < 2 * nn1;
    if (amode == 2) {   // receiver 0 (senders 1 .. N - 1), then receiver a (senders (a + 1 + j) mod N)
      i = q < nn1 ? 0 : a;
      sd = q < nn1 ? q + 1 : a + 1 + (q - nn1);
      if (sd >= N) sd -= N;
    } else if (q < a) {
      i = q;
      sd = a;
    } else if (q < a + nn1) {   // receiver a, sender (a + 1 + j) mod N with j = q - a
      i = a;
      sd = q + 1 < N ? q + 1 : q + 1 - N;
    } else {
      i = q - nn1 + 1;
      sd = a;
    }
    if (!valid) {
      i = 0;
      sd = 1;
    }
  }
  const int mrow = valid ? mol : 0;
  const int rr = mrow * N + i, rs = mrow * N + sd;   // receiver / sender rows (graph.py:10-13)
  ECNF_DCHECK(rr < net.MPW * N && rs < net.MPW * N && rr >= 0 && rs >= 0, 1);
  ECNF_DCHECK(tile * 32 < net.MPW * net.EP, 2);
  // split kernels: the row this lane's receiver-segment part is stored to — macc for the part in the tile where
  // the segment starts, the cross buffer (one row per molecule tile) for its continuation in the next tile
  float* agg_dst = nullptr;
  if constexpr (Geo<NF, NT, P, BN>::kSplit) {
    if (net.cross && !psb) {
      const int tloc = tile - mrow * (net.EP >> 5);
      agg_dst = tloc == ((i * nn1) >> 5) ? s.macc + rr * s.ld_m : s.cross + (mrow * (net.EP >> 5) + tloc) * s.ld_m;
      ECNF_DCHECK(tloc >= 0 && mrow * (net.EP >> 5) + tloc < net.MPW * (net.EP >> 5), 4);
    }
  }
#ifdef ECNF_STAMPS
  unsigned long long t_sub = __builtin_amdgcn_s_memtime();
#endif

  // r_ij = x_i - x_j, lengths = safe_norm (egnn.py:73-74, numerical.py:7-10)
  float r[D], dr[D];
  float x2 = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    r[d] = s.xc[rr * D + d] - s.xc[rs * D + d];
    x2 += r[d] * r[d];
  }
  const bool zero = (x2 == 0.f);
  const float length = sqrtf(zero ? 1.0f : x2);
  const float len2 = length * length;
  float dlength = 0.f, dlen2 = 0.f;
  if constexpr (NT) {
    float rdr = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      dr[d] = s.xc[(RP + rr) * D + d] - s.xc[(RP + rs) * D + d];
      rdr += r[d] * dr[d];
    }
    dlength = zero ? 0.f : rdr / length;
    dlen2 = 2.0f * length * dlength;
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) dr[d] = 0.f;
  }

  if constexpr (Geo<NF, NT, P, BN>::kSplit) {
    // phi_e layer 1 from the per-node halves: pre = P_s[s] + P_r[r] + |r|^2 w_d  (egnn.py:76,79), SiLU, split
    SplitX<NF> XA, XB;
    f32x16 acc[NF];
    // (pair tiles: the molecule's P row copied to hin before the edge phase; the P rows hold the waves' slices)
    const float* Ps = psb ? s.hin + mrow * 2 * M : s.P + rs * s.ld_P;
    const float* Pr = psb ? s.hin + mrow * 2 * M + M : s.P + rr * s.ld_P + M;
    // 4 NF rounds of 4 consecutive features (16-B LDS reads of w_d, P_s, P_r), two rounds per step behind
    // scheduling fences with the next step's reads issued first: the per-round read -> s_waitcnt lgkmcnt(0) ->
    // 2-element SiLU chain form exposed the LDS latency and a wait state after every transcendental
    constexpr int NQ = 4 * NF, GQ = 2, NG = NQ / GQ;
    auto rd3 = [&](int q, f32x4 (&o)[3]) {
      const int row = (q >> 2) * 32 + 8 * (q & 3) + 4 * kk;
      o[0] = *reinterpret_cast<const f32x4*>(s.vecs + (2 * L - 1) * (NF * 32) + row);
      o[1] = *reinterpret_cast<const f32x4*>(Ps + row);
      o[2] = *reinterpret_cast<const f32x4*>(Pr + row);
    };
    f32x4 lb[2][GQ][3];
    static_for<GQ>([&](auto Ic) { rd3(decltype(Ic)::value, lb[0][decltype(Ic)::value]); });
    static_for<NG>([&](auto Gc) {
      constexpr int g = decltype(Gc)::value;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (g + 1 < NG)
        static_for<GQ>([&](auto Ic) { rd3((g + 1) * GQ + decltype(Ic)::value, lb[(g + 1) & 1][decltype(Ic)::value]); });
      static_for<GQ>([&](auto Ic) {
        constexpr int q = g * GQ + decltype(Ic)::value, fb = q >> 2, qq = q & 3;
        const f32x4(&o)[3] = lb[g & 1][decltype(Ic)::value];
        static_for<2>([&](auto Hc) {
          constexpr int e = 2 * decltype(Hc)::value;
          const float u0 = o[1][e] + o[2][e] + len2 * o[0][e];   // log2 domain (silu_u)
          const float u1 = o[1][e + 1] + o[2][e + 1] + len2 * o[0][e + 1];
          put_pair<NF, fb, 4 * qq + e>(XA, silu_u(u0), silu_u(u1));
        });
      });
    });
    __builtin_amdgcn_sched_barrier(0);
    STAMP_LANE0(s, kStEdgeLayer1, t_sub);
    // phi_e layers 2..L
    const unsigned* Ws = launder_uniform(WPP == 3 ? bw.Ws3 : bw.Ws);
    const float* ci = bw.cinv;
    ChainInv ie, ix;
    static_for<2 * 4 - 1>([&](auto Lc) {
      constexpr int l = decltype(Lc)::value;
      ie.v[l] = l < L - 1 ? ci[l] : 1.0f;
      ix.v[l] = l < L ? ci[L - 1 + l] : 1.0f;
    });
    chain_split<NF, L - 1, WPP>(XA, XB, acc, Ws, s.vecs, ie, lane);
    STAMP_LANE0(s, kStEdgeChainE, t_sub);
    // phi_x layers 1..L on the (ungated) messages
    auto phi_x = [&](f32x16 (&m)[NF], f32x16 (&)[NF]) {
      STAMP_LANE0(s, kStEdgeAgg, t_sub);
      static_for<NF>([&](auto Fc) {
        constexpr int fb = decltype(Fc)::value;
        static_for<8>([&](auto Ic) {
          constexpr int i = decltype(Ic)::value;
          put_pair<NF, fb, 2 * i>(XA, m[fb][2 * i], m[fb][2 * i + 1]);
        });
      });
      const unsigned* Wx = launder_uniform((WPP == 3 ? bw.Ws3 : bw.Ws) + (size_t)(L - 1) * SplitPlan<NF, 1>::GL * WPP * 256);
      STAMP_LANE0(s, kStEdgePhiXIn, t_sub);
      chain_split<NF, L, WPP>(XA, XB, m, Wx, s.vecs + (L - 1) * NF * 32, ix, lane);
      STAMP_LANE0(s, kStEdgePhiX, t_sub);
    };
    // (one call site, the pair tiles branching inside the tail: two, each with its own copy of the phi_x chain, spilled)
    if constexpr (NT == 0 && NF == 4)
      edge_tail_pc<NF, NT, L, D>(net, bw, s, acc, acc, valid, rr, agg_dst, r, dr, length, dlength, lane, agg, phi_x,
                                 true, pctx);
    else
      edge_tail<NF, NT, L, D>(net, bw, s, acc, acc, valid, rr, agg_dst, r, dr, length, dlength, lane, agg, phi_x);
    STAMP_LANE0(s, kStEdgeTail, t_sub);
    return;
  }
  if constexpr (Geo<NF, NT, P, BN>::kL2T) {
    // phi_e.0 from the log2-domain per-node halves: u = P_s[s] + P_r[r] + |r|^2 w_d', y' = u / (1 + 2^u) and its
    // tangent dy' = r du (1 - ln2 (u - y')), split straight into the chain's input buffers (16-B LDS reads)
    constexpr float kNegLn2 = -0.69314718055994531f;
    SplitX<NF> XA, XB, XAT, XBT;
    f32x16 X[NF], XT[NF];
    // (pair tiles: the molecule's primal and tangent P rows copied to hin, as the primal kernels')
    const float* pcp = s.hin + mrow * 2 * M;
    const float* pct = s.hin + (net.MPW + mrow) * 2 * M;
    const float* Ps = psb ? pcp : s.P + rs * s.ld_P;
    const float* Pr = psb ? pcp + M : s.P + rr * s.ld_P + M;
    const float* PsT = psb ? pct : s.P + (RP + rs) * s.ld_P;
    const float* PrT = psb ? pct + M : s.P + (RP + rr) * s.ld_P + M;
    // as the primal split kernels: one round of 4 features per fenced step, the next round's 5 reads issued first
    constexpr int NQ = 4 * NF;
    auto rd5 = [&](int q, f32x4 (&o)[5]) {
      const int row = (q >> 2) * 32 + 8 * (q & 3) + 4 * kk;
      o[0] = *reinterpret_cast<const f32x4*>(s.vecs + (2 * L - 1) * (NF * 32) + row);
      o[1] = *reinterpret_cast<const f32x4*>(Ps + row);
      o[2] = *reinterpret_cast<const f32x4*>(Pr + row);
      o[3] = *reinterpret_cast<const f32x4*>(PsT + row);
      o[4] = *reinterpret_cast<const f32x4*>(PrT + row);
    };
    f32x4 lb[2][5];
    rd5(0, lb[0]);
    static_for<NQ>([&](auto Qc) {
      constexpr int q = decltype(Qc)::value, fb = q >> 2, qq = q & 3;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (q + 1 < NQ) rd5(q + 1, lb[(q + 1) & 1]);
      const f32x4(&o)[5] = lb[q & 1];
      static_for<2>([&](auto Hc) {
        constexpr int e = 2 * decltype(Hc)::value;
        float y[2], d[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float u = o[1][e + h] + o[2][e + h] + len2 * o[0][e + h];
          const float du = o[3][e + h] + o[4][e + h] + dlen2 * o[0][e + h];
          const float r = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
          y[h] = u * r;
          d[h] = r * du * fmaf(u - y[h], kNegLn2, 1.0f);
        }
        put_pair<NF, fb, 4 * qq + e>(XA, y[0], y[1]);
        put_pair<NF, fb, 4 * qq + e>(XAT, d[0], d[1]);
      });
    });
    __builtin_amdgcn_sched_barrier(0);
    STAMP_LANE0(s, kStEdgeLayer1, t_sub);
    ChainInv ie, ix;
    static_for<2 * 4 - 1>([&](auto Lc) {
      constexpr int l = decltype(Lc)::value;
      ie.v[l] = l < L - 1 ? bw.cinv[l] : 1.0f;
      ix.v[l] = l < L ? bw.cinv[L - 1 + l] : 1.0f;
    });
    chain_split<NF, L - 1, 1, 3>(XA, XB, X, launder_uniform(bw.Ws3), s.vecs, ie, lane, XAT, XBT, XT);
    STAMP_LANE0(s, kStEdgeChainE, t_sub);
    // the tail stays in the log2 domain as in the primal split kernels: gate / shift with the -ln2-folded w_g', w_x'
    // (staged in vecs), the aggregate's -ln2 / sqrt(N-1) in the split phi_h.0 weights, phi_x fed the messages as is
    auto phi_x = [&](f32x16 (&Y)[NF], f32x16 (&YT)[NF]) {
      STAMP_LANE0(s, kStEdgeAgg, t_sub);
      const unsigned* Wx = launder_uniform(bw.Ws3 + (size_t)(L - 1) * SplitPlan<NF, 1>::GL * 3 * 256);
      static_for<NF>([&](auto Fc) {
        constexpr int fb = decltype(Fc)::value;
        static_for<8>([&](auto Ic) {
          constexpr int i = decltype(Ic)::value;
          put_pair<NF, fb, 2 * i>(XA, Y[fb][2 * i], Y[fb][2 * i + 1]);
          put_pair<NF, fb, 2 * i>(XAT, YT[fb][2 * i], YT[fb][2 * i + 1]);
        });
      });
      STAMP_LANE0(s, kStEdgePhiXIn, t_sub);
      chain_split<NF, L, 1, 3>(XA, XB, Y, Wx, s.vecs + (L - 1) * NF * 32, ix, lane, XAT, XBT, YT);
      STAMP_LANE0(s, kStEdgePhiX, t_sub);
    };
    // (a < 0: block-1 dual tiles of the exact trace store tangents only)
    if constexpr (NF == 4)
      edge_tail_pc<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg, phi_x,
                                 a < 0, pctx);
    else
      edge_tail<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg, phi_x, a < 0);
    STAMP_LANE0(s, kStEdgeTail, t_sub);
    return;
  }
  if constexpr (Geo<NF, NT, P, BN>::kWideT) {
    // M = 256 tangent kernels: phi_e.0 per edge, then the sequential dual chains (chain_dual_seq)
    f32x16 X[NF], XT[NF];
    edge_layer1_dual<NF>(net, bw, s, rr, rs, len2, dlen2, X, XT, lane);
    STAMP_LANE0(s, kStEdgeLayer1, t_sub);
    chain_dual_seq<NF, L - 1>(X, XT, launder_uniform(bw.Ws3), s.vecs, bw.cinv, lane, true);
    STAMP_LANE0(s, kStEdgeChainE, t_sub);
    edge_tail<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg,
                            [&](f32x16 (&Y)[NF], f32x16 (&YT)[NF]) {
                              const unsigned* Wx =
                                  launder_uniform(bw.Ws3 + (size_t)(L - 1) * SplitPlan<NF, 1>::GL * 3 * 256);
                              chain_dual_seq<NF, L>(Y, YT, Wx, s.vecs + (L - 1) * NF * 32, bw.cinv + (L - 1), lane,
                                                    false);
                            });
    STAMP_LANE0(s, kStEdgeTail, t_sub);
    return;
  }
  if constexpr (Geo<NF, NT, P, BN>::kWideT32) {
    // the same in strict fp32 (natural-domain activations and biases, the fp32 chain fragments)
    f32x16 X[NF], XT[NF];
    edge_layer1_dual_f32<NF>(net, bw, s, rr, rs, len2, dlen2, X, XT, lane);
    STAMP_LANE0(s, kStEdgeLayer1, t_sub);
    chain_dual_seq_f32<NF, L - 1>(X, XT, launder_uniform(bw.We), s.vecs, lane);
    STAMP_LANE0(s, kStEdgeChainE, t_sub);
    edge_tail<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg,
                            [&](f32x16 (&Y)[NF], f32x16 (&YT)[NF]) {
                              const float* Wx = launder_uniform(bw.We + (size_t)(L - 1) * NF * NF * 1024);
                              chain_dual_seq_f32<NF, L>(Y, YT, Wx, s.vecs + (L - 1) * NF * 32, lane);
                            });
    STAMP_LANE0(s, kStEdgeTail, t_sub);
    return;
  }
  // phi_e layer 1 from the per-node halves: pre = P_s[s] + P_r[r] + |r|^2 w_d  (egnn.py:76,79)
  f32x16 X[NF], XT[NF];
  const float* Ps = s.P + rs * s.ld_P;
  const float* Pr = s.P + rr * s.ld_P + M;
  const float* PsT = s.P + (RP + rs) * s.ld_P;
  const float* PrT = s.P + (RP + rr) * s.ld_P + M;
#pragma unroll
  for (int fb = 0; fb < NF; ++fb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(s.vecs + (2 * L - 1) * (NF * 32) + fb * 32 + 8 * q + 4 * kk);
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int row = fb * 32 + 8 * q + 4 * kk + e4;
        const float p = Ps[row] + Pr[row] + len2 * w[e4];
        float y, yT = 0.f;
        if constexpr (NT) {
          const float pT = PsT[row] + PrT[row] + dlen2 * w[e4];
          silu_dual<NT>(p, pT, y, yT);
          XT[fb][4 * q + e4] = yT;
        } else {
          silu_dual<NT>(p, 0.f, y, yT);
        }
        X[fb][4 * q + e4] = y;
      }
    }
  STAMP_LANE0(s, kStEdgeLayer1, t_sub);
  // phi_e layers 2..L.  The weight pointer is laundered through an empty asm so the (tile-invariant) weight
  // loads are not hoisted out of the tile loop into thousands of live registers.
  if constexpr (Geo<NF, NT, P, BN>::kSplitT) {
    // split-fp16 chains with tangents (chain_split_tangent; the staged chain biases are the log2-domain copies)
    ChainInv ie, ix;
    static_for<2 * 4 - 1>([&](auto Lc) {
      constexpr int l = decltype(Lc)::value;
      ie.v[l] = l < L - 1 ? bw.cinv[l] : 1.0f;
      ix.v[l] = l < L ? bw.cinv[L - 1 + l] : 1.0f;
    });
    chain_split_tangent<NF, L - 1>(X, XT, launder_uniform(bw.Ws3), s.vecs, ie, lane);
    STAMP_LANE0(s, kStEdgeChainE, t_sub);
    edge_tail<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg,
                            [&](f32x16 (&Y)[NF], f32x16 (&YT)[NF]) {
                              const unsigned* Wx =
                                  launder_uniform(bw.Ws3 + (size_t)(L - 1) * SplitPlan<NF, 1>::GL * 3 * 256);
                              chain_split_tangent<NF, L>(Y, YT, Wx, s.vecs + (L - 1) * NF * 32, ix, lane);
                            });
  } else {
  const float* We = launder_uniform(bw.We);
  chain_segment<NF, NT, L - 1>(X, XT, We, s.vecs, lane);
  STAMP_LANE0(s, kStEdgeChainE, t_sub);
  edge_tail<NF, NT, L, D>(net, bw, s, X, XT, valid, rr, agg_dst, r, dr, length, dlength, lane, agg,
                          [&](f32x16 (&Y)[NF], f32x16 (&YT)[NF]) {
                            const float* Wx = launder_uniform(bw.We + (L - 1) * NF * NF * 1024);
                            chain_segment<NF, NT, L>(Y, YT, Wx, s.vecs + (L - 1) * NF * 32, lane);
                          });
  }
  STAMP_LANE0(s, kStEdgeTail, t_sub);
}

// ---------------------------------------------------------------------------------------------------
// Column-split team mode (team cols; the M = 256 split primal kernels, kColsNW = 8 waves): every member
// workgroup of a molecule's team runs ONE edge tile per block, and its waves split each chain layer of that tile by
// output block (wave w: blocks [w NJ, (w + 1) NJ), NJ = NF / kColsNW), exchanging the layer through an LDS image (Lds::xs): split pieces
// in the MFMA B-operand layout between layers, fp32 after a segment's last layer.  Per output element the arithmetic
// is chain_split's (the same MFMA sequence from the bias column, the same log2-domain SiLU, pair split and fp32 last
// layer), and the gate / phi_x-output dot products read the whole fp32 layer back and sum in the batch order
// (edge_tail, edge_shift), so a cols-mode solve is bitwise equal to the batch path's.
// ---------------------------------------------------------------------------------------------------
// column-split team mode: the LDS image of one chain layer of the tile, [NF][2][pieces][64] u32x4 split pieces or
// [NF][4][64] f32x4, right after the feature ids (carve_lds; Net::xs_floats).  Derived from the carve-up where it is
// used, not held in Lds (one more pointer there spilled in the single-evaluation vf_kernel)
__device__ __forceinline__ float* lds_xs(const Net& net, const Lds& s) {
  return reinterpret_cast<float*>(s.feat) + align4(net.MPW * net.N);
}

// the whole split layer image -> registers (u32x4 [fb][u][piece] at ((fb 2 + u) pieces + piece) 64 + lane)
template <int NF>
__device__ __forceinline__ void xs_load(const float* xs, SplitX<NF>& X, int lane) {
  const u32x4* p = reinterpret_cast<const u32x4*>(xs);
  static_for<NF>([&](auto Fc) {
    constexpr int fb = decltype(Fc)::value;
    static_for<2>([&](auto Uc) {
      constexpr int u = decltype(Uc)::value;
      static_for<kPieces>([&](auto Pc) {
        constexpr int pc = decltype(Pc)::value;
        X.v[fb][u][pc] = p[((fb * 2 + u) * kPieces + pc) * 64 + lane];
      });
    });
  });
}

// fp32 accumulator-layout block fb <-> the image (f32x4 [fb][q] at (fb 4 + q) 64 + lane: registers 4q .. 4q + 3)
__device__ __forceinline__ void mi_store(float* xs, const f32x16& a, int fb, int lane) {
  f32x4* p = reinterpret_cast<f32x4*>(xs);
  static_for<4>([&](auto Qc) {
    constexpr int q = decltype(Qc)::value;
    p[(fb * 4 + q) * 64 + lane] = f32x4{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
  });
}
template <int NF>
__device__ __forceinline__ void mi_load(const float* xs, f32x16 (&m)[NF], int lane) {
  const f32x4* p = reinterpret_cast<const f32x4*>(xs);
  static_for<NF>([&](auto Fc) {
    constexpr int fb = decltype(Fc)::value;
    static_for<4>([&](auto Qc) {
      constexpr int q = decltype(Qc)::value;
      const f32x4 v = p[(fb * 4 + q) * 64 + lane];
      m[fb][4 * q] = v[0];
      m[fb][4 * q + 1] = v[1];
      m[fb][4 * q + 2] = v[2];
      m[fb][4 * q + 3] = v[3];
    });
  });
}

// the log2-domain SiLU of this wave's blocks (chain_split stages A-C: y' = u r, r = 1 / (1 + 2^u)); SPLIT: the pairs
// split into the image's pieces (the next layer's input), else fp32 in place (a segment's last layer)
template <int NJ, bool SPLIT>
__device__ __forceinline__ void cols_act(f32x16 (&acc)[NJ], float* xs, int j0, int lane) {
  u32x4* p = reinterpret_cast<u32x4*>(xs);
  static_for<NJ>([&](auto Jc) {
    constexpr int jj = decltype(Jc)::value;
    static_for<2>([&](auto Uc) {
      constexpr int u = decltype(Uc)::value;
      u32x4 w[kPieces];
      static_for<4>([&](auto Wc) {
        constexpr int wd = decltype(Wc)::value, r = 8 * u + 2 * wd;
        const f32x2 uv = {acc[jj][r], acc[jj][r + 1]};
        f32x2 ev = {__builtin_amdgcn_exp2f(uv[0]), __builtin_amdgcn_exp2f(uv[1])};
        const f32x2 sv = ev + 1.0f;
        ev[0] = __builtin_amdgcn_rcpf(sv[0]);
        ev[1] = __builtin_amdgcn_rcpf(sv[1]);
        const f32x2 yv = uv * ev;
        if constexpr (SPLIT) {
          unsigned pc[kPieces];
          split_pair(yv[0], yv[1], pc);
#pragma unroll
          for (int i = 0; i < kPieces; ++i) w[i][wd] = pc[i];
        } else {
          acc[jj][r] = yv[0];
          acc[jj][r + 1] = yv[1];
        }
      });
      if constexpr (SPLIT) {
#pragma unroll
        for (int i = 0; i < kPieces; ++i) p[(((j0 + jj) * 2 + u) * kPieces + i) * 64 + lane] = w[i];
      }
    });
  });
}

constexpr int kColsPF = 8;   // weight groups in flight per wave in the column-split chain (its fragments come from L2)
// NL chained layers on the tile, the waves split by output block (wave w: blocks j0 .. j0 + NJ - 1, j0 = w NJ).
// Input: the full split layer X (registers; also in the image); output: the last layer's fp32 activations of EVERY
// block in m (read back from the image).  Per layer and block the MFMA sequence of chain_split (kBI: C = the bias
// column, then the k-steps (fb, u) in order, three cross terms each, smallest first) and its activation; two
// workgroup barriers per layer (after the MFMAs: every wave has read the image; after the stores).  The wave's
// weight groups (chain_split's packed layout: [layer][jb][fb][u][piece], 1 KiB per piece) stream as ONE sequence over
// the layers, kColsPF groups ahead, so the next layer's first fragments are in flight across the barriers and
// the activation (each wave reads its own blocks' fragments from L2: nothing is shared in L1 as in the batch path).
template <int NF, int NL>
__device__ __forceinline__ void cols_segment(SplitX<NF>& X, f32x16 (&m)[NF], const unsigned* __restrict__ W,
                                             const float* bias, float* xs, int wave, int lane) {
  constexpr int NJ = NF / kColsNW, GB = 2 * NF, GL = GB * NF, NG = NJ * GB, NQ = NL * NG, PF = kColsPF;
  const int j0 = wave * NJ, kk = lane >> 5;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(W), (short)0,
                                                                         0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  const int gbase = __builtin_amdgcn_readfirstlane(j0 * GB);   // this wave's first group of a layer
  // byte offset of the wave's q-th group: layer q / NG, its group q % NG from gbase
  auto woff = [&](int q) { return (((q / NG) * GL + gbase + (q % NG)) * kPieces) * kPieceBytes; };
  u32x4 wbuf[PF + 1][kPieces];
  static_for<PF>([&](auto Qc) {
    constexpr int q = decltype(Qc)::value;
#pragma unroll
    for (int p = 0; p < kPieces; ++p) wbuf[q][p] = wload(rsrc, voff, woff(q) + p * kPieceBytes);
  });
  f32x16 acc[NJ];
  static_for<NQ>([&](auto Qc) {
    constexpr int q = decltype(Qc)::value, l = q / NG, g = q % NG, jj = g / GB, fb = (g % GB) >> 1, u = g & 1;
    if constexpr (g == 0) {   // the layer's accumulators start at its bias column (chain_split kBI)
      static_for<NJ>([&](auto Jc) {
        constexpr int j = decltype(Jc)::value;
        static_for<4>([&](auto Rc) {
          constexpr int r4 = decltype(Rc)::value;
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + l * NF * 32 + 4 * kk + (j0 + j) * 32 + 8 * r4);
          acc[j][4 * r4] = b4[0];
          acc[j][4 * r4 + 1] = b4[1];
          acc[j][4 * r4 + 2] = b4[2];
          acc[j][4 * r4 + 3] = b4[3];
        });
      });
      __builtin_amdgcn_s_setprio(kChainPrio);
    }
    if constexpr (q + PF < NQ) {
#pragma unroll
      for (int p = 0; p < kPieces; ++p) wbuf[(q + PF) % (PF + 1)][p] = wload(rsrc, voff, woff(q + PF) + p * kPieceBytes);
    }
    static_for<kTerms>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      acc[jj] = mfma_split(wbuf[q % (PF + 1)][term_w(t)], X.v[fb][u][term_x(t)], acc[jj]);
    });
    if constexpr (g == NG - 1) {   // the layer's MFMAs are issued: activation and exchange
      __builtin_amdgcn_s_setprio(0);
      __syncthreads();
      if constexpr (l + 1 < NL) {
        cols_act<NJ, true>(acc, xs, j0, lane);
        __syncthreads();
        xs_load<NF>(xs, X, lane);
      } else {
        cols_act<NJ, false>(acc, xs, j0, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) mi_store(xs, acc[j], j0 + j, lane);
        __syncthreads();
        mi_load<NF>(xs, m, lane);
      }
    }
  });
}

// one edge tile of the column-split team mode (all waves of the workgroup; NT = 0, split primal kernels, packed
// receiver runs).  Geometry, layer 1, gate, aggregation and shifts as edge_tile / edge_tail (kSplit path); the
// aggregation of each message block by the wave that owns it, the shifts stored by wave 0.
template <int NF, int L, int D>
__device__ __forceinline__ void edge_tile_cols(const Net& net, const BlockW& bw, const Lds& s, int tile, int wave,
                                               int lane, bool agg) {
  static_assert(NF % kColsNW == 0, "cols mode deals the output blocks over the workgroup's waves");
  constexpr int NJ = NF / kColsNW, M = NF * 32;
  const int kk = lane >> 5, li = lane & 31, j0 = wave * NJ;
  const int N = net.N, nn1 = N - 1;
  const int mol = (tile * 32) / net.EP;
  const int e_in = tile * 32 + li - mol * net.EP;
  const int i0 = e_in / net.SR, jr = e_in - i0 * net.SR;
  const bool valid = (mol < net.MPW) && (i0 < N) && (jr < nn1);
  const int i = valid ? i0 : 0;
  int sd = i + 1 + (valid ? jr : 0);
  if (sd >= N) sd -= N;
  const int mrow = valid ? mol : 0;
  const int rr = mrow * N + i, rs = mrow * N + sd;   // receiver / sender rows (graph.py:10-13)
  float* agg_dst = nullptr;
  if (net.cross) {
    const int tloc = tile - mrow * (net.EP >> 5);
    agg_dst = tloc == ((i * nn1) >> 5) ? s.macc + rr * s.ld_m : s.cross + (mrow * (net.EP >> 5) + tloc) * s.ld_m;
  }
  float r[D], dr[D];
  float x2 = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    r[d] = s.xc[rr * D + d] - s.xc[rs * D + d];
    x2 += r[d] * r[d];
    dr[d] = 0.f;
  }
  const bool zero = (x2 == 0.f);
  const float length = sqrtf(zero ? 1.0f : x2);
  const float len2 = length * length;
  float* xs = lds_xs(net, s);
#ifdef ECNF_STAMPS   // diagnostic build: wave 0's sub-phases (the edge stamp slots of edge_tile)
  unsigned long long t_sub = __builtin_amdgcn_s_memtime();
#endif
  // phi_e layer 1 from the per-node halves for this wave's blocks (egnn.py:76,79): u = P_s[s] + P_r[r] + |r|^2 w_d'
  {
    const float* Ps = s.P + rs * s.ld_P;
    const float* Pr = s.P + rr * s.ld_P + M;
    u32x4* p = reinterpret_cast<u32x4*>(xs);
    static_for<NJ>([&](auto Jc) {
      constexpr int jj = decltype(Jc)::value;
      const int fb = j0 + jj;
      u32x4 w[2][kPieces];
      static_for<4>([&](auto Qc) {
        constexpr int q = decltype(Qc)::value;
        const int row = fb * 32 + 8 * q + 4 * kk;
        const f32x4 wv = *reinterpret_cast<const f32x4*>(s.vecs + (2 * L - 1) * (NF * 32) + row);
        const f32x4 ps = *reinterpret_cast<const f32x4*>(Ps + row);
        const f32x4 pr = *reinterpret_cast<const f32x4*>(Pr + row);
        static_for<2>([&](auto Hc) {
          constexpr int e = 2 * decltype(Hc)::value, R = 4 * q + e, u = R >> 3, wd = (R & 7) >> 1;
          const float u0 = ps[e] + pr[e] + len2 * wv[e];   // log2 domain (silu_u)
          const float u1 = ps[e + 1] + pr[e + 1] + len2 * wv[e + 1];
          unsigned pc[kPieces];
          split_pair(silu_u(u0), silu_u(u1), pc);
#pragma unroll
          for (int k = 0; k < kPieces; ++k) w[u][k][wd] = pc[k];
        });
      });
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < kPieces; ++k) p[((fb * 2 + u) * kPieces + k) * 64 + lane] = w[u][k];
    });
  }
  __syncthreads();
  SplitX<NF> X;
  xs_load<NF>(xs, X, lane);
  f32x16 m[NF];
  // phi_e layers 2..L
  STAMP_LANE0(s, kStEdgeLayer1, t_sub);
  cols_segment<NF, L - 1>(X, m, launder_uniform(bw.Ws), s.vecs, xs, wave, lane);
  STAMP_LANE0(s, kStEdgeChainE, t_sub);
  SegScan sc;
  sc.init(valid ? rr : -1, li);
  const bool writer = valid && sc.tail;
  if (agg) {
    // gate e_ij = sigmoid(m_ij . w_g + b_g) over every block, edge_tail's lds_dot (the same summation order: cols
    // results stay bitwise the batch path's; egnn.py:99-101)
    float part, partT;
    lds_dot<NF, 0>(s.vecs + (2 * L) * (NF * 32), m, m, kk, part, partT);
    part += __shfl_xor(part, 32);
    const float g = sigmoidf_(part + bw.bg);
    // this wave's message blocks: scatter_sum(m_ij e_ij) (egnn.py:102-104), segment parts stored as edge_tail does
    static_for<NF>([&](auto Fc) {
      constexpr int fb = decltype(Fc)::value;
      if (fb / NJ == wave) {
        float v[16];
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16) v[r16] = m[fb][r16] * g;
        sc.sum_many<16>(v);
        if (writer) {
          if (agg_dst) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              *reinterpret_cast<f32x4*>(agg_dst + fb * 32 + 8 * q + 4 * kk) =
                  f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
          } else {
            float* mrow = s.macc + rr * s.ld_m + 4 * kk;   // (edge_tail's validated form)
            asm volatile("" : "+v"(mrow));
#pragma unroll
            for (int r16 = 0; r16 < 16; ++r16) lds_add(mrow + fb * 32 + acc_row(r16, 0), v[r16]);
          }
        }
      }
    });
  }
  // phi_x layers 1..L on the (ungated) messages, split in full by every wave
  static_for<NF>([&](auto Fc) {
    constexpr int fb = decltype(Fc)::value;
    static_for<8>([&](auto Ic) {
      constexpr int k = decltype(Ic)::value;
      put_pair<NF, fb, 2 * k>(X, m[fb][2 * k], m[fb][2 * k + 1]);
    });
  });
  STAMP_LANE0(s, kStEdgeAgg, t_sub);
  cols_segment<NF, L>(X, m, launder_uniform(bw.Ws + (size_t)(L - 1) * SplitPlan<NF, 1>::GL * kPieces * 256),
                      s.vecs + (L - 1) * NF * 32, xs, wave, lane);
  // phi_x output Dense(1) and the shifts (egnn.py:83-94): every wave computes them, wave 0 stores
  STAMP_LANE0(s, kStEdgePhiX, t_sub);
  edge_shift<NF, 0, L, D>(net, bw, s, m, m, writer, sc, rr, r, dr, length, 0.f, lane, wave == 0);
  __syncthreads();   // the image is rewritten by the next tile's layer 1
  STAMP_LANE0(s, kStEdgeTail, t_sub);
}

// ---------------------------------------------------------------------------------------------------
// Team (latency) mode: G workgroups integrate ONE molecule together (a batch far below the CU count, e.g. the
// reference's one-molecule-per-call sampling timer, examples/load_checkpoint_measure_sampling_time.py:101-119).
// Every member runs the same solver and node phases redundantly (deterministic, so bitwise identical in every
// member); the molecule's edge tiles are dealt round-robin over the members (tile t -> member t mod G) and, after each
// block's edge phase, the members exchange their parts of the edge aggregates through global memory:
//   * message rows (macc) from the member holding the tile where the receiver's segment starts; with stored segment
//     parts (Net::cross) the continuation rows (cross) from the member holding their tile, else (atomically
//     accumulated parts) plus the other tile's member's row;
//   * shift rows (dxacc) from the one or two members holding the receiver's tiles.
// A receiver's segment touches at most two tiles and a missing part is an exact zero, so the rebuilt aggregates are
// bitwise those of a single workgroup running every tile: results are bitwise independent of G.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility; cdna_hip_programming.md Guideline 16 R1): owned rows
// stored write-through (sc1, 16 B), every storing wave drains (vmcnt(0)), a workgroup barrier, one lane's agent-scope
// atomic add on the molecule's arrival counter; one lane polls it (relaxed sc1 loads, s_sleep) until all G members
// arrived for this exchange, one agent-scope acquire, vmcnt(0), barrier, then plain loads.  Slots are double
// buffered by exchange parity (a member can run at most one exchange ahead of the slowest).  Polls are bounded: a
// timeout marks the molecule (status ECNF_E_HIP) instead of hanging the grid.
// ---------------------------------------------------------------------------------------------------
struct TeamP {
  int G;               // workgroups per molecule (<= 1: off)
  int slot;            // floats per exchange slot: (1 + NT) N M (messages, tangent rows after the primal ones)
                       // + (EP / 32) M (continuation rows of the split primal kernels) + (1 + NT) align4(N D)
  float* buf;          // [molecules][2][G][slot]
  unsigned* ctr;       // [molecules] arrival counters (zeroed before every launch)
  int* timeout;        // [molecules] set when an exchange timed out (zeroed before every launch)
  int cols;            // 1: column-split mode (edge_tile_cols; G = tiles per molecule, one tile per member)
  // teamed slots (device memory, nullptr: every slot): slots [0, *nteam) run as teams of G workgroups (blocks
  // [0, G *nteam)), the slots after them alone, one workgroup each (the re-dealt adaptive solve's tail teams,
  // ecnf_hip.hip redeal_kernel)
  const int* nteam;
  int nteam_max;       // host bound of *nteam (the launch's grid: B + nteam_max (G - 1) workgroups)
  // stop-and-team (the re-dealt solve's second launch, ecnf_hip.hip dispatch_integrate): *fin counts the molecules
  // finished in this launch; once at most stop_left of the *nsl occupied slots are unfinished, every molecule stops at
  // its next step boundary (state stored) and a third launch resumes the survivors as teams.  A team decides through
  // its member 0, whose verdict travels in the exchange slot (team_stop_flag), so all members stop at the same step
  int* fin;            // (nullptr: off)
  const int* nsl;
  int stop_left;
};

// the solver loop's sizes (MPW, ND), the LDS offset of the solver state, and a team's stop verdict (stop-and-team,
// read from member 0's exchange slot at the last exchange), in static LDS: written once and read at every use site
// (LDS loads after barriers), so they occupy no SGPRs across the evaluations (kept in SGPRs, they were spilled through
// VGPRs to scratch in the 256-register kernels).  ONE 16-B array: a static LDS variable of another size would move
// the dynamic LDS base off its 16-B alignment, and every ds_read_b128 of the carve-up with it
__device__ __forceinline__ int* solver_sizes() {
  __shared__ int sz[4];   // [MPW, ND, solver-state offset in floats from the dynamic LDS base, team stop verdict]
  return sz;
}
__device__ __forceinline__ int* team_stop_flag() { return solver_sizes() + 3; }

struct TeamCtx {
  TeamP p;
  int r;               // this workgroup's rank in its team
  int T;               // the team's molecule slot
  int G;               // workgroups of this slot's team (1: the slot runs alone, no exchange)
};

typedef ECNF_GLOBAL unsigned* gu32_p;

// one exchange of the edge aggregates (MPW = 1; all threads of the workgroup, after the edge phase's barrier)
template <int NT, int NTHR>
__device__ __forceinline__ void team_exchange(const Net& net, const Lds& s, const TeamCtx& tm, int epoch,
                                              bool pairs = false) {
  const int G = tm.G;
  if (G <= 1) return;   // a slot that runs alone holds every aggregate already
  const int tid = opaque_tid();
  const int N = net.N, M = net.M, D = net.D, r = tm.r, nn1 = N - 1, SR = net.SR, RP = net.RP;
  const int tpm = net.EP >> 5, M4 = M >> 2;
  // slot layout: messages [1 + NT][N][M] (tangent rows after the primal rows), continuation rows [tpm][M] (split
  // primal kernels), shift rows [1 + NT][N][D] (tangent after primal).  The tangent kernels aggregate with LDS atomics
  // (no continuation rows), so a receiver's primal and tangent rows come from the same one or two members.
  const int off_x = (1 + NT) * N * M, off_d = off_x + tpm * M;
  const int ND = N * D, ND4 = (ND + 3) & ~3;   // shift rows [1 + NT][ND4]: whole 16-B stores inside the slot
  const int off_f = off_d + (1 + NT) * ND4;    // member 0's stop verdict (stop-and-team), one 16-B chunk
  float* base = tm.p.buf + ((size_t)tm.T * 2 + (epoch & 1)) * G * tm.p.slot;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  const int mine = r * tm.p.slot * 4;   // byte offset of this member's slot
  auto st16 = [&](int fo, f32x4 v) {   // write-through (sc1) 16-B store of slot float fo
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, fo * 4, mine, 16);
  };
  // the tiles that hold receiver i's edges (block-1 pair tiles: atom i's pairs, PairPlan13; no continuation rows)
  auto first_tile = [&](int i) { return pairs ? PairPlan13::tile_lo(i) : (i * SR) >> 5; };
  auto last_tile = [&](int i) { return pairs ? PairPlan13::tile_hi(i) : (i * SR + nn1 - 1) >> 5; };
  const bool cross = net.cross && !pairs;
  // ---- publish the rows this member owns
  for (int idx = tid; idx < (1 + NT) * N * M4; idx += NTHR) {
    const int w = idx / (N * M4), iw = idx - w * (N * M4);   // w = 1: the tangent row RP + i
    const int i = iw / M4, c = (iw - i * M4) * 4;
    const bool own = first_tile(i) % G == r ||
                     (!cross && last_tile(i) != first_tile(i) && last_tile(i) % G == r);   // (its second part)
    if (own) st16((w * N + i) * M + c, *reinterpret_cast<const f32x4*>(s.macc + (w * RP + i) * s.ld_m + c));
  }
  if (cross)
    for (int idx = tid; idx < tpm * M4; idx += NTHR) {
      const int t = idx / M4, c = (idx - t * M4) * 4;
      if (t % G == r) st16(off_x + t * M + c, *reinterpret_cast<const f32x4*>(s.cross + t * s.ld_m + c));
    }
  for (int idx = tid; idx < (ND + 3) >> 2; idx += NTHR)   // every member: its whole (partial) shift rows
    st16(off_d + 4 * idx, *reinterpret_cast<const f32x4*>(s.dxacc + 4 * idx));
  if constexpr (NT)   // ... and the tangent shift rows (LDS rows RP .. RP + N - 1; RP D is a multiple of 4 floats)
    for (int idx = tid; idx < (ND + 3) >> 2; idx += NTHR)
      st16(off_d + ND4 + 4 * idx, *reinterpret_cast<const f32x4*>(s.dxacc + RP * D + 4 * idx));
  if (tm.p.fin && r == 0 && tid == 0) {   // stop-and-team: member 0's verdict for every member
    const int left = *tm.p.nsl - __hip_atomic_load((ECNF_GLOBAL int*)tm.p.fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float v = left <= tm.p.stop_left ? 1.0f : 0.0f;
    st16(off_f, f32x4{v, v, v, v});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its write-through stores
  __syncthreads();
  // ---- arrive, then wait for the whole team.  A timeout is sticky: once any member has flagged the molecule (a member
  // not running), every later wait of every member sees the flag at its first poll (and every 256th after) and gives
  // up at once, so a broken team costs one poll budget, not one per exchange.
  if (tid == 0) {
    gu32_p ctr = (gu32_p)(tm.p.ctr + tm.T);
    ECNF_GLOBAL int* tflag = (ECNF_GLOBAL int*)(tm.p.timeout + tm.T);
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned want = (unsigned)G * (unsigned)(epoch + 1);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if ((spins & 255u) == 0 && __hip_atomic_load(tflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {   // seconds: a member is not running (not co-resident); give up, flag it
        __hip_atomic_store(tflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (tm.p.fin && tid == 0) *team_stop_flag() = base[off_f] != 0.0f ? 1 : 0;   // member 0's slot (slot 0)
  __syncthreads();
  // ---- rebuild the aggregates a single workgroup would hold
  const float* slot0 = base;
  auto ld16 = [&](int member, int fo) {
    return *reinterpret_cast<const f32x4*>(slot0 + (size_t)member * tm.p.slot + fo);
  };
  // message rows (items 0 .. nmsg - 1: receiver i, 4 columns), then the crossing continuation rows (tile t, 4
  // columns), in batches of kB items per thread whose loads are all issued before their LDS stores: the slots were
  // written through by other XCDs' workgroups, so every load is a memory round trip, and one per loop trip
  // serialised ~14 of them per exchange
  constexpr int kB = 8;
  const int nmsg = (1 + NT) * N * M4, ntot = nmsg + (cross ? tpm * M4 : 0);
  for (int base = tid; base < ntot; base += kB * NTHR) {
    f32x4 v[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int idx = base + u * NTHR;
      v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idx < nmsg) {
        const int w = idx / (N * M4), iw = idx - w * (N * M4);
        const int i = iw / M4, c = (iw - i * M4) * 4;
        const int o0 = first_tile(i) % G, o1 = last_tile(i) % G;
        v[u] = ld16(o0, (w * N + i) * M + c);
        // atomically accumulated parts (no cross rows): 0 + a + b, whichever member holds each (exact in any order)
        if (!cross && o1 != o0) v[u] += ld16(o1, (w * N + i) * M + c);
      } else if (idx < ntot) {
        const int t = (idx - nmsg) / M4, c = (idx - nmsg - t * M4) * 4;
        v[u] = ld16(t % G, off_x + t * M + c);
      }
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int idx = base + u * NTHR;
      if (idx < nmsg) {
        const int w = idx / (N * M4), iw = idx - w * (N * M4);
        const int i = iw / M4, c = (iw - i * M4) * 4;
        *reinterpret_cast<f32x4*>(s.macc + (w * RP + i) * s.ld_m + c) = v[u];
      } else if (idx < ntot) {
        const int t = (idx - nmsg) / M4, c = (idx - nmsg - t * M4) * 4;
        *reinterpret_cast<f32x4*>(s.cross + t * s.ld_m + c) = v[u];
      }
    }
  }
  for (int idx = tid; idx < (1 + NT) * ND; idx += NTHR) {
    const int w = idx / ND, iw = idx - w * ND, i = iw / D;
    const int o0 = first_tile(i) % G, o1 = last_tile(i) % G;
    float v = slot0[(size_t)o0 * tm.p.slot + off_d + w * ND4 + iw];
    if (o1 != o0) v += slot0[(size_t)o1 * tm.p.slot + off_d + w * ND4 + iw];
    s.dxacc[w * RP * D + iw] = v;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------------
// one full evaluation.  x_in/tan_in/v_out/tan_out: LDS [MPW][N*D]; t_in: LDS [MPW] (actual time).
// Must be called by all Geo<NF, NT, P>::NTHR threads of the workgroup (NW waves); returns after a barrier.
// ---------------------------------------------------------------------------------------------------
template <int NF, int NT, int L, int D, int P, bool TEAM = false, bool COLS = false, bool BN = false>
__device__ __forceinline__ void egnn_eval(const Net& net, const Lds& s, const float* x_in, const float* t_in, const float* tan_in,
                          float* v_out, float* tan_out, const int* act = nullptr, int sparse_a = -1,
                          float* pcache = nullptr, int pmode = 0, const TeamCtx* tm = nullptr,
                          int* tepoch = nullptr) {
  constexpr int kNW = kernel_waves<NF, NT, P, COLS>(), kNT = kernel_threads<NF, NT, P, COLS>();
  constexpr bool kSplitG = Geo<NF, NT, P, BN>::kSplit;
  constexpr bool kSplitN = Geo<NF, NT, P, BN>::kSplitN;   // split node GEMMs (primal split kernels and tangent kernels)
  // block-1 pair tiles compiled (Net::pairs turns them on): the M = 128 split primal and split tangent kernels
  constexpr bool kPairs = (kSplitG || Geo<NF, NT, P, BN>::kL2T) && NF == 4 && !COLS;
  // the exact trace's sparse blocks (primal + dual tiles, see the edge loop) in the M <= 128 split tangent kernels;
  // not compiled for the L = 2 shapes (M, D) = (128, 3), (64, 2), where the primal tile's code beside the dual
  // tile's spilled 36 B per lane (tests/test_kernel_resources.py).  The BASELINE shapes (LJ13 128/3/3, ALDP 64/2/3,
  // DW4 128/3/2) have it.
  // (team kernels: tangent teams run Hutchinson solves only, ecnf_hip.hip team_size)
  constexpr bool kSparseX = Geo<NF, NT, P, BN>::kL2T && !(L == 2 && (NF == 4 || D == 2)) && !TEAM;
  const int tid = opaque_tid(), lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: task indices stay in SGPRs
  const int N = net.N, H = net.H, T = net.T, M = NF * 32, RP = net.RP, MPW = net.MPW, ND = net.ND;
  const int nvalid = MPW * N;
  const int R = RP * (1 + NT);

  // ---- prologue: input mean, centring (egnn.py:160), embedding (build_cnf.py:79-83) ----
  // (runtime divisors pass opaque_u at each loop: their division constants are formed here instead of being hoisted
  // above the previous evaluation and kept live, i.e. spilled, across it)
  for (int idx = tid, MD = opaque_u(MPW * D); idx < MD * (1 + NT); idx += kNT) {
    const int which = idx / MD, md = idx - which * MD, m = md / D, d = md - m * D;
    const float* src = (which == 0 ? x_in : tan_in) + m * ND + d;
    float acc = 0.f;
    for (int i = 0; i < N; ++i) acc += src[i * D];
    s.mean[idx] = acc / (float)N;
  }
  for (int idx = tid, To = opaque_u(T); idx < MPW * To; idx += kNT) {
    const int m = idx / To, k = idx - m * To, half = To >> 1;
    const float ts = t_in[m] * 1000.0f;                   // build_cnf.py:23
    const float arg = ts * net.freqs[k < half ? k : k - half];
    s.temb[idx] = k < half ? sinf(arg) : cosf(arg);
  }
  __syncthreads();
  for (int idx = tid, VD = opaque_u(nvalid * D), No = opaque_u(N); idx < VD * (1 + NT); idx += kNT) {
    const int which = idx / VD, nd = idx - which * VD, n = nd / D, d = nd - n * D;
    const int m = n / No;
    const float* src = which == 0 ? x_in : tan_in;
    const float v = src[m * ND + (n - m * No) * D + d] - s.mean[which * MPW * D + m * D + d];
    const int row = which * RP + n;
    s.xc[row * D + d] = v;
  }
  for (int idx = tid, HT = opaque_u(H + T), No = opaque_u(N); idx < R * HT; idx += kNT) {
    const int row = idx / HT, c = idx - row * HT;
    float v = 0.f;
    if (row < nvalid) {
      const int m = row / No;
      v = c < H ? gptr(net.emb)[s.feat[row] * H + c] : s.temb[m * T + (c - H)];
    }
    s.hin[row * s.ld_hin + c] = v;
  }
  __syncthreads();
  STAMP(s, kStPrologue);

  const int ntiles = (MPW * net.EP) >> 5;
  for (int k = 0; k < net.K; ++k) {
    const BlockW& bw = net.blk[k];
    // fresh (opaque) thread indices per phase group: per-thread addresses of the node phases are then computed after
    // the edge phase instead of being hoisted above it and kept live (spilled) through it
    int tid = opaque_tid(), lane = tid & 63;
    // the last block's h update (gate, aggregation, phi_h) is dead: the field is x_K - x_c - mean (egnn.py:176-188)
    const bool need_h = k + 1 < net.K;
    // stage this block's chain biases and the w_d / w_g / w_x vectors in LDS (read by every edge tile)
    {
      const float* be = (kSplitG || Geo<NF, NT, P, BN>::kSplitT || Geo<NF, NT, P, BN>::kWideT) ? bw.be_u : bw.be;
      const float* wd = (kSplitG || Geo<NF, NT, P, BN>::kL2T) ? bw.wd_u : bw.wd;
      const float* wg = (kSplitG || Geo<NF, NT, P, BN>::kL2T) ? bw.wg_u : bw.wg;
      const float* wx = (kSplitG || Geo<NF, NT, P, BN>::kL2T) ? bw.wx_u : bw.wx;
      for (int idx = tid; idx < (2 * L + 2) * M; idx += kNT) {
        const int v = idx / M, c = idx - v * M;
        float val;
        if (v < 2 * L - 1) val = gptr(be)[idx];
        else if (v == 2 * L - 1) val = gptr(wd)[c];
        else if (v == 2 * L) val = gptr(wg)[c];
        else val = gptr(wx)[c];
        s.vecs[idx] = val;
      }
    }
    // h <- Dense([h | temb])  (egnn.py:166-167)
    node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(s.hin, s.ld_hin, H + T, nullptr, 0, 0, bw.Wn, bw.Wn_s, bw.ninv, H, bw.bn, H,
                                      false, nullptr, 0, s.hb, s.ld_hb, RP, nvalid, wave, lane);
    __syncthreads();
    STAMP(s, kStNodeDense);
    // block-1 pair tiles (not in the exact trace, whose block 1 runs dual tiles at one atom): every atom of a molecule
    // has the same P row, held per molecule in hin (dead until the node update) so that the P rows can hold the waves'
    // transposition slices; macc restarts from +0 (the pairs' aggregates are atomic, the receiver segments' first parts
    // were stores)
    const bool pairs = kPairs && k == 0 && net.pairs && sparse_a < 0;
    // per-node halves of phi_e layer 1 (the M = 256 tangent kernels compute layer 1 per edge)
    bool pcopied = false;
    if constexpr (!Geo<NF, NT, P, BN>::kNoP) {
      constexpr bool kPu = kSplitG || Geo<NF, NT, P, BN>::kL2T;   // log2-domain P
      if (NT == 0 && pairs) {
        // primal pair blocks: P for one row per molecule only, as one 32-row tile (its rows past MPW read whatever
        // follows and are not stored): the molecules' hb rows gathered behind the P copies, the P GEMM writing the
        // copies directly.  Each P row is the same MFMA sequence as in the full GEMM (bitwise), on half the tasks
        float* hbc = s.hin + MPW * 2 * M;
        for (int idx = tid; idx < MPW * H; idx += kNT) {
          const int m = idx / H, c = idx - m * H;
          hbc[m * s.ld_hb + c] = s.hb[m * N * s.ld_hb + c];
        }
        for (int idx = tid; idx < R * M; idx += kNT) {
          const int row = idx / M, c = idx - row * M;
          s.macc[row * s.ld_m + c] = 0.f;
        }
        __syncthreads();
        node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(hbc, s.ld_hb, H, nullptr, 0, 0, bw.Wp, bw.Wp_s, bw.pinv,
                                          2 * M, kPu ? bw.bp_u : bw.bp, 2 * M, false, nullptr, 0, s.hin, 2 * M, 32, MPW,
                                          wave, lane);
        __syncthreads();
        pcopied = true;
      } else {
        node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(s.hb, s.ld_hb, H, nullptr, 0, 0, bw.Wp, bw.Wp_s, bw.pinv, 2 * M,
                                          kPu ? bw.bp_u : bw.bp, 2 * M, false, nullptr, 0, s.P, s.ld_P, RP, nvalid, wave,
                                          lane);
        __syncthreads();
      }
    }
    if (pairs && !pcopied) {
      for (int idx = tid; idx < (1 + NT) * MPW * 2 * M; idx += kNT) {   // primal rows, then the tangent rows
        const int w = idx / (MPW * 2 * M), m = (idx - w * MPW * 2 * M) / (2 * M), c = idx % (2 * M);
        s.hin[idx] = s.P[(w * RP + m * N) * s.ld_P + c];
      }
      for (int idx = tid; idx < R * M; idx += kNT) {
        const int row = idx / M, c = idx - row * M;
        s.macc[row * s.ld_m + c] = 0.f;
      }
      __syncthreads();
    }
    STAMP(s, kStPGemm);
    // edges
    // tile t runs on wave t mod NW, i.e. SIMD t mod 4: every SIMD gets ceil/floor(ntiles / 4) tiles
    {
      // act (LDS [MPW], the solver's per-molecule flags; nullptr = every slot): the edge tiles of molecules whose
      // adaptive solve has finished, and of slots that pad the last workgroup, are skipped and the remaining tiles
      // are dealt round-robin over the waves, so a workgroup's tail after its faster molecules finish runs at the
      // cost of the molecules still integrating.  Skipped molecules' outputs are never committed; every molecule's
      // tiles and node rows are its own, so the others' results are unchanged (bitwise).
      const int elane = opaque_tid() & 63;
      const int tpm = net.EP >> 5;
      unsigned amask = MPW >= 32 ? 0xffffffffu : (1u << MPW) - 1u;
      if (act) {
        amask = 0;
        for (int m = 0; m < MPW; ++m) amask |= (act[m] != 0 ? 1u : 0u) << m;
      }
      amask = __builtin_amdgcn_readfirstlane(amask);
      const int nact = __builtin_popcount(amask);
      auto nth_active = [&](int q) {
        unsigned mm = amask;
        for (int i = 0; i < q; ++i) mm &= mm - 1u;   // drop the q lowest active molecules
        return __builtin_ctz(mm);
      };
      // exact trace (sparse_a = the unit tangent's atom; joint_field): two blocks need only 2(N - 1) edge tangents.
      //  * block 1: h carries no tangent yet (embedding and time only), so an edge's tangent is nonzero only if it
      //    touches atom a (dr = 0 otherwise, and the chains, gate and shift of a zero input tangent are exactly 0);
      //  * the last block (K > 1): it updates x only, and the trace reads the JVP at atoms a and 0 only
      //    (joint_field: tout[k] - tout[k mod D]), so only the edges into those two atoms need tangents (the other
      //    atoms' tangent rows go stale; nothing reads them).
      // There every edge runs as a primal tile and the 2(N - 1) edges as dual tiles storing tangents only: per
      // molecule tpm primal + ceil(2(N - 1) / 32) dual tiles instead of tpm dual tiles (dual tiles dealt first)
      int ndt = 0;
      const int amode = k == 0 ? 1 : 2;
      if constexpr (kSparseX)
        if (sparse_a >= 0 && (k == 0 || k + 1 == net.K)) ndt = (2 * (N - 1) + 31) >> 5;
      // primal aggregates of the sparse blocks cached over the JVP passes of one evaluation (pcache, joint_field):
      // pass 1 stores them after the edge phase (pmode 1), later passes load them here and run only the dual tiles
      // (pmode 2).  Dual tiles store tangent rows only, so the loaded primal rows are not raced.
      const int pstride = N * M + 2 * N * D;
      const bool pload = ndt && pcache && pmode == 2;
      if (pload) {
        for (int idx = tid; idx < MPW * N * M; idx += kNT) {
          const int r = idx / M, c = idx - r * M, m = r / N;
          if ((amask >> m) & 1u && k == 0) s.macc[r * s.ld_m + c] = pcache[m * pstride + (r - m * N) * M + c];
        }
        for (int idx = tid; idx < MPW * N * D; idx += kNT) {
          const int r = idx / D, m = r / N;
          if ((amask >> m) & 1u)
            s.dxacc[idx] = pcache[m * pstride + N * M + (k == 0 ? 0 : N * D) + (idx - m * N * D)];
        }
      }
      const int nd = nact * ndt;
      const int tpb = pairs ? PairPlan13::kTiles : tpm;   // this block's tiles per molecule
      float* psb = pairs ? s.P + wave * 1024 : nullptr;
      const int nrun = nd + (pload ? 0 : nact * tpb);
      // team mode (MPW = 1): this member runs tiles t = r, r + G, ... of the molecule (team_exchange)
      const int tstep = TEAM ? tm->G : 1, tfirst = TEAM ? tm->r : 0;
      if constexpr (COLS) {
        // column-split team mode: member r runs tile r (G = tiles per molecule) with all of its waves
        static_assert(TEAM && NT == 0 && Geo<NF, NT, P, BN>::kSplit, "cols mode: team primal split kernels");
        for (int vt = tfirst; vt < nrun; vt += tstep) {
          const int q = vt / tpm;
          edge_tile_cols<NF, L, D>(net, bw, s, nth_active(q) * tpm + (vt - q * tpm), wave, elane, need_h);
        }
      } else {
      for (int vt = tfirst + wave * tstep; vt < nrun; vt += kNW * tstep) {
        if constexpr (kSparseX) {
          if (vt < nd) {
            const int q = vt / ndt;
            edge_tile<NF, NT, L, D, P, kPieces, BN>(net, bw, s, nth_active(q), elane, need_h, sparse_a, vt - q * ndt, amode);
            continue;
          }
        }
        const int v2 = vt - nd, q = v2 / tpb;
        const int tile = nth_active(q) * tpb + (v2 - q * tpb);
        if constexpr (kSparseX) {
          if (ndt) {
            edge_tile<NF, 0, L, D, P, 3>(net, bw, s, tile, elane, need_h);   // exact weights, as the dual tiles
            continue;
          }
        }
        // (one call site: the pair tiles branch inside the tile around one copy of its chains; a second inlined copy
        // for block 1 grew the kernel by 40 KB of code and ran 6.7x slower)
        edge_tile<NF, NT, L, D, P, kPieces, BN>(net, bw, s, tile, elane, need_h, -1, 0, 1, psb);
      }
      }   // !COLS
    }
    __syncthreads();
    if constexpr (TEAM) {   // team mode: rebuild the molecule's aggregates from every member's tiles
      STAMP(s, kStEdge);
      team_exchange<NT, kNT>(net, s, *tm, *tepoch, pairs);
      ++*tepoch;
      STAMP(s, kStTeam);
    }
    if constexpr (kSparseX) {
      // first JVP pass of an exact-trace evaluation: cache the sparse block's primal aggregates (see the edge loop)
      if (pcache && pmode == 1 && sparse_a >= 0 && (k == 0 || k + 1 == net.K)) {
        const int pstride = N * M + 2 * N * D;
        if (k == 0)
          for (int idx = tid; idx < MPW * N * M; idx += kNT) {
            const int r = idx / M, c = idx - r * M, m = r / N;
            pcache[m * pstride + (r - m * N) * M + c] = s.macc[r * s.ld_m + c];
          }
        for (int idx = tid; idx < MPW * N * D; idx += kNT) {
          const int m = idx / (N * D);
          pcache[m * pstride + N * M + (k == 0 ? 0 : N * D) + (idx - m * N * D)] = s.dxacc[idx];
        }
        __syncthreads();
      }
    }
    STAMP(s, kStEdge);
    tid = opaque_tid();
    lane = tid & 63;
    // node update: x += shift_i / (N-1) (egnn.py:95,113); m_i /= sqrt(N-1) (egnn.py:104)
    for (int idx = tid; idx < R * D; idx += kNT) {
      s.xc[idx] += s.dxacc[idx] / net.nn1;
      s.dxacc[idx] = 0.f;
    }
    if (!need_h) {   // last block: no h update
      __syncthreads();
      STAMP(s, kStNodeUpd);
      continue;
    }
    if constexpr (kSplitG) {
      // the split phi_h.0 weights carry the message scale -ln2 / sqrt(N-1) (log2-domain messages, chain_split.hpp;
      // egnn.py:104), so only the continuation parts of the segments that cross a tile boundary are added here:
      // one (molecule, crossing) row per wave trip, wave-uniform indices
      if (net.cross && !pairs) {
        const int nx = net.ncross, tpm = net.EP >> 5;
        for (int j = wave; j < MPW * nx; j += kNW) {
          const int m = j / nx, q = j - m * nx;
          float* dst = s.macc + (m * N + net.xs_i[q]) * s.ld_m;
          const float* src = s.cross + (m * tpm + net.xs_t[q]) * s.ld_m;
          for (int c = lane; c < M; c += 64) dst[c] += src[c];
        }
      }
    } else if constexpr (!Geo<NF, NT, P, BN>::kL2T) {   // kL2T: the scale is in the split phi_h.0 weights
      for (int idx = tid; idx < R * M; idx += kNT) {
        const int row = idx / M, c = idx - row * M;
        s.macc[row * s.ld_m + c] = s.macc[row * s.ld_m + c] / net.sqrt_nn1;
      }
    }
    __syncthreads();
    if constexpr (kSplitG || kPairs) {
      if (net.cross || pairs) {   // the cross buffer (pair tiles: the P copies) overlaid hin's time-embedding columns
        for (int idx = tid; idx < nvalid * T; idx += kNT) {
          const int row = idx / T, c = idx - row * T;
          s.hin[row * s.ld_hin + H + c] = s.temb[(row / N) * T + c];
        }
      }
    }
    STAMP(s, kStNodeUpd);
    // phi_h = MLP((M,)*L + (H,)) on [m_i | h], residual (egnn.py:105-111)
    if constexpr (Geo<NF, NT, P, BN>::kWideT) {
      // in place on macc (no P region in these kernels), then macc restarts from +0 for the next block's aggregates
      node_gemm_inplace<NT, kNW>(s.macc, s.ld_m, M, s.hb, s.ld_hb, H, bw.Wh_sn0, bw.hinv_n0, bw.bh[0], M, true,
                                 s.macc, s.ld_m, RP, nvalid, wave, lane);
      __syncthreads();
      for (int l = 1; l < L; ++l) {
        node_gemm_inplace<NT, kNW>(s.macc, s.ld_m, M, nullptr, 0, 0, bw.Wh_s[l], bw.hinv[l], bw.bh[l], M, true, s.macc,
                                   s.ld_m, RP, nvalid, wave, lane);
        __syncthreads();
      }
      node_gemm<NT, kNW, true>(s.macc, s.ld_m, M, nullptr, 0, 0, bw.Wh[L], bw.Wh_s[L], bw.hinv[L], H, bw.bh[L], H, false,
                               s.hb, s.ld_hb, s.hin, s.ld_hin, RP, nvalid, wave, lane);
      __syncthreads();
      for (int idx = tid; idx < R * M; idx += kNT) {
        const int row = idx / M, c = idx - row * M;
        s.macc[row * s.ld_m + c] = 0.f;
      }
      __syncthreads();
      STAMP(s, kStPhiH);
      continue;
    }
    if constexpr (Geo<NF, NT, P, BN>::kWideT32) {   // the same in fp32 (macc already carries the 1 / sqrt(N - 1))
      node_gemm_inplace_f32<NT, kNW>(s.macc, s.ld_m, M, s.hb, s.ld_hb, H, bw.Wh[0], M, bw.bh[0], M, true, s.macc,
                                     s.ld_m, RP, nvalid, wave, lane);
      __syncthreads();
      for (int l = 1; l < L; ++l) {
        node_gemm_inplace_f32<NT, kNW>(s.macc, s.ld_m, M, nullptr, 0, 0, bw.Wh[l], M, bw.bh[l], M, true, s.macc,
                                       s.ld_m, RP, nvalid, wave, lane);
        __syncthreads();
      }
      node_gemm<NT, kNW, false>(s.macc, s.ld_m, M, nullptr, 0, 0, bw.Wh[L], nullptr, 1.0f, H, bw.bh[L], H, false,
                                s.hb, s.ld_hb, s.hin, s.ld_hin, RP, nvalid, wave, lane);
      __syncthreads();
      for (int idx = tid; idx < R * M; idx += kNT) {
        const int row = idx / M, c = idx - row * M;
        s.macc[row * s.ld_m + c] = 0.f;
      }
      __syncthreads();
      STAMP(s, kStPhiH);
      continue;
    }
    float* Q0 = s.P;
    float* Q1 = s.P + (kSplitN ? M + 4 : M + 1);   // 16-B aligned rows for the split node GEMMs
    constexpr bool kHu = kSplitG || Geo<NF, NT, P, BN>::kL2T;   // log2-domain messages, scale in phi_h.0
    node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(s.macc, s.ld_m, M, s.hb, s.ld_hb, H, bw.Wh[0], kHu ? bw.Wh_s[0] : bw.Wh_sn0,
                                      kHu ? bw.hinv[0] : bw.hinv_n0, M, bw.bh[0], M, true, nullptr, 0, Q0, s.ld_P, RP,
                                      nvalid, wave, lane);
    __syncthreads();
    if (!(kSplitG && net.cross)) {   // atomically accumulated aggregates restart from +0
      for (int idx = tid; idx < R * M; idx += kNT) {
        const int row = idx / M, c = idx - row * M;
        s.macc[row * s.ld_m + c] = 0.f;
      }
    }
    for (int l = 1; l < L; ++l) {
      node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(Q0, s.ld_P, M, nullptr, 0, 0, bw.Wh[l], bw.Wh_s[l], bw.hinv[l], M, bw.bh[l], M,
                                        true, nullptr, 0, Q1, s.ld_P, RP, nvalid, wave, lane);
      __syncthreads();
      float* tq = Q0; Q0 = Q1; Q1 = tq;
    }
    node_gemm<NT, kNW, kSplitN, Geo<NF, NT, P, BN>::kNodePFA>(Q0, s.ld_P, M, nullptr, 0, 0, bw.Wh[L], bw.Wh_s[L], bw.hinv[L], H, bw.bh[L], H,
                                      false, s.hb, s.ld_hb, s.hin, s.ld_hin, RP, nvalid, wave, lane);
    __syncthreads();
    STAMP(s, kStPhiH);
  }

  // ---- epilogue: v = ((x_K - x_c0) - mean(x_in)) * final_scaling  (egnn.py:183-188) ----
  for (int idx = tid; idx < nvalid * D * (1 + NT); idx += kNT) {
    const int which = idx / (nvalid * D), nd = idx - which * nvalid * D, n = nd / D, d = nd - n * D;
    const int m = n / N;
    const int row = which * RP + n;
    // x_c0 recomputed from the (unchanged) input exactly as the prologue computed it (no [R][D] LDS copy)
    const float* src = which == 0 ? x_in : tan_in;
    const float mu = s.mean[which * MPW * D + m * D + d];
    const float xc0 = src[m * ND + (n - m * N) * D + d] - mu;
    const float v = ((s.xc[row * D + d] - xc0) - mu) * net.fs;
    float* dst = which == 0 ? v_out : tan_out;
    dst[m * ND + (n - m * N) * D + d] = v;
  }
  __syncthreads();
  STAMP(s, kStEpilogue);
}

}  // namespace ecnf
