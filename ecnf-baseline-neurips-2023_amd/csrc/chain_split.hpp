// chain_split.hpp — the edge-MLP chain on the 16-bit matrix cores, fp32-accurate by operand splitting (gfx950).
//
// Why: on gfx950 v_mfma_f32_32x32x2_f32 runs at the fp32 VECTOR rate and shares the SIMD's vector issue, so every
// SiLU / scan instruction of the fp32-MFMA chain adds to its time (measured: tools/micro/chain_bench.hip).  The
// 16-bit MFMAs (v_mfma_f32_32x32x16_f16, 32 cycles for 16x the fp32 MFMA's k-depth) run on the matrix cores and
// leave 24 of their 32 cycles of vector issue free.
//
// Accuracy: every fp32 operand x is split into two fp16 values by round-to-nearest, x = x0 + x1,
// |x - x0| <= 2^-11 |x|, and x1 = fp16(x - x0) carries the rest to 2^-22 |x| (one v_cvt_pk_f16_f32 and two v_fma_mix
// per pair of values).  A product keeps the three cross terms w1x0, w0x1, w0x0 (smallest first) and accumulates them
// in fp32 inside the MFMA; the dropped w1x1 and the piece roundings are <= 2^-21 |w x|.  Node-GEMM weights are split
// on the host after scaling each matrix by a power of two s (max |w s| in [2^12, 2^13)), so both weight pieces are
// normal fp16 numbers; their epilogue multiplies the accumulator by 1/s (exact) in the FMA that adds the bias.
// Edge-chain weights are split unscaled and every output block's accumulator starts at its bias column, so the
// activation needs no FMA (-1 VALU per element; LJ13 26.70 -> 26.01 ms); the host refuses |w| >= 2^15.  Activations
// and unscaled weights keep their pieces' absolute error <= 2^-25 below 2^-14 (fp16 subnormals): per dot product of
// K = 128 terms that is <= 128 * 2^-25 * max|x| absolute, i.e. ~1e-6 relative for O(0.1) weights.  (The round-1 form,
// three bf16 pieces and six cross terms, ran LJ13 in 56.8 ms against 36.5 ms for the fp16 pair.)
//
// Layout: one 32-edge tile per wave, features on MFMA rows, edges on lanes (as the fp32 chain).  A k-step of
// 16 input features of block fb is accumulator registers 8u..8u+7 (u = 0, 1): lane (c, h) holds features
// f(8u+j, h) = ((8u+j)&3) + 8((8u+j)>>2) + 4h of edge c, exactly the 16-bit B-operand slot k = 8h + j, so the
// weights are packed in that permuted k order on the host and activations never move between lanes.
//
// Schedule (one layer = NF output blocks x NF input blocks x 2 k-steps = 2 NF^2 groups of kTerms MFMAs, output-block
// major): block jb accumulates in groups [2NF jb, 2NF (jb+1)); block jb-1 is activated (bias, SiLU, split into
// the OTHER activation buffer) one pair of elements per group meanwhile, and the last block of a layer during the
// first 2NF-2 groups of the next, before group (jb 0, fb NF-1) reads it.  The final layer's SiLU stays fp32 in
// place (the tail needs fp32 messages).  Weight groups stream PF groups ahead, contiguous across layers.
#pragma once
// (included by egnn_eval.hpp inside namespace ecnf)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const ECNF_GLOBAL u32x4* gu32x4_p;

constexpr int kPieces = 2;
constexpr int kTerms = 3;
// cross term t: (weight piece, activation piece), smallest first: w1 x0, w0 x1, w0 x0
__host__ __device__ constexpr int term_w(int t) { return t == 0 ? 1 : 0; }
__host__ __device__ constexpr int term_x(int t) { return t == 1 ? 1 : 0; }
// bytes of one split group / k-step fragment set: kPieces x 64 lanes x 16 B
constexpr int kPieceBytes = 1024;
constexpr int kGroupU32 = kPieces * 256;

// activations of one tile in split form: [input block][k-step u][piece] -> 8 16-bit values (4 u32) per lane
template <int NF>
struct SplitX {
  u32x4 v[NF][2][kPieces];
};

__device__ __forceinline__ f32x16 mfma_split(u32x4 a, u32x4 b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                0, 0);
}

// y0, y1 -> kPieces packed 16-bit pairs (RNE), y = sum of the pieces per element
__device__ __forceinline__ void split_pair(float y0, float y1, unsigned (&p)[kPieces]) {
  p[0] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){y0, y1}, f16x2));
  // p1 = fp16(y - fp16 piece 0) per half: the mixed-precision FMA reads the f16 half directly, the difference is
  // exact in fp32 and rounded once (hipcc does not form v_fma_mix from C here)
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo)
      : "v"(p[0]), "v"(y0), "v"(y1));
  p[1] = lo;
}

// SiLU in the log2 domain.  The split kernels carry every pre-activation as u = -log2(e) t (the host folds the
// factor into the biases and the first layer's weights) and every activation as y' = -log2(e) silu(t):
//   y' = u / (1 + 2^u)
// (v_exp_f32, v_add, v_rcp_f32, v_mul).  A layer fed y' needs no change of its weights: W y + b = -ln2 W y' + b,
// so u_next = W y' - log2(e) b.  The consumers of a chain's last layer (gate and phi_x-output vectors, the message
// aggregate) take the -ln 2 on the host / in the node update.
__device__ __forceinline__ float silu_u(float u) {
  return u * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

// store elements (r, r+1) of block j (accumulator register order) into split buffer X
template <int NF, int J, int R>
__device__ __forceinline__ void put_pair(SplitX<NF>& X, float y0, float y1) {
  static_assert((R & 1) == 0, "pairs start at even registers");
  unsigned p[kPieces];
  split_pair(y0, y1, p);
  constexpr int u = R >> 3, w = (R & 7) >> 1;
#pragma unroll
  for (int i = 0; i < kPieces; ++i) X.v[J][u][i][w] = p[i];
}

// The activation of a layer's output block runs as a 3-stage software pipeline across MFMA groups, so the VALU that
// fills each MFMA gap has no dependency on the VALU of the same gap (no transcendental-latency stalls):
//   stage A (group gA): u = acc (+ the bias and 1/s for 3-piece weights); e = 2^u   (v_exp)
//   stage B (group gB): r = 1 / (1 + e)                                              (v_add, v_rcp)
//   stage C (group gC): y' = u r, split into the next layer's input buffer (v_mul, v_cvt_pk, 2 v_fma_mix), or kept
//                       fp32 in place in acc for the segment's last layer
// An item is one pair of elements (rows 2p, 2p+1 of the accumulator registers) of output block j of layer l.
// Groups are output-block major: block jb of a layer accumulates in groups [jb GB, (jb + 1) GB), GB = 2 NF.
// Constraints per item: gA after the block's last MFMA group; gA before layer l+1 re-zeroes acc[j] (group
// (l+1) GL + j GB); gC before layer l+1 first reads input block j (group (l+1) GL + 2 j).  Items spread evenly
// over that window, gB = gA + 1, gC = gA + 2 where the window allows (compressed into fewer groups otherwise).
template <int NF, int NL>
struct SplitPlan {
  static constexpr int GB = 2 * NF;        // groups per output block
  static constexpr int GL = NF * GB;       // groups per layer
  static constexpr int G = NL * GL;        // MFMA groups of the segment
  static constexpr int PPB = 8;            // element pairs per block (16 accumulator registers)
  static constexpr int NI = NL * NF * PPB; // items
  struct Item { int l, j, p, gA, gB, gC; };
  static constexpr int imin(int a, int b) { return a < b ? a : b; }
  static constexpr int imax(int a, int b) { return a > b ? a : b; }
  static constexpr Item item(int id) {
    const int l = id / (NF * PPB), j = (id / PPB) % NF, p = id % PPB;
    const int base = l * GL + (j + 1) * GB;                 // first group after the block's last MFMA
    const int deadline = (l + 1) * GL + 2 * j - 1;          // last group that may still write input block j
    const int span = imax(1, deadline - base - 1);          // groups with room for gC = gA + 2
    const int rate = (PPB + span - 1) / span;               // items per stage-A group
    const int gA = base + p / rate;
    const int gC = imax(gA, imin(gA + 2, deadline));
    const int gB = imin(gA + 1, gC);
    return Item{l, j, p, gA, gB, gC};
  }
  static constexpr int last_group() {
    int m = G - 1;
    for (int i = 0; i < NI; ++i) m = imax(m, item(i).gC);
    return m;
  }
  // number of items with stage S (0 = A, 1 = B, 2 = C) in group g, and the id of the k-th one
  static constexpr int stage_g(const Item& it, int S) { return S == 0 ? it.gA : S == 1 ? it.gB : it.gC; }
  static constexpr int count(int g, int S) {
    int n = 0;
    for (int i = 0; i < NI; ++i) n += stage_g(item(i), S) == g;
    return n;
  }
  static constexpr int nth(int g, int S, int k) {
    for (int i = 0; i < NI; ++i)
      if (stage_g(item(i), S) == g && k-- == 0) return i;
    return -1;
  }
  // the same restricted to items whose previous stage sits in the same group (late = true: compressed windows, which
  // must follow that stage inside the group) or in an earlier one (late = false); S = 1, 2
  static constexpr bool is_late(const Item& it, int S) { return stage_g(it, S - 1) == stage_g(it, S); }
  static constexpr int count_l(int g, int S, bool late) {
    int n = 0;
    for (int i = 0; i < NI; ++i) n += stage_g(item(i), S) == g && is_late(item(i), S) == late;
    return n;
  }
  static constexpr int nth_l(int g, int S, bool late, int k) {
    for (int i = 0; i < NI; ++i)
      if (stage_g(item(i), S) == g && is_late(item(i), S) == late && k-- == 0) return i;
    return -1;
  }
  // LDS address (floats, lane half 0) of the two biases of item id; the lane half adds 4
  static constexpr int bias_off(int id) {
    const Item it = item(id);
    const int r = 2 * it.p;
    return it.l * NF * 32 + it.j * 32 + 8 * (r >> 2) + (r & 3);
  }
};

// per-layer 1 / weight scale of a chain segment (wave-uniform)
struct ChainInv {
  float v[2 * 4 - 1];
};

constexpr int kChainPrio = 1;        // wave priority inside the chain (s_setprio; 2 or 3: no further change)
constexpr int kSplitPF = 3;          // weight groups in flight ahead of the MFMAs (PF 2 ... 10: no difference)
constexpr int kSplitPF3 = 3;         // ... for the 3-piece (exact-weight) chains (2 / 3 equal; 5 spilled 119 registers)
constexpr int kSplitPF3Narrow = 2;   // ... at M = 64, where the kernel runs 2 waves per SIMD (ALDP 50.5 -> 50.2 ms)

__device__ __forceinline__ u32x4 wload(__amdgpu_buffer_rsrc_t rsrc, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
}

template <int I, typename A, typename B>
__device__ __forceinline__ auto& pick(A& a, B& b) {
  if constexpr (I == 0) return a; else return b;
}

// NL chained layers Y = silu(X W_l + b_l).  Input in XA (split form); on return acc holds the last layer's
// activations y' (log2 domain, silu_u) in fp32 (accumulator layout).  XA / XB are both clobbered.
// Weights: packed split fragments [layer][group][piece][lane] (16 B), read as buffer loads with the group
// offset in an SGPR, PF groups ahead; biases: LDS [NL][M] (log2 domain), each item's two (adjacent) rows read one
// group before its stage A; inv.v[l]: 1 / the weight scale of layer l (3-piece weights).
// NT = 1 (forward-mode tangent, the divergence kernels): XAT / XBT / accT carry the tangent of every activation
// through the same layers.  Each weight fragment feeds 2 kTerms MFMAs (primal and tangent interleaved); the
// tangent of a layer is du = accT inv (no bias) and dy' = silu'(t) du = r (1 - ln2 u (1 - r)) du with the primal's
// r = 1 / (1 + 2^u) (silu'(t) = sigma(t) (1 + t (1 - sigma(t))), t = -ln2 u).
// WP: weight pieces per fragment group.  kPieces (2): the primal kernels' unscaled pieces, accumulators started at
// the bias column.  3 (the divergence kernels, kWExact): the weights scaled by a power of two per layer and split into
// three fp16 pieces w0 + w1 + w2 that hold the fp32 weight EXACTLY, the primal MFMAs adding the fourth term w2 x0
// (smallest first) and the activation applying 1/s and the bias in an FMA.  Two pieces represent a weight only to
// 2^-22 (and unscaled small weights far worse, in fp16 subnormals): a FIXED perturbation of the network, which the
// exact trace sums coherently over its N*D diagonal entries (LJ13: +1.2e-6 relative in tr J, 8x the fp32 rounding
// error; tools/diag/trace_precision.py).  The tangent MFMAs keep three terms on pieces 0 and 1.
template <int NF, int NL, int NT = 0, int WP = kPieces>
__device__ __forceinline__ void chain_split(SplitX<NF>& XA, SplitX<NF>& XB, f32x16 (&acc)[NF],
                                            const unsigned* __restrict__ Wpk, const float* __restrict__ bias,
                                            const ChainInv& inv, int lane, SplitX<NF>& XAT, SplitX<NF>& XBT,
                                            f32x16 (&accT)[NF]) {
  using Plan = SplitPlan<NF, NL>;
  static_assert(WP == kPieces || WP == 3, "2-piece weights, or the exact 3-piece weights");
  static_assert(NT == 0 || NT == 1, "primal, or primal + one tangent");
  constexpr bool kBI = WP == kPieces;   // accumulators start at the bias column (unscaled weights)
  // the chain wave issues first on its SIMD while its partner wave is in VALU / LDS work (A/B: 26.14 -> 25.99 ms)
  __builtin_amdgcn_s_setprio(kChainPrio);
  constexpr int GB = Plan::GB, GL = Plan::GL, G = Plan::G, NI = Plan::NI,
                PF = WP == 3 ? (NF <= 2 ? kSplitPF3Narrow : kSplitPF3) : kSplitPF;
  constexpr int GE = Plan::last_group() + 1;   // groups including the VALU-only tail
  const int kk = lane >> 5;
  const float* lbias = bias + 4 * kk;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(Wpk), (short)0,
                                                                         0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  u32x4 wbuf[PF + 1][WP];
#pragma unroll
  for (int gg = 0; gg < PF && gg < G; ++gg)
#pragma unroll
    for (int p = 0; p < WP; ++p) wbuf[gg][p] = wload(rsrc, voff, (gg * WP + p) * kPieceBytes);
  // per-item pipeline registers (SSA after unrolling: only live items occupy registers)
  f32x2 bv[NI], uv[NI], ev[NI], dv[NI];
  // kBI: each output block's accumulator starts at its (log2-domain) bias column and the weights are unscaled, so
  // stage A needs no FMA; a block's 16 biases (rows acc_row(r, kk)) are 4 x 16-B LDS reads, issued 2 groups ahead
  auto bias_block = [&](int off) {
    f32x16 c;
    static_for<4>([&](auto Qc) {
      constexpr int q = decltype(Qc)::value;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(lbias + off + 8 * q);
      c[4 * q] = b4[0];
      c[4 * q + 1] = b4[1];
      c[4 * q + 2] = b4[2];
      c[4 * q + 3] = b4[3];
    });
    return c;
  };
  f32x16 cb = {};
  if constexpr (kBI) {
    cb = bias_block(0);
  } else {
    static_for<Plan::count(0, 0)>([&](auto Kc) {
      constexpr int id = Plan::nth(0, 0, decltype(Kc)::value);
      bv[id] = *reinterpret_cast<const f32x2*>(lbias + Plan::bias_off(id));
    });
  }
  static_for<GE>([&](auto GGc) {
    constexpr int gg = decltype(GGc)::value;
    constexpr bool mfma_group = gg < G;
    constexpr int l = gg / GL, g = gg % GL, jb = g / GB, fb = (g % GB) >> 1, u = g & 1;
    constexpr int nbias = kBI ? 0 : Plan::count(gg + 1, 0);
    constexpr int nxt = l * NF + jb + 1;   // the next output block of the segment
    constexpr bool load_cb = kBI && mfma_group && (g % GB) == GB - 2 && nxt < NL * NF;
    if constexpr (load_cb) cb = bias_block((nxt / NF) * NF * 32 + (nxt % NF) * 32);
    if constexpr (gg + PF < G) {
#pragma unroll
      for (int p = 0; p < WP; ++p)
        wbuf[(gg + PF) % (PF + 1)][p] = wload(rsrc, voff, ((gg + PF) * WP + p) * kPieceBytes);
    }
    // biases of the next group's stage-A items
    static_for<nbias>([&](auto Kc) {
      constexpr int id = Plan::nth(gg + 1, 0, decltype(Kc)::value);
      bv[id] = *reinterpret_cast<const f32x2*>(lbias + Plan::bias_off(id));
    });
    auto mfma_t = [&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      auto& Xin = pick<l & 1>(XA, XB);
      const u32x4* A = wbuf[gg % (PF + 1)];
      const u32x4* B = Xin.v[fb][u];
      const u32x4* BT = pick<l & 1>(XAT, XBT).v[fb][u];
      constexpr int pa = term_w(t), pb = term_x(t);   // cross terms, smallest first
      if constexpr (fb == 0 && u == 0 && t == 0) {
        const f32x16 z = {};
        if constexpr (WP == 3) {   // the exact-weight term w2 x0 first
          acc[jb] = mfma_split(A[2], B[0], z);
          acc[jb] = mfma_split(A[pa], B[pb], acc[jb]);
        } else {
          acc[jb] = mfma_split(A[pa], B[pb], kBI ? cb : z);
        }
        if constexpr (NT) accT[jb] = mfma_split(A[pa], BT[pb], z);
      } else {
        if constexpr (WP == 3 && t == 0) acc[jb] = mfma_split(A[2], B[0], acc[jb]);
        acc[jb] = mfma_split(A[pa], B[pb], acc[jb]);
        if constexpr (NT) accT[jb] = mfma_split(A[pa], BT[pb], accT[jb]);
      }
    };
    // stage A
    auto stageA = [&]() { static_for<Plan::count(gg, 0)>([&](auto Kc) {
      constexpr int id = Plan::nth(gg, 0, decltype(Kc)::value);
      constexpr typename Plan::Item it = Plan::item(id);
      constexpr int r = 2 * it.p;
      if constexpr (kBI) {
        uv[id][0] = acc[it.j][r];
        uv[id][1] = acc[it.j][r + 1];
      } else {
        uv[id][0] = fmaf(acc[it.j][r], inv.v[it.l], bv[id][0]);
        uv[id][1] = fmaf(acc[it.j][r + 1], inv.v[it.l], bv[id][1]);
      }
      ev[id][0] = __builtin_amdgcn_exp2f(uv[id][0]);
      ev[id][1] = __builtin_amdgcn_exp2f(uv[id][1]);
      if constexpr (NT) {
        if constexpr (kBI) {
          dv[id][0] = accT[it.j][r];
          dv[id][1] = accT[it.j][r + 1];
        } else {
          dv[id][0] = accT[it.j][r] * inv.v[it.l];
          dv[id][1] = accT[it.j][r + 1] * inv.v[it.l];
        }
      }
    }); };
    // stage B: the add as packed fp32 where the compiler keeps the pair in an aligned register pair (bit-identical;
    // LJ13 27.14 -> 27.02 ms, profiles/round2/e3)
    auto stageB = [&](auto Late) { static_for<Plan::count_l(gg, 1, decltype(Late)::value)>([&](auto Kc) {
      constexpr int id = Plan::nth_l(gg, 1, decltype(Late)::value, decltype(Kc)::value);
      const f32x2 s = ev[id] + 1.0f;
      ev[id][0] = __builtin_amdgcn_rcpf(s[0]);
      ev[id][1] = __builtin_amdgcn_rcpf(s[1]);
    }); };
    // stage C
    auto stageC = [&](auto Late) { static_for<Plan::count_l(gg, 2, decltype(Late)::value)>([&](auto Kc) {
      constexpr int id = Plan::nth_l(gg, 2, decltype(Late)::value, decltype(Kc)::value);
      constexpr typename Plan::Item it = Plan::item(id);
      const f32x2 yv = uv[id] * ev[id];
      const float y0 = yv[0], y1 = yv[1];
      if constexpr (it.l < NL - 1) {
        put_pair<NF, it.j, 2 * it.p>(pick<(it.l + 1) & 1>(XA, XB), y0, y1);
      } else {
        acc[it.j][2 * it.p] = y0;
        acc[it.j][2 * it.p + 1] = y1;
      }
      if constexpr (NT) {
        constexpr float kNegLn2 = -0.69314718055994531f;
        // u (1 - r) = u - y' (y' = u r): 4 VALU per element instead of 5
        const f32x2 dd = (ev[id] * dv[id]) * __builtin_elementwise_fma(uv[id] - (f32x2){y0, y1}, (f32x2)kNegLn2,
                                                                      (f32x2)1.0f);
        const float d0 = dd[0], d1 = dd[1];
        if constexpr (it.l < NL - 1) {
          put_pair<NF, it.j, 2 * it.p>(pick<(it.l + 1) & 1>(XAT, XBT), d0, d1);
        } else {
          accT[it.j][2 * it.p] = d0;
          accT[it.j][2 * it.p + 1] = d1;
        }
      }
    }); };
    // Emission order pinned per MFMA gap: one stage per MFMA of the group (stage C, B, A after the 1st, 2nd, 3rd
    // MFMA term: each ~20 cycles of issue for one item, inside the 24 free issue cycles of a 32-cycle MFMA), every
    // gap closed by a sched_barrier.  Stage C consumes the rcp of the previous group, stage A reads an accumulator
    // finished at least one group earlier, so no gap waits on its own MFMA.  (A sched_group_barrier form left 2/3 of
    // the gaps empty and bunched 40-100 issue cycles into the others.)
    if constexpr (mfma_group) {
      __builtin_amdgcn_sched_barrier(0);
      static_for<kTerms>([&](auto Tc) {
        constexpr int t = decltype(Tc)::value;
        constexpr int stage = 2 - (t * 3) / kTerms;   // C, B, A
        mfma_t(Tc);
        // items whose windows were compressed (two stages in one group) run in A, B, C order after stage A
        if constexpr (stage == 2) stageC(std::false_type{});
        if constexpr (stage == 1) stageB(std::false_type{});
        if constexpr (stage == 0) {
          stageA();
          stageB(std::true_type{});
          stageC(std::true_type{});
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    } else {
      stageA();
      stageB(std::false_type{});
      stageB(std::true_type{});
      stageC(std::false_type{});
      stageC(std::true_type{});
    }
  });
  __builtin_amdgcn_s_setprio(0);
}

// primal-only chain (the tangent arguments alias the primal ones and are never touched)
template <int NF, int NL, int WP = kPieces>
__device__ __forceinline__ void chain_split(SplitX<NF>& XA, SplitX<NF>& XB, f32x16 (&acc)[NF],
                                            const unsigned* __restrict__ Wpk, const float* __restrict__ bias,
                                            const ChainInv& inv, int lane) {
  chain_split<NF, NL, 0, WP>(XA, XB, acc, Wpk, bias, inv, lane, XA, XB, acc);
}

// the tangent kernels' chain segment on natural-domain fp32 activations (fp32-MFMA accumulator layout, as
// chain_segment): X, XT -> log2 domain, split, NL dual layers, back to the natural domain in place.  Biases: the
// log2-domain copies (the NT kernels stage be_u); weights: the same split fragments as the primal kernels.
template <int NF, int NL>
__device__ __forceinline__ void chain_split_tangent(f32x16 (&X)[NF], f32x16 (&XT)[NF], const unsigned* __restrict__ Wpk,
                                                    const float* __restrict__ bias, const ChainInv& inv, int lane) {
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.69314718055994531f;
  SplitX<NF> XA, XB, XAT, XBT;
  static_for<NF>([&](auto Fc) {
    constexpr int fb = decltype(Fc)::value;
    static_for<8>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value;
      put_pair<NF, fb, 2 * i>(XA, kNegLog2e * X[fb][2 * i], kNegLog2e * X[fb][2 * i + 1]);
      put_pair<NF, fb, 2 * i>(XAT, kNegLog2e * XT[fb][2 * i], kNegLog2e * XT[fb][2 * i + 1]);
    });
  });
  chain_split<NF, NL, 1, 3>(XA, XB, X, Wpk, bias, inv, lane, XAT, XBT, XT);
#pragma unroll
  for (int fb = 0; fb < NF; ++fb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      X[fb][r] *= kNegLn2;
      XT[fb][r] *= kNegLn2;
    }
}

// ---------------------------------------------------------------------------------------------------
// M = 256 tangent kernels (QM9): the forward-mode edge chain with the primal and the tangent in SEQUENTIAL passes
// per layer.  chain_split_tangent interleaves both on every weight fragment, which needs split input + output
// buffers and accumulators for both (6 x 128 registers at NF = 8); here a layer is
//   1. primal pass:  acc  = b' + W X'    (X' split block by block into XA just before its first k-step is needed;
//                                         the accumulators start at the log2-domain bias column)
//   2. tangent pass: accT = W X'_T      (the same fragments streamed again)
//   3. activation:   X'  = u / (1 + 2^u),  X'_T = r (1 - ln2 u (1 - r)) du   (u = acc, du = accT, r = 1/(1+2^u))
// so at most acc + XAT + accT (3 x 128 registers) are live.  X, XT: the log2-domain activations in fp32
// accumulator layout (in_log2 = false: natural-domain input, scaled by -log2 e first); on return the natural-domain
// output (x -ln 2).  Weights: the primal chain's split fragments [layer][group (jb, fb, u)][piece][lane].
// ---------------------------------------------------------------------------------------------------
template <int NF>
__device__ __forceinline__ void split_blocks(const f32x16 (&X)[NF], SplitX<NF>& S) {
  static_for<NF>([&](auto Fc) {
    constexpr int fb = decltype(Fc)::value;
    static_for<8>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value;
      put_pair<NF, fb, 2 * i>(S, X[fb][2 * i], X[fb][2 * i + 1]);
    });
  });
}

// weight groups in flight in dual_pass: 3 pieces x (PF + 1) slots beside the split input, the accumulators and the
// other operand's fp32 activations (512-register waves)
constexpr int kDualPF = 2;
// one pass of one layer over the 3-piece exact weights (chain_split WP = 3): acc[jb] = sum over (fb, u) of
// W[l][jb][fb][u] X'[fb][u] with the w2 x0 term in the PRIMAL pass (the tangent pass keeps three terms)
template <int NF, bool PRIMAL>
__device__ __forceinline__ void dual_pass(const SplitX<NF>& X, f32x16 (&acc)[NF], __amdgpu_buffer_rsrc_t rsrc,
                                          int voff, int layer_soff) {
  constexpr int G = 2 * NF * NF, PF = kDualPF, WP = 3;
  u32x4 wbuf[PF + 1][WP];
  static_for<PF>([&](auto Gc) {
    constexpr int gg = decltype(Gc)::value;
#pragma unroll
    for (int p = 0; p < WP; ++p) wbuf[gg][p] = wload(rsrc, voff, layer_soff + (gg * WP + p) * kPieceBytes);
  });
  static_for<G>([&](auto Gc) {
    constexpr int gg = decltype(Gc)::value;
    constexpr int jb = gg / (2 * NF), fb = (gg % (2 * NF)) >> 1, u = gg & 1;
    if constexpr (gg + PF < G) {
#pragma unroll
      for (int p = 0; p < WP; ++p)
        wbuf[(gg + PF) % (PF + 1)][p] = wload(rsrc, voff, layer_soff + ((gg + PF) * WP + p) * kPieceBytes);
    }
    if constexpr (fb == 0 && u == 0) acc[jb] = f32x16{};
    const u32x4* A = wbuf[gg % (PF + 1)];
    if constexpr (PRIMAL) acc[jb] = mfma_split(A[2], X.v[fb][u][0], acc[jb]);
    static_for<kTerms>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      acc[jb] = mfma_split(A[term_w(t)], X.v[fb][u][term_x(t)], acc[jb]);
    });
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <int NF, int NL>
__device__ __forceinline__ void chain_dual_seq(f32x16 (&X)[NF], f32x16 (&XT)[NF], const unsigned* __restrict__ Wpk,
                                               const float* __restrict__ bias, const float* cinv, int lane,
                                               bool in_log2, bool out_log2 = false) {
  constexpr float kNegLog2e = -1.4426950408889634f, kNegLn2 = -0.69314718055994531f;
  constexpr int WP = 3;   // exact 3-piece weights (chain_split WP = 3)
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(Wpk), (short)0,
                                                                         0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  const float* lbias = bias + 4 * (lane >> 5);
  if (!in_log2) {
#pragma unroll
    for (int fb = 0; fb < NF; ++fb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        X[fb][r] *= kNegLog2e;
        XT[fb][r] *= kNegLog2e;
      }
  }
  // a runtime layer loop with scheduling fences between the phases: only one pass's operands are live at a time
  for (int l = 0; l < NL; ++l) {
    const int soff = l * (2 * NF * NF) * WP * kPieceBytes;
    {
      SplitX<NF> XA;
      split_blocks<NF>(X, XA);
      __builtin_amdgcn_sched_barrier(0);
      dual_pass<NF, true>(XA, X, rsrc, voff, soff);    // X <- s W X' (primal, exact weights)
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      SplitX<NF> XAT;
      split_blocks<NF>(XT, XAT);
      __builtin_amdgcn_sched_barrier(0);
      dual_pass<NF, false>(XAT, XT, rsrc, voff, soff);  // XT <- s W X'_T
    }
    __builtin_amdgcn_sched_barrier(0);
    const float il = cinv[l];   // 1 / the layer's weight scale (read where used: nothing live across the passes)
    const float* lb = lbias + l * NF * 32;
#pragma unroll
    for (int fb = 0; fb < NF; ++fb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // the biases of registers 4q .. 4q+3 (rows acc_row(r, kk) = 8q + 4kk + 0..3): one 16-B LDS read
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(lb + fb * 32 + 8 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * q + i;
          const float u = fmaf(X[fb][r], il, b4[i]);   // u = W X' + b'
          const float rr = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
          const float y = u * rr;
          X[fb][r] = y;
          XT[fb][r] = rr * (XT[fb][r] * il) * fmaf(u - y, kNegLn2, 1.0f);
        }
      }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (out_log2) return;   // the split tangent kernels' log2-domain tail (w_g', w_x' carry the -ln 2)
#pragma unroll
  for (int fb = 0; fb < NF; ++fb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      X[fb][r] *= kNegLn2;
      XT[fb][r] *= kNegLn2;
    }
}
