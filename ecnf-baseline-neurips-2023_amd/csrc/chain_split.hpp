// chain_split.hpp — the edge-MLP chain on the 16-bit matrix cores, fp32-accurate by operand splitting (gfx950).
//
// Why: on gfx950 v_mfma_f32_32x32x2_f32 runs at the fp32 VECTOR rate and shares the SIMD's vector issue, so every
// SiLU / scan instruction of the fp32-MFMA chain adds to its time (measured: tools/micro/chain_bench.hip).  The
// 16-bit MFMAs (v_mfma_f32_32x32x16_{f16,bf16}, 32 cycles for 16x the fp32 MFMA's k-depth) run on the matrix cores
// and leave 24 of their 32 cycles of vector issue free.
//
// Accuracy (default, fp16 pieces): every fp32 operand x is split into two fp16 values by round-to-nearest,
// x = x0 + x1, |x - x0| <= 2^-11 |x|, and x1 = fp16(x - x0) carries the rest to 2^-22 |x| (one v_cvt_pk_f16_f32
// and two v_fma_mix per pair of values).  A product keeps the three cross terms w1x0, w0x1, w0x0 (smallest first)
// and accumulates them in fp32 inside the MFMA; the dropped w1x1 and the piece roundings are <= 2^-21 |w x|.
// Weights are split on the host after scaling each matrix by a power of two s (max |w s| in [2^12, 2^13)), so
// both weight pieces are normal fp16 numbers; the epilogue multiplies the accumulator by 1/s (exact) in the FMA
// that adds the bias.  Activations are split unscaled: fp16 holds |x| < 65504, and below 2^-14 the fp16
// subnormals keep the absolute error of a piece <= 2^-25.
// -DECNF_SPLIT_BF16 builds the earlier form: three bf16 pieces (x0 + x1 + x2, |x2| <= 2^-17 |x|), six cross terms
// (w2x0, w1x1, w0x2, w1x0, w0x1, w0x0), no scaling (bf16 has fp32's exponent range).
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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const ECNF_GLOBAL u32x4* gu32x4_p;

#ifdef ECNF_SPLIT_BF16
constexpr int kPieces = 3;
constexpr int kTerms = 6;
#else
constexpr int kPieces = 2;
constexpr int kTerms = 3;
#endif
// cross term t: (weight piece, activation piece), smallest first
__host__ __device__ constexpr int term_w(int t) {
  return kPieces == 3 ? (t == 0 ? 2 : (t == 1 || t == 3) ? 1 : 0) : (t == 0 ? 1 : 0);
}
__host__ __device__ constexpr int term_x(int t) {
  return kPieces == 3 ? (t == 2 ? 2 : (t == 1 || t == 4) ? 1 : 0) : (t == 1 ? 1 : 0);
}
// bytes of one split group / k-step fragment set: kPieces x 64 lanes x 16 B
constexpr int kPieceBytes = 1024;
constexpr int kGroupU32 = kPieces * 256;

// activations of one tile in split form: [input block][k-step u][piece] -> 8 16-bit values (4 u32) per lane
template <int NF>
struct SplitX {
  u32x4 v[NF][2][kPieces];
};

__device__ __forceinline__ f32x16 mfma_split(u32x4 a, u32x4 b, const f32x16& c) {
#ifdef ECNF_SPLIT_BF16
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                0, 0);
#endif
}

// y0, y1 -> kPieces packed 16-bit pairs (RNE), y = sum of the pieces per element
__device__ __forceinline__ void split_pair(float y0, float y1, unsigned (&p)[kPieces]) {
#ifdef ECNF_SPLIT_BF16
  p[0] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){y0, y1}, bf16x2));
  float r0 = y0 - __builtin_bit_cast(float, p[0] << 16);
  float r1 = y1 - __builtin_bit_cast(float, p[0] & 0xffff0000u);
  p[1] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
  r0 -= __builtin_bit_cast(float, p[1] << 16);
  r1 -= __builtin_bit_cast(float, p[1] & 0xffff0000u);
  p[2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
#else
  p[0] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){y0, y1}, f16x2));
  // p1 = fp16(y - fp16 piece 0) per half: the mixed-precision FMA reads the f16 half directly, the difference is
  // exact in fp32 and rounded once (hipcc does not form v_fma_mix from C here)
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo)
      : "v"(p[0]), "v"(y0), "v"(y1));
  p[1] = lo;
#endif
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

template <int NF>
struct SplitPlan {
  static constexpr int GB = 2 * NF;        // groups per output block
  static constexpr int GL = NF * GB;       // groups per layer
  // groups of the next layer available to the last block: its split (stage 2) runs one group after its SiLU
  // (stage 1) and must land before group (jb 0, fb NF-1) reads it
  static constexpr int WIN = 2 * NF - 3 > 0 ? 2 * NF - 3 : 1;
  // activation work of group g of a layer: {block, layer offset, first pair, end pair}; block -1 = none.
  // pairs are 0..7 (16 elements of a block)
  struct Task { int j, dl, p0, p1; };
  static constexpr Task task(int g, bool has_prev) {
    const int jb = g / GB, k = g % GB;
    // block jb-1 during the first GB-1 groups of block jb (its stage 2 then lands inside this layer)
    if (jb >= 1) return k < GB - 1 ? Task{jb - 1, 0, (8 * k) / (GB - 1), (8 * (k + 1)) / (GB - 1)} : Task{-1, 0, 0, 0};
    if (has_prev && k < WIN) return Task{NF - 1, -1, (8 * k) / WIN, (8 * (k + 1)) / WIN};
    return Task{-1, 0, 0, 0};
  }
  // MFMA slot (1..5 of the group's 6) after which pair number i of n is issued
  static constexpr int slot(int i, int n) { return 1 + (i * 5) / (n > 0 ? n : 1); }
};

// element pair activation: y = silu(acc + b) (Dense then SiLU, mlp.py:14), either split into X or fp32 in place;
// b2 = the biases of rows (R, R+1), inv = 1 / (the layer's weight scale)
template <int NF, int J, int R, bool SPLIT>
__device__ __forceinline__ void act_pair(f32x16 (&acc)[NF], SplitX<NF>& X, f32x2 b2, float inv) {
#ifdef ECNF_SPLIT_CHEAP_ACT   // timing experiment: keep the data flow, drop the arithmetic
  if constexpr (SPLIT) {
    X.v[J][R >> 3][0][(R & 7) >> 1] = __builtin_bit_cast(unsigned, acc[J][R]);
    X.v[J][R >> 3][1][(R & 7) >> 1] = __builtin_bit_cast(unsigned, acc[J][R + 1]);
  }
  return;
#endif
  const float t0 = fmaf(acc[J][R], inv, b2[0]);
  const float t1 = fmaf(acc[J][R + 1], inv, b2[1]);
  const float y0 = t0 * sigmoidf_(t0);
  const float y1 = t1 * sigmoidf_(t1);
  if constexpr (SPLIT) {
#ifdef ECNF_SPLIT_NO_SPLIT
    X.v[J][R >> 3][0][(R & 7) >> 1] = __builtin_bit_cast(unsigned, y0) ^ __builtin_bit_cast(unsigned, y1);
#else
    put_pair<NF, J, R>(X, y0, y1);
#endif
  } else {
    acc[J][R] = y0;
    acc[J][R + 1] = y1;
  }
}

// the activation in two stages, one group apart (software pipelined for ILP):
//   stage 1: y = silu(acc + b) -> y2 (kept fp32 in place in acc for the final layer)
//   stage 2: split y2 into the three bf16 pieces of the next layer's input
template <int NF, int J, int R, bool SPLIT>
__device__ __forceinline__ f32x2 act_stage1(f32x16 (&acc)[NF], f32x2 b2, float inv) {
  const float t0 = fmaf(acc[J][R], inv, b2[0]);
  const float t1 = fmaf(acc[J][R + 1], inv, b2[1]);
  const float y0 = t0 * sigmoidf_(t0);
  const float y1 = t1 * sigmoidf_(t1);
  if constexpr (!SPLIT) {
    acc[J][R] = y0;
    acc[J][R + 1] = y1;
  }
  return f32x2{y0, y1};
}

template <int I, typename A, typename B>
__device__ __forceinline__ auto& pick(A& a, B& b) {
  if constexpr (I == 0) return a; else return b;
}

#ifndef ECNF_SPLIT_PF
#define ECNF_SPLIT_PF 3
#endif

__device__ __forceinline__ u32x4 wload(__amdgpu_buffer_rsrc_t rsrc, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
}

// per-layer 1 / weight scale of a chain segment (wave-uniform)
struct ChainInv {
  float v[2 * 4 - 1];
};

// NL chained layers Y = silu(X W_l + b_l).  Input in XA (split form); on return acc holds the last layer's
// activations in fp32 (accumulator layout).  XA / XB are both clobbered.
// Weights: packed split fragments [layer][group][piece][lane] (16 B), read as buffer loads with the group
// offset in an SGPR; biases: LDS [NL][M], each activated pair's two (adjacent) rows read one group ahead;
// inv.v[l]: 1 / the weight scale of layer l.
// Each group's MFMAs and activation VALU are emitted together and interleaved by sched_group_barrier: the
// weight loads first, then MFMA / VALU alternately, so the VALU fills the MFMAs' free issue cycles.
template <int NF, int NL>
__device__ __forceinline__ void chain_split(SplitX<NF>& XA, SplitX<NF>& XB, f32x16 (&acc)[NF],
                                            const unsigned* __restrict__ Wpk, const float* __restrict__ bias,
                                            const ChainInv& inv, int lane) {
  using Plan = SplitPlan<NF>;
  constexpr int GB = Plan::GB, GL = Plan::GL, G = NL * GL, M = NF * 32, PF = ECNF_SPLIT_PF;
  constexpr int kMaxPair = 8;
  const int kk = lane >> 5;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(Wpk), (short)0,
                                                                         0x7fffffff, 0x00020000);
  const int voff = lane * 16;
  // task of global group gg (any layer), and the LDS bias address of its pair i
  auto task_of = [](int gg2) constexpr { return Plan::task(gg2 % GL, gg2 / GL > 0); };
  auto bias_row = [](int gg2, int i) constexpr {
    const typename Plan::Task t = Plan::task(gg2 % GL, gg2 / GL > 0);
    const int r = 2 * (t.p0 + i);
    return (gg2 / GL + t.dl) * M + t.j * 32 + 8 * (r >> 2) + (r & 3);
  };
  u32x4 wbuf[PF + 1][kPieces];
#pragma unroll
  for (int gg = 0; gg < PF && gg < G; ++gg)
#pragma unroll
    for (int p = 0; p < kPieces; ++p) wbuf[gg][p] = wload(rsrc, voff, (gg * kPieces + p) * kPieceBytes);
  f32x2 bcur[kMaxPair], bnext[kMaxPair];
  f32x2 ybuf[2][kMaxPair];                                // stage-1 results, by group parity
  {
    constexpr typename Plan::Task t0 = Plan::task(0, false);
    if constexpr (t0.j >= 0)
      static_for<t0.p1 - t0.p0>([&](auto Ic) {
        bcur[Ic] = *reinterpret_cast<const f32x2*>(bias + bias_row(0, Ic) + 4 * kk);
      });
  }
  static_for<G>([&](auto GGc) {
    constexpr int gg = decltype(GGc)::value;
    constexpr int l = gg / GL, g = gg % GL, jb = g / GB, fb = (g % GB) >> 1, u = g & 1;
    constexpr typename Plan::Task tk = task_of(gg);
    constexpr int tl = l + tk.dl;                          // layer whose block is activated here
    constexpr bool split_out = tl < NL - 1;                // final layer stays fp32 in acc
    constexpr int npair = tk.j >= 0 ? tk.p1 - tk.p0 : 0;
    auto& Xin = pick<l & 1>(XA, XB);
    if constexpr (gg + PF < G) {
#pragma unroll
      for (int p = 0; p < kPieces; ++p)
        wbuf[(gg + PF) % (PF + 1)][p] = wload(rsrc, voff, ((gg + PF) * kPieces + p) * kPieceBytes);
    }
    // biases of the next group's pairs
    constexpr int nnext = (gg + 1 < G && task_of(gg + 1).j >= 0) ? task_of(gg + 1).p1 - task_of(gg + 1).p0 : 0;
    static_for<nnext>([&](auto Ic) {
      bnext[Ic] = *reinterpret_cast<const f32x2*>(bias + bias_row(gg + 1, Ic) + 4 * kk);
    });
    const u32x4* A = wbuf[gg % (PF + 1)];
    const u32x4* B = Xin.v[fb][u];
    static_for<kTerms>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      constexpr int pa = term_w(t), pb = term_x(t);   // cross terms, smallest first
      if constexpr (fb == 0 && u == 0 && t == 0) {
        const f32x16 z = {};
        acc[jb] = mfma_split(A[pa], B[pb], z);
      } else {
        acc[jb] = mfma_split(A[pa], B[pb], acc[jb]);
      }
    });
#ifndef ECNF_SPLIT_NO_ACT
    // stage 2 of the previous group's pairs (split into that layer's output buffer)
    if constexpr (gg > 0) {
      constexpr typename Plan::Task tp = task_of(gg - 1);
      constexpr int lp = (gg - 1) / GL + tp.dl;
      if constexpr (tp.j >= 0 && lp < NL - 1) {
        auto& Xp = pick<(lp + 1) & 1>(XA, XB);
        static_for<tp.p1 - tp.p0>([&](auto Ic) {
          constexpr int i = decltype(Ic)::value;
          put_pair<NF, tp.j, 2 * (tp.p0 + i)>(Xp, ybuf[(gg - 1) & 1][i][0], ybuf[(gg - 1) & 1][i][1]);
        });
      }
    }
    // stage 1 of this group's pairs
    static_for<npair>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value;
      ybuf[gg & 1][i] = act_stage1<NF, (tk.j < 0 ? 0 : tk.j), 2 * (tk.p0 + i), split_out>(acc, bcur[i], inv.v[tl]);
    });
#endif
    // schedule: weight loads, bias reads, then MFMA / VALU alternating
    constexpr int nvalu = npair * 16 + (kPieces == 3 ? 12 : 1) *
                                            ((gg > 0 && task_of(gg - 1).j >= 0) ? task_of(gg - 1).p1 - task_of(gg - 1).p0 : 0);
    constexpr int per = (nvalu + kTerms - 1) / kTerms;
#ifndef ECNF_SPLIT_NO_SGB
    if constexpr (gg + PF < G) __builtin_amdgcn_sched_group_barrier(0x020, kPieces, 0);
    if constexpr (nnext > 0) __builtin_amdgcn_sched_group_barrier(0x100, nnext, 0);
    static_for<kTerms>([&](auto) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if constexpr (per > 0) __builtin_amdgcn_sched_group_barrier(0x002, per, 0);
    });
#endif
    __builtin_amdgcn_sched_barrier(0);
    static_for<nnext>([&](auto Ic) { bcur[Ic] = bnext[Ic]; });
  });
  {
    constexpr typename Plan::Task tp = task_of(G - 1);
    constexpr int lp = (G - 1) / GL + tp.dl;
    if constexpr (tp.j >= 0 && lp < NL - 1) {
      auto& Xp = pick<(lp + 1) & 1>(XA, XB);
      static_for<tp.p1 - tp.p0>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        put_pair<NF, tp.j, 2 * (tp.p0 + i)>(Xp, ybuf[(G - 1) & 1][i][0], ybuf[(G - 1) & 1][i][1]);
      });
    }
  }
  // the final layer's last block
  static_for<8>([&](auto Ic) {
    constexpr int i = decltype(Ic)::value;
    const f32x2 b2 = *reinterpret_cast<const f32x2*>(bias + (NL - 1) * M + (NF - 1) * 32 + 8 * ((2 * i) >> 2) +
                                                     ((2 * i) & 3) + 4 * kk);
    act_pair<NF, NF - 1, 2 * i, false>(acc, XA, b2, inv.v[NL - 1]);
  });
}
