// chain_split.hpp — the edge-MLP chain on the bf16 matrix cores, fp32-accurate by operand splitting (gfx950).
//
// Why: on gfx950 v_mfma_f32_32x32x2_f32 runs at the fp32 VECTOR rate and shares the SIMD's vector issue, so every
// SiLU / scan instruction of the fp32-MFMA chain adds to its time (measured: tools/micro/chain_bench.hip).  The
// bf16 MFMA (v_mfma_f32_32x32x16_bf16, 32 cycles for 16x the fp32 MFMA's k-depth) runs on the matrix cores and
// leaves 24 of its 32 cycles of vector issue free.
//
// Accuracy: every fp32 operand x is split into three bf16 values by round-to-nearest, x = x0 + x1 + x2 with
// |x1| <= 2^-9 |x|, |x2| <= 2^-17 |x| (exact for all normal x); a product keeps the six cross terms with
// i + j <= 2 (w2x0, w1x1, w0x2, w1x0, w0x1, w0x0, smallest first) and accumulates them in fp32 inside the MFMA.
// The dropped terms are <= 2^-25 |w x|, below fp32's own rounding of the product, so a layer matches the fp32
// GEMM to fp32 summation-order noise (tests/test_gpu_parity.py states the tolerances; DESIGN.md the measured
// errors against the fp64 oracle).
//
// Layout: one 32-edge tile per wave, features on MFMA rows, edges on lanes (as the fp32 chain).  A k-step of
// 16 input features of block fb is accumulator registers 8u..8u+7 (u = 0, 1): lane (c, h) holds features
// f(8u+j, h) = ((8u+j)&3) + 8((8u+j)>>2) + 4h of edge c, exactly the bf16 B-operand slot k = 8h + j, so the
// weights are packed in that permuted k order on the host and activations never move between lanes.
//
// Schedule (one layer = NF output blocks x NF input blocks x 2 k-steps = 2 NF^2 groups of 6 MFMAs, output-block
// major): block jb accumulates in groups [2NF jb, 2NF (jb+1)); block jb-1 is activated (bias, SiLU, split into
// the OTHER activation buffer) one pair of elements per group meanwhile, and the last block of a layer during the
// first 2NF-2 groups of the next, before group (jb 0, fb NF-1) reads it.  The final layer's SiLU stays fp32 in
// place (the tail needs fp32 messages).  Weight groups stream PF groups ahead, contiguous across layers.
#pragma once
// (included by egnn_eval.hpp inside namespace ecnf)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const ECNF_GLOBAL u32x4* gu32x4_p;

// activations of one tile in split form: [input block][k-step u][piece] -> 8 bf16 (4 u32) per lane
template <int NF>
struct SplitX {
  u32x4 v[NF][2][3];
};

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// y0, y1 -> three packed bf16 pairs (RNE), y = p0 + p1 + p2 per element
__device__ __forceinline__ void split3(float y0, float y1, unsigned& p0, unsigned& p1, unsigned& p2) {
  p0 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){y0, y1}, bf16x2));
  float r0 = y0 - __builtin_bit_cast(float, p0 << 16);
  float r1 = y1 - __builtin_bit_cast(float, p0 & 0xffff0000u);
  p1 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
  r0 -= __builtin_bit_cast(float, p1 << 16);
  r1 -= __builtin_bit_cast(float, p1 & 0xffff0000u);
  p2 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
}

// store elements (r, r+1) of block j (accumulator register order) into split buffer X
template <int NF, int J, int R>
__device__ __forceinline__ void put_pair(SplitX<NF>& X, float y0, float y1) {
  static_assert((R & 1) == 0, "pairs start at even registers");
  unsigned p0, p1, p2;
  split3(y0, y1, p0, p1, p2);
  constexpr int u = R >> 3, w = (R & 7) >> 1;
  X.v[J][u][0][w] = p0;
  X.v[J][u][1][w] = p1;
  X.v[J][u][2][w] = p2;
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
// b2 = the biases of rows (R, R+1)
template <int NF, int J, int R, bool SPLIT>
__device__ __forceinline__ void act_pair(f32x16 (&acc)[NF], SplitX<NF>& X, f32x2 b2) {
#ifdef ECNF_SPLIT_CHEAP_ACT   // timing experiment: keep the data flow, drop the arithmetic
  if constexpr (SPLIT) {
    X.v[J][R >> 3][0][(R & 7) >> 1] = __builtin_bit_cast(unsigned, acc[J][R]);
    X.v[J][R >> 3][1][(R & 7) >> 1] = __builtin_bit_cast(unsigned, acc[J][R + 1]);
  }
  return;
#endif
  const float t0 = acc[J][R] + b2[0];
  const float t1 = acc[J][R + 1] + b2[1];
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
__device__ __forceinline__ f32x2 act_stage1(f32x16 (&acc)[NF], f32x2 b2) {
  const float t0 = acc[J][R] + b2[0];
  const float t1 = acc[J][R + 1] + b2[1];
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

// NL chained layers Y = silu(X W_l + b_l).  Input in XA (split form); on return acc holds the last layer's
// activations in fp32 (accumulator layout).  XA / XB are both clobbered.
// Weights: packed split-bf16 fragments [layer][group][piece][lane] (16 B), read as buffer loads with the group
// offset in an SGPR; biases: LDS [NL][M], each activated pair's two (adjacent) rows read one group ahead.
// Each group's MFMAs and activation VALU are emitted together and interleaved by sched_group_barrier: the
// weight loads first, then MFMA / VALU alternately, so the VALU fills the MFMAs' free issue cycles.
template <int NF, int NL>
__device__ __forceinline__ void chain_split(SplitX<NF>& XA, SplitX<NF>& XB, f32x16 (&acc)[NF],
                                            const unsigned* __restrict__ Wpk, const float* __restrict__ bias,
                                            int lane) {
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
  u32x4 wbuf[PF + 1][3];
#pragma unroll
  for (int gg = 0; gg < PF && gg < G; ++gg)
#pragma unroll
    for (int p = 0; p < 3; ++p) wbuf[gg][p] = wload(rsrc, voff, (gg * 3 + p) * 1024);
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
      for (int p = 0; p < 3; ++p) wbuf[(gg + PF) % (PF + 1)][p] = wload(rsrc, voff, ((gg + PF) * 3 + p) * 1024);
    }
    // biases of the next group's pairs
    constexpr int nnext = (gg + 1 < G && task_of(gg + 1).j >= 0) ? task_of(gg + 1).p1 - task_of(gg + 1).p0 : 0;
    static_for<nnext>([&](auto Ic) {
      bnext[Ic] = *reinterpret_cast<const f32x2*>(bias + bias_row(gg + 1, Ic) + 4 * kk);
    });
    const u32x4* A = wbuf[gg % (PF + 1)];
    const u32x4* B = Xin.v[fb][u];
    static_for<6>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      // cross terms, smallest first: (2,0) (1,1) (0,2) (1,0) (0,1) (0,0)  [weight piece, activation piece]
      constexpr int pa = t == 0 ? 2 : (t == 1 || t == 3) ? 1 : 0;
      constexpr int pb = t == 2 ? 2 : (t == 1 || t == 4) ? 1 : 0;
      if constexpr (fb == 0 && u == 0 && t == 0) {
        const f32x16 z = {};
        acc[jb] = mfma_bf16(A[pa], B[pb], z);
      } else {
        acc[jb] = mfma_bf16(A[pa], B[pb], acc[jb]);
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
      ybuf[gg & 1][i] = act_stage1<NF, (tk.j < 0 ? 0 : tk.j), 2 * (tk.p0 + i), split_out>(acc, bcur[i]);
    });
#endif
    // schedule: weight loads, bias reads, then MFMA / VALU alternating
    constexpr int nvalu = npair * 16 + 12 * ((gg > 0 && task_of(gg - 1).j >= 0) ? task_of(gg - 1).p1 - task_of(gg - 1).p0 : 0);
    constexpr int per = (nvalu + 5) / 6;
#ifndef ECNF_SPLIT_NO_SGB
    if constexpr (gg + PF < G) __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
    if constexpr (nnext > 0) __builtin_amdgcn_sched_group_barrier(0x100, nnext, 0);
    static_for<6>([&](auto) {
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
    act_pair<NF, NF - 1, 2 * i, false>(acc, XA, b2);
  });
}
