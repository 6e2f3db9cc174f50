// The production split chain (chain_split.hpp) in isolation: 4 waves/CU, each runs TILES x (2-layer + 3-layer
// segments) on synthetic activations with the real weight packing size and LDS biases.  Cycles per layer.
#include "../../ecnf-baseline-neurips-2023_amd/csrc/egnn_eval.hpp"
#include <cstdio>
#include <vector>
using namespace ecnf;
#ifndef TILES
#define TILES 16
#endif
#ifndef WAVES   // waves per workgroup (= per CU: the launch reserves 120 KiB of LDS per workgroup)
#define WAVES 4
#endif
constexpr int NF = 4, M = 128;
constexpr size_t kLayerU32 = (size_t)2 * NF * NF * kGroupU32;

__global__ __launch_bounds__(64 * WAVES) void kern(const unsigned* __restrict__ W, const float* __restrict__ b, float* out,
                                            unsigned long long* cyc) {
  __shared__ float bias[5 * M];
  for (int i = threadIdx.x; i < 5 * M; i += 64 * WAVES) bias[i] = b[i];
  extern __shared__ float pad[];
  if (threadIdx.x == 0) pad[0] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  SplitX<NF> XA, XB;
  f32x16 acc[NF];
  for (int f = 0; f < NF; ++f)
    for (int u = 0; u < 2; ++u)
      for (int p = 0; p < kPieces; ++p) XA.v[f][u][p] = u32x4{0x3f803f80u + lane, 0x3f00u + f, 0x3e803e80u + u, 0x3c003c00u + p};
  ChainInv inv;
  for (int l = 0; l < 7; ++l) inv.v[l] = 1.0f / 4096;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#ifdef TWO_TILES   // two tiles per wave share every weight fragment (chain_split NT = 2): TILES / 2 pairs
  SplitX<NF> XA2, XB2;
  f32x16 acc2[NF];
  for (int f = 0; f < NF; ++f)
    for (int u = 0; u < 2; ++u)
      for (int p = 0; p < kPieces; ++p) XA2.v[f][u][p] = u32x4{0x3f803f81u + lane, 0x3f01u + f, 0x3e803e81u + u, 0x3c013c00u + p};
  for (int t = 0; t < TILES / 2; ++t) {
    chain_split<NF, 2, 2>(XA, XB, acc, launder_uniform(W), bias, inv, lane, XA2, XB2, acc2);
    static_for<NF>([&](auto Fc) {
      constexpr int fb = decltype(Fc)::value;
      static_for<8>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        put_pair<NF, fb, 2 * i>(XA, acc[fb][2 * i], acc[fb][2 * i + 1]);
        put_pair<NF, fb, 2 * i>(XA2, acc2[fb][2 * i], acc2[fb][2 * i + 1]);
      });
    });
    chain_split<NF, 3, 2>(XA, XB, acc, launder_uniform(W + 2 * kLayerU32), bias + 2 * M, inv, lane, XA2, XB2, acc2);
    static_for<NF>([&](auto Fc) {
      constexpr int fb = decltype(Fc)::value;
      static_for<8>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        put_pair<NF, fb, 2 * i>(XA, acc[fb][2 * i], acc[fb][2 * i + 1]);
        put_pair<NF, fb, 2 * i>(XA2, acc2[fb][2 * i], acc2[fb][2 * i + 1]);
      });
    });
  }
  for (int f = 0; f < NF; ++f)
    for (int r = 0; r < 16; ++r) acc[f][r] += acc2[f][r];
#else
  for (int t = 0; t < TILES; ++t) {
    chain_split<NF, 2>(XA, XB, acc, launder_uniform(W), bias, inv, lane);
    static_for<NF>([&](auto Fc) {
      constexpr int fb = decltype(Fc)::value;
      static_for<8>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        put_pair<NF, fb, 2 * i>(XA, acc[fb][2 * i], acc[fb][2 * i + 1]);
      });
    });
    chain_split<NF, 3>(XA, XB, acc, launder_uniform(W + 2 * kLayerU32), bias + 2 * M, inv, lane);
    static_for<NF>([&](auto Fc) {
      constexpr int fb = decltype(Fc)::value;
      static_for<8>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        put_pair<NF, fb, 2 * i>(XA, acc[fb][2 * i], acc[fb][2 * i + 1]);
      });
    });
  }
#endif
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int f = 0; f < NF; ++f)
    for (int r = 0; r < 16; ++r) s += acc[f][r];
  out[blockIdx.x * 64 * WAVES + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * WAVES + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  const size_t nW = 5 * kLayerU32;
  std::vector<unsigned> hw(nW);
  for (size_t i = 0; i < nW; ++i) hw[i] = 0x3c003c00u + (unsigned)(i * 2654435761u % 4096);
  std::vector<float> hb(5 * M);
  for (int i = 0; i < 5 * M; ++i) hb[i] = 0.01f * (i % 7);
  unsigned* W; float *b, *out; unsigned long long* cyc;
  (void)hipMalloc(&W, nW * 4); (void)hipMalloc(&b, 5 * M * 4); (void)hipMalloc(&out, 256 * 64 * WAVES * 4);   // one float per thread
  (void)hipMalloc(&cyc, 256 * WAVES * 8);   // one slot per wave
  (void)hipMemcpy(W, hw.data(), nW * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, hb.data(), 5 * M * 4, hipMemcpyHostToDevice);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
  std::vector<unsigned long long> hc(256 * WAVES);
  for (int rep = 0; rep < 4; ++rep) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(64 * WAVES), 120 * 1024, 0, W, b, out, cyc);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(hc.data(), cyc, 256 * WAVES * 8, hipMemcpyDeviceToHost);
    double m = 0; for (auto c : hc) m += c; m /= hc.size();
    if (rep == 3) printf("split chain: %.0f cycles/layer per wave (tile-layers %d per wave; MFMA-bound %d per tile-layer), %.3f ms\n", m / (TILES * 5.0), TILES * 5, 32 * kTerms * 32, ms);
  }
  return 0;
}
