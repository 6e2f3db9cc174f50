// Microbenchmark of the edge-MLP chain in isolation: every wave runs TILES x (phi_e 2 layers + phi_x 3 layers)
// of chain_segment<4, 0, *> on register-resident activations, weights streamed from a 2 MB buffer (5 layers of
// fragment-packed 128x128), biases from LDS.  Reports cycles per MFMA per SIMD.
#include "../../ecnf-baseline-neurips-2023_amd/csrc/egnn_eval.hpp"
#include <cstdio>
#include <vector>
#include <algorithm>
using namespace ecnf;

#ifndef WAVES
#define WAVES 8
#endif
#ifndef TILES
#define TILES 64
#endif

__global__ __launch_bounds__(64 * WAVES) void chain_kernel(const float* __restrict__ W, const float* __restrict__ b,
                                                           float* out, unsigned long long* cyc, float seed) {
  __shared__ float bias[5 * 128];
  for (int i = threadIdx.x; i < 5 * 128; i += 64 * WAVES) bias[i] = b[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f32x16 X[4], XT[4];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) X[f][r] = seed * (0.01f * (f * 16 + r) - 0.3f) + 1e-3f * lane;
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < TILES; ++t) {
    const float* w0 = launder_uniform(W);
    chain_segment<4, 0, 2>(X, XT, w0, bias, lane);
    const float* w1 = launder_uniform(W + 2 * 128 * 128);
    chain_segment<4, 0, 3>(X, XT, w1, bias + 2 * 128, lane);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += X[f][r];
  out[blockIdx.x * 64 * WAVES + threadIdx.x] = s;
  if (lane == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID (id 4), 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID (id 20)
    if ((threadIdx.x >> 6) == 0) {
      cyc[4 * 256 * WAVES + blockIdx.x * 4 + 0] = r0;
      cyc[4 * 256 * WAVES + blockIdx.x * 4 + 1] = r1;
      cyc[4 * 256 * WAVES + blockIdx.x * 4 + 2] = hw;
      cyc[4 * 256 * WAVES + blockIdx.x * 4 + 3] = xcc;
    }
    cyc[blockIdx.x * WAVES + (threadIdx.x >> 6)] = t1 - t0;
    cyc[256 * WAVES + blockIdx.x * WAVES + (threadIdx.x >> 6)] = r1 - r0;
  }
}

int main() {
  const int nW = 5 * 128 * 128;
  std::vector<float> hw(nW), hb(5 * 128);
  for (int i = 0; i < nW; ++i) hw[i] = ((i * 2654435761u) % 1000) * 1e-4f - 0.05f;
  for (int i = 0; i < 5 * 128; ++i) hb[i] = 0.01f * (i % 7);
  float *W, *b, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&W, nW * 4); (void)hipMalloc(&b, 5 * 128 * 4);
  (void)hipMalloc(&out, 256 * 64 * WAVES * 4); (void)hipMalloc(&cyc, (4 * 256 * WAVES + 1024) * 8);
  (void)hipMemcpy(W, hw.data(), nW * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, hb.data(), 5 * 128 * 4, hipMemcpyHostToDevice);
  std::vector<unsigned long long> hc(4 * 256 * WAVES + 1024);
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(64 * WAVES), 0, 0, W, b, out, cyc, 1.0f);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(hc.data(), cyc, (4 * 256 * WAVES + 1024) * 8, hipMemcpyDeviceToHost);
    double m = 0, rt = 0; for (int i = 0; i < 256 * WAVES; ++i) { m += hc[i]; rt += hc[256 * WAVES + i]; }
    m /= 256 * WAVES; rt /= 256 * WAVES;
    const double mfma_per_wave = TILES * 5.0 * 256;
    // cycles per MFMA per SIMD: each SIMD runs WAVES/4 waves
    printf("WAVES=%d TILES=%d: %.1f cycles/MFMA/SIMD (wave mean %.0f cyc, %.1f us real -> %.3f GHz), %.3f ms, %.1f TFLOP/s\n", WAVES, TILES,
           m / (mfma_per_wave * WAVES / 4), m, rt / 100.0, m / (rt * 10.0), ms, 256.0 * WAVES * mfma_per_wave * 4096 / (ms * 1e-3) / 1e12);
    if (rep == 2) {
      unsigned long long smin = ~0ull;
      for (int g = 0; g < 256; ++g) smin = std::min(smin, hc[4 * 256 * WAVES + g * 4]);
      for (int g = 0; g < 256; ++g) {
        const unsigned long long* q = &hc[4 * 256 * WAVES + g * 4];
        const unsigned hw = (unsigned)q[2];
        printf("wg %3d xcc %llu se %u cu %2u start %6.1f us dur %7.1f us\n", g, q[3] & 15, (hw >> 13) & 7,
               (hw >> 8) & 15, (q[0] - smin) / 100.0, (q[1] - q[0]) / 100.0);
      }
    }
  }
  return 0;
}
