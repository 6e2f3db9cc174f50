// Microbenchmark: cycles per v_mfma_f32_32x32x2_f32 for one wave per SIMD with K independent VALU ops
// (and optionally transcendentals) interleaved per MFMA.  Two accumulators alternate (no dependent stall).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KV, int KT>
__global__ __launch_bounds__(256) void kern(float* out, unsigned long long* cyc, int iters, float seed) {
  f32x16 a0 = {}, a1 = {};
  float a = seed + threadIdx.x * 1e-3f, b = seed * 0.5f;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = seed + i;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, a0, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < KV; ++k) v[k & 7] = v[k & 7] * 1.0001f + 0.5f;
#pragma unroll
      for (int k = 0; k < KT; ++k) v[(k + 3) & 7] = __expf(v[(k + 3) & 7]);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, a1, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < KV; ++k) v[(k + 5) & 7] = v[(k + 5) & 7] * 0.9999f + 0.25f;
#pragma unroll
      for (int k = 0; k < KT; ++k) v[(k + 1) & 7] = __builtin_amdgcn_rcpf(v[(k + 1) & 7]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a0[i] + a1[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KV, int KT>
void run(float* out, unsigned long long* cyc, unsigned long long* h, int iters) {
  hipLaunchKernelGGL((kern<KV, KT>), dim3(256), dim3(256), 0, 0, out, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  hipMemcpy(h, cyc, 256 * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  m /= 256;
  printf("VALU/MFMA=%d TRANS/MFMA=%d : %.1f cycles per MFMA\n", KV, KT, m / (iters * 32.0));
}

int main() {
  float* out; unsigned long long* cyc; unsigned long long h[256];
  hipMalloc(&out, 256 * 256 * 4); hipMalloc(&cyc, 256 * 8);
  const int it = 2000;
  run<0, 0>(out, cyc, h, it); run<0, 0>(out, cyc, h, it);
  run<2, 0>(out, cyc, h, it); run<4, 0>(out, cyc, h, it); run<8, 0>(out, cyc, h, it);
  run<12, 0>(out, cyc, h, it); run<16, 0>(out, cyc, h, it);
  run<0, 1>(out, cyc, h, it); run<0, 2>(out, cyc, h, it); run<0, 4>(out, cyc, h, it);
  run<4, 2>(out, cyc, h, it); run<8, 2>(out, cyc, h, it);
  return 0;
}
