// Microbenchmark 2: two waves per SIMD (8 waves per workgroup, one workgroup per CU).  Waves 0-3: MFMA-only
// stream (v_mfma_f32_32x32x2_f32, two accumulators).  Waves 4-7: VALU-only stream (fma + exp/rcp) or idle.
// Does the VALU wave run concurrently with the fp32 MFMA wave on the same SIMD?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>   // 0: MFMA waves only, 1: MFMA + VALU waves, 2: VALU waves only
__global__ __launch_bounds__(512) void kern(float* out, unsigned long long* cyc, int iters, float seed) {
  const int wave = threadIdx.x >> 6;
  float s = 0.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < 4) {
    if (MODE != 2) {
      f32x16 a0 = {}, a1 = {};
      float a = seed + threadIdx.x * 1e-3f, b = seed * 0.5f;
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, a1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) s += a0[i] + a1[i];
    }
  } else {
    if (MODE != 0) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = seed + i + threadIdx.x;
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = v[k] * 1.0001f + 0.5f;
#pragma unroll
          for (int k = 0; k < 2; ++k) v[k + 3] = __builtin_amdgcn_rcpf(__expf(-v[k + 3]) + 1.0f);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int MODE>
void run(float* out, unsigned long long* cyc, unsigned long long* h, int iters, const char* name) {
  hipLaunchKernelGGL((kern<MODE>), dim3(256), dim3(512), 0, 0, out, cyc, iters, 1.0f);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h, cyc, 256 * 8 * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0;
  for (int i = 0; i < 256; ++i) {
    for (int w = 0; w < 4; ++w) m0 += h[i * 8 + w];
    for (int w = 4; w < 8; ++w) m1 += h[i * 8 + w];
  }
  m0 /= 1024 * (iters * 32.0);
  m1 /= 1024 * (iters * 16.0);
  printf("%-22s MFMA waves: %.1f cyc/MFMA   VALU waves: %.1f cyc per (8 fma + 2 sigmoid) block\n", name, m0, m1);
}

int main() {
  float* out; unsigned long long* cyc; unsigned long long h[256 * 8];
  (void)hipMalloc(&out, 256 * 512 * 4); (void)hipMalloc(&cyc, 256 * 8 * 8);
  run<0>(out, cyc, h, 2000, "warmup");
  run<0>(out, cyc, h, 2000, "mfma only");
  run<2>(out, cyc, h, 2000, "valu only");
  run<1>(out, cyc, h, 2000, "mfma + valu waves");
  return 0;
}
