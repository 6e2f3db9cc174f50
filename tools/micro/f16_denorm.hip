// Does v_mfma_f32_32x32x16_f16 honour fp16 subnormal inputs on gfx950, and does the v_fma_mix split of
// chain_split.hpp reconstruct x = p0 + p1 to 2^-22?  Prints PASS/FAIL lines.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/micro/f16_denorm.hip -o tools/micro/f16_denorm
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../ecnf-baseline-neurips-2023_amd/csrc/egnn_eval.hpp"
using namespace ecnf;

__global__ void mfma_denorm(float a_val_f32, float* out) {
  const int l = threadIdx.x;
  u32x4 a, b;
  const _Float16 av = (_Float16)a_val_f32, one = (_Float16)1.0f;
  const unsigned ap = __builtin_bit_cast(unsigned short, av) | ((unsigned)__builtin_bit_cast(unsigned short, av) << 16);
  const unsigned bp = __builtin_bit_cast(unsigned short, one) | ((unsigned)__builtin_bit_cast(unsigned short, one) << 16);
  for (int i = 0; i < 4; ++i) { a[i] = ap; b[i] = bp; }
  f32x16 c = {};
  c = mfma_split(a, b, c);
  out[l] = c[0];
}

__global__ void split_check(const float* x, float* rec, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned p[kPieces];
  split_pair(x[2 * i], x[2 * i + 1], p);
  float r0 = 0.f, r1 = 0.f;
  for (int k = kPieces - 1; k >= 0; --k) {
    r0 += (float)__builtin_bit_cast(_Float16, (unsigned short)(p[k] & 0xffff));
    r1 += (float)__builtin_bit_cast(_Float16, (unsigned short)(p[k] >> 16));
  }
  rec[2 * i] = r0;
  rec[2 * i + 1] = r1;
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4);
  bool ok = true;
  for (float v : {std::ldexp(1.0f, -20), std::ldexp(3.0f, -24), std::ldexp(1.0f, -14), 0.5f}) {
    hipLaunchKernelGGL(mfma_denorm, dim3(1), dim3(64), 0, 0, v, d);
    float h[64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const float expect = 16.0f * v;
    const bool pass = h[0] == expect;
    ok &= pass;
    printf("%s mfma f16 input %.6g x 16 -> %.9g (expect %.9g)\n", pass ? "PASS" : "FAIL", v, h[0], expect);
  }
  const int n = 1 << 20;
  std::vector<float> x(n);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (s >> 8) * (1.0f / 16777216.0f);
    s = s * 1664525u + 1013904223u;
    const int e = (int)(s >> 27) - 20;   // magnitudes 2^-20 .. 2^11
    x[i] = (u - 0.5f) * std::ldexp(1.0f, e);
  }
  float *dx, *dr;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dr, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(split_check, dim3(n / 2 / 256), dim3(256), 0, 0, dx, dr, n);
  std::vector<float> r(n);
  hipMemcpy(r.data(), dr, n * 4, hipMemcpyDeviceToHost);
  // bound: |x - p0 - p1| <= max(2^-22 |x|, 2^-25) (relative above 2^-3, the fp16 subnormal spacing below)
  double worst = 0, worst_abs = 0, worst_ratio = 0;
  for (int i = 0; i < n; ++i) {
    const double err = std::fabs((double)r[i] - (double)x[i]);
    const double ax = std::fabs((double)x[i]);
    if (ax >= 0.125) worst = std::max(worst, err / ax);
    else worst_abs = std::max(worst_abs, err);
    worst_ratio = std::max(worst_ratio, err / std::max(std::ldexp(ax, -22), std::ldexp(1.0, -25)));
  }
  const bool pass = worst_ratio <= 1.0;
  ok &= pass;
  printf("%s split reconstruct: max rel err %.3g (2^%.1f) for |x| >= 2^-3, max abs err %.3g below; "
         "err / max(2^-22 |x|, 2^-25) <= %.3f\n", pass ? "PASS" : "FAIL", worst, std::log2(worst), worst_abs, worst_ratio);
  return ok ? 0 : 1;
}
