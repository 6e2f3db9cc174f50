// Feasibility microbenchmark for a split-bf16 (3 pieces, 6 cross terms) edge chain on gfx950:
// 4 waves/CU (one per SIMD), each streams bf16 A fragments (3 pieces per 16-deep k-step) from a 480 KB weight
// region through L2/L1 and issues 6*NS v_mfma_f32_32x32x16_bf16 per group (NS = activation streams sharing each
// A fragment), optionally with NFILL elements of SiLU + 3-way bf16 split per group interleaved between the MFMAs.
// Reports cycles per group (ideal: 6*NS*32 cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <utility>
#include <type_traits>

#ifndef NS
#define NS 2
#endif
#ifndef NPF
#define NPF 3
#endif
#ifndef NFILL
#define NFILL 0
#endif
#ifndef NWAVES
#define NWAVES 4
#endif
#ifndef LOADSRC
#define LOADSRC 0   // 0: global (L2/L1), 1: none (fragments stay in registers), 2: LDS
#endif
constexpr int kGroups = 32;   // per layer (NF = 4: 4 fb x 2 u x 4 jb)
constexpr int kLayers = 5;
constexpr int kTiles = 16;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gu32x4_p;

template <typename Fn, int... I>
__device__ __forceinline__ void sfor_impl(Fn&& f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename Fn>
__device__ __forceinline__ void sfor(Fn&& f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// SiLU then RNE split of two values into three packed bf16 pairs
__device__ __forceinline__ void act_split(float a0, float a1, float b, unsigned& p0, unsigned& p1, unsigned& p2) {
  float t0 = a0 + b, t1 = a1 + b;
  float y0 = t0 * __builtin_amdgcn_rcpf(1.0f + __expf(-t0));
  float y1 = t1 * __builtin_amdgcn_rcpf(1.0f + __expf(-t1));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 h = __builtin_convertvector((f32x2){y0, y1}, bf16x2);
  p0 = __builtin_bit_cast(unsigned, h);
  float r0 = y0 - __builtin_bit_cast(float, p0 << 16), r1 = y1 - __builtin_bit_cast(float, p0 & 0xffff0000u);
  h = __builtin_convertvector((f32x2){r0, r1}, bf16x2);
  p1 = __builtin_bit_cast(unsigned, h);
  r0 = r0 - __builtin_bit_cast(float, p1 << 16); r1 = r1 - __builtin_bit_cast(float, p1 & 0xffff0000u);
  h = __builtin_convertvector((f32x2){r0, r1}, bf16x2);
  p2 = __builtin_bit_cast(unsigned, h);
}

__global__ __launch_bounds__(64 * NWAVES) void kern(const unsigned* __restrict__ W, float* out, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  __shared__ u32x4 lw[8 * 3 * 64];   // 24 KB: 8 groups of fragments
  for (int i = threadIdx.x; i < 8 * 3 * 64; i += 64 * NWAVES) lw[i] = ((const u32x4*)W)[i];
  __syncthreads();
  u32x4 X[NS][4][2][3];     // [stream][fb][u][piece]
  f32x16 acc[NS][4];
  for (int s = 0; s < NS; ++s)
    for (int f = 0; f < 4; ++f)
      for (int u = 0; u < 2; ++u)
        for (int p = 0; p < 3; ++p) X[s][f][u][p] = u32x4{0x3f803f80u + lane + s, 0x3f00u + f, 0x3e803e80u + u, 0x3c003c00u + p};
  for (int s = 0; s < NS; ++s)
    for (int j = 0; j < 4; ++j) acc[s][j] = f32x16{};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < kTiles; ++t) {
    for (int l = 0; l < kLayers; ++l) {
      unsigned long long wv = (unsigned long long)(W + (size_t)l * kGroups * 3 * 64 * 4);
      const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)wv), hi = __builtin_amdgcn_readfirstlane((unsigned)(wv >> 32));
      gu32x4_p wp = (gu32x4_p)(((unsigned long long)hi << 32) | lo);
      wp += lane;
      u32x4 wb[NPF + 1][3];
      sfor<NPF>([&](auto Gc) { constexpr int g = decltype(Gc)::value;
        for (int p = 0; p < 3; ++p) wb[g][p] = wp[(g * 3 + p) * 64]; });
      sfor<kGroups>([&](auto Gc) {
        constexpr int g = decltype(Gc)::value;
        constexpr int jb = g & 3, u = (g >> 2) & 1, fb = g >> 3;
        if constexpr (g + NPF < kGroups && LOADSRC == 0) {
          for (int p = 0; p < 3; ++p) wb[(g + NPF) % (NPF + 1)][p] = wp[((g + NPF) * 3 + p) * 64];
        }
        if constexpr (g + NPF < kGroups && LOADSRC == 2) {
          for (int p = 0; p < 3; ++p) wb[(g + NPF) % (NPF + 1)][p] = lw[((((g + NPF) % 8) * 3 + p) * 64) + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        const u32x4* A = wb[g % (NPF + 1)];
        sfor<NS>([&](auto Sc) {
          constexpr int s = decltype(Sc)::value;
          acc[s][jb] = mfma(A[2], X[s][fb][u][0], acc[s][jb]);
          acc[s][jb] = mfma(A[1], X[s][fb][u][1], acc[s][jb]);
          acc[s][jb] = mfma(A[0], X[s][fb][u][2], acc[s][jb]);
          acc[s][jb] = mfma(A[1], X[s][fb][u][0], acc[s][jb]);
          acc[s][jb] = mfma(A[0], X[s][fb][u][1], acc[s][jb]);
          acc[s][jb] = mfma(A[0], X[s][fb][u][0], acc[s][jb]);
        });
        // NFILL elements of activation work: from a finished block into a block not read in the next groups
        sfor<(NFILL + 1) / 2>([&](auto Ec) {
          constexpr int e = decltype(Ec)::value;
          constexpr int s = e % NS, src = (jb + 2) & 3, dst = (fb + 2) & 3, r = (2 * e) & 15;
          unsigned p0, p1, p2;
          act_split(acc[s][src][r], acc[s][src][r + 1], 0.01f * e, p0, p1, p2);
          X[s][dst][(e >> 2) & 1][0][(e >> 1) & 3] = p0;
          X[s][dst][(e >> 2) & 1][1][(e >> 1) & 3] = p1;
          X[s][dst][(e >> 2) & 1][2][(e >> 1) & 3] = p2;
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int s = 0; s < NS; ++s)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) sum += acc[s][j][r];
  out[blockIdx.x * 64 * NWAVES + threadIdx.x] = sum;
  if (lane == 0) cyc[blockIdx.x * NWAVES + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  const size_t nW = (size_t)kLayers * kGroups * 3 * 64 * 4;   // u32
  std::vector<unsigned> hw(nW);
  for (size_t i = 0; i < nW; ++i) hw[i] = 0x3c003c00u + (unsigned)(i * 2654435761u % 4096);
  unsigned* W; float* out; unsigned long long* cyc;
  (void)hipMalloc(&W, nW * 4); (void)hipMalloc(&out, 256 * 64 * NWAVES * 4); (void)hipMalloc(&cyc, 256 * NWAVES * 8);
  (void)hipMemcpy(W, hw.data(), nW * 4, hipMemcpyHostToDevice);
  std::vector<unsigned long long> hc(256 * NWAVES);
  for (int rep = 0; rep < 4; ++rep) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(64 * NWAVES), 0, 0, W, out, cyc);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(hc.data(), cyc, 256 * NWAVES * 8, hipMemcpyDeviceToHost);
    double m = 0, mx = 0; for (auto c : hc) { m += c; mx = c > mx ? c : mx; } m /= hc.size();
    const double groups = (double)kTiles * kLayers * kGroups;
    if (rep == 3)
      printf("NS=%d NPF=%d NFILL=%d NWAVES=%d: %.1f cycles/group mean (%.1f max), ideal %d; %.3f ms; %.1f f32-equiv TFLOP/s\n", NS, NPF, NFILL, NWAVES,
             m / groups, mx / groups, 6 * NS * 32 * NWAVES / 4, ms,
             256.0 * NWAVES * NS * groups * 2 * 32 * 32 * 16 / (ms * 1e-3) / 1e12);
  }
  return 0;
}
