// Which SIMD does each wave of a workgroup run on?  Reads HW_ID (SIMD_ID bits 5:4, CU_ID 11:8) for every wave of
// 512- and 256-thread workgroups; prints the wave -> SIMD map of the first workgroups.  Build:
//   hipcc -O2 --offload-arch=gfx950 tools/micro/wave_simd.hip -o tools/micro/wave_simd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(unsigned* out) {
  if ((threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
    out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = hw;
  }
}

int main() {
  for (int threads : {512, 256}) {
    const int blocks = 512, waves = threads / 64;
    unsigned* d;
    hipMalloc(&d, blocks * waves * 4);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, d);
    std::vector<unsigned> h(blocks * waves);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int same_rr = 0;
    for (int b = 0; b < blocks; ++b) {
      bool rr = true;
      for (int w = 0; w < waves; ++w) rr &= (((h[b * waves + w] >> 4) & 3) == (unsigned)((((h[b * waves] >> 4) & 3) + w) & 3));
      same_rr += rr;
    }
    printf("%d threads: %d of %d workgroups map wave w to SIMD (simd0 + w) mod 4\n", threads, same_rr, blocks);
    for (int b = 0; b < 4; ++b) {
      printf("  wg %d:", b);
      for (int w = 0; w < waves; ++w) printf(" w%d->simd%u(cu%u)", w, (h[b * waves + w] >> 4) & 3, (h[b * waves + w] >> 8) & 15);
      printf("\n");
    }
    hipFree(d);
  }
  return 0;
}
