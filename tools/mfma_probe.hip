// Calibration probe: the MFMA rate one CU sustains with nothing but back-to-back
// v_mfma_f32_16x16x32_f16 (16 independent accumulators per wave, operands in registers, random
// fp16 values), 256 / 512 / 1024 workgroups of 4 or 8 waves, no LDS, no memory in the loop.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma_loop(const f16x8* seed, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8 a = seed[lane], b = seed[64 + lane];
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  std::vector<_Float16> h(128 * 8);
  srand(1);
  for (auto& x : h) x = (_Float16)((rand() % 2001 - 1000) / 1000.0f);
  f16x8* seed;
  float* out;
  hipMalloc(&seed, h.size() * 2);
  hipMemcpy(seed, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMalloc(&out, 1024 * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int threads : {256, 512}) {
    for (int grid : {256, 512, 1024}) {
      mfma_loop<16><<<grid, threads>>>(seed, out, 100);
      hipDeviceSynchronize();
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        mfma_loop<16><<<grid, threads>>>(seed, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double flops = 2.0 * 16 * 16 * 32 * 16.0 * iters * (threads / 64) * grid;
      printf("{\"threads\": %d, \"grid\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", threads, grid, best, flops / best / 1e9);
    }
  }
  return 0;
}
