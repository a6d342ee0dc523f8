// Per-CU LDS-DMA fill-rate probe (gfx950): how fast can one workgroup per CU stream operand tiles
// from global memory into an LDS ring with global_load_lds_dwordx4 -- the GEMM main loops' operand
// path -- as a function of the bytes kept in flight and of where the source lives (an L2-sized
// panel re-read by every workgroup of an XCD, or a large buffer streamed from HBM).
// No MFMA work: an upper bound for the fill side of the main loop.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/fill_probe tools/fill_probe.hip
// Run:   tools/fill_probe  -> one JSON line per (source, stage bytes, stages in flight, waves)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Each workgroup moves `steps` stages of STAGE_KB KiB into a ring of NS stages, keeping IN_FLIGHT
// stages outstanding (counted vmcnt, raw barrier as in the GEMM ring). Source offset of stage s
// cycles through `span` bytes starting at a per-workgroup base (span small: L2-resident re-reads;
// span large: HBM streaming).
template <int NW, int STAGE_KB, int NS, int IN_FLIGHT>
__global__ __launch_bounds__(NW * 64, 1) void fill_kernel(const uint8_t* src, size_t span, size_t wg_stride, int steps,
                                                          unsigned long long* sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PIECES = STAGE_KB / NW;   // 1 KiB wave-instructions per wave per stage
  static_assert(PIECES >= 1 && IN_FLIGHT < NS, "geometry");
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint8_t* base = src + (size_t)blockIdx.x * wg_stride;
  auto issue = [&](int s) {
    const size_t off = ((size_t)s * STAGE_KB * 1024) % span;
    uint8_t* dst = smem + (s % NS) * STAGE_KB * 1024;
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const int piece = wid * PIECES + j;
      __builtin_amdgcn_global_load_lds((const void*)(base + off + piece * 1024 + lane * 16),
                                       (void*)(dst + piece * 1024), 16, 0, 0);
    }
  };
  for (int s = 0; s < IN_FLIGHT && s < steps; ++s) issue(s);
  unsigned acc = 0;
  for (int s = 0; s < steps; ++s) {
    if (s + IN_FLIGHT < steps) {
      issue(s + IN_FLIGHT);
      // stage s retired once only the IN_FLIGHT younger stages remain
      if constexpr (IN_FLIGHT == 1) wait_vmcnt<PIECES>();
      else if constexpr (IN_FLIGHT == 2) wait_vmcnt<2 * PIECES>();
      else wait_vmcnt<3 * PIECES>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    acc += smem[(s % NS) * STAGE_KB * 1024 + threadIdx.x * 4];   // touch the landed stage
  }
  if (acc == 0xFFFFFFFFu) sink[blockIdx.x] = acc;
}

template <int NW, int STAGE_KB, int NS, int IN_FLIGHT>
void run(const char* label, const uint8_t* buf, size_t span, size_t wg_stride, int cus, int steps) {
  auto k = fill_kernel<NW, STAGE_KB, NS, IN_FLIGHT>;
  const int lds = NS * STAGE_KB * 1024;
  CHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  unsigned long long* sink;
  CHK(hipMalloc(&sink, cus * 8));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  k<<<cus, NW * 64, lds>>>(buf, span, wg_stride, steps, sink);   // warm-up
  CHK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a));
    k<<<cus, NW * 64, lds>>>(buf, span, wg_stride, steps, sink);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  const double ms = ts[2];
  const double bytes_per_cu = (double)steps * STAGE_KB * 1024;
  printf("{\"source\": \"%s\", \"waves\": %d, \"stage_kb\": %d, \"in_flight\": %d, \"kb_in_flight\": %d, "
         "\"gbps_per_cu\": %.1f, \"tbps_chip\": %.2f}\n",
         label, NW, STAGE_KB, IN_FLIGHT, IN_FLIGHT * STAGE_KB, bytes_per_cu / ms / 1e6, bytes_per_cu * cus / ms / 1e9);
  fflush(stdout);
  CHK(hipFree(sink));
}

int main() {
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t big = (size_t)4 << 30;   // 4 GiB: far past the 256 MiB Infinity Cache
  uint8_t* buf;
  CHK(hipMalloc(&buf, big));
  CHK(hipMemset(buf, 1, big));
  const int steps = 400;
  // L2: every workgroup re-reads the same 1 MiB panel (one copy per XCD's L2)
  const size_t l2span = (size_t)1 << 20;
  // HBM: each workgroup streams its own 16 MiB slice once
  const size_t hspan = (size_t)16 << 20, hstride = hspan;
  run<8, 64, 2, 1>("L2 panel", buf, l2span, 0, cus, steps);
  run<8, 32, 4, 3>("L2 panel", buf, l2span, 0, cus, steps);
  run<8, 48, 3, 2>("L2 panel", buf, l2span, 0, cus, steps);
  run<4, 32, 4, 3>("L2 panel", buf, l2span, 0, cus, steps);
  // Infinity Cache: each workgroup re-reads its own 512 KiB slice (32 per XCD = 16 MiB > the 4 MiB
  // L2, 128 MiB in all < the 256 MiB Infinity Cache)
  const size_t mspan = (size_t)512 << 10;
  run<8, 64, 2, 1>("MALL slices", buf, mspan, mspan, cus, steps);
  run<8, 32, 4, 3>("MALL slices", buf, mspan, mspan, cus, steps);
  run<8, 48, 3, 2>("MALL slices", buf, mspan, mspan, cus, steps);
  run<8, 64, 2, 1>("HBM stream", buf, hspan, hstride, cus, 256);
  run<8, 32, 4, 3>("HBM stream", buf, hspan, hstride, cus, 256);
  run<8, 48, 3, 2>("HBM stream", buf, hspan, hstride, cus, 256);
  CHK(hipFree(buf));
  return 0;
}
