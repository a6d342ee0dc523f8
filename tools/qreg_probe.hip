// Main-loop probe for the search filter GEMM's next form (DESIGN.md "Open after round 5"): each
// wave keeps its 64 queries x 512 dims of fp16 in registers for the whole launch and only the
// index rows stream through LDS (BN rows per tile, double-buffered LDS-DMA, XOR-swizzled chunks),
// so a tile costs BN KiB of LDS fill plus 4 x BN KiB of fragment reads per workgroup against
// 64 x BN x 512 x 2 x 4 FLOP. The "epilogue" is a running per-query maximum (what a threshold
// compare costs), stored per lane so the host can check it. Not product code: the timing answers
// whether this form beats G2's 256 x 192 loop (filter GEMM ~0.49 MFMA busy).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/qreg_probe tools/qreg_probe.hip
// Run:   tools/qreg_probe [rows]  -> JSON lines (check, then timing)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 512;           // dims (halves per row)
constexpr int QW = 64;           // queries per wave
constexpr int NW = 4;            // waves per workgroup (one per SIMD)
constexpr int QG = QW * NW;      // queries per workgroup
constexpr int KS = D / 32;       // 16 k-steps of the 16x16x32 MFMA

// LDS position of chunk c (16 B) of tile row r: chunks XOR-swizzled by r & 15 so the 16 rows a
// fragment read touches at one chunk land on 16 distinct 16-B slots
__device__ __forceinline__ int pos(int r, int c) { return c ^ (r & 15); }

template <int BN>
__global__ __launch_bounds__(NW * 64, 1) void qreg_kernel(const _Float16* Q, const _Float16* X, int64_t N, int nqg,
                                                          int nrange, float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BN * 1024];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the nqg query groups of one row range run on one XCD (blockIdx % 8), so each index tile comes
  // from HBM once per XCD and the other groups read it from L2
  const int b = blockIdx.x;
  const int xcd = b % 8, j = b / 8;
  const int qg = j % nqg, nr = xcd + 8 * (j / nqg);
  if (nr >= nrange) return;
  const int64_t per = ((N + nrange - 1) / nrange + BN - 1) / BN * BN;
  const int64_t r0 = (int64_t)nr * per, r1 = std::min<int64_t>(N, r0 + per);
  const int ntile = r1 > r0 ? (int)((r1 - r0 + BN - 1) / BN) : 0;

  // this wave's queries: A-fragments a[mb][ks] = query q0 + 16 mb + (lane & 15), dims 32 ks + 8 (lane >> 4) ..
  const int q0 = qg * QG + wid * QW;
  f16x8 a[4][KS];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      a[mb][ks] = *(const f16x8*)(Q + (int64_t)(q0 + mb * 16 + (lane & 15)) * D + ks * 32 + 8 * (lane >> 4));

  // DMA: wave w fills tile rows w * BN / NW ..; lane L of a row's instruction writes LDS chunk L,
  // which holds the row's chunk L ^ (row & 15)
  constexpr int RPW = BN / NW;
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wid * RPW + i;
      const int64_t row = std::min<int64_t>(r0 + (int64_t)t * BN + r, N - 1);
      __builtin_amdgcn_global_load_lds((const void*)(X + row * D + pos(r, lane) * 8),
                                       (void*)(smem + buf * BN * 1024 + r * 1024), 16, 0, 0);
    }
  };
  float rm[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if (ntile > 0) issue(0, 0);
  for (int t = 0; t < ntile; ++t) {
    const int buf = t & 1;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 1 < ntile) issue(t + 1, buf ^ 1);
    const uint8_t* tb = smem + buf * BN * 1024;
    const int rows_left = (int)std::min<int64_t>(BN, r1 - r0 - (int64_t)t * BN);
    // index fragments two 16-row blocks deep: block nb + 1's reads are issued between block nb's
    // MFMAs (the MFMA statements clobber memory so the reads stay where they are placed)
    f16x8 bfr[2][KS];
    auto rd = [&](int nb, int ks) {
      const int r = nb * 16 + (lane & 15);
      bfr[nb & 1][ks] = *(const f16x8*)(tb + r * 1024 + pos(r, ks * 4 + (lane >> 4)) * 16);
    };
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) rd(0, ks);
#pragma unroll
    for (int nb = 0; nb < BN / 16; ++nb) {
      f32x4 acc[4];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          // the query fragments are AGPR operands (all 256 of them stay in the accumulator file),
          // leaving the VGPRs to the index fragments in flight; the first k-step starts from C = 0
          if (ks == 0)
            asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0"
                         : "=v"(acc[mb])
                         : "v"(bfr[nb & 1][ks]), "a"(a[mb][ks])
                         : "memory");
          else
            asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0"
                         : "+v"(acc[mb])
                         : "v"(bfr[nb & 1][ks]), "a"(a[mb][ks])
                         : "memory");
        }
        if (nb + 1 < BN / 16) {
          rd(nb + 1, ks);
          // keep block nb's fragment live past the read of block nb + 1's: the two never share
          // registers, so no LDS return overwrites an operand of an in-flight MFMA
          asm volatile("" ::"v"(bfr[nb & 1][ks]));
        }
      }
      // the MFMA results' read hazard (inline asm: the compiler inserts no wait states)
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])::"memory");
      // C[i = tile row nb*16 + 4 (lane >> 4) + e][j = query lane & 15]
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (nb * 16 + 4 * (lane >> 4) + e < rows_left) rm[mb] = fmaxf(rm[mb], acc[mb][e]);
    }
  }
  // out[b][wid][mb][lane]
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) out[(((int64_t)b * NW + wid) * 4 + mb) * 64 + lane] = rm[mb];
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 4000000;
  const int nq = 2560, nqg = nq / QG;   // 10 query groups
  constexpr int BN = 64;
  int ncu = 256;
  const int nrange = 24;                // 10 x 24 = 240 workgroups, one per CU
  const int nwg = 8 * nqg * ((nrange + 7) / 8);
  (void)ncu;
  std::vector<_Float16> hq((size_t)nq * D);
  srand(1);
  for (auto& v : hq) v = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.09f);
  _Float16 *dq, *dx;
  float* dout;
  CHK(hipMalloc(&dq, hq.size() * 2));
  CHK(hipMalloc(&dx, (size_t)N * D * 2));
  CHK(hipMalloc(&dout, (size_t)nwg * NW * 4 * 64 * 4));
  CHK(hipMemcpy(dq, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  // index rows: a deterministic pattern generated on the host in chunks
  {
    const int64_t CH = 1 << 20;
    std::vector<_Float16> hx((size_t)CH * D);
    for (int64_t r0 = 0; r0 < N; r0 += CH) {
      const int64_t n = std::min(CH, N - r0);
      for (int64_t i = 0; i < n * D; ++i) {
        const uint32_t h = (uint32_t)((r0 * D + i) * 2654435761u);
        hx[i] = (_Float16)(((h >> 8) / 16777216.0f - 0.5f) * 0.09f);
      }
      CHK(hipMemcpy(dx + r0 * D, hx.data(), (size_t)n * D * 2, hipMemcpyHostToDevice));
    }
  }
  auto run = [&]() {
    qreg_kernel<BN><<<nwg, NW * 64, 0, 0>>>(dq, dx, N, nqg, nrange, dout);
    CHK(hipGetLastError());
  };
  run();
  CHK(hipDeviceSynchronize());
  // check: the max over rows of a few queries against the host (fp32 sums of fp16 products)
  std::vector<float> hout((size_t)nwg * NW * 4 * 64);
  CHK(hipMemcpy(hout.data(), dout, hout.size() * 4, hipMemcpyDeviceToHost));
  std::vector<float> gmax(nq, -INFINITY);
  for (int b = 0; b < nwg; ++b) {
    const int xcd = b % 8, j = b / 8, qg = j % nqg, nr = xcd + 8 * (j / nqg);
    if (nr >= nrange) continue;
    for (int w = 0; w < NW; ++w)
      for (int mb = 0; mb < 4; ++mb)
        for (int l = 0; l < 64; ++l) {
          const int q = qg * QG + w * QW + mb * 16 + (l & 15);
          gmax[q] = std::max(gmax[q], hout[(((size_t)b * NW + w) * 4 + mb) * 64 + l]);
        }
  }
  const int64_t NC = std::min<int64_t>(N, 200000);
  double worst = 0;
  if (NC == N) {
    std::vector<_Float16> hx((size_t)N * D);
    CHK(hipMemcpy(hx.data(), dx, hx.size() * 2, hipMemcpyDeviceToHost));
    for (int q : {0, 1, 17, 255, 256, 1000, 2559}) {
      float best = -INFINITY;
      for (int64_t r = 0; r < N; ++r) {
        float s = 0.f;
        for (int k = 0; k < D; ++k) s += (float)hq[(size_t)q * D + k] * (float)hx[(size_t)r * D + k];
        best = std::max(best, s);
      }
      worst = std::max(worst, (double)fabsf(best - gmax[q]));
    }
    printf("{\"check_rows\": %lld, \"max_abs_diff\": %.3e}\n", (long long)N, worst);
  }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) run();
  const int reps = 10;
  CHK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) run();
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double flop = 2.0 * nq * (double)N * D;
  printf("{\"rows\": %lld, \"queries\": %d, \"BN\": %d, \"workgroups\": %d, \"ms\": %.3f, \"tflops\": %.1f, "
         "\"index_gbs\": %.0f}\n",
         (long long)N, nq, BN, nwg, ms, flop / ms / 1e9, (double)N * D * 2 / ms / 1e6);
  return 0;
}
