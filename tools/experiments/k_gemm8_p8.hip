// EXPERIMENT (round 4, not built into libclm): the 256 x 256 "8-phase" structure of
// cdna_hip_programming.md §5 (four quadrant phases per K-tile, row groups staggered by one barrier,
// s_setprio 1 MFMA segments). Bit-identical to config 1 on every shape (integer and random data),
// no faster (tools/pp_probe.py, profiles/r04_v6_p8_probe.jsonl; main loop / full, us): 8192^3
// 845.8 / 881.0 vs config 1 858.1 / 885.6 (hipBLASLt 716.5); v_qkv 46.6 / 59.3 vs 42.8 / 55.3;
// L/14 fc1 518.8 / 697.5 vs 491.8 / 637.7; the configs[4] search 56.2 k QPS vs 70.5 k.
// P8 MFMA GEMM for gfx950 (config 12 of clm_gemm): 256 x 256 tiles, 8 waves (2 row groups x 4
// column waves, 128 x 64 per wave), one K-tile of 64 in four phases -- one 64 x 32 quadrant of
// the wave tile each -- with the two waves of a SIMD (waves w and w + 4: the row groups) offset
// by one barrier interval. Same operand layout, epilogues and persistent tile order as
// gemm_kernel (k_gemm.hip), and the same per-element MFMA order (16x16x32 over K in order), so
// the results are bit-identical to every other config.
//
// A phase, per wave:  M: LDS-DMA pieces of the next K-tile + the ds_reads of this quadrant's
// register subtile  | barrier |  C: 16 MFMAs at s_setprio 1  | barrier.
// Group 1 runs one interval behind group 0, so in every interval one wave per SIMD issues only
// MFMAs while its partner reads LDS and issues DMA (cdna_hip_programming.md §5, the 256^2
// 8-phase template). Quadrant order (0,0) (0,1) (1,1) (1,0): the loads before each phase are the
// A-subtile (8 ds_read_b128) and / or the B-subtile (4) that change.
//
// LDS: two K-tile buffers of 256 A rows + 256 B rows x 128 B (128 KiB), XOR chunk swizzle on the
// DMA source. DMA of K-tile s+1 (8 pieces per wave) goes out in the M parts of phases 1-3 of
// K-tile s into the buffer of K-tile s-1, whose last reader (group 1, phase 4 of s-1) retired its
// reads before the barrier that ends that interval; every wave waits for its own pieces at the end
// of its phase-4 M part, two or more intervals after issuing them and before the barrier that
// precedes the first read of K-tile s+1.
#include <algorithm>

#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void sbar8() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool BF, int EPI>
__global__ __launch_bounds__(512, 2) void gemm8_kernel(GemmArgs ga) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  using C = Cfg<BM, BN, WM, WN, 2>;   // TM = 8, TN = 4, STAGE_BYTES = 64 KiB
  constexpr int TM = C::TM, TN = C::TN;
  GemmArgs g = ga;
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;             // row group: SIMD partners w, w + 4 are in different groups
  const int wm = grp, wn = wid & 3;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntn * ntm, G = gridDim.x;
  const TileWalk tw = tile_walk(ntiles, G);
  if (tw.count <= 0) return;            // the whole workgroup leaves together
  const int n_my = tw.count;
  const int nk = g.K / BK;
  const int S = n_my * nk;

  auto coords = [&](int i, int& m0, int& n0) {
    const int t = tw.first + i * tw.stride;
    int tm, tn;
    if (g.m_fastest) {
      tm = t % ntm;
      tn = t / ntm;
    } else {
      const int group = t / (GM * ntn);
      const int first_m = group * GM;
      const int gsz = min(GM, ntm - first_m);
      const int r = t - group * GM * ntn;
      tm = first_m + r % gsz;
      tn = r / gsz;
    }
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // loader (as G2): 8 pieces of 8 rows x 128 B per wave and K-tile: A rows wid*32 + j*8, j < 4,
  // then B rows wid*32 + (j-4)*8
  const int r8 = lane >> 3, pc = lane & 7;
  const uint32_t lda2 = (uint32_t)g.lda * 2, ldw2 = (uint32_t)g.ldw * 2;
  const uint32_t ch0 = (uint32_t)((pc ^ ((r8 >> 1) & 7)) << 4);
  const uint32_t ch1 = (uint32_t)((pc ^ ((4 + (r8 >> 1)) & 7)) << 4);
  const uint32_t la0 = r8 * lda2 + ch0, lw0 = r8 * ldw2 + ch0, dch = ch1 - ch0;
  __amdgpu_buffer_rsrc_t ra, rw;
  int ld_i = 0, ld_kt = 0;
  auto point = [&](int i) {
    int m0, n0;
    coords(i, m0, n0);
    ra = buf_rsrc(g.A + (int64_t)m0 * g.lda, min(BM, g.M - m0) * (int)lda2);
    rw = buf_rsrc(g.W + (int64_t)n0 * g.ldw, min(BN, g.N - n0) * (int)ldw2);
  };
  point(0);
  auto piece = [&](int buf, int j) {   // j compile-time after unrolling
    uint8_t* base = smem + buf * C::STAGE_BYTES;
    const int so = __builtin_amdgcn_readfirstlane(ld_kt * BK * 2);
    const int p = wid * 4 + (j & 3);   // piece index inside its operand (0..31), 8 rows each
    if (j < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(base + p * 1024), 16,
                                               (la0 + (uint32_t)(p & 1) * dch) + (uint32_t)(p * 8) * lda2, so, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(base + BM * 128 + p * 1024), 16,
                                               (lw0 + (uint32_t)(p & 1) * dch) + (uint32_t)(p * 8) * ldw2, so, 0, 0);
  };
  auto advance = [&]() {
    if (++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };

  u32x4 asub[2][4], bsub[2][2];
  auto read_a = [&](const uint8_t* sa, int qr) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int row = wm * 128 + qr * 64 + mb * 16 + (lane & 15);
        asub[kk][mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
    }
  };
  auto read_b = [&](const uint8_t* sa, int qc) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int row = wn * 64 + qc * 32 + nb * 16 + (lane & 15);
        bsub[kk][nb] = *(const u32x4*)(sa + BM * 128 + row * 128 + swz(row, c) * 16);
      }
    }
  };
  f32x4 acc[TM][TN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto quad = [&](int qr, int qc) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[qr * 4 + mb][qc * 2 + nb] = mfma16<BF>(bsub[kk][nb], asub[kk][mb], acc[qr * 4 + mb][qc * 2 + nb]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto keep_live = [&]() {
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
  };
  zero();

  // prologue: K-tile 0 landed everywhere
#pragma unroll
  for (int j = 0; j < 8; ++j) piece(0, j);
  advance();
  wait_vmcnt<0>();
  lds_barrier();
  if (grp) sbar8();   // group 1 runs one interval behind

  int pm0 = 0, pn0 = 0;
  int s = 0;
  for (int ti = 0; ti < n_my; ++ti) {
    int m0, n0;
    coords(ti, m0, n0);
    for (int kt = 0; kt < nk; ++kt, ++s) {
      const uint8_t* sa = smem + (s & 1) * C::STAGE_BYTES;
      const int nb_ = (s + 1) & 1;
      const bool dma = s + 1 < S;
      // ---- phase 1: quadrant (0, 0); DMA pieces 0-2 of K-tile s+1; a finished tile's epilogue
      if (dma) { piece(nb_, 0); piece(nb_, 1); piece(nb_, 2); }
      if (kt == 0 && ti > 0) {
        if (g.debug & 1) keep_live();
        else epilogue<BF, EPI, BM, BN, WM, WN, 2>(g, acc, pm0, pn0, wm, wn, lane);
        zero();
      }
      read_a(sa, 0);
      read_b(sa, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sbar8();
      quad(0, 0);
      sbar8();
      // ---- phase 2: quadrant (0, 1); DMA pieces 3-5
      if (dma) { piece(nb_, 3); piece(nb_, 4); piece(nb_, 5); }
      read_b(sa, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sbar8();
      quad(0, 1);
      sbar8();
      // ---- phase 3: quadrant (1, 1); DMA pieces 6-7
      if (dma) { piece(nb_, 6); piece(nb_, 7); advance(); }
      read_a(sa, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sbar8();
      quad(1, 1);
      sbar8();
      // ---- phase 4: quadrant (1, 0); own pieces of K-tile s+1 landed before the barrier
      read_b(sa, 0);
      wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sbar8();
      quad(1, 0);
      sbar8();
    }
    pm0 = m0;
    pn0 = n0;
  }
  if (g.debug & 1) keep_live();
  else epilogue<BF, EPI, BM, BN, WM, WN, 2>(g, acc, pm0, pn0, wm, wn, lane);
  if (!grp) sbar8();   // balance group 1's leading barrier
}

template <bool BF, int EPI>
hipError_t launch8(const GemmArgs& g, hipStream_t s) {
  constexpr int LDS = 2 * (256 + 256) * BK * 2;
  auto kern = gemm8_kernel<BF, EPI>;
  static unsigned dev_done = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  static int cus_of[32] = {};
  int& cus = cus_of[dev & 31];
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
  }
  const int tiles = ((g.N + 255) / 256) * ((g.M + 255) / 256);
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, cus);
  kern<<<dim3(nwg), dim3(512), LDS, s>>>(g);
  return hipGetLastError();
}

template <bool BF>
hipError_t by_epi8(int epi, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return launch8<BF, EPI_STORE>(g, s);
    case EPI_GELU: return launch8<BF, EPI_GELU>(g, s);
    case EPI_RESID: return launch8<BF, EPI_RESID>(g, s);
    case EPI_PATCH: return launch8<BF, EPI_PATCH>(g, s);
    case EPI_SCORE: return launch8<BF, EPI_SCORE>(g, s);
    case EPI_FILTER: return launch8<BF, EPI_FILTER>(g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t gemm8_launch(bool bf16, int epi, const GemmArgs& g, hipStream_t s) {
  return bf16 ? by_epi8<true>(epi, g, s) : by_epi8<false>(epi, g, s);
}
}  // namespace clm
