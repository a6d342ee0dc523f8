// EXPERIMENT (round 4, not built into libclm): the ping-pong main loop below, measured against the
// shipped gemm_kernel / G2 configs on the encoder shapes (tools/pp_probe.py; bit-identical outputs
// on every shape and epilogue; profiles/r04_v1_pp_probe.jsonl, r04_v1_pp_variants.jsonl):
//   v_fc1 main loop 65.8 us (256 x 128 PP) vs 57.5-59.9 (G2 256 x 128, lockstep); full 82.9 vs 75.2.
//   Timing-only builds of the PP loop: no operand DMA 47.4 us, no fragment reads 47.3, neither 37.7
//   (1.60 PF/s: the staggered MFMA segments themselves are fast), DMA issued between the MFMAs of
//   the computing wave 94.5. The memory segment (16 ds_read_b128 + 6 LDS-DMA pieces per wave) takes
//   ~2x the 512-cycle MFMA segment it must hide behind: the per-CU LDS-DMA fill (~24 KB per interval
//   at ~40-55 B/clk) and the fragment reads share the segment. To build it with -DPP_* timing
//   variants: see git history of tools/experiments and tools/ppv.sh.
// PP ("ping-pong") MFMA GEMM for gfx950 (configs 12-16 of clm_gemm): the encoder's dense
// GEMMs (TF/models/clip/modeling_clip.py:294-297, 332, 343-344) with the same operand layout,
// epilogues and persistent tile order as gemm_kernel (k_gemm.hip); the main loop differs.
//
// Why: in gemm_kernel / G2 all 8 waves of a workgroup run in lockstep (one barrier per K-step),
// so every SIMD alternates between an LDS-read burst (both of its waves waiting on fragments)
// and an MFMA burst (both waves competing for the one matrix pipe), and the 16x16x32 MFMA leaves
// only 8 of its 16 cycles for other instructions of the SIMD (MI355X_MICROARCH.md, cycle
// constants). Here the two waves that share a SIMD (waves w and w + 4: a workgroup's waves are
// dealt cyclically over the 4 SIMDs) are staggered by one barrier interval:
//
//   interval t:    group 0 (waves 0-3)            group 1 (waves 4-7)
//   2s             M(s): frags of stage s,         C(s-1): MFMAs of stage s-1
//                  DMA of stage s+2
//   2s+1           C(s): MFMAs of stage s          M(s): frags of stage s, DMA of stage s+2
//
// so in every interval one wave per SIMD issues nothing but MFMAs (at s_setprio 1) while its
// partner reads LDS fragments, issues the LDS-DMA of a later stage and waits on its counters.
// Group g computes rows [g * BM/2, (g+1) * BM/2) of the tile (the waves form a (WM) x (WN) grid
// over the tile, WM even, rows of group 1 below those of group 0).
//
// LDS ring: 3 stages of (BM + BN) x 64 (A rows, then W rows; 128-byte rows, XOR chunk swizzle on
// the source address so the image is lane-linear for the DMA and ds_read_b128 is conflict-free).
// Hazards (t = barrier interval):
//  * RAW: stage s+1 is read from t = 2s+2 on; each wave waits for its own pieces of stage s+1
//    (counted vmcnt) at the end of its M(s) segment, i.e. before the barrier that ends t = 2s+1
//    at the latest, so every piece has landed and a barrier has passed before the first read;
//  * WAR: stage s+2 goes into the buffer of stage s-1, whose last reader (group 1, t = 2s-1)
//    retired its reads (lgkmcnt(0)) before the barrier that ends t = 2s-1; the first DMA into it
//    (group 0) is issued at t = 2s.
// The persistent ring crosses tile boundaries: a tile's epilogue runs in the wave's first M
// segment of the next tile (after that segment's DMA, so the stores stay in flight under the
// counted waits), i.e. while the partner wave computes.
#include <algorithm>

#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void sbar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(512, 2) void gemm3_kernel(GemmArgs ga) {
  constexpr int ST = 3;
  using C = Cfg<BM, BN, WM, WN, ST>;
  static_assert(C::NW == 8 && WM % 2 == 0, "8 waves, rows split between the two wave groups");
  static_assert(C::LDS <= 160 * 1024, "3-stage ring must fit the CU's LDS");
  constexpr int LA = BM / 64, LB = BN / 64;   // DMA pieces (8 rows x 128 B) per wave per stage
  static_assert(BM % 64 == 0 && BN % 64 == 0, "pieces split evenly over 8 waves");
  constexpr int L = LA + LB;
  constexpr int TM = C::TM, TN = C::TN;
  GemmArgs g = ga;
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntn * ntm, G = gridDim.x;
  const TileWalk tw = tile_walk(ntiles, G);
  if (tw.count <= 0) return;   // the whole workgroup leaves together: no barrier is left waiting
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

  // loader (as G2): SGPR descriptors from the tile's first row whose record count ends at the
  // matrix's last row (rows past M / N read as zeros), one VGPR offset per piece, K in SOFFSET
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
  auto dma_next = [&](int buf) {
    uint8_t* base = smem + buf * C::STAGE_BYTES;
    const int so = __builtin_amdgcn_readfirstlane(ld_kt * BK * 2);
#pragma unroll
    for (int j = 0; j < LA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(base + (wid * LA + j) * 1024), 16,
                                               (la0 + (uint32_t)((wid * LA + j) & 1) * dch) + (uint32_t)((wid * LA + j) * 8) * lda2,
                                               so, 0, 0);
#pragma unroll
    for (int j = 0; j < LB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(base + BM * 128 + (wid * LB + j) * 1024), 16,
                                               (lw0 + (uint32_t)((wid * LB + j) & 1) * dch) + (uint32_t)((wid * LB + j) * 8) * ldw2,
                                               so, 0, 0);
    if (++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };

#ifdef PP_DMA_IN_C
  // timing experiment: piece q of the 2L pieces per stage a group-0 wave issues (the 8L pieces of
  // a stage over waves 0-3); the loader advances after the last one
  auto dma_piece2 = [&](int buf, int q) {
    uint8_t* base = smem + buf * C::STAGE_BYTES;
    const int so = __builtin_amdgcn_readfirstlane(ld_kt * BK * 2);
    const int p = wid * 2 * L + q;
    if (p < BM / 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(base + p * 1024), 16,
                                               (la0 + (uint32_t)(p & 1) * dch) + (uint32_t)(p * 8) * lda2, so, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(base + p * 1024), 16,
                                               (lw0 + (uint32_t)(p & 1) * dch) + (uint32_t)((p - BM / 8) * 8) * ldw2, so, 0, 0);
    if (q == 2 * L - 1 && ++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };
#endif
  u32x4 af[2][TM], bw[2][TN];
  auto read_frags = [&](const uint8_t* sa) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int mb = 0; mb < TM; ++mb) {
        const int row = wm * (BM / WM) + mb * 16 + (lane & 15);
        af[kk][mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) {
        const int row = wn * (BN / WN) + nb * 16 + (lane & 15);
        bw[kk][nb] = *(const u32x4*)(sa + BM * 128 + row * 128 + swz(row, c) * 16);
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
  zero();

  // prologue: stages 0 and 1 in flight, stage 0 landed everywhere
  dma_next(0);
  if (S > 1) dma_next(1);
  if (S > 1) wait_vmcnt<L>();
  else wait_vmcnt<0>();
  lds_barrier();
  if (grp) sbar();   // group 1 runs one interval behind

  constexpr int E0 = epi_min_stores<EPI, TM, TN>();
  constexpr int E = E0 + L > 63 ? 63 - L : E0;
  const bool vec_epi = (g.N % 4) == 0 && (g.ldo % 4) == 0 && !(g.debug & 1);
  int pm0 = 0, pn0 = 0;   // previous tile (epilogue pending)
  int s = 0;
  bool epi_prev = false;   // an epilogue ran in the previous M segment
  for (int ti = 0; ti < n_my; ++ti) {
    int m0, n0;
    coords(ti, m0, n0);
    for (int kt = 0; kt < nk; ++kt, ++s) {
      // ---- M segment
#if defined(PP_NO_DMA)
      const bool dma = false;
#elif defined(PP_DMA_IN_C)
      const bool dma = false;
#else
      const bool dma = s + 2 < S;
      if (dma) dma_next((s + 2) % ST);
#endif
#ifndef PP_NO_READS
      read_frags(smem + (s % ST) * C::STAGE_BYTES);
#endif
      bool epi_now = false;
      if (kt == 0 && ti > 0) {
        if (g.debug & 1) {
#pragma unroll
          for (int mb = 0; mb < TM; ++mb)
#pragma unroll
            for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
        } else {
          epilogue<BF, EPI, BM, BN, WM, WN, ST>(g, acc, pm0, pn0, wm, wn, lane);
          epi_now = vec_epi;
        }
        zero();
      }
      // own pieces of stage s+1 landed; younger: DMA(s+2) and this / the previous segment's stores
      if (s + 1 < S) {
        const bool st = epi_now || epi_prev;
        if (dma) {
          if (st) wait_vmcnt<L + E>();
          else wait_vmcnt<L>();
        } else {
          if (st) wait_vmcnt<E>();
          else wait_vmcnt<0>();
        }
      }
      epi_prev = epi_now;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sbar();
      // ---- C segment
      __builtin_amdgcn_s_setprio(1);
#ifdef PP_DMA_IN_C
      // timing experiment: group 0 issues all of stage s+2's pieces between its MFMAs
      {
        const bool d2 = grp == 0 && s + 2 < S;
        int q = 0;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int mb = 0; mb < TM; ++mb)
#pragma unroll
            for (int nb = 0; nb < TN; ++nb) {
              acc[mb][nb] = mfma16<BF>(bw[kk][nb], af[kk][mb], acc[mb][nb]);
              if (d2 && ((kk * TM + mb) * TN + nb) % 3 == 1 && q < 2 * L) {
                __builtin_amdgcn_sched_barrier(0);
                dma_piece2((s + 2) % ST, q++);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
        if (d2) { while (q < 2 * L) dma_piece2((s + 2) % ST, q++); }
        if (grp == 0 && s + 1 < S) {
          if (d2) wait_vmcnt<2 * L>();
          else wait_vmcnt<0>();
        }
      }
#else
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int mb = 0; mb < TM; ++mb)
#pragma unroll
          for (int nb = 0; nb < TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[kk][nb], af[kk][mb], acc[mb][nb]);
#endif
      __builtin_amdgcn_s_setprio(0);
      sbar();
    }
    pm0 = m0;
    pn0 = n0;
  }
  if (g.debug & 1) {
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
  } else {
    epilogue<BF, EPI, BM, BN, WM, WN, ST>(g, acc, pm0, pn0, wm, wn, lane);
  }
  if (!grp) sbar();   // balance group 1's leading barrier
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN>
hipError_t launch_cfg3(const GemmArgs& g, hipStream_t s) {
  using C = Cfg<BM, BN, WM, WN, 3>;
  auto kern = gemm3_kernel<BF, EPI, BM, BN, WM, WN>;
  static unsigned dev_done = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  static int cus_of[32] = {};
  int& cus = cus_of[dev & 31];
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
  }
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM);
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, cus);   // one workgroup per CU
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}

template <bool BF, int EPI>
hipError_t by_id3(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 12: return launch_cfg3<BF, EPI, 256, 128, 4, 2>(g, s);
    case 13: return launch_cfg3<BF, EPI, 128, 256, 2, 4>(g, s);
    case 14: return launch_cfg3<BF, EPI, 192, 128, 4, 2>(g, s);
    case 15: return launch_cfg3<BF, EPI, 128, 192, 2, 4>(g, s);
    case 16: return launch_cfg3<BF, EPI, 128, 128, 4, 2>(g, s);
    default: return hipErrorInvalidValue;
  }
}
template <bool BF>
hipError_t by_epi3(int epi, int id, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return by_id3<BF, EPI_STORE>(id, g, s);
    case EPI_GELU: return by_id3<BF, EPI_GELU>(id, g, s);
    case EPI_RESID: return by_id3<BF, EPI_RESID>(id, g, s);
    case EPI_PATCH: return by_id3<BF, EPI_PATCH>(id, g, s);
    case EPI_SCORE: return by_id3<BF, EPI_SCORE>(id, g, s);
    case EPI_FILTER: return by_id3<BF, EPI_FILTER>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t gemm3_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s) {
  return bf16 ? by_epi3<true>(epi, id, g, s) : by_epi3<false>(epi, id, g, s);
}
}  // namespace clm
