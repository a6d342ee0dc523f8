// G2 MFMA GEMM for gfx950 (configs 8-11 of clm_gemm): one wave per SIMD with large per-wave
// tiles, for the encoder's dense qkv / out / fc1 / fc2 GEMMs (TF/models/clip/modeling_clip.py:
// 294-297, 332, 343-344). Same operand layout, epilogues and persistent tile order as
// k_gemm.hip's gemm_kernel; the main loop differs (see below).
#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

// ---------------------------------------------------------------------------------------
// G2: one wave per SIMD, large per-wave tiles (4 waves, 2 x 2, each (BM/2) x (BN/2): 128 x 128
// at 256 x 256 = 256 fp32 accumulators per lane). Two-buffer LDS ring filled by
// buffer_load ... lds (one 32-bit VGPR offset per 8-row piece, the K advance in SOFFSET, the
// tile base in the SGPR descriptor). Per K-step s (buffer s&1, two 32-deep halves kk0/kk1):
//   read kk1 fragments of s | MFMAs kk0 of s (fragments prefetched in step s-1)
//   | wait DMA(s+1) + barrier | DMA(s+2) into buffer s&1 | read kk0 fragments of s+1
//   | MFMAs kk1 of s | tile end: epilogue.
// The LDS latency of every fragment read is covered by 64 MFMAs of the other half, the only
// MFMA-idle window per step is the barrier, and DMA(s+2) is issued before a tile end's
// epilogue stores, so the next wait never drains them (counted vmcnt).
template <int BM, int BN, int WM, int WN>
struct Cfg2 {
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int TM = BM / WM / 16;
  static constexpr int TN = BN / WN / 16;
  static constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  static constexpr int LDS = 2 * STAGE_BYTES;   // two-buffer ring: DMA lead of one K-step
  static constexpr int LA = BM / 8 / NW;
  static constexpr int LB = BN / 8 / NW;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "rows must split evenly over waves");
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <bool BF, int EPI, int BM, int BN, int WM, int WN>
__device__ __forceinline__ void gemm2_body(const GemmArgs& ga, int bid, int G) {
  using C = Cfg2<BM, BN, WM, WN>;
  GemmArgs g = ga;   // varlen: the device-resident row count (the grid was sized for ga.M)
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  constexpr int L = C::LA + C::LB;   // vmcnt units (DMA instructions) per K-step
  constexpr int TM = C::TM, TN = C::TN;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntn * ntm;
  const TileWalk tw = tile_walk(ntiles, bid, G);
  if (tw.count <= 0) return;   // varlen: fewer live tiles than the grid
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

  // loader: descriptors at the tile's first row whose record count ends at the matrix's last
  // row (rows past M / N read as zeros by the range check, which covers the VGPR offset);
  // per-lane byte offsets of a piece = lane part (16-B chunk XOR-swizzled on the source so the
  // LDS image is lane-linear; the swizzle depends only on the parity of the piece's 8-row index) + piece rows
  const int r8 = lane >> 3, pc = lane & 7;
  const uint32_t lda2 = (uint32_t)g.lda * 2, ldw2 = (uint32_t)g.ldw * 2;
  // (a runtime-indexed la[2] here made hipcc's host pass drop every kernel of this file from
  // the object's fatbin without an error: keep the parity select arithmetic)
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
    for (int j = 0; j < C::LA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(base + (wid * C::LA + j) * 1024), 16,
                                               (la0 + (uint32_t)((wid * C::LA + j) & 1) * dch) + (uint32_t)((wid * C::LA + j) * 8) * lda2,
                                               so, 0, 0);
#pragma unroll
    for (int j = 0; j < C::LB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(base + BM * 128 + (wid * C::LB + j) * 1024), 16,
                                               (lw0 + (uint32_t)((wid * C::LB + j) & 1) * dch) + (uint32_t)((wid * C::LB + j) * 8) * ldw2,
                                               so, 0, 0);
    if (++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };
  auto read_frags = [&](const uint8_t* sa, int kk, u32x4 (&af)[TM], u32x4 (&bw)[TN]) {
    const int c = kk * 4 + (lane >> 4);
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int row = wm * (BM / WM) + mb * 16 + (lane & 15);
      af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
    }
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      const int row = wn * (BN / WN) + nb * 16 + (lane & 15);
      bw[nb] = *(const u32x4*)(sa + BM * 128 + row * 128 + swz(row, c) * 16);
    }
  };
  f32x4 acc[TM][TN];
  auto mma = [&](const u32x4 (&af)[TM], const u32x4 (&bw)[TN]) {
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], acc[mb][nb]);
  };

  dma_next(0);
  if (S > 1) dma_next(1);
  if (S >= 2) wait_vmcnt<L>();   // DMA(0) retired, DMA(1) in flight
  else wait_vmcnt<0>();
  lds_barrier();
  u32x4 a0[TM], b0[TN], a1[TM], b1[TN];
  read_frags(smem, 0, a0, b0);

  constexpr int E0 = epi_min_stores<EPI, TM, TN>();
  constexpr int E = E0 > 63 ? 63 : E0;
  const bool vec_epi = (g.N % 4) == 0 && (g.ldo % 4) == 0 && !(g.debug & 1);
  int s = 0;     // K-step of the ring (all tiles of this workgroup)
  int cur = 0;   // its LDS buffer, s % 2
  for (int ti = 0; ti < n_my; ++ti) {
    int m0, n0;
    coords(ti, m0, n0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt, ++s) {
      read_frags(smem + cur * C::STAGE_BYTES, 1, a1, b1);
      mma(a0, b0);
      const int nxt = cur ^ 1;
      if (s + 1 < S) {
        // DMA(s+1) retired -- kk1 fragments of s landed, and after the barrier no wave reads
        // buffer `cur` any more. The previous tile's E epilogue stores were issued after DMA(s+1)
        // of its last step, so at kt = 0 they may stay in flight.
        if (kt == 0 && ti > 0 && vec_epi) wait_vmcnt<E>();
        else wait_vmcnt<0>();
        lds_barrier();
        if (s + 2 < S) dma_next(cur);
        read_frags(smem + nxt * C::STAGE_BYTES, 0, a0, b0);
      }
      mma(a1, b1);
      cur = nxt;
    }
    if (g.debug & 1) {
#pragma unroll
      for (int mb = 0; mb < TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
    } else {
      epilogue<BF, EPI, BM, BN, WM, WN, 2>(g, acc, m0, n0, wm, wn, lane);
    }
  }
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, 1) void gemm2_kernel(GemmArgs ga) {
  gemm2_body<BF, EPI, BM, BN, WM, WN>(ga, blockIdx.x, gridDim.x);
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN>
hipError_t launch_cfg2(const GemmArgs& g, hipStream_t s) {
  using C = Cfg2<BM, BN, WM, WN>;
  auto kern = gemm2_kernel<BF, EPI, BM, BN, WM, WN>;
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
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, cus);   // <= one per CU
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}


template <bool BF, int EPI>
hipError_t by_id(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 8: return launch_cfg2<BF, EPI, 256, 192, 4, 2>(g, s);
    case 9: return launch_cfg2<BF, EPI, 256, 128, 4, 2>(g, s);
    case 10: return launch_cfg2<BF, EPI, 192, 256, 2, 4>(g, s);
    case 11: return launch_cfg2<BF, EPI, 128, 256, 2, 4>(g, s);
    default: return hipErrorInvalidValue;
  }
}
template <bool BF>
hipError_t by_epi(int epi, int id, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return by_id<BF, EPI_STORE>(id, g, s);
    case EPI_GELU: return by_id<BF, EPI_GELU>(id, g, s);
    case EPI_RESID: return by_id<BF, EPI_RESID>(id, g, s);
    case EPI_PATCH: return by_id<BF, EPI_PATCH>(id, g, s);
    case EPI_SCORE: return by_id<BF, EPI_SCORE>(id, g, s);
    case EPI_FILTER: return by_id<BF, EPI_FILTER>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t gemm2_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s) {
  return bf16 ? by_epi<true>(epi, id, g, s) : by_epi<false>(epi, id, g, s);
}

}  // namespace clm
