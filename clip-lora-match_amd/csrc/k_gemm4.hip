// G4 MFMA GEMM for gfx950 (configs 13 / 14 of clm_gemm): 256 x BN tiles (BN = 256 or 128) on FOUR
// waves, one per SIMD, each holding a 128 x BN/2 register tile whose fp32 accumulators live in the
// AGPR half of the 512-entry register file (64 / 32 f32x4 = 256 / 128 AGPRs per lane). Same operand
// layout, persistent tile walk and two-buffer buffer_load ... lds ring as G2 (k_gemm2.hip); what
// changes is the per-wave tile: 16 (BN = 256) fragment reads feed 64 MFMAs per 32-deep half K-step,
// where G2's 64 x 64 / 64 x 96 wave tiles feed 16 / 24 with 8 / 10 -- half the fragment bytes per
// MFMA, the memory work DESIGN §2 found the main loops bound by. The CLIP Linears this serves:
// TF/models/clip/modeling_clip.py:294-297 (q/k/v), 332 (out_proj), 343-344 (fc1 / fc2); the
// caller is /root/reference/models/clip_model.py:89-150.
//
// Register allocation: the MFMA builtins keep the compiler's hazard handling; an empty asm with an
// "a" operand after each MFMA pins every accumulator to the AGPR class, and the epilogues read one
// 16 x 16 block at a time into VGPRs (an "+v" asm on a copy) -- the generic gemm_common epilogue,
// which materialises whole accumulator rows in VGPRs, spills at this tile size (412-748 B of
// scratch; the same main loop alone fits in 176 VGPRs + 256 AGPRs).
#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

typedef __attribute__((address_space(3))) void* lds_ptr4_t;

template <int BN>
struct Cfg4 {
  static constexpr int BM = 256, WM = 2, WN = 2, NW = 4, NT = 256;
  static constexpr int TM = BM / WM / 16;   // 8
  static constexpr int TN = BN / WN / 16;   // 8 or 4
  static constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  static constexpr int LDS = 2 * STAGE_BYTES;
  static constexpr int LA = BM / 8 / NW;     // 8 DMA pieces of A per wave and K-step
  static constexpr int LB = BN / 8 / NW;     // 8 or 4 of W
};

// one 16 x 16 accumulator block into VGPRs, read at its point of use
__device__ __forceinline__ f32x4 take(const f32x4& a) {
  f32x4 v = a;
  asm volatile("" : "+v"(v));
  return v;
}

// STORE / GELU: bias (+ quick-GELU), 16-bit, 16-B stores (v_permlane16_swap pairs column blocks as
// gemm_common's wide path does)
template <bool BF, int EPI, int BN>
__device__ __forceinline__ void epi4_store(const GemmArgs& g, const f32x4 (&acc)[8][BN / 32], int m0, int n0, int wm,
                                           int wn, int lane) {
  using C = Cfg4<BN>;
  constexpr int TN = C::TN;
  const int nrec = (g.debug & 2) ? 0 : 0x7FFFFFF0;
  const int wrow = m0 + wm * 128 + (lane & 15);
  const int wcol = n0 + wn * (BN / 2) + (lane >> 4) * 4;
  float4 cv[TN];
#pragma unroll
  for (int nb = 0; nb < TN; ++nb) {
    const int n = wcol + nb * 16;
    cv[nb] = (g.bias && n < g.N) ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto finish = [&](const f32x4& a, int nb) {
    float v[4] = {a[0] + cv[nb].x, a[1] + cv[nb].y, a[2] + cv[nb].z, a[3] + cv[nb].w};
    if constexpr (epi_gelu(EPI)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = quick_gelu(v[j]);
    }
    return u32x2{pack2<BF>(v[0], v[1]), pack2<BF>(v[2], v[3])};
  };
  // 16-B stores only (gemm4_supports: N, ldo multiples of 8, out 16-B aligned): a second, 8-B store
  // path in this kernel made the compiler drain vmcnt at every tile start (the epilogue's stores
  // could no longer stay in flight under the next tile's first K-steps)
  const auto ob = buf_rsrc((const u16*)g.out + (int64_t)m0 * g.ldo, nrec);
  const int q = lane >> 4;
  const int wcol8 = n0 + wn * (BN / 2) + (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = wrow + mb * 16;
#pragma unroll
    for (int nb = 0; nb < TN; nb += 2) {
      const u32x2 p0 = finish(take(acc[mb][nb]), nb), p1 = finish(take(acc[mb][nb + 1]), nb + 1);
      const auto rx = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
      const int col = wcol8 + nb * 16;
      const uint32_t off = (m < g.M && col < g.N) ? (uint32_t)(((m - m0) * g.ldo + col) * 2) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{rx[0], ry[0], rx[1], ry[1]}, ob, off, 0, 0);
    }
  }
}

// RESID: out (fp32) += acc + bias, h + (acc + b) as gemm_common's RESID epilogue (same bits);
// software-pipelined over row-blocks (block mb + 1's residual loads issued before block mb's stores)
template <int BN>
__device__ __forceinline__ void epi4_resid(const GemmArgs& g, const f32x4 (&acc)[8][BN / 32], int m0, int n0, int wm,
                                           int wn, int lane) {
  using C = Cfg4<BN>;
  constexpr int TN = C::TN;
  const int nrec = (g.debug & 2) ? 0 : 0x7FFFFFF0;
  const int wrow = m0 + wm * 128 + (lane & 15);
  const int wcol = n0 + wn * (BN / 2) + (lane >> 4) * 4;
  const auto ob = buf_rsrc((const float*)g.out + (int64_t)m0 * g.ldo, nrec);
  auto off = [&](int mb, int nb) {
    const int m = wrow + mb * 16, n = wcol + nb * 16;
    return (m < g.M && n < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + n) * 4) : BUF_OOB;
  };
  float4 cv[TN];
#pragma unroll
  for (int nb = 0; nb < TN; ++nb) {
    const int n = wcol + nb * 16;
    cv[nb] = (g.bias && n < g.N) ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  u32x4 hc[TN], hn[TN];
#pragma unroll
  for (int nb = 0; nb < TN; ++nb) hc[nb] = __builtin_amdgcn_raw_buffer_load_b128(ob, off(0, nb), 0, 0);
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    if (mb + 1 < 8) {
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) hn[nb] = __builtin_amdgcn_raw_buffer_load_b128(ob, off(mb + 1, nb), 0, 0);
    }
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      const f32x4 a = take(acc[mb][nb]);
      const float4 c = cv[nb];
      const float r0 = __uint_as_float(hc[nb][0]) + (a[0] + c.x);
      const float r1 = __uint_as_float(hc[nb][1]) + (a[1] + c.y);
      const float r2 = __uint_as_float(hc[nb][2]) + (a[2] + c.z);
      const float r3 = __uint_as_float(hc[nb][3]) + (a[3] + c.w);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(r0), __float_as_uint(r1), __float_as_uint(r2), __float_as_uint(r3)}, ob, off(mb, nb), 0,
          0);
    }
    if (mb + 1 < 8) {
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) hc[nb] = hn[nb];
    }
  }
}

template <int N> struct IC4 { static constexpr int value = N; };

// Main loop, per K-step (two 32-deep halves kk0 / kk1 of the two-buffer ring, G2's order):
//   read kk1 fragments | 64 MFMAs on kk0 (fragments read one step earlier) | wait DMA + barrier |
//   DMA of the K-step two ahead into the buffer just released | read the next kk0 fragments |
//   64 MFMAs on kk1
// At one wave per SIMD no other wave fills the MFMA pipe while a wave issues its 16 LDS-DMA pieces
// (~60 cycles each among MFMAs), so the steady loop is kept branch-free -- the DMA target (this
// tile's K-step kt + 2 or the next tile's kt + 2 - nk, zeros past the last tile) is a select of
// descriptors, the tile's first K-step is peeled -- and sched_group_barrier interleaves the DMA
// pieces and fragment reads one per MFMA. The accumulators are pinned to AGPRs once per K-step.
template <bool BF, int EPI, int BN>
__device__ __forceinline__ void gemm4_body(const GemmArgs& ga, int bid, int G) {
  using C = Cfg4<BN>;
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN;
  constexpr int NP = C::LA + C::LB;   // DMA pieces per wave and K-step
  GemmArgs g = ga;   // varlen: the device-resident row count (the grid was sized for ga.M)
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / 2, wn = wid % 2;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const TileWalk tw = tile_walk(ntn * ntm, bid, G);
  if (tw.count <= 0) return;
  const int n_my = tw.count;
  const int nk = g.K / BK;   // >= 2 (gemm4_supports)

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

  // loader (G2's): descriptors at the tile's first row, record count ending at the matrix's last
  // row (rows past M / N read as zeros); per piece one VGPR offset, the K advance in SOFFSET
  const int r8 = lane >> 3, pc = lane & 7;
  const uint32_t lda2 = (uint32_t)g.lda * 2, ldw2 = (uint32_t)g.ldw * 2;
  const uint32_t ch0 = (uint32_t)((pc ^ ((r8 >> 1) & 7)) << 4);
  const uint32_t ch1 = (uint32_t)((pc ^ ((4 + (r8 >> 1)) & 7)) << 4);
  const uint32_t la0 = r8 * lda2 + ch0, lw0 = r8 * ldw2 + ch0, dch = ch1 - ch0;
  // tile i's descriptors; past the last tile every record is out of range (the DMA writes zeros
  // into a buffer no later step reads)
  auto tile_rsrc = [&](int i, __amdgpu_buffer_rsrc_t& ra, __amdgpu_buffer_rsrc_t& rw) {
    if (i < n_my) {
      int m0, n0;
      coords(i, m0, n0);
      ra = buf_rsrc(g.A + (int64_t)m0 * g.lda, min(BM, g.M - m0) * (int)lda2);
      rw = buf_rsrc(g.W + (int64_t)n0 * g.ldw, min(BN, g.N - n0) * (int)ldw2);
    } else {
      ra = buf_rsrc(g.A, 0);
      rw = buf_rsrc(g.W, 0);
    }
  };
  auto dma = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rw, int ktgt, int buf) {
    uint8_t* base = smem + buf * C::STAGE_BYTES;
    const int so = __builtin_amdgcn_readfirstlane(ktgt * BK * 2);
#pragma unroll
    for (int j = 0; j < C::LA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr4_t)(base + (wid * C::LA + j) * 1024), 16,
                                               (la0 + (uint32_t)((wid * C::LA + j) & 1) * dch) + (uint32_t)((wid * C::LA + j) * 8) * lda2,
                                               so, 0, 0);
#pragma unroll
    for (int j = 0; j < C::LB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr4_t)(base + BM * 128 + (wid * C::LB + j) * 1024), 16,
                                               (lw0 + (uint32_t)((wid * C::LB + j) & 1) * dch) + (uint32_t)((wid * C::LB + j) * 8) * ldw2,
                                               so, 0, 0);
  };
  auto read_frags = [&](const uint8_t* sa, int kk, u32x4 (&af)[TM], u32x4 (&bw)[TN]) {
    const int c = kk * 4 + (lane >> 4);
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int row = wm * 128 + mb * 16 + (lane & 15);
      af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
    }
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      const int row = wn * (BN / 2) + nb * 16 + (lane & 15);
      bw[nb] = *(const u32x4*)(sa + BM * 128 + row * 128 + swz(row, c) * 16);
    }
  };
  f32x4 acc[TM][TN];
  auto mma = [&](const u32x4 (&af)[TM], const u32x4 (&bw)[TN], auto firstc) {
    constexpr bool FIRST = decltype(firstc)::value != 0;   // C = 0: the tile's first half K-step
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb)
        acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mb][nb]);
  };
  auto pin = [&]() {   // the accumulators stay in AGPRs
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) asm volatile("" : "+a"(acc[mb][nb]));
  };

  __amdgpu_buffer_rsrc_t ra, rw, rna, rnw;   // this tile's and the next tile's descriptors
  tile_rsrc(0, ra, rw);
  tile_rsrc(1, rna, rnw);
  dma(ra, rw, 0, 0);
  dma(ra, rw, 1, 1);
  wait_vmcnt<0>();
  lds_barrier();
  u32x4 a0[TM], b0[TN], a1[TM], b1[TN];
  read_frags(smem, 0, a0, b0);

  constexpr int E0 = EPI == EPI_RESID ? TM * TN : TM * TN / 2;   // stores of one tile's epilogue
  constexpr int E = E0 > 63 ? 63 : E0;
  int cur = 0;
  // one K-step (kt of this tile; FIRST: kt == 0, which may leave the previous epilogue's stores in
  // flight -- they are younger than the DMA waited for)
  auto step = [&](int kt, auto firstc) {
    constexpr bool FIRST = decltype(firstc)::value != 0;
    read_frags(smem + cur * C::STAGE_BYTES, 1, a1, b1);
    mma(a0, b0, firstc);
#pragma unroll
    for (int j = 0; j < TM + TN; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 LDS read
    }
    if constexpr (FIRST) wait_vmcnt<E>();
    else wait_vmcnt<0>();
    lds_barrier();
    const bool same = kt + 2 < nk;
    dma(same ? ra : rna, same ? rw : rnw, same ? kt + 2 : kt + 2 - nk, cur);
    cur ^= 1;
    read_frags(smem + cur * C::STAGE_BYTES, 0, a0, b0);
    mma(a1, b1, IC4<0>{});
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // 1 VMEM (LDS-DMA piece)
    }
#pragma unroll
    for (int j = 0; j < TM + TN; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 LDS read
    }
    pin();
  };
  for (int ti = 0; ti < n_my; ++ti) {
    int m0, n0;
    coords(ti, m0, n0);
    step(0, IC4<1>{});
    for (int kt = 1; kt < nk; ++kt) step(kt, IC4<0>{});
    if (g.debug & 1) {
#pragma unroll
      for (int mb = 0; mb < TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"a"(acc[mb][nb]));
    } else if constexpr (EPI == EPI_RESID) {
      epi4_resid<BN>(g, acc, m0, n0, wm, wn, lane);
    } else {
      epi4_store<BF, EPI, BN>(g, acc, m0, n0, wm, wn, lane);
    }
    ra = rna;
    rw = rnw;
    tile_rsrc(ti + 2, rna, rnw);
  }
  wait_vmcnt<0>();   // the zero-filling DMA past the last tile and the last stores
}

template <bool BF, int EPI, int BN>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(GemmArgs ga) {
  gemm4_body<BF, EPI, BN>(ga, blockIdx.x, gridDim.x);
}

template <bool BF, int EPI, int BN>
hipError_t launch_cfg4(const GemmArgs& g, hipStream_t s) {
  using C = Cfg4<BN>;
  auto kern = gemm4_kernel<BF, EPI, BN>;
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
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + C::BM - 1) / C::BM);
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, cus);   // <= one per CU
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}

template <bool BF, int EPI>
hipError_t by_id4(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 13: return launch_cfg4<BF, EPI, 256>(g, s);
    case 14: return launch_cfg4<BF, EPI, 128>(g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

bool gemm4_supports(int epi, const GemmArgs& g) {
  if (g.K % BK || g.K < 2 * BK || g.ksplit > 1 || (g.N % 4) || (g.ldo % 4)) return false;
  if (epi == EPI_RESID) return true;
  return (epi == EPI_STORE || epi == EPI_GELU) && (g.N % 8) == 0 && (g.ldo % 8) == 0 && ((uintptr_t)g.out & 15) == 0;
}

hipError_t gemm4_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s) {
  if (!gemm4_supports(epi, g)) return hipErrorInvalidValue;
  switch (epi) {
    case EPI_STORE: return bf16 ? by_id4<true, EPI_STORE>(id, g, s) : by_id4<false, EPI_STORE>(id, g, s);
    case EPI_GELU: return bf16 ? by_id4<true, EPI_GELU>(id, g, s) : by_id4<false, EPI_GELU>(id, g, s);
    case EPI_RESID: return bf16 ? by_id4<true, EPI_RESID>(id, g, s) : by_id4<false, EPI_RESID>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace clm
