// EXPERIMENT (round 4, not built into libclm): G2's main loop on v_mfma_f32_32x32x16 (configs
// 12-16 while it was built). Exact on small-integer operands against the 16x16x32 kernels on every
// encoder shape and epilogue (the 32 x 32 C layout and the permlane32 16-B stores are right), but
// no faster (tools/pp_probe.py, profiles/r04_v2_w32_probe.jsonl, fp16, batch 256, main loop / full
// us): v_fc1 60.1 / 76.8 vs G2 55.9 / 71.1; v_fc2 (128 x 192, 2 WG/CU) 68.5 / 81.4 vs 57.7 / 68.6
// (160 x 128); 256 x 256 on v_qkv 43.4 / 57.0 vs 44.3 / 58.4, t_qkv 29.7 / 43.3 vs 31.0 / 45.9.
// The wide shape's 3/4 free issue cycles (vs 1/2) do not move these loops: they are not bound by
// MFMA issue slots. Kept for the record (and the 32 x 32 epilogue), not in the build.
// W32 MFMA GEMM for gfx950 (configs 12-15 of clm_gemm): G2's main loop (k_gemm2.hip: two-buffer
// LDS ring filled by buffer_load ... lds, fragments of one K-half read while the other half's
// MFMAs run, one barrier per K-step) on v_mfma_f32_32x32x16_{f16,bf16} instead of 16x16x32.
//
// Why: the encoder GEMMs are issue-bound (PMC: 37-46 % of the waves' cycles are issue stalls,
// MFMA pipe 31-34 % busy). A 16x16x32 MFMA holds its SIMD's issue for 8 of its 16 cycles, a
// 32x32x16 for 8 of its 32 (MI355X_MICROARCH.md, cycle constants): at equal FLOPs the wide shape
// leaves 3/4 instead of 1/2 of the issue cycles to the fragment reads, the LDS-DMA and the loop's
// scalar work of both waves of a SIMD. The LDS image and its XOR swizzle are G2's: the 32x32x16
// fragment reads (lanes 0-31 one 16-B chunk of rows 0-31, lanes 32-63 the next chunk) are
// conflict-free in it as well (each ds_read_b128 lane group covers 8 row pairs x 2 parities).
//
// Operands swapped as in every GEMM here (W rows on the MFMA A port): a lane holds output row
// m = lane & 31 of a 32 x 32 block and, in accumulator registers 4g .. 4g + 3, output columns
// 8g + 4 (lane >> 5) .. + 3 (g = 0..3). The 32x32x16 MFMA sums 16 products per step instead of
// 32, so its results are not bit-identical to the 16x16x32 kernels' (rounding of the partial
// sums); a model uses one MFMA shape for every GEMM of a role (see pick_config).
#include <algorithm>

#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool BF>
__device__ __forceinline__ f32x16 mfma32(const u32x4& a, const u32x4& b, f32x16 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

template <int BM, int BN, int WM, int WN>
struct Cfg32 {
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int TM = BM / WM / 32;   // 32-row blocks per wave
  static constexpr int TN = BN / WN / 32;   // 32-col blocks per wave
  static constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  static constexpr int LDS = 2 * STAGE_BYTES;
  static constexpr int LA = BM / 8 / NW;
  static constexpr int LB = BN / 8 / NW;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "rows must split evenly over waves");
  static_assert(TM >= 1 && TN >= 1 && BM % (32 * WM) == 0 && BN % (32 * WN) == 0, "32 x 32 blocks");
};

// ---- epilogue from 32 x 32 accumulators ---------------------------------------------------------
// fragment (mb, nb, g) of a lane: row m = wrow + 32 mb, columns n .. n + 3 with n = wcol + 32 nb + 8 g
template <bool BF, int EPI, int TM, int TN>
__device__ __forceinline__ void epilogue32(const GemmArgs& g, const f32x16 (&acc)[TM][TN], int m0, int n0, int wrow,
                                           int wcol, int lane) {
  const int nrec = (g.debug & 2) ? 0 : 0x7FFFFFF0;
  auto frag = [&](int mb, int nb, int q) {
    return float4{acc[mb][nb][4 * q], acc[mb][nb][4 * q + 1], acc[mb][nb][4 * q + 2], acc[mb][nb][4 * q + 3]};
  };
  if ((g.N % 4) != 0 || (g.ldo % 4) != 0) {   // ragged N: element by element (same arithmetic)
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int m = wrow + mb * 32;
      if (m >= g.M) continue;
      const float rs = (EPI == EPI_SCORE || EPI == EPI_FILTER) && g.rscale ? g.rscale[m] : 1.f;
      int64_t prow = m;
      const float* aux = nullptr;
      if constexpr (EPI == EPI_PATCH) {
        const int b = m / g.group, p = m - b * g.group;
        prow = (int64_t)b * (g.group + 1) + 1 + p;
        aux = g.aux + (int64_t)(1 + p) * g.aux_ld;
      }
#pragma unroll
      for (int nb = 0; nb < TN; ++nb)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int nj = wcol + nb * 32 + 8 * q + j;
            if (nj >= g.N) continue;
            float x = acc[mb][nb][4 * q + j];
            if constexpr (epi_stores16(EPI) || EPI == EPI_RESID)
              if (g.bias) x += g.bias[nj];
            if constexpr (epi_stores16(EPI) && !epi_gelu(EPI)) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(x);
            else if constexpr (epi_gelu(EPI)) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(quick_gelu(x));
            else if constexpr (EPI == EPI_RESID) ((float*)g.out)[(int64_t)m * g.ldo + nj] += x;
            else if constexpr (EPI == EPI_PATCH) ((float*)g.out)[prow * g.ldo + nj] = x + aux[nj];
            else if constexpr (EPI == EPI_SCORE) ((float*)g.out)[(int64_t)m * g.ldo + nj] = x * rs * (g.cscale ? g.cscale[nj] : 1.f);
            else {
              const float sc = x * rs * g.cscale[nj];
              if (sc >= g.theta[(int64_t)m * g.theta_ld]) {
                const int slot = atomicAdd(g.cnt + m, 1);
                if (slot < g.cap) {
                  g.cand_s[(int64_t)m * g.cap + slot] = sc;
                  g.cand_i[(int64_t)m * g.cap + slot] = g.base + nj;
                }
              }
            }
          }
    }
    return;
  }
  auto colvec = [&](const float* v, int n, float dflt) {
    return (v && n < g.N) ? *(const float4*)(v + n) : make_float4(dflt, dflt, dflt, dflt);
  };
  if constexpr (epi_stores16(EPI)) {
    // v_permlane32_swap pairs lane l (columns 8q .. 8q+3) with lane l + 32 (8q+4 .. 8q+7): after the
    // swap of the q = 2p and 2p + 1 pieces, lanes 0-31 hold columns 16p .. 16p+7 and lanes 32-63
    // columns 16p+8 .. 16p+15 of their row: one 16-B store each
    const auto ob = buf_rsrc((const u16*)g.out + (int64_t)m0 * g.ldo, nrec);
    const bool wide = (g.N % 8) == 0 && (g.ldo % 8) == 0 && ((uintptr_t)g.out & 15) == 0;
    const int h = lane >> 5;
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      float4 bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[q] = colvec(g.bias, wcol + nb * 32 + 8 * q, 0.f);
#pragma unroll
      for (int mb = 0; mb < TM; ++mb) {
        const int m = wrow + mb * 32;
        u32x2 pk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 a = frag(mb, nb, q);
          float v[4] = {a.x + bv[q].x, a.y + bv[q].y, a.z + bv[q].z, a.w + bv[q].w};
          if constexpr (epi_gelu(EPI)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = quick_gelu(v[j]);
          }
          pk[q] = u32x2{pack2<BF>(v[0], v[1]), pack2<BF>(v[2], v[3])};
        }
        if (wide) {
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const auto rx = __builtin_amdgcn_permlane32_swap(pk[2 * p].x, pk[2 * p + 1].x, false, false);
            const auto ry = __builtin_amdgcn_permlane32_swap(pk[2 * p].y, pk[2 * p + 1].y, false, false);
            const int col = wcol - 4 * h + nb * 32 + 16 * p + 8 * h;
            const uint32_t off = (m < g.M && col < g.N) ? (uint32_t)(((m - m0) * g.ldo + col) * 2) : BUF_OOB;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{rx[0], ry[0], rx[1], ry[1]}, ob, off, 0, 0);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = wcol + nb * 32 + 8 * q;
            const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)(((m - m0) * g.ldo + n) * 2) : BUF_OOB;
            __builtin_amdgcn_raw_buffer_store_b64(pk[q], ob, off, 0, 0);
          }
        }
      }
    }
  } else if constexpr (EPI == EPI_RESID || EPI == EPI_PATCH) {
    // read-modify-write per row-block: all of a block's loads issued before its stores
    const int64_t orow0 = EPI == EPI_PATCH ? (int64_t)m0 + m0 / g.group + 1 : m0;
    const auto ob = buf_rsrc((const float*)g.out + orow0 * g.ldo, nrec);
    const auto ab = buf_rsrc(EPI == EPI_PATCH ? (const void*)g.aux : g.out);
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int m = wrow + mb * 32;
      int64_t orow = m;
      int arow = 0;
      if constexpr (EPI == EPI_PATCH) {
        const int b = m / g.group;
        orow = (int64_t)m + b + 1;
        arow = 1 + (m - b * g.group);
      }
      u32x4 hv[TN][4];
      uint32_t oo[TN][4];
#pragma unroll
      for (int nb = 0; nb < TN; ++nb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = wcol + nb * 32 + 8 * q;
          const bool ok = m < g.M && n < g.N;
          oo[nb][q] = ok ? (uint32_t)(((orow - orow0) * g.ldo + n) * 4) : BUF_OOB;
          const uint32_t ao = ok ? (uint32_t)(((int64_t)arow * g.aux_ld + n) * 4) : BUF_OOB;
          hv[nb][q] = EPI == EPI_RESID ? __builtin_amdgcn_raw_buffer_load_b128(ob, oo[nb][q], 0, 0)
                                       : __builtin_amdgcn_raw_buffer_load_b128(ab, ao, 0, 0);
        }
#pragma unroll
      for (int nb = 0; nb < TN; ++nb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 a = frag(mb, nb, q);
          const float4 c = EPI == EPI_RESID ? colvec(g.bias, wcol + nb * 32 + 8 * q, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float r0 = __uint_as_float(hv[nb][q][0]) + (a.x + c.x);
          const float r1 = __uint_as_float(hv[nb][q][1]) + (a.y + c.y);
          const float r2 = __uint_as_float(hv[nb][q][2]) + (a.z + c.z);
          const float r3 = __uint_as_float(hv[nb][q][3]) + (a.w + c.w);
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{__float_as_uint(r0), __float_as_uint(r1), __float_as_uint(r2), __float_as_uint(r3)}, ob, oo[nb][q], 0, 0);
        }
    }
  } else {   // EPI_SCORE / EPI_FILTER: score = dot * rscale[m] * cscale[n], in this order
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int m = wrow + mb * 32;
      const float rs = (g.rscale && m < g.M) ? g.rscale[m] : 1.f;
      if constexpr (EPI == EPI_SCORE) {
        const auto ob = buf_rsrc((const float*)g.out + (int64_t)m0 * g.ldo, nrec);
#pragma unroll
        for (int nb = 0; nb < TN; ++nb)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = wcol + nb * 32 + 8 * q;
            const float4 c = colvec(g.cscale, n, 1.f);
            const float4 a = frag(mb, nb, q);
            const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + n) * 4) : BUF_OOB;
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4{__float_as_uint(a.x * rs * c.x), __float_as_uint(a.y * rs * c.y), __float_as_uint(a.z * rs * c.z),
                      __float_as_uint(a.w * rs * c.w)},
                ob, off, 0, 0);
          }
      } else {
        if (m >= g.M) continue;
        const float th = g.theta[(int64_t)m * g.theta_ld];
#pragma unroll
        for (int nb = 0; nb < TN; ++nb)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = wcol + nb * 32 + 8 * q;
            if (n >= g.N) continue;
            const float4 c = colvec(g.cscale, n, 1.f);
            const float4 a = frag(mb, nb, q);
            const float sc[4] = {a.x * rs * c.x, a.y * rs * c.y, a.z * rs * c.z, a.w * rs * c.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (sc[j] >= th) {
                const int slot = atomicAdd(g.cnt + m, 1);
                if (slot < g.cap) {
                  g.cand_s[(int64_t)m * g.cap + slot] = sc[j];
                  g.cand_i[(int64_t)m * g.cap + slot] = g.base + n + j;
                }
              }
            }
          }
      }
    }
  }
}

template <int EPI, int TM, int TN>
constexpr int epi32_min_stores() {
  return epi_stores16(EPI) ? TM * TN * 2 : EPI == EPI_FILTER ? 0 : TM * TN * 4;
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN, int WGPC>
__global__ __launch_bounds__(WM * WN * 64, WGPC * WM * WN / 4) void gemm32_kernel(GemmArgs ga) {
  using C = Cfg32<BM, BN, WM, WN>;
  GemmArgs g = ga;   // varlen: the device-resident row count (the grid was sized for ga.M)
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  constexpr int L = C::LA + C::LB;
  constexpr int TM = C::TM, TN = C::TN;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntn * ntm, G = gridDim.x;
  const TileWalk tw = tile_walk(ntiles, G);
  if (tw.count <= 0) return;
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
  // K-half kh of a stage: 16-deep steps k16 = 2 kh, 2 kh + 1; chunk of lane = 2 k16 + (lane >> 5)
  auto read_frags = [&](const uint8_t* sa, int kh, u32x4 (&af)[2][TM], u32x4 (&bw)[2][TN]) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int c = (2 * kh + s2) * 2 + (lane >> 5);
#pragma unroll
      for (int mb = 0; mb < TM; ++mb) {
        const int row = wm * (BM / WM) + mb * 32 + (lane & 31);
        af[s2][mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) {
        const int row = wn * (BN / WN) + nb * 32 + (lane & 31);
        bw[s2][nb] = *(const u32x4*)(sa + BM * 128 + row * 128 + swz(row, c) * 16);
      }
    }
  };
  f32x16 acc[TM][TN];
  auto mma = [&](const u32x4 (&af)[2][TM], const u32x4 (&bw)[2][TN]) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int mb = 0; mb < TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < TN; ++nb) acc[mb][nb] = mfma32<BF>(bw[s2][nb], af[s2][mb], acc[mb][nb]);
  };

  dma_next(0);
  if (S > 1) dma_next(1);
  if (S >= 2) wait_vmcnt<L>();
  else wait_vmcnt<0>();
  lds_barrier();
  u32x4 a0[2][TM], b0[2][TN], a1[2][TM], b1[2][TN];
  read_frags(smem, 0, a0, b0);

  constexpr int E0 = epi32_min_stores<EPI, TM, TN>();
  constexpr int E = E0 > 63 ? 63 : E0;
  const bool vec_epi = (g.N % 4) == 0 && (g.ldo % 4) == 0 && !(g.debug & 1);
  const int wrow_l = wm * (BM / WM) + (lane & 31), wcol_l = wn * (BN / WN) + 4 * (lane >> 5);
  int s = 0, cur = 0;
  for (int ti = 0; ti < n_my; ++ti) {
    int m0, n0;
    coords(ti, m0, n0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
    for (int kt = 0; kt < nk; ++kt, ++s) {
      read_frags(smem + cur * C::STAGE_BYTES, 1, a1, b1);
      mma(a0, b0);
      const int nxt = cur ^ 1;
      if (s + 1 < S) {
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
        for (int nb = 0; nb < TN; ++nb)
#pragma unroll
          for (int q = 0; q < 4; ++q)   // 16-byte pieces: the host pass rejects a 64-byte "v" operand
            asm volatile("" ::"v"(f32x4{acc[mb][nb][4 * q], acc[mb][nb][4 * q + 1], acc[mb][nb][4 * q + 2],
                                        acc[mb][nb][4 * q + 3]}));
    } else {
      epilogue32<BF, EPI, TM, TN>(g, acc, m0, n0, m0 + wrow_l, n0 + wcol_l, lane);
    }
  }
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN, int WGPC>
hipError_t launch_cfg32(const GemmArgs& g, hipStream_t s) {
  using C = Cfg32<BM, BN, WM, WN>;
  static_assert(C::LDS * WGPC <= 160 * 1024, "LDS of the resident workgroups");
  auto kern = gemm32_kernel<BF, EPI, BM, BN, WM, WN, WGPC>;
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
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, cus * WGPC);
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}

template <bool BF, int EPI>
hipError_t by_id32(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 12: return launch_cfg32<BF, EPI, 256, 128, 4, 2, 1>(g, s);
    case 13: return launch_cfg32<BF, EPI, 128, 256, 2, 4, 1>(g, s);
    case 14: return launch_cfg32<BF, EPI, 256, 256, 4, 2, 1>(g, s);
    case 15: return launch_cfg32<BF, EPI, 128, 192, 2, 2, 2>(g, s);
    case 16: return launch_cfg32<BF, EPI, 192, 128, 2, 2, 2>(g, s);
    default: return hipErrorInvalidValue;
  }
}
template <bool BF>
hipError_t by_epi32(int epi, int id, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return by_id32<BF, EPI_STORE>(id, g, s);
    case EPI_GELU: return by_id32<BF, EPI_GELU>(id, g, s);
    case EPI_RESID: return by_id32<BF, EPI_RESID>(id, g, s);
    case EPI_PATCH: return by_id32<BF, EPI_PATCH>(id, g, s);
    case EPI_SCORE: return by_id32<BF, EPI_SCORE>(id, g, s);
    case EPI_FILTER: return by_id32<BF, EPI_FILTER>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t gemm32_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s) {
  return bf16 ? by_epi32<true>(epi, id, g, s) : by_epi32<false>(epi, id, g, s);
}
}  // namespace clm
