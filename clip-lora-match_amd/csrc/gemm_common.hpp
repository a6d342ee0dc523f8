// Shared pieces of the MFMA GEMM kernels (k_gemm.hip, k_gemm2.hip): tile geometry, counted
// vmcnt waits, and the fused epilogues (bias / quick-GELU / fp32 residual / patch rows /
// cosine scores / filtered candidates) from the MFMA accumulators.
#pragma once
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace clm {
namespace gemm_detail {
// grouped raster: row panels per group. 4: an XCD's 32 concurrent tiles cover 4 row panels x 8
// column tiles, fewer unique operand bytes per round than 8 x 4 (Infinity-Cache traffic is the main
// loops' bound): pair step +0.9 % vs 8, 16 -3.7 %, 2 +0.2 %
// (profiles/r02_v6_gemm_raster_ab.txt)
constexpr int GM = 4;
constexpr int BK = 64;

// Persistent tile walk of workgroup bid (of G) over `ntiles` tiles with G workgroups: workgroup xb
// (the bijective XCD remap) takes tiles xb, xb + G, ... (a banded walk, one band of the tile order
// per XCD group, left the L2 hit rate and the pair step unchanged: profiles/r02_v6_gemm_band_ab.txt)
struct TileWalk { int first, stride, count; };
__device__ __forceinline__ TileWalk tile_walk(int ntiles, int bid, int G) {
  const int xb = xcd_remap(bid, G);
  return TileWalk{xb, G, xb < ntiles ? (ntiles - 1 - xb) / G + 1 : 0};
}

template <int BM, int BN, int WM, int WN, int STAGES>
struct Cfg {
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int TM = BM / WM / 16;  // 16-row blocks per wave
  static constexpr int TN = BN / WN / 16;  // 16-col blocks per wave
  static constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  static constexpr int LDS = STAGES * STAGE_BYTES;
  static constexpr int LA = BM / 8 / NW;   // A DMA pieces (8 rows) per wave per K-tile
  static constexpr int LB = BN / 8 / NW;
  static constexpr int L = LA + LB;        // vmcnt units per K-tile
  // workgroups per CU the LDS ring allows, and the waves per SIMD that makes: given to
  // __launch_bounds__ so the register allocation does not cost that occupancy
  static constexpr int WG_PER_CU = (160 * 1024) / LDS;
  static constexpr int WAVES_PER_EU = WG_PER_CU * NW / 4 < 1 ? 1 : (WG_PER_CU * NW / 4 > 8 ? 8 : WG_PER_CU * NW / 4);
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "rows must split evenly over waves");
  static_assert(TM >= 1 && TN >= 1, "wave tile too small");
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is a 6-bit counter");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ragged-N epilogue (N or ldo not a multiple of 4): element by element, same arithmetic
// as the vector paths (score = dot * rscale * cscale in that order)
template <bool BF, int EPI, int TM, int TN>
__device__ __forceinline__ void epilogue_scalar(const GemmArgs& g, const f32x4 (&acc)[TM][TN], int wrow, int wcol) {
#pragma unroll
  for (int mb = 0; mb < TM; ++mb) {
    const int m = wrow + mb * 16;
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
    for (int nb = 0; nb < TN; ++nb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nj = wcol + nb * 16 + j;
        if (nj >= g.N) break;
        float x = acc[mb][nb][j];
        if constexpr (epi_stores16(EPI) || EPI == EPI_RESID)
          if (g.bias) x += g.bias[nj];
        if constexpr (epi_stores16(EPI) && !epi_gelu(EPI)) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(x);
        else if constexpr (epi_gelu(EPI)) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(quick_gelu(x));
        else if constexpr (EPI == EPI_RESID) ((float*)g.out)[(int64_t)m * g.ldo + nj] += x;
        else if constexpr (EPI == EPI_PATCH) ((float*)g.out)[prow * g.ldo + nj] = x + aux[nj];
        else if constexpr (EPI == EPI_SCORE) {
          const float v = x * rs * (g.cscale ? g.cscale[nj] : 1.f);
          if (g.out16) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = (u16)f16_down(v);
          else ((float*)g.out)[(int64_t)m * g.ldo + nj] = v;
        }
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
  }
}

// Residual prefetch (EPI_RESID in gemm_kernel): the fp32 residual values of the first P row-blocks
// a lane's epilogue adds to, loaded into registers while the tile's last K-step still computes --
// that part of the read-modify-write's reads overlaps the main loop instead of following it. Same
// buffer offsets as the epilogue (out-of-range lanes read BUF_OOB: zeros, never stored).
template <int BM, int BN, int WM, int WN, int P>
__device__ __forceinline__ void resid_prefetch(const GemmArgs& g, int m0, int n0, int wm, int wn, int lane,
                                               u32x4 (&h)[P][BN / WN / 16]) {
  const auto ob = buf_rsrc((const float*)g.out + (int64_t)m0 * g.ldo);
  const int wrow = m0 + wm * (BM / WM) + (lane & 15);
  const int wcol = n0 + wn * (BN / WN) + (lane >> 4) * 4;
#pragma unroll
  for (int mb = 0; mb < P; ++mb)
#pragma unroll
    for (int nb = 0; nb < BN / WN / 16; ++nb) {
      const int m = wrow + mb * 16, n = wcol + nb * 16;
      const uint32_t oo = (m < g.M && n < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + n) * 4) : BUF_OOB;
      h[mb][nb] = __builtin_amdgcn_raw_buffer_load_b128(ob, oo, 0, 0);
    }
}

// Epilogue of one BM x BN tile from the accumulators. PRE > 0 (EPI_RESID only): the residual
// values of row-blocks 0 .. PRE-1 are already in hpre (resid_prefetch).
template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES, int PRE = 0>
__device__ __forceinline__ void epilogue(const GemmArgs& g, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane, int64_t out_off = 0,
                                         const u32x4 (*hpre)[BN / WN / 16] = nullptr) {
  static_assert(PRE == 0 || EPI == EPI_RESID, "residual prefetch: RESID epilogue only");
  using C = Cfg<BM, BN, WM, WN, STAGES>;
  // lane owns C[m, n..n+3], m = wrow + 16*mb, n = wcol + 16*nb.
  // Every global load of the epilogue (bias / cscale / row scales, residual, pos rows) is
  // issued in a batch BEFORE the stores it feeds: vmcnt counts loads and stores together in
  // issue order, so a load placed after a store waits for that store's round trip, and a
  // per-block load -> store sequence costs one full memory latency per 16x16 block.
  // (An LDS-staged full-row variant measured slower on every encoder shape:
  // profiles/r01_v5_gemm_split_staged_epilogue.jsonl.)
  const int nrec = (g.debug & 2) ? 0 : 0x7FFFFFF0;   // diagnostic: drop every epilogue store
  const int wrow = m0 + wm * (BM / WM) + (lane & 15);
  const int wcol = n0 + wn * (BN / WN) + (lane >> 4) * 4;
  if ((g.N % 4) != 0 || (g.ldo % 4) != 0) {   // ragged N: scalar tail path
    epilogue_scalar<BF, EPI, C::TM, C::TN>(g, acc, wrow, wcol);
    return;
  }
  // per-column vectors, loaded once per nb (they do not depend on the row); the RESID/PATCH
  // path with TN > 4 loads them per row-block instead (VGPR budget, see below)
  // (PRE: the first blocks load nothing, so the bias vectors are hoisted too)
  constexpr bool HOIST = !(EPI == EPI_RESID || EPI == EPI_PATCH) || C::TN <= 4 || PRE > 0;
  float4 cv[C::TN];
#pragma unroll
  for (int nb = 0; nb < C::TN; ++nb) {
    if constexpr (!HOIST || EPI == EPI_FILTER) break;   // FILTER: loaded after its skip test
    const int n = wcol + nb * 16;
    if constexpr (EPI == EPI_SCORE || EPI == EPI_FILTER)
      cv[nb] = (g.cscale && n < g.N) ? *(const float4*)(g.cscale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
    else
      cv[nb] = (g.bias && n < g.N) ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  if constexpr (epi_stores16(EPI)) {
    auto finish = [&](int mb, int nb) {
      float v[4] = {acc[mb][nb][0] + cv[nb].x, acc[mb][nb][1] + cv[nb].y, acc[mb][nb][2] + cv[nb].z,
                    acc[mb][nb][3] + cv[nb].w};
      if constexpr (epi_gelu(EPI)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = quick_gelu(v[j]);
      }
      return u32x2{pack2<BF>(v[0], v[1]), pack2<BF>(v[2], v[3])};
    };
    const auto ob = buf_rsrc((const u16*)g.out + (int64_t)m0 * g.ldo, nrec);   // tile-relative offsets
    const bool wide = (C::TN % 2) == 0 && (g.N % 8) == 0 && (g.ldo % 8) == 0 && ((uintptr_t)g.out & 15) == 0;
    if (wide) {
      // 16-B stores: v_permlane16_swap trades the odd 16-lane groups' block-nb words with the
      // even groups' block-(nb+1) words, so lane group q holds 8 consecutive columns
      // (nb + (q & 1)) * 16 + (q >> 1) * 8 .. +7 of its row
      const int q = lane >> 4;
      const int wcol8 = n0 + wn * (BN / WN) + (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int m = wrow + mb * 16;
#pragma unroll
        for (int nb = 0; nb < C::TN; nb += 2) {
          const u32x2 p0 = finish(mb, nb), p1 = finish(mb, nb + 1);
          const auto rx = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
          const auto ry = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
          const int col = wcol8 + nb * 16;
          const uint32_t off = (m < g.M && col < g.N) ? (uint32_t)(((m - m0) * g.ldo + col) * 2) : BUF_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{rx[0], ry[0], rx[1], ry[1]}, ob, off, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int m = wrow + mb * 16;
#pragma unroll
        for (int nb = 0; nb < C::TN; ++nb) {
          const int n = wcol + nb * 16;
          const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)(((m - m0) * g.ldo + n) * 2) : BUF_OOB;
          __builtin_amdgcn_raw_buffer_store_b64(finish(mb, nb), ob, off, 0, 0);
        }
      }
    }
  } else if constexpr (EPI == EPI_RESID || EPI == EPI_PATCH) {
    // read-modify-write, software-pipelined over row-blocks: block mb+1's loads are issued
    // before block mb's stores, so no store waits on another store's round trip and only
    // two blocks of loaded rows (2 * TN float4) are live.
    // No branches: out-of-range lanes use BUF_OOB.
    // Patch rows skip each image's class row: out row = m + m / group + 1 (vision embeddings).
    const int64_t orow0 = EPI == EPI_PATCH ? (int64_t)m0 + m0 / g.group + 1 : m0;
    const auto ob = buf_rsrc((const float*)g.out + orow0 * g.ldo, nrec);
    const auto ab = buf_rsrc(EPI == EPI_PATCH ? (const void*)g.aux : g.out);   // pos rows (PATCH)
    auto offs = [&](int mb, int nb, uint32_t& oo, uint32_t& ao) {
      const int m = wrow + mb * 16, n = wcol + nb * 16;
      int64_t orow = m;
      int arow = 0;
      if constexpr (EPI == EPI_PATCH) {
        const int b = m / g.group;
        orow = (int64_t)m + b + 1;
        arow = 1 + (m - b * g.group);
      }
      const bool ok = m < g.M && n < g.N;
      oo = ok ? (uint32_t)(((orow - orow0) * g.ldo + n) * 4) : BUF_OOB;
      ao = ok ? (uint32_t)(((int64_t)arow * g.aux_ld + n) * 4) : BUF_OOB;
    };
    auto load_blk = [&](int mb, u32x4 (&h)[C::TN]) {
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) {
        uint32_t oo, ao;
        offs(mb, nb, oo, ao);
        h[nb] = EPI == EPI_RESID ? __builtin_amdgcn_raw_buffer_load_b128(ob, oo, 0, 0)
                                 : __builtin_amdgcn_raw_buffer_load_b128(ab, ao, 0, 0);
        if constexpr (!HOIST) {
          const int n = wcol + nb * 16;
          cv[nb] = (g.bias && n < g.N) ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    };
    // pipelining holds 2 * TN float4 of loaded rows; where that would cost a wave per SIMD
    // (TN > 4, or PATCH's extra address VALU) one block at a time is loaded, then stored.
    // With P = PRE prefetched blocks, block P is loaded before the first store and the
    // pipelining (or the block-by-block loads) takes over from there.
    constexpr int P = EPI == EPI_RESID ? PRE : 0;
    constexpr bool PIPE = EPI == EPI_RESID && C::TN <= 4;
    u32x4 hc[C::TN], hn[C::TN];
    if constexpr (P > 0) {
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) hc[nb] = hpre[0][nb];
      if (P < C::TM) load_blk(P, hn);
    } else {
      load_blk(0, hc);
    }
#pragma unroll
    for (int mb = 0; mb < C::TM; ++mb) {
      if (PIPE && mb >= P && mb + 1 < C::TM) load_blk(mb + 1, hn);
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) {
        uint32_t oo, ao;
        offs(mb, nb, oo, ao);
        const float4 c = cv[nb];
        const float r0 = __uint_as_float(hc[nb][0]) + (acc[mb][nb][0] + c.x);
        const float r1 = __uint_as_float(hc[nb][1]) + (acc[mb][nb][1] + c.y);
        const float r2 = __uint_as_float(hc[nb][2]) + (acc[mb][nb][2] + c.z);
        const float r3 = __uint_as_float(hc[nb][3]) + (acc[mb][nb][3] + c.w);
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(r0), __float_as_uint(r1), __float_as_uint(r2), __float_as_uint(r3)}, ob, oo, 0, 0);
      }
      if (mb + 1 < C::TM) {
        if (mb + 1 < P) {
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) hc[nb] = hpre[(mb + 1) < P ? mb + 1 : 0][nb];
        } else if (PIPE || mb + 1 == P) {
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) hc[nb] = hn[nb];
        } else {
          load_blk(mb + 1, hc);
        }
      }
    }
  } else {   // EPI_SCORE / EPI_FILTER: score = dot * rscale[m] * cscale[n], in this order
    float rs[C::TM], th[C::TM];
#pragma unroll
    for (int mb = 0; mb < C::TM; ++mb) {
      const int m = wrow + mb * 16;
      rs[mb] = (g.rscale && m < g.M) ? g.rscale[m] : 1.f;
      if constexpr (EPI == EPI_FILTER) th[mb] = m < g.M ? g.theta[(int64_t)m * g.theta_ld] : 0.f;
    }
    if constexpr (EPI == EPI_SCORE) {
      if constexpr (C::TN == 8) {
        if (g.out16 == 2) {
          // the largest of each lane's 4 consecutive scores, fp16 rounded toward -inf: a row's
          // tile of BN columns becomes BN / 4 group maxima, lane (wn, q)'s 8 blocks contiguous at
          // n0 / 4 + wn * (BN / WN) / 4 + q * 8 (a permutation of the groups: the k-th value and
          // count passes read a row's values as a multiset). NaN-propagating maximum.
          const auto oh = buf_rsrc((const u16*)g.out + out_off + (int64_t)m0 * g.ldo, nrec);
          const int q = lane >> 4;
          const int ccol = n0 / 4 + wn * (BN / WN) / 4 + q * 8;
#pragma unroll
          for (int mb = 0; mb < C::TM; ++mb) {
            const int m = wrow + mb * 16;
            uint32_t w[4];
#pragma unroll
            for (int nb = 0; nb < 8; nb += 2) {
              float mx2[2];
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const float4 c = cv[nb + u];
                const f32x4 a = acc[mb][nb + u];
                mx2[u] = __builtin_elementwise_maximum(
                    __builtin_elementwise_maximum(a[0] * rs[mb] * c.x, a[1] * rs[mb] * c.y),
                    __builtin_elementwise_maximum(a[2] * rs[mb] * c.z, a[3] * rs[mb] * c.w));
              }
              w[nb / 2] = f16_down(mx2[0]) | (f16_down(mx2[1]) << 16);
            }
            // every column of the lane's blocks is < N when its first one is (N % 256 == 0 here)
            const uint32_t off = (m < g.M && wcol < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + ccol) * 2) : BUF_OOB;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, oh, off, 0, 0);
          }
          return;
        }
      }
      if (g.out16) {   // fp16 scores rounded toward -inf, 8 B per lane and block
        const auto oh = buf_rsrc((const u16*)g.out + out_off + (int64_t)m0 * g.ldo, nrec);
#pragma unroll
        for (int mb = 0; mb < C::TM; ++mb) {
          const int m = wrow + mb * 16;
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) {
            const int n = wcol + nb * 16;
            const float4 c = cv[nb];
            const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + n) * 2) : BUF_OOB;
            const uint32_t h0 = f16_down(acc[mb][nb][0] * rs[mb] * c.x), h1 = f16_down(acc[mb][nb][1] * rs[mb] * c.y);
            const uint32_t h2 = f16_down(acc[mb][nb][2] * rs[mb] * c.z), h3 = f16_down(acc[mb][nb][3] * rs[mb] * c.w);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{h0 | (h1 << 16), h2 | (h3 << 16)}, oh, off, 0, 0);
          }
        }
        return;
      }
      const auto ob = buf_rsrc((const float*)g.out + out_off + (int64_t)m0 * g.ldo, nrec);
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int m = wrow + mb * 16;
#pragma unroll
        for (int nb = 0; nb < C::TN; ++nb) {
          const int n = wcol + nb * 16;
          const float4 c = cv[nb];
          const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)(((int64_t)(m - m0) * g.ldo + n) * 4) : BUF_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{__float_as_uint(acc[mb][nb][0] * rs[mb] * c.x), __float_as_uint(acc[mb][nb][1] * rs[mb] * c.y),
                    __float_as_uint(acc[mb][nb][2] * rs[mb] * c.z), __float_as_uint(acc[mb][nb][3] * rs[mb] * c.w)},
              ob, off, 0, 0);
        }
      }
    } else {
      // Skip test: with cmin = min cscale >= 0 and cmax = max cscale finite, every score of a
      // 16 x 16 block, (acc * rs) * c, is at most (mx * rs) * (mx >= 0 ? cmax : cmin), mx = the
      // block's largest accumulator on the lane (fp32 multiplication is monotonic; same operation
      // order as the scores), so a row block / block that no lane of the wave can append from is
      // skipped whole, before its cscale loads. Out-of-range columns (clamped operand rows) only
      // raise mx. The appended (score, row) set is exactly the unskipped path's.
      if (g.cbound) {
        const float cmin = key_float(g.cbound[0]), cmax = key_float(g.cbound[1]);
        const bool cok = cmin >= 0.f && cmax <= 3.4028235e38f;   // NaN fails both
#pragma unroll
        for (int mb = 0; mb < C::TM; ++mb) {
          const int m = wrow + mb * 16;
          const bool live = m < g.M;
          const bool rok = cok && rs[mb] >= 0.f && rs[mb] <= 3.4028235e38f && th[mb] >= -3.4028235e38f;
          float bmx[C::TN];
          float mx = -3.4028235e38f;
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) {
            bmx[nb] = fmaxf(fmaxf(acc[mb][nb][0], acc[mb][nb][1]), fmaxf(acc[mb][nb][2], acc[mb][nb][3]));
            mx = fmaxf(mx, bmx[nb]);
          }
          auto reach = [&](float v) { return live && (!rok || (v * rs[mb]) * (v >= 0.f ? cmax : cmin) >= th[mb]); };
          if (!__any(reach(mx))) continue;
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) {
            if (!__any(reach(bmx[nb]))) continue;
            const int n = wcol + nb * 16;
            if (!live || n >= g.N) continue;
            const float4 c = g.cscale ? *(const float4*)(g.cscale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float sc[4] = {acc[mb][nb][0] * rs[mb] * c.x, acc[mb][nb][1] * rs[mb] * c.y,
                                 acc[mb][nb][2] * rs[mb] * c.z, acc[mb][nb][3] * rs[mb] * c.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (sc[j] >= th[mb]) {
                const int slot = atomicAdd(g.cnt + m, 1);
                if (slot < g.cap) {
                  g.cand_s[(int64_t)m * g.cap + slot] = sc[j];
                  g.cand_i[(int64_t)m * g.cap + slot] = g.base + n + j;
                }
              }
            }
          }
        }
        return;
      }
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) {
        const int n = wcol + nb * 16;
        cv[nb] = (g.cscale && n < g.N) ? *(const float4*)(g.cscale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
      }
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int m = wrow + mb * 16;
        if (m >= g.M) continue;
#pragma unroll
        for (int nb = 0; nb < C::TN; ++nb) {
          const int n = wcol + nb * 16;
          if (n >= g.N) continue;
          const float4 c = cv[nb];
          const float sc[4] = {acc[mb][nb][0] * rs[mb] * c.x, acc[mb][nb][1] * rs[mb] * c.y,
                               acc[mb][nb][2] * rs[mb] * c.z, acc[mb][nb][3] * rs[mb] * c.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (sc[j] >= th[mb]) {
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

// Stores (vector-memory instructions) one tile's epilogue issues per wave at least, on the
// vector paths; the main loop's counted vmcnt leaves this many in flight after a tile end
// (a smaller count than actually issued only over-waits). FILTER stores in branches: 0.
// EPI_SCORE with TN == 8 may run the group-maxima form (GemmArgs::out16 == 2: one 16-B store per
// row-block, TM in all), so it counts TM.
template <int EPI, int TM, int TN>
constexpr int epi_min_stores() {
  return epi_stores16(EPI) ? TM * TN / 2 : EPI == EPI_FILTER ? 0 : (EPI == EPI_SCORE && TN == 8) ? TM : TM * TN;
}

}  // namespace gemm_detail

// G2 kernels (k_gemm2.hip): configs 8-11
hipError_t gemm2_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s);
// G4 kernels (k_gemm4.hip): configs 13 (256 x 256) / 14 (256 x 128), 4 waves of 128 x BN/2
bool gemm4_supports(int epi, const GemmArgs& g);
hipError_t gemm4_launch(bool bf16, int epi, int id, const GemmArgs& g, hipStream_t s);
}  // namespace clm
