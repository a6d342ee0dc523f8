// MFMA GEMM for gfx950: C[M,N] = A[M,K] . W[N,K]^T, bf16/fp16 operands, fp32 accumulate.
//
// Replaces the ATen CPU addmm/conv that the reference runs for every
// nn.Linear / patch-embed conv of the CLIP towers (TF/models/clip/modeling_clip.py:
// 294-297 q/k/v, 332 out_proj, 343-344 fc1/fc2, 148-154 patch conv, and the
// score matmul of src/embedding/search.py:96 / similarity.py:32), with the
// bias, quick-GELU, residual-add, positional-embedding and cosine-scaling
// epilogues fused.
//
// Structure (templated tile BM x BN x 64, WM x WN waves, STAGES-deep LDS ring):
//  * both operand tiles stream HBM/L2 -> LDS by global_load_lds_dwordx4 (16 B per
//    lane, lane-linear 1 KiB per wave-instruction = 8 rows of 128 B); the XOR chunk
//    swizzle is applied to the per-lane SOURCE address so that the ds_read_b128
//    fragment reads (16 rows per lane group) are bank-conflict free;
//  * STAGES = 3: two K-tiles stay in flight across the (raw) barrier, retired by a
//    counted s_waitcnt vmcnt(L) -- never vmcnt(0) in the steady state;
//  * operands are SWAPPED in the MFMA (W rows feed the A port): the 16x16 C-block
//    then has the output row m on the lane and 4 consecutive output columns in the
//    lane's 4 accumulator registers, so every epilogue access is a 4-wide vector
//    (8 B bf16 / 16 B fp32) instead of 2-byte scatter;
//  * workgroup ids are remapped XCD-aware so the N-tiles sharing one A row-panel
//    (and its L2 lines) run on one XCD.
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace clm {

namespace {
constexpr int BK = 64;

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
        if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_RESID)
          if (g.bias) x += g.bias[nj];
        if constexpr (EPI == EPI_STORE) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(x);
        else if constexpr (EPI == EPI_GELU) ((u16*)g.out)[(int64_t)m * g.ldo + nj] = from_f32<BF>(quick_gelu(x));
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
  }
}

// Epilogue of one BM x BN tile from the accumulators.
template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
__device__ __forceinline__ void epilogue(const GemmArgs& g, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane) {
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
  constexpr bool HOIST = !(EPI == EPI_RESID || EPI == EPI_PATCH) || C::TN <= 4;
  float4 cv[C::TN];
#pragma unroll
  for (int nb = 0; nb < C::TN; ++nb) {
    if constexpr (!HOIST) break;
    const int n = wcol + nb * 16;
    if constexpr (EPI == EPI_SCORE || EPI == EPI_FILTER)
      cv[nb] = (g.cscale && n < g.N) ? *(const float4*)(g.cscale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
    else
      cv[nb] = (g.bias && n < g.N) ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) {
    auto finish = [&](int mb, int nb) {
      float v[4] = {acc[mb][nb][0] + cv[nb].x, acc[mb][nb][1] + cv[nb].y, acc[mb][nb][2] + cv[nb].z,
                    acc[mb][nb][3] + cv[nb].w};
      if constexpr (EPI == EPI_GELU) {
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
    // (TN > 4, or PATCH's extra address VALU) one block at a time is loaded, then stored
    constexpr bool PIPE = EPI == EPI_RESID && C::TN <= 4;
    u32x4 hc[C::TN], hn[C::TN];
    load_blk(0, hc);
#pragma unroll
    for (int mb = 0; mb < C::TM; ++mb) {
      if (PIPE && mb + 1 < C::TM) load_blk(mb + 1, hn);
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
        if constexpr (PIPE) {
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
      const auto ob = buf_rsrc((const float*)g.out + (int64_t)m0 * g.ldo, nrec);
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
template <int EPI, int TM, int TN>
constexpr int epi_min_stores() {
  return (EPI == EPI_STORE || EPI == EPI_GELU) ? TM * TN / 2 : EPI == EPI_FILTER ? 0 : TM * TN;
}

// Persistent: workgroup b takes tiles xb, xb + G, xb + 2G, ... (G = gridDim.x <= tiles,
// xb = XCD-aware remap of b), and its LDS-DMA ring runs ACROSS tile boundaries: the first
// K-tiles of tile i+1 are issued before tile i's epilogue, so they land while the epilogue
// runs, and the epilogue's stores drain under tile i+1's main loop (counted vmcnt that
// leaves them in flight). A one-tile-per-workgroup grid is the plain non-persistent GEMM.
template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(WM * WN * 64, (Cfg<BM, BN, WM, WN, STAGES>::WAVES_PER_EU)) void gemm_kernel(GemmArgs g) {
  using C = Cfg<BM, BN, WM, WN, STAGES>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntn * ntm, G = gridDim.x;
  const int xb = xcd_remap(blockIdx.x, G);
  const int n_my = (ntiles - 1 - xb) / G + 1;
  const int nk = g.K / BK;
  const int S = n_my * nk;   // K-steps of all this workgroup's tiles, one ring

  auto coords = [&](int i, int& m0, int& n0) {
    const int t = i * G + xb;
    int tm, tn;
    if (g.m_fastest) {          // every query tile of one index tile back to back (search)
      tm = t % ntm;
      tn = t / ntm;
    } else {                    // grouped raster: GM row-panels x all N-tiles per group, M inner,
      constexpr int GM = 8;     // so an XCD's concurrent tiles share A panels and W tiles in L2
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

  // loader state: per-lane DMA sources of the tile being loaded (piece j of this wave covers
  // tile rows (wid*LA + j)*8 .. +8), re-pointed when the ring crosses into the next tile
  const int r8 = lane >> 3, pc = lane & 7;
  const u16* a_src[C::LA];
  const u16* w_src[C::LB];
  auto point = [&](int i) {
    int m0, n0;
    coords(i, m0, n0);
#pragma unroll
    for (int j = 0; j < C::LA; ++j) {
      const int row = (wid * C::LA + j) * 8 + r8;
      a_src[j] = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + (pc ^ ((row >> 1) & 7)) * 8;
    }
#pragma unroll
    for (int j = 0; j < C::LB; ++j) {
      const int row = (wid * C::LB + j) * 8 + r8;
      w_src[j] = g.W + (int64_t)min(n0 + row, g.N - 1) * g.ldw + (pc ^ ((row >> 1) & 7)) * 8;
    }
  };
  int ld_i = 0, ld_kt = 0;
  point(0);
  auto stage_next = [&](int buf) {   // DMA of the ring's next K-step into LDS buffer buf
    uint8_t* base = smem + buf * C::STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < C::LA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + ld_kt * BK),
                                       (void*)(base + (wid * C::LA + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < C::LB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(w_src[j] + ld_kt * BK),
                                       (void*)(base + BM * 128 + (wid * C::LB + j) * 1024), 16, 0, 0);
    if (++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };

  const int wm = wid / WN, wn = wid % WN;
  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < S) stage_next(s);

  // stores a tile end leaves in flight (the ragged scalar path stores in branches: none counted)
  constexpr int E = epi_min_stores<EPI, C::TM, C::TN>();
  const bool vec_epi = (g.N % 4) == 0 && (g.ldo % 4) == 0 && !(g.debug & 1);
  int c_i = 0, c_kt = 0, m0, n0;
  coords(0, m0, n0);
  bool prev_end = false;
  for (int s = 0; s < S; ++s) {
    // retire K-step s's DMA, leaving younger ones in flight: the STAGES-2 later K-steps' DMA
    // and, right after a tile end, that epilogue's stores (issued after this DMA)
    const bool more = s + STAGES - 2 < S;
    const bool pe = prev_end && vec_epi;
    if (more) {
      if (pe) wait_vmcnt<C::L * (STAGES - 2) + E>();
      else wait_vmcnt<C::L * (STAGES - 2)>();
    } else {
      if (pe) wait_vmcnt<E>();
      else wait_vmcnt<0>();
    }
    lds_barrier();
    if (s + STAGES - 1 < S) stage_next((s + STAGES - 1) % STAGES);
    const uint8_t* sa = smem + (s % STAGES) * C::STAGE_BYTES;
    const uint8_t* sb = sa + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      u32x4 af[C::TM], bw[C::TN];
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int row = wm * (BM / WM) + mb * 16 + (lane & 15);
        af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) {
        const int row = wn * (BN / WN) + nb * 16 + (lane & 15);
        bw[nb] = *(const u32x4*)(sb + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < C::TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], acc[mb][nb]);
    }
    prev_end = ++c_kt == nk;
    if (prev_end) {
      if (g.debug & 1) {   // timing diagnostic: main loop only
#pragma unroll
        for (int mb = 0; mb < C::TM; ++mb)
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
      } else {
        epilogue<BF, EPI, BM, BN, WM, WN, STAGES>(g, acc, m0, n0, wm, wn, lane);
      }
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c_kt = 0;
      if (++c_i < n_my) coords(c_i, m0, n0);
    }
  }
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_cfg(const GemmArgs& g, hipStream_t s) {
  using C = Cfg<BM, BN, WM, WN, STAGES>;
  auto kern = gemm_kernel<BF, EPI, BM, BN, WM, WN, STAGES>;
  static unsigned dev_done = 0;   // >64 KiB dynamic LDS needs the opt-in attribute, once per device
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  // persistent grid: at most one workgroup per resident slot (occupancy x CUs, per device)
  static int slots[32] = {};
  int& sl = slots[dev & 31];
  if (sl == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, C::NT, C::LDS) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
    sl = per_cu * cus;
  }
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM);
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, sl);   // debug bit 2: one tile per workgroup
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}

// tile configurations (index = GemmArgs-independent id, also the `config` of clm_gemm)
template <bool BF, int EPI>
hipError_t launch_id(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 0: return launch_cfg<BF, EPI, 128, 128, 2, 2, 2>(g, s);
    case 1: return launch_cfg<BF, EPI, 128, 128, 2, 2, 3>(g, s);
    case 2: return launch_cfg<BF, EPI, 256, 128, 4, 2, 3>(g, s);
    case 3: return launch_cfg<BF, EPI, 128, 256, 2, 4, 3>(g, s);
    case 4: return launch_cfg<BF, EPI, 256, 256, 4, 2, 2>(g, s);
    case 5: return launch_cfg<BF, EPI, 64, 128, 1, 2, 3>(g, s);
    case 6: return launch_cfg<BF, EPI, 128, 192, 2, 2, 2>(g, s);
    case 7: return launch_cfg<BF, EPI, 192, 128, 2, 2, 2>(g, s);
    case 8: return launch_cfg<BF, EPI, 256, 128, 4, 2, 2>(g, s);
    case 9: return launch_cfg<BF, EPI, 192, 192, 2, 2, 2>(g, s);
    case 10: return launch_cfg<BF, EPI, 128, 256, 2, 4, 2>(g, s);
    default: return hipErrorInvalidValue;
  }
}

constexpr int NCFG = 11;

// Tile choice: a cost model calibrated on the sweep (profiles/r01_v3_gemm_sweep.jsonl).
// time(cfg) ~ rounds(cfg) x round_cost(cfg), rounds = ceil(tiles / resident workgroups),
// round_cost = BM*BN*(workgroups per CU) / efficiency(cfg) with the efficiencies measured on
// 4096^3 (bf16, TF/s / 1000). Narrow GEMMs (N = 512, 768) pick 192x128 (one round instead of
// two 128x128 rounds); wide ones pick 256x256 or 256x128 / 128x256. $CLM_GEMM_CFG overrides.
struct CfgModel { int id, bm, bn, wg_per_cu; double eff; };
constexpr CfgModel MODELS[] = {
  {0, 128, 128, 2, 0.975}, {4, 256, 256, 1, 1.18}, {6, 128, 192, 2, 0.955}, {7, 192, 128, 2, 0.955},
  {8, 256, 128, 1, 1.025}, {10, 128, 256, 1, 1.056}};
int pick_config(int M, int N) {
  static int forced = -2;
  if (forced == -2) {
    const char* e = getenv("CLM_GEMM_CFG");
    forced = e ? atoi(e) : -1;
  }
  if (forced >= 0 && forced < NCFG) return forced;
  int best = 0;
  double best_cost = 1e300;
  for (const CfgModel& c : MODELS) {
    const int64_t tiles = (int64_t)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    const int64_t slots = 256LL * c.wg_per_cu;
    const int64_t rounds = (tiles + slots - 1) / slots;
    const double cost = rounds * (double)c.bm * c.bn * c.wg_per_cu / c.eff;
    if (cost < best_cost * 0.999) { best_cost = cost; best = c.id; }
  }
  return best;
}

template <bool BF>
hipError_t dispatch(int epi, int id, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return launch_id<BF, EPI_STORE>(id, g, s);
    case EPI_GELU: return launch_id<BF, EPI_GELU>(id, g, s);
    case EPI_RESID: return launch_id<BF, EPI_RESID>(id, g, s);
    case EPI_PATCH: return launch_id<BF, EPI_PATCH>(id, g, s);
    case EPI_SCORE: return launch_id<BF, EPI_SCORE>(id, g, s);
    case EPI_FILTER: return launch_id<BF, EPI_FILTER>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

int gemm_num_configs() { return NCFG; }

hipError_t gemm_cfg(bool bf16, int epi, int config, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K <= 0 || (g.K % BK) != 0 || (g.lda % 8) != 0 || (g.ldw % 8) != 0) return hipErrorInvalidValue;
  const int id = config >= 0 ? config : pick_config(g.M, g.N);
  return bf16 ? dispatch<true>(epi, id, g, s) : dispatch<false>(epi, id, g, s);
}

hipError_t gemm(bool bf16, int epi, const GemmArgs& g, hipStream_t s) { return gemm_cfg(bf16, epi, -1, g, s); }

}  // namespace clm
