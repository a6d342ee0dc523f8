// Residual GEMM with the next LayerNorm fused (gfx950): for the encoder's out_proj -> LN2 and
// fc2 -> next layer's LN1 (TF/models/clip/modeling_clip.py:362-384: hidden = residual + mlp(..);
// the next layer opens with layer_norm1(hidden)),
//   h[m, :] += A[m, :] . W^T + bias            (fp32 residual stream, N = d)
//   y[m, :]  = LayerNorm(h[m, :]; gamma, beta)  (16-bit input of the next q/k/v or fc1 GEMM)
// in one launch, so the standalone LayerNorm pass over h (4 B read + 2 B written per element, 48
// launches per pair step) is gone and y leaves the epilogue straight from the accumulators.
//
// A workgroup owns BM WHOLE rows (BN = d): 8 waves, wave w all BM rows x the d/8 columns
// [w*d/8, (w+1)*d/8), so the row statistics are in-tile: per-lane partial sums, one 4-lane
// cross-row reduction, eight per-wave partials through LDS, summed by every wave in wave order
// (all waves hold bit-identical statistics, and a row's bits do not depend on its tile).
//
// Main loop: 32-deep K-steps (64-byte LDS rows; the whole 832-row vision stage is 52 KiB, so a
// 3-deep ring fits in 160 KiB beside the statistics), both operands by global_load_lds_dwordx4
// (1 KiB = 16 rows x 64 B per wave-instruction, lane-linear LDS image), the 16-B chunk XOR
// swizzle chunk ^ F[(row >> 2) & 3], F = {0, 2, 3, 1}, on the per-lane SOURCE address: the
// ds_read_b128 fragment reads of 16 rows x 4 chunks then hit 16 distinct bank quads in each of
// the instruction's four 16-lane groups. W rows feed the MFMA A port (lane: output row m =
// lane & 15, 4 consecutive columns), as in k_gemm.hip, so every epilogue access is a vector.
//
// Every CU of one XCD streams the same W (1.2 MB out_proj, 4.7 MB fc2) at nearly the same K
// offset, so W is an L2 hit after the first CU's miss; A is each tile's own rows.
#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

constexpr int RK = 32;
typedef __attribute__((address_space(3))) void* lds_ptr_t;   // K-step depth (elements): one 64-byte LDS row per operand row

// LayerNorm arithmetic, spelled out (explicit fma, fixed association): a row's statistics
// partition its d values as the tiles do -- 8 column slabs of d / 8 (one per wave), 4 interleaved
// 4-column groups per slab (one per 16-lane row of the MFMA C layout), each group summed over its
// 16-column blocks in order; groups combine as (g0 + g1) + (g2 + g3), slabs in order from slab 0.
__device__ __forceinline__ float rl_sum4(float a, float b, float c, float d) { return (a + b) + (c + d); }
__device__ __forceinline__ float rl_sqdev(float a, float b, float c, float d, float mean) {
  const float d0 = a - mean, d1 = b - mean, d2 = c - mean, d3 = d - mean;
  return __builtin_fmaf(d0, d0, d1 * d1) + __builtin_fmaf(d2, d2, d3 * d3);
}
__device__ __forceinline__ float rl_norm(float x, float mean, float rstd, float g, float b) {
  return __builtin_fmaf((x - mean) * rstd, g, b);
}

// physical 16-B slot of logical chunk c in LDS row r (64-byte rows, 4 chunks)
__device__ __forceinline__ int swz64(int r, int c) { return c ^ ((0x78 >> (((r >> 2) & 3) * 2)) & 3); }

template <int BM, int D>
struct RlCfg {
  static constexpr int NW = 8, NT = NW * 64;
  static constexpr int WN = D / NW;            // columns per wave
  static constexpr int TM = BM / 16, TN = WN / 16;
  static constexpr int P = (BM + D) / 16;      // 1-KiB DMA pieces per K-step
  static constexpr int PHI = (P + NW - 1) / NW, PLO = P / NW, NHI = P % NW;   // pieces per wave
  static constexpr int STAGE = (BM + D) * RK * 2;
  static constexpr int RED = 2 * NW * BM * 4;  // row sums, row squared deviations
  static constexpr int STAGES = (163840 - RED) / STAGE > 4 ? 4 : (163840 - RED) / STAGE;
  static constexpr int LDS = STAGES * STAGE + RED;
  static_assert(BM % 16 == 0 && WN % 16 == 0 && TN % 2 == 0, "tile geometry");
  static_assert(STAGES >= 2, "LDS ring");
  static_assert(PHI * (STAGES - 2) <= 63, "vmcnt");
};

template <bool BF, int BM, int D>
__global__ __launch_bounds__(512, 2) void resid_ln_kernel(ResLnArgs aa) {
  using C = RlCfg<BM, D>;
  constexpr int TM = C::TM, TN = C::TN, ST = C::STAGES;
  ResLnArgs a = aa;
  if (a.m_dev) a.M = __builtin_amdgcn_readfirstlane(*a.m_dev);
  const int m0 = blockIdx.x * BM;
  if (m0 >= a.M) return;   // varlen: the grid was sized for the largest row count
  __shared__ __attribute__((aligned(16))) uint8_t smem[C::LDS];
  float* red_s = (float*)(smem + ST * C::STAGE);
  float* red_v = red_s + C::NW * BM;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool hi = wid < C::NHI;   // this wave issues PHI pieces per K-step (else PLO)
  const int nk = a.K / RK;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int c = lane >> 4;

  // loader: piece i of this wave = stacked rows 16 (wid + 8 i) .. +16 (A rows 0..BM-1, then W);
  // lane: row (lane >> 2) of the piece, physical slot lane & 3 <- logical chunk slot ^ F
  const u16* src[C::PHI];
  {
    const int pr = lane >> 2;
    const int ch = (lane & 3) ^ ((0x78 >> (((lane >> 4) & 3) * 2)) & 3);
#pragma unroll
    for (int i = 0; i < C::PHI; ++i) {
      const int j = wid + C::NW * i;
      if (j < BM / 16) {
        const int m = min(m0 + j * 16 + pr, a.M - 1);
        src[i] = a.A + (int64_t)m * a.lda + ch * 8;
      } else {
        const int n = (j - BM / 16) * 16 + pr;
        src[i] = a.W + (int64_t)min(n, D - 1) * a.ldw + ch * 8;   // (past D: a lo wave's unused slot)
      }
    }
  }
  auto stage = [&](int kt) {
    uint8_t* base = smem + (kt % ST) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::PHI; ++i) {
      if (i == C::PHI - 1 && C::NHI != 0 && !hi) break;
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * RK), (void*)(base + (wid + C::NW * i) * 1024), 16, 0,
                                       0);
    }
  };

#pragma unroll
  for (int s = 0; s < ST - 1; ++s)
    if (s < nk) stage(s);

  for (int s = 0; s < nk; ++s) {
    // retire K-step s's pieces; the ST - 2 younger K-steps stay in flight
    if (s + ST - 2 < nk) {
      if (C::NHI == 0 || hi) wait_vmcnt<C::PHI * (ST - 2)>();
      else wait_vmcnt<C::PLO * (ST - 2)>();
    } else {
      wait_vmcnt<0>();
    }
    lds_barrier();
    if (s + ST - 1 < nk) stage(s + ST - 1);
    const uint8_t* sa = smem + (s % ST) * C::STAGE;
    const uint8_t* sb = sa + BM * 64 + wid * C::WN * 64;
    u32x4 af[TM], bw[TN];
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int r = mb * 16 + (lane & 15);
      af[mb] = *(const u32x4*)(sa + r * 64 + swz64(r, c) * 16);
    }
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      const int r = nb * 16 + (lane & 15);
      bw[nb] = *(const u32x4*)(sb + r * 64 + swz64(r, c) * 16);
    }
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], acc[mb][nb]);
  }


  if (a.debug & 1) {   // timing diagnostic: main loop only
#pragma unroll
    for (int mb = 0; mb < TM; ++mb)
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
    return;
  }
  // ---- epilogue: h += acc + bias (the RESID arithmetic, h + (acc + b)), then LayerNorm(h) ----
  // lane: rows m0 + 16 mb + (lane & 15), columns wcol + 16 nb .. +3
  const int wcol = wid * C::WN + (lane >> 4) * 4;
  const auto hb = buf_rsrc(a.h + (int64_t)m0 * a.ldh);
  auto hoff = [&](int mb, int nb) -> uint32_t {
    const int r = mb * 16 + (lane & 15);
    return m0 + r < a.M ? (uint32_t)(((int64_t)r * a.ldh + wcol + nb * 16) * 4) : BUF_OOB;
  };
  float4 bv[TN];
#pragma unroll
  for (int nb = 0; nb < TN; ++nb)
    bv[nb] = a.bias ? *(const float4*)(a.bias + wcol + nb * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
  // residual read-modify-write, software-pipelined over row-blocks (block mb+1's loads are issued
  // before block mb's stores); the row sums accumulate per lane as the blocks complete
  float rs[TM];
  {
    u32x4 hc[TN], hn[TN];
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) hc[nb] = __builtin_amdgcn_raw_buffer_load_b128(hb, hoff(0, nb), 0, 0);
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      if (mb + 1 < TM) {
#pragma unroll
        for (int nb = 0; nb < TN; ++nb) hn[nb] = __builtin_amdgcn_raw_buffer_load_b128(hb, hoff(mb + 1, nb), 0, 0);
      }
      float s = 0.f;
#pragma unroll
      for (int nb = 0; nb < TN; ++nb) {
        f32x4& x = acc[mb][nb];
        x[0] = __uint_as_float(hc[nb][0]) + (x[0] + bv[nb].x);
        x[1] = __uint_as_float(hc[nb][1]) + (x[1] + bv[nb].y);
        x[2] = __uint_as_float(hc[nb][2]) + (x[2] + bv[nb].z);
        x[3] = __uint_as_float(hc[nb][3]) + (x[3] + bv[nb].w);
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])}, hb,
            hoff(mb, nb), 0, 0);
        s += rl_sum4(x[0], x[1], x[2], x[3]);
      }
      rs[mb] = s;
      if (mb + 1 < TM) {
#pragma unroll
        for (int nb = 0; nb < TN; ++nb) hc[nb] = hn[nb];
      }
    }
  }
  if (a.debug & 2) {   // timing diagnostic: residual read-modify-write only, no LayerNorm
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) asm volatile("" ::"v"(rs[mb]));
    return;
  }
  // row statistics: lanes l, l^16, l^32, l^48 share a row; then the 8 waves' partials in order
  auto row_total = [&](float (&part)[TM], float* red, float (&tot)[TM]) {
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const float v = cross_rows_reduce<false>(part[mb]);
      if (lane < 16) red[wid * BM + mb * 16 + lane] = v;
    }
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const int r = mb * 16 + (lane & 15);
      float t = red[r];
#pragma unroll
      for (int w = 1; w < C::NW; ++w) t += red[w * BM + r];
      tot[mb] = t;
    }
  };
  float mean[TM], rstd[TM];
  row_total(rs, red_s, mean);
#pragma unroll
  for (int mb = 0; mb < TM; ++mb) {
    mean[mb] = mean[mb] / D;
    float v = 0.f;
#pragma unroll
    for (int nb = 0; nb < TN; ++nb) {
      v += rl_sqdev(acc[mb][nb][0], acc[mb][nb][1], acc[mb][nb][2], acc[mb][nb][3], mean[mb]);
    }
    rs[mb] = v;
  }
  row_total(rs, red_v, rstd);
#pragma unroll
  for (int mb = 0; mb < TM; ++mb) rstd[mb] = 1.0f / sqrtf(rstd[mb] / D + a.eps);

  // y = (h - mean) * rstd * gamma + beta, 16-B stores: v_permlane16_swap pairs blocks nb, nb+1 so
  // lane group q holds 8 consecutive columns (nb + (q & 1)) * 16 + (q >> 1) * 8 .. +7 (k_gemm.hip)
  const auto yb = buf_rsrc(a.y + (int64_t)m0 * a.ldy);
  const int q = lane >> 4;
  const int wcol8 = wid * C::WN + (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
  for (int nb = 0; nb < TN; nb += 2) {
    float4 g0 = *(const float4*)(a.gamma + wcol + nb * 16), b0 = *(const float4*)(a.beta + wcol + nb * 16);
    float4 g1 = *(const float4*)(a.gamma + wcol + nb * 16 + 16), b1 = *(const float4*)(a.beta + wcol + nb * 16 + 16);
#pragma unroll
    for (int mb = 0; mb < TM; ++mb) {
      const f32x4& x0 = acc[mb][nb];
      const f32x4& x1 = acc[mb][nb + 1];
      const float mu = mean[mb], rsd = rstd[mb];
      const u32x2 p0{pack2<BF>(rl_norm(x0[0], mu, rsd, g0.x, b0.x), rl_norm(x0[1], mu, rsd, g0.y, b0.y)),
                     pack2<BF>(rl_norm(x0[2], mu, rsd, g0.z, b0.z), rl_norm(x0[3], mu, rsd, g0.w, b0.w))};
      const u32x2 p1{pack2<BF>(rl_norm(x1[0], mu, rsd, g1.x, b1.x), rl_norm(x1[1], mu, rsd, g1.y, b1.y)),
                     pack2<BF>(rl_norm(x1[2], mu, rsd, g1.z, b1.z), rl_norm(x1[3], mu, rsd, g1.w, b1.w))};
      const auto rx = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
      const int r = mb * 16 + (lane & 15);
      const uint32_t off = m0 + r < a.M ? (uint32_t)(((int64_t)r * a.ldy + wcol8 + nb * 16) * 2) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{rx[0], ry[0], rx[1], ry[1]}, yb, off, 0, 0);
    }
  }
}

template <bool BF, int BM, int D>
hipError_t launch(const ResLnArgs& a, hipStream_t s) {
  const int grid = (a.M + BM - 1) / BM;
  resid_ln_kernel<BF, BM, D><<<dim3(grid), dim3(RlCfg<BM, D>::NT), 0, s>>>(a);
  return hipGetLastError();
}

template <bool BF, int D>
hipError_t launch_d(int bm, const ResLnArgs& a, hipStream_t s) {
  switch (bm) {
    case 32: return launch<BF, 32, D>(a, s);
    case 64: return launch<BF, 64, D>(a, s);
    case 80: return launch<BF, 80, D>(a, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

bool resid_ln_supported(int d, int K) { return (d == 512 || d == 768) && K > 0 && K % RK == 0; }

// rows per workgroup: the fewest rounds of the 256 CUs (whole-row tiles, one per CU), then the
// smaller tile; up to 4096 rows, 32-row tiles. $CLM_RESLN_BM forces 64 / 80 (tools, tests).
int resid_ln_bm(int M) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("CLM_RESLN_BM");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 64 || forced == 80) return forced;
  if (M <= 32 * 128) return 32;   // few rows (the pruned last layer's pooled rows): more workgroups
  const int r64 = ((M + 63) / 64 + 255) / 256, r80 = ((M + 79) / 80 + 255) / 256;
  return r80 < r64 ? 80 : 64;
}

hipError_t resid_ln(bool bf16, const ResLnArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  if (!resid_ln_supported(a.N, a.K) || (a.lda % 8) || (a.ldw % 8) || (a.ldh % 4) ||
      (a.ldy % 8) || !a.gamma || !a.beta || ((uintptr_t)a.y & 15) || ((uintptr_t)a.h & 15))
    return hipErrorInvalidValue;
  const int bm = a.bm ? a.bm : resid_ln_bm(a.M);
  if (a.N == 768) return bf16 ? launch_d<true, 768>(bm, a, s) : launch_d<false, 768>(bm, a, s);
  return bf16 ? launch_d<true, 512>(bm, a, s) : launch_d<false, 512>(bm, a, s);
}

}  // namespace clm
