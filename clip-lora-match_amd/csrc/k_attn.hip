// Multi-head attention for the CLIP towers on gfx950 MFMA.
//
// Replaces CLIPAttention's sdpa/eager core (TF/models/clip/modeling_clip.py:
// 259-277, 298-335): softmax(Q K^T * 64^-1/2 [+ causal mask]) V per (batch, head),
// head_dim 64, T = 50 (B/32 image), 77 (text, causal), 577 (L/14@336 image).
// The 64^-1/2 scale is folded into the q_proj weights at load (a power of two,
// so the product is bit-identical to scaling the scores).
//
// Key tiles of 64: K and V staged in LDS row-major with the 128-B-row XOR swizzle (K read
// as ds_read_b128 fragments, V through ds_read_b64_tr_b16, see v_frag_trT). Scores are
// computed transposed, S^T = K Q^T, so each lane owns one query: the fp32 softmax reduces
// in-lane plus two cross-lane steps (v_permlane16/32_swap), and P stays in registers as the B operand of
// O^T = V^T P^T. attn_kernel (T > 128) runs an online softmax over double-buffered tiles;
// attn_small_kernel (T <= 128) holds every key and does one exact pass.
#include "kernels.hpp"

namespace clm {

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));

// V^T operand of O^T = V^T P^T, from a ROW-MAJOR V tile ([64 keys][128 B], 16-B chunks
// XOR-swizzled by (key>>1)&7 like K) with two ds_read_b64_tr_b16 (per 16-lane group, lane
// 4q+p addresses key row q, dims 4p..4p+3, and lane i receives dim i of the 4 rows): lane l holds
// V[key0 + 4*(l>>4) + 0..3][dim0 + (l&15)] and V[key0 + 16 + 4*(l>>4) + 0..3][dim0 + (l&15)],
// the key order in which the lane holds P (S^T C layout of key blocks 2kk and 2kk+1).
__device__ __forceinline__ u32x4 v_frag_trT(const uint8_t* tile, int kbase, int nb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int chunk = nb * 2 + (p >> 1);
  const int ka = kbase + g * 4 + q, kb = ka + 16;
  const uint8_t* pa = tile + ka * 128 + ((chunk ^ ((ka >> 1) & 7)) << 4) + (p & 1) * 8;
  const uint8_t* pb = tile + kb * 128 + ((chunk ^ ((kb >> 1) & 7)) << 4) + (p & 1) * 8;
  const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  const u32x2 a = __builtin_bit_cast(u32x2, ra), b = __builtin_bit_cast(u32x2, rb);
  return u32x4{a.x, a.y, b.x, b.y};
}

// T > 128 (ViT-L/14@336: T = 577). One workgroup = (128-query block, head, batch): 4 waves x
// two 16-query blocks, so every K fragment (ds_read_b128) and V fragment (ds_read_b64_tr_b16)
// read from LDS feeds two MFMAs. Scores are computed transposed, S^T = K Q^T, so a lane owns
// ONE query and 16 of the tile's 64 keys: the softmax max / sum are 15 in-lane ops + 2
// cross-lane steps, and P stays in registers as the B operand of O^T = V^T P^T (no LDS round
// trip). K / V tiles of 64 keys are double-buffered in LDS and the next tile is loaded into
// registers while the current one computes: one barrier per tile.
template <bool BF, bool CAUSAL>
__global__ __launch_bounds__(256, CAUSAL ? 2 : 3) void attn_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                      int T, int d) {
  constexpr int RB = 2;   // 16-query blocks per wave
  constexpr float L2E = 1.4426950408889634f;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 16384];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4;
  const u16* base = qkv + (int64_t)b * T * ldq;
  const int qw = qb * 64 * RB + wid * 16 * RB;   // first query of this wave

  u32x4 qa[RB][2];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = min(qw + rb * 16 + (lane & 15), T - 1);
    const u16* qp = base + (int64_t)r * ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qa[rb][kk] = *(const u32x4*)(qp + kk * 32 + 8 * g);
  }
  f32x4 o[RB][4];   // O^T: lane holds query (lane&15), dims nb*16 + 4g + 0..3
  float mrow[RB], lrow[RB];   // running max (log2 domain) and sum for this lane's query
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mrow[rb] = -INFINITY;
    lrow[rb] = 0.f;
  }

  const int ntiles = (T + 63) / 64;
  const int nkt = CAUSAL ? min((qb * 64 * RB + 64 * RB - 1) / 64 + 1, ntiles) : ntiles;
  u32x4 kr[2], vr[2];   // this thread's 2 chunks of the next K / V tile
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = tid + 256 * i, key = ci >> 3, c = ci & 7, kg = kt * 64 + key;
      kr[i] = u32x4{0u, 0u, 0u, 0u};
      vr[i] = u32x4{0u, 0u, 0u, 0u};
      if (kg < T) {
        const u16* rp = base + (int64_t)kg * ldq + h * 64 + c * 8;
        kr[i] = *(const u32x4*)(rp + d);
        vr[i] = *(const u32x4*)(rp + 2 * d);
      }
    }
  };
  auto stage = [&](int buf) {
    uint8_t* sK = smem + buf * 16384;
    uint8_t* sV = sK + 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = tid + 256 * i, key = ci >> 3, c = ci & 7;
      *(u32x4*)(sK + key * 128 + swz(key, c) * 16) = kr[i];
      *(u32x4*)(sV + key * 128 + swz(key, c) * 16) = vr[i];
    }
  };
  load(0);
  stage(0);
  if (nkt > 1) load(1);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const uint8_t* sK = smem + (kt & 1) * 16384;
    const uint8_t* sV = sK + 8192;
    f32x4 sc[RB][4];   // S^T: lane holds query (lane&15), keys kt*64 + nb*16 + 4g + 0..3
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) sc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = nb * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + g;
        const u32x4 kb = *(const u32x4*)(sK + krow * 128 + swz(krow, c) * 16);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) sc[rb][nb] = mfma16<BF>(kb, qa[rb][kk], sc[rb][nb]);
      }
    }
    const bool masked = CAUSAL || (kt + 1) * 64 > T;
    u32x4 pb[RB][2];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      if (masked) {
        const int qi = qw + rb * 16 + (lane & 15);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kj = kt * 64 + nb * 16 + 4 * g + j;
            if (!(kj < T && (!CAUSAL || kj <= qi))) sc[rb][nb][j] = -INFINITY;
          }
      }
      float tmax = sc[rb][0][0];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j) tmax = fmaxf(tmax, sc[rb][nb][j]);
      tmax = cross_rows_reduce<true>(tmax);
      const float mnew = fmaxf(mrow[rb], tmax * L2E);
      const float muse = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(mrow[rb] - muse);
      mrow[rb] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[rb][nb][j], L2E, -muse));
          sc[rb][nb][j] = p;
          rs += p;
        }
      rs = cross_rows_reduce<false>(rs);
      lrow[rb] = lrow[rb] * alpha + rs;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j) o[rb][nb][j] *= alpha;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const f32x4 lo = sc[rb][2 * kk], hi = sc[rb][2 * kk + 1];
        pb[rb][kk] = u32x4{pack2<BF>(lo[0], lo[1]), pack2<BF>(lo[2], lo[3]),
                           pack2<BF>(hi[0], hi[1]), pack2<BF>(hi[2], hi[3])};
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const u32x4 va = v_frag_trT(sV, kk * 32, nb, lane);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) o[rb][nb] = mfma16<BF>(va, pb[rb][kk], o[rb][nb]);
      }
    }
    // publish tile kt+1 (loaded during this tile) into the other buffer -- every wave finished
    // reading that buffer (tile kt-1) before the previous barrier -- and start loading kt+2
    if (kt + 1 < nkt) {
      stage((kt + 1) & 1);
      if (kt + 2 < nkt) load(kt + 2);
    }
    __syncthreads();
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int qi = qw + rb * 16 + (lane & 15);
    if (qi >= T) continue;
    const float inv = 1.0f / lrow[rb];
    u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + 4 * g;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      *(u32x2*)(op + nb * 16) = u32x2{pack2<BF>(o[rb][nb][0] * inv, o[rb][nb][1] * inv),
                                      pack2<BF>(o[rb][nb][2] * inv, o[rb][nb][3] * inv)};
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool BF>
__device__ __forceinline__ f32x16 mfma32(const u32x4& a, const u32x4& b, f32x16 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

// max / sum of v over lanes l and l ^ 32 (v_permlane32_swap: a VALU exchange, no LDS round trip;
// with both operands v the two results are v's lower and upper halves, each broadcast)
__device__ __forceinline__ float pair32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// V^T operand (32 dims x 16 keys) of a 32x32x16 PV MFMA, from the row-major swizzled V tile.
// Lane l (hi = l >> 5) holds dim dim0 + (l & 31) and logical k = 8 hi + t, t = 0..7, standing for
// key k16 + 4 hi + t (t < 4) or k16 + 8 + 4 hi + (t - 4): the order in which the 32x32 S^T
// accumulator leaves P in the lane (C row 8 (r >> 2) + 4 hi + (r & 3)), so P feeds the MFMA
// straight from registers. Two ds_read_b64_tr_b16, each 16-lane group reading 4 key rows x 16 dims.
__device__ __forceinline__ u32x4 v_frag32(const uint8_t* tile, int k16, int dim0, int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hi = gg >> 1, dh = gg & 1;
  const int chunk = (dim0 >> 3) + 2 * dh + (p >> 1);
  const int ka = k16 + 4 * hi + q, kb = ka + 8;
  const uint8_t* pa = tile + ka * 128 + ((chunk ^ ((ka >> 1) & 7)) << 4) + (p & 1) * 8;
  const uint8_t* pb = tile + kb * 128 + ((chunk ^ ((kb >> 1) & 7)) << 4) + (p & 1) * 8;
  const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  const u32x2 a = __builtin_bit_cast(u32x2, ra), b = __builtin_bit_cast(u32x2, rb);
  return u32x4{a.x, a.y, b.x, b.y};
}

// T > 128, non-causal (ViT-L/14@336: T = 577) on 32x32x16 MFMAs. One workgroup = 4 waves x 32
// queries of one (batch, head); the workgroups of a (batch, head) are consecutive on one XCD
// (xcd_remap), so its K / V rows are fetched into that XCD's L2 once. Per 64-key tile:
//   S^T = K Q^T as 2 key blocks of 32: lane l holds query (l & 31) and 32 of the tile's keys, the
//     other 32 in lane l ^ 32 -> row max = in-lane v_max3 chain + one v_permlane32_swap;
//   online softmax in the log2 domain; O and the running sum are rescaled only when some row's
//     max grew (wave vote; exp2(0) = 1 otherwise, so skipping is exact); row sums stay per lane
//     until the end;
//   O^T += V^T P^T: P packed from the accumulators is the B operand as it lies (v_frag32 reads V
//     in the matching key order).
// K / V tiles double-buffered in LDS, the next tile loaded into registers during this one's
// MFMAs (one barrier per tile). Waves whose 32 queries all lie past T only stage tiles.
// SUB32: each 32-key half of the tile is its own online-softmax step (16 scores per lane live
// instead of 32, so the kernel fits 128 VGPRs = 4 waves per SIMD; a half past T is skipped)
template <bool BF, bool SUB32>
__global__ __launch_bounds__(256, SUB32 ? 4 : 2) void attn_long_kernel(const u16* qkv, int64_t ldq, u16* out,
                                                                       int64_t ldo, int T, int d, int H, int nqb) {
  constexpr float L2E = 1.4426950408889634f;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 16384];
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int qb = wg % nqb, bh = wg / nqb, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, hi = lane >> 5;
  const u16* base = qkv + (int64_t)b * T * ldq;
  const int qw = qb * 128 + wid * 32;   // first query of this wave
  const bool active = qw < T;
  const int qi = qw + (lane & 31);

  u32x4 qf[4];   // Q^T operand: query qi, dims 16 s + 8 hi + 0..7
  {
    const u16* qp = base + (int64_t)min(qi, T - 1) * ldq + h * 64 + 8 * hi;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *(const u32x4*)(qp + 16 * s);
  }
  f32x16 o[2];   // O^T: query qi, dims db * 32 + 8 (r >> 2) + 4 hi + (r & 3)
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -INFINITY, l = 0.f;   // running max (log2 domain, shared by lanes l, l^32); lane-partial sum

  const int nkt = (T + 63) / 64;
  u32x4 kr[2], vr[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = tid + 256 * i, key = ci >> 3, c = ci & 7, kg = kt * 64 + key;
      kr[i] = u32x4{0u, 0u, 0u, 0u};
      vr[i] = u32x4{0u, 0u, 0u, 0u};
      if (kg < T) {
        const u16* rp = base + (int64_t)kg * ldq + h * 64 + c * 8;
        kr[i] = *(const u32x4*)(rp + d);
        vr[i] = *(const u32x4*)(rp + 2 * d);
      }
    }
  };
  auto stage = [&](int buf) {
    uint8_t* sK = smem + buf * 16384;
    uint8_t* sV = sK + 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = tid + 256 * i, key = ci >> 3, c = ci & 7;
      *(u32x4*)(sK + key * 128 + swz(key, c) * 16) = kr[i];
      *(u32x4*)(sV + key * 128 + swz(key, c) * 16) = vr[i];
    }
  };
  load(0);
  stage(0);
  if (nkt > 1) load(1);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    if (SUB32 && active) {
      const uint8_t* sK = smem + (kt & 1) * 16384;
      const uint8_t* sV = sK + 8192;
      const int kleft = T - kt * 64;   // valid keys in this tile (>= 1)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if (kb * 32 >= kleft) break;   // wave-uniform
        f32x16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
        const int krow = kb * 32 + (lane & 31);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const u32x4 kf = *(const u32x4*)(sK + krow * 128 + swz(krow, 2 * s + hi) * 16);
          sc = mfma32<BF>(kf, qf[s], sc);
        }
        if (kleft < kb * 32 + 32) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kb * 32 + 8 * (r >> 2) + 4 * hi + (r & 3) >= kleft) sc[r] = -INFINITY;
        }
        float tmax = sc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, sc[r]);
        tmax = pair32_max(tmax);
        const float mnew = fmaxf(m, tmax * L2E);   // finite: every processed half holds a valid key
        if (__any(mnew > m)) {
          const float alpha = __builtin_amdgcn_exp2f(m - mnew);
          l *= alpha;
#pragma unroll
          for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
          m = mnew;
        }
        u32x4 pf[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float p[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            p[t] = __builtin_amdgcn_exp2f(fmaf(sc[8 * hf + t], L2E, -m));
            l += p[t];
          }
          pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int db = 0; db < 2; ++db) o[db] = mfma32<BF>(v_frag32(sV, kb * 32 + 16 * hf, db * 32, lane), pf[hf], o[db]);
      }
    }
    if (!SUB32 && active) {
      const uint8_t* sK = smem + (kt & 1) * 16384;
      const uint8_t* sV = sK + 8192;
      const int kleft = T - kt * 64;   // valid keys in this tile (>= 1)
      f32x16 sc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
        const int krow = kb * 32 + (lane & 31);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const u32x4 kf = *(const u32x4*)(sK + krow * 128 + swz(krow, 2 * s + hi) * 16);
          sc[kb] = mfma32<BF>(kf, qf[s], sc[kb]);
        }
      }
      if (kleft < 64) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kb * 32 + 8 * (r >> 2) + 4 * hi + (r & 3) >= kleft) sc[kb][r] = -INFINITY;
      }
      float tmax = sc[0][0];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[kb][r]);
      tmax = pair32_max(tmax);
      const float mnew = fmaxf(m, tmax * L2E);   // finite: every tile holds a valid key
      if (__any(mnew > m)) {
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);   // 0 on the first tile, 1 where no growth
        l *= alpha;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
        m = mnew;
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        u32x4 pf[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float p[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            p[t] = __builtin_amdgcn_exp2f(fmaf(sc[kb][8 * hf + t], L2E, -m));
            l += p[t];
          }
          pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int db = 0; db < 2; ++db) o[db] = mfma32<BF>(v_frag32(sV, kb * 32 + 16 * hf, db * 32, lane), pf[hf], o[db]);
      }
    }
    if (kt + 1 < nkt) {
      stage((kt + 1) & 1);
      if (kt + 2 < nkt) load(kt + 2);
    }
    __syncthreads();
  }
  if (!active) return;
  l = pair32_sum(l);
  if (qi >= T) return;
  const float inv = 1.0f / l;
  u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + 4 * hi;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(u32x2*)(op + db * 32 + 8 * g) = u32x2{pack2<BF>(o[db][4 * g] * inv, o[db][4 * g + 1] * inv),
                                              pack2<BF>(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
}

// V^T operand as v_frag32, from a V tile whose 16-B chunks are XOR-swizzled by
// ((key >> 1) & 1) << 2 instead of K's (key >> 1) & 7: a ds_read_b64_tr_b16 bank group (32 lanes)
// covers 4 consecutive key rows x 4 chunks, and this swizzle puts rows k and k + 2 in opposite
// 64-B halves of the 128-B row, so the 32 lanes hit 32 distinct 8-B bank slots (K's swizzle maps
// rows k and k + 2 onto the same four chunks: a 2-way conflict on every V read).
__device__ __forceinline__ int swz_v(int row, int chunk) { return chunk ^ (((row >> 1) & 1) << 2); }
__device__ __forceinline__ u32x4 v_frag32v(const uint8_t* tile, int k16, int dim0, int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hi = gg >> 1, dh = gg & 1;
  const int chunk = (dim0 >> 3) + 2 * dh + (p >> 1);
  const int ka = k16 + 4 * hi + q, kb = ka + 8;
  const uint8_t* pa = tile + ka * 128 + (swz_v(ka, chunk) << 4) + (p & 1) * 8;
  const uint8_t* pb = tile + kb * 128 + (swz_v(kb, chunk) << 4) + (p & 1) * 8;
  // inline asm, not the builtin: with global_load_lds DMAs in flight the compiler puts an
  // s_waitcnt vmcnt(0) before every builtin transposed read (it cannot tell the DMA's buffer from
  // this one), which would stall each tile on the next tile's DMA. The caller waits on lgkmcnt
  // (lds_wait) before using the fragment.
  const uint32_t la = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)pa);
  const uint32_t lb = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const uint8_t*)pb);
  u32x2 a, b;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(a) : "v"(la));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(b) : "v"(lb));
  return u32x4{a.x, a.y, b.x, b.y};
}
// every LDS read issued so far has landed; the fragments are tied to the wait so that no use of
// them is scheduled above it
__device__ __forceinline__ void lds_wait(u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b));
}

// T > 128, non-causal (ViT-L/14@336: T = 577), the default form. Same work split and MFMA shapes
// as attn_long_kernel<BF, true> (4 waves x 32 queries of one (batch, head); 32-key online-softmax
// steps on 32x32x16 MFMAs, S^T = K Q^T so a lane owns one query), rebuilt around its measured
// bound -- vector-instruction issue (profiles/r05_v4_attn_pmc_summary.json: 2,459 VALU
// instructions per wave, VALU active 21 % of every one of 4 waves per SIMD, MFMA busy 31 %):
//   * K / V tiles stream HBM/L2 -> LDS by global_load_lds_dwordx4 (no register staging, no
//     ds_write, no zero fill): each wave issues 2 K + 2 V pieces of 8 rows x 128 B per 64-key tile,
//     rows past T clamped to T - 1 (their scores are masked to -inf, so P = 0 multiplies finite
//     V rows); double-buffered, the DMA of tile kt + 1 issued right after the barrier that opens
//     tile kt (every wave is then done with its buffer): one barrier per tile;
//   * lazy max: P = exp2(S log2e - m) against the running max m as it stands, and the lane's sum of
//     its 16 probabilities checked instead of a max over the scores. Only when some lane's sum
//     exceeds 2^15 (a score more than ~11 log2-units above m, or m still -inf on the first step:
//     the sum is then inf / NaN) does the wave take the exact rescale path (max over scores,
//     v_permlane32_swap, O and the sum scaled by exp2(m - m_new), P recomputed). The fast path thus
//     drops the 11-instruction max chain, the cross-lane swap and the vote on m per 32 keys; every
//     P stays <= 2^15 (fp16-safe) and O / l is unchanged in exact arithmetic (a common factor);
//   * V swizzled by swz_v (conflict-free transposed reads; K keeps swz for its ds_read_b128).
template <bool BF>
__global__ __launch_bounds__(256, 4) void attn_long_dma_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                               int T, int d, int H, int nqb) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr float RS_MAX = 32768.f;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 16384];
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int qb = wg % nqb, bh = wg / nqb, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, lane = tid & 63, hi = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u16* base = qkv + (int64_t)b * T * ldq + h * 64;
  const int qw = qb * 128 + wid * 32;   // first query of this wave
  const bool active = qw < T;
  const int qi = qw + (lane & 31);

  // this lane's DMA slots: piece j of the wave covers tile rows (2 wid + j) * 8 .. + 7; lane ->
  // row + (lane >> 3), LDS chunk position lane & 7, which holds the global chunk swz^-1 of it
  const int r8 = lane >> 3, pc = lane & 7;
  int kc[2], vc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (2 * wid + j) * 8 + r8;
    kc[j] = d + swz(row, pc) * 8;
    vc[j] = 2 * d + swz_v(row, pc) * 8;
  }
  auto issue = [&](int kt, int buf) {
    uint8_t* sK = smem + buf * 16384;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kg = min(kt * 64 + (2 * wid + j) * 8 + r8, T - 1);
      const u16* rp = base + (int64_t)kg * ldq;
      __builtin_amdgcn_global_load_lds((const void*)(rp + kc[j]), (void*)(sK + (2 * wid + j) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(rp + vc[j]), (void*)(sK + 8192 + (2 * wid + j) * 1024), 16, 0,
                                       0);
    }
  };

  u32x4 qf[4];   // Q^T operand: query qi, dims 16 s + 8 hi + 0..7
  {
    const u16* qp = base + (int64_t)min(qi, T - 1) * ldq + 8 * hi;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *(const u32x4*)(qp + 16 * s);
  }
  f32x16 o[2];   // O^T: query qi, dims db * 32 + 8 (r >> 2) + 4 hi + (r & 3)
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -INFINITY, l = 0.f;   // running shift (log2 domain, equal in lanes l, l ^ 32); lane-partial sum

  const int nkt = (T + 63) / 64;
  issue(0, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    // this wave's pieces of tile kt landed; then every wave's, and every wave is done with tile
    // kt - 1's buffer
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 1 < nkt) issue(kt + 1, (kt + 1) & 1);
    if (!active) continue;
    const uint8_t* sK = smem + (kt & 1) * 16384;
    const uint8_t* sV = sK + 8192;
    const int kleft = T - kt * 64;   // valid keys in this tile (>= 1)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (kb * 32 >= kleft) break;   // wave-uniform
      f32x16 sc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = 0.f;
      const int krow = kb * 32 + (lane & 31);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const u32x4 kf = *(const u32x4*)(sK + krow * 128 + swz(krow, 2 * s + hi) * 16);
        sc = mfma32<BF>(kf, qf[s], sc);
      }
      if (kleft < kb * 32 + 32) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kb * 32 + 8 * (r >> 2) + 4 * hi + (r & 3) >= kleft) sc[r] = -INFINITY;
      }
      u32x4 pf[2];
      float rs = 0.f;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float p[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          p[t] = __builtin_amdgcn_exp2f(fmaf(sc[8 * hf + t], L2E, -m));
          rs += p[t];
        }
        pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
      }
      if (__any(!(rs <= RS_MAX))) {   // rare: rescale to the exact running max, recompute P
        float tmax = sc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, sc[r]);
        tmax = pair32_max(tmax);
        const float mnew = fmaxf(m, tmax * L2E);   // finite: every processed half holds a valid key
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
        m = mnew;
        rs = 0.f;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float p[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            p[t] = __builtin_amdgcn_exp2f(fmaf(sc[8 * hf + t], L2E, -m));
            rs += p[t];
          }
          pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
        }
      }
      l += rs;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        u32x4 v0 = v_frag32v(sV, kb * 32 + 16 * hf, 0, lane), v1 = v_frag32v(sV, kb * 32 + 16 * hf, 32, lane);
        lds_wait(v0, v1);
        o[0] = mfma32<BF>(v0, pf[hf], o[0]);
        o[1] = mfma32<BF>(v1, pf[hf], o[1]);
      }
    }
  }
  if (!active) return;
  l = pair32_sum(l);
  if (qi >= T) return;
  const float inv = 1.0f / l;
  u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + 4 * hi;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(u32x2*)(op + db * 32 + 8 * g) = u32x2{pack2<BF>(o[db][4 * g] * inv, o[db][4 * g + 1] * inv),
                                              pack2<BF>(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
}

// T <= 128 (ViT-B/32: vision T = 50, text T = 77 causal): one workgroup per (head, batch),
// ceil(T/16) waves x 16 queries; all key tiles (<= 2 x 64) of K and V staged once. Scores are
// transposed as in attn_kernel (lane = one query, 16 keys per tile), and since every key is
// resident the softmax is a single exact pass over <= 32 in-lane values: no online rescale,
// P straight from registers into O^T = V^T P^T.
// NT = key tiles held (1 for T <= 64: 16 KB of LDS per workgroup instead of 32, so twice as
// many workgroups -- and their global loads -- are in flight per CU)
template <bool BF, bool CAUSAL, int NT>
__global__ __launch_bounds__(512) void attn_small_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                         int T, int d) {
  constexpr float L2E = 1.4426950408889634f;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NT * 8192 * 2];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4;
  const int nthr = blockDim.x;
  uint8_t* sK = smem;                     // [NT tiles][64 keys][128 B] swizzled
  uint8_t* sV = smem + NT * 8192;         // [NT tiles][64 keys][128 B] swizzled, like sK
  const u16* base = qkv + (int64_t)b * T * ldq;
  const int ntiles = (T + 63) / 64;
  for (int ci = tid; ci < ntiles * 512; ci += nthr) {
    const int key = ci >> 3, c = ci & 7;
    u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = u32x4{0u, 0u, 0u, 0u};
    if (key < T) {
      const u16* rp = base + (int64_t)key * ldq + h * 64 + c * 8;
      kv = *(const u32x4*)(rp + d);
      vv = *(const u32x4*)(rp + 2 * d);
    }
    const int kt = key >> 6, kr = key & 63;
    *(u32x4*)(sK + kt * 8192 + kr * 128 + swz(kr, c) * 16) = kv;
    *(u32x4*)(sV + kt * 8192 + kr * 128 + swz(kr, c) * 16) = vv;
  }
  const int q0 = wid * 16, qi = q0 + (lane & 15);
  u32x4 qa[2];
  {
    const u16* qp = base + (int64_t)min(qi, T - 1) * ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qa[kk] = *(const u32x4*)(qp + kk * 32 + 8 * g);
  }
  __syncthreads();
  const int nkt = CAUSAL ? min((q0 + 15) / 64 + 1, ntiles) : ntiles;
  f32x4 sc[NT][4];   // S^T: lane holds query qi, keys kt*64 + nb*16 + 4g + 0..3
  float tmax = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    if (kt >= nkt) break;
    const uint8_t* tK = sK + kt * 8192;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      sc[kt][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = nb * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + g;
        sc[kt][nb] = mfma16<BF>(*(const u32x4*)(tK + krow * 128 + swz(krow, c) * 16), qa[kk], sc[kt][nb]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = kt * 64 + nb * 16 + 4 * g + j;
        if (!(kj < T && (!CAUSAL || kj <= qi))) sc[kt][nb][j] = -INFINITY;
        tmax = fmaxf(tmax, sc[kt][nb][j]);
      }
    }
  }
  tmax = cross_rows_reduce<true>(tmax);
  const float m2 = tmax * L2E;   // key 0 is always visible: finite
  float rs = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    if (kt >= nkt) break;
    u32x4 pb[2];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[kt][nb][j], L2E, -m2));
        sc[kt][nb][j] = p;
        rs += p;
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const f32x4 lo = sc[kt][2 * kk], hi = sc[kt][2 * kk + 1];
      pb[kk] = u32x4{pack2<BF>(lo[0], lo[1]), pack2<BF>(lo[2], lo[3]), pack2<BF>(hi[0], hi[1]),
                     pack2<BF>(hi[2], hi[3])};
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb] = mfma16<BF>(v_frag_trT(sV + kt * 8192, kk * 32, nb, lane), pb[kk], o[nb]);
  }
  rs = cross_rows_reduce<false>(rs);
  if (qi >= T) return;
  const float inv = 1.0f / rs;
  u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + 4 * g;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    *(u32x2*)(op + nb * 16) = u32x2{pack2<BF>(o[nb][0] * inv, o[nb][1] * inv), pack2<BF>(o[nb][2] * inv, o[nb][3] * inv)};
}
}  // namespace

hipError_t attention(bool bf16, bool causal, const u16* qkv, int64_t ldq, u16* out, int64_t ldo, int B, int T,
                     int H, int d, hipStream_t s) {
  if (B <= 0 || T <= 0) return hipSuccess;
  if (d != H * 64 || (ldq % 8) || (ldo % 8)) return hipErrorInvalidValue;
  if (T <= 128) {
    dim3 g2(H, B), b2(64 * ((T + 15) / 16));
    // NT = 1 for T <= 64 measured no faster in the pipeline (0.46-0.48 ms of attention per step
    // either way, pairs/s 0.7 % lower: profiles/r02_v4_attn_ab.txt), so both sizes hold 2 tiles
    const bool one = false;
#define CLM_SMALL(BFV, CV)                                                                    \
    (one ? (attn_small_kernel<BFV, CV, 1><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d), 0)     \
         : (attn_small_kernel<BFV, CV, 2><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d), 0))
    if (bf16) {
      if (causal) CLM_SMALL(true, true); else CLM_SMALL(true, false);
    } else {
      if (causal) CLM_SMALL(false, true); else CLM_SMALL(false, false);
    }
#undef CLM_SMALL
    return hipGetLastError();
  }
  // $CLM_ATTN_LONG: 0 = the 16x16x32 attn_kernel, 1 = attn_long_kernel with 64-key softmax
  // steps, 2 = its SUB32 form (L/14: 6.53 vs 6.91 ms per step, profiles/r02_v4_attn_ab.txt),
  // 3 (default) = attn_long_dma_kernel
  static const int long_mode = getenv("CLM_ATTN_LONG") ? atoi(getenv("CLM_ATTN_LONG")) : 3;
  if (!causal && long_mode) {
    const int nqb = (T + 127) / 128;
    const int64_t nwg = (int64_t)nqb * H * B;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    if (long_mode == 3) {
      if (bf16) attn_long_dma_kernel<true><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
      else attn_long_dma_kernel<false><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
    } else if (long_mode == 2) {
      if (bf16) attn_long_kernel<true, true><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
      else attn_long_kernel<false, true><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
    } else {
      if (bf16) attn_long_kernel<true, false><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
      else attn_long_kernel<false, false><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
    }
    return hipGetLastError();
  }
  dim3 grid((T + 127) / 128, H, B), block(256);
  if (bf16) {
    if (causal) attn_kernel<true, true><<<grid, block, 0, s>>>(qkv, ldq, out, ldo, T, d);
    else attn_kernel<true, false><<<grid, block, 0, s>>>(qkv, ldq, out, ldo, T, d);
  } else {
    if (causal) attn_kernel<false, true><<<grid, block, 0, s>>>(qkv, ldq, out, ldo, T, d);
    else attn_kernel<false, false><<<grid, block, 0, s>>>(qkv, ldq, out, ldo, T, d);
  }
  return hipGetLastError();
}

}  // namespace clm
