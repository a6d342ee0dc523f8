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
typedef __attribute__((address_space(3))) void* lds_ptr_t;

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

// this lane's V^T read address (LDS bytes, tile at tile0) for dims db * 32 .., key rows 4 hi + q:
// lane l (hi = l >> 5) reads dim db * 32 + (l & 31)'s keys in the order the S^T accumulator holds P.
// The swizzle term depends only on (q >> 1) & 1, so each key block k16 (and its +8 partner) is an
// immediate offset on this one address.
__device__ __forceinline__ uint32_t v_lane_base(uint32_t tile0, int db, int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hi = gg >> 1, dh = gg & 1;
  const int chunk = db * 4 + 2 * dh + (p >> 1);
  const int ka = 4 * hi + q;
  return tile0 + ka * 128 + (swz_v(ka, chunk) << 4) + (p & 1) * 8;
}
// V^T fragment (32 dims x 16 keys) at byte offset OFF from the lane's base: two
// ds_read_b64_tr_b16 (rows k16 + 4 hi + q and + 8). Inline asm, not the builtin: with LDS DMAs in
// flight the compiler puts an s_waitcnt vmcnt(0) before every builtin transposed read (it cannot
// tell the DMA's buffer from this one), which would stall each tile on the next tile's DMA; the
// caller waits on lgkmcnt (lds_wait) before using the fragment.
template <int OFF>
__device__ __forceinline__ u32x4 v_frag32v(uint32_t va) {
  u32x2 a, b;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(a) : "v"(va), "i"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(b) : "v"(va), "i"(OFF + 8 * 128));
  return u32x4{a.x, a.y, b.x, b.y};
}
// every LDS read issued so far has landed; the fragments are tied to the wait so that no use of
// them is scheduled above it
__device__ __forceinline__ void lds_wait(u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b));
}
template <int N> struct IC { static constexpr int value = N; };

// T > 128, non-causal (ViT-L/14@336: T = 577), the default form. Same work split and MFMA shapes
// as attn_long_kernel<BF, true> (4 waves x 32 queries of one (batch, head); 32-key online-softmax
// steps on 32x32x16 MFMAs, S^T = K Q^T so a lane owns one query), rebuilt around its measured
// bound -- vector-instruction issue (profiles/r05_v4_attn_pmc_summary.json: 2,459 VALU
// instructions per wave, VALU active 21 % of every one of 4 waves per SIMD, MFMA busy 31 %):
//   * K / V tiles stream HBM/L2 -> LDS by buffer_load ... lds (no register staging, no ds_write,
//     no zero fill, no per-tile address arithmetic): each wave issues 2 K + 2 V pieces of 8 rows x
//     128 B per 64-key tile from a per-tile buffer resource over the rows left, so rows past T
//     read as zeros (their scores are masked to -inf anyway); double-buffered, the DMA of tile
//     kt + 1 issued right after the barrier that opens tile kt (every wave is then done with its
//     buffer): one barrier per tile. The tile loop is unrolled by two so both buffers' LDS
//     offsets are immediates of the fragment reads;
//   * lazy max: P = exp2(S log2e - m) against the running max m as it stands, and the lane's sum of
//     its 16 probabilities checked instead of a max over the scores. Only when some lane's sum
//     exceeds 2^15 (a score more than ~11 log2-units above m, or m still -inf on the first step:
//     the sum is then inf / NaN) does the wave take the exact rescale path (max over scores,
//     v_permlane32_swap, O and the sum scaled by exp2(m - m_new), P recomputed). The fast path thus
//     drops the 11-instruction max chain, the cross-lane swap and the vote on m per 32 keys; every
//     P stays <= 2^15 (fp16-safe) and O / l is unchanged in exact arithmetic (a common factor);
//   * V swizzled by swz_v (conflict-free transposed reads; K keeps swz for its ds_read_b128).
// QL2E (bf16 only): q arrives pre-scaled by log2(e) as well (the engine folds it into the q_proj
// weights, attention_folds_log2e), so the scores are already in the log2 domain, and the running
// shift m -- kept as a bf16 value -- enters the score accumulator through a fifth MFMA of the QK
// chain (A = a column of ones, B = -m in k-slot 0): the fast path is then P = exp2(acc), without
// the 16 v_fma_f32 per 32 keys that apply log2 e and subtract m (one 32-cycle MFMA instead of 64
// cycles of vector issue).
template <bool BF, bool QL2E>
__global__ __launch_bounds__(256, 4) void attn_long_dma_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                               int T, int d, int H, int nqb) {
  static_assert(BF || !QL2E, "the folded form keeps the shift in bf16");
  constexpr float L2E = QL2E ? 1.0f : 1.4426950408889634f;
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
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)smem);

  // this lane's DMA byte offsets: piece j of the wave covers tile rows (2 wid + j) * 8 .. + 7;
  // lane -> row + (lane >> 3), LDS chunk position lane & 7, which holds the global chunk that the
  // swizzle maps there
  const int r8 = lane >> 3, pc = lane & 7;
  const uint32_t ldq2 = (uint32_t)ldq * 2;
  uint32_t ko[2], vo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (2 * wid + j) * 8 + r8;
    ko[j] = row * ldq2 + (uint32_t)(d + swz(row, pc) * 8) * 2;
    vo[j] = row * ldq2 + (uint32_t)(2 * d + swz_v(row, pc) * 8) * 2;
  }
  auto issue = [&](int kt, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const auto rs = buf_rsrc(base + (int64_t)kt * 64 * ldq, (T - kt * 64) * (int)ldq2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + BUF * 16384 + (2 * wid + j) * 1024), 16, ko[j], 0,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + BUF * 16384 + 8192 + (2 * wid + j) * 1024), 16,
                                               vo[j], 0, 0, 0);
    }
  };

  u32x4 qf[4];   // Q^T operand: query qi, dims 16 s + 8 hi + 0..7
  {
    const u16* qp = base + (int64_t)min(qi, T - 1) * ldq + 8 * hi;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *(const u32x4*)(qp + 16 * s);
  }
  // K fragment rows: key kb * 32 + (lane & 31), chunk 2 s + hi (the kb / buffer parts are immediates)
  uint32_t kaddr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) kaddr[s] = (lane & 31) * 128 + swz(lane & 31, 2 * s + hi) * 16;
  const uint32_t va0 = v_lane_base(lds0, 0, lane), va1 = v_lane_base(lds0, 1, lane);

  f32x16 o[2];   // O^T: query qi, dims db * 32 + 8 (r >> 2) + 4 hi + (r & 3)
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = QL2E ? 0.f : -INFINITY;   // running shift (log2 domain, equal in lanes l, l ^ 32)
  float l = 0.f;                      // lane-partial sum
  // QL2E: the shift's MFMA operands (k-slot 0 of lanes 0..31; every other slot zero)
  const u32x4 ones = u32x4{hi ? 0u : 0x3F80u, 0u, 0u, 0u};
  u32x4 negm = u32x4{0u, 0u, 0u, 0u};

  // S^T of keys KB * 32 .. of the tile in buffer BUF (QL2E: minus the shift as it stands)
  auto qk = [&](auto bufc, auto kbc, f32x16& sc) {
    constexpr int BUF = decltype(bufc)::value, KB = decltype(kbc)::value;
    constexpr int KOFF = BUF * 16384 + KB * 4096;
    u32x4 kf[4];   // all four K fragments in flight before the first QK MFMA
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[s] = *(const u32x4*)(smem + KOFF + kaddr[s]);
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = 0.f;
    if constexpr (QL2E) sc = mfma32<BF>(ones, negm, sc);   // sc = -m
#pragma unroll
    for (int s = 0; s < 4; ++s) sc = mfma32<BF>(kf[s], qf[s], sc);
  };
  // keys past T (kleft valid keys in the tile): register r holds key KB*32 + 8(r>>2) + 4hi + (r&3)
  auto mask = [&](f32x16& sc, int kleft, int KB) {
    const int lim = kleft - KB * 32 - 4 * hi;   // one lane value against immediates
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (8 * (r >> 2) + (r & 3) >= lim) sc[r] = -INFINITY;
  };
  // P (packed for the PV MFMA) and the lane's sum of one 32-key step; the rare exact rescale
  // (QL2E: always on the first step, m = 0 being no running max)
  auto softmax = [&](const f32x16& sc, bool first, u32x4 (&pf)[2]) -> float {
    float rs = 0.f;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float p[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        p[t] = __builtin_amdgcn_exp2f(QL2E ? sc[8 * hf + t] : fmaf(sc[8 * hf + t], L2E, -m));
        rs += p[t];
      }
      pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
    }
    if ((QL2E && first) || __any(!(rs <= RS_MAX))) {
      float tmax = sc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, sc[r]);
      tmax = pair32_max(tmax);   // finite: every processed step holds a valid key
      float dm;                  // the shift's growth; sc is relative to the old shift (QL2E)
      if constexpr (QL2E) {
        // the new shift, rounded to bf16 (it re-enters the MFMA as a bf16 operand); the
        // difference of two bf16 values is exact in fp32
        const uint32_t mb = pack2<true>(m + (first ? tmax : fmaxf(tmax, 0.f)), 0.f) & 0xFFFFu;
        const float mnew = __uint_as_float(mb << 16);
        dm = mnew - m;
        m = mnew;
        negm = u32x4{hi ? 0u : (mb ^ 0x8000u), 0u, 0u, 0u};
      } else {
        const float mnew = fmaxf(m, tmax * L2E);
        dm = mnew - m;   // +inf on the first step: alpha = 0 scales the zero O and sum
        m = mnew;
      }
      // QL2E's first step: O and the sum are still zero, and dm = m_new can be below -128 (every
      // logit of the first 32 keys under about -88.7), where exp2(-dm) is +inf and 0 * inf NaN
      const float alpha = (QL2E && first) ? 0.f : __builtin_amdgcn_exp2f(-dm);
      l *= alpha;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
      rs = 0.f;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float p[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          p[t] = __builtin_amdgcn_exp2f(QL2E ? sc[8 * hf + t] - dm : fmaf(sc[8 * hf + t], L2E, -m));
          rs += p[t];
        }
        pf[hf] = u32x4{pack2<BF>(p[0], p[1]), pack2<BF>(p[2], p[3]), pack2<BF>(p[4], p[5]), pack2<BF>(p[6], p[7])};
      }
    }
    return rs;
  };
  // O^T += V^T P^T for keys KB * 32 .. of the tile in buffer BUF
  auto pv = [&](auto bufc, auto kbc, const u32x4 (&pf)[2]) {
    constexpr int BUF = decltype(bufc)::value, KB = decltype(kbc)::value;
    constexpr int VOFF = BUF * 16384 + 8192 + KB * 32 * 128;
    {
      u32x4 v0 = v_frag32v<VOFF>(va0), v1 = v_frag32v<VOFF>(va1);
      lds_wait(v0, v1);
      o[0] = mfma32<BF>(v0, pf[0], o[0]);
      o[1] = mfma32<BF>(v1, pf[0], o[1]);
    }
    {
      u32x4 v0 = v_frag32v<VOFF + 16 * 128>(va0), v1 = v_frag32v<VOFF + 16 * 128>(va1);
      lds_wait(v0, v1);
      o[0] = mfma32<BF>(v0, pf[1], o[0]);
      o[1] = mfma32<BF>(v1, pf[1], o[1]);
    }
  };
  const int nkt = (T + 63) / 64;
  // one 64-key tile: two 32-key steps. (Software-pipelined -- both QK chains first, the second
  // under the first step's softmax -- needs 160 VGPRs, i.e. 3 waves per SIMD: 6.03 vs 5.31 ms of
  // L/14 attention per step, profiles/r05_v6_attn_ab.txt.)
  auto tile = [&](int kt, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    // this wave's pieces of tile kt landed; then every wave's, and every wave is done with tile
    // kt - 1's buffer
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 1 < nkt) issue(kt + 1, IC<1 - BUF>{});
    if (!active) return;
    const int kleft = T - kt * 64;   // valid keys in this tile (>= 1)
    f32x16 sc;
    u32x4 pf[2];
    qk(bufc, IC<0>{}, sc);
    if (kleft < 32) mask(sc, kleft, 0);
    l += softmax(sc, kt == 0, pf);
    pv(bufc, IC<0>{}, pf);
    if (kleft > 32) {
      qk(bufc, IC<1>{}, sc);
      if (kleft < 64) mask(sc, kleft, 1);
      l += softmax(sc, false, pf);
      pv(bufc, IC<1>{}, pf);
    }
  };
  issue(0, IC<0>{});
  for (int kt = 0; kt < nkt; kt += 2) {
    tile(kt, IC<0>{});
    if (kt + 1 < nkt) tile(kt + 1, IC<1>{});
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
// $CLM_ATTN_LONG (T > 128, non-causal): 0 = the 16x16x32 attn_kernel, 1 = attn_long_kernel with
// 64-key softmax steps, 2 = its SUB32 form (L/14: 6.53 vs 6.91 ms per step,
// profiles/r02_v4_attn_ab.txt), 3 (default) = attn_long_dma_kernel
int attn_long_mode() {
  static const int m = getenv("CLM_ATTN_LONG") ? atoi(getenv("CLM_ATTN_LONG")) : 3;
  return m;
}
}  // namespace

// attn_long_dma_kernel's per-tile buffer resources take 32-bit byte offsets over a sequence's
// rows: sequences up to 65,535 tokens (rows of <= 3 x 1024 16-bit values: < 2^31 bytes)
constexpr int ATTN_DMA_MAX_T = 65535;

bool attention_folds_log2e(bool bf16, bool causal, int T) {
  return bf16 && !causal && T > 128 && T <= ATTN_DMA_MAX_T && attn_long_mode() == 3;
}

hipError_t attention(bool bf16, bool causal, const u16* qkv, int64_t ldq, u16* out, int64_t ldo, int B, int T,
                     int H, int d, hipStream_t s, bool q_log2e) {
  if (d != H * 64 || (ldq % 8) || (ldo % 8)) return hipErrorInvalidValue;
  if (q_log2e && !attention_folds_log2e(bf16, causal, T)) return hipErrorInvalidValue;
  if (B <= 0 || T <= 0) return hipSuccess;
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
  // longer sequences than the DMA kernel's offsets cover take the SUB32 register-staged kernel
  const int long_mode = (attn_long_mode() == 3 && (T > ATTN_DMA_MAX_T || (int64_t)T * ldq * 2 >= (1ll << 31)))
                            ? 2 : attn_long_mode();
  if (q_log2e && long_mode != 3) return hipErrorInvalidValue;   // only that kernel takes log2-domain q
  if (!causal && long_mode) {
    const int nqb = (T + 127) / 128;
    const int64_t nwg = (int64_t)nqb * H * B;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    if (long_mode == 3) {
      if (q_log2e) attn_long_dma_kernel<true, true><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
      else if (bf16) attn_long_dma_kernel<true, false><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
      else attn_long_dma_kernel<false, false><<<(unsigned)nwg, 256, 0, s>>>(qkv, ldq, out, ldo, T, d, H, nqb);
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
