// Multi-head attention for the CLIP towers on gfx950 MFMA.
//
// Replaces CLIPAttention's sdpa/eager core (TF/models/clip/modeling_clip.py:
// 259-277, 298-335): softmax(Q K^T * 64^-1/2 [+ causal mask]) V per (batch, head),
// head_dim 64, T = 50 (B/32 image), 77 (text, causal), 577 (L/14@336 image).
// The 64^-1/2 scale is folded into the q_proj weights at load (a power of two,
// so the product is bit-identical to scaling the scores).
//
// One workgroup = (64-row query block, head, batch); 4 waves x 16 query rows.
// Key tiles of 64: K and V staged in LDS row-major with the 128-B-row XOR swizzle (K read
// as ds_read_b128 B-fragments, V through ds_read_b64_tr_b16, see v_frag_tr); online softmax
// in fp32 with 16-lane group
// reductions on the MFMA C layout; P goes through a per-wave LDS tile to become
// the A operand of PV.
#include "kernels.hpp"

namespace clm {

namespace {

// PV B-operand (16x16x32: lane l holds V[key0 + (l>>4)*8 + 0..7][dim0 + (l&15)]) from a
// ROW-MAJOR V tile ([64 keys][128 B], 16-B chunks XOR-swizzled by (key>>1)&7 like K) with two
// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses key row q, dims 4p..4p+3, and lane
// i receives dim i of the 4 rows. V is then staged with one 16-B LDS write per chunk, instead
// of eight 8-way bank-conflicted 2-B writes into a transposed image.
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 v_frag_tr(const uint8_t* tile, int kbase, int nb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int chunk = nb * 2 + (p >> 1);
  const int ka = kbase + g * 8 + q, kb = ka + 4;
  const uint8_t* pa = tile + ka * 128 + ((chunk ^ ((ka >> 1) & 7)) << 4) + (p & 1) * 8;
  const uint8_t* pb = tile + kb * 128 + ((chunk ^ ((kb >> 1) & 7)) << 4) + (p & 1) * 8;
  const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  const u32x2 a = __builtin_bit_cast(u32x2, ra), b = __builtin_bit_cast(u32x2, rb);
  return u32x4{a.x, a.y, b.x, b.y};
}

template <bool BF, bool CAUSAL>
__global__ __launch_bounds__(256) void attn_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                   int T, int d) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[8192 + 8192 + 4 * 2048];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint8_t* sK = smem;
  uint8_t* sV = smem + 8192;   // [64 keys][128 B] swizzled, like sK
  uint8_t* sP = smem + 16384 + wid * 2048;
  const u16* base = qkv + (int64_t)b * T * ldq;
  const int q0 = qb * 64 + wid * 16;

  u32x4 qa[2];
  {
    const int r = min(q0 + (lane & 15), T - 1);
    const u16* qp = base + (int64_t)r * ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qa[kk] = *(const u32x4*)(qp + kk * 32 + 8 * (lane >> 4));
  }
  f32x4 o[4];
  float mrow[4], lrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = f32x4{0.f, 0.f, 0.f, 0.f}; mrow[j] = -INFINITY; lrow[j] = 0.f; }

  const int ntiles = (T + 63) / 64;
  const int nkt = CAUSAL ? min(qb + 1, ntiles) : ntiles;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ci = tid + 256 * i, key = ci >> 3, c = ci & 7;
      const int kg = kt * 64 + key;
      u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = u32x4{0u, 0u, 0u, 0u};
      if (kg < T) {
        const u16* rp = base + (int64_t)kg * ldq + h * 64 + c * 8;
        kv = *(const u32x4*)(rp + d);
        vv = *(const u32x4*)(rp + 2 * d);
      }
      *(u32x4*)(sK + key * 128 + swz(key, c) * 16) = kv;
      *(u32x4*)(sV + key * 128 + swz(key, c) * 16) = vv;
    }
    __syncthreads();

    f32x4 sc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      sc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = nb * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + (lane >> 4);
        const u32x4 kb = *(const u32x4*)(sK + krow * 128 + swz(krow, c) * 16);
        sc[nb] = mfma16<BF>(qa[kk], kb, sc[nb]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qi = q0 + (lane >> 4) * 4 + j;
      float tmax = -INFINITY;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int kj = kt * 64 + nb * 16 + (lane & 15);
        const bool ok = kj < T && (!CAUSAL || kj <= qi);
        const float v = ok ? sc[nb][j] : -INFINITY;
        sc[nb][j] = v;
        tmax = fmaxf(tmax, v);
      }
      tmax = group16_max(tmax);
      const float mnew = fmaxf(mrow[j], tmax);
      const float alpha = (mrow[j] == -INFINITY) ? 0.f : __expf(mrow[j] - mnew);
      mrow[j] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float p = __expf(sc[nb][j] - mnew);
        sc[nb][j] = p;
        rs += p;
      }
      rs = group16_sum(rs);
      lrow[j] = lrow[j] * alpha + rs;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb][j] *= alpha;
    }
    // P (C layout: row=(lane>>4)*4+j, key=nb*16+(lane&15)) -> per-wave LDS [16][64]
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (lane >> 4) * 4 + j, key = nb * 16 + (lane & 15);
        *(u16*)(sP + row * 128 + swz(row, key >> 3) * 16 + (key & 7) * 2) = from_f32<BF>(sc[nb][j]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row = lane & 15, c = kk * 4 + (lane >> 4);
      const u32x4 pa = *(const u32x4*)(sP + row * 128 + swz(row, c) * 16);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb] = mfma16<BF>(pa, v_frag_tr(sV, kk * 32, nb, lane), o[nb]);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qi = q0 + (lane >> 4) * 4 + j;
    if (qi >= T) continue;
    const float inv = 1.0f / lrow[j];
    u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + (lane & 15);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) op[nb * 16] = from_f32<BF>(o[nb][j] * inv);
  }
}
// T <= 128: one workgroup per (head, batch), ceil(T/16) waves x 16 query rows; all
// key tiles (<= 2 x 64) of K and V staged once.
template <bool BF, bool CAUSAL>
__global__ __launch_bounds__(512) void attn_small_kernel(const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                                                         int T, int d) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 8192 + 2 * 8192 + 8 * 2048];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nthr = blockDim.x;
  uint8_t* sK = smem;                     // [2 tiles][64 keys][128 B] swizzled
  uint8_t* sV = smem + 2 * 8192;          // [2 tiles][64 keys][128 B] swizzled, like sK
  uint8_t* sP = smem + 4 * 8192 + wid * 2048;
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
  const int q0 = wid * 16;
  u32x4 qa[2];
  {
    const int r = min(q0 + (lane & 15), T - 1);
    const u16* qp = base + (int64_t)r * ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qa[kk] = *(const u32x4*)(qp + kk * 32 + 8 * (lane >> 4));
  }
  __syncthreads();
  f32x4 o[4];
  float mrow[4], lrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = f32x4{0.f, 0.f, 0.f, 0.f}; mrow[j] = -INFINITY; lrow[j] = 0.f; }
  const int nkt = CAUSAL ? min((q0 + 15) / 64 + 1, ntiles) : ntiles;
  for (int kt = 0; kt < nkt; ++kt) {
    const uint8_t* tK = sK + kt * 8192;
    f32x4 sc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      sc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int krow = nb * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + (lane >> 4);
        sc[nb] = mfma16<BF>(qa[kk], *(const u32x4*)(tK + krow * 128 + swz(krow, c) * 16), sc[nb]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qi = q0 + (lane >> 4) * 4 + j;
      float tmax = -INFINITY;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int kj = kt * 64 + nb * 16 + (lane & 15);
        const bool ok = kj < T && (!CAUSAL || kj <= qi);
        const float v = ok ? sc[nb][j] : -INFINITY;
        sc[nb][j] = v;
        tmax = fmaxf(tmax, v);
      }
      tmax = group16_max(tmax);
      const float mnew = fmaxf(mrow[j], tmax);
      const float alpha = (mrow[j] == -INFINITY) ? 0.f : __expf(mrow[j] - mnew);
      mrow[j] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float p = __expf(sc[nb][j] - mnew);
        sc[nb][j] = p;
        rs += p;
      }
      rs = group16_sum(rs);
      lrow[j] = lrow[j] * alpha + rs;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb][j] *= alpha;
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (lane >> 4) * 4 + j, key = nb * 16 + (lane & 15);
        *(u16*)(sP + row * 128 + swz(row, key >> 3) * 16 + (key & 7) * 2) = from_f32<BF>(sc[nb][j]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row = lane & 15, c = kk * 4 + (lane >> 4);
      const u32x4 pa = *(const u32x4*)(sP + row * 128 + swz(row, c) * 16);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) o[nb] = mfma16<BF>(pa, v_frag_tr(sV + kt * 8192, kk * 32, nb, lane), o[nb]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // P reads done before next tile's P writes
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qi = q0 + (lane >> 4) * 4 + j;
    if (qi >= T) continue;
    const float inv = 1.0f / lrow[j];
    u16* op = out + ((int64_t)b * T + qi) * ldo + h * 64 + (lane & 15);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) op[nb * 16] = from_f32<BF>(o[nb][j] * inv);
  }
}
}  // namespace

hipError_t attention(bool bf16, bool causal, const u16* qkv, int64_t ldq, u16* out, int64_t ldo, int B, int T,
                     int H, int d, hipStream_t s) {
  if (B <= 0 || T <= 0) return hipSuccess;
  if (d != H * 64 || (ldq % 8) || (ldo % 8)) return hipErrorInvalidValue;
  if (T <= 128) {
    dim3 g2(H, B), b2(64 * ((T + 15) / 16));
    if (bf16) {
      if (causal) attn_small_kernel<true, true><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d);
      else attn_small_kernel<true, false><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d);
    } else {
      if (causal) attn_small_kernel<false, true><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d);
      else attn_small_kernel<false, false><<<g2, b2, 0, s>>>(qkv, ldq, out, ldo, T, d);
    }
    return hipGetLastError();
  }
  dim3 grid((T + 63) / 64, H, B), block(256);
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
