// Row-wise kernels of the encode path (gfx950): LayerNorm (+ fused text
// embedding gather, + fused LoRA down-projection), patchify with the
// CLIPProcessor rescale/normalise fused, CLS assembly, and the pooled-row
// LN -> projection -> L2-normalise tail.
//
// Reference arithmetic (TF = transformers/):
//   LayerNorm eps 1e-5             TF/models/clip/modeling_clip.py:358,360,605,607,504
//   text embeddings gather+add     modeling_clip.py:232-256
//   vision embeddings cls/pos      modeling_clip.py:202-218
//   rescale/normalize              TF/image_transforms.py rescale (f64 mul -> f32), normalize
//   pooled CLS / first-EOS row     modeling_clip.py:561-582, 650-651
//   projection + L2 norm           modeling_clip.py:712-713,750-751; models/clip_model.py:116,148
//   PEFT LoRA down-projection x.A^T (lora_A), models/clip_model.py:78
#include "kernels.hpp"

namespace clm {

namespace {

// ------------------------------------------------------------------ LN ------
// One wave per row; lane owns NP float2 pairs at e = (i*64 + lane)*2.
template <bool BF, int NP>
__global__ __launch_bounds__(256) void ln_kernel(LnArgs aa) {
  LnArgs a = aa;   // varlen: the device-resident row count (the grid was sized for aa.M)
  if (a.m_dev) a.M = __builtin_amdgcn_readfirstlane(*a.m_dev);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.M) return;
  const int d = NP * 128;
  float x[NP][2];
  if (a.mode == 0) {
    const float* src = a.src + (int64_t)row * a.lds;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const float2 v = *(const float2*)(src + (i * 64 + lane) * 2);
      x[i][0] = v.x; x[i][1] = v.y;
    }
  } else {
    const int src = a.rowmap ? a.rowmap[row] : row;   // packed row -> b * L + position
    const int tokid = a.ids[src];
    const float* tk = a.tok + (int64_t)tokid * d;
    const float* ps = a.pos + (int64_t)(src % a.L) * d;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int e = (i * 64 + lane) * 2;
      const float2 t = *(const float2*)(tk + e);
      const float2 p = *(const float2*)(ps + e);
      x[i][0] = t.x + p.x; x[i][1] = t.y + p.y;
    }
  }
  auto ln = [&](const float* g, const float* b) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) s += x[i][0] + x[i][1];
    const float mean = wave_sum(s) / d;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const float d0 = x[i][0] - mean, d1 = x[i][1] - mean;
      v += d0 * d0 + d1 * d1;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(v) / d + a.eps);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int e = (i * 64 + lane) * 2;
      const float2 gg = *(const float2*)(g + e);
      const float2 bb = *(const float2*)(b + e);
      x[i][0] = (x[i][0] - mean) * rstd * gg.x + bb.x;
      x[i][1] = (x[i][1] - mean) * rstd * gg.y + bb.y;
    }
  };
  auto store_h = [&]() {
    float* h = a.hf + (int64_t)row * a.ldh;
#pragma unroll
    for (int i = 0; i < NP; ++i) *(float2*)(h + (i * 64 + lane) * 2) = make_float2(x[i][0], x[i][1]);
  };
  if (a.g2) {
    ln(a.g1, a.b1);
    store_h();
    ln(a.g2, a.b2);
  } else {
    if (a.mode == 1) store_h();
    ln(a.g1, a.b1);
  }
  u16* y = a.y + (int64_t)row * a.ldy;
#pragma unroll
  for (int i = 0; i < NP; ++i) *(uint32_t*)(y + (i * 64 + lane) * 2) = pack2<BF>(x[i][0], x[i][1]);

}

// d % 256 == 0: lane owns NQ float4 at e = (i*64 + lane)*4 (16-B loads, 8-B bf16 stores: half
// the memory instructions of the float2 form above; HBM-bound).
template <bool BF, int NQ, int R = 2>
__device__ __forceinline__ void ln4_body(const LnArgs& aa, int bid) {
  LnArgs a = aa;   // varlen: the device-resident row count (the grid was sized for aa.M)
  if (a.m_dev) a.M = __builtin_amdgcn_readfirstlane(*a.m_dev);
  // R rows per wave (every row's loads issued before any is reduced; gamma / beta loaded
  // once per wave and reused); the 16-B paired store path below takes rows in pairs
  static_assert(R % 2 == 0, "rows per wave come in pairs");
  const int lane = threadIdx.x & 63;
  const int row0 = (bid * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= a.M) return;
  constexpr int d = NQ * 256;
  float4 x[R][NQ];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = min(row0 + r, a.M - 1);
    if (a.mode == 0) {
      const float* src = a.src + (int64_t)row * a.lds;
#pragma unroll
      for (int i = 0; i < NQ; ++i) x[r][i] = *(const float4*)(src + (i * 64 + lane) * 4);
    } else {
      const int src = a.rowmap ? a.rowmap[row] : row;   // packed row -> b * L + position
      const int tokid = a.ids[src];
      const float* tk = a.tok + (int64_t)tokid * d;
      const float* ps = a.pos + (int64_t)(src % a.L) * d;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int e = (i * 64 + lane) * 4;
        const float4 t = *(const float4*)(tk + e), p = *(const float4*)(ps + e);
        x[r][i] = make_float4(t.x + p.x, t.y + p.y, t.z + p.z, t.w + p.w);
      }
    }
  }
  auto ln = [&](const float* g, const float* b) {
    float4 gg[NQ], bb[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      gg[i] = *(const float4*)(g + (i * 64 + lane) * 4);
      bb[i] = *(const float4*)(b + (i * 64 + lane) * 4);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NQ; ++i) s += (x[r][i].x + x[r][i].y) + (x[r][i].z + x[r][i].w);
      const float mean = wave_sum(s) / d;
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const float d0 = x[r][i].x - mean, d1 = x[r][i].y - mean, d2 = x[r][i].z - mean, d3 = x[r][i].w - mean;
        v += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
      const float rstd = 1.0f / sqrtf(wave_sum(v) / d + a.eps);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        x[r][i].x = (x[r][i].x - mean) * rstd * gg[i].x + bb[i].x;
        x[r][i].y = (x[r][i].y - mean) * rstd * gg[i].y + bb[i].y;
        x[r][i].z = (x[r][i].z - mean) * rstd * gg[i].z + bb[i].z;
        x[r][i].w = (x[r][i].w - mean) * rstd * gg[i].w + bb[i].w;
      }
    }
  };
  auto store_h = [&]() {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (row0 + r >= a.M) break;
      float* h = a.hf + (int64_t)(row0 + r) * a.ldh;
#pragma unroll
      for (int i = 0; i < NQ; ++i) *(float4*)(h + (i * 64 + lane) * 4) = x[r][i];
    }
  };
  if (a.g2) {
    ln(a.g1, a.b1);
    store_h();
    ln(a.g2, a.b2);
  } else {
    if (a.mode == 1) store_h();
    ln(a.g1, a.b1);
  }
  if (row0 + R - 1 < a.M && (a.ldy % 8) == 0) {
    // 16-B stores for each pair of the wave's rows: lane pairs (2l, 2l+1) swap one 8-B half by
    // DPP, then the even lane stores row 0's 8 consecutive values, the odd lane row 1's (one
    // store instruction per chunk for both rows instead of two 8-B ones; same values)
    const bool odd = lane & 1;
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      u16* y0 = a.y + (int64_t)(row0 + r) * a.ldy;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const u32x2 p0{pack2<BF>(x[r][i].x, x[r][i].y), pack2<BF>(x[r][i].z, x[r][i].w)};
        const u32x2 p1{pack2<BF>(x[r + 1][i].x, x[r + 1][i].y), pack2<BF>(x[r + 1][i].z, x[r + 1][i].w)};
        const u32x2 snd = odd ? p0 : p1;
        const u32x2 rcv{(uint32_t)__builtin_amdgcn_update_dpp(0, (int)snd.x, 0xB1, 0xF, 0xF, false),
                        (uint32_t)__builtin_amdgcn_update_dpp(0, (int)snd.y, 0xB1, 0xF, 0xF, false)};
        const int e = (i * 64 + (lane & ~1)) * 4;   // the pair's first column
        if (!odd) *(u32x4*)(y0 + e) = u32x4{p0.x, p0.y, rcv.x, rcv.y};
        else *(u32x4*)(y0 + a.ldy + e) = u32x4{rcv.x, rcv.y, p1.x, p1.y};
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (row0 + r >= a.M) break;
    u16* y = a.y + (int64_t)(row0 + r) * a.ldy;
#pragma unroll
    for (int i = 0; i < NQ; ++i)
      *(u32x2*)(y + (i * 64 + lane) * 4) = u32x2{pack2<BF>(x[r][i].x, x[r][i].y), pack2<BF>(x[r][i].z, x[r][i].w)};
  }
}

template <bool BF, int NQ, int R = 2>
__global__ __launch_bounds__(256) void ln4_kernel(LnArgs a) {
  ln4_body<BF, NQ, R>(a, blockIdx.x);
}

template <bool BF>
hipError_t ln_dispatch(const LnArgs& a, hipStream_t s) {
  dim3 grid((a.M + 3) / 4), block(256);
  dim3 grid2((a.M + 7) / 8);   // ln4_kernel: 2 rows per wave
  switch (a.d) {
    case 128: ln_kernel<BF, 1><<<grid, block, 0, s>>>(a); break;
    case 256: ln4_kernel<BF, 1><<<grid2, block, 0, s>>>(a); break;
    case 512: ln4_kernel<BF, 2><<<grid2, block, 0, s>>>(a); break;
    case 768: ln4_kernel<BF, 3><<<grid2, block, 0, s>>>(a); break;
    case 1024: ln4_kernel<BF, 4><<<grid2, block, 0, s>>>(a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// -------------------------------------------------------------- patchify ---
// Fast path (p % 8 == 0): one thread per (patch row, ky, 8-pixel run) reads the run's
// 8 pixels of all channels once (24 B u8 / 3 x 32 B f32) and writes one 16-B chunk
// per channel at k = c*p*p + ky*p + kx0 (conv weight flatten order [c][ky][kx]).
template <bool BF>
__global__ __launch_bounds__(256) void patchify_fast_kernel(const void* pix, int layout, int B, int S, int p,
                                                            const float* lut, u16* P, int Kp) {
  __shared__ float slut[3 * 256];
  for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) slut[i] = lut[i];
  __syncthreads();
  const int G = S / p, runs = p / 8, pp = p * p;
  const int64_t total = (int64_t)B * G * G * p * runs;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < total;
       w += (int64_t)gridDim.x * blockDim.x) {
    const int run = (int)(w % runs);
    int64_t q = w / runs;
    const int ky = (int)(q % p);
    const int64_t r = q / p;                 // patch row = b*G*G + py*G + px
    const int b = (int)(r / (G * G));
    const int pi = (int)(r - (int64_t)b * G * G);
    const int py = pi / G, px = pi - py * G;
    const int yy = py * p + ky, xx = px * p + run * 8;
    float v[3][8];
    if (layout == 0) {
      const uint8_t* src = (const uint8_t*)pix + (((int64_t)b * S + yy) * S + xx) * 3;
      const uint2 w0 = *(const uint2*)src, w1 = *(const uint2*)(src + 8), w2 = *(const uint2*)(src + 16);
      const uint32_t d[6] = {w0.x, w0.y, w1.x, w1.y, w2.x, w2.y};
#pragma unroll
      for (int e = 0; e < 24; ++e) {
        const uint32_t u = (d[e >> 2] >> ((e & 3) * 8)) & 0xffu;
        v[e % 3][e / 3] = slut[(e % 3) * 256 + u];
      }
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* src = (const float*)pix + (((int64_t)b * 3 + c) * S + yy) * S + xx;
        const float4 a0 = *(const float4*)src, a1 = *(const float4*)(src + 4);
        v[c][0] = a0.x; v[c][1] = a0.y; v[c][2] = a0.z; v[c][3] = a0.w;
        v[c][4] = a1.x; v[c][5] = a1.y; v[c][6] = a1.z; v[c][7] = a1.w;
      }
    }
    u16* dst = P + r * Kp + ky * p + run * 8;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint4 o;
      o.x = pack2<BF>(v[c][0], v[c][1]); o.y = pack2<BF>(v[c][2], v[c][3]);
      o.z = pack2<BF>(v[c][4], v[c][5]); o.w = pack2<BF>(v[c][6], v[c][7]);
      *(uint4*)(dst + c * pp) = o;
    }
  }
}

// zero the K padding columns [C*p*p, Kp) (only when Kp > C*p*p)
__global__ void pad_cols_kernel(u16* P, int64_t rows, int k0, int Kp) {
  const int w = Kp - k0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * w; i += (int64_t)gridDim.x * blockDim.x)
    P[(i / w) * Kp + k0 + (i % w)] = 0;
}

// Generic path (any p, any C): one thread per 8 consecutive K entries of one patch row.
template <bool BF>
__global__ __launch_bounds__(256) void patchify_kernel(const void* pix, int layout, int B, int S, int p,
                                                       int C, const float* lut, u16* P, int Kp) {
  const int G = S / p;
  const int64_t rows = (int64_t)B * G * G;
  const int chunks = Kp / 8;
  const int64_t total = rows * chunks;
  const int pp = p * p, kreal = C * pp;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < total;
       w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = w / chunks;
    const int kc = (int)(w - r * chunks);
    const int b = (int)(r / (G * G));
    const int pi = (int)(r - (int64_t)b * G * G);
    const int py = pi / G, px = pi - py * G;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = kc * 8 + e;
      float val = 0.f;
      if (k < kreal) {
        const int c = k / pp, rem = k - c * pp;
        const int ky = rem / p, kx = rem - ky * p;
        const int yy = py * p + ky, xx = px * p + kx;
        if (layout == 0) {
          const uint8_t u = ((const uint8_t*)pix)[(((int64_t)b * S + yy) * S + xx) * C + c];
          val = lut[c * 256 + u];
        } else {
          val = ((const float*)pix)[(((int64_t)b * C + c) * S + yy) * S + xx];
        }
      }
      v[e] = val;
    }
    uint4 o;
    o.x = pack2<BF>(v[0], v[1]); o.y = pack2<BF>(v[2], v[3]);
    o.z = pack2<BF>(v[4], v[5]); o.w = pack2<BF>(v[6], v[7]);
    *(uint4*)(P + r * Kp + kc * 8) = o;
  }
}

__global__ void write_cls_kernel(float* h, int64_t ldh, int B, int T, int d, const float* cls,
                                 const float* pos) {
  const int b = blockIdx.x;
  for (int e = threadIdx.x; e < d; e += blockDim.x) h[(int64_t)b * T * ldh + e] = cls[e] + pos[e];
}

// ------------------------------------------------------- pool + projection --

// The pooled row of item b: 0 (vision CLS), or with ids the first EOS token (argmax(ids) for
// the legacy eos_token_id == 2 rule) -- CLIPTextTransformer's pooling
// (TF/models/clip/modeling_clip.py:558-580; vision CLS: :650). Whole wave, uniform result.
__device__ __forceinline__ int pooled_row(const int32_t* ids, int b, int T, int eos, int lane) {
  if (!ids) return 0;
  const int32_t* id = ids + (int64_t)b * T;
  int best = INT_MAX, bestv = INT_MIN;
  for (int t = lane; t < T; t += 64) {
    const int v = id[t];
    if (eos == 2) { if (v > bestv) { bestv = v; best = t; } }
    else if (v == eos && t < best) best = t;
  }
  if (eos == 2) {
    for (int o = 32; o > 0; o >>= 1) {
      const int ov = __shfl_xor(bestv, o, 64), ob = __shfl_xor(best, o, 64);
      if (ov > bestv || (ov == bestv && ob < best)) { bestv = ov; best = ob; }
    }
  } else {
    for (int o = 32; o > 0; o >>= 1) best = min(best, __shfl_xor(best, o, 64));
  }
  return best == INT_MAX ? 0 : best;   // (ids == eos).argmax() is 0 when absent
}

// Last-layer pruning: one wave per item copies its pooled row of the residual stream h and of
// the attention output O into the compact hc [B][d] / Oc [B][ldoc] (see run_layers).
__global__ __launch_bounds__(64) void gather_pooled_kernel(const float* h, int64_t ldh, const u16* O, int64_t ldo,
                                                           int T, int d, const int32_t* ids, int eos, float* hc,
                                                           u16* Oc, int64_t ldoc, const int* offs) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int64_t row = offs ? (int64_t)offs[b + 1] - 1 : (int64_t)b * T + pooled_row(ids, b, T, eos, lane);
  for (int e = lane * 4; e < d; e += 256) {
    *(float4*)(hc + (int64_t)b * d + e) = *(const float4*)(h + row * ldh + e);
    *(u32x2*)(Oc + (int64_t)b * ldoc + e) = *(const u32x2*)(O + row * ldo + e);
  }
}

// Grid (B/PRB row blocks) x (D/64 column blocks), 16 waves. Each block LayerNorms its PRB
// pooled rows into LDS (layout [i][row]: one ds_read_b128 = 4 rows of element i), then thread
// (c, part) accumulates column c over a sixteenth of d for all PRB rows with coalesced projT
// [d][D] reads; the 16 parts are summed through LDS in part order. (4 parts of d/4 left each
// thread a 192-long dependent chain of loads and FMAs: ~30 us per launch at B = 256.) The
// un-normalised rows go to `tmp`; finish_rows_kernel applies the L2 norm.
constexpr int PRB = 8, PP = 16;
__global__ __launch_bounds__(64 * PP) void pool_project_kernel(const float* h, int64_t ldh, int B, int T, int d,
                                                               const int32_t* ids, int eos, const float* g,
                                                               const float* bt, float eps, const float* projT, int D,
                                                               float* tmp, const int* offs) {
  // Batch invariance: a row's arithmetic must not depend on its slot r in the PRB group.
  // With implicit contraction the compiler fuses (or SLP-packs unfused) the unrolled
  // per-slot chains differently, 1-ulp apart; so no implicit contraction here, and every
  // intended FMA is an explicit fmaf.
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* y = sm;                   // [d][PRB]
  float* part_sum = sm + d * PRB;  // [PP][PRB][64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = blockIdx.x * PRB;
  for (int rr = wid; rr < PRB; rr += PP) {
    const int b = b0 + rr;
    if (b >= B) {
      for (int e = lane; e < d; e += 64) y[e * PRB + rr] = 0.f;
      continue;
    }
    const int64_t prow = offs ? (int64_t)offs[b + 1] - 1 : (int64_t)b * T + pooled_row(ids, b, T, eos, lane);
    const float* x = h + prow * ldh;
    float s = 0.f;
    for (int e = lane; e < d; e += 64) s += x[e];
    const float mean = wave_sum(s) / d;
    float v = 0.f;
    for (int e = lane; e < d; e += 64) { const float t = x[e] - mean; v = fmaf(t, t, v); }
    const float rstd = 1.0f / sqrtf(wave_sum(v) / d + eps);
    for (int e = lane; e < d; e += 64) y[e * PRB + rr] = fmaf((x[e] - mean) * rstd, g[e], bt[e]);
  }
  __syncthreads();
  const int c = lane, part = wid;
  const int j = blockIdx.y * 64 + c;
  const int i0 = part * (d / PP), i1 = i0 + d / PP;
  float acc[PRB];
#pragma unroll
  for (int r = 0; r < PRB; ++r) acc[r] = 0.f;
  if (j < D) {
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
      const float w = projT[(int64_t)i * D + j];
      const float4 ya = *(const float4*)(y + i * PRB), yb = *(const float4*)(y + i * PRB + 4);
      acc[0] = fmaf(ya.x, w, acc[0]); acc[1] = fmaf(ya.y, w, acc[1]);
      acc[2] = fmaf(ya.z, w, acc[2]); acc[3] = fmaf(ya.w, w, acc[3]);
      acc[4] = fmaf(yb.x, w, acc[4]); acc[5] = fmaf(yb.y, w, acc[5]);
      acc[6] = fmaf(yb.z, w, acc[6]); acc[7] = fmaf(yb.w, w, acc[7]);
    }
  }
#pragma unroll
  for (int r = 0; r < PRB; ++r) part_sum[(part * PRB + r) * 64 + c] = acc[r];
  __syncthreads();
  if (wid < PRB && j < D) {   // wave r sums row r's 16 parts, in part order
    const int r = wid, b = b0 + r;
    if (b < B) {
      float t = part_sum[r * 64 + c];
#pragma unroll
      for (int q = 1; q < PP; ++q) t += part_sum[(q * PRB + r) * 64 + c];
      tmp[(int64_t)b * D + j] = t;
    }
  }
}

// Varlen text plan: live rows per caption (its pooled row + 1: with the causal mask no later row
// reaches the pooled one), their prefix sums, the packed-row -> [B, L] map and the fused-attention
// tiles (greedy: whole captions in order, <= 256 rows per tile).
// live rows per caption, one wave per caption (pooled_row's rule): its own launch, so the id
// reads of all captions are in flight at once
__global__ __launch_bounds__(256) void text_lens_kernel(const int32_t* ids, int B, int L, int eos, int* lens) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int p = pooled_row(ids, b, L, eos, threadIdx.x & 63);
  if ((threadIdx.x & 63) == 0) lens[b] = p + 1;
}

// One workgroup, everything parallel but the walk over tiles: block prefix sum of the lengths in
// LDS, then per caption b (a thread each) the end of a tile that would start at b (binary search
// in the prefix sums), then thread 0 chains the tiles from caption 0 (one LDS read per tile).
// (A sequential per-caption pass in one wave cost 40-110 us at B = 256.)
constexpr int PLAN_MAX_B = 4096;
__global__ __launch_bounds__(256) void text_plan_kernel(int B, int L, const int* lens, int* offs, int* tiles,
                                                        int* counts) {
  __shared__ int s_off[PLAN_MAX_B + 1];
  __shared__ int s_next[PLAN_MAX_B];
  __shared__ int s_part[256];
  const int tid = threadIdx.x;
  const int C = (B + 255) / 256;   // captions per thread, contiguous
  const int b0 = min(tid * C, B), b1 = min(b0 + C, B);
  int sum = 0;
  for (int b = b0; b < b1; ++b) { s_off[b] = sum; sum += lens[b]; }
  s_part[tid] = sum;
  __syncthreads();
  if (tid < 64) {   // exclusive scan of the 256 chunk sums: 4 per lane, then a wave scan
    const int v0 = s_part[tid * 4], v1 = s_part[tid * 4 + 1], v2 = s_part[tid * 4 + 2], v3 = s_part[tid * 4 + 3];
    const int own = v0 + v1 + v2 + v3;
    int t = own;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(t, o, 64);
      if (tid >= o) t += y;
    }
    const int ex = t - own;
    s_part[tid * 4] = ex;
    s_part[tid * 4 + 1] = ex + v0;
    s_part[tid * 4 + 2] = ex + v0 + v1;
    s_part[tid * 4 + 3] = ex + v0 + v1 + v2;
    if (tid == 63) {
      s_off[B] = t;
      counts[0] = t;
    }
  }
  __syncthreads();
  for (int b = b0; b < b1; ++b) s_off[b] += s_part[tid];
  __syncthreads();
  for (int b = tid; b < B; b += 256) {   // largest e with s_off[e] - s_off[b] <= 256
    int lo = b + 1, hi = B;
    const int lim = s_off[b] + 256;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_off[mid] <= lim) lo = mid; else hi = mid - 1;
    }
    s_next[b] = lo;
  }
  __syncthreads();
  if (tid == 0) {
    int nt = 0;
    for (int first = 0; first < B; first = s_next[first]) tiles[nt++] = first | ((s_next[first] - first) << 16);
    counts[1] = nt;
  }
  for (int b = tid; b <= B; b += 256) offs[b] = s_off[b];
}

// packed row r -> b * L + (r - offs[b]) (text_plan's row map), in parallel: workgroup w owns
// captions [16 w, 16 w + 16) and their rows (contiguous in the packed order); each thread finds its
// rows' caption by a 4-step binary search over the 17 offsets in LDS, and stores coalesced. (Filled
// inside the one-workgroup plan kernel, caption by caption, this took ~50 of its 61 us per call.)
constexpr int ROWMAP_CAPS = 16;
__global__ __launch_bounds__(256) void text_rowmap_kernel(int B, int L, const int* offs, int* rowmap) {
  __shared__ int s_o[ROWMAP_CAPS + 1];
  const int b0 = blockIdx.x * ROWMAP_CAPS, nb = min(ROWMAP_CAPS, B - b0);
  if (threadIdx.x <= nb) s_o[threadIdx.x] = offs[b0 + threadIdx.x];
  __syncthreads();
  const int o0 = s_o[0], n = s_o[nb] - o0;
  for (int p = threadIdx.x; p < n; p += 256) {
    const int r = o0 + p;
    int lo = 0, hi = nb - 1;   // the last j with s_o[j] <= r
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_o[mid] <= r) lo = mid; else hi = mid - 1;
    }
    rowmap[r] = (b0 + lo) * L + (r - s_o[lo]);
  }
}

// out[b] = tmp[b] / ||tmp[b]||_2 (models/clip_model.py:116,148) or a plain copy; f32 or f16 out
__global__ __launch_bounds__(256) void finish_rows_kernel(const float* tmp, int B, int D, void* out, int out_dtype,
                                                          int normalize) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* r = tmp + (int64_t)b * D;
  float s = 0.f;
  for (int e = lane; e < D; e += 64) s = fmaf(r[e], r[e], s);
  const float nrm = normalize ? sqrtf(wave_sum(s)) : 1.f;
  for (int e = lane; e < D; e += 64) {
    const float o = normalize ? r[e] / nrm : r[e];
    if (out_dtype == 0) ((float*)out)[(int64_t)b * D + e] = o;
    else ((u16*)out)[(int64_t)b * D + e] = f32_to_f16(o);
  }
}

// ------------------------------------------------------------ index rows ---
__global__ __launch_bounds__(256) void rows_to_f16_kernel(const void* src, int src_dtype, int64_t n, int dim,
                                                          u16* dst, float* inv_norm, int norm_src) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  auto load = [&](int e) {
    return src_dtype == 0 ? ((const float*)src)[row * dim + e] : f16_to_f32(((const u16*)src)[row * dim + e]);
  };
  // norm_src 2: round v / ||v|| (unit rows: no fp16 overflow, no subnormal loss of tiny rows)
  float scale = 1.f;
  if (norm_src == 2) {
    float s0 = 0.f;
    for (int e = lane; e < dim; e += 64) {
      const float v = load(e);
      s0 += v * v;
    }
    scale = 1.0f / sqrtf(wave_sum(s0));
  }
  float s = 0.f;
  for (int e = lane; e < dim; e += 64) {
    const float v = load(e) * scale;
    const u16 hv = f32_to_f16(v);
    dst[row * dim + e] = hv;
    const float r = norm_src == 1 ? v : f16_to_f32(hv);
    s += r * r;
  }
  s = wave_sum(s);
  if (lane == 0) inv_norm[row] = 1.0f / sqrtf(s);
}

__global__ __launch_bounds__(256) void sample_rows_kernel(const u16* rows, const float* inv, int64_t n, int dim,
                                                          int64_t S, u16* out_rows, float* out_inv) {
  const int64_t sidx = blockIdx.x;
  const int64_t src = sidx * n / S;
  const uint4* a = (const uint4*)(rows + src * dim);
  uint4* b = (uint4*)(out_rows + sidx * dim);
  for (int e = threadIdx.x; e < dim / 8; e += blockDim.x) b[e] = a[e];
  if (threadIdx.x == 0) out_inv[sidx] = inv[src];
}

__global__ __launch_bounds__(256) void l2n_kernel(float* rows, int64_t n, int dim) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  float* r = rows + row * dim;
  float s = 0.f;
  for (int e = lane; e < dim; e += 64) s += r[e] * r[e];
  const float nrm = sqrtf(wave_sum(s));
  for (int e = lane; e < dim; e += 64) r[e] = r[e] / nrm;
}

// Query fusion (SeekerService._build_query_embedding, seeker_service.py:148-157): one wave per
// row, out = v / ||v|| with v = wa*a + wb*b (b == nullptr: v = a, the single-modality branch).
// The weighted sum is rounded like the reference's (two products, then one add: no FMA contraction).
__global__ __launch_bounds__(256) void fuse_rows_kernel(const float* a, float wa, const float* b, float wb,
                                                         int64_t n, int dim, float* out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* ra = a + row * dim;
  const float* rb = b ? b + row * dim : nullptr;
  float* ro = out + row * dim;
  float s = 0.f;
  for (int e = lane; e < dim; e += 64) {
    const float v = rb ? __fadd_rn(__fmul_rn(wa, ra[e]), __fmul_rn(wb, rb[e])) : ra[e];
    s += v * v;
  }
  const float nrm = sqrtf(wave_sum(s));
  for (int e = lane; e < dim; e += 64) {
    const float v = rb ? __fadd_rn(__fmul_rn(wa, ra[e]), __fmul_rn(wb, rb[e])) : ra[e];
    ro[e] = v / nrm;
  }
}

__global__ __launch_bounds__(256) void f32_to_f16_kernel(const float* src, int64_t total, u16* dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = f32_to_f16(src[i]);
}

}  // namespace

hipError_t layernorm(bool bf16, const LnArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  return bf16 ? ln_dispatch<true>(a, s) : ln_dispatch<false>(a, s);
}

hipError_t patchify(bool bf16, const void* pix, int layout, int B, int S, int p, int C, const float* lut,
                    u16* P, int Kp, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (Kp % 8) return hipErrorInvalidValue;
  const int G = S / p;
  if (C == 3 && p % 8 == 0 && (S * 3) % 8 == 0) {
    const int64_t total = (int64_t)B * G * G * p * (p / 8);
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 32);
    if (bf16) patchify_fast_kernel<true><<<blocks, 256, 0, s>>>(pix, layout, B, S, p, lut, P, Kp);
    else patchify_fast_kernel<false><<<blocks, 256, 0, s>>>(pix, layout, B, S, p, lut, P, Kp);
    if (Kp > 3 * p * p) {
      const int64_t rows = (int64_t)B * G * G;
      pad_cols_kernel<<<(int)std::min<int64_t>((rows * (Kp - 3 * p * p) + 255) / 256, 4096), 256, 0, s>>>(
          P, rows, 3 * p * p, Kp);
    }
    return hipGetLastError();
  }
  const int64_t total = (int64_t)B * G * G * (Kp / 8);
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
  if (bf16) patchify_kernel<true><<<blocks, 256, 0, s>>>(pix, layout, B, S, p, C, lut, P, Kp);
  else patchify_kernel<false><<<blocks, 256, 0, s>>>(pix, layout, B, S, p, C, lut, P, Kp);
  return hipGetLastError();
}

hipError_t write_cls(float* h, int64_t ldh, int B, int T, int d, const float* cls, const float* pos,
                     hipStream_t s) {
  if (B <= 0) return hipSuccess;
  write_cls_kernel<<<B, 256, 0, s>>>(h, ldh, B, T, d, cls, pos);
  return hipGetLastError();
}

hipError_t gather_pooled(const float* h, int64_t ldh, const u16* O, int64_t ldo, int B, int T, int d,
                         const int32_t* ids, int eos, float* hc, u16* Oc, int64_t ldoc, hipStream_t s,
                         const int* offs) {
  if (B <= 0) return hipSuccess;
  if ((d % 4) || (ldh % 4) || (ldo % 4) || (ldoc % 4)) return hipErrorInvalidValue;
  gather_pooled_kernel<<<B, 64, 0, s>>>(h, ldh, O, ldo, T, d, ids, eos, hc, Oc, ldoc, offs);
  return hipGetLastError();
}

hipError_t pool_project(const float* h, int64_t ldh, int B, int T, int d, const int32_t* ids, int eos,
                        const float* g, const float* bta, float eps, const float* projT, int D, float* tmp, void* out,
                        int out_dtype, int normalize, hipStream_t s, const int* offs) {
  if (B <= 0) return hipSuccess;
  if (d % PP) return hipErrorInvalidValue;
  const size_t sm = (size_t)(d * PRB + PP * PRB * 64) * sizeof(float);
  dim3 grid((B + PRB - 1) / PRB, (D + 63) / 64);
  pool_project_kernel<<<grid, 64 * PP, sm, s>>>(h, ldh, B, T, d, ids, eos, g, bta, eps, projT, D, tmp, offs);
  finish_rows_kernel<<<(B + 3) / 4, 256, 0, s>>>(tmp, B, D, out, out_dtype, normalize);
  return hipGetLastError();
}

hipError_t text_plan(const int32_t* ids, int B, int L, int eos, int* lens, int* offs, int* rowmap, int* tiles,
                     int* counts, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (L < 1 || L > 256) return hipErrorInvalidValue;
  if (B > PLAN_MAX_B) return hipErrorInvalidValue;
  text_lens_kernel<<<(B + 3) / 4, 256, 0, s>>>(ids, B, L, eos, lens);
  text_plan_kernel<<<1, 256, 0, s>>>(B, L, lens, offs, tiles, counts);
  text_rowmap_kernel<<<(B + ROWMAP_CAPS - 1) / ROWMAP_CAPS, 256, 0, s>>>(B, L, offs, rowmap);
  return hipGetLastError();
}

hipError_t rows_to_f16(const void* src, int src_dtype, int64_t n, int dim, u16* dst, float* inv_norm,
                       hipStream_t s, int norm_src) {
  if (n <= 0) return hipSuccess;
  rows_to_f16_kernel<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(src, src_dtype, n, dim, dst, inv_norm, norm_src);
  return hipGetLastError();
}

hipError_t sample_rows(const u16* rows, const float* inv, int64_t n, int dim, int64_t S, u16* out_rows,
                       float* out_inv, hipStream_t s) {
  if (S <= 0) return hipSuccess;
  if (dim % 8) return hipErrorInvalidValue;
  sample_rows_kernel<<<(unsigned)S, 64, 0, s>>>(rows, inv, n, dim, S, out_rows, out_inv);
  return hipGetLastError();
}

hipError_t l2_normalize_rows(float* rows, int64_t n, int dim, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  l2n_kernel<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(rows, n, dim);
  return hipGetLastError();
}

hipError_t fuse_rows(const float* a, float wa, const float* b, float wb, int64_t n, int dim, float* out,
                     hipStream_t s) {
  if (n <= 0) return hipSuccess;
  fuse_rows_kernel<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(a, wa, b, wb, n, dim, out);
  return hipGetLastError();
}

hipError_t f32_to_f16_rows(const float* src, int64_t n, int dim, u16* dst, hipStream_t s) {
  const int64_t total = n * dim;
  if (total <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  f32_to_f16_kernel<<<blocks, 256, 0, s>>>(src, total, dst);
  return hipGetLastError();
}

}  // namespace clm
