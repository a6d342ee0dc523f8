// Image preprocessing for inputs of any size: shortest-edge BICUBIC resize + centre crop to S x S,
// uint8 HWC RGB in, uint8 [n, S, S, 3] out (the layout clm_encode_image's u8 path normalises inside
// patchify). The arithmetic is PIL's ImagingResample for 8-bit images (Pillow 12.2.0
// src/libImaging/Resample.c, what CLIPImageProcessor runs, models/clip_model.py:108-110), restated
// in oracle/image_ref.py:
//   pass 1 (horizontal) into a uint8 intermediate, pass 2 (vertical); per output coordinate a tap
//   window [min, min + n) with 22-bit fixed-point weights; acc = 2^21 + sum(px * w) in int32,
//   out = clamp(acc >> 22, 0, 255).
// Only the window the crop keeps is computed: the S kept columns of pass 1 over the source rows the
// S kept rows need, then pass 2 for the S x S crop. Each output pixel depends only on its taps, so
// the crop equals PIL's full resize followed by transformers' centre crop bit for bit.
// Tap tables are built on the host (capi.cpp, double precision in PIL's operation order).
#include <algorithm>

#include "kernels.hpp"

namespace clm {
namespace {

constexpr int RS_BITS = 22;

__device__ __forceinline__ uint8_t clip8(int acc) {
  const int v = acc >> RS_BITS;     // arithmetic shift: floor, as PIL's lookup index
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pass 1: tmp[i][row][ox][c] = clip8(sum_j src[i][r0 + row][xmin[ox] + j][c] * xk[ox][j]),
// one thread per (row, ox) of image blockIdx.y, all three channels.
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ src,
                                                       const ResizeDesc* __restrict__ desc,
                                                       const int32_t* __restrict__ coef, int S,
                                                       uint8_t* __restrict__ tmp) {
  const ResizeDesc d = desc[blockIdx.y];
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= d.rows * S) return;
  const int row = t / S, ox = t - row * S;
  const int32_t* xmin = coef + d.coef_off;
  const int32_t* xn = xmin + S;
  const int32_t* xk = xmin + 4 * S + (int64_t)ox * d.kh;
  const uint8_t* p = src + d.src_off + ((int64_t)(d.r0 + row) * d.W + xmin[ox]) * 3;
  int a0 = 1 << (RS_BITS - 1), a1 = a0, a2 = a0;
  const int n = xn[ox];
  for (int j = 0; j < n; ++j) {
    const int w = xk[j];
    a0 += (int)p[3 * j + 0] * w;
    a1 += (int)p[3 * j + 1] * w;
    a2 += (int)p[3 * j + 2] * w;
  }
  uint8_t* o = tmp + d.tmp_off + ((int64_t)row * S + ox) * 3;
  o[0] = clip8(a0);
  o[1] = clip8(a1);
  o[2] = clip8(a2);
}

// pass 2: out[i][oy][ox][c] = clip8(sum_j tmp[i][ymin[oy] + j][ox][c] * yk[oy][j]), one thread per
// output pixel (consecutive threads: consecutive ox, so the tap rows are read coalesced).
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ tmp,
                                                       const ResizeDesc* __restrict__ desc,
                                                       const int32_t* __restrict__ coef, int S,
                                                       uint8_t* __restrict__ out) {
  const ResizeDesc d = desc[blockIdx.y];
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= S * S) return;
  const int oy = t / S, ox = t - oy * S;
  const int32_t* ymin = coef + d.coef_off + 2 * S;
  const int32_t* yn = ymin + S;
  const int32_t* yk = coef + d.coef_off + 4 * S + (int64_t)S * d.kh + (int64_t)oy * d.kv;
  const uint8_t* p = tmp + d.tmp_off + ((int64_t)ymin[oy] * S + ox) * 3;
  const int64_t step = (int64_t)S * 3;
  int a0 = 1 << (RS_BITS - 1), a1 = a0, a2 = a0;
  const int n = yn[oy];
  for (int j = 0; j < n; ++j) {
    const int w = yk[j];
    a0 += (int)p[0] * w;
    a1 += (int)p[1] * w;
    a2 += (int)p[2] * w;
    p += step;
  }
  uint8_t* o = out + ((int64_t)blockIdx.y * S * S + t) * 3;
  o[0] = clip8(a0);
  o[1] = clip8(a1);
  o[2] = clip8(a2);
}

// Counter-based synthetic images (benchmarks / tests of the index build, BASELINE configs[2]):
// byte b of image `row` is a function of (seed, row, b) only, so any shard of any batch split
// regenerates the same pixels. 16 bytes per thread (two splitmix64 outputs), 16-B stores.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_images_kernel(uint64_t seed, int64_t row0, int64_t per_image,
                                                           int64_t total16, uint8_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total16; t += (int64_t)gridDim.x * 256) {
    const int64_t byte = t * 16;
    const int64_t img = byte / per_image;
    const uint64_t key = seed ^ ((uint64_t)(row0 + img) * 0xD1B54A32D192ED03ull);
    const uint64_t w = (uint64_t)(byte - img * per_image) >> 3;
    u32x4 v;
    const uint64_t a = splitmix64(key + w), b = splitmix64(key + w + 1);
    v.x = (uint32_t)a; v.y = (uint32_t)(a >> 32); v.z = (uint32_t)b; v.w = (uint32_t)(b >> 32);
    *(u32x4*)(out + byte) = v;
  }
}

}  // namespace

hipError_t synth_images(uint64_t seed, int64_t row0, int n, int S, uint8_t* out, hipStream_t s) {
  const int64_t per_image = (int64_t)S * S * 3;
  if (n <= 0) return hipSuccess;
  if (per_image % 16) return hipErrorInvalidValue;
  const int64_t total16 = per_image * n / 16;
  const unsigned blocks = (unsigned)std::min<int64_t>((total16 + 255) / 256, 8192);
  synth_images_kernel<<<blocks, 256, 0, s>>>(seed, row0, per_image, total16, out);
  return hipGetLastError();
}

hipError_t resize_crop(const uint8_t* src, const ResizeDesc* desc, int n, int S, int max_rows,
                       const int32_t* coef, uint8_t* tmp, uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 gh((unsigned)(((int64_t)max_rows * S + 255) / 256), (unsigned)n);
  resize_h_kernel<<<gh, 256, 0, s>>>(src, desc, coef, S, tmp);
  const dim3 gv((unsigned)((S * S + 255) / 256), (unsigned)n);
  resize_v_kernel<<<gv, 256, 0, s>>>(tmp, desc, coef, S, out);
  return hipGetLastError();
}

}  // namespace clm
