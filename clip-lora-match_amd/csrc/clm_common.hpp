// Common device/host helpers for libclm (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Raw buffer descriptor over [base, base + 2 GiB) built from wave-uniform inputs (made
// provable with readfirstlane, so hipcc emits no waterfall loop). A lane passing
// BUF_OOB as its byte offset has its store dropped / its load return 0 by the hardware
// range check: predication without branches (a branch per store makes the waitcnt pass
// fall back to vmcnt(0) in front of every store).
constexpr uint32_t BUF_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int num_records = 0x7FFFFFF0) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, num_records, 0x00020000);
}

namespace clm {

constexpr int WAVE = 64;

// ---- scalar conversions (RNE; NaN preserved by the hardware cvt) ----------
__device__ __forceinline__ float bf16_to_f32(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float f16_to_f32(u16 v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ u16 f32_to_bf16(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ u16 f32_to_f16(float f) { return __builtin_bit_cast(u16, (_Float16)f); }

template <bool BF> __device__ __forceinline__ float to_f32(u16 v) { return BF ? bf16_to_f32(v) : f16_to_f32(v); }
template <bool BF> __device__ __forceinline__ u16 from_f32(float f) { return BF ? f32_to_bf16(f) : f32_to_f16(f); }

// pack two floats into one dword of two 16-bit values (lo first), RNE.
// The two-element vector conversion is ONE v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32; the form
// with two scalar casts + shift / or compiles (ROCm 7.2) to two half-used v_cvt_pk_bf16_f32,
// a shift and an SDWA or -- 4 VALU per pair (3 for fp16) in every epilogue and in attention's
// P packing. Same instruction, same rounding: results are bit-identical.
// (-DCLM_PACK_SCALAR builds the old form for A/B runs.)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
template <bool BF> __device__ __forceinline__ uint32_t pack2(float a, float b) {
#ifdef CLM_PACK_SCALAR
  return (uint32_t)from_f32<BF>(a) | ((uint32_t)from_f32<BF>(b) << 16);
#else
  if constexpr (BF)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
  else
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, f16x2_t));
#endif
}

// one 16x16x32 MFMA on 8-element fragments held as raw 16-byte vectors
template <bool BF>
__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, f32x4 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// ---- wave reductions (64 lanes) ---------------------------------------------
// Butterfly all-reduce on the VALU: DPP quad_perm [1,0,3,2] / [2,3,0,1], row_half_mirror and
// row_mirror inside each 16-lane row, then v_permlane16_swap / v_permlane32_swap across rows
// (no ds_bpermute round trips through the LDS crossbar). Every lane combines the same two
// partial values at every step (a + b == b + a), so all 64 lanes hold bit-identical results.
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <bool MAX> __device__ __forceinline__ float op2(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }
template <bool MAX> __device__ __forceinline__ float row16_reduce(float v) {
  v = op2<MAX>(v, dpp_f<0xB1>(v));    // quad_perm [1,0,3,2]
  v = op2<MAX>(v, dpp_f<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op2<MAX>(v, dpp_f<0x141>(v));   // row_half_mirror: the other quad of the 8
  v = op2<MAX>(v, dpp_f<0x140>(v));   // row_mirror: the other 8 of the row
  return v;
}
// over the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 (the 16-lane rows of a wave)
template <bool MAX> __device__ __forceinline__ float cross_rows_reduce(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op2<MAX>(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op2<MAX>(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
template <bool MAX> __device__ __forceinline__ float wave_reduce(float v) {
  return cross_rows_reduce<MAX>(row16_reduce<MAX>(v));
}
__device__ __forceinline__ float wave_sum(float v) { return wave_reduce<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_reduce<true>(v); }
// reductions inside aligned groups of 16 lanes (MFMA C-layout rows)
__device__ __forceinline__ float group16_sum(float v) { return row16_reduce<false>(v); }
__device__ __forceinline__ float group16_max(float v) { return row16_reduce<true>(v); }

// fp16 bits of the largest fp16 value <= v (round toward -inf; NaN stays NaN): RNE, then one
// step down when that rounded up
__device__ __forceinline__ uint32_t f16_down(float v) {
  const _Float16 h = (_Float16)v;
  uint32_t b = __builtin_bit_cast(uint16_t, h);
  if ((float)h > v) b = b == 0u ? 0x8001u : (b & 0x8000u) ? b + 1u : b - 1u;
  return b;
}

__device__ __forceinline__ float quick_gelu(float x) {
  // TF/activations.py:123  x * sigmoid(1.702 x), as x * rcp(1 + 2^(-1.702 log2(e) x)):
  // v_exp_f32 + v_rcp_f32 (1 ulp) instead of an IEEE division (4 v_div_* + v_fma per value,
  // which made the fc1 epilogue cost as much as a third of its main loop). Limits stay exact:
  // x -> -inf gives 2^+big = inf, rcp = 0, -0; x -> +inf gives x.
  const float t = __builtin_amdgcn_exp2f(-2.4554669595930157f * x);
  return x * __builtin_amdgcn_rcpf(1.0f + t);
}

// XOR swizzle of 16-byte chunks inside 128-byte LDS rows: conflict-free
// ds_read_b128 for MFMA fragment reads of 16 consecutive rows.
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming §5 T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

}  // namespace clm
