// Fused q/k/v projection + attention for short sequences (T <= 128: ViT-B/32 images T = 50,
// captions L <= 77, causal): one launch per encoder layer instead of the qkv GEMM + the
// attention kernel.
//
// Replaces, per layer, CLIPAttention's q_proj / k_proj / v_proj and its sdpa/eager core
// (TF/models/clip/modeling_clip.py:294-297 and 259-277 / 298-335). A tile is G = 256 / T whole
// sequences (256 rows) x ONE head's q, k and v columns (192 = 3 x 64 W rows, gathered from the
// fused [3d, K] weight), so the tile's epilogue holds everything that head's attention needs.
// The q / k / v values are rounded to the compute dtype exactly as the STORE epilogue rounds
// them (acc + bias, one v_cvt_pk), staged in LDS instead of HBM, and attended with the
// arithmetic of attn_small_kernel (k_attn.hip): S^T = K Q^T, one exact softmax pass over <= 2
// key tiles, O^T = V^T P^T. The output O is bit-identical to the two-kernel path
// (tests/test_gpu_encode.py::test_fused_qkv_attention_bit_identical), and the [M, 3d] QKV
// tensor never goes to HBM (vision: 59 MB written + read back per layer at batch 256).
//
// Main loop: the gemm_kernel structure (k_gemm.hip) at 256 x 192 x 64, 8 waves (4 x 2, 64 x 96
// per wave), 2-stage global_load_lds ring, swapped MFMA operands (so the accumulator
// MFMA order, hence every q/k/v value, equals the qkv GEMM's). One tile per workgroup: the
// 96 KB staging image reuses the ring's LDS.
#include <algorithm>

#include "gemm_common.hpp"

namespace clm {

namespace {
using namespace gemm_detail;

constexpr int FA_BM = 256, FA_BN = 192, FA_WM = 4, FA_WN = 2, FA_NW = 8;
constexpr int FA_TM = FA_BM / FA_WM / 16, FA_TN = FA_BN / FA_WN / 16;   // 4 x 6 blocks per wave
constexpr int FA_LA = FA_BM / 8 / FA_NW, FA_LB = FA_BN / 8 / FA_NW;      // DMA pieces per wave
constexpr int FA_STAGE = (FA_BM + FA_BN) * 128;
constexpr int FA_LDS = 2 * FA_STAGE;   // 112 KB ring; the staging image (96 KB) overlays it
constexpr int FA_SEC = FA_BM * 128;    // one staged section (q, k or v): [256 rows][128 B]
static_assert(3 * FA_SEC <= FA_LDS, "q/k/v staging must fit in the ring's LDS");
static_assert(FA_BM % (8 * FA_NW) == 0 && FA_BN % (8 * FA_NW) == 0, "rows split evenly over waves");

// The staged q / k / v sections ([256 rows][128 B]) swizzle their 16-B chunks by row & 7 (the
// DMA ring's (row >> 1) & 7 pairs rows 2j and 2j + 1 on one chunk): 8 consecutive rows then hold a
// chunk at 8 distinct positions, so the 16-B staging writes (8-lane groups of consecutive rows),
// the q / k fragment reads (ds_read_b128 at any sequence offset) and the transposed V reads
// (32 lanes = 8 consecutive rows x 2 chunks x 2 halves) are all bank-conflict free.
__device__ __forceinline__ int swz_s(int row, int chunk) { return chunk ^ (row & 7); }

// V^T operand of O^T = V^T P^T from the staged V section (rows = tile rows): k_attn.hip's
// v_frag_trT on absolute tile rows, clamped to the image (a clamped row only ever meets a masked
// key, whose P is exactly 0)
__device__ __forceinline__ u32x4 v_frag_rows(const uint8_t* sec, int kbase, int nb, int lane) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int chunk = nb * 2 + (p >> 1);
  const int ka = min(kbase + g * 4 + q, FA_BM - 1), kb = min(kbase + 16 + g * 4 + q, FA_BM - 1);
  const uint8_t* pa = sec + ka * 128 + (swz_s(ka, chunk) << 4) + (p & 1) * 8;
  const uint8_t* pb = sec + kb * 128 + (swz_s(kb, chunk) << 4) + (p & 1) * 8;
  const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  const u32x2 x = __builtin_bit_cast(u32x2, ra), y = __builtin_bit_cast(u32x2, rb);
  return u32x4{x.x, x.y, y.x, y.y};
}

struct FaArgs {
  const u16* X; int64_t ldx;   // [B*T, K] LayerNorm output (compute dtype)
  const u16* W; int64_t ldw;   // [3d, K] fused q/k/v weight (q rows pre-scaled by 64^-1/2)
  const float* bias;           // [3d]
  u16* out; int64_t ldo;       // [B*T, >= d] attention output
  int B, T, H, d, K, G;        // G = sequences per tile
  // varlen (VL): packed sequences of lens[b] rows at offs[b]; tiles[t] = first | count << 16;
  // counts = {live rows, live tiles}
  const int* lens; const int* offs; const int* tiles; const int* counts;
};

// workgroup `bid` of the `nwg` that serve one problem (gemm_attn_kernel: the whole grid)
template <bool BF, bool CAUSAL, bool VL>
__device__ __forceinline__ void gemm_attn_body(const FaArgs& a, int bid, int nwg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the H head tiles of one row panel run back to back on one XCD (they share the A panel in L2)
  int t, s0, nseq;
  int64_t m0, M;
  if constexpr (VL) {   // grid sized for the worst case: only the live tiles run
    const int live = __builtin_amdgcn_readfirstlane(a.counts[1]) * a.H;
    if (bid >= live) return;
    t = xcd_remap(bid, live);
    const int tw = __builtin_amdgcn_readfirstlane(a.tiles[t / a.H]);
    s0 = tw & 0xFFFF;
    nseq = tw >> 16;
    m0 = __builtin_amdgcn_readfirstlane(a.offs[s0]);
    M = __builtin_amdgcn_readfirstlane(a.counts[0]);
  } else {
    t = xcd_remap(bid, nwg);
    s0 = (t / a.H) * a.G;
    nseq = min(a.G, a.B - s0);
    m0 = (int64_t)s0 * a.T;
    M = (int64_t)a.B * a.T;
  }
  const int h = t % a.H;
  const int nk = (a.K + BK - 1) / BK;   // K % 64 == 32: the last step multiplies its first 32 columns
  const bool half_last = (a.K % BK) != 0;

  // ---- main loop: acc[256 x 192] = X[m0 .. m0 + 255, :] . W[head h's q, k, v rows]^T --------
  const int r8 = lane >> 3, pc = lane & 7;
  const u16* a_src[FA_LA];
  const u16* w_src[FA_LB];
#pragma unroll
  for (int j = 0; j < FA_LA; ++j) {
    const int row = (wid * FA_LA + j) * 8 + r8;
    a_src[j] = a.X + min(m0 + row, M - 1) * a.ldx + (pc ^ ((row >> 1) & 7)) * 8;
  }
#pragma unroll
  for (int j = 0; j < FA_LB; ++j) {
    const int row = (wid * FA_LB + j) * 8 + r8;   // tile column: section row / 64, head dim row % 64
    const int64_t wrow = (int64_t)(row >> 6) * a.d + h * 64 + (row & 63);
    w_src[j] = a.W + wrow * a.ldw + (pc ^ ((row >> 1) & 7)) * 8;
  }
  auto stage = [&](int kt, int buf) {
    uint8_t* base = smem + buf * FA_STAGE;
#pragma unroll
    for (int j = 0; j < FA_LA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + kt * BK), (void*)(base + (wid * FA_LA + j) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int j = 0; j < FA_LB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(w_src[j] + kt * BK),
                                       (void*)(base + FA_BM * 128 + (wid * FA_LB + j) * 1024), 16, 0, 0);
  };

  const int wm = wid / FA_WN, wn = wid % FA_WN;
  // the epilogue's bias vectors, loaded before the main loop (their latency hides under it instead
  // of opening the q/k/v staging)
  float4 bv[FA_TN];
#pragma unroll
  for (int nb = 0; nb < FA_TN; ++nb) {
    const int col = wn * (FA_BN / FA_WN) + nb * 16 + 4 * g;
    bv[nb] = a.bias ? *(const float4*)(a.bias + (col >> 6) * a.d + h * 64 + (col & 63)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  f32x4 acc[FA_TM][FA_TN];
#pragma unroll
  for (int i = 0; i < FA_TM; ++i)
#pragma unroll
    for (int j = 0; j < FA_TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  for (int s = 0; s < nk; ++s) {
    wait_vmcnt<0>();   // K-step s landed (the only DMA in flight)
    lds_barrier();     // ... for every wave, and every wave is done reading buffer (s + 1) & 1
    if (s + 1 < nk) stage(s + 1, (s + 1) & 1);
    const uint8_t* sa = smem + (s & 1) * FA_STAGE;
    const uint8_t* sb = sa + FA_BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk == 1 && half_last && s == nk - 1) break;
      const int c = kk * 4 + g;
      u32x4 af[FA_TM], bw[FA_TN];
#pragma unroll
      for (int mb = 0; mb < FA_TM; ++mb) {
        const int row = wm * (FA_BM / FA_WM) + mb * 16 + (lane & 15);
        af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < FA_TN; ++nb) {
        const int row = wn * (FA_BN / FA_WN) + nb * 16 + (lane & 15);
        bw[nb] = *(const u32x4*)(sb + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < FA_TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < FA_TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], acc[mb][nb]);
    }
  }

  // ---- q / k / v -> compute dtype, staged in LDS (sections [256 rows][128 B], swizzled) -----
  // lane holds row wm*64 + mb*16 + (lane & 15), columns wn*96 + nb*16 + 4g .. +3 of the tile:
  // section (q, k, v) = column / 64, head dim = column % 64
  lds_barrier();   // every wave has read its last fragments out of the ring
  // 16-B writes: v_permlane16_swap trades the odd 16-lane groups' block-nb words with the even
  // groups' block-(nb + 1) words, so lane group q holds the 8 consecutive columns
  // (nb + (q & 1)) * 16 + (q >> 1) * 8 .. + 7 of its row (one chunk of one section)
  static_assert(FA_TN % 2 == 0, "column blocks are swapped in pairs");
#pragma unroll
  for (int mb = 0; mb < FA_TM; ++mb) {
    const int row = wm * (FA_BM / FA_WM) + mb * 16 + (lane & 15);
#pragma unroll
    for (int nb = 0; nb < FA_TN; nb += 2) {
      const u32x2 p0{pack2<BF>(acc[mb][nb][0] + bv[nb].x, acc[mb][nb][1] + bv[nb].y),
                     pack2<BF>(acc[mb][nb][2] + bv[nb].z, acc[mb][nb][3] + bv[nb].w)};
      const u32x2 p1{pack2<BF>(acc[mb][nb + 1][0] + bv[nb + 1].x, acc[mb][nb + 1][1] + bv[nb + 1].y),
                     pack2<BF>(acc[mb][nb + 1][2] + bv[nb + 1].z, acc[mb][nb + 1][3] + bv[nb + 1].w)};
      const auto rx = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
      const int col = wn * (FA_BN / FA_WN) + (nb + (g & 1)) * 16 + (g >> 1) * 8;
      const int dim = col & 63;
      *(u32x4*)(smem + (col >> 6) * FA_SEC + row * 128 + (swz_s(row, dim >> 3) << 4)) = u32x4{rx[0], ry[0], rx[1], ry[1]};
    }
  }
  lds_barrier();

  // ---- attention: units of (sequence, 16-query block), round-robin over the 8 waves --------
  constexpr float L2E = 1.4426950408889634f;
  const uint8_t* sQ = smem;
  const uint8_t* sK = smem + FA_SEC;
  const uint8_t* sV = smem + 2 * FA_SEC;
  // units (sequence i, 16-query block) in order, unit u to wave u % 8
  int u = 0, i = 0, qb = 0, nqb = 0, seq_t = 0, seq_r0 = 0;
  auto load_seq = [&]() {   // sequence i: its length and first tile row
    if constexpr (VL) {
      seq_t = a.lens[s0 + i];
      seq_r0 = a.offs[s0 + i] - (int)m0;
    } else {
      seq_t = a.T;
      seq_r0 = i * a.T;
    }
    nqb = (seq_t + 15) / 16;
    qb = 0;
  };
  if (nseq > 0) load_seq();
  for (; i < nseq; ++u) {
    const int q0 = qb * 16, T = seq_t, r0 = seq_r0;
    const bool mine = (u % FA_NW) == wid;
    if (++qb == nqb && ++i < nseq) load_seq();
    if (!mine) continue;
    const int ntiles = (T + 63) / 64;
    const int qi = q0 + (lane & 15);       // this lane's query
    u32x4 qa[2];
    {
      const int qrow = r0 + min(qi, T - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) qa[kk] = *(const u32x4*)(sQ + qrow * 128 + swz_s(qrow, kk * 4 + g) * 16);
    }
    const int nkt = CAUSAL ? min((q0 + 15) / 64 + 1, ntiles) : ntiles;
    f32x4 sc[2][4];   // S^T: lane holds query qi, keys kt*64 + nb*16 + 4g + 0..3
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      if (kt >= nkt) break;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        sc[kt][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int krow = min(r0 + kt * 64 + nb * 16 + (lane & 15), FA_BM - 1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int c = kk * 4 + g;
          sc[kt][nb] = mfma16<BF>(*(const u32x4*)(sK + krow * 128 + swz_s(krow, c) * 16), qa[kk], sc[kt][nb]);
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
    for (int kt = 0; kt < 2; ++kt) {
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
        for (int nb = 0; nb < 4; ++nb)
          o[nb] = mfma16<BF>(v_frag_rows(sV, r0 + kt * 64 + kk * 32, nb, lane), pb[kk], o[nb]);
    }
    rs = cross_rows_reduce<false>(rs);
    if (qi < T) {
      const float inv = 1.0f / rs;
      u16* op = a.out + (m0 + r0 + qi) * a.ldo + h * 64 + 4 * g;   // row of sequence i, query qi
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        *(u32x2*)(op + nb * 16) = u32x2{pack2<BF>(o[nb][0] * inv, o[nb][1] * inv), pack2<BF>(o[nb][2] * inv, o[nb][3] * inv)};
    }
  }
}

template <bool BF, bool CAUSAL, bool VL>
__global__ __launch_bounds__(FA_NW * 64, 2) void gemm_attn_kernel(FaArgs a) {
  gemm_attn_body<BF, CAUSAL, VL>(a, blockIdx.x, gridDim.x);
}

template <bool BF, bool CAUSAL, bool VL>
hipError_t launch(const FaArgs& a, int tiles, hipStream_t s) {
  auto kern = gemm_attn_kernel<BF, CAUSAL, VL>;
  static unsigned dev_done = 0;   // >64 KiB dynamic LDS needs the opt-in attribute, once per device
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, FA_LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  kern<<<dim3(tiles), dim3(FA_NW * 64), FA_LDS, s>>>(a);
  return hipGetLastError();
}
}  // namespace

bool gemm_attn_supported(int T, int H, int d, int K) {
  return T >= 1 && T <= 128 && d == H * 64 && K > 0 && K % 32 == 0;
}

namespace {
// FaArgs + workgroup count of a fixed-length launch; false if the shapes are unsupported
bool fixed_args(const AttnProblem& p, FaArgs& a, int& grid) {
  if (!gemm_attn_supported(p.T, p.H, p.d, p.K) || (p.ldx % 8) || (p.ldw % 8) || (p.ldo % 4) || p.ldx < p.K ||
      p.ldw < p.K || p.ldo < p.d)
    return false;
  a = FaArgs{};
  a.X = p.X; a.ldx = p.ldx; a.W = p.W; a.ldw = p.ldw; a.bias = p.bias; a.out = p.out; a.ldo = p.ldo;
  a.B = p.B; a.T = p.T; a.H = p.H; a.d = p.d; a.K = p.K; a.G = FA_BM / p.T;
  const int64_t tiles = (int64_t)((p.B + a.G - 1) / a.G) * p.H;
  if (tiles > 0x7FFFFFFF) return false;
  grid = (int)tiles;
  return true;
}
// ... of a varlen launch (packed sequences; grid sized for the worst case)
bool varlen_args(const AttnProblem& p, FaArgs& a, int& grid) {
  if (!gemm_attn_supported(p.T, p.H, p.d, p.K) || p.B > 0xFFFF || (p.ldx % 8) || (p.ldw % 8) || (p.ldo % 4) ||
      p.ldx < p.K || p.ldw < p.K || p.ldo < p.d || !p.lens || !p.offs || !p.tiles || !p.counts)
    return false;
  a = FaArgs{};
  a.X = p.X; a.ldx = p.ldx; a.W = p.W; a.ldw = p.ldw; a.bias = p.bias; a.out = p.out; a.ldo = p.ldo;
  a.B = p.B; a.T = p.T; a.H = p.H; a.d = p.d; a.K = p.K; a.G = 0;
  a.lens = p.lens; a.offs = p.offs; a.tiles = p.tiles; a.counts = p.counts;
  // text_plan closes a tile only when the next sequence does not fit, so every tile but the last
  // holds more than 256 - L rows: at most ceil(rows / (257 - L)) + 1 tiles, and at most B
  const int64_t max_tiles = std::min<int64_t>(p.B, ((int64_t)p.B * p.T + (256 - p.T)) / (257 - p.T) + 1);
  const int64_t g = max_tiles * p.H;
  if (g > 0x7FFFFFFF) return false;
  grid = (int)g;
  return true;
}
}  // namespace

hipError_t gemm_attn(bool bf16, bool causal, const u16* X, int64_t ldx, const u16* W, int64_t ldw, const float* bias,
                     u16* out, int64_t ldo, int B, int T, int H, int d, int K, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  AttnProblem p{X, ldx, W, ldw, bias, out, ldo, B, T, H, d, K, nullptr, nullptr, nullptr, nullptr};
  FaArgs a;
  int tiles;
  if (!fixed_args(p, a, tiles)) return hipErrorInvalidValue;
  if (bf16) return causal ? launch<true, true, false>(a, tiles, s) : launch<true, false, false>(a, tiles, s);
  return causal ? launch<false, true, false>(a, tiles, s) : launch<false, false, false>(a, tiles, s);
}

hipError_t gemm_attn_varlen(bool bf16, bool causal, const u16* X, int64_t ldx, const u16* W, int64_t ldw,
                            const float* bias, u16* out, int64_t ldo, int B, int L, int H, int d, int K,
                            const int* lens, const int* offs, const int* tiles, const int* counts, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  AttnProblem p{X, ldx, W, ldw, bias, out, ldo, B, L, H, d, K, lens, offs, tiles, counts};
  FaArgs a;
  int grid;
  if (!varlen_args(p, a, grid)) return hipErrorInvalidValue;
  if (bf16) return causal ? launch<true, true, true>(a, grid, s) : launch<true, false, true>(a, grid, s);
  return causal ? launch<false, true, true>(a, grid, s) : launch<false, false, true>(a, grid, s);
}

}  // namespace clm
