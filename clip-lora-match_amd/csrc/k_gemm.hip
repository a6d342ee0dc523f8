// MFMA GEMM for gfx950: C[M,N] = A[M,K] . W[N,K]^T, bf16/fp16 operands, fp32 accumulate.
//
// Replaces the ATen CPU addmm/conv that the reference runs for every
// nn.Linear / patch-embed conv of the CLIP towers (TF/models/clip/modeling_clip.py:
// 294-297 q/k/v, 332 out_proj, 343-344 fc1/fc2, 148-154 patch conv, and the
// score matmul of src/embedding/search.py:96 / similarity.py:32), with the
// bias, quick-GELU, residual-add, positional-embedding and cosine-scaling
// epilogues fused.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 blocks of
// v_mfma_f32_16x16x32_{bf16,f16}. Both operand tiles are staged HBM/L2 -> LDS
// by global_load_lds_dwordx4 (16 B per lane, lane-linear LDS image), with the
// XOR chunk swizzle applied to the per-lane SOURCE address so fragment reads
// (ds_read_b128, 16 rows per lane group) are bank-conflict free. Two LDS
// stages: tile k+1 streams in while tile k feeds the MFMAs. Workgroup ids are
// remapped XCD-aware so the N-tiles sharing one A row-panel run on one XCD.
#include "kernels.hpp"

namespace clm {

namespace {
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KiB

template <bool BF, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, ntn * ntm);
  const int tm = t / ntn, tn = t % ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // each wave stages 32 rows of A and 32 rows of W per K-tile (4 x 1 KiB DMA each)
  const int r8 = lane >> 3, pc = lane & 7;
  const u16* a_src[4];
  const u16* w_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wid * 32 + i * 8 + r8;
    const int c = pc ^ ((row >> 1) & 7);
    const int gm = min(m0 + row, g.M - 1);
    const int gn = min(n0 + row, g.N - 1);
    a_src[i] = g.A + (int64_t)gm * g.lda + c * 8;
    w_src[i] = g.W + (int64_t)gn * g.ldw + c * 8;
  }
  auto stage = [&](int kt, int s) {
    uint8_t* base = smem + s * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + kt * BK),
                                       (void*)(base + (wid * 32 + i * 8) * 128), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(w_src[i] + kt * BK),
                                       (void*)(base + BM * 128 + (wid * 32 + i * 8) * 128), 16, 0, 0);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, s ^ 1);
    const uint8_t* sa = smem + s * STAGE_BYTES;
    const uint8_t* sb = sa + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      u32x4 af[4], bfr[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int row = wm * 64 + mb * 16 + (lane & 15);
        af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int row = wn * 64 + nb * 16 + (lane & 15);
        bfr[nb] = *(const u32x4*)(sb + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma16<BF>(af[mb], bfr[nb], acc[mb][nb]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: C layout col = lane&15, row = (lane>>4)*4 + j -------------
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = n0 + wn * 64 + nb * 16 + (lane & 15);
      if (n >= g.N) continue;
      float bias = 0.f;
      if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_RESID)
        if (g.bias) bias = g.bias[n];
      float cs = 1.f;
      if constexpr (EPI == EPI_SCORE) cs = g.cscale ? g.cscale[n] : 1.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + mb * 16 + (lane >> 4) * 4 + j;
        if (m >= g.M) continue;
        const float v = acc[mb][nb][j];
        if constexpr (EPI == EPI_STORE) {
          ((u16*)g.out)[(int64_t)m * g.ldo + n] = from_f32<BF>(v + bias);
        } else if constexpr (EPI == EPI_GELU) {
          ((u16*)g.out)[(int64_t)m * g.ldo + n] = from_f32<BF>(quick_gelu(v + bias));
        } else if constexpr (EPI == EPI_RESID) {
          float* o = (float*)g.out + (int64_t)m * g.ldo + n;
          *o = *o + (v + bias);
        } else if constexpr (EPI == EPI_PATCH) {
          const int b = m / g.group, p = m - b * g.group;
          const int64_t row = (int64_t)b * (g.group + 1) + 1 + p;
          ((float*)g.out)[row * g.ldo + n] = v + g.aux[(int64_t)(1 + p) * g.aux_ld + n];
        } else {  // EPI_SCORE
          const float rs = g.rscale ? g.rscale[m] : 1.f;
          ((float*)g.out)[(int64_t)m * g.ldo + n] = v * rs * cs;
        }
      }
    }
  }
}

template <bool BF>
hipError_t launch(int epi, const GemmArgs& g, hipStream_t s) {
  const int nwg = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM);
  dim3 grid(nwg), block(256);
  switch (epi) {
    case EPI_STORE: gemm_nt_kernel<BF, EPI_STORE><<<grid, block, 0, s>>>(g); break;
    case EPI_GELU: gemm_nt_kernel<BF, EPI_GELU><<<grid, block, 0, s>>>(g); break;
    case EPI_RESID: gemm_nt_kernel<BF, EPI_RESID><<<grid, block, 0, s>>>(g); break;
    case EPI_PATCH: gemm_nt_kernel<BF, EPI_PATCH><<<grid, block, 0, s>>>(g); break;
    case EPI_SCORE: gemm_nt_kernel<BF, EPI_SCORE><<<grid, block, 0, s>>>(g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
}  // namespace

hipError_t gemm(bool bf16, int epi, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K <= 0 || (g.K % BK) != 0 || (g.lda % 8) != 0 || (g.ldw % 8) != 0) return hipErrorInvalidValue;
  return bf16 ? launch<true>(epi, g, s) : launch<false>(epi, g, s);
}

}  // namespace clm
