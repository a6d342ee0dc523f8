// G3 MFMA GEMM for gfx950 (config 23 of clm_gemm): the 256 x 256 eight-phase ping-pong schedule
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T3+T4+T5) for the encoder's large
// qkv / fc1 / fc2 / patch GEMMs (TF/models/clip/modeling_clip.py:294-297, 343-344, 148-154).
// Same operand layout (C = A . W^T, both K-contiguous), fused epilogues (gemm_common.hpp) and
// tile raster as k_gemm.hip.
//
// Geometry: 8 waves = 2 groups (wave rows wr = 0, 1: 128 output rows each) x 4 (64 columns
// each); per wave 8 x 4 accumulator blocks of 16 x 16 (MFMA 16x16x32, W rows on the A port so a
// lane holds 4 consecutive output columns of one row).
//
// LDS: two K-tile buffers (64 deep), each split into four HALF-TILES of 128 rows x 128 B:
//   A0 / A1 = the first / second 64 rows of BOTH wave groups' 128-row slices,
//   B0 / B1 = the first / second 32 columns of every wave's 64-column slice,
// so each wave's quadrant (64 rows x 32 columns) of a K-tile reads exactly one A half and one
// B half. A K-tile runs as four phases, one quadrant each:
//   phase 0: read A0 + B0 fragments | MFMA rows 0-63  x cols 0-31
//   phase 1: read B1                 | MFMA rows 0-63  x cols 32-63
//   phase 2: read A1                 | MFMA rows 64-127 x cols 32-63
//   phase 3: (no reads)              | MFMA rows 64-127 x cols 0-31
// Every phase also issues ONE half-tile of LDS-DMA (2 buffer_load ... lds per wave), so half
// X of K-tile t is issued at phase 4t-5 (A0), 4t-4 (B0), 4t-3 (B1), 4t-2 (A1): 4-5 phases
// ahead of its first read, 3-5 phases after the last read of the half it overwrites (K-tile
// t-2, same buffer). Before each phase's first barrier a counted vmcnt retires the halves
// issued up to 3 phases earlier -- everything the next phase reads -- leaving up to three
// half-tiles (6 DMA instructions) in flight; the loop never drains to vmcnt(0).
// Ping-pong: wave group 1 runs one barrier behind group 0, so on every SIMD one wave issues
// its fragment reads and DMA while the other runs its 16-MFMA cluster (s_setprio(1) around the
// cluster keeps hipcc from hoisting MFMAs across the barriers, T5).
// RAW for a staged half: its issuers' vmcnt precedes a barrier that every reader passes before
// the read (the staggered group passes it one barrier later, still before its read phase).
#include "gemm_common.hpp"

namespace clm {
namespace {
using namespace gemm_detail;

typedef __attribute__((address_space(3))) void* lds_ptr3_t;

constexpr int G3_BM = 256, G3_BN = 256;
constexpr int G3_HALF = 128 * 128;            // one half-tile: 128 rows x 128 B
constexpr int G3_BUF = 4 * G3_HALF;           // A0, A1, B0, B1
constexpr int G3_LDS = 2 * G3_BUF;            // 128 KiB

__device__ __forceinline__ void wait_vm_halves(int c) {   // c half-tiles (2 DMA each) may stay in flight
  if (c >= 3) wait_vmcnt<6>();
  else if (c == 2) wait_vmcnt<4>();
  else if (c == 1) wait_vmcnt<2>();
  else wait_vmcnt<0>();
}

template <bool BF, int EPI>
__global__ __launch_bounds__(512, 1) void gemm3_kernel(GemmArgs g) {
  using C = Cfg<G3_BM, G3_BN, 2, 4, 2>;   // epilogue geometry: 2 x 4 waves, 8 x 4 blocks each
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wn = wid & 3;
  const int ntn = (g.N + G3_BN - 1) / G3_BN, ntm = (g.M + G3_BM - 1) / G3_BM;
  const int ntiles = ntn * ntm;
  const int t = xcd_remap(blockIdx.x, ntiles);
  int tm, tn;
  if (g.m_fastest) {
    tm = t % ntm;
    tn = t / ntm;
  } else {   // grouped raster: GM row-panels x all N-tiles per group, M inner
    constexpr int GM = 8;
    const int group = t / (GM * ntn);
    const int first_m = group * GM;
    const int gsz = min(GM, ntm - first_m);
    const int r = t - group * GM * ntn;
    tm = first_m + r % gsz;
    tn = r / gsz;
  }
  const int m0 = tm * G3_BM, n0 = tn * G3_BN;
  const int nk = g.K / BK;

  // ---- loader: per-lane byte offsets of this wave's 2 pieces (8 LDS rows each) of every half
  const int r8 = lane >> 3, pc = lane & 7;
  const uint32_t lda2 = (uint32_t)g.lda * 2, ldw2 = (uint32_t)g.ldw * 2;
  const __amdgpu_buffer_rsrc_t ra = buf_rsrc(g.A + (int64_t)m0 * g.lda, min(G3_BM, g.M - m0) * (int)lda2);
  const __amdgpu_buffer_rsrc_t rw = buf_rsrc(g.W + (int64_t)n0 * g.ldw, min(G3_BN, g.N - n0) * (int)ldw2);
  uint32_t off[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rl = (wid * 2 + j) * 8 + r8;                       // LDS row inside a half, 0..127
    const uint32_t ch = (uint32_t)((pc ^ ((rl >> 1) & 7)) << 4);  // source-side XOR chunk swizzle
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ta = (rl >> 6) * 128 + h * 64 + (rl & 63);        // tile row of A half h
      const int tb = (rl >> 5) * 64 + h * 32 + (rl & 31);         // tile column of B half h
      off[h][j] = (uint32_t)ta * lda2 + ch;
      off[2 + h][j] = (uint32_t)tb * ldw2 + ch;
    }
  }
  // half x: 0 = A0, 1 = A1, 2 = B0, 3 = B1 of K-tile kt into buffer kt & 1
  auto issue = [&](int x, int kt) {
    uint8_t* dst = smem + (kt & 1) * G3_BUF + x * G3_HALF + wid * 2048;
    const int so = __builtin_amdgcn_readfirstlane(kt * BK * 2);
    const __amdgpu_buffer_rsrc_t rs = x < 2 ? ra : rw;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr3_t)(dst + j * 1024), 16, off[x][j], so, 0, 0);
  };
  // the half scheduled at global phase q (q >= -5): A0(t) at 4t-5, B0(t) 4t-4, B1(t) 4t-3, A1(t) 4t-2,
  // i.e. phase p of K-tile kt issues B0(kt+1), B1(kt+1), A1(kt+1), A0(kt+2) for p = 0, 1, 2, 3
  auto issued = [&](int q) { return q >= -5 && (q + 5) / 4 < nk; };
  auto issue_phase = [&](int p, int kt) {   // p compile-time after unrolling
    if (p == 3) { if (kt + 2 < nk) issue(0, kt + 2); }
    else if (kt + 1 < nk) issue(p == 0 ? 2 : p == 1 ? 3 : 1, kt + 1);
  };

  // ---- fragments
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const uint8_t* half) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int row = wr * 64 + mb * 16 + (lane & 15);
        fa[mb][kk] = *(const u32x4*)(half + row * 128 + swz(row, c) * 16);
      }
    }
  };
  auto read_b = [&](const uint8_t* half, u32x4 (&fb)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int row = wn * 32 + nb * 16 + (lane & 15);
        fb[nb][kk] = *(const u32x4*)(half + row * 128 + swz(row, c) * 16);
      }
    }
  };
  auto cluster = [&](int mh, int nh, const u32x4 (&fb)[2][2]) {   // one quadrant x K 64: 16 MFMAs
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mh * 4 + mb][nh * 2 + nb] = mfma16<BF>(fb[nb][kk], fa[mb][kk], acc[mh * 4 + mb][nh * 2 + nb]);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: halves of phases -5 .. -1, retire those phase 0 reads (A0(0), B0(0))
  issue(0, 0);
  issue(2, 0);
  issue(3, 0);
  issue(1, 0);
  if (nk > 1) issue(0, 1);
  wait_vm_halves((int)issued(-3) + (int)issued(-2) + (int)issued(-1));
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const uint8_t* buf = smem + (kt & 1) * G3_BUF;
    const int q0 = kt * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = q0 + p;
      if (p == 0) { read_a(buf + 0 * G3_HALF); read_b(buf + 2 * G3_HALF, fb0); }
      else if (p == 1) read_b(buf + 3 * G3_HALF, fb1);
      else if (p == 2) read_a(buf + 1 * G3_HALF);
      issue_phase(p, kt);
      // retire every half issued up to phase q-3: all that phase q+1 reads
      wait_vm_halves((int)issued(q) + (int)issued(q - 1) + (int)issued(q - 2));
      __builtin_amdgcn_s_barrier();
      if (p == 0) cluster(0, 0, fb0);
      else if (p == 1) cluster(0, 1, fb1);
      else if (p == 2) cluster(1, 1, fb1);
      else cluster(1, 0, fb0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();   // balance group 1's extra barrier

  if (g.debug & 1) {
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
    return;
  }
  epilogue<BF, EPI, G3_BM, G3_BN, 2, 4, 2>(g, acc, m0, n0, wr, wn, lane);
  (void)sizeof(C);
}

template <bool BF, int EPI>
hipError_t launch3(const GemmArgs& g, hipStream_t s) {
  auto kern = gemm3_kernel<BF, EPI>;
  static unsigned dev_done = 0;   // >64 KiB dynamic LDS needs the opt-in attribute, once per device
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  const int tiles = ((g.N + G3_BN - 1) / G3_BN) * ((g.M + G3_BM - 1) / G3_BM);
  kern<<<dim3(tiles), dim3(512), G3_LDS, s>>>(g);
  return hipGetLastError();
}

template <bool BF>
hipError_t by_epi3(int epi, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return launch3<BF, EPI_STORE>(g, s);
    case EPI_GELU: return launch3<BF, EPI_GELU>(g, s);
    case EPI_RESID: return launch3<BF, EPI_RESID>(g, s);
    case EPI_PATCH: return launch3<BF, EPI_PATCH>(g, s);
    case EPI_SCORE: return launch3<BF, EPI_SCORE>(g, s);
    case EPI_FILTER: return launch3<BF, EPI_FILTER>(g, s);
    case EPI_STORE_LN: return launch3<BF, EPI_STORE_LN>(g, s);
    case EPI_GELU_LN: return launch3<BF, EPI_GELU_LN>(g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t gemm3_launch(bool bf16, int epi, const GemmArgs& g, hipStream_t s) {
  if (g.m_dev) return hipErrorInvalidValue;   // varlen rows: gemm_kernel / G2 only
  if (g.M > 0 && (int64_t)g.lda * 2 * 256 > 0x7FFFFFF0LL) return hipErrorInvalidValue;   // descriptor range
  return bf16 ? by_epi3<true>(epi, g, s) : by_epi3<false>(epi, g, s);
}
}  // namespace clm
