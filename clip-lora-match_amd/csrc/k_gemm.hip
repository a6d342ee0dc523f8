// MFMA GEMM for gfx950: C[M,N] = A[M,K] . W[N,K]^T, bf16/fp16 operands, fp32 accumulate.
//
// Replaces the ATen CPU addmm/conv that the reference runs for every
// nn.Linear / patch-embed conv of the CLIP towers (TF/models/clip/modeling_clip.py:
// 294-297 q/k/v, 332 out_proj, 343-344 fc1/fc2, 148-154 patch conv, and the
// score matmul of src/embedding/search.py:96 / similarity.py:32), with the
// bias, quick-GELU, residual-add, positional-embedding and cosine-scaling
// epilogues fused.
//
// Structure (templated tile BM x BN x 64, WM x WN waves, STAGES-deep LDS ring):
//  * both operand tiles stream HBM/L2 -> LDS by global_load_lds_dwordx4 (16 B per
//    lane, lane-linear 1 KiB per wave-instruction = 8 rows of 128 B); the XOR chunk
//    swizzle is applied to the per-lane SOURCE address so that the ds_read_b128
//    fragment reads (16 rows per lane group) are bank-conflict free;
//  * STAGES = 3: two K-tiles stay in flight across the (raw) barrier, retired by a
//    counted s_waitcnt vmcnt(L) -- never vmcnt(0) in the steady state;
//  * operands are SWAPPED in the MFMA (W rows feed the A port): the 16x16 C-block
//    then has the output row m on the lane and 4 consecutive output columns in the
//    lane's 4 accumulator registers, so every epilogue access is a 4-wide vector
//    (8 B bf16 / 16 B fp32) instead of 2-byte scatter;
//  * workgroup ids are remapped XCD-aware so the N-tiles sharing one A row-panel
//    (and its L2 lines) run on one XCD.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "gemm_common.hpp"

namespace clm {

namespace {
using namespace gemm_detail;
// Persistent: workgroup b walks its tiles (tile_walk, G = gridDim.x <= tiles workgroups), and its LDS-DMA ring runs ACROSS tile boundaries: the first
// K-tiles of tile i+1 are issued before tile i's epilogue, so they land while the epilogue
// runs, and the epilogue's stores drain under tile i+1's main loop (counted vmcnt that
// leaves them in flight). A one-tile-per-workgroup grid is the plain non-persistent GEMM.
template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
__device__ __forceinline__ void gemm_body(const GemmArgs& ga, int bid, int G) {
  using C = Cfg<BM, BN, WM, WN, STAGES>;
  GemmArgs g = ga;   // varlen: the device-resident row count (the grid was sized for ga.M)
  if (g.m_dev) g.M = __builtin_amdgcn_readfirstlane(*g.m_dev);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (g.N + BN - 1) / BN, ntm = (g.M + BM - 1) / BM;
  const int ks = g.ksplit > 1 ? g.ksplit : 1;   // split-K: work unit = (tile, K slice)
  const int ntiles = ntn * ntm * ks;
  const TileWalk tw = tile_walk(ntiles, bid, G);
  if (tw.count <= 0) return;   // varlen: fewer live tiles than the grid
  const int n_my = tw.count;
  // K % 64 == 32 (unmerged LoRA's 32-wide K-extension granule): the last K-step's DMA still moves
  // 64 columns (operand rows are readable to round_up(K, 64)) but only its first 32 are multiplied
  const int nk = (g.K + BK - 1) / BK / ks;
  const bool half_last = (g.K % BK) != 0;
  const int S = n_my * nk;   // K-steps of all this workgroup's tiles, one ring

  auto coords = [&](int i, int& m0, int& n0, int& k0) {
    int t = tw.first + i * tw.stride;
    k0 = 0;
    if (ks > 1) {   // the slices of one tile are adjacent units (same XCD under the remap)
      k0 = (t % ks) * nk * BK;
      t /= ks;
    }
    int tm, tn;
    if (g.m_fastest) {          // every query tile of one index tile back to back (search)
      tm = t % ntm;
      tn = t / ntm;
    } else {                    // grouped raster: GM row-panels x all N-tiles per group, M inner,
                                // so an XCD's concurrent tiles share A panels and W tiles in L2
      const int group = t / (GM * ntn);
      const int first_m = group * GM;
      const int gsz = min(GM, ntm - first_m);
      const int r = t - group * GM * ntn;
      tm = first_m + r % gsz;
      tn = r / gsz;
    }
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // loader state: per-lane DMA sources of the tile being loaded (piece j of this wave covers
  // tile rows (wid*LA + j)*8 .. +8), re-pointed when the ring crosses into the next tile
  const int r8 = lane >> 3, pc = lane & 7;
  const u16* a_src[C::LA];
  const u16* w_src[C::LB];
  auto point = [&](int i) {
    int m0, n0, k0;
    coords(i, m0, n0, k0);
#pragma unroll
    for (int j = 0; j < C::LA; ++j) {
      const int row = (wid * C::LA + j) * 8 + r8;
      a_src[j] = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + k0 + (pc ^ ((row >> 1) & 7)) * 8;
    }
#pragma unroll
    for (int j = 0; j < C::LB; ++j) {
      const int row = (wid * C::LB + j) * 8 + r8;
      w_src[j] = g.W + (int64_t)min(n0 + row, g.N - 1) * g.ldw + k0 + (pc ^ ((row >> 1) & 7)) * 8;
    }
  };
  int ld_i = 0, ld_kt = 0;
  point(0);
  auto stage_next = [&](int buf) {   // DMA of the ring's next K-step into LDS buffer buf
    uint8_t* base = smem + buf * C::STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < C::LA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + ld_kt * BK),
                                       (void*)(base + (wid * C::LA + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < C::LB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(w_src[j] + ld_kt * BK),
                                       (void*)(base + BM * 128 + (wid * C::LB + j) * 1024), 16, 0, 0);
    if (++ld_kt == nk) {
      ld_kt = 0;
      if (++ld_i < n_my) point(ld_i);
    }
  };

  const int wm = wid / WN, wn = wid % WN;
  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < S) stage_next(s);

  // stores a tile end leaves in flight (the ragged scalar path stores in branches: none counted)
  constexpr int E0 = epi_min_stores<EPI, C::TM, C::TN>();
  constexpr int E = E0 + C::L * (STAGES - 2) > 63 ? 63 - C::L * (STAGES - 2) : E0;   // 6-bit vmcnt: over-wait
  const bool vec_epi = (g.N % 4) == 0 && (g.ldo % 4) == 0 && !(g.debug & 1);
  int c_i = 0, c_kt = 0, m0, n0, k0;
  coords(0, m0, n0, k0);
  int since_end = STAGES;   // K-steps since the last tile end
  // residual prefetch (RESID, 2-stage ring): the first PB row-blocks of the residual tile,
  // issued right after the DMA of a tile's last K-step, so their reads land while that K-step
  // computes (resid_prefetch). Only the 128 x 192 tile (TN = 6: the towers' concurrent RESID
  // GEMMs) takes it, one row-block (24 VGPRs + the hoisted bias, no spill): +1.3 % pairs/s in the
  // pair step; on the TN = 4 tiles it measured neutral (192 x 128) or slower (160 x 128, -8 %)
  // (profiles/r03_v6_resid_prefetch_*)
  constexpr int PB = (EPI == EPI_RESID && STAGES == 2 && C::TN == 6) ? 1 : 0;
  constexpr bool PRE = PB > 0;
  constexpr int XP = PB * C::TN;   // prefetch loads: the youngest ops at the next wait
  u32x4 hpre[PRE ? PB : 1][C::TN];
  const bool pre_on = PRE && ks == 1 && nk >= 2 && vec_epi;
  bool hp_pending = false;
  for (int s = 0; s < S; ++s) {
    // retire K-step s's DMA, leaving younger ones in flight: the STAGES-2 later K-steps' DMA
    // and, for STAGES-1 steps after a tile end, that epilogue's stores (the DMA of those steps
    // was issued before the stores; the first DMA issued after them is waited STAGES steps on),
    // or the residual prefetch issued after this step's DMA
    const bool more = s + STAGES - 2 < S;
    ++since_end;
    const bool pe = vec_epi && since_end <= STAGES - 1;
    if (PRE && hp_pending) {   // STAGES == 2: only the XP prefetch loads are younger than DMA(s)
      wait_vmcnt<XP>();
      hp_pending = false;
    } else if (more) {
      if (pe) wait_vmcnt<C::L * (STAGES - 2) + E>();
      else wait_vmcnt<C::L * (STAGES - 2)>();
    } else {
      if (pe) wait_vmcnt<E>();
      else wait_vmcnt<0>();
    }
    lds_barrier();
    if (s + STAGES - 1 < S) stage_next((s + STAGES - 1) % STAGES);
    if constexpr (PRE) {
      if (pre_on && c_kt == nk - 2) {
        resid_prefetch<BM, BN, WM, WN, PRE ? PB : 1>(g, m0, n0, wm, wn, lane, hpre);
        hp_pending = true;
      }
    }
    const uint8_t* sa = smem + (s % STAGES) * C::STAGE_BYTES;
    const uint8_t* sb = sa + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk == 1 && half_last && c_kt == nk - 1) break;
      const int c = kk * 4 + (lane >> 4);
      u32x4 af[C::TM], bw[C::TN];
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb) {
        const int row = wm * (BM / WM) + mb * 16 + (lane & 15);
        af[mb] = *(const u32x4*)(sa + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < C::TN; ++nb) {
        const int row = wn * (BN / WN) + nb * 16 + (lane & 15);
        bw[nb] = *(const u32x4*)(sb + row * 128 + swz(row, c) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < C::TM; ++mb)
#pragma unroll
        for (int nb = 0; nb < C::TN; ++nb) acc[mb][nb] = mfma16<BF>(bw[nb], af[mb], acc[mb][nb]);
    }
    if (++c_kt == nk) {
      since_end = 0;
      if (g.debug & 1) {   // timing diagnostic: main loop only
#pragma unroll
        for (int mb = 0; mb < C::TM; ++mb)
#pragma unroll
          for (int nb = 0; nb < C::TN; ++nb) asm volatile("" ::"v"(acc[mb][nb]));
      } else {
        if constexpr (PRE) {
          if (pre_on) epilogue<BF, EPI, BM, BN, WM, WN, STAGES, PB>(g, acc, m0, n0, wm, wn, lane, 0, hpre);
          else epilogue<BF, EPI, BM, BN, WM, WN, STAGES>(g, acc, m0, n0, wm, wn, lane, 0);
        } else {
          epilogue<BF, EPI, BM, BN, WM, WN, STAGES>(g, acc, m0, n0, wm, wn, lane,
                                                    ks > 1 ? (int64_t)(k0 / (nk * BK)) * g.split_stride : 0);
        }
      }
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c_kt = 0;
      if (++c_i < n_my) coords(c_i, m0, n0, k0);
    }
  }
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(WM * WN * 64, (Cfg<BM, BN, WM, WN, STAGES>::WAVES_PER_EU)) void gemm_kernel(GemmArgs ga) {
  gemm_body<BF, EPI, BM, BN, WM, WN, STAGES>(ga, blockIdx.x, gridDim.x);
}

template <bool BF, int EPI, int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_cfg(const GemmArgs& g, hipStream_t s) {
  using C = Cfg<BM, BN, WM, WN, STAGES>;
  auto kern = gemm_kernel<BF, EPI, BM, BN, WM, WN, STAGES>;
  static unsigned dev_done = 0;   // >64 KiB dynamic LDS needs the opt-in attribute, once per device
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  // persistent grid: at most one workgroup per resident slot (occupancy x CUs, per device)
  static int slots[32] = {};
  int& sl = slots[dev & 31];
  if (sl == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, C::NT, C::LDS) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
    sl = per_cu * cus;
  }
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM) * (g.ksplit > 1 ? g.ksplit : 1);
  const int nwg = (g.debug & 4) ? tiles : std::min(tiles, sl);   // debug bit 2: one tile per workgroup
  kern<<<dim3(nwg), dim3(C::NT), C::LDS, s>>>(g);
  return hipGetLastError();
}

// tile configurations (index = GemmArgs-independent id, also the `config` of clm_gemm); every one
// is picked by pick_config for some shape. Configs that never won inside the encode pipeline
// (other gemm_kernel / G2 tiles, G2's deferred-store and 3-buffer twins, the 256 x 256
// eight-phase G3) were removed; their A/B records stay under profiles/ (r01_v8_*, r01_v10_*,
// r02_v4_*, r02_v9_tile_family_ab.txt).
template <bool BF, int EPI>
hipError_t launch_id(int id, const GemmArgs& g, hipStream_t s) {
  switch (id) {
    case 0: return launch_cfg<BF, EPI, 128, 128, 2, 2, 2>(g, s);
    case 1: return launch_cfg<BF, EPI, 256, 256, 4, 2, 2>(g, s);
    case 2: return launch_cfg<BF, EPI, 128, 64, 4, 1, 3>(g, s);
    case 3: return launch_cfg<BF, EPI, 128, 192, 2, 2, 2>(g, s);
    case 4: return launch_cfg<BF, EPI, 192, 128, 2, 2, 2>(g, s);
    case 5: return launch_cfg<BF, EPI, 256, 128, 4, 2, 2>(g, s);
    case 6: return launch_cfg<BF, EPI, 128, 256, 2, 4, 2>(g, s);
    case 7: return launch_cfg<BF, EPI, 160, 128, 2, 2, 2>(g, s);
    case 8: case 9: case 10: case 11: return gemm2_launch(BF, EPI, id, g, s);
    case 12: return launch_cfg<BF, EPI, 64, 64, 4, 1, 3>(g, s);
    case 13: case 14: return gemm4_launch(BF, EPI, id, g, s);
    default: return hipErrorInvalidValue;
  }
}

constexpr int NCFG = 15;
static_assert(GEMM_CFG_SKINNY == 12, "config 12 is the 64 x 64 tile");
static_assert(GEMM_CFG_SPLITK == 2, "config 2 is the 128 x 64 tile");

// Tile choice: a cost model per kernel family, time(cfg) ~ rounds(cfg) x round_cost(cfg),
// rounds = ceil(tiles / resident workgroups), round_cost = BM*BN*(workgroups per CU) /
// efficiency(cfg). Which family serves which epilogue was measured INSIDE the encode pipeline
// (tools/trace_cfgs.sh: every config forced for every GEMM of the sequential encode under a
// kernel trace; profiles/r01_v8_pipeline_cfg_sweep.jsonl) -- a warm-cache repeated-GEMM sweep
// ranks them differently:
//  * the quick-GELU fc1 GEMMs -> G2 (k_gemm2.hip): 8-10 % faster there in every pipeline
//    trace (its epilogue VALU overlaps the co-resident waves' MFMAs better); efficiencies
//    fitted on the ViT-B/32 qkv GEMM;
//  * everything else -> gemm_kernel: qkv (STORE) ties or loses on G2 inside the pipeline
//    although G2 wins by ~13 % in a warm-cache repeated-GEMM sweep; the narrow fp32
//    read-modify-write outputs (out_proj / fc2 RESID, patch PATCH) take the 2-workgroups-per-CU
//    tiles (192x128 / 128x192), whose co-resident workgroups overlap one tile's residual round
//    trip with the other's MFMAs.
// $CLM_GEMM_CFG forces a config (tools and tests).
struct CfgModel { int id, bm, bn, wg_per_cu; double eff; };
constexpr CfgModel MODELS_G2[] = {
  {8, 256, 192, 1, 2.569}, {9, 256, 128, 1, 2.349}, {10, 192, 256, 1, 2.521}, {11, 128, 256, 1, 2.340}};
// 160x128 (config 7): the N = 512 / 768 RESID / PATCH shapes fill one round of 2-WG/CU slots
// (480 / 496 tiles of 512, against 402 / 412 with 192x128): v_out 28.7 vs 32.0 µs, v_fc2 67.7
// vs 74.9, t_out 24.0 vs 25.8, t_fc2 49.5 vs 53.7 (profiles/r02_v4_gemm_160x128.txt) -- when the
// GEMM has the chip to itself; while the two towers run concurrently (gemm_set_concurrent) it is
// skipped: the 192x128 / 128x192 single round leaves ~20 % of the slots to the other stream
// (profiles/r02_v9_tile_family_ab.txt)
constexpr CfgModel MODELS[] = {
  {0, 128, 128, 2, 0.975}, {1, 256, 256, 1, 1.18}, {3, 128, 192, 2, 0.955}, {4, 192, 128, 2, 0.955},
  {5, 256, 128, 1, 1.025}, {6, 128, 256, 1, 1.056}, {7, 160, 128, 2, 0.93}};
thread_local bool g_concurrent = false;
// $CLM_GEMM_CONCURRENT=1: pick the concurrent-tower tiles on every launch (the PMC passes of
// tools/pmc.sh serialise the step but must count the tiles the timed two-stream step runs)
bool env_concurrent() {
  static const int v = getenv("CLM_GEMM_CONCURRENT") ? atoi(getenv("CLM_GEMM_CONCURRENT")) : 0;
  return v != 0;
}
template <int NM>
int pick_from(const CfgModel (&models)[NM], int M, int N) {
  const int skip = (g_concurrent || env_concurrent()) ? 7 : -1;
  int best = models[0].id;
  double best_cost = 1e300;
  for (const CfgModel& c : models) {
    if (c.id == skip) continue;
    const int64_t tiles = (int64_t)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    const int64_t slots = 256LL * c.wg_per_cu;
    const int64_t rounds = (tiles + slots - 1) / slots;
    const double cost = rounds * (double)c.bm * c.bn * c.wg_per_cu / c.eff;
    if (cost < best_cost * 0.999) { best_cost = cost; best = c.id; }
  }
  return best;
}
int pick_config(int epi, int M, int N) {
  static int forced = -2;
  if (forced == -2) {
    const char* e = getenv("CLM_GEMM_CFG");
    forced = e ? atoi(e) : -1;
  }
  if (forced >= 0 && forced < NCFG) return forced;
  // the search's filter GEMM (K = 512, no stores): G2's loop, 256 x 192 -- configs[4] search
  // 95.9 k QPS vs 86.4 k with gemm_kernel 256 x 256 (profiles/r04_v7_search_cfg_ab.txt)
  if (epi == EPI_FILTER) return pick_from(MODELS_G2, M, N);
  // Large M x N plain stores (>= 4 full rounds of 256 x 256 tiles, e.g. ViT-L/14@336 batch 128: qkv
  // 73,856 x 3,072): G4's one-wave-per-SIMD 256 x 256 tile (config 13), 439 vs 457 us for config 1
  // with its stores (profiles/r06_v3_g4_probe.jsonl; $CLM_G4_STORE=0 keeps config 1)
  static const int g4_store = getenv("CLM_G4_STORE") ? atoi(getenv("CLM_G4_STORE")) : 1;
  if (epi == EPI_STORE && g4_store && (int64_t)((M + 255) / 256) * ((N + 255) / 256) >= 4 * 256) return 13;
  if (epi != EPI_GELU) return pick_from(MODELS, M, N);
  // Large M (>= 4 full rounds of 256 x 256 tiles, e.g. ViT-L/14@336 batch 128: fc1 73,856 x 4,096):
  // quantisation no longer favours G2's narrower tiles: gemm_kernel 256 x 256 takes 636 us there
  // against 874 for G2 256 x 128 (tools/quant_probe.py, profiles/r02_v6_l14_gemm_probe.txt)
  if ((int64_t)((M + 255) / 256) * ((N + 255) / 256) >= 4 * 256) return 1;
  return pick_from(MODELS_G2, M, N);
}

template <bool BF>
hipError_t dispatch(int epi, int id, const GemmArgs& g, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: return launch_id<BF, EPI_STORE>(id, g, s);
    case EPI_GELU: return launch_id<BF, EPI_GELU>(id, g, s);
    case EPI_RESID: return launch_id<BF, EPI_RESID>(id, g, s);
    case EPI_PATCH: return launch_id<BF, EPI_PATCH>(id, g, s);
    case EPI_SCORE: return launch_id<BF, EPI_SCORE>(id, g, s);
    case EPI_FILTER: return launch_id<BF, EPI_FILTER>(id, g, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

int gemm_num_configs() { return NCFG; }

hipError_t gemm_cfg(bool bf16, int epi, int config, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K <= 0 || (g.K % 32) != 0 || (g.lda % 8) != 0 || (g.ldw % 8) != 0) return hipErrorInvalidValue;
  int id = config >= 0 ? config : pick_config(epi, g.M, g.N);
  if (g.K % BK) {   // the half last K-step: gemm_kernel configs without split-K only
    if (g.ksplit > 1) return hipErrorInvalidValue;
    if (id >= 8 && id <= 11) {
      if (config >= 0) return hipErrorInvalidValue;
      id = pick_from(MODELS, g.M, g.N);
    }
  }
  // G4 (configs 13 / 14): STORE / GELU (N, ldo multiples of 8) / RESID (of 4), whole K-steps
  if (id >= 13 && !gemm4_supports(epi, g)) {
    if (config >= 0) return hipErrorInvalidValue;
    id = pick_from(MODELS, g.M, g.N);
  }
  return bf16 ? dispatch<true>(epi, id, g, s) : dispatch<false>(epi, id, g, s);
}

hipError_t gemm(bool bf16, int epi, const GemmArgs& g, hipStream_t s) {
  if (g.ksplit > 1) return hipErrorInvalidValue;   // split-K: gemm_splitk_resid only
  return gemm_cfg(bf16, epi, -1, g, s);
}

namespace {
// out[m, n] += sum_s ws[s][m][n] (slice order) + bias[n]: the RESID epilogue's arithmetic,
// h + (acc + bias), with acc summed over the K slices; 4 columns per thread
__global__ __launch_bounds__(256) void splitk_resid_kernel(const float* ws, int slices, int M, int N, const float* bias,
                                                          float* out, int64_t ldo) {
  const int n4 = N / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)M * n4) return;
  const int m = (int)(i / n4), n = (int)(i - (int64_t)m * n4) * 4;
  const int64_t stride = (int64_t)M * N;
  float4 acc = *(const float4*)(ws + (int64_t)m * N + n);
  for (int s = 1; s < slices; ++s) {
    const float4 p = *(const float4*)(ws + s * stride + (int64_t)m * N + n);
    acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
  }
  const float4 b = bias ? *(const float4*)(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4* o = (float4*)(out + (int64_t)m * ldo + n);
  float4 h = *o;
  h.x = h.x + (acc.x + b.x); h.y = h.y + (acc.y + b.y); h.z = h.z + (acc.z + b.z); h.w = h.w + (acc.w + b.w);
  *o = h;
}
}  // namespace

hipError_t gemm_splitk_resid(bool bf16, const GemmArgs& g, int slices, float* ws, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (slices < 1 || g.K <= 0 || g.K % (BK * slices) || (g.N % 4) || (g.ldo % 4) || !ws) return hipErrorInvalidValue;
  GemmArgs p = g;   // slice partials: EPI_SCORE with no scales stores acc * 1 * 1 = acc exactly
  p.out = ws; p.ldo = g.N; p.bias = nullptr; p.rscale = nullptr; p.cscale = nullptr;
  p.ksplit = slices; p.split_stride = (int64_t)g.M * g.N;
  // 128 x 64 tiles (4 waves): the few rows still spread over many workgroups
  hipError_t e = gemm_cfg(bf16, EPI_SCORE, GEMM_CFG_SPLITK, p, s);
  if (e != hipSuccess) return e;
  const int64_t n = (int64_t)g.M * (g.N / 4);
  splitk_resid_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(ws, slices, g.M, g.N, g.bias, (float*)g.out, g.ldo);
  return hipGetLastError();
}

void gemm_set_concurrent(bool on) { g_concurrent = on; }

}  // namespace clm
