// Host-callable launchers of the gfx950 kernels in k_*.hip.
#pragma once
#include "clm_common.hpp"

namespace clm {

// ---------------------------------------------------------------- GEMM ------
// C[M,N] = A[M,K] . W[N,K]^T  (both operands K-contiguous, nn.Linear layout),
// bf16 or fp16 operands, fp32 accumulate, fused epilogue. K % 64 == 0, or K % 64 == 32 (gemm_kernel
// configs 0-7 without split-K, and gemm_attn): every operand row must then be readable (and finite)
// to round_up(K, 64) -- the last K-step's DMA moves 64 columns, its MFMAs use the first 32.
enum Epi {
  EPI_STORE = 0,  // out16[m,n] = acc + bias[n]
  EPI_GELU = 1,   // out16[m,n] = quick_gelu(acc + bias[n])
  EPI_RESID = 2,  // outf[m,n] += acc + bias[n]            (fp32 residual stream)
  EPI_PATCH = 3,  // outf[b*(G+1)+1+p, n] = acc + aux[(1+p)*aux_ld + n], m = b*G+p
  EPI_SCORE = 4,  // outf[m,n] = acc * rscale[m] * cscale[n]  (cosine scores)
  EPI_FILTER = 5   // s = acc*rscale[m]*cscale[n]; if s >= theta[m]: append (s, base+n) to row m's
                   // candidate list (atomic slot in cnt[m], capacity cap)
};
constexpr bool epi_stores16(int e) { return e == EPI_STORE || e == EPI_GELU; }
constexpr bool epi_gelu(int e) { return e == EPI_GELU; }

struct GemmArgs {
  const u16* A; int64_t lda;
  const u16* W; int64_t ldw;
  int M, N, K;
  void* out; int64_t ldo;
  const float* bias;
  const float* aux; int64_t aux_ld; int group;
  const float* rscale; const float* cscale;
  // EPI_FILTER
  const float* theta; int64_t theta_ld; int* cnt; float* cand_s; int64_t* cand_i; int cap; int64_t base;
  // optional: order keys {min, max} of cscale[0, N) (value_bounds); lets a wave whose largest
  // accumulator cannot reach any of its rows' thresholds skip the per-element filter
  const unsigned* cbound;
  int m_fastest;   // tile order: 1 = consecutive workgroups walk M (share one W tile)
  // split-K (gemm_kernel configs only, EPI_SCORE as the fp32 partial store): ksplit > 1 cuts K
  // into ksplit equal slices; slice s of every tile writes out + s * split_stride
  int ksplit; int64_t split_stride;
  // EPI_SCORE: 1 = store the scores as fp16 rounded toward -inf (f16_down: never above the fp32
  // score, so a k-th largest taken over them bounds the fp32 one from below), out as u16 [M, ldo];
  // 2 (gemm_kernel config 1 only, N % 256 == 0) = one fp16 (rounded down) per 4 consecutive
  // columns, their maximum, out as u16 [M, ldo >= N / 4] in a per-tile permuted column order
  int out16;
  // varlen rows (packed text tower): if set, the row count is *m_dev (device-resident, <= M, which
  // sizes the grid), so a captured graph replays with data-dependent row counts
  const int* m_dev;
  int debug;       // diagnostics only: 1 = skip the epilogue (accumulators kept live), 2 = drop its
                   // stores, 4 = one tile per workgroup (non-persistent grid)
};

hipError_t gemm(bool bf16, int epi, const GemmArgs& g, hipStream_t s);
// Few-row residual GEMM (the pruned last layer: M = pooled rows): out[m,n] += acc + bias with K cut
// into `slices` (deterministic: the fp32 partials [slices][M][N] go to ws and are summed in slice
// order by one reduce kernel, so a row's result does not depend on M). slices must divide K / 64.
hipError_t gemm_splitk_resid(bool bf16, const GemmArgs& g, int slices, float* ws, hipStream_t s);
// fp32 workspace bytes gemm_splitk_resid needs
inline size_t gemm_splitk_ws_bytes(int M, int N, int slices) { return (size_t)slices * M * N * 4; }
// explicit tile configuration (config < 0: heuristic); configs: k_gemm.hip launch_id.
// GEMM_CFG_SPLITK: the 128 x 64 tile (4 waves), for few-row GEMMs (the pooled last layer)
constexpr int GEMM_CFG_SPLITK = 2;
// GEMM_CFG_SKINNY: 64 x 64 tiles (4 waves), for N <= 64 (the unmerged-LoRA down-projections): twice
// the workgroups of 128 x 64 over the same rows
constexpr int GEMM_CFG_SKINNY = 12;
hipError_t gemm_cfg(bool bf16, int epi, int config, const GemmArgs& g, hipStream_t s);
int gemm_num_configs();
// host-side hint for the tile heuristic of the calling thread: true while two towers are being
// launched on concurrent streams (clm_encode_pair). Then the RESID / PATCH GEMMs keep the
// 192x128 / 128x192 tiles, whose single round leaves ~20 % of the workgroup slots to the
// other stream; alone, the slot-filling 160x128 tiles are faster (profiles/r02_v4_gemm_160x128.txt)
void gemm_set_concurrent(bool on);

// ----------------------------------------------------------- row ops -------
// LayerNorm over rows of a fp32 matrix, one wave per row.
//   mode 0: x = src rows                         (src = h)
//   mode 1: x = tok[ids[r]] + pos[r % L]         (text embedding gather), h written
// If g2 != null: h_out = LN(x; g1,b1) is written to hf (fp32) and y = LN(h_out; g2,b2)
// else: (mode 1 writes hf = x) y = LN(x; g1,b1).
// y (compute dtype) gets row stride ldy.
struct LnArgs {
  int mode;
  const float* src; int64_t lds;       // mode 0 source rows
  const int32_t* ids; const float* tok; const float* pos; int L;   // mode 1
  float* hf; int64_t ldh;              // fp32 output rows (may alias src)
  const float* g1; const float* b1;
  const float* g2; const float* b2;
  u16* y; int64_t ldy;
  int M, d; float eps;
  // varlen rows (packed text tower): rows r < *m_dev only (M sizes the grid); mode 1 reads token
  // rowmap[r] = b * L + position of the padded [B, L] ids instead of r
  const int* m_dev; const int* rowmap;
};
hipError_t layernorm(bool bf16, const LnArgs& a, hipStream_t s);

// shortest-edge bicubic resize + centre crop (k_image.hip), PIL / CLIPImageProcessor arithmetic.
// Per image: source HWC RGB bytes at src + src_off (row stride 3 W); the crop needs source rows
// [r0, r0 + rows), whose horizontally resampled S columns go to tmp + tmp_off ([rows][S][3]).
// coef + coef_off holds int32 xmin[S] | xn[S] | ymin[S] (relative to r0) | yn[S] | xk[S][kh] |
// yk[S][kv] (22-bit fixed-point taps).
struct ResizeDesc {
  int64_t src_off;
  int64_t tmp_off;
  int32_t W, r0, rows, kh, kv, coef_off;
};
hipError_t resize_crop(const uint8_t* src, const ResizeDesc* desc, int n, int S, int max_rows,
                       const int32_t* coef, uint8_t* tmp, uint8_t* out, hipStream_t s);

// n synthetic uint8 [S, S, 3] images, image i's bytes a function of (seed, row0 + i) only
// (S * S * 3 % 16 == 0; out 16-B aligned)
hipError_t synth_images(uint64_t seed, int64_t row0, int n, int S, uint8_t* out, hipStream_t s);

// patchify + (u8 rescale/normalise via lut | f32 copy) -> P[B*G*G, Kp] (compute dtype)
hipError_t patchify(bool bf16, const void* pix, int layout, int B, int S, int p, int C,
                    const float* lut /*[C*256]*/, u16* P, int Kp, hipStream_t s);

// h[b*T + 0, :] = cls + pos[0]
hipError_t write_cls(float* h, int64_t ldh, int B, int T, int d, const float* cls,
                     const float* pos, hipStream_t s);

// pooled row -> LN -> projection (fp32, projT [d, D]) -> optional L2 norm -> out
//   ids == null: row b*T (CLS); else row b*T + (first eos in ids[b]) (argmax if eos==2)
//   tmp: [B, D] fp32 workspace
// Last-layer pruning: hc[b] = h[b*T + prow_b], Oc[b][:d] = O[b*T + prow_b][:d], prow_b the
// pooled row (0, or the first EOS of ids).
// offs (varlen packed text rows, see text_plan): item b's pooled row is offs[b + 1] - 1 (its last
// live row, the first EOS) instead of b * T + pooled_row(ids)
hipError_t gather_pooled(const float* h, int64_t ldh, const u16* O, int64_t ldo, int B, int T, int d,
                         const int32_t* ids, int eos, float* hc, u16* Oc, int64_t ldoc, hipStream_t s,
                         const int* offs = nullptr);
hipError_t pool_project(const float* h, int64_t ldh, int B, int T, int d, const int32_t* ids,
                        int eos, const float* g, const float* bta, float eps, const float* projT,
                        int D, float* tmp, void* out, int out_dtype, int normalize, hipStream_t s,
                        const int* offs = nullptr);
// Varlen text plan (causal text tower, CLIPTextTransformer pools the first EOS row: rows after it
// cannot reach the pooled output). Per caption b of ids [B, L]: lens[b] = pooled row + 1 live
// rows, offs[b] = their exclusive prefix sum (offs[B] = total), rowmap[offs[b] + p] = b * L + p,
// the fused-attention tiles (whole captions, <= 256 rows each; tiles[t] = first caption |
// captions << 16) and counts = {live rows, tiles}. Three launches (lengths: a wave per caption;
// prefix / tiles: one workgroup; row map: a workgroup per 16 captions); B <= 4096.
hipError_t text_plan(const int32_t* ids, int B, int L, int eos, int* lens, int* offs, int* rowmap, int* tiles,
                     int* counts, hipStream_t s);

// ----------------------------------------------------------- attention -----
// qkv [B*T, 3d] (q pre-scaled by head_dim^-0.5), out [B*T, ldo] compute dtype.
// q_log2e: q carries log2(e) as well (the scores arrive in the log2 domain); valid only where
// attention_folds_log2e(bf16, causal, T) -- the kernel chosen for that shape takes that form
// (k_attn.hip attn_long_dma_kernel<true, true>: bf16, non-causal, T > 128) -- else
// hipErrorInvalidValue. The engine folds log2 e into the q_proj weights of such towers.
bool attention_folds_log2e(bool bf16, bool causal, int T);
hipError_t attention(bool bf16, bool causal, const u16* qkv, int64_t ldq, u16* out, int64_t ldo,
                     int B, int T, int H, int d, hipStream_t s, bool q_log2e = false);
// fused q/k/v projection + attention (k_gemm_attn.hip), T <= 128: out = attention(X . Wqkv^T +
// bias) without materialising QKV; bit-identical to gemm(EPI_STORE) + attention()
bool gemm_attn_supported(int T, int H, int d, int K);
hipError_t gemm_attn(bool bf16, bool causal, const u16* X, int64_t ldx, const u16* W, int64_t ldw, const float* bias,
                     u16* out, int64_t ldo, int B, int T, int H, int d, int K, hipStream_t s);
// the same over packed variable-length sequences (text_plan's lens / offs / tiles / counts; B
// sequences of <= L <= 128 rows, rows X[offs[b] ..]); grid sized for the worst case
hipError_t gemm_attn_varlen(bool bf16, bool causal, const u16* X, int64_t ldx, const u16* W, int64_t ldw,
                            const float* bias, u16* out, int64_t ldo, int B, int L, int H, int d, int K,
                            const int* lens, const int* offs, const int* tiles, const int* counts, hipStream_t s);
// one fused q/k/v + attention problem (gemm_attn / gemm_attn_varlen); lens == null: fixed length T
struct AttnProblem {
  const u16* X; int64_t ldx; const u16* W; int64_t ldw; const float* bias; u16* out; int64_t ldo;
  int B, T, H, d, K;
  const int *lens, *offs, *tiles, *counts;   // varlen (text_plan) or null
};

// ----------------------------------------------------------- search --------
// rows f32|f16 [n, dim] -> fp16 dst + fp32 inverse norms of the fp16-rounded rows
// (norm_src = 0) or of the source rows (norm_src = 1); norm_src = 2: dst = fp16(v / ||v||)
// and the inverse norms of those rounded unit rows
hipError_t rows_to_f16(const void* src, int src_dtype, int64_t n, int dim, u16* dst,
                       float* inv_norm, hipStream_t s, int norm_src);
// per-row top-k over scores [nq, C] (row stride lds): out sorted by (score desc,
// idx asc); idx = base + column.
hipError_t topk_rows(const float* scores, int64_t lds, int64_t nq, int64_t C, int k,
                     int64_t base, float* out_s, int64_t* out_i, int64_t ldo, hipStream_t s);
// top-k of any k (k > 1024, or candidate lists longer than one LDS sort): exact k-th key by radix
// select, the k composites collected, sorted (LDS runs + merge passes), emitted. idx == null: the
// global index of column j is base + j; else idx[row * ldi + j] (< 0: an empty slot, never taken
// before a score). Rows with fewer than k entries end in (-inf, -1). nq <= 65535; ws of
// topk_any_ws_bytes(nq, k) device bytes.
size_t topk_any_ws_bytes(int64_t nq, int k);
hipError_t topk_any(const float* scores, int64_t lds, const int64_t* idx, int64_t ldi, int64_t nq, int64_t C, int k,
                    int64_t base, float* out_s, int64_t* out_i, int64_t ldo, void* ws, hipStream_t s);
// cnt[q] = number of scores in row q [C] (row stride lds) that are >= th[q]
hipError_t count_ge(const float* scores, int64_t lds, int64_t nq, int64_t C, const float* th, int* cnt, hipStream_t s);
// the same over fp16 scores (GemmArgs::out16 score matrices)
hipError_t count_ge16(const u16* scores, int64_t lds, int64_t nq, int64_t C, const float* th, int* cnt, hipStream_t s);
hipError_t kth_thresholds16(const u16* scores, int64_t lds, int64_t nq, int64_t C, int k, float margin, float* th,
                            hipStream_t s);
// merge `parts` candidate lists per row: in [nq, parts*k_in] -> out [nq, k]
hipError_t topk_merge(const float* in_s, const int64_t* in_i, int64_t nq, int parts, int k_in,
                      int k, float* out_s, int64_t* out_i, hipStream_t s);
hipError_t l2_normalize_rows(float* rows, int64_t n, int dim, hipStream_t s);
hipError_t fuse_rows(const float* a, float wa, const float* b, float wb, int64_t n, int dim, float* out,
                     hipStream_t s);
// strided row sample: out[s] = rows[s * n / S] (fp16 rows + fp32 inverse norms)
hipError_t sample_rows(const u16* rows, const float* inv, int64_t n, int dim, int64_t S, u16* out_rows,
                       float* out_inv, hipStream_t s);
hipError_t f32_to_f16_rows(const float* src, int64_t n, int dim, u16* dst, hipStream_t s);
hipError_t f16_to_f32_rows(const u16* src, int64_t n, int dim, float* dst, hipStream_t s);

// exact (fp64) cosine re-scoring (k_search.hip): every path scores a (query, row) pair through
// one device routine, so the exact scores are bit-identical across paths
hipError_t query_norms(const float* q, int64_t nq, int dim, double* qn, hipStream_t s);
// out[qi, j] = fp32(cos64(q[qi], rows[j])), rows f32 or f16 [rn, dim]
hipError_t exact_scores(const float* q, const double* qn, int64_t nq, const void* rows, bool rows_f16, int64_t rn,
                        int dim, float* out, int64_t ldo, hipStream_t s);
// per query: candidates (fp16-pass score, global index) [nq, cap] with counts cnt[nq] -> keep
// those within `margin` of the k-th, re-score exactly, emit top k by (score desc, index asc);
// queries with cnt > cap are left untouched
hipError_t rescore_select(const float* cand_s, const int64_t* cand_i, const int* cnt, int cap, const float* q,
                          const double* qn, int dim, const void* rows, bool rows_f16, int64_t offset, float margin,
                          int64_t nq, int k, float* out_s, int64_t* out_i, hipStream_t s);
// overflowed lists: candidates [nq, cap] (global indices; cnt[q] <= cap) -> per chunk of
// RESCORE_WIDE_CHUNK candidates the top k by (exact score desc, index asc), part_s / part_i
// [nq, ceil(cap / chunk) * k] (-inf / -1 padded), merged by topk_merge; ceil(cap / chunk) * k <= 8192
constexpr int RESCORE_WIDE_CHUNK = 4096;
hipError_t rescore_wide(const int64_t* cand_i, const int* cnt, int64_t cap, const float* q, const double* qn, int dim,
                        const void* rows, bool rows_f16, int64_t offset, int64_t nq, int k, float* part_s,
                        int64_t* part_i, hipStream_t s);
// dst row j = src row idx[j] (scatter: dst row idx[j] = src row j), row_bytes per row
hipError_t gather_rows(const void* src, int64_t src_stride, const int64_t* idx, int64_t n, int64_t row_bytes,
                       void* dst, int64_t dst_stride, bool scatter, hipStream_t s);
// th[q] = ts[q * ld + k - 1] - margin
hipError_t filter_thresholds(const float* ts, int64_t ld, int64_t nq, int k, float margin, float* th, hipStream_t s);
// th[q] = (k-th largest of scores row q [C], duplicates counted) - margin, bit-identical to
// topk_rows + filter_thresholds; k <= 8, C >= k
hipError_t kth_thresholds(const float* scores, int64_t lds, int64_t nq, int64_t C, int k, float margin, float* th,
                          hipStream_t s);
// keys[0] / keys[1] = order key (float_key) of min / max over v[0, n); a NaN anywhere makes the
// decoded min or max NaN. keys: 2 device u32
hipError_t value_bounds(const float* v, int64_t n, unsigned* keys, hipStream_t s);
// small-batch search scan (k_search.hip scan16_kernel): nq <= 16 unit-rounded fp16 queries q16
// [nq, dim] (inverse norms qinv) against the fp16 index rows [N, dim] (inverse norms inv), one
// streaming pass: out [N, ldo] = fp16-pass scores (acc * qinv * inv), row-major with the queries
// of a row contiguous (ldo = 1, 2, 4, 8 or 16 >= nq), cmax [nq, nchunk] = each 256-row chunk's
// largest score (nchunk = ceil(N / 256)); dim % 64 == 0, 64 <= dim <= 1024
// wtop (optional) [nq, ldw]: wave w's 8 largest chunk maxima per query at columns 8 w .. 8 w + 7
// (-inf padded); scan16_waves gives the wave count W (ldw >= 8 W)
struct Scan16Args {
  const u16* rows; const float* inv; int64_t N; int dim;
  const u16* q16; const float* qinv; int nq;
  float* out; int64_t ldo;
  float* cmax; int64_t nchunk;
  float* wtop; int64_t ldw;
};
hipError_t scan16(const Scan16Args& a, hipStream_t s);
void scan16_shape(int dim, int* nw, int* depth);
int scan16_grid(int64_t nchunk, int nw, int cus);
int64_t scan16_waves(int64_t nchunk, int dim);
// append every (score, base + row) of column q of scores [C rows, ldq] (ldq a power of two, 1..16,
// >= nq) at or above th[q] to q's candidate list [cap] (cnt[q] counts them all)
hipError_t collect_ge(const float* scores, int ldq, int nq, int64_t C, const float* th, int* cnt, int cap, float* cs,
                      int64_t* ci, int64_t base, hipStream_t s);
__host__ __device__ inline unsigned float_key(float f) {
  const unsigned b = __builtin_bit_cast(unsigned, f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__host__ __device__ inline float key_float(unsigned k) {
  return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

}  // namespace clm
