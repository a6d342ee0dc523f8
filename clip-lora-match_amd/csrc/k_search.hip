// Exact top-k selection for the cosine search (gfx950).
//
// Replaces torch.topk(sims, k, largest=True, sorted=True) of
// src/embedding/search.py:98-99 and similarity.py:57 over the score rows the
// EPI_SCORE GEMM writes. The order is defined as (score desc, index asc):
// CPU torch.topk leaves ties unordered (SURVEY §7 hard part 2), this fixes it.
//
// topk_rows: one 1024-thread workgroup per query row. Radix select on the
// order-preserving 32-bit key of the fp32 score (digits 11/11/10 bits, LDS
// histograms), stopping as soon as the bin holding the k-th key has <= CAP
// members; then one collection pass gathers every key above that bin plus the
// bin's members IN INDEX ORDER (block prefix sums, so a tie group larger than
// CAP keeps its smallest indices), and a bitonic sort of 64-bit
// (key, ~index) composites in LDS emits the sorted k.
// topk_merge: sort of parts*k_in candidates per row (chunk / shard merge).
#include <algorithm>

#include "kernels.hpp"

namespace clm {

namespace {
constexpr int NT = 1024;
constexpr int CAP = 4096;
constexpr int SORT_MAX = 8192;
constexpr int WIDE_CH = 4096;   // rescore_wide chunk (kernels.hpp RESCORE_WIDE_CHUNK)

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// in-place descending bitonic sort of n (power of two) u64 keys, all threads of the block
__device__ void bitonic_desc(uint64_t* a, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < n / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const uint64_t x = a[lo], y = a[hi];
        if ((x < y) == desc) { a[lo] = y; a[hi] = x; }
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void topk_rows_kernel(const float* S, int64_t lds, int64_t C, int k,
                                                       int64_t base, float* os, int64_t* oi, int64_t ldo) {
  __shared__ uint32_t hist[2048];
  __shared__ uint64_t cand[SORT_MAX];
  __shared__ uint32_t s_prefix, s_bin_cnt;
  __shared__ int s_pbits, s_kk, s_nsure, s_nbin;
  __shared__ int wsum[NT / 64];
  __shared__ int lanecum[64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t row = blockIdx.x;
  const float* s = S + row * lds;

  if (tid == 0) { s_prefix = 0; s_pbits = 0; s_kk = k; }
  __syncthreads();

  // ---- radix select ---------------------------------------------------------
  for (int pass = 0; pass < 3; ++pass) {
    const int pbits = s_pbits;
    const uint32_t prefix = s_prefix;
    const int width = pass < 2 ? 11 : 10;
    const int shift = 32 - pbits - width;
    const int nb = 1 << width;
    for (int i = tid; i < nb; i += NT) hist[i] = 0;
    __syncthreads();
    for (int64_t i = tid; i < C; i += NT) {
      const uint32_t key = fkey(s[i]);
      if (pbits == 0 || (key >> (32 - pbits)) == prefix) atomicAdd(&hist[(key >> shift) & (nb - 1)], 1u);
    }
    __syncthreads();
    if (wid == 0) {  // find the bin (from the top) holding the kk-th key
      const int per = nb / 64;
      const int hi_bin = nb - 1 - lane * per;  // lane covers bins (hi_bin-per, hi_bin]
      int gs = 0;
      for (int q = 0; q < per; ++q) gs += hist[hi_bin - q];
      int cum = gs;  // inclusive scan over lanes
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(cum, o, 64);
        if (lane >= o) cum += v;
      }
      lanecum[lane] = cum;
      const int kk = s_kk;
      const unsigned long long m = __ballot(cum >= kk);
      const int first = m ? __ffsll((long long)m) - 1 : 63;
      if (lane == first) {
        int above = cum - gs;
        int bin = hi_bin;
        for (int q = 0; q < per; ++q) {
          const int b = hi_bin - q;
          if (above + (int)hist[b] >= kk || q == per - 1) { bin = b; break; }
          above += hist[b];
        }
        s_kk = kk - above;
        s_prefix = (prefix << width) | (uint32_t)bin;
        s_pbits = pbits + width;
        s_bin_cnt = hist[bin];
      }
    }
    __syncthreads();
    if (s_bin_cnt <= (uint32_t)CAP) break;
  }

  // ---- collection ------------------------------------------------------------
  const int pbits = s_pbits;
  const uint32_t prefix = s_prefix;
  const int drop = 32 - pbits;
  if (tid == 0) { s_nsure = 0; s_nbin = 0; }
  __syncthreads();
  uint64_t* sure = cand;            // < k entries (k <= 1024)
  uint64_t* binb = cand + 1024;     // <= CAP entries, index order
  for (int64_t b0 = 0; b0 < C; b0 += NT) {
    const int64_t i = b0 + tid;
    bool is_sure = false, is_bin = false;
    uint32_t key = 0;
    if (i < C) {
      key = fkey(s[i]);
      const uint32_t top = drop >= 32 ? 0u : (key >> drop);
      is_sure = top > prefix;
      is_bin = top == prefix;
    }
    const uint64_t comp = ((uint64_t)key << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
    if (is_sure) sure[atomicAdd(&s_nsure, 1)] = comp;
    const unsigned long long m = __ballot(is_bin);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(m);
    __syncthreads();
    int off = s_nbin;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    if (is_bin && off + rank < CAP) binb[off + rank] = comp;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < NT / 64; ++w) tot += wsum[w];
      s_nbin = s_nbin + tot;
    }
    __syncthreads();
  }
  const int nsure = s_nsure;
  const int nbin = min(s_nbin, CAP);
  // compact: sure (nsure <= 1024) then bin list, pad to a power of two
  int total = nsure + nbin;
  int n2 = 1;
  while (n2 < total) n2 <<= 1;
  // move bin entries to follow the sure entries (sure region is fixed 1024)
  // read all into registers first to avoid overlap hazards
  uint64_t tmp[(1024 + CAP) / NT];
#pragma unroll
  for (int q = 0; q < (1024 + CAP) / NT; ++q) {
    const int j = tid + q * NT;
    uint64_t v = 0;
    if (j < nsure) v = sure[j];
    else if (j < total) v = binb[j - nsure];
    tmp[q] = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < (1024 + CAP) / NT; ++q) {
    const int j = tid + q * NT;
    if (j < SORT_MAX) cand[j] = tmp[q];
  }
  for (int j = (1024 + CAP) + tid; j < n2; j += NT) cand[j] = 0;
  __syncthreads();
  if (n2 > 1) bitonic_desc(cand, n2);
  for (int j = tid; j < k; j += NT) {
    float sc = -INFINITY;
    int64_t ix = -1;
    if (j < total) {
      const uint64_t v = cand[j];
      sc = kfloat((uint32_t)(v >> 32));
      ix = base + (int64_t)(0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFu));
    }
    os[row * ldo + j] = sc;
    oi[row * ldo + j] = ix;
  }
}

// ---- exact (fp64) cosine re-scoring ---------------------------------------------------------
// The reference ranks fp32 rows by fp32 dot products of fp32-normalised vectors
// (search.py:36,68,93,96; similarity.py:30-32). The MFMA pass ranks fp16-rounded operands, so
// its scores are within MARGIN/2 of the exact cosine; these kernels recompute the cosine of
// the caller's own fp32 (or fp16) rows in fp64 -- fp32 x fp32 products are exact in fp64 --
// and round once to fp32. Every kernel goes through cos_wave, with one fixed element -> lane
// mapping and reduction order, so a (query, row) pair scores bit-identically on every path.
template <typename R>
__device__ __forceinline__ float row_elem(const R* r, int64_t e) {
  if constexpr (sizeof(R) == 2) return f16_to_f32(r[e]);
  else return r[e];
}

// lane-partial fp64 sums over elements e = lane + 64 i, then one xor-tree over the wave
template <typename R>
__device__ __forceinline__ void dot_wave(const float* q, const R* r, int dim, int lane, double& dot, double& rr) {
  double a = 0.0, b = 0.0;
  for (int e = lane; e < dim; e += 64) {
    const double rv = (double)row_elem(r, e);
    a = fma((double)q[e], rv, a);
    b = fma(rv, rv, b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  dot = a;
  rr = b;
}

__device__ __forceinline__ float cos_from(double dot, double qn, double rr) {
  return (float)(dot / (qn * sqrt(rr)));
}

// qn[q] = ||q||_2 in fp64 (same lane mapping as dot_wave)
__global__ __launch_bounds__(256) void qnorm_kernel(const float* q, int64_t nq, int dim, double* qn) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nq) return;
  double d, s;
  dot_wave(q + row * dim, q + row * dim, dim, lane, d, s);
  if (lane == 0) qn[row] = sqrt(s);
}

// out[qi, j] = cos(q[qi], rows[r0 + j]) for j < rn, qi < nq: one wave per row, queries looped
template <typename R>
__global__ __launch_bounds__(256) void exact_scores_kernel(const float* q, const double* qn, int64_t nq,
                                                           const R* rows, int64_t rn, int dim, float* out,
                                                           int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= rn) return;
  const R* r = rows + j * dim;
  for (int64_t qi = 0; qi < nq; ++qi) {
    double d, rr;
    dot_wave(q + qi * dim, r, dim, lane, d, rr);
    if (lane == 0) out[qi * ldo + j] = cos_from(d, qn[qi], rr);
  }
}

// Per query (one 1024-thread workgroup): sort the filter candidates (fp16-pass score, global
// index) desc, keep those within `margin` of the k-th -- a superset of the exact top-k, since
// |fp16-pass score - exact cosine| <= margin / 2 -- re-score them exactly and emit the top k
// by (exact score desc, index asc). cnt[q] > cap marks an incomplete list: nothing is written
// for that query (the host redoes it with the full exact scan).
template <typename R>
__global__ __launch_bounds__(NT) void rescore_select_kernel(const float* cs, const int64_t* ci, const int* cnt,
                                                            int cap, const float* q, const double* qn, int dim,
                                                            const R* rows, int64_t offset, float margin, int k,
                                                            float* os, int64_t* oi) {
  __shared__ uint64_t keys[SORT_MAX];
  __shared__ int s_m;
  const int64_t row = blockIdx.x;
  const int c = cnt[row];
  if (c > cap) return;
  int n2 = 1;
  while (n2 < c) n2 <<= 1;
  for (int j = threadIdx.x; j < n2; j += NT) {
    uint64_t v = 0;
    if (j < c) {
      const int64_t ix = ci[row * cap + j];
      v = ((uint64_t)fkey(cs[row * cap + j]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)ix);
    }
    keys[j] = v;
  }
  __syncthreads();
  if (n2 > 1) bitonic_desc(keys, n2);
  const float thr = c >= k ? kfloat((uint32_t)(keys[k - 1] >> 32)) - margin : -INFINITY;
  if (threadIdx.x == 0) s_m = c;
  __syncthreads();
  for (int j = threadIdx.x; j < c; j += NT)
    if (kfloat((uint32_t)(keys[j] >> 32)) < thr && (j == 0 || kfloat((uint32_t)(keys[j - 1] >> 32)) >= thr))
      s_m = j;
  __syncthreads();
  const int m = s_m;
  // exact scores of the m survivors, one wave per candidate, written back in place
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* qr = q + row * dim;
  const double qnr = qn[row];
  for (int j = wid; j < m; j += NT / 64) {
    const uint32_t low = (uint32_t)(keys[j] & 0xFFFFFFFFu);
    const int64_t gix = (int64_t)(0xFFFFFFFFu - low);
    double d, rr;
    dot_wave(qr, rows + (gix - offset) * dim, dim, lane, d, rr);
    const float sc = cos_from(d, qnr, rr);
    if (lane == 0) keys[j] = ((uint64_t)fkey(sc) << 32) | low;
  }
  __syncthreads();
  int m2 = 1;
  while (m2 < m) m2 <<= 1;
  for (int j = m + threadIdx.x; j < m2; j += NT) keys[j] = 0;
  __syncthreads();
  if (m2 > 1) bitonic_desc(keys, m2);
  for (int j = threadIdx.x; j < k; j += NT) {
    if (j < m) {
      const uint64_t v = keys[j];
      os[row * k + j] = kfloat((uint32_t)(v >> 32));
      oi[row * k + j] = (int64_t)(0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFu));
    } else {
      os[row * k + j] = -INFINITY;
      oi[row * k + j] = -1;
    }
  }
}

// Overflowed candidate lists (more rows inside the window than CAND_CAP: near-duplicate rows)
// are rebuilt by the host with a capacity that holds all of them and cut into chunks of WIDE_CH
// candidates; per (chunk, query) one workgroup computes every candidate's exact score through
// dot_wave / cos_from (the bits of every other path), sorts the chunk's (exact key, index) in
// LDS and emits its top k (-inf / -1 padding); topk_merge_kernel then merges the chunks' lists.
// The list holds the exact top-k of the index (as rescore_select's does), so the result is the
// full exact scan's.
template <typename R>
__global__ __launch_bounds__(NT) void rescore_wide_kernel(const int64_t* ci, const int* cnt, int64_t cap,
                                                          const float* q, const double* qn, int dim, const R* rows,
                                                          int64_t offset, int k, int nch, float* os, int64_t* oi) {
  __shared__ uint64_t keys[WIDE_CH];
  const int64_t row = blockIdx.y;
  const int ch = blockIdx.x;
  const int64_t c = min((int64_t)cnt[row], cap);
  const int64_t j0 = (int64_t)ch * WIDE_CH;
  const int n = (int)max<int64_t>(0, min<int64_t>(c - j0, WIDE_CH));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* qr = q + row * dim;
  const double qnr = qn[row];
  for (int j = wid; j < n; j += NT / 64) {
    const int64_t gix = ci[row * cap + j0 + j];
    double d, rr;
    dot_wave(qr, rows + (gix - offset) * dim, dim, lane, d, rr);
    const float sc = cos_from(d, qnr, rr);
    if (lane == 0) keys[j] = ((uint64_t)fkey(sc) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)gix);
  }
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int j = n + threadIdx.x; j < n2; j += NT) keys[j] = 0;
  __syncthreads();
  if (n2 > 1) bitonic_desc(keys, n2);
  float* o_s = os + (row * nch + ch) * k;
  int64_t* o_i = oi + (row * nch + ch) * k;
  for (int j = threadIdx.x; j < k; j += NT) {
    if (j < n) {
      const uint64_t v = keys[j];
      o_s[j] = kfloat((uint32_t)(v >> 32));
      o_i[j] = (int64_t)(0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFu));
    } else {
      o_s[j] = -INFINITY;
      o_i[j] = -1;
    }
  }
}

// row gather / scatter of `row_bytes` per row: dst[j] = src[idx[j]] (scatter: dst[idx[j]] = src[j])
__global__ void gather_rows_kernel(const uint8_t* src, int64_t src_stride, const int64_t* idx, int64_t row_bytes,
                                   uint8_t* dst, int64_t dst_stride, int scatter) {
  const int64_t j = blockIdx.x, r = idx[j];
  const uint8_t* sp = src + (scatter ? j : r) * src_stride;
  uint8_t* dp = dst + (scatter ? r : j) * dst_stride;
  for (int64_t b = threadIdx.x; b < row_bytes; b += blockDim.x) dp[b] = sp[b];
}

// filter threshold: th[q] = fp16-pass k-th score of q (ts[q * ld + k - 1]) - margin
__global__ void theta_kernel(const float* ts, int64_t ld, int64_t nq, int k, float margin, float* th) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nq) th[i] = ts[i * ld + k - 1] - margin;
}

// Threshold of the sampled bounded search: th[row] = (k-th largest of row, by the fkey order, with
// multiplicity) - margin, the value topk_rows + theta_kernel give, in one streaming pass instead of
// a radix select's 2-3 passes with LDS-atomic histograms. 256 threads per row: each keeps the 8
// largest keys of its strided elements in registers (sorted, insertion on the rare key above the
// 8th), then each wave and finally wave 0 pops the maximum k times (lowest lane first among equal
// keys, so duplicates count). k <= KTH_MAX.
constexpr int KTH_MAX = 8;
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
// H16: fp16 score rows (GemmArgs::out16), 8 values per 16-B load; fkey of the value widened to
// fp32 (exact), so the keys order as the fp16 values do
template <bool H16>
__global__ __launch_bounds__(256) void kth_threshold_kernel(const void* Sv, int64_t lds, int64_t C, int k, float margin,
                                                            float* th) {
  __shared__ uint32_t part[4 * KTH_MAX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* S = (const float*)Sv;
  const float* s = S + (int64_t)blockIdx.x * lds;
  uint32_t t[KTH_MAX];
#pragma unroll
  for (int j = 0; j < KTH_MAX; ++j) t[j] = 0u;
  auto insert = [&](uint32_t x) {
    if (x <= t[KTH_MAX - 1]) return;
    t[KTH_MAX - 1] = x;
#pragma unroll
    for (int j = KTH_MAX - 1; j > 0; --j)
      if (t[j] > t[j - 1]) { const uint32_t a = t[j]; t[j] = t[j - 1]; t[j - 1] = a; }
  };
  if constexpr (H16) {   // the caller checked lds % 8 == 0 and 16-B alignment
    const u16* sh = (const u16*)Sv + (int64_t)blockIdx.x * lds;
    const int64_t C8 = C >> 3;
    const u32x4* s8 = (const u32x4*)sh;
    auto hv = [](uint32_t w, int hi) {
      return (float)__builtin_bit_cast(_Float16, (uint16_t)(hi ? (w >> 16) : (w & 0xFFFFu)));
    };
    int64_t i = tid;
    for (; i + 256 < C8; i += 512) {   // two 16-B loads (16 values) in flight before the inserts
      const u32x4 a = s8[i], b = s8[i + 256];
      float v[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = hv(a[j], 0); v[2 * j + 1] = hv(a[j], 1);
        v[8 + 2 * j] = hv(b[j], 0); v[9 + 2 * j] = hv(b[j], 1);
      }
      float mx = v[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = __builtin_elementwise_maximum(mx, v[j]);
      if (!(mx == mx) || fkey(mx) > t[KTH_MAX - 1]) {
#pragma unroll
        for (int j = 0; j < 16; ++j) insert(fkey(v[j]));
      }
    }
    for (; i < C8; i += 256) {
      const u32x4 a = s8[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) { insert(fkey(hv(a[j], 0))); insert(fkey(hv(a[j], 1))); }
    }
    for (int64_t j = (C8 << 3) + tid; j < C; j += 256) insert(fkey((float)__builtin_bit_cast(_Float16, sh[j])));
  } else if ((lds & 3) == 0 && ((uintptr_t)S & 15) == 0) {
    const int64_t C4 = C >> 2;
    const float4* s4 = (const float4*)s;
    int64_t i = tid;
    for (; i + 768 < C4; i += 1024) {   // four 16-B loads in flight before the inserts
      const float4 a = s4[i], b = s4[i + 256], c = s4[i + 512], e = s4[i + 768];
      // a block whose 16 values are all below the current 8th largest is one test, no inserts
      // (NaN-propagating maximum: a block holding a NaN takes the per-value path, as the plain loop)
      auto mx2 = [](float x, float y) { return __builtin_elementwise_maximum(x, y); };
      const float mx = mx2(mx2(mx2(mx2(a.x, a.y), mx2(a.z, a.w)), mx2(mx2(b.x, b.y), mx2(b.z, b.w))),
                           mx2(mx2(mx2(c.x, c.y), mx2(c.z, c.w)), mx2(mx2(e.x, e.y), mx2(e.z, e.w))));
      if (!(mx == mx) || fkey(mx) > t[KTH_MAX - 1]) {
        insert(fkey(a.x)); insert(fkey(a.y)); insert(fkey(a.z)); insert(fkey(a.w));
        insert(fkey(b.x)); insert(fkey(b.y)); insert(fkey(b.z)); insert(fkey(b.w));
        insert(fkey(c.x)); insert(fkey(c.y)); insert(fkey(c.z)); insert(fkey(c.w));
        insert(fkey(e.x)); insert(fkey(e.y)); insert(fkey(e.z)); insert(fkey(e.w));
      }
    }
    for (; i < C4; i += 256) {
      const float4 v = s4[i];
      insert(fkey(v.x)); insert(fkey(v.y)); insert(fkey(v.z)); insert(fkey(v.w));
    }
    for (int64_t j = (C4 << 2) + tid; j < C; j += 256) insert(fkey(s[j]));
  } else {
    for (int64_t i = tid; i < C; i += 256) insert(fkey(s[i]));
  }
  // wave top-k: pop the wave maximum k times
  uint32_t m = 0;
  for (int r = 0; r < k; ++r) {
    m = wave_max_u32(t[0]);
    const unsigned long long who = __ballot(t[0] == m);
    if (lane == __ffsll((long long)who) - 1) {
#pragma unroll
      for (int j = 0; j < KTH_MAX - 1; ++j) t[j] = t[j + 1];
      t[KTH_MAX - 1] = 0u;
    }
    if (lane == 0) part[wid * KTH_MAX + r] = m;
  }
  __syncthreads();
  if (wid == 0) {
    uint32_t v = (lane < 4 * KTH_MAX && (lane % KTH_MAX) < k) ? part[lane] : 0u;
    for (int r = 0; r < k; ++r) {
      m = wave_max_u32(v);
      const unsigned long long who = __ballot(v == m);
      if (lane == __ffsll((long long)who) - 1) v = 0u;
    }
    if (lane == 0) th[blockIdx.x] = kfloat(m) - margin;
  }
}

__global__ void upcast_f16_kernel(const u16* src, int64_t total, float* dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = f16_to_f32(src[i]);
}

__global__ __launch_bounds__(NT) void topk_merge_kernel(const float* in_s, const int64_t* in_i, int n_in,
                                                        int k, float* os, int64_t* oi) {
  __shared__ uint64_t cand[SORT_MAX];
  const int64_t row = blockIdx.x;
  int n2 = 1;
  while (n2 < n_in) n2 <<= 1;
  for (int j = threadIdx.x; j < n2; j += NT) {
    uint64_t v = 0;
    if (j < n_in) {
      const int64_t ix = in_i[row * n_in + j];
      if (ix >= 0)
        v = ((uint64_t)fkey(in_s[row * n_in + j]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)ix);
    }
    cand[j] = v;
  }
  __syncthreads();
  if (n2 > 1) bitonic_desc(cand, n2);
  for (int j = threadIdx.x; j < k; j += NT) {
    const uint64_t v = j < n_in ? cand[j] : 0;
    if (v == 0) { os[row * k + j] = -INFINITY; oi[row * k + j] = -1; continue; }
    os[row * k + j] = kfloat((uint32_t)(v >> 32));
    oi[row * k + j] = (int64_t)(0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFu));
  }
}
// ---- top-k for any k (topk_any: k > 1024, or more merge candidates than one LDS sort holds) ----------
// Every entry's 64-bit composite is (key << 32) | (0xFFFFFFFF - global index): descending composite
// order is (score desc, index asc).
// 1. kth_exact_kernel: per row, the exact kk-th largest composite (kk = min(k, C)) as two 32-bit
//    radix selects (11 / 11 / 10-bit passes each): the key T of the kk-th entry, then among the
//    entries with key T the low word Lo of the one that is kk-th overall (ties on the score are
//    broken by the global index whatever order the columns hold them in -- merge inputs are lists).
// 2. collect_kernel: every composite >= (T, Lo) of the row -- exactly kk -- into a segment of Kp (a
//    power of two) u64, 0-padded (order irrelevant).
// 3. sort_runs_kernel: LDS bitonic sort (descending) of runs of min(Kp, RUN); merge_runs_kernel:
//    merge passes doubling the run length until it is Kp (merge path by binary search, stable:
//    equal composites -- only the 0 pads -- keep A before B).
// 4. emit_kernel: the first k composites as (score, global index), (-inf, -1) for pads.
constexpr int RUN = 8192;

__device__ __forceinline__ bool any_valid(const int64_t* ix, int64_t j) { return !ix || ix[j] >= 0; }
__device__ __forceinline__ uint32_t any_lo(const int64_t* ix, int64_t base, int64_t j) {
  return 0xFFFFFFFFu - (uint32_t)(ix ? ix[j] : base + j);
}

// radix select over `get(i, v)` (true: entry i takes part with 32-bit value v) of the kk-th largest
// value, three passes 11 / 11 / 10 bits; returns the value and the number of entries equal to it
// that belong to the top kk (s_kk). All threads of the block call it.
template <typename Get>
__device__ void radix_kth(int64_t C, int kk, uint32_t* hist, uint32_t& s_prefix, int& s_pbits, int& s_kk, Get get) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) { s_prefix = 0; s_pbits = 0; s_kk = kk; }
  __syncthreads();
  for (int pass = 0; pass < 3; ++pass) {
    const int pbits = s_pbits;
    const uint32_t prefix = s_prefix;
    const int width = pass < 2 ? 11 : 10;
    const int shift = 32 - pbits - width;
    const int nb = 1 << width;
    for (int i = tid; i < nb; i += NT) hist[i] = 0;
    __syncthreads();
    for (int64_t i = tid; i < C; i += NT) {
      uint32_t v;
      if (get(i, v) && (pbits == 0 || (v >> (32 - pbits)) == prefix)) atomicAdd(&hist[(v >> shift) & (nb - 1)], 1u);
    }
    __syncthreads();
    if (wid == 0) {   // the bin (from the top) holding the kk-th value, as topk_rows_kernel
      const int per = nb / 64;
      const int hi_bin = nb - 1 - lane * per;
      int gs = 0;
      for (int q = 0; q < per; ++q) gs += hist[hi_bin - q];
      int cum = gs;
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(cum, o, 64);
        if (lane >= o) cum += v;
      }
      const int k2 = s_kk;
      const unsigned long long m = __ballot(cum >= k2);
      const int first = m ? __ffsll((long long)m) - 1 : 63;
      if (lane == first) {
        int above = cum - gs;
        int bin = hi_bin;
        for (int q = 0; q < per; ++q) {
          const int b = hi_bin - q;
          if (above + (int)hist[b] >= k2 || q == per - 1) { bin = b; break; }
          above += hist[b];
        }
        s_kk = k2 - above;
        s_prefix = (prefix << width) | (uint32_t)bin;
        s_pbits = pbits + width;
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void kth_exact_kernel(const float* S, int64_t lds, const int64_t* I, int64_t ldi,
                                                       int64_t C, int k, int64_t base, uint32_t* thr) {
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_prefix;
  __shared__ int s_pbits, s_kk;
  const int64_t row = blockIdx.x;
  const float* s = S + row * lds;
  const int64_t* ix = I ? I + row * ldi : nullptr;
  int64_t nvalid = C;
  if (ix) {   // entries that can be taken (empty merge slots cannot)
    __shared__ int s_nv;
    if (threadIdx.x == 0) s_nv = 0;
    __syncthreads();
    int c = 0;
    for (int64_t i = threadIdx.x; i < C; i += NT) c += ix[i] >= 0;
    atomicAdd(&s_nv, c);
    __syncthreads();
    nvalid = s_nv;
  }
  const int kk = (int)min((int64_t)k, nvalid);
  if (kk <= 0) {   // nothing to take: a threshold above every composite
    if (threadIdx.x == 0) { thr[2 * row] = 0xFFFFFFFFu; thr[2 * row + 1] = 0xFFFFFFFFu; }
    return;
  }
  radix_kth(C, kk, hist, s_prefix, s_pbits, s_kk, [&](int64_t i, uint32_t& v) {
    if (!any_valid(ix, i)) return false;
    v = fkey(s[i]);
    return true;
  });
  const uint32_t T = s_prefix;
  const int need = s_kk;
  __syncthreads();
  radix_kth(C, need, hist, s_prefix, s_pbits, s_kk, [&](int64_t i, uint32_t& v) {
    if (!any_valid(ix, i) || fkey(s[i]) != T) return false;
    v = any_lo(ix, base, i);
    return true;
  });
  if (threadIdx.x == 0) { thr[2 * row] = T; thr[2 * row + 1] = s_prefix; }
}

__global__ __launch_bounds__(NT) void collect_kernel(const float* S, int64_t lds, const int64_t* I, int64_t ldi,
                                                     int64_t C, int64_t base, const uint32_t* thr, uint64_t* seg,
                                                     int64_t Kp) {
  __shared__ int s_n;
  const int64_t row = blockIdx.x;
  const float* s = S + row * lds;
  const int64_t* ix = I ? I + row * ldi : nullptr;
  uint64_t* out = seg + row * Kp;
  for (int64_t j = threadIdx.x; j < Kp; j += NT) out[j] = 0;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint64_t lim = ((uint64_t)thr[2 * row] << 32) | thr[2 * row + 1];
  for (int64_t i = threadIdx.x; i < C; i += NT) {
    if (!any_valid(ix, i)) continue;
    const uint64_t comp = ((uint64_t)fkey(s[i]) << 32) | any_lo(ix, base, i);
    if (comp >= lim) {
      const int at = atomicAdd(&s_n, 1);
      if (at < Kp) out[at] = comp;
    }
  }
}

__global__ __launch_bounds__(NT) void sort_runs_kernel(uint64_t* seg, int64_t Kp, int run) {
  __shared__ uint64_t a[RUN];
  uint64_t* p = seg + (int64_t)blockIdx.y * Kp + (int64_t)blockIdx.x * run;
  for (int j = threadIdx.x; j < run; j += NT) a[j] = p[j];
  __syncthreads();
  bitonic_desc(a, run);
  for (int j = threadIdx.x; j < run; j += NT) p[j] = a[j];
}

__global__ __launch_bounds__(256) void merge_runs_kernel(const uint64_t* src, uint64_t* dst, int64_t Kp, int64_t L,
                                                         int64_t total) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
    const int64_t row = p / Kp, q = p - row * Kp;
    const int64_t r = q / L, pos = q - r * L;
    const uint64_t x = src[p];
    const uint64_t* other = src + row * Kp + (r ^ 1) * L;
    const bool b_side = r & 1;
    int64_t lo = 0, hi = L;   // other-run elements that precede x: > x (x in A) or >= x (x in B)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const uint64_t o = other[mid];
      if (b_side ? o >= x : o > x) lo = mid + 1;
      else hi = mid;
    }
    dst[row * Kp + (r & ~(int64_t)1) * L + pos + lo] = x;
  }
}

__global__ __launch_bounds__(256) void emit_kernel(const uint64_t* seg, int64_t Kp, int64_t nq, int k, float* os,
                                                   int64_t* oi, int64_t ldo) {
  const int64_t total = nq * k;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
    const int64_t row = p / k, j = p - row * k;
    const uint64_t v = j < Kp ? seg[row * Kp + j] : 0;
    if (v == 0) {
      os[row * ldo + j] = -INFINITY;
      oi[row * ldo + j] = -1;
    } else {
      os[row * ldo + j] = kfloat((uint32_t)(v >> 32));
      oi[row * ldo + j] = (int64_t)(0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFu));
    }
  }
}

int64_t any_kp(int k) {
  int64_t kp = 2;
  while (kp < k) kp <<= 1;
  return kp;
}
}  // namespace

size_t topk_any_ws_bytes(int64_t nq, int k) {
  const int64_t kp = any_kp(k);
  return (size_t)nq * 8 + 256 + 2 * (size_t)nq * kp * 8;
}

hipError_t topk_any(const float* scores, int64_t lds, const int64_t* idx, int64_t ldi, int64_t nq, int64_t C, int k,
                    int64_t base, float* out_s, int64_t* out_i, int64_t ldo, void* ws, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || C < 0 || C > 0xFFFFFFFFll || nq > 65535 || !ws) return hipErrorInvalidValue;
  const int64_t kp = any_kp(k);
  uint32_t* thr = (uint32_t*)ws;   // per row {T, Lo}
  uint64_t* seg = (uint64_t*)(((uintptr_t)(thr + 2 * nq) + 255) & ~(uintptr_t)255);
  uint64_t* seg2 = seg + nq * kp;
  kth_exact_kernel<<<(unsigned)nq, NT, 0, s>>>(scores, lds, idx, ldi, C, k, base, thr);
  collect_kernel<<<(unsigned)nq, NT, 0, s>>>(scores, lds, idx, ldi, C, base, thr, seg, kp);
  const int run = (int)std::min<int64_t>(kp, RUN);
  sort_runs_kernel<<<dim3((unsigned)(kp / run), (unsigned)nq), NT, 0, s>>>(seg, kp, run);
  uint64_t *a = seg, *b = seg2;
  for (int64_t L = run; L < kp; L <<= 1) {
    const int64_t total = nq * kp;
    merge_runs_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, 65536), 256, 0, s>>>(a, b, kp, L, total);
    std::swap(a, b);
  }
  emit_kernel<<<(unsigned)std::min<int64_t>((nq * k + 255) / 256, 65536), 256, 0, s>>>(a, kp, nq, k, out_s, out_i, ldo);
  return hipGetLastError();
}

namespace {
// cnt[row] = #{ j < C : S[row, j] >= th[row] } (one 256-thread workgroup per row)
__global__ __launch_bounds__(256) void count_ge_kernel(const float* S, int64_t lds, int64_t C, const float* th,
                                                       int* cnt) {
  __shared__ int part[4];
  const int64_t row = blockIdx.x;
  const float t = th[row];
  const float* s = S + row * lds;
  int c = 0;
  if ((lds & 3) == 0 && ((uintptr_t)S & 15) == 0) {   // 16-B loads, four in flight per thread
    const int64_t C4 = C >> 2;
    const float4* s4 = (const float4*)s;
    int64_t i = threadIdx.x;
    for (; i + 768 < C4; i += 1024) {
      const float4 a = s4[i], b = s4[i + 256], d = s4[i + 512], e = s4[i + 768];
      c += (a.x >= t) + (a.y >= t) + (a.z >= t) + (a.w >= t) + (b.x >= t) + (b.y >= t) + (b.z >= t) + (b.w >= t) +
           (d.x >= t) + (d.y >= t) + (d.z >= t) + (d.w >= t) + (e.x >= t) + (e.y >= t) + (e.z >= t) + (e.w >= t);
    }
    for (; i < C4; i += 256) {
      const float4 a = s4[i];
      c += (a.x >= t) + (a.y >= t) + (a.z >= t) + (a.w >= t);
    }
    for (int64_t j = (C4 << 2) + threadIdx.x; j < C; j += 256) c += s[j] >= t;
  } else {
    for (int64_t j = threadIdx.x; j < C; j += 256) c += s[j] >= t;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[row] = part[0] + part[1] + part[2] + part[3];
}
// fp16 score rows (GemmArgs::out16): 8 values per 16-B load
__device__ __forceinline__ float f16v(uint32_t w, int hi) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(hi ? (w >> 16) : (w & 0xFFFFu)));
}
__global__ __launch_bounds__(256) void count_ge16_kernel(const u16* S, int64_t lds, int64_t C, const float* th,
                                                         int* cnt) {
  __shared__ int part[4];
  const int64_t row = blockIdx.x;
  const float t = th[row];
  const u16* s = S + row * lds;
  int c = 0;
  const int64_t C8 = C >> 3;
  const u32x4* s8 = (const u32x4*)s;
  int64_t i = threadIdx.x;
  for (; i + 256 < C8; i += 512) {
    const u32x4 a = s8[i], b = s8[i + 256];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      c += (f16v(a[j], 0) >= t) + (f16v(a[j], 1) >= t) + (f16v(b[j], 0) >= t) + (f16v(b[j], 1) >= t);
  }
  for (; i < C8; i += 256) {
    const u32x4 a = s8[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) c += (f16v(a[j], 0) >= t) + (f16v(a[j], 1) >= t);
  }
  for (int64_t j = (C8 << 3) + threadIdx.x; j < C; j += 256)
    c += (float)__builtin_bit_cast(_Float16, s[j]) >= t;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[row] = part[0] + part[1] + part[2] + part[3];
}
}  // namespace

hipError_t count_ge16(const u16* scores, int64_t lds, int64_t nq, int64_t C, const float* th, int* cnt,
                      hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if ((lds & 7) || ((uintptr_t)scores & 15)) return hipErrorInvalidValue;
  count_ge16_kernel<<<(unsigned)nq, 256, 0, s>>>(scores, lds, C, th, cnt);
  return hipGetLastError();
}

hipError_t count_ge(const float* scores, int64_t lds, int64_t nq, int64_t C, const float* th, int* cnt, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  count_ge_kernel<<<(unsigned)nq, 256, 0, s>>>(scores, lds, C, th, cnt);
  return hipGetLastError();
}

hipError_t topk_rows(const float* scores, int64_t lds, int64_t nq, int64_t C, int k, int64_t base, float* out_s,
                     int64_t* out_i, int64_t ldo, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || k > 1024 || C < 0 || C > 0xFFFFFFFFll) return hipErrorInvalidValue;
  topk_rows_kernel<<<(unsigned)nq, NT, 0, s>>>(scores, lds, C, k, base, out_s, out_i, ldo);
  return hipGetLastError();
}

hipError_t topk_merge(const float* in_s, const int64_t* in_i, int64_t nq, int parts, int k_in, int k,
                      float* out_s, int64_t* out_i, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  const int n_in = parts * k_in;
  if (n_in > SORT_MAX || k < 1 || k > 1024) return hipErrorInvalidValue;
  topk_merge_kernel<<<(unsigned)nq, NT, 0, s>>>(in_s, in_i, n_in, k, out_s, out_i);
  return hipGetLastError();
}

hipError_t query_norms(const float* q, int64_t nq, int dim, double* qn, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  qnorm_kernel<<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(q, nq, dim, qn);
  return hipGetLastError();
}

hipError_t exact_scores(const float* q, const double* qn, int64_t nq, const void* rows, bool rows_f16, int64_t rn,
                        int dim, float* out, int64_t ldo, hipStream_t s) {
  if (nq <= 0 || rn <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((rn + 3) / 4);
  if (rows_f16)
    exact_scores_kernel<u16><<<grid, 256, 0, s>>>(q, qn, nq, (const u16*)rows, rn, dim, out, ldo);
  else
    exact_scores_kernel<float><<<grid, 256, 0, s>>>(q, qn, nq, (const float*)rows, rn, dim, out, ldo);
  return hipGetLastError();
}

hipError_t rescore_select(const float* cand_s, const int64_t* cand_i, const int* cnt, int cap, const float* q,
                          const double* qn, int dim, const void* rows, bool rows_f16, int64_t offset, float margin,
                          int64_t nq, int k, float* out_s, int64_t* out_i, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (cap > SORT_MAX || k < 1 || k > 1024) return hipErrorInvalidValue;
  if (rows_f16)
    rescore_select_kernel<u16><<<(unsigned)nq, NT, 0, s>>>(cand_s, cand_i, cnt, cap, q, qn, dim, (const u16*)rows,
                                                           offset, margin, k, out_s, out_i);
  else
    rescore_select_kernel<float><<<(unsigned)nq, NT, 0, s>>>(cand_s, cand_i, cnt, cap, q, qn, dim,
                                                             (const float*)rows, offset, margin, k, out_s, out_i);
  return hipGetLastError();
}

hipError_t rescore_wide(const int64_t* cand_i, const int* cnt, int64_t cap, const float* q, const double* qn, int dim,
                        const void* rows, bool rows_f16, int64_t offset, int64_t nq, int k, float* part_s,
                        int64_t* part_i, hipStream_t s) {
  static_assert(WIDE_CH == RESCORE_WIDE_CHUNK, "chunk size");
  if (nq <= 0) return hipSuccess;
  const int64_t nch = (cap + WIDE_CH - 1) / WIDE_CH;
  if (k < 1 || k > WIDE_CH || nch < 1 || nch * k > SORT_MAX || nq > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nch, (unsigned)nq);
  if (rows_f16)
    rescore_wide_kernel<u16><<<grid, NT, 0, s>>>(cand_i, cnt, cap, q, qn, dim, (const u16*)rows, offset, k, (int)nch,
                                                 part_s, part_i);
  else
    rescore_wide_kernel<float><<<grid, NT, 0, s>>>(cand_i, cnt, cap, q, qn, dim, (const float*)rows, offset, k,
                                                   (int)nch, part_s, part_i);
  return hipGetLastError();
}

hipError_t gather_rows(const void* src, int64_t src_stride, const int64_t* idx, int64_t n, int64_t row_bytes,
                       void* dst, int64_t dst_stride, bool scatter, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  gather_rows_kernel<<<(unsigned)n, 256, 0, s>>>((const uint8_t*)src, src_stride, idx, row_bytes, (uint8_t*)dst,
                                                 dst_stride, scatter ? 1 : 0);
  return hipGetLastError();
}

hipError_t filter_thresholds(const float* ts, int64_t ld, int64_t nq, int k, float margin, float* th, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  theta_kernel<<<(unsigned)((nq + 255) / 256), 256, 0, s>>>(ts, ld, nq, k, margin, th);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void value_bounds_kernel(const float* v, int64_t n, unsigned* keys) {
  unsigned lo = 0xFFFFFFFFu, hi = 0u;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const unsigned k = float_key(v[i]);
    lo = min(lo, k);
    hi = max(hi, k);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (unsigned)__shfl_xor((int)lo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(keys, lo);
    atomicMax(keys + 1, hi);
  }
}

hipError_t value_bounds(const float* v, int64_t n, unsigned* keys, hipStream_t s) {
  hipError_t e = hipMemsetD32Async((hipDeviceptr_t)keys, 0xFFFFFFFFu, 1, s);
  if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)(keys + 1), 0u, 1, s);
  if (e != hipSuccess || n <= 0) return e;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  value_bounds_kernel<<<blocks, 256, 0, s>>>(v, n, keys);
  return hipGetLastError();
}

hipError_t kth_thresholds(const float* scores, int64_t lds, int64_t nq, int64_t C, int k, float margin, float* th,
                          hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || k > KTH_MAX || C < k) return hipErrorInvalidValue;
  kth_threshold_kernel<false><<<(unsigned)nq, 256, 0, s>>>(scores, lds, C, k, margin, th);
  return hipGetLastError();
}

hipError_t kth_thresholds16(const u16* scores, int64_t lds, int64_t nq, int64_t C, int k, float margin, float* th,
                            hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || k > KTH_MAX || C < k || (lds & 7) || ((uintptr_t)scores & 15)) return hipErrorInvalidValue;
  kth_threshold_kernel<true><<<(unsigned)nq, 256, 0, s>>>(scores, lds, C, k, margin, th);
  return hipGetLastError();
}

hipError_t f16_to_f32_rows(const u16* src, int64_t n, int dim, float* dst, hipStream_t s) {
  const int64_t total = n * dim;
  if (total <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  upcast_f16_kernel<<<blocks, 256, 0, s>>>(src, total, dst);
  return hipGetLastError();
}

namespace {
// ------------------------------------------------------------------------------------------
// Small query batches (nq <= 16) against a large index: the reference's own call pattern, one
// query per search_with_embedding call (src/embedding/search.py:93-99, seeker_service.py:183-186).
// The MFMA filter GEMM pads such a batch to 256-row query tiles; this pass streams the fp16 index
// once at HBM rate instead (10.24 GB for configs[4]'s 10 M x 512), every wave on its own rows:
//  * the index is cut into chunks of 256 rows; wave w of the W in the grid takes chunks w, w + W,
//    ... (each 256 x dim x 2 bytes contiguous), 16-row blocks through a per-wave D-deep LDS ring
//    filled by buffer_load ... lds (one 1 KiB wave-instruction per 512 row bytes, whole rows, the
//    16-B chunks XOR-swizzled on the source so the fragment reads are conflict-free) plus one DMA of
//    the block's 16 inverse norms. No barriers: a wave reads only the blocks it loaded;
//  * per block, dim / 32 v_mfma_f32_16x16x32_f16 with the (<= 16) unit-rounded fp16 queries held in
//    registers on the A port and the index rows on the B port: lane l ends with queries 4 (l >> 4)
//    .. +3 of row l & 15, scored as the EPI_SCORE epilogue does (acc * qinv[q] * inv[row]), stored
//    into the row-major [N, ldq] score matrix (a block's scores one contiguous piece: 16 B per lane
//    for ldq >= 4) and max-reduced into the chunk's maxima;
//  * cmax[q][chunk] = the largest fp16-pass score of the chunk (NaN scores ignored, rows past N
//    -inf). The k-th largest chunk maximum is at most the k-th largest score of the whole index
//    (k chunks whose maxima reach it hold k distinct rows), so th = that - margin bounds the
//    candidates exactly as the sampled threshold does (capi.cpp search_small).
// Counted vmcnt: in the steady state the DMA of block i is older than one score store and D - 2
// (DMA + store) groups; the first and last D - 1 blocks, and the extra chunk-maximum stores, only
// ever make the wait longer (vmcnt(0) there).
constexpr int SCAN_CHUNK = 256;
// cache policy of the index stream's LDS-DMA: nt (non-temporal; each row is read once per call):
// single-query device time 1.763 -> 1.682 ms at 10 M x 512, 0.729 -> 0.764 of HBM, nq = 1..16 all
// 4-6 % faster (profiles/r06_v15_scan16_nt_ab.txt)
#ifndef CLM_SCAN_AUX
#define CLM_SCAN_AUX 2
#endif
template <int KS, int D>
__device__ __forceinline__ void scan16_body(const Scan16Args& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  constexpr int RB = KS * 64;            // row bytes (dim = 32 KS)
  constexpr int BLK = 16 * RB + 1024;    // a block's LDS image: 16 rows, then its inverse norms
  constexpr int F0 = 1 + (D - 2) * (KS + 2);
  constexpr int F = F0 > 63 ? 63 : F0;
  // lane: row rr of a 16-row block (B port / C column), query group g: queries 4 g .. 4 g + 3
  // (C rows); on the A port the lane carries query rr
  const int lane = threadIdx.x & 63, g = lane >> 4, rr = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int64_t W = (int64_t)gridDim.x * nw;
  const int64_t w = (int64_t)blockIdx.x * nw + wid;
  const int64_t nchunk = a.nchunk;
  const int64_t my = w < nchunk ? (nchunk - 1 - w) / W + 1 : 0;
  const int64_t nb = my * (SCAN_CHUNK / 16);
  const int ldq = (int)a.ldo;   // scores per row: 1, 2, 4, 8 or 16 (>= nq)
  // the wave's 8 largest chunk maxima of queries 4 g + u (sorted descending, every lane of the
  // group), written at the end: the k-th largest over every wave's list is the k-th largest chunk
  // maximum for k <= 8, without a pass over [nq, nchunk] (one workgroup per query spent 74 us on it
  // at 10 M rows)
  float top[4][KTH_MAX];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < KTH_MAX; ++j) top[u][j] = -INFINITY;
  auto write_top = [&]() {
    const auto tb = buf_rsrc(a.wtop + w * KTH_MAX);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < KTH_MAX; ++j) {
        const int q = 4 * g + u;
        const uint32_t to = (rr == 0 && q < a.nq) ? (uint32_t)(((int64_t)q * a.ldw + j) * 4) : BUF_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(top[u][j]), tb, to, 0, 0);
      }
  };
  if (nb == 0) {
    if (a.wtop) write_top();
    return;
  }
  uint8_t* ring = smem + wid * D * BLK;
  // chunk swizzle: 16 consecutive rows at one chunk position land on 16 distinct bank quads
  auto sw = [](int r) { return RB >= 256 ? (r & 15) : ((r >> 1) & 7); };
  u32x4 qf[KS];   // A port: query rr, dims (4 s + g) * 8 .. + 7
  {
    const u16* qp = a.q16 + (int64_t)min(rr, a.nq - 1) * (KS * 32) + g * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = rr < a.nq ? *(const u32x4*)(qp + s * 32) : u32x4{0u, 0u, 0u, 0u};
  }
  float qs[4];   // inverse norms of queries 4 g + u
#pragma unroll
  for (int u = 0; u < 4; ++u) qs[u] = 4 * g + u < a.nq ? a.qinv[4 * g + u] : 0.f;
  uint32_t doff[KS];   // DMA: instruction t, lane -> LDS slot t * 1 KiB + 16 lane of the block image
#pragma unroll
  for (int t = 0; t < KS; ++t) {
    const int o = t * 1024 + lane * 16, r = o / RB, p = (o % RB) / 16;
    doff[t] = (uint32_t)(r * RB + ((p ^ sw(r)) * 16));
  }
  const uint32_t ioff = lane < 4 ? (uint32_t)lane * 16 : BUF_OOB;
  uint32_t foff[KS];   // B port: row rr of the block, chunk 4 s + g
#pragma unroll
  for (int s = 0; s < KS; ++s) foff[s] = (uint32_t)(rr * RB + (((4 * s + g) ^ sw(rr)) * 16));
  auto row0_of = [&](int64_t i) { return (w + (i >> 4) * W) * SCAN_CHUNK + (i & 15) * 16; };
  auto issue = [&](int64_t i, int buf) {
    const int64_t r0 = row0_of(i);
    const int left = (int)max<int64_t>(0, min<int64_t>(16, a.N - r0));
    const auto rs = buf_rsrc(a.rows + r0 * (KS * 32), left * RB);
    const auto ri = buf_rsrc(a.inv + r0, left * 4);
    uint8_t* base = ring + buf * BLK;
#pragma unroll
    for (int t = 0; t < KS; ++t)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(base + t * 1024), 16, doff[t], 0, 0, CLM_SCAN_AUX);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ri, (lds_ptr_t)(base + 16 * RB), 16, ioff, 0, 0, CLM_SCAN_AUX);
  };
#pragma unroll
  for (int j = 0; j < D - 1; ++j)
    if (j < nb) issue(j, j);
  float run[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int buf = 0;
  for (int64_t i = 0; i < nb; ++i) {
    if (i < D - 1 || i > nb - D) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(F) : "memory");
    // the buffer of block i - 1 is free: its fragment reads were consumed by last block's MFMAs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + D - 1 < nb) issue(i + D - 1, buf == 0 ? D - 1 : buf - 1);
    const uint8_t* blk = ring + buf * BLK;
    u32x4 af[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = *(const u32x4*)(blk + foff[s]);
    // the row's inverse norm through an asm read: the compiler's LDS-DMA alias tracking put a
    // vmcnt(0) (every DMA in flight, the whole ring) in front of this read when it was a plain load
    uint32_t ivb;
    asm volatile("ds_read_b32 %0, %1" : "=v"(ivb) : "v"((uint32_t)(uintptr_t)(blk + 16 * RB + rr * 4)) : "memory");
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma16<false>(qf[s], af[s], acc);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ivb));
    const float iv = __uint_as_float(ivb);
    const int64_t r0 = row0_of(i);
    const bool live = r0 + rr < a.N;
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = live ? acc[u] * qs[u] * iv : -INFINITY;
      run[u] = fmaxf(run[u], v[u]);
    }
    // scores [N, ldq], the row's queries contiguous: a block's 16 rows are one contiguous piece
    const auto ob = buf_rsrc(a.out + r0 * ldq);
    if (ldq >= 4) {
      const uint32_t oo = (live && 4 * g < a.nq) ? (uint32_t)((rr * ldq + 4 * g) * 4) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                   __float_as_uint(v[2]), __float_as_uint(v[3])}, ob, oo, 0, 0);
    } else if (ldq == 2) {
      const uint32_t oo = (live && g == 0) ? (uint32_t)(rr * 8) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v[0]), __float_as_uint(v[1])}, ob, oo, 0, 0);
    } else {
      const uint32_t oo = (live && g == 0) ? (uint32_t)(rr * 4) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), ob, oo, 0, 0);
    }
    if ((i & 15) == 15) {   // chunk end: its maximum per query (the 16 row lanes of each group)
      const int64_t chunk = w + (i >> 4) * W;
      const auto cb = buf_rsrc(a.cmax + chunk);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float m = group16_max(run[u]);
        run[u] = -INFINITY;
        const int q = 4 * g + u;
        const uint32_t co = (rr == 0 && q < a.nq) ? (uint32_t)((int64_t)q * nchunk * 4) : BUF_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), cb, co, 0, 0);
        if (m > top[u][KTH_MAX - 1]) {   // never NaN: fmaxf dropped NaN scores
          top[u][KTH_MAX - 1] = m;
#pragma unroll
          for (int j = KTH_MAX - 1; j > 0; --j)
            if (top[u][j] > top[u][j - 1]) { const float t = top[u][j]; top[u][j] = top[u][j - 1]; top[u][j - 1] = t; }
        }
      }
    }
    buf = buf + 1 == D ? 0 : buf + 1;
  }
  if (a.wtop) write_top();
}

// (the body lives in a __device__ function: written inline in the kernel, hipcc's host pass left
// every instantiation's launch stub undefined)
template <int KS, int D>
__global__ __launch_bounds__(256, 1) void scan16_kernel(Scan16Args a) {
  scan16_body<KS, D>(a);
}

// candidates of the small-batch search: every (score, global row) of the score matrix S [C rows,
// ldq] (ldq a power of two >= nq; query q in column q) at or above th[q], appended to q's list
// (capacity cap; cnt[q] counts them all, so cnt > cap marks an overflow). The list order is the
// atomics' (rescore_select sorts by (score, index)).
__global__ __launch_bounds__(256) void collect_ge_kernel(const float* S, int lq, int nq, int64_t C, const float* th,
                                                         int* cnt, int cap, float* cs, int64_t* ci, int64_t base) {
  const int ldq = 1 << lq;
  float t[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) t[q] = q < nq ? th[q] : INFINITY;
  const int64_t n4 = ((C << lq) + 3) >> 2;   // float4 groups, the last one possibly partial
  for (int64_t e4 = (int64_t)blockIdx.x * 256 + threadIdx.x; e4 < n4; e4 += (int64_t)gridDim.x * 256) {
    float v[4];
    const int64_t e0 = e4 * 4;
    if (e0 + 4 <= (C << lq)) {
      const float4 x = *(const float4*)(S + e0);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = e0 + u < (C << lq) ? S[e0 + u] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = e0 + u;
      const int q = (int)(e & (ldq - 1));
      float tq = t[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) tq = q == j ? t[j] : tq;
      if (v[u] >= tq && q < nq) {
        const int slot = atomicAdd(cnt + q, 1);
        if (slot < cap) {
          cs[(int64_t)q * cap + slot] = v[u];
          ci[(int64_t)q * cap + slot] = base + (e >> lq);
        }
      }
    }
  }
}

}  // namespace
int scan16_grid(int64_t nchunk, int nw, int cus) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(cus, (nchunk + nw - 1) / nw));
}
namespace {

template <int KS, int D>
hipError_t scan16_launch(const Scan16Args& a, int nw, hipStream_t st) {
  auto kern = scan16_kernel<KS, D>;
  const int lds = nw * D * (16 * KS * 64 + 1024);
  static unsigned dev_done = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!(__atomic_load_n(&dev_done, __ATOMIC_ACQUIRE) & (1u << (dev & 31)))) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&dev_done, 1u << (dev & 31), __ATOMIC_RELEASE);
  }
  static int cus_of[32] = {};
  int& cus = cus_of[dev & 31];
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
  }
  const int grid = scan16_grid(a.nchunk, nw, cus);
  if ((int64_t)grid * nw * KTH_MAX > a.ldw && a.wtop) return hipErrorInvalidValue;
  kern<<<dim3(grid), dim3(nw * 64), lds, st>>>(a);
  return hipGetLastError();
}

template <int KS>
hipError_t scan16_depth(const Scan16Args& a, int nw, int depth, hipStream_t st) {
  switch (depth) {
    case 2: return scan16_launch<KS, 2>(a, nw, st);
    case 3: return scan16_launch<KS, 3>(a, nw, st);
    case 4: return scan16_launch<KS, 4>(a, nw, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

// waves per workgroup and ring depth for a row width: one wave per CU with the deepest ring the
// LDS and the 6-bit vmcnt hold (4 blocks: 3 in flight, 51 KiB at 512 dims) -- at 10 M x 512 that
// streamed 1.83 ms per query against 1.87-1.93 for 2-4 waves with 2-4 blocks each
// (profiles/r06_v1_scan16_shape_ab.txt: the many-wave forms split the 39 k chunks less evenly);
// $CLM_SCAN_NW / $CLM_SCAN_D (A/B)
void scan16_shape(int dim, int* nw, int* depth) {
  const int blk = 16 * dim * 2 + 1024;
  static const int env_nw = getenv("CLM_SCAN_NW") ? atoi(getenv("CLM_SCAN_NW")) : 0;
  static const int env_d = getenv("CLM_SCAN_D") ? atoi(getenv("CLM_SCAN_D")) : 0;
  int w = env_nw > 0 ? std::min(env_nw, 4) : 1;
  int d = env_d > 0 ? std::min(std::max(env_d, 2), 4) : 4;
  while (d > 2 && w * d * blk > 160 * 1024) --d;
  while (w > 1 && w * d * blk > 160 * 1024) --w;
  *nw = w * d * blk <= 160 * 1024 ? w : 0;
  *depth = d;
}

int64_t scan16_waves(int64_t nchunk, int dim) {
  int nw = 0, d = 0;
  scan16_shape(dim, &nw, &d);
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  (void)hipGetLastError();
  return (int64_t)scan16_grid(nchunk, std::max(nw, 1), cus) * std::max(nw, 1);
}

hipError_t scan16(const Scan16Args& a, hipStream_t st) {
  if (a.N <= 0 || a.nq <= 0) return hipSuccess;
  if (a.nq > 16 || a.dim % 64 || a.dim < 64 || a.dim > 1024 || a.ldo < a.nq || a.ldo > 16 ||
      (a.ldo & (a.ldo - 1)) || (int64_t)(a.nq - 1) * a.nchunk * 4 + 4 > 0x7FFFFFF0 ||
      a.nchunk != (a.N + SCAN_CHUNK - 1) / SCAN_CHUNK)
    return hipErrorInvalidValue;
  int nw = 0, d = 0;
  scan16_shape(a.dim, &nw, &d);
  if (nw < 1) return hipErrorInvalidValue;
  switch (a.dim / 32) {
    case 2: return scan16_depth<2>(a, nw, d, st);
    case 4: return scan16_depth<4>(a, nw, d, st);
    case 6: return scan16_depth<6>(a, nw, d, st);
    case 8: return scan16_depth<8>(a, nw, d, st);
    case 10: return scan16_depth<10>(a, nw, d, st);
    case 12: return scan16_depth<12>(a, nw, d, st);
    case 14: return scan16_depth<14>(a, nw, d, st);
    case 16: return scan16_depth<16>(a, nw, d, st);
    case 18: return scan16_depth<18>(a, nw, d, st);
    case 20: return scan16_depth<20>(a, nw, d, st);
    case 22: return scan16_depth<22>(a, nw, d, st);
    case 24: return scan16_depth<24>(a, nw, d, st);
    case 26: return scan16_depth<26>(a, nw, d, st);
    case 28: return scan16_depth<28>(a, nw, d, st);
    case 30: return scan16_depth<30>(a, nw, d, st);
    case 32: return scan16_depth<32>(a, nw, d, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t collect_ge(const float* scores, int ldq, int nq, int64_t C, const float* th, int* cnt, int cap, float* cs,
                      int64_t* ci, int64_t base, hipStream_t s) {
  if (nq <= 0 || C <= 0) return hipSuccess;
  int lq = 0;
  while ((1 << lq) < ldq) ++lq;
  if ((1 << lq) != ldq || ldq > 16 || nq > ldq || ((uintptr_t)scores & 15)) return hipErrorInvalidValue;
  const int64_t n4 = ((C << lq) + 3) / 4;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 4096));
  collect_ge_kernel<<<gx, 256, 0, s>>>(scores, lq, nq, C, th, cnt, cap, cs, ci, base);
  return hipGetLastError();
}

}  // namespace clm
