// Host-side sanitizer harness of the C-ABI (ASan / UBSan build of the C-ABI
// layer). Built by `make sanitize` with the HOST half of every translation unit under
// -fsanitize=address,undefined (device code is compiled normally: GPU sanitizers are not
// available on this pool), and run without Python, so no preload is needed.
//
//  * every run: argument validation of each entry point (null pointers, bad shapes, bad
//    dtypes), error strings, version / layout queries;
//  * with a HIP device: the resident-index lifecycle (create, f16 + f32 appends that grow the
//    capacity, search on the scan and bounded paths, read-back, offset, reset, destroy),
//    clm_cosine_scores / clm_topk_merge / clm_l2_normalize / clm_fuse_queries on host buffers,
//    each checked against a scalar host reference.
// Exit code 0 = all checks passed (the sanitizers abort the process on their own findings).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "clm.h"

// leaks LeakSanitizer reports at exit from inside the ROCm runtime (HSA / HIP objects that
// live for the process) are not ours; anything allocated by libclm or this harness still counts
extern "C" const char* __lsan_default_suppressions() { return "leak:libhsa-runtime64\nleak:libamdhip64\n"; }

static int failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, #cond, \
                   clm_last_error());                                            \
      ++failures;                                                                \
    }                                                                            \
  } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static float frand() {   // xorshift64*, uniform in [-1, 1)
  rng_state ^= rng_state >> 12;
  rng_state ^= rng_state << 25;
  rng_state ^= rng_state >> 27;
  return (float)((rng_state * 2685821657736338717ull) >> 40) / (float)(1ull << 23) - 1.0f;
}

static void argument_checks() {
  CHECK(clm_version() && std::strlen(clm_version()) > 0);
  CHECK(clm_model_desc_size() == (int32_t)sizeof(clm_model_desc));
  clm_ctx* ctx = nullptr;
  CHECK(clm_ctx_create(0, nullptr, &ctx) == CLM_E_ARG);
  CHECK(std::strlen(clm_last_error()) > 0);
  CHECK(clm_ctx_destroy(nullptr) == CLM_OK);
  CHECK(clm_load_tensor(nullptr, "x", nullptr, CLM_F32, nullptr, 0) == CLM_E_ARG);
  CHECK(clm_finalize(nullptr) != CLM_OK);
  CHECK(clm_encode_image(nullptr, nullptr, CLM_PIX_U8_HWC, 1, nullptr, CLM_F32, 1, nullptr) != CLM_OK);
  CHECK(clm_encode_text(nullptr, nullptr, 1, 77, nullptr, CLM_F32, 1, nullptr) != CLM_OK);
  clm_index* idx = nullptr;
  CHECK(clm_index_create(0, 16, 100, &idx) != CLM_OK);    // dim % 64 != 0
  CHECK(clm_index_create(0, 16, 131072, &idx) != CLM_OK);   // dim > 65536
  CHECK(clm_index_destroy(nullptr) == CLM_OK);
  CHECK(clm_index_size(nullptr) < 0);
  CHECK(clm_index_search(nullptr, nullptr, CLM_F32, 1, 1, nullptr, nullptr, nullptr) != CLM_OK);
  int64_t st[4];
  CHECK(clm_index_stats2(nullptr, st, 4) != CLM_OK);
  CHECK(clm_gemm(0, 99, CLM_EPI_STORE, -1, nullptr, 64, nullptr, 64, 1, 1, 64, nullptr, 1, nullptr, nullptr, nullptr,
                 nullptr) == CLM_E_ARG);
  CHECK(clm_attention(0, 99, 0, nullptr, nullptr, 64, 1, 1, 1, nullptr) == CLM_E_ARG);
  CHECK(clm_layernorm(0, CLM_BF16, nullptr, 100, 4, 100, nullptr, nullptr, 1e-5f, nullptr, 100, nullptr) == CLM_E_ARG);
  CHECK(clm_topk_merge(0, nullptr, nullptr, 1, 0, 1, 1, nullptr, nullptr, nullptr) != CLM_OK);
  CHECK(clm_l2_normalize(0, nullptr, 1, 0, nullptr) != CLM_OK);
}

static double cos64(const float* a, const float* b, int dim) {
  double ab = 0, aa = 0, bb = 0;
  for (int e = 0; e < dim; ++e) {
    ab += (double)a[e] * b[e];
    aa += (double)a[e] * a[e];
    bb += (double)b[e] * b[e];
  }
  return ab / std::sqrt(aa * bb);
}

static void device_checks() {
  const int dim = 128, nq = 5, k = 7;
  // index: f16 rows first (upcast into the fp32 copy when the f32 rows arrive), capacity grows
  clm_index* idx = nullptr;
  CHECK(clm_index_create(0, 8, dim, &idx) == CLM_OK);
  if (!idx) return;
  const int n16 = 300, n32 = 2000, n = n16 + n32;
  std::vector<float> rows((size_t)n * dim);
  for (auto& v : rows) v = frand();
  std::vector<uint16_t> h16((size_t)n16 * dim);
  for (size_t i = 0; i < h16.size(); ++i) {
    const _Float16 h = (_Float16)rows[i];
    std::memcpy(&h16[i], &h, 2);
    rows[i] = (float)h;   // the fp16 rows as given are the reference rows
  }
  CHECK(clm_index_append(idx, h16.data(), CLM_F16, n16, nullptr) == CLM_OK);
  CHECK(clm_index_append(idx, rows.data() + (size_t)n16 * dim, CLM_F32, n32, nullptr) == CLM_OK);
  CHECK(clm_index_size(idx) == n);
  std::vector<float> back((size_t)n * dim);
  CHECK(clm_index_read(idx, 0, n, back.data(), nullptr) == CLM_OK);
  CHECK(std::memcmp(back.data(), rows.data(), back.size() * 4) == 0);
  CHECK(clm_index_read(idx, n - 1, 2, back.data(), nullptr) != CLM_OK);   // past the end

  std::vector<float> q((size_t)nq * dim);
  for (auto& v : q) v = frand();
  std::vector<float> sc((size_t)nq * k);
  std::vector<int64_t> ix((size_t)nq * k);
  for (int pass = 0; pass < 2; ++pass) {   // exact scan, then the bounded path
    if (pass == 1) setenv("CLM_SEARCH_BOUNDED", "1", 1);
    CHECK(clm_index_search(idx, q.data(), CLM_F32, nq, k, sc.data(), ix.data(), nullptr) == CLM_OK);
    for (int i = 0; i < nq; ++i) {
      // host reference: exact cosines, (score desc, index asc)
      std::vector<std::pair<double, int64_t>> all(n);
      for (int j = 0; j < n; ++j) all[j] = {cos64(&q[(size_t)i * dim], &rows[(size_t)j * dim], dim), j};
      std::partial_sort(all.begin(), all.begin() + k, all.end(), [](const auto& a, const auto& b) {
        return a.first > b.first || (a.first == b.first && a.second < b.second);
      });
      for (int t = 0; t < k; ++t) {
        CHECK(ix[(size_t)i * k + t] == all[t].second);
        CHECK(sc[(size_t)i * k + t] == (float)all[t].first);
      }
    }
    unsetenv("CLM_SEARCH_BOUNDED");
  }
  CHECK(clm_index_set_offset(idx, 1000) == CLM_OK);
  CHECK(clm_index_search(idx, q.data(), CLM_F32, 1, 1, sc.data(), ix.data(), nullptr) == CLM_OK);
  CHECK(ix[0] >= 1000);
  int64_t st[4] = {-1, -1, -1, -1};
  CHECK(clm_index_stats2(idx, st, 4) == CLM_OK && st[0] >= 0);
  CHECK(clm_index_reset(idx) == CLM_OK && clm_index_size(idx) == 0);
  CHECK(clm_index_search(idx, q.data(), CLM_F32, nq, 3, sc.data(), ix.data(), nullptr) == CLM_OK);
  CHECK(ix[0] == -1 && std::isinf(sc[0]));   // empty index: (-inf, -1) slots
  CHECK(clm_index_destroy(idx) == CLM_OK);

  // near-duplicate rows: 3000 copies of one row (and 3000 others) overflow the bounded path's
  // 2048-candidate lists; those queries take the whole-list pass (overflow_wide), k = 7 and 1024
  {
    const int nd = 6000, ndup = 3000, nqd = 4;
    std::vector<float> drows((size_t)nd * dim);
    for (auto& v : drows) v = frand();
    for (int j = 1; j < ndup; ++j) std::memcpy(&drows[(size_t)(2 * j) * dim], &drows[0], dim * 4);   // even rows
    clm_index* di = nullptr;
    CHECK(clm_index_create(0, nd, dim, &di) == CLM_OK);
    if (di) {
      CHECK(clm_index_append(di, drows.data(), CLM_F32, nd, nullptr) == CLM_OK);
      std::vector<float> dq((size_t)nqd * dim);
      for (auto& v : dq) v = frand();
      std::memcpy(dq.data(), drows.data(), dim * 4);
      std::memcpy(dq.data() + 2 * dim, drows.data(), dim * 4);
      setenv("CLM_SEARCH_BOUNDED", "1", 1);
      for (int kk : {7, 1024}) {
        int64_t s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
        CHECK(clm_index_stats2(di, s0, 4) == CLM_OK);
        std::vector<float> dsc((size_t)nqd * kk);
        std::vector<int64_t> dix((size_t)nqd * kk);
        CHECK(clm_index_search(di, dq.data(), CLM_F32, nqd, kk, dsc.data(), dix.data(), nullptr) == CLM_OK);
        CHECK(clm_index_stats2(di, s1, 4) == CLM_OK && s1[3] - s0[3] >= 2);   // the two duplicate queries
        for (int i = 0; i < nqd; ++i) {
          std::vector<std::pair<double, int64_t>> all(nd);
          for (int j = 0; j < nd; ++j) all[j] = {cos64(&dq[(size_t)i * dim], &drows[(size_t)j * dim], dim), j};
          std::partial_sort(all.begin(), all.begin() + kk, all.end(), [](const auto& a, const auto& b) {
            return a.first > b.first || (a.first == b.first && a.second < b.second);
          });
          for (int t = 0; t < kk; ++t) {
            CHECK(dix[(size_t)i * kk + t] == all[t].second);
            CHECK(dsc[(size_t)i * kk + t] == (float)all[t].first);
          }
        }
      }
      unsetenv("CLM_SEARCH_BOUNDED");
      CHECK(clm_index_destroy(di) == CLM_OK);
    }
  }

  // exact cosine matrix on host buffers, any dim
  const int cd = 77, cn = 33;
  std::vector<float> cq((size_t)nq * cd), cc((size_t)cn * cd), cout((size_t)nq * cn);
  for (auto& v : cq) v = frand();
  for (auto& v : cc) v = frand();
  CHECK(clm_cosine_scores(0, cq.data(), nq, cc.data(), cn, cd, cout.data(), nullptr) == CLM_OK);
  for (int i = 0; i < nq; ++i)
    for (int j = 0; j < cn; ++j) CHECK(cout[(size_t)i * cn + j] == (float)cos64(&cq[(size_t)i * cd], &cc[(size_t)j * cd], cd));

  // two sorted lists per query merge into one
  const int parts = 2, kin = 4, km = 5;
  std::vector<float> ms = {0.9f, 0.5f, 0.4f, 0.1f, 0.8f, 0.5f, 0.3f, 0.2f};
  std::vector<int64_t> mi = {3, 9, 1, 7, 4, 2, 8, 6};
  std::vector<float> os(km);
  std::vector<int64_t> oi(km);
  CHECK(clm_topk_merge(0, ms.data(), mi.data(), 1, parts, kin, km, os.data(), oi.data(), nullptr) == CLM_OK);
  const int64_t want[km] = {3, 4, 2, 9, 1};
  for (int t = 0; t < km; ++t) CHECK(oi[t] == want[t]);

  // a merge past one LDS sort (topk_any): 5 lists of 3000 with ties and empty slots, k = 4500,
  // against a host sort by (score desc, index asc)
  {
    const int P = 5, KI = 3000, K = 4500, NQ = 2;
    std::vector<float> bs((size_t)NQ * P * KI);
    std::vector<int64_t> bi(bs.size());
    for (size_t j = 0; j < bs.size(); ++j) {
      bs[j] = (float)((int)(frand() * 64.f)) / 64.f;   // many exact ties
      bi[j] = (j % 997 == 5) ? -1 : (int64_t)((j * 7919) % 1000003);
    }
    std::vector<float> bos((size_t)NQ * K);
    std::vector<int64_t> boi((size_t)NQ * K);
    CHECK(clm_topk_merge(0, bs.data(), bi.data(), NQ, P, KI, K, bos.data(), boi.data(), nullptr) == CLM_OK);
    for (int q = 0; q < NQ; ++q) {
      std::vector<std::pair<float, int64_t>> v;
      for (int j = 0; j < P * KI; ++j) {
        const size_t o = (size_t)q * P * KI + j;
        if (bi[o] >= 0) v.push_back({bs[o], bi[o]});
      }
      std::sort(v.begin(), v.end(), [](const std::pair<float, int64_t>& x, const std::pair<float, int64_t>& y) {
        return x.first != y.first ? x.first > y.first : x.second < y.second;
      });
      int bad = 0;
      for (int t = 0; t < K; ++t) bad += (boi[(size_t)q * K + t] != v[t].second || bos[(size_t)q * K + t] != v[t].first);
      CHECK(bad == 0);
    }
  }

  // l2 normalise and query fusion in place on host rows
  std::vector<float> a((size_t)3 * dim), b((size_t)3 * dim);
  for (auto& v : a) v = frand();
  for (auto& v : b) v = frand();
  std::vector<float> fused(a.size());
  CHECK(clm_fuse_queries(0, a.data(), 0.7f, b.data(), 0.3f, 3, dim, fused.data(), nullptr) == CLM_OK);
  CHECK(clm_l2_normalize(0, a.data(), 3, dim, nullptr) == CLM_OK);
  for (int r = 0; r < 3; ++r) {
    double s2 = 0, f2 = 0;
    for (int e = 0; e < dim; ++e) {
      s2 += (double)a[(size_t)r * dim + e] * a[(size_t)r * dim + e];
      f2 += (double)fused[(size_t)r * dim + e] * fused[(size_t)r * dim + e];
    }
    CHECK(std::fabs(s2 - 1.0) < 1e-5 && std::fabs(f2 - 1.0) < 1e-5);
  }
}

int main() {
  argument_checks();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    device_checks();
    std::printf("host_check: argument + device checks, %d failure(s)\n", failures);
  } else {
    (void)hipGetLastError();
    std::printf("host_check: argument checks (no HIP device), %d failure(s)\n", failures);
  }
  return failures ? 1 : 0;
}
