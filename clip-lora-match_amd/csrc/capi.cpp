// libclm C-ABI (include/clm.h): context, weight packing, encode drivers, HBM index.
//
// Host runtime behind the reference's Python API:
//   load_clip_model            models/clip_model.py:37-82     -> clm_ctx_create/_load_tensor/_finalize
//   PEFT LoRA (r, alpha/r)     models/lora_adapter.py:21-43    -> merged or K-extension packing
//   encode_image/encode_text   models/clip_model.py:89-150     -> clm_encode_image/_text
//   TextSearchIndex            src/embedding/search.py:24-115  -> clm_index_*
// Weights arrive by transformers / PEFT state-dict name; finalize() fuses q/k/v
// into one [3d, K] matrix (q rows pre-scaled by 64^-1/2), folds LoRA either into
// the weights (W + (alpha/r) B A, fp32 then cast) or as K-extension columns
// [W | (alpha/r) B] against activations [X | X A^T], and uploads everything in
// the compute dtype (bf16/fp16), keeping LayerNorm, biases, embeddings and the
// projections in fp32.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "clm.h"
#include "kernels.hpp"

using namespace clm;

namespace {

thread_local std::string g_err;
// clm_debug_set / $CLM_GEMM_DEBUG: GemmArgs::debug of clm_gemm (micro-benchmarks only)
int g_gemm_debug = getenv("CLM_GEMM_DEBUG") ? atoi(getenv("CLM_GEMM_DEBUG")) : 0;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(CLM_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

uint16_t host_f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
uint16_t host_f32_to_f16(float f) {
  _Float16 h = (_Float16)f;
  uint16_t r;
  std::memcpy(&r, &h, 2);
  return r;
}
float host_f16_to_f32(uint16_t v) {
  _Float16 h;
  std::memcpy(&h, &v, 2);
  return (float)h;
}
float host_bf16_to_f32(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

struct LayerW {
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  // k_*: the weight's row stride and the K of GEMMs that need whole 64-wide K-steps (G2, split-K);
  // kl_*: the logical K, in + round_up(r, 32) in unmerged-LoRA mode (gemm_kernel and the fused
  // attention run the 32-wide last K-step), = k_* otherwise
  u16* w_qkv = nullptr; float* b_qkv = nullptr; int k_qkv = 0, kl_qkv = 0;
  u16* w_out = nullptr; float* b_out = nullptr; int k_out = 0, kl_out = 0;
  u16* w_fc1 = nullptr; float* b_fc1 = nullptr; int k_fc1 = 0, kl_fc1 = 0;
  u16* w_fc2 = nullptr; float* b_fc2 = nullptr; int k_fc2 = 0, kl_fc2 = 0;
  // unmerged LoRA: the stacked A of each GEMM input in the compute dtype, [RPAD, in] with zero rows
  // past r_* (the down-projection GEMM writes all RPAD extension columns: the pad ones get zeros)
  u16* a_qkv = nullptr; int r_qkv = 0;
  u16* a_out = nullptr; int r_out = 0;
  u16* a_fc1 = nullptr; int r_fc1 = 0;
  u16* a_fc2 = nullptr; int r_fc2 = 0;
};

struct Tower {
  bool vision = false;
  bool q_log2e = false;   // q_proj weights carry log2(e) (attention_folds_log2e)
  int d = 0, L = 0, H = 0, mlp = 0;
  std::vector<LayerW> layers;
  float *projT = nullptr, *fin_g = nullptr, *fin_b = nullptr;
  // vision
  u16* patch_w = nullptr; int kp = 0;
  float *cls = nullptr, *pos = nullptr, *pre_g = nullptr, *pre_b = nullptr, *lut = nullptr;
  // text
  float *tok = nullptr, *tpos = nullptr;
  // workspace
  int64_t maxM = 0;
  float* h = nullptr;
  u16 *X = nullptr, *QKV = nullptr, *O = nullptr, *Hm = nullptr, *P = nullptr;
  float* pooled = nullptr;  // [max_batch, proj_dim] un-normalised projections
  float* hc = nullptr;      // [max_batch, d] pooled residual rows of the pruned last layer
  u16* Oc = nullptr;        // [max_batch, ldo] their attention-output rows
  // varlen text plan (text_plan): per caption live rows / offsets, packed-row map, fused-attention
  // tiles, {live rows, tiles}; a sub-batch view at b0 uses lens / tiles + b0, offs / counts + 2 b0
  int *vl_lens = nullptr, *vl_offs = nullptr, *vl_rowmap = nullptr, *vl_tiles = nullptr, *vl_counts = nullptr;
  int64_t ldx = 0, ldo = 0, ldm = 0;
};

// K-extension width of the unmerged LoRA mode: the storage (weight columns, activation columns;
// rows stay whole 64-wide K-steps), of which GEMMs multiply round_up(sum r, 32) (LORA_GRANULE)
constexpr int RPAD = 64;
constexpr int LORA_GRANULE = 32;

}  // namespace

struct clm_ctx {
  int dev = 0;
  clm_model_desc desc{};
  bool finalized = false;
  bool lora_enabled = true;
  std::unordered_map<std::string, HostTensor> host;
  std::vector<void*> allocs;       // weights + workspace
  Tower vis, txt;
  // host<->device staging
  void* stage_in = nullptr; size_t stage_in_bytes = 0;
  void* stage_out = nullptr; size_t stage_out_bytes = 0;
  int32_t* ids_dev = nullptr;
  // two-tower concurrency + graph replay (clm_encode_pair)
  // Each tower's batch is cut into `split` sub-batches on their own streams (disjoint row
  // ranges of the tower workspace): one sub-batch's write-bound GEMM epilogues and
  // latency-bound LN/attention launches overlap another's MFMA main loops.
  static constexpr int MAX_SPLIT = 4;
  hipStream_t ps[2 * MAX_SPLIT] = {};
  hipEvent_t pev[2 * MAX_SPLIT] = {};
  hipEvent_t ev_fork = nullptr, ev_done = nullptr;
  typedef std::tuple<const void*, int, int, const void*, int, int, void*, void*, int, int, int> PairKey;
  std::map<PairKey, hipGraphExec_t> graphs;
  int last_pair_path = -1;   // clm_pair_path: 0 = two tower streams (-1: no encode_pair yet)
  // kernel timing (clm_prof_*): events recorded on the launch stream
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  struct Rec { int cat; double work; size_t e0, e1; };
  std::vector<Rec> recs;

  // operand type of a tower's GEMMs / attention (CLM_COMPUTE_MIXED: bf16 vision, fp16 text)
  bool bf16(bool vision) const {
    return desc.compute_dtype == CLM_BF16 || (vision && desc.compute_dtype == CLM_COMPUTE_MIXED);
  }

  template <typename T>
  int dalloc(T** p, size_t count) {
    void* q = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(&q, count * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(CLM_E_OOM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed");
    }
    allocs.push_back(q);
    *p = (T*)q;
    return CLM_OK;
  }
  void drop_graphs() {
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    graphs.clear();
  }
  void free_all() {
    drop_graphs();
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
    if (stage_in) (void)hipFree(stage_in);
    if (stage_out) (void)hipFree(stage_out);
    stage_in = stage_out = nullptr;
    stage_in_bytes = stage_out_bytes = 0;
    vis = Tower();
    txt = Tower();
    ids_dev = nullptr;
  }
};

struct clm_index {
  int dev = 0;
  int64_t cap = 0, n = 0, dim = 0, offset = 0;
  // MFMA-pass operands: fp16 rows (f16 appends: the rows as given; f32 appends: the rows
  // normalised in fp32, then rounded) + fp32 inverse norms of those fp16 rows
  u16* rows = nullptr;
  float* inv = nullptr;
  // the caller's fp32 rows, kept once any f32 rows were appended (f16 appends upcast into it):
  // the exact re-scoring reads these; without them the fp16 rows ARE the caller's rows
  float* rows32 = nullptr;
  // search workspaces (grown on demand): ws = query staging, ws2 = per-query-block buffers,
  // ws3 = chunked score matrices of the exact scans
  void* ws = nullptr; size_t ws_bytes = 0;
  void* ws2 = nullptr; size_t ws2_bytes = 0;
  void* ws3 = nullptr; size_t ws3_bytes = 0;
  // ws4 = the overflow passes' gathered queries / candidate lists (overflow_wide, exact re-scan)
  void* ws4 = nullptr; size_t ws4_bytes = 0;
  // strided row sample for the threshold pass, rebuilt when n changes
  u16* samp = nullptr; float* samp_inv = nullptr; int64_t samp_S = 0, samp_n = -1, samp_cap = 0;
  // order keys {min, max} of inv[0, n) for the filter GEMM's skip test, rebuilt with the sample
  unsigned* inv_keys = nullptr; int64_t inv_keys_n = -1;
  // queries served by: [0] sampled bounded search, [1] the full exact scan, [2] overflow re-runs,
  // [3] bounded search with the chunked fp16 scan as step 1
  // [4] / [5]: queries whose filter pass ran on G2 256 x 192 / gemm_kernel 256 x 256 (dense blocks)
  // [6]: queries served by the small-batch streaming search (search_small)
  int64_t search_stats[7] = {0, 0, 0, 0, 0, 0, 0};
};

namespace {

const HostTensor* find(const clm_ctx* c, const std::string& n) {
  auto it = c->host.find(n);
  return it == c->host.end() ? nullptr : &it->second;
}

int need(const clm_ctx* c, const std::string& n, int64_t numel, const HostTensor** out) {
  const HostTensor* t = find(c, n);
  if (!t) return fail(CLM_E_MISSING, "missing tensor '" + n + "'");
  if ((int64_t)t->data.size() != numel)
    return fail(CLM_E_ARG, "tensor '" + n + "' has " + std::to_string(t->data.size()) + " elements, expected " +
                               std::to_string(numel));
  *out = t;
  return CLM_OK;
}

int upload_f32(clm_ctx* c, const std::vector<float>& v, float** dst) {
  int r = c->dalloc(dst, v.size());
  if (r) return r;
  HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  return CLM_OK;
}

int upload_16(clm_ctx* c, const std::vector<float>& v, u16** dst, bool bf) {
  std::vector<u16> h(v.size());
  if (bf)
    for (size_t i = 0; i < v.size(); ++i) h[i] = host_f32_to_bf16(v[i]);
  else
    for (size_t i = 0; i < v.size(); ++i) h[i] = host_f32_to_f16(v[i]);
  int r = c->dalloc(dst, h.size());
  if (r) return r;
  HIPCHK(hipMemcpy(*dst, h.data(), h.size() * sizeof(u16), hipMemcpyHostToDevice));
  return CLM_OK;
}

// the stacked LoRA A [r_ext, in] (fp32 host) as the [RPAD, in] 16-bit W operand of the
// down-projection GEMM, rows r_ext .. RPAD-1 zero
int upload_lora_a(clm_ctx* c, const std::vector<float>& A, int r_ext, int in, u16** dst, bool bf) {
  std::vector<float> pad((size_t)RPAD * in, 0.f);
  std::copy(A.begin(), A.begin() + (size_t)r_ext * in, pad.begin());
  return upload_16(c, pad, dst, bf);
}

int get_f32(clm_ctx* c, const std::string& n, int64_t numel, float** dst) {
  const HostTensor* t;
  int r = need(c, n, numel, &t);
  if (r) return r;
  return upload_f32(c, t->data, dst);
}

// A linear's weight block for a (possibly fused) GEMM: rows [row0, row0+out) of W,
// its LoRA pair (if targeted and enabled), and the extension offset for unmerged mode.
struct LinearSpec {
  std::string path;
  int in, out;
  bool lora;
};

// Build a fused [sum(out), K] weight (fp32 host) for linears sharing one input.
// merged: W += s * B A.  unmerged: K = in + RPAD, columns [in + off, in + off + r) = s * B.
// Also returns the stacked A [r_ext, in] for the unmerged mode.
int build_fused(clm_ctx* c, const std::vector<LinearSpec>& specs, float q_scale, std::vector<float>& W,
                std::vector<float>& bias, int& K, std::vector<float>& A_stack, int& r_ext, int& K_log) {
  const clm_model_desc& d = c->desc;
  const bool unmerged = d.lora_mode == CLM_LORA_UNMERGED;
  const int in = specs[0].in;
  int total_out = 0;
  r_ext = 0;
  for (auto& s : specs) {
    total_out += s.out;
    if (s.lora) r_ext += d.lora_r;
  }
  K = (unmerged && r_ext > 0) ? in + RPAD : in;
  K_log = (unmerged && r_ext > 0) ? in + (r_ext + LORA_GRANULE - 1) / LORA_GRANULE * LORA_GRANULE : in;
  if (r_ext > RPAD) return fail(CLM_E_ARG, "LoRA rank too large for the K-extension (sum r > 64)");
  W.assign((size_t)total_out * K, 0.f);
  bias.assign(total_out, 0.f);
  A_stack.assign((size_t)r_ext * in, 0.f);
  const float scaling = d.lora_r > 0 ? d.lora_alpha / (float)d.lora_r : 0.f;
  int row0 = 0, roff = 0;
  for (size_t si = 0; si < specs.size(); ++si) {
    const LinearSpec& s = specs[si];
    const HostTensor *w, *b;
    int r = need(c, s.path + ".weight", (int64_t)s.out * s.in, &w);
    if (r) return r;
    r = need(c, s.path + ".bias", s.out, &b);
    if (r) return r;
    const float qs = si == 0 ? q_scale : 1.0f;   // the first linear's scale (q_proj: see build_tower)
    for (int o = 0; o < s.out; ++o) {
      std::memcpy(&W[(size_t)(row0 + o) * K], &w->data[(size_t)o * s.in], s.in * sizeof(float));
      bias[row0 + o] = b->data[o];
    }
    if (s.lora) {
      const HostTensor *A, *B;
      const std::string base = "base_model.model." + s.path;
      r = need(c, base + ".lora_A.weight", (int64_t)d.lora_r * s.in, &A);
      if (r) return r;
      r = need(c, base + ".lora_B.weight", (int64_t)s.out * d.lora_r, &B);
      if (r) return r;
      if (!unmerged) {
        for (int o = 0; o < s.out; ++o) {
          float* wr = &W[(size_t)(row0 + o) * K];
          for (int j = 0; j < d.lora_r; ++j) {
            const float bj = scaling * B->data[(size_t)o * d.lora_r + j];
            const float* ar = &A->data[(size_t)j * s.in];
            for (int i = 0; i < s.in; ++i) wr[i] += bj * ar[i];
          }
        }
      } else {
        for (int o = 0; o < s.out; ++o)
          for (int j = 0; j < d.lora_r; ++j)
            W[(size_t)(row0 + o) * K + s.in + roff + j] = scaling * B->data[(size_t)o * d.lora_r + j];
        std::memcpy(&A_stack[(size_t)roff * in], A->data.data(), (size_t)d.lora_r * in * sizeof(float));
      }
      roff += d.lora_r;
    }
    if (qs != 1.0f) {
      for (int o = 0; o < s.out; ++o) {
        float* wr = &W[(size_t)(row0 + o) * K];
        for (int i = 0; i < K; ++i) wr[i] *= qs;
        bias[row0 + o] *= qs;
      }
    }
    row0 += s.out;
  }
  if (!unmerged) r_ext = 0;
  return CLM_OK;
}

int build_tower(clm_ctx* c, Tower& T, bool vision) {
  const clm_model_desc& d = c->desc;
  const clm_tower_desc& td = vision ? d.vision : d.text;
  T.vision = vision;
  T.d = td.hidden; T.L = td.layers; T.H = td.heads; T.mlp = td.mlp;
  if (T.d != T.H * 64) return fail(CLM_E_ARG, "head_dim must be 64");
  if (T.d % 128 || T.d > 1024 || T.mlp % 64) return fail(CLM_E_ARG, "hidden must be a multiple of 128 (<=1024), mlp of 64");
  const std::string pre = vision ? "vision_model" : "text_model";
  const bool lora_on = c->lora_enabled && d.lora_r > 0;
  const uint32_t tg = lora_on ? d.lora_targets : 0u;
  const bool unmerged = d.lora_mode == CLM_LORA_UNMERGED;
  // q_proj carries the 64^-1/2 score scale (head_dim 64: a power of two, bit-identical to scaling
  // the scores), and log2(e) too where the tower's attention kernel takes its scores in the log2
  // domain (attention_folds_log2e: the L/14 image tower's T = 577)
  const int Tseq = vision ? (d.image_size / d.patch) * (d.image_size / d.patch) + 1 : 0;
  T.q_log2e = vision && attention_folds_log2e(c->bf16(true), false, Tseq);
  const float qscale = T.q_log2e ? 0.125f * 1.4426950408889634f : 0.125f;
  int r;
  T.layers.resize(T.L);
  for (int l = 0; l < T.L; ++l) {
    LayerW& Lw = T.layers[l];
    const std::string p = pre + ".encoder.layers." + std::to_string(l);
    if ((r = get_f32(c, p + ".layer_norm1.weight", T.d, &Lw.ln1_g))) return r;
    if ((r = get_f32(c, p + ".layer_norm1.bias", T.d, &Lw.ln1_b))) return r;
    if ((r = get_f32(c, p + ".layer_norm2.weight", T.d, &Lw.ln2_g))) return r;
    if ((r = get_f32(c, p + ".layer_norm2.bias", T.d, &Lw.ln2_b))) return r;
    std::vector<float> W, b, A;
    int K, rext, KL;
    // q, k, v share the LN1 output: one fused GEMM
    std::vector<LinearSpec> qkv = {{p + ".self_attn.q_proj", T.d, T.d, (tg & CLM_LORA_Q) != 0},
                                   {p + ".self_attn.k_proj", T.d, T.d, (tg & CLM_LORA_K) != 0},
                                   {p + ".self_attn.v_proj", T.d, T.d, (tg & CLM_LORA_V) != 0}};
    if ((r = build_fused(c, qkv, qscale, W, b, K, A, rext, KL))) return r;
    if ((r = upload_16(c, W, &Lw.w_qkv, c->bf16(vision))) || (r = upload_f32(c, b, &Lw.b_qkv))) return r;
    Lw.k_qkv = K; Lw.kl_qkv = KL; Lw.r_qkv = rext;
    if (unmerged && rext && (r = upload_lora_a(c, A, rext, T.d, &Lw.a_qkv, c->bf16(vision)))) return r;

    std::vector<LinearSpec> outp = {{p + ".self_attn.out_proj", T.d, T.d, (tg & CLM_LORA_OUT) != 0}};
    if ((r = build_fused(c, outp, 1.0f, W, b, K, A, rext, KL))) return r;
    if ((r = upload_16(c, W, &Lw.w_out, c->bf16(vision))) || (r = upload_f32(c, b, &Lw.b_out))) return r;
    Lw.k_out = K; Lw.kl_out = KL; Lw.r_out = rext;
    if (unmerged && rext && (r = upload_lora_a(c, A, rext, T.d, &Lw.a_out, c->bf16(vision)))) return r;

    std::vector<LinearSpec> fc1 = {{p + ".mlp.fc1", T.d, T.mlp, (tg & CLM_LORA_FC1) != 0}};
    if ((r = build_fused(c, fc1, 1.0f, W, b, K, A, rext, KL))) return r;
    if ((r = upload_16(c, W, &Lw.w_fc1, c->bf16(vision))) || (r = upload_f32(c, b, &Lw.b_fc1))) return r;
    Lw.k_fc1 = K; Lw.kl_fc1 = KL; Lw.r_fc1 = rext;
    if (unmerged && rext && (r = upload_lora_a(c, A, rext, T.d, &Lw.a_fc1, c->bf16(vision)))) return r;

    std::vector<LinearSpec> fc2 = {{p + ".mlp.fc2", T.mlp, T.d, (tg & CLM_LORA_FC2) != 0}};
    if ((r = build_fused(c, fc2, 1.0f, W, b, K, A, rext, KL))) return r;
    if ((r = upload_16(c, W, &Lw.w_fc2, c->bf16(vision))) || (r = upload_f32(c, b, &Lw.b_fc2))) return r;
    Lw.k_fc2 = K; Lw.kl_fc2 = KL; Lw.r_fc2 = rext;
    if (unmerged && rext && (r = upload_lora_a(c, A, rext, T.mlp, &Lw.a_fc2, c->bf16(vision)))) return r;
  }
  // projection, transposed to [d, D] for coalesced reads in pool_project
  {
    const HostTensor* pw;
    const std::string pn = vision ? "visual_projection.weight" : "text_projection.weight";
    if ((r = need(c, pn, (int64_t)d.proj_dim * T.d, &pw))) return r;
    std::vector<float> pt((size_t)T.d * d.proj_dim);
    for (int j = 0; j < d.proj_dim; ++j)
      for (int i = 0; i < T.d; ++i) pt[(size_t)i * d.proj_dim + j] = pw->data[(size_t)j * T.d + i];
    if ((r = upload_f32(c, pt, &T.projT))) return r;
  }
  const int64_t B = d.max_batch;
  if (vision) {
    const int G = d.image_size / d.patch, Tn = G * G + 1;
    if ((r = get_f32(c, pre + ".post_layernorm.weight", T.d, &T.fin_g))) return r;
    if ((r = get_f32(c, pre + ".post_layernorm.bias", T.d, &T.fin_b))) return r;
    if ((r = get_f32(c, pre + ".pre_layrnorm.weight", T.d, &T.pre_g))) return r;
    if ((r = get_f32(c, pre + ".pre_layrnorm.bias", T.d, &T.pre_b))) return r;
    if ((r = get_f32(c, pre + ".embeddings.class_embedding", T.d, &T.cls))) return r;
    if ((r = get_f32(c, pre + ".embeddings.position_embedding.weight", (int64_t)Tn * T.d, &T.pos))) return r;
    const int kreal = d.channels * d.patch * d.patch;
    T.kp = (int)round_up(kreal, 64);
    const HostTensor* pw;
    if ((r = need(c, pre + ".embeddings.patch_embedding.weight", (int64_t)T.d * kreal, &pw))) return r;
    std::vector<float> wp((size_t)T.d * T.kp, 0.f);
    for (int o = 0; o < T.d; ++o) std::memcpy(&wp[(size_t)o * T.kp], &pw->data[(size_t)o * kreal], kreal * 4);
    if ((r = upload_16(c, wp, &T.patch_w, c->bf16(true)))) return r;
    // CLIPImageProcessor rescale (float64 multiply -> float32) then (x - mean) / std in float32
    std::vector<float> lut((size_t)d.channels * 256);
    for (int ch = 0; ch < d.channels; ++ch)
      for (int u = 0; u < 256; ++u) {
        const float x = (float)((double)u * (1.0 / 255.0));
        lut[(size_t)ch * 256 + u] = (x - d.mean[ch % 3]) / d.std[ch % 3];
      }
    if ((r = upload_f32(c, lut, &T.lut))) return r;
    T.maxM = B * Tn;
    if ((r = c->dalloc(&T.P, (size_t)B * G * G * T.kp))) return r;
  } else {
    if ((r = get_f32(c, pre + ".final_layer_norm.weight", T.d, &T.fin_g))) return r;
    if ((r = get_f32(c, pre + ".final_layer_norm.bias", T.d, &T.fin_b))) return r;
    if ((r = get_f32(c, pre + ".embeddings.token_embedding.weight", (int64_t)d.vocab * T.d, &T.tok))) return r;
    if ((r = get_f32(c, pre + ".embeddings.position_embedding.weight", (int64_t)d.max_pos * T.d, &T.tpos))) return r;
    T.maxM = B * d.max_pos;
  }
  T.ldx = T.d + RPAD;
  T.ldo = T.d + RPAD;
  T.ldm = T.mlp + RPAD;
  if ((r = c->dalloc(&T.h, (size_t)T.maxM * T.d))) return r;
  if ((r = c->dalloc(&T.X, (size_t)T.maxM * T.ldx))) return r;
  if ((r = c->dalloc(&T.QKV, (size_t)T.maxM * 3 * T.d))) return r;
  if ((r = c->dalloc(&T.O, (size_t)T.maxM * T.ldo))) return r;
  if ((r = c->dalloc(&T.Hm, (size_t)T.maxM * T.ldm))) return r;
  if ((r = c->dalloc(&T.pooled, (size_t)B * d.proj_dim))) return r;
  if ((r = c->dalloc(&T.hc, (size_t)B * T.d))) return r;
  if ((r = c->dalloc(&T.Oc, (size_t)B * T.ldo))) return r;
  if (!T.vision) {
    if ((r = c->dalloc(&T.vl_lens, (size_t)B))) return r;
    if ((r = c->dalloc(&T.vl_offs, (size_t)2 * B + 1))) return r;
    if ((r = c->dalloc(&T.vl_rowmap, (size_t)T.maxM))) return r;
    if ((r = c->dalloc(&T.vl_tiles, (size_t)B))) return r;
    if ((r = c->dalloc(&T.vl_counts, (size_t)2 * B))) return r;
  }
  return CLM_OK;
}

int ensure_stage(void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return CLM_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return fail(CLM_E_OOM, "staging allocation failed");
  }
  *cap = bytes;
  return CLM_OK;
}

// time one launch when profiling is on: returns the event-pair slot or -1
struct ProfScope {
  clm_ctx* c; hipStream_t st; int cat; double work; size_t e0 = 0; bool on = false;
  ProfScope(clm_ctx* c_, hipStream_t st_, int cat_, double work_) : c(c_), st(st_), cat(cat_), work(work_) {
    if (!c->prof) return;
    if (c->ev_used + 2 > c->ev_pool.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) { (void)hipGetLastError(); return; }
        c->ev_pool.push_back(e);
      }
    }
    e0 = c->ev_used;
    c->ev_used += 2;
    on = hipEventRecord(c->ev_pool[e0], st) == hipSuccess;
  }
  ~ProfScope() {
    if (!on) return;
    if (hipEventRecord(c->ev_pool[e0 + 1], st) == hipSuccess) c->recs.push_back({cat, work, e0, e0 + 1});
  }
};
#define PROF(cat, work) ProfScope prof_scope_##__LINE__(c, st, cat, work)

#define KCHK(x)                                                                                   \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return fail(CLM_E_HIP, std::string("kernel launch ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

// LN into X for a layer's q/k/v (or fc1) GEMM input
LnArgs ln_into_x(clm_ctx* c, Tower& T, int64_t M, const float* g, const float* b, float* h = nullptr) {
  LnArgs a{};
  if (!h) h = T.h;
  a.mode = 0; a.src = h; a.lds = T.d; a.hf = h; a.ldh = T.d;
  a.g1 = g; a.b1 = b; a.y = T.X; a.ldy = T.ldx;
  a.M = (int)M; a.d = T.d; a.eps = c->desc.ln_eps;
  return a;
}

// Unmerged LoRA, the down-projection of a GEMM input (PEFT lora_A, models/clip_model.py:78):
// X[:, K : K + RPAD) = X[:, :K] . A^T as a skinny MFMA GEMM (N = RPAD, 64 x 64 tiles, fp32
// accumulate, rounded once to the compute dtype), so the consumer GEMM's K-extension
// [X | X A^T] . [W | (alpha/r) B]^T adds the low-rank update in its own main loop. The input's
// rows are read once more (19.7 MB for the vision q/k/v input at batch 256, ~3 us); the round-4
// VALU form (24 wave reductions per row inside the LayerNorm / a row-per-wave kernel) cost
// 1.6 ms per pair step (profiles/r05_v2_unmerged_trace.txt).
hipError_t lora_down_gemm(bool bf, u16* X, int64_t ldx, int M, int K, const u16* A, const int* mdev,
                          hipStream_t st) {
  GemmArgs g{};
  g.A = X; g.lda = ldx; g.W = A; g.ldw = K; g.M = M; g.N = RPAD; g.K = K;
  g.out = X + K; g.ldo = ldx; g.m_dev = mdev;
  static const int cfg = getenv("CLM_LORA_DOWN_CFG") ? atoi(getenv("CLM_LORA_DOWN_CFG")) : GEMM_CFG_SKINNY;   // A/B
  return gemm_cfg(bf, EPI_STORE, cfg, g, st);
}

// Last-layer pruning (default; $CLM_NO_PRUNE=1 runs every row): the encoders return only the
// pooled row of each item (vision CLS row 0, text first-EOS row: TF/models/clip/
// modeling_clip.py:558-580, 650), and after the last layer's attention every op is row-wise
// (out_proj, LN2, fc1, fc2 + their LoRA). So the last layer runs q/k/v and attention on all
// B*S rows, then out_proj .. fc2 on the B pooled rows only (gathered into T.hc / T.Oc): the
// pooled embeddings are the same rows through the same kernels.
bool prune_last_layer() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLM_NO_PRUNE");
    v = (e && atoi(e)) ? 0 : 1;
  }
  return v == 1 && !(g_gemm_debug & 8);   // clm_debug_set bit 8: every row (tests)
}

// Varlen text (default; $CLM_TEXT_VARLEN=0 or clm_debug_set bit 32: every padded row): the text
// tower is causal and pools each caption's first-EOS row, so rows after it cannot reach the
// output. Only each caption's live rows (through its first EOS) are packed and encoded; the
// embeddings are bit-identical to encoding all L rows (rows are independent in every kernel but
// attention, whose keys of a live query are all live; tests/test_gpu_encode.py). Needs the fused
// attention kernel (unmerged LoRA included: its down-projection GEMMs read the live row count too).
bool text_varlen_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLM_TEXT_VARLEN");
    v = (e && !atoi(e)) ? 0 : 1;
  }
  return v == 1 && !(g_gemm_debug & 32);
}

// q/k/v projection + attention fused into one launch for T <= 128 (k_gemm_attn.hip) unless
// $CLM_FUSED_ATTN=0 or clm_debug_set bit 16 (tests: the two-kernel path, bit-identical)
bool fused_attention(int T, int H, int d, int K) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLM_FUSED_ATTN");
    v = (e && !atoi(e)) ? 0 : 1;
  }
  return v == 1 && !(g_gemm_debug & 16) && gemm_attn_supported(T, H, d, K);
}

// Per-call state of one tower's encoder pass (run_layers).
struct LayerRun {
  Tower* T;
  int B, S;
  bool causal, vl, bf;
  const int32_t* ids;
  const int* mdev;            // varlen: device-resident live row count (T.vl_counts)
  double Mx, attn_pairs;      // executed rows / attention pairs (profiling)
};

int make_run(clm_ctx* c, Tower& T, int B, int S, bool causal, const int32_t* ids, bool vl, hipStream_t st,
             LayerRun* r) {
  *r = LayerRun{&T, B, S, causal, vl, c->bf16(T.vision), ids, vl ? T.vl_counts : nullptr, (double)B * S,
                (double)B * S * S};
  // varlen (packed live text rows): the row-wise kernels read the live row count from
  // T.vl_counts; the profiled pass (no graph, may sync) counts the executed rows and attention pairs
  if (vl && c->prof) {
    std::vector<int> lens(B);
    HIPCHK(hipMemcpyAsync(lens.data(), T.vl_lens, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    r->Mx = r->attn_pairs = 0;
    for (int v : lens) { r->Mx += v; r->attn_pairs += (double)v * v; }
  }
  return CLM_OK;
}

double attn_flops(const LayerRun& R, int l) {
  const Tower& T = *R.T;
  return 2.0 * R.Mx * 3 * T.d * T.layers[l].kl_qkv + 4.0 * T.H * R.attn_pairs * 64;
}

// layer l's q/k/v projection + attention of one tower: T.X -> T.O
int attn_step(clm_ctx* c, const LayerRun& R, int l, hipStream_t st) {
  Tower& T = *R.T;
  LayerW& Lw = T.layers[l];
  const bool bf = R.bf;
  GemmArgs g{};
  g.A = T.X; g.lda = T.ldx; g.M = R.B * R.S; g.N = 3 * T.d; g.K = Lw.kl_qkv; g.out = T.QKV; g.ldo = 3 * T.d;
  g.W = Lw.w_qkv; g.ldw = Lw.k_qkv; g.bias = Lw.b_qkv;
  if (R.vl) {   // packed live rows of variable-length captions
    PROF(CLM_PROF_GEMM, attn_flops(R, l));
    KCHK(gemm_attn_varlen(bf, R.causal, g.A, g.lda, g.W, g.ldw, g.bias, T.O, T.ldo, R.B, R.S, T.H, T.d, g.K,
                          T.vl_lens, T.vl_offs, T.vl_tiles, T.vl_counts, st));
  } else if (fused_attention(R.S, T.H, T.d, g.K)) {
    // one launch: the q/k/v GEMM's tiles attend their own sequences (GEMM + attention FLOPs)
    PROF(CLM_PROF_GEMM, attn_flops(R, l));
    KCHK(gemm_attn(bf, R.causal, g.A, g.lda, g.W, g.ldw, g.bias, T.O, T.ldo, R.B, R.S, T.H, T.d, g.K, st));
  } else {
    { PROF(CLM_PROF_GEMM, 2.0 * g.M * g.N * g.K); KCHK(gemm(bf, EPI_STORE, g, st)); }
    { PROF(CLM_PROF_ATTN, 4.0 * R.B * T.H * (double)R.S * R.S * 64);
      KCHK(attention(bf, R.causal, T.QKV, 3 * T.d, T.O, T.ldo, R.B, R.S, T.H, T.d, st, T.q_log2e)); }
  }
  return CLM_OK;
}

// the pruned last layer's residual GEMMs have only B (pooled) rows: K is split into slices of
// >= 4 K-steps (a fixed count per shape, so a row's bits do not depend on B), partials in the
// QKV workspace, which is idle by then (B * S rows * 3d 16-bit values); 75 µs of idle chip per
// launch before (profiles/r02_v5_pooled_splitk_ab.txt)
int pooled_resid(clm_ctx* c, const LayerRun& R, GemmArgs& g, hipStream_t st) {
  const int nk = g.K / 64;
  int slices = 1;
  for (int sl = nk / 4; sl >= 2; --sl)
    if (nk % sl == 0 && gemm_splitk_ws_bytes(1, g.N, sl) <= (size_t)R.S * 3 * R.T->d * 2) { slices = sl; break; }
  PROF(CLM_PROF_GEMM, 2.0 * g.M * g.N * g.K);
  if (slices > 1) KCHK(gemm_splitk_resid(R.bf, g, slices, (float*)R.T->QKV, st));
  else KCHK(gemm_cfg(R.bf, EPI_RESID, GEMM_CFG_SPLITK, g, st));
  return CLM_OK;
}

// The four row-wise GEMMs and two LayerNorms of layer l after its attention, as (M rows of) one
// tower: out_proj (+= h), LN2 -> X, fc1 (GELU) -> Hm, fc2 (+= h), next layer's LN1 -> X.
struct PostOps {
  GemmArgs out, fc1, fc2;
  LnArgs ln2, ln1;
  bool has_ln1;
  double rows;   // executed rows (profiling)
};
PostOps post_ops(clm_ctx* c, const LayerRun& R, int l, int64_t M, float* h, u16* O, bool pooled) {
  Tower& T = *R.T;
  LayerW& Lw = T.layers[l];
  const int* mdev = pooled ? nullptr : R.mdev;
  PostOps p{};
  p.rows = pooled ? (double)M : R.Mx;
  GemmArgs& g = p.out;
  // pooled rows: split-K over whole 64-wide K-steps (the extension's pad columns are zero on both sides)
  g.A = O; g.lda = T.ldo; g.W = Lw.w_out; g.ldw = Lw.k_out; g.M = (int)M; g.N = T.d; g.K = pooled ? Lw.k_out : Lw.kl_out;
  g.out = h; g.ldo = T.d; g.bias = Lw.b_out; g.m_dev = mdev;
  p.ln2 = ln_into_x(c, T, M, Lw.ln2_g, Lw.ln2_b, h);
  p.ln2.m_dev = mdev;
  GemmArgs& f = p.fc1;
  f.A = T.X; f.lda = T.ldx; f.M = (int)M; f.N = T.mlp; f.K = Lw.k_fc1; f.out = T.Hm; f.ldo = T.ldm;
  f.W = Lw.w_fc1; f.ldw = Lw.k_fc1; f.bias = Lw.b_fc1; f.m_dev = mdev;
  GemmArgs& f2 = p.fc2;
  f2.A = T.Hm; f2.lda = T.ldm; f2.W = Lw.w_fc2; f2.ldw = Lw.k_fc2; f2.M = (int)M; f2.N = T.d;
  f2.K = pooled ? Lw.k_fc2 : Lw.kl_fc2;
  f2.out = h; f2.ldo = T.d; f2.bias = Lw.b_fc2; f2.m_dev = mdev;
  p.has_ln1 = l + 1 < T.L;
  if (p.has_ln1) {
    LayerW& Ln = T.layers[l + 1];
    p.ln1 = ln_into_x(c, T, M, Ln.ln1_g, Ln.ln1_b);
    p.ln1.m_dev = mdev;
  }
  return p;
}

// layer l after its attention, one tower. The last layer is pruned to the pooled rows
// (prune_last_layer): they are gathered into T.hc / T.Oc first and *pooled_rows is set.
int post_attn_step(clm_ctx* c, const LayerRun& R, int l, bool* pooled_rows, hipStream_t st) {
  Tower& T = *R.T;
  LayerW& Lw = T.layers[l];
  const bool bf = R.bf;
  const bool pooled = prune_last_layer() && l + 1 == T.L;
  int64_t M = (int64_t)R.B * R.S;
  float* h = T.h;
  u16* O = T.O;
  if (pooled) {
    { PROF(CLM_PROF_OTHER, (double)R.B * T.d * 6.0);
      KCHK(gather_pooled(T.h, T.d, T.O, T.ldo, R.B, R.S, T.d, R.ids, c->desc.eos_token_id, T.hc, T.Oc, T.ldo, st,
                         R.vl ? T.vl_offs : nullptr)); }
    M = R.B;
    h = T.hc;
    O = T.Oc;
    *pooled_rows = true;
  }
  PostOps p = post_ops(c, R, l, M, h, O, pooled);
  const int* mdev = pooled ? nullptr : R.mdev;
  if (Lw.r_out) { PROF(CLM_PROF_GEMM, 2.0 * p.rows * RPAD * T.d);
    KCHK(lora_down_gemm(bf, O, T.ldo, (int)M, T.d, Lw.a_out, mdev, st)); }
  if (pooled) {
    int r = pooled_resid(c, R, p.out, st);
    if (r) return r;
  } else {
    PROF(CLM_PROF_GEMM, 2.0 * p.rows * p.out.N * p.out.K); KCHK(gemm(bf, EPI_RESID, p.out, st));
  }
  { PROF(CLM_PROF_LN, p.rows * T.d * 6.0); KCHK(layernorm(bf, p.ln2, st)); }
  if (Lw.r_fc1) { PROF(CLM_PROF_GEMM, 2.0 * p.rows * RPAD * T.d);
    KCHK(lora_down_gemm(bf, T.X, T.ldx, (int)M, T.d, Lw.a_fc1, mdev, st)); }
  { PROF(CLM_PROF_GEMM, 2.0 * p.rows * p.fc1.N * p.fc1.K);   // pooled rows: 128 x 64 tiles (4 waves) fill the chip
    KCHK(pooled ? gemm_cfg(bf, EPI_GELU, GEMM_CFG_SPLITK, p.fc1, st) : gemm(bf, EPI_GELU, p.fc1, st)); }
  if (Lw.r_fc2) { PROF(CLM_PROF_GEMM, 2.0 * p.rows * RPAD * T.mlp);
    KCHK(lora_down_gemm(bf, T.Hm, T.ldm, (int)M, T.mlp, Lw.a_fc2, mdev, st)); }
  if (pooled) {
    int r = pooled_resid(c, R, p.fc2, st);
    if (r) return r;
  } else {
    PROF(CLM_PROF_GEMM, 2.0 * p.rows * p.fc2.N * p.fc2.K); KCHK(gemm(bf, EPI_RESID, p.fc2, st));
  }
  if (p.has_ln1) {
    { PROF(CLM_PROF_LN, p.rows * T.d * 6.0); KCHK(layernorm(bf, p.ln1, st)); }
    const LayerW& Ln = T.layers[l + 1];
    if (Ln.r_qkv) { PROF(CLM_PROF_GEMM, 2.0 * p.rows * RPAD * T.d);
      KCHK(lora_down_gemm(bf, T.X, T.ldx, (int)M, T.d, Ln.a_qkv, mdev, st)); }
  }
  return CLM_OK;
}

// encoder layers on the residual stream T.h; the first layer's LN1 output must already be in T.X.
// Returns with the pooled rows in T.hc (pruned: *pooled_rows = true) or all rows in T.h.
// (LayerNorm folded into the next GEMM -- producer moments in the residual epilogue, consumer
// W diag(gamma) + epilogue correction -- was parity-green but 3 % slower end to end and was
// removed: profiles/r02_v2_ln_fold_ab.txt.)
int run_layers(clm_ctx* c, Tower& T, int B, int S, bool causal, const int32_t* ids, bool* pooled_rows,
               hipStream_t st, bool vl = false) {
  *pooled_rows = false;
  LayerRun R;
  int r = make_run(c, T, B, S, causal, ids, vl, st, &R);
  for (int l = 0; !r && l < T.L; ++l) {
    r = attn_step(c, R, l, st);
    if (!r) r = post_attn_step(c, R, l, pooled_rows, st);
  }
  return r;
}

// the tower with its workspace pointers moved to sub-batch b0 (items of `rows` sequence rows)
Tower ws_view(const Tower& T0, int b0, int rows, int patches, int proj_dim) {
  Tower T = T0;
  const int64_t r0 = (int64_t)b0 * rows;
  T.h += r0 * T.d; T.X += r0 * T.ldx; T.QKV += r0 * 3 * T.d; T.O += r0 * T.ldo; T.Hm += r0 * T.ldm;
  if (T.P) T.P += (int64_t)b0 * patches * T.kp;
  T.pooled += (int64_t)b0 * proj_dim;
  T.hc += (int64_t)b0 * T.d;
  T.Oc += (int64_t)b0 * T.ldo;
  if (T.vl_lens) {
    T.vl_lens += b0; T.vl_tiles += b0; T.vl_offs += 2 * b0; T.vl_counts += 2 * b0; T.vl_rowmap += r0;
  }
  return T;
}

// image tower up to the first layer: patchify -> patch GEMM (+pos) -> class rows -> pre-LN + LN1 -> T.X
int image_prologue(clm_ctx* c, Tower& T, const void* pix, int layout, int B, hipStream_t st) {
  const clm_model_desc& d = c->desc;
  const bool bf = c->bf16(T.vision);
  const int G = d.image_size / d.patch, Tn = G * G + 1;
  { PROF(CLM_PROF_OTHER, (double)B * G * G * T.kp * 2.0 + (double)B * d.image_size * d.image_size * d.channels);
    KCHK(patchify(bf, pix, layout, B, d.image_size, d.patch, d.channels, T.lut, T.P, T.kp, st)); }
  GemmArgs g{};
  g.A = T.P; g.lda = T.kp; g.W = T.patch_w; g.ldw = T.kp; g.M = B * G * G; g.N = T.d; g.K = T.kp;
  g.out = T.h; g.ldo = T.d; g.aux = T.pos; g.aux_ld = T.d; g.group = G * G;
  { PROF(CLM_PROF_GEMM, 2.0 * g.M * g.N * g.K); KCHK(gemm(bf, EPI_PATCH, g, st)); }
  { PROF(CLM_PROF_OTHER, (double)B * T.d * 4.0); KCHK(write_cls(T.h, T.d, B, Tn, T.d, T.cls, T.pos, st)); }
  LnArgs a = ln_into_x(c, T, (int64_t)B * Tn, T.pre_g, T.pre_b);
  a.g2 = T.layers[0].ln1_g; a.b2 = T.layers[0].ln1_b;  // pre_layrnorm (in place) then layer-0 LN1
  { PROF(CLM_PROF_LN, (double)B * Tn * T.d * 10.0); KCHK(layernorm(bf, a, st)); }
  if (T.layers[0].r_qkv) { PROF(CLM_PROF_GEMM, 2.0 * B * Tn * RPAD * T.d);
    KCHK(lora_down_gemm(bf, T.X, T.ldx, B * Tn, T.d, T.layers[0].a_qkv, nullptr, st)); }
  return CLM_OK;
}

// pooled class rows -> post-LN -> projection (-> L2 norm) -> out
int image_epilogue(clm_ctx* c, Tower& T, int B, bool pooled_rows, void* out, int out_dtype, int normalize,
                   hipStream_t st) {
  const clm_model_desc& d = c->desc;
  const int G = d.image_size / d.patch, Tn = G * G + 1;
  PROF(CLM_PROF_OTHER, (double)B * (T.d * 4.0 + d.proj_dim * 4.0) + (double)T.d * d.proj_dim * 4.0);
  KCHK(pool_project(pooled_rows ? T.hc : T.h, T.d, B, pooled_rows ? 1 : Tn, T.d, nullptr, d.eos_token_id, T.fin_g,
                    T.fin_b, d.ln_eps, T.projT, d.proj_dim, T.pooled, out, out_dtype == CLM_F32 ? 0 : 1, normalize,
                    st));
  return CLM_OK;
}

int encode_image_chunk(clm_ctx* c, Tower& T, const void* pix, int layout, int B, void* out, int out_dtype,
                       int normalize, hipStream_t st) {
  const int G = c->desc.image_size / c->desc.patch;
  int r = image_prologue(c, T, pix, layout, B, st);
  bool pooled_rows = false;
  if (!r) r = run_layers(c, T, B, G * G + 1, false, nullptr, &pooled_rows, st);
  if (!r) r = image_epilogue(c, T, B, pooled_rows, out, out_dtype, normalize, st);
  return r;
}

// text tower up to the first layer: varlen plan (text_plan) -> token + position gather -> LN1 -> T.X.
// *vl: whether the live rows are packed (varlen path)
int text_prologue(clm_ctx* c, Tower& T, const int32_t* ids_dev, int B, int L, bool* vl_out, hipStream_t st) {
  const clm_model_desc& d = c->desc;
  const bool bf = c->bf16(T.vision);
  LnArgs a{};
  a.mode = 1; a.ids = ids_dev; a.tok = T.tok; a.pos = T.tpos; a.L = L;
  a.hf = T.h; a.ldh = T.d; a.g1 = T.layers[0].ln1_g; a.b1 = T.layers[0].ln1_b;
  a.y = T.X; a.ldy = T.ldx; a.M = B * L; a.d = T.d; a.eps = d.ln_eps;
  bool vl = text_varlen_enabled() && T.vl_lens && B <= 4096 &&   // text_plan: <= 4096 captions per chunk
            fused_attention(L, T.H, T.d, T.layers.empty() ? 0 : T.layers[0].k_qkv);
  if (vl) {
    { PROF(CLM_PROF_OTHER, (double)B * L * 8.0);
      KCHK(text_plan(ids_dev, B, L, d.eos_token_id, T.vl_lens, T.vl_offs, T.vl_rowmap, T.vl_tiles, T.vl_counts, st)); }
    a.m_dev = T.vl_counts;
    a.rowmap = T.vl_rowmap;
  }
  *vl_out = vl;
  { PROF(CLM_PROF_LN, (double)B * L * T.d * 14.0); KCHK(layernorm(bf, a, st)); }
  if (T.layers[0].r_qkv) { PROF(CLM_PROF_GEMM, 2.0 * B * L * RPAD * T.d);
    KCHK(lora_down_gemm(bf, T.X, T.ldx, B * L, T.d, T.layers[0].a_qkv, vl ? T.vl_counts : nullptr, st)); }
  return CLM_OK;
}

// pooled first-EOS rows -> final LN -> projection (-> L2 norm) -> out
int text_epilogue(clm_ctx* c, Tower& T, const int32_t* ids_dev, int B, int L, bool vl, bool pooled_rows, void* out,
                  int out_dtype, int normalize, hipStream_t st) {
  const clm_model_desc& d = c->desc;
  PROF(CLM_PROF_OTHER, (double)B * (T.d * 4.0 + d.proj_dim * 4.0 + L * 4.0) + (double)T.d * d.proj_dim * 4.0);
  KCHK(pool_project(pooled_rows ? T.hc : T.h, T.d, B, pooled_rows ? 1 : L, T.d, pooled_rows ? nullptr : ids_dev,
                    d.eos_token_id, T.fin_g, T.fin_b, d.ln_eps, T.projT, d.proj_dim, T.pooled, out,
                    out_dtype == CLM_F32 ? 0 : 1, normalize, st, vl && !pooled_rows ? T.vl_offs : nullptr));
  return CLM_OK;
}

int encode_text_chunk(clm_ctx* c, Tower& T, const int32_t* ids_dev, int B, int L, void* out, int out_dtype,
                      int normalize, hipStream_t st) {
  bool vl = false, pooled_rows = false;
  int r = text_prologue(c, T, ids_dev, B, L, &vl, st);
  if (!r) r = run_layers(c, T, B, L, true, ids_dev, &pooled_rows, st, vl);
  if (!r) r = text_epilogue(c, T, ids_dev, B, L, vl, pooled_rows, out, out_dtype, normalize, st);
  return r;
}

size_t dtype_size(int dt) {
  switch (dt) {
    case CLM_F32: case CLM_I32: return 4;
    case CLM_F16: case CLM_BF16: return 2;
    case CLM_U8: return 1;
    case CLM_I64: return 8;
  }
  return 0;
}

}  // namespace

extern "C" {

const char* clm_last_error(void) { return g_err.c_str(); }
const char* clm_version(void) { return "clm 0.1.0 gfx950"; }
int32_t clm_model_desc_size(void) { return (int32_t)sizeof(clm_model_desc); }

int clm_gemm(int hip_device, int dtype, int epilogue, int config, const void* A, int64_t lda, const void* W,
             int64_t ldw, int M, int N, int K, void* out, int64_t ldo, const float* bias, const float* rscale,
             const float* cscale, void* stream) {
  if (dtype != CLM_BF16 && dtype != CLM_F16) return fail(CLM_E_ARG, "dtype must be bf16 or f16");
  if (epilogue != EPI_STORE && epilogue != EPI_GELU && epilogue != EPI_RESID && epilogue != EPI_SCORE)
    return fail(CLM_E_ARG, "bad epilogue");
  if (config >= gemm_num_configs()) return fail(CLM_E_ARG, "bad config");
  // K % 64 == 32 (the unmerged-LoRA granule): rows must be readable to round_up(K, 64)
  const int64_t kr = (K + 63) / 64 * 64;
  if (M < 0 || N < 0 || K <= 0 || K % 32 || (K % 64 && (lda < kr || ldw < kr)))
    return fail(CLM_E_ARG, "bad shape (K % 64 == 0, or K % 64 == 32 with lda, ldw >= round_up(K, 64))");
  DeviceGuard g(hip_device);
  GemmArgs a{};
  a.A = (const u16*)A; a.lda = lda; a.W = (const u16*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.out = out; a.ldo = ldo; a.bias = bias; a.rscale = rscale; a.cscale = cscale;
  a.debug = g_gemm_debug;
  hipError_t e = gemm_cfg(dtype == CLM_BF16, epilogue, config, a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("gemm: ") + hipGetErrorString(e));
  return CLM_OK;
}

int clm_gemm_num_configs(void) { return gemm_num_configs(); }

// The sampled search's score matrix forms (search_bounded): fp16 A / W, score = acc * rscale[m] *
// cscale[n] stored as fp16 rounded toward -inf (mode 1, [M, ldo] u16) or as the maxima of each
// group of 4 consecutive columns, rounded the same way (mode 2: [M, ldo >= N / 4] u16, a row's
// groups in a fixed permutation; config 1 and N % 256 == 0, as the search runs it).
int clm_gemm_scores16(int hip_device, int config, const void* A, int64_t lda, const void* W, int64_t ldw, int M,
                      int N, int K, const float* rscale, const float* cscale, void* out, int64_t ldo, int mode,
                      void* stream) {
  if (mode != 1 && mode != 2) return fail(CLM_E_ARG, "mode must be 1 (fp16 scores) or 2 (group maxima)");
  if (config >= gemm_num_configs()) return fail(CLM_E_ARG, "bad config");
  if (M < 0 || N < 0 || K <= 0 || K % 64) return fail(CLM_E_ARG, "bad shape (K % 64 == 0)");
  if (mode == 2 && (config != 1 || N % 256 || ldo < N / 4 || ldo % 8))
    return fail(CLM_E_ARG, "group maxima: config 1, N % 256 == 0, ldo >= N / 4, ldo % 8 == 0");
  if (mode == 1 && ldo < N) return fail(CLM_E_ARG, "ldo < N");
  DeviceGuard g(hip_device);
  GemmArgs a{};
  a.A = (const u16*)A; a.lda = lda; a.W = (const u16*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.out = out; a.ldo = ldo; a.rscale = rscale; a.cscale = cscale; a.out16 = mode;
  hipError_t e = gemm_cfg(false, EPI_SCORE, config, a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("gemm: ") + hipGetErrorString(e));
  return CLM_OK;
}

void clm_debug_set(int flags) { g_gemm_debug = flags; }

int clm_attention_ex(int hip_device, int dtype, int flags, const void* qkv, void* out, int64_t ldo, int B, int T,
                     int H, void* stream) {
  if (dtype != CLM_BF16 && dtype != CLM_F16) return fail(CLM_E_ARG, "dtype must be bf16 or f16");
  if (B < 0 || T < 0 || H <= 0) return fail(CLM_E_ARG, "bad shape");
  DeviceGuard g(hip_device);
  if (flags & ~(CLM_ATTN_CAUSAL | CLM_ATTN_Q_LOG2E)) return fail(CLM_E_ARG, "unknown attention flags");
  const bool bf = dtype == CLM_BF16, cz = (flags & CLM_ATTN_CAUSAL) != 0, l2e = (flags & CLM_ATTN_Q_LOG2E) != 0;
  if (l2e && !attention_folds_log2e(bf, cz, T))
    return fail(CLM_E_ARG, "CLM_ATTN_Q_LOG2E: the kernel for this dtype / mask / T takes q without log2(e)");
  hipError_t e = attention(bf, cz, (const u16*)qkv, 3LL * H * 64, (u16*)out, ldo, B, T, H, H * 64,
                           (hipStream_t)stream, l2e);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("attention: ") + hipGetErrorString(e));
  return CLM_OK;
}

// the original entry point: `causal` is a 0 / non-0 switch (any non-zero value is the causal mask)
int clm_attention(int hip_device, int dtype, int causal, const void* qkv, void* out, int64_t ldo, int B, int T,
                  int H, void* stream) {
  return clm_attention_ex(hip_device, dtype, causal ? CLM_ATTN_CAUSAL : 0, qkv, out, ldo, B, T, H, stream);
}

int clm_layernorm(int hip_device, int dtype, const float* src, int64_t lds, int64_t M, int d, const float* gamma,
                  const float* beta, float eps, void* y, int64_t ldy, void* stream) {
  if (dtype != CLM_BF16 && dtype != CLM_F16) return fail(CLM_E_ARG, "dtype must be bf16 or f16");
  if (M < 0 || M > 0x7FFFFFFF || d <= 0 || d % 128 || d > 1024 || lds < d || ldy < d || (lds % 4) || (ldy % 4))
    return fail(CLM_E_ARG, "bad shape");
  if (M == 0) return CLM_OK;
  DeviceGuard g(hip_device);
  LnArgs a{};
  a.mode = 0; a.src = src; a.lds = lds; a.hf = nullptr; a.ldh = 0;
  a.g1 = gamma; a.b1 = beta; a.y = (u16*)y; a.ldy = ldy; a.M = (int)M; a.d = d; a.eps = eps;
  hipError_t e = layernorm(dtype == CLM_BF16, a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("layernorm: ") + hipGetErrorString(e));
  return CLM_OK;
}

int clm_prof_enable(clm_ctx* ctx, int enable) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  DeviceGuard g(ctx->dev);
  (void)hipDeviceSynchronize();
  ctx->prof = enable != 0;
  ctx->recs.clear();
  ctx->ev_used = 0;
  return CLM_OK;
}

int clm_prof_read(clm_ctx* ctx, int category, double* ms, double* work, int64_t* launches) {
  if (!ctx || category < 0 || category >= CLM_PROF_NCAT) return fail(CLM_E_ARG, "bad argument");
  DeviceGuard g(ctx->dev);
  double t = 0, w = 0;
  int64_t n = 0;
  for (auto& r : ctx->recs) {
    if (r.cat != category) continue;
    HIPCHK(hipEventSynchronize(ctx->ev_pool[r.e1]));
    float m = 0.f;
    HIPCHK(hipEventElapsedTime(&m, ctx->ev_pool[r.e0], ctx->ev_pool[r.e1]));
    t += m; w += r.work; ++n;
  }
  if (ms) *ms = t;
  if (work) *work = w;
  if (launches) *launches = n;
  return CLM_OK;
}

int clm_ctx_create(int hip_device, const clm_model_desc* desc, clm_ctx** out) {
  if (!desc || !out) return fail(CLM_E_ARG, "null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    (void)hipGetLastError();
    return fail(CLM_E_HIP, "no HIP device available");
  }
  if (hip_device < 0 || hip_device >= ndev) return fail(CLM_E_ARG, "bad device index");
  if (desc->compute_dtype != CLM_BF16 && desc->compute_dtype != CLM_F16 && desc->compute_dtype != CLM_COMPUTE_MIXED)
    return fail(CLM_E_ARG, "compute_dtype must be CLM_BF16, CLM_F16 or CLM_COMPUTE_MIXED");
  if (desc->max_batch <= 0 || desc->patch <= 0 || desc->image_size % desc->patch)
    return fail(CLM_E_ARG, "bad max_batch / patch / image_size");
  if (desc->max_pos > 77 * 4 || desc->proj_dim > 1024) return fail(CLM_E_ARG, "bad max_pos / proj_dim");
  if (desc->lora_r < 0 || desc->lora_r > 64) return fail(CLM_E_ARG, "lora_r must be in [0, 64]");
  clm_ctx* c = new clm_ctx();
  c->dev = hip_device;
  c->desc = *desc;
  *out = c;
  return CLM_OK;
}

int clm_ctx_destroy(clm_ctx* ctx) {
  if (!ctx) return CLM_OK;
  DeviceGuard g(ctx->dev);
  (void)hipDeviceSynchronize();
  ctx->free_all();
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : {ctx->ev_fork, ctx->ev_done})
    if (e) (void)hipEventDestroy(e);
  for (int i = 0; i < 2 * clm_ctx::MAX_SPLIT; ++i) {
    if (ctx->pev[i]) (void)hipEventDestroy(ctx->pev[i]);
    if (ctx->ps[i]) (void)hipStreamDestroy(ctx->ps[i]);
  }
  delete ctx;
  return CLM_OK;
}

int clm_load_tensor(clm_ctx* ctx, const char* name, const void* host_ptr, int dtype, const int64_t* shape,
                    int ndim) {
  if (!ctx || !name || (!host_ptr && ndim > 0) || ndim < 0 || ndim > 8) return fail(CLM_E_ARG, "bad argument");
  int64_t n = 1;
  HostTensor t;
  for (int i = 0; i < ndim; ++i) {
    if (shape[i] < 0) return fail(CLM_E_ARG, "negative dim");
    n *= shape[i];
    t.shape.push_back(shape[i]);
  }
  t.data.resize(n);
  if (dtype == CLM_F32) {
    std::memcpy(t.data.data(), host_ptr, n * sizeof(float));
  } else if (dtype == CLM_F16) {
    const uint16_t* p = (const uint16_t*)host_ptr;
    for (int64_t i = 0; i < n; ++i) t.data[i] = host_f16_to_f32(p[i]);
  } else if (dtype == CLM_BF16) {
    const uint16_t* p = (const uint16_t*)host_ptr;
    for (int64_t i = 0; i < n; ++i) t.data[i] = host_bf16_to_f32(p[i]);
  } else {
    return fail(CLM_E_ARG, "tensor dtype must be f32/f16/bf16");
  }
  ctx->host[name] = std::move(t);
  ctx->finalized = false;
  return CLM_OK;
}

int clm_finalize(clm_ctx* ctx) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  DeviceGuard g(ctx->dev);
  (void)hipDeviceSynchronize();
  ctx->free_all();
  ctx->finalized = false;
  int r = build_tower(ctx, ctx->vis, true);
  if (!r) r = build_tower(ctx, ctx->txt, false);
  if (!r) r = ctx->dalloc(&ctx->ids_dev, (size_t)ctx->desc.max_batch * ctx->desc.max_pos);
  if (r) {
    ctx->free_all();
    return r;
  }
  ctx->finalized = true;
  return CLM_OK;
}

int clm_set_lora(clm_ctx* ctx, int r, float alpha, uint32_t targets) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  if (r < 0 || r > 64) return fail(CLM_E_ARG, "lora_r must be in [0, 64]");
  if (targets & ~(uint32_t)(CLM_LORA_Q | CLM_LORA_K | CLM_LORA_V | CLM_LORA_OUT | CLM_LORA_FC1 | CLM_LORA_FC2))
    return fail(CLM_E_ARG, "unknown LoRA target bits");
  ctx->desc.lora_r = r;
  ctx->desc.lora_alpha = alpha;
  ctx->desc.lora_targets = r > 0 ? targets : 0u;
  ctx->finalized = false;   // the adapter tensors are loaded next, then clm_finalize
  return CLM_OK;
}

int clm_set_lora_enabled(clm_ctx* ctx, int enabled) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  ctx->lora_enabled = enabled != 0;
  return clm_finalize(ctx);
}

int clm_encode_image(clm_ctx* ctx, const void* pixels, int pix_layout, int n, void* out, int out_dtype,
                     int normalize, void* stream) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  if (!ctx->finalized) return fail(CLM_E_STATE, "clm_finalize has not been called");
  if (n < 0 || (n > 0 && (!pixels || !out))) return fail(CLM_E_ARG, "bad pixels/out/n");
  if (pix_layout != CLM_PIX_U8_HWC && pix_layout != CLM_PIX_F32_CHW) return fail(CLM_E_ARG, "bad pix_layout");
  if (out_dtype != CLM_F32 && out_dtype != CLM_F16) return fail(CLM_E_ARG, "out_dtype must be f32 or f16");
  if (n == 0) return CLM_OK;
  DeviceGuard g(ctx->dev);
  hipStream_t st = (hipStream_t)stream;
  const clm_model_desc& d = ctx->desc;
  const size_t pix_bytes = (size_t)d.image_size * d.image_size * d.channels * (pix_layout == CLM_PIX_U8_HWC ? 1 : 4);
  const size_t out_row = (size_t)d.proj_dim * dtype_size(out_dtype);
  const bool in_dev = is_device_ptr(pixels), out_dev = is_device_ptr(out);
  const int mb = d.max_batch;
  if (!in_dev) {
    int r = ensure_stage(&ctx->stage_in, &ctx->stage_in_bytes, pix_bytes * mb);
    if (r) return r;
  }
  if (!out_dev) {
    int r = ensure_stage(&ctx->stage_out, &ctx->stage_out_bytes, out_row * mb);
    if (r) return r;
  }
  for (int i0 = 0; i0 < n; i0 += mb) {
    const int B = std::min(mb, n - i0);
    const void* src = (const uint8_t*)pixels + (size_t)i0 * pix_bytes;
    if (!in_dev) {
      HIPCHK(hipMemcpyAsync(ctx->stage_in, src, pix_bytes * B, hipMemcpyHostToDevice, st));
      src = ctx->stage_in;
    }
    void* dst = out_dev ? (void*)((uint8_t*)out + (size_t)i0 * out_row) : ctx->stage_out;
    int r = encode_image_chunk(ctx, ctx->vis, src, pix_layout, B, dst, out_dtype, normalize, st);
    if (r) return r;
    if (!out_dev) {
      HIPCHK(hipMemcpyAsync((uint8_t*)out + (size_t)i0 * out_row, ctx->stage_out, out_row * B, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    } else if (!in_dev) {
      HIPCHK(hipStreamSynchronize(st));  // staging buffer reused next chunk
    }
  }
  return CLM_OK;
}

int clm_encode_text(clm_ctx* ctx, const int32_t* ids, int n, int L, void* out, int out_dtype, int normalize,
                    void* stream) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  if (!ctx->finalized) return fail(CLM_E_STATE, "clm_finalize has not been called");
  const clm_model_desc& d = ctx->desc;
  if (n < 0 || (n > 0 && (!ids || !out))) return fail(CLM_E_ARG, "bad ids/out/n");
  if (L <= 0 || L > d.max_pos)
    return fail(CLM_E_ARG, "sequence length " + std::to_string(L) + " outside [1, " + std::to_string(d.max_pos) + "]");
  if (out_dtype != CLM_F32 && out_dtype != CLM_F16) return fail(CLM_E_ARG, "out_dtype must be f32 or f16");
  if (n == 0) return CLM_OK;
  DeviceGuard g(ctx->dev);
  hipStream_t st = (hipStream_t)stream;
  const size_t out_row = (size_t)d.proj_dim * dtype_size(out_dtype);
  const bool in_dev = is_device_ptr(ids), out_dev = is_device_ptr(out);
  const int mb = d.max_batch;
  if (!out_dev) {
    int r = ensure_stage(&ctx->stage_out, &ctx->stage_out_bytes, out_row * mb);
    if (r) return r;
  }
  for (int i0 = 0; i0 < n; i0 += mb) {
    const int B = std::min(mb, n - i0);
    const int32_t* src = ids + (size_t)i0 * L;
    if (!in_dev) {
      for (int64_t q = 0; q < (int64_t)B * L; ++q)
        if (src[q] < 0 || src[q] >= d.vocab) return fail(CLM_E_ARG, "token id out of range");
      HIPCHK(hipMemcpyAsync(ctx->ids_dev, src, sizeof(int32_t) * B * L, hipMemcpyHostToDevice, st));
      src = ctx->ids_dev;
    }
    void* dst = out_dev ? (void*)((uint8_t*)out + (size_t)i0 * out_row) : ctx->stage_out;
    int r = encode_text_chunk(ctx, ctx->txt, src, B, L, dst, out_dtype, normalize, st);
    if (r) return r;
    if (!out_dev) {
      HIPCHK(hipMemcpyAsync((uint8_t*)out + (size_t)i0 * out_row, ctx->stage_out, out_row * B, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    } else if (!in_dev) {
      HIPCHK(hipStreamSynchronize(st));
    }
  }
  return CLM_OK;
}

// Sub-batch launches of one encode_pair on ps[0..2*split): images on ps[2j], captions on
// ps[2j+1]. `fork` has been recorded on ps[0]; every other stream waits on it, and ps[0]
// waits on every other stream's pev at the end (join).
static int pair_launch(clm_ctx* c, int split, hipEvent_t fork, const void* pixels, int layout, int n_img,
                       const int32_t* ids, int n_txt, int L, void* oi, void* ot, int out_dtype, int normalize) {
  const clm_model_desc& d = c->desc;
  const int Tn = d.image_size / d.patch * (d.image_size / d.patch) + 1;
  const size_t pix_bytes = (size_t)d.image_size * d.image_size * d.channels * (layout == CLM_PIX_U8_HWC ? 1 : 4);
  const size_t out_row = (size_t)d.proj_dim * dtype_size(out_dtype);
  for (int i = 1; i < 2 * split; ++i) HIPCHK(hipStreamWaitEvent(c->ps[i], fork, 0));
  struct Concurrent {   // tile heuristic hint for the duration of the launches (k_gemm.hip)
    explicit Concurrent(bool on) { gemm_set_concurrent(on); }
    ~Concurrent() { gemm_set_concurrent(false); }
  } conc(n_img > 0 && n_txt > 0);
  const int G = d.image_size / d.patch;
  for (int j = 0; j < split; ++j) {
    const int i0 = (int)((int64_t)n_img * j / split), i1 = (int)((int64_t)n_img * (j + 1) / split);
    const int t0 = (int)((int64_t)n_txt * j / split), t1 = (int)((int64_t)n_txt * (j + 1) / split);
    if (i1 > i0) {
      Tower T = ws_view(c->vis, i0, Tn, G * G, d.proj_dim);
      int r = encode_image_chunk(c, T, (const uint8_t*)pixels + i0 * pix_bytes, layout, i1 - i0,
                                 (uint8_t*)oi + i0 * out_row, out_dtype, normalize, c->ps[2 * j]);
      if (r) return r;
    }
    if (t1 > t0) {
      Tower T = ws_view(c->txt, t0, L, 0, d.proj_dim);
      int r = encode_text_chunk(c, T, ids + (int64_t)t0 * L, t1 - t0, L, (uint8_t*)ot + t0 * out_row, out_dtype,
                                normalize, c->ps[2 * j + 1]);
      if (r) return r;
    }
  }
  for (int i = 1; i < 2 * split; ++i) {
    HIPCHK(hipEventRecord(c->pev[i], c->ps[i]));
    HIPCHK(hipStreamWaitEvent(c->ps[0], c->pev[i], 0));
  }
  return CLM_OK;
}

int clm_pair_path(const clm_ctx* ctx) { return ctx ? ctx->last_pair_path : -1; }

int clm_encode_pair(clm_ctx* ctx, const void* pixels, int pix_layout, int n_img, const int32_t* ids, int n_txt,
                    int L, void* out_img, void* out_txt, int out_dtype, int normalize, int flags, void* stream) {
  if (!ctx) return fail(CLM_E_ARG, "null ctx");
  if (!ctx->finalized) return fail(CLM_E_STATE, "clm_finalize has not been called");
  const clm_model_desc& d = ctx->desc;
  if (n_img < 0 || n_txt < 0 || n_img > d.max_batch || n_txt > d.max_batch)
    return fail(CLM_E_ARG, "clm_encode_pair: 0 <= n <= max_batch per tower");
  if (pix_layout != CLM_PIX_U8_HWC && pix_layout != CLM_PIX_F32_CHW) return fail(CLM_E_ARG, "bad pix_layout");
  if (out_dtype != CLM_F32 && out_dtype != CLM_F16) return fail(CLM_E_ARG, "out_dtype must be f32 or f16");
  if (n_txt && (L <= 0 || L > d.max_pos)) return fail(CLM_E_ARG, "bad sequence length");
  if ((n_img && (!is_device_ptr(pixels) || !is_device_ptr(out_img))) ||
      (n_txt && (!is_device_ptr(ids) || !is_device_ptr(out_txt))))
    return fail(CLM_E_ARG, "clm_encode_pair needs device buffers");
  if (n_img == 0 && n_txt == 0) return CLM_OK;
  DeviceGuard g(ctx->dev);
  hipStream_t st = (hipStream_t)stream;
  if (!ctx->ps[0]) {
    for (int i = 0; i < 2 * clm_ctx::MAX_SPLIT; ++i) {
      HIPCHK(hipStreamCreateWithFlags(&ctx->ps[i], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&ctx->pev[i], hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming));
  }
  // sub-batches per tower: flags, else CLM_PAIR_SPLIT, else by batch size
  static const int env_split = getenv("CLM_PAIR_SPLIT") ? atoi(getenv("CLM_PAIR_SPLIT")) : 0;
  int split = (flags >> CLM_PAIR_SPLIT_SHIFT) & 15;
  // default 1: with persistent GEMM grids (one workgroup per CU slot) more concurrent
  // sub-batch streams only contend; measured 43.9k vs 41.3k (2) vs 38.2k (4) pairs/s at B=256
  if (!split) split = env_split > 0 ? env_split : 1;
  split = std::max(1, std::min({split, clm_ctx::MAX_SPLIT, std::max(n_img, n_txt)}));
  const bool use_graph = (flags & CLM_PAIR_GRAPH) && !ctx->prof;
  ctx->last_pair_path = 0;   // one stream per tower piece (the only path; round 5's grouped launches were removed)
  HIPCHK(hipEventRecord(ctx->ev_fork, st));
  HIPCHK(hipStreamWaitEvent(ctx->ps[0], ctx->ev_fork, 0));
  if (!use_graph) {
    int r = pair_launch(ctx, split, ctx->ev_fork, pixels, pix_layout, n_img, ids, n_txt, L, out_img, out_txt,
                        out_dtype, normalize);
    if (r) return r;
  } else {
    // the diagnostic flags change which kernels run (varlen / fused / pruned): part of the key
    clm_ctx::PairKey key(pixels, pix_layout, n_img, ids, n_txt, L, out_img, out_txt, out_dtype, normalize,
                         split | (g_gemm_debug << 8));
    auto it = ctx->graphs.find(key);
    if (it == ctx->graphs.end()) {
      if (ctx->graphs.size() >= 16) ctx->drop_graphs();
      // capture the pure kernel DAG on ps[0]; the fork edge from the origin stream is the
      // wait on ev_fork above (outside the capture); inside, ev_done is the fork point
      HIPCHK(hipStreamBeginCapture(ctx->ps[0], hipStreamCaptureModeRelaxed));
      hipError_t e1 = hipEventRecord(ctx->ev_done, ctx->ps[0]);
      int r = e1 == hipSuccess ? pair_launch(ctx, split, ctx->ev_done, pixels, pix_layout, n_img, ids, n_txt, L,
                                             out_img, out_txt, out_dtype, normalize)
                               : CLM_OK;
      hipGraph_t graph = nullptr;
      hipError_t e3 = hipStreamEndCapture(ctx->ps[0], &graph);
      if (r) { if (graph) (void)hipGraphDestroy(graph); return r; }
      if (e1 != hipSuccess || e3 != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return fail(CLM_E_HIP, std::string("graph capture: ") + hipGetErrorString(e3 != hipSuccess ? e3 : e1));
      }
      hipGraphExec_t exec = nullptr;
      hipError_t e4 = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (e4 != hipSuccess) return fail(CLM_E_HIP, std::string("graph instantiate: ") + hipGetErrorString(e4));
      it = ctx->graphs.emplace(key, exec).first;
    }
    HIPCHK(hipGraphLaunch(it->second, ctx->ps[0]));
  }
  HIPCHK(hipEventRecord(ctx->ev_done, ctx->ps[0]));
  HIPCHK(hipStreamWaitEvent(st, ctx->ev_done, 0));
  return CLM_OK;
}

// ------------------------------------------------------------------ index ---
// HBM-resident cosine index behind TextSearchIndex / top_k_similar (src/embedding/search.py:
// 24-115, similarity.py:36-58). Search = an fp16 MFMA pass that bounds the candidates, then an
// exact fp64 re-score of the candidates against the caller's own rows (see clm_index_search).
int clm_index_create(int hip_device, int64_t capacity, int dim, clm_index** out) {
  if (!out || capacity < 0 || dim <= 0 || dim % 64 || dim > 65536)
    return fail(CLM_E_ARG, "bad capacity/dim (dim must be a multiple of 64, <= 65536)");
  DeviceGuard g(hip_device);
  clm_index* x = new clm_index();
  x->dev = hip_device;
  x->cap = std::max<int64_t>(capacity, 1);
  x->dim = dim;
  if (hipMalloc(&x->rows, (size_t)x->cap * dim * sizeof(u16)) != hipSuccess ||
      hipMalloc(&x->inv, (size_t)x->cap * sizeof(float)) != hipSuccess) {
    (void)hipGetLastError();
    if (x->rows) (void)hipFree(x->rows);
    delete x;
    return fail(CLM_E_OOM, "index allocation failed");
  }
  *out = x;
  return CLM_OK;
}

int clm_index_destroy(clm_index* x) {
  if (!x) return CLM_OK;
  DeviceGuard g(x->dev);
  (void)hipDeviceSynchronize();
  for (void* p : {(void*)x->rows, (void*)x->inv, (void*)x->rows32, x->ws, x->ws2, x->ws3, x->ws4, (void*)x->samp,
                  (void*)x->samp_inv, (void*)x->inv_keys})
    if (p) (void)hipFree(p);
  delete x;
  return CLM_OK;
}

static int index_grow(clm_index* x, int64_t need_rows) {
  if (need_rows <= x->cap) return CLM_OK;
  int64_t nc = std::max<int64_t>(need_rows, x->cap * 2);
  u16* nr = nullptr;
  float* ni = nullptr;
  float* n32 = nullptr;
  if (hipMalloc(&nr, (size_t)nc * x->dim * sizeof(u16)) != hipSuccess ||
      hipMalloc(&ni, (size_t)nc * sizeof(float)) != hipSuccess ||
      (x->rows32 && hipMalloc(&n32, (size_t)nc * x->dim * sizeof(float)) != hipSuccess)) {
    (void)hipGetLastError();
    if (nr) (void)hipFree(nr);
    if (ni) (void)hipFree(ni);
    return fail(CLM_E_OOM, "index grow failed");
  }
  HIPCHK(hipMemcpy(nr, x->rows, (size_t)x->n * x->dim * sizeof(u16), hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(ni, x->inv, (size_t)x->n * sizeof(float), hipMemcpyDeviceToDevice));
  if (n32) {
    HIPCHK(hipMemcpy(n32, x->rows32, (size_t)x->n * x->dim * sizeof(float), hipMemcpyDeviceToDevice));
    (void)hipFree(x->rows32);
    x->rows32 = n32;
  }
  (void)hipFree(x->rows);
  (void)hipFree(x->inv);
  x->rows = nr;
  x->inv = ni;
  x->cap = nc;
  return CLM_OK;
}

// rescore_select / topk_merge order ties by a 32-bit image of the global row index
constexpr int64_t MAX_GLOBAL_ROWS = (int64_t)0xFFFFFFFF;

int clm_index_append(clm_index* x, const void* rows, int dtype, int64_t n, void* stream) {
  if (!x || n < 0 || (n > 0 && !rows)) return fail(CLM_E_ARG, "bad argument");
  if (dtype != CLM_F32 && dtype != CLM_F16) return fail(CLM_E_ARG, "rows must be f32 or f16");
  if (n == 0) return CLM_OK;
  if (x->offset + x->n + n > MAX_GLOBAL_ROWS)
    return fail(CLM_E_ARG, "index append: global row indices must stay below 2^32 (offset + rows)");
  DeviceGuard g(x->dev);
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipStreamSynchronize(st));
  int r = index_grow(x, x->n + n);
  if (r) return r;
  x->samp_n = -1;   // the threshold sample is rebuilt from the new row set
  x->inv_keys_n = -1;
  if (dtype == CLM_F32 && !x->rows32) {
    // first fp32 rows: keep an fp32 copy from now on; the rows so far were fp16 as given
    if (hipMalloc(&x->rows32, (size_t)x->cap * x->dim * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      x->rows32 = nullptr;
      return fail(CLM_E_OOM, "fp32 row copy allocation failed");
    }
    KCHK(f16_to_f32_rows(x->rows, x->n, (int)x->dim, x->rows32, st));
  }
  const size_t bytes = (size_t)n * x->dim * dtype_size(dtype);
  const void* src = rows;
  void* tmp = nullptr;
  if (!is_device_ptr(rows)) {
    if (hipMalloc(&tmp, bytes) != hipSuccess) { (void)hipGetLastError(); return fail(CLM_E_OOM, "staging failed"); }
    HIPCHK(hipMemcpyAsync(tmp, rows, bytes, hipMemcpyHostToDevice, st));
    src = tmp;
  }
  hipError_t e = hipSuccess;
  if (x->rows32) {
    float* dst = x->rows32 + (size_t)x->n * x->dim;
    e = dtype == CLM_F32 ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st)
                         : f16_to_f32_rows((const u16*)src, n, (int)x->dim, dst, st);
  }
  // fp16 MFMA operands: f32 rows are normalised first (no fp16 overflow / subnormal loss);
  // f16 rows are kept as given (exact) with the inverse norms of those rows
  if (e == hipSuccess)
    e = rows_to_f16(src, dtype == CLM_F32 ? 0 : 1, n, (int)x->dim, x->rows + (size_t)x->n * x->dim, x->inv + x->n,
                    st, dtype == CLM_F32 ? 2 : 0);
  if (tmp) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(tmp);
  }
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("index append: ") + hipGetErrorString(e));
  x->n += n;
  return CLM_OK;
}

// Shard persistence (TextSearchIndex.save_shard / load_shard): the index's internal state as it
// is, so a reload skips the fp32 normalisation and fp16 rounding of every row and searches bit for
// bit as the index that was saved.
int clm_index_has_f32(const clm_index* x) { return x ? (x->rows32 != nullptr) : -1; }

static hipMemcpyKind copy_kind(const void* dst, const void* src) {
  const bool d = is_device_ptr(dst), s = is_device_ptr(src);
  return d ? (s ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice) : (s ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
}

int clm_index_export(clm_index* x, int64_t start, int64_t n, uint16_t* rows16, float* inv, float* rows32,
                     void* stream) {
  if (!x || start < 0 || n < 0 || start + n > x->n || (n > 0 && (!rows16 || !inv)))
    return fail(CLM_E_ARG, "index export: bad range or null destination");
  if (rows32 && !x->rows32) return fail(CLM_E_STATE, "index export: the index keeps no fp32 rows");
  if (n == 0) return CLM_OK;
  DeviceGuard g(x->dev);
  hipStream_t st = (hipStream_t)stream;
  const size_t cnt = (size_t)n * x->dim;
  HIPCHK(hipMemcpyAsync(rows16, x->rows + (size_t)start * x->dim, cnt * 2, copy_kind(rows16, x->rows), st));
  HIPCHK(hipMemcpyAsync(inv, x->inv + start, (size_t)n * 4, copy_kind(inv, x->inv), st));
  if (rows32)
    HIPCHK(hipMemcpyAsync(rows32, x->rows32 + (size_t)start * x->dim, cnt * 4, copy_kind(rows32, x->rows32), st));
  HIPCHK(hipStreamSynchronize(st));
  return CLM_OK;
}

int clm_index_import(clm_index* x, const uint16_t* rows16, const float* inv, const float* rows32, int64_t n,
                     void* stream) {
  if (!x || n < 0 || (n > 0 && (!rows16 || !inv))) return fail(CLM_E_ARG, "index import: bad argument");
  if (n == 0) return CLM_OK;
  if (x->offset + x->n + n > MAX_GLOBAL_ROWS)
    return fail(CLM_E_ARG, "index import: global row indices must stay below 2^32 (offset + rows)");
  DeviceGuard g(x->dev);
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipStreamSynchronize(st));
  int r = index_grow(x, x->n + n);
  if (r) return r;
  x->samp_n = -1;
  x->inv_keys_n = -1;
  const size_t cnt = (size_t)n * x->dim;
  if (rows32 && !x->rows32) {   // as clm_index_append: the first fp32 rows start the fp32 copy
    if (hipMalloc(&x->rows32, (size_t)x->cap * x->dim * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      x->rows32 = nullptr;
      return fail(CLM_E_OOM, "fp32 row copy allocation failed");
    }
    KCHK(f16_to_f32_rows(x->rows, x->n, (int)x->dim, x->rows32, st));
  }
  u16* d16 = x->rows + (size_t)x->n * x->dim;
  HIPCHK(hipMemcpyAsync(d16, rows16, cnt * 2, copy_kind(d16, rows16), st));
  HIPCHK(hipMemcpyAsync(x->inv + x->n, inv, (size_t)n * 4, copy_kind(x->inv, inv), st));
  if (x->rows32) {
    float* d32 = x->rows32 + (size_t)x->n * x->dim;
    if (rows32) HIPCHK(hipMemcpyAsync(d32, rows32, cnt * 4, copy_kind(d32, rows32), st));
    else KCHK(f16_to_f32_rows(d16, n, (int)x->dim, d32, st));   // fp16 rows are the caller's rows
  }
  HIPCHK(hipStreamSynchronize(st));
  x->n += n;
  return CLM_OK;
}

int64_t clm_index_size(const clm_index* x) { return x ? x->n : -1; }

int clm_index_reset(clm_index* x) {
  if (!x) return fail(CLM_E_ARG, "null index");
  x->n = 0;
  x->samp_n = -1;   // never reuse a sample of the previous rows
  x->inv_keys_n = -1;
  return CLM_OK;
}

int clm_index_set_offset(clm_index* x, int64_t off) {
  if (!x || off < 0) return fail(CLM_E_ARG, "bad argument");
  if (off + x->n > MAX_GLOBAL_ROWS)
    return fail(CLM_E_ARG, "index offset: global row indices must stay below 2^32 (offset + rows)");
  x->offset = off;
  return CLM_OK;
}

int clm_index_read(clm_index* x, int64_t start, int64_t n, float* dst, void* stream) {
  if (!x || start < 0 || n < 0 || start + n > x->n || (n > 0 && !dst)) return fail(CLM_E_ARG, "bad range");
  if (n == 0) return CLM_OK;
  DeviceGuard g(x->dev);
  hipStream_t st = (hipStream_t)stream;
  const size_t cnt = (size_t)n * x->dim;
  std::vector<float> f(cnt);
  if (x->rows32) {
    HIPCHK(hipMemcpyAsync(f.data(), x->rows32 + (size_t)start * x->dim, cnt * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    std::vector<u16> h(cnt);
    HIPCHK(hipMemcpyAsync(h.data(), x->rows + (size_t)start * x->dim, cnt * 2, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (size_t i = 0; i < cnt; ++i) f[i] = host_f16_to_f32(h[i]);
  }
  if (is_device_ptr(dst)) {
    HIPCHK(hipMemcpy(dst, f.data(), cnt * 4, hipMemcpyHostToDevice));
  } else {
    std::memcpy(dst, f.data(), cnt * 4);
  }
  return CLM_OK;
}

static int grow(void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return CLM_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(CLM_E_OOM, "search workspace allocation failed");
  }
  *cap = bytes;
  return CLM_OK;
}

// Grow-only per-device scratch for the entry points that stage host buffers (resize_crop,
// cosine_scores, topk_merge, l2_normalize, fuse_queries): no hipMalloc / hipFree per call -- hipFree
// synchronises the whole device, which stalled work queued on other streams (the concurrent tower
// stream) behind a single-image encode. A caller holds the device's lock until its stream has
// drained the scratch (every such entry point synchronises its stream before returning).
struct Scratch {
  std::mutex mu;
  void* p = nullptr;
  size_t bytes = 0;
};
// A call that needed more than SCRATCH_KEEP bytes (a one-off host-staged score matrix, a resize
// of large photos) frees its scratch once its stream has drained it, so that peak does not stay
// allocated for the life of the process (the caller holds scr.mu)
constexpr size_t SCRATCH_KEEP = (size_t)256 << 20;
static void scratch_trim(Scratch& scr) {
  if (scr.bytes <= SCRATCH_KEEP) return;
  (void)hipFree(scr.p);
  (void)hipGetLastError();
  scr.p = nullptr;
  scr.bytes = 0;
}
static Scratch& scratch_of_current_device() {
  static Scratch s[64];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) { (void)hipGetLastError(); d = 0; }
  return s[d & 63];
}

// The MFMA pass scores fp16 unit-rounded operands: |fp16-pass score - exact cosine| <= 2.05e-3
// (each side's rounding moves a cosine by <= 2u, u = 2^-11, plus fp32 accumulation of <= 1024
// products). Every row of the exact top-k therefore has an fp16-pass score within 2 x 2.05e-3 of
// the fp16-pass k-th best; the candidates are taken that wide (plus slack) and re-scored exactly.
constexpr float RESCORE_MARGIN = 5e-3f;
// ... while the fp32 accumulation error stays inside the slack: dim * 2^-24 <= 4.9e-4 for dim <= 8192
// (every score within 1.95e-3 + 4.9e-4 of the exact cosine, twice that < RESCORE_MARGIN). Wider
// rows are always searched by the exact scan.
constexpr int MARGIN_MAX_DIM = 8192;
constexpr int CAND_CAP = 2048;

// Chunked scan: score chunks [nqb, ch] -- fp16 MFMA (EPI_SCORE GEMM) or exact fp64 cosines
// (exact_scores) -- radix top-k per chunk row, merge of the chunk lists. Any k <= 1024, any N.
static int search_scan(clm_index* x, bool exact, const u16* q16, const float* qinv, const float* q32,
                       const double* qn, int64_t nq, int k, float* osc, int64_t* oix, hipStream_t st) {
  const int dim = (int)x->dim;
  const int64_t N = x->n;
  const size_t budget = (size_t)512 << 20;
  const int64_t max_chunks = std::max<int64_t>(1, 8192 / k);
  int64_t ch = 1;
  if (N > 0) {
    ch = std::max<int64_t>((N + max_chunks - 1) / max_chunks, std::min<int64_t>(N, 1 << 17));
    ch = round_up(ch, 128);
  }
  const int64_t nchunks = N > 0 ? (N + ch - 1) / ch : 0;
  int64_t nqb = std::max<int64_t>(1, std::min<int64_t>(nq, (int64_t)(budget / ((size_t)ch * 4))));
  nqb = std::min<int64_t>(nqb, 4096);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t o_sc = take((size_t)nqb * ch * 4);
  const size_t o_cs = take((size_t)nqb * std::max<int64_t>(nchunks, 1) * k * 4);
  const size_t o_ci = take((size_t)nqb * std::max<int64_t>(nchunks, 1) * k * 8);
  int r = grow(&x->ws3, &x->ws3_bytes, off);
  if (r) return r;
  uint8_t* w = (uint8_t*)x->ws3;
  float* sc = (float*)(w + o_sc);
  float* cs = (float*)(w + o_cs);
  int64_t* ci = (int64_t*)(w + o_ci);
  for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
    const int64_t nb = std::min(nqb, nq - q0);
    if (N == 0) {
      KCHK(topk_rows(sc, 1, nb, 0, k, 0, osc + q0 * k, oix + q0 * k, k, st));
      continue;
    }
    for (int64_t c = 0; c < nchunks; ++c) {
      const int64_t r0 = c * ch, rn = std::min(ch, N - r0);
      if (exact) {
        const void* rp = x->rows32 ? (const void*)(x->rows32 + r0 * dim) : (const void*)(x->rows + r0 * dim);
        KCHK(exact_scores(q32 + q0 * dim, qn + q0, nb, rp, !x->rows32, rn, dim, sc, ch, st));
      } else {
        GemmArgs ga{};
        ga.A = q16 + q0 * dim; ga.lda = dim; ga.W = x->rows + r0 * dim; ga.ldw = dim;
        ga.M = (int)nb; ga.N = (int)rn; ga.K = dim; ga.out = sc; ga.ldo = ch;
        ga.rscale = qinv + q0; ga.cscale = x->inv + r0;
        KCHK(gemm(false, EPI_SCORE, ga, st));
      }
      if (nchunks == 1) {
        KCHK(topk_rows(sc, ch, nb, rn, k, x->offset + r0, osc + q0 * k, oix + q0 * k, k, st));
      } else {
        KCHK(topk_rows(sc, ch, nb, rn, k, x->offset + r0, cs + c * k, ci + c * k, nchunks * k, st));
      }
    }
    if (nchunks > 1) KCHK(topk_merge(cs, ci, nb, (int)nchunks, k, k, osc + q0 * k, oix + q0 * k, st));
  }
  return CLM_OK;
}

// Exact scan for k > 1024 (torch.topk of search.py:98 / similarity.py:57 takes any k <= N): every
// row of a query block scored exactly into one [nqb, N] matrix, then topk_any (exact k-th key,
// collection, LDS run sort + merge passes). The block is sized so the scores and topk_any's
// workspace stay within a 1 GiB budget (at least one query).
static int search_scan_large(clm_index* x, const float* q32, const double* qn, int64_t nq, int k, float* osc,
                             int64_t* oix, hipStream_t st) {
  const int dim = (int)x->dim;
  const int64_t N = x->n;
  const size_t budget = (size_t)1 << 30;
  const size_t per_q = (size_t)std::max<int64_t>(N, 1) * 4 + topk_any_ws_bytes(1, k);
  int64_t nqb = std::max<int64_t>(1, std::min<int64_t>(nq, (int64_t)(budget / per_q)));
  nqb = std::min<int64_t>(nqb, 65535);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t o_sc = take((size_t)nqb * std::max<int64_t>(N, 1) * 4);
  const size_t o_ws = take(topk_any_ws_bytes(nqb, k));
  int r = grow(&x->ws3, &x->ws3_bytes, off);
  if (r) return r;
  uint8_t* w = (uint8_t*)x->ws3;
  float* sc = (float*)(w + o_sc);
  for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
    const int64_t nb = std::min(nqb, nq - q0);
    if (N > 0) {
      const void* rp = x->rows32 ? (const void*)x->rows32 : (const void*)x->rows;
      KCHK(exact_scores(q32 + q0 * dim, qn + q0, nb, rp, !x->rows32, N, dim, sc, N, st));
    }
    KCHK(topk_any(sc, std::max<int64_t>(N, 1), nullptr, 0, nb, N, k, x->offset, osc + q0 * k, oix + q0 * k, k,
                  w + o_ws, st));
  }
  return CLM_OK;
}

// The filter GEMM's cscale bounds (GemmArgs::cbound) for the current rows, computed once per row set
// on the stream. Null (no skip test) when $CLM_FILTER_SKIP=0 (A/B) or the 8 bytes cannot be had.
static const unsigned* inv_keys_of(clm_index* x, hipStream_t st) {
  static const bool on = !getenv("CLM_FILTER_SKIP") || atoi(getenv("CLM_FILTER_SKIP")) != 0;
  if (!on) return nullptr;
  if (!x->inv_keys && hipMalloc(&x->inv_keys, 2 * sizeof(unsigned)) != hipSuccess) {
    (void)hipGetLastError();
    x->inv_keys = nullptr;
    return nullptr;
  }
  if (x->inv_keys_n != x->n) {
    if (value_bounds(x->inv, x->n, x->inv_keys, st) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    x->inv_keys_n = x->n;
  }
  return x->inv_keys;
}

// Overflowed queries, wide path: their fp16 rows, inverse norms, fp32 rows, norms and filter
// thresholds are gathered, the EPI_FILTER GEMM streams the index once more for just them with a
// capacity of cap[j] (the first pass's count plus headroom), and rescore_wide + topk_merge pick the
// exact top k from the whole list; results are scattered back to the queries' rows. Queries whose
// list still exceeds its capacity are appended to `full` (the exact scan redoes them).
static int overflow_wide(clm_index* x, const std::vector<int64_t>& qs, const std::vector<int64_t>& cap,
                         const u16* q16, const float* qinv, const float* q32, const double* qn, const float* th,
                         int k, float* osc, int64_t* oix, std::vector<int64_t>& full, hipStream_t st) {
  const int dim = (int)x->dim;
  const int64_t n = (int64_t)qs.size();
  const void* xrows = x->rows32 ? (const void*)x->rows32 : (const void*)x->rows;
  int64_t cap_max = 0;
  for (int64_t c : cap) cap_max = std::max(cap_max, c);
  cap_max = round_up(cap_max, RESCORE_WIDE_CHUNK);
  const int64_t nch = cap_max / RESCORE_WIDE_CHUNK;
  // queries per group: candidate lists (12 B per slot) within ~1 GB, at most 4096
  const int64_t G = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(n, 4096), (int64_t)(1 << 30) / (cap_max * 12)));
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t p_x = take((size_t)G * 8), p_q16 = take((size_t)G * dim * 2), p_qi = take((size_t)G * 4),
               p_q32 = take((size_t)G * dim * 4), p_qn = take((size_t)G * 8), p_th = take((size_t)G * 4),
               p_cnt = take((size_t)G * 4), p_cs = take((size_t)G * cap_max * 4), p_ci = take((size_t)G * cap_max * 8),
               p_ps = take((size_t)G * nch * k * 4), p_pi = take((size_t)G * nch * k * 8),
               p_s = take((size_t)G * k * 4), p_i = take((size_t)G * k * 8);
  if (int rg = grow(&x->ws4, &x->ws4_bytes, off)) return rg;
  uint8_t* w = (uint8_t*)x->ws4;
  int64_t* gx = (int64_t*)(w + p_x);
  int* cnt = (int*)(w + p_cnt);
  std::vector<int> hcnt;
  hipError_t e = hipSuccess;
  int r = CLM_OK;
  for (int64_t g0 = 0; g0 < n && e == hipSuccess && r == CLM_OK; g0 += G) {
    const int64_t ng = std::min(G, n - g0);
    e = hipMemcpyAsync(gx, qs.data() + g0, (size_t)ng * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = gather_rows(q16, (int64_t)dim * 2, gx, ng, (int64_t)dim * 2, w + p_q16, (int64_t)dim * 2, false, st);
    if (e == hipSuccess) e = gather_rows(qinv, 4, gx, ng, 4, w + p_qi, 4, false, st);
    if (e == hipSuccess) e = gather_rows(q32, (int64_t)dim * 4, gx, ng, (int64_t)dim * 4, w + p_q32, (int64_t)dim * 4, false, st);
    if (e == hipSuccess) e = gather_rows(qn, 8, gx, ng, 8, w + p_qn, 8, false, st);
    if (e == hipSuccess) e = gather_rows(th, 4, gx, ng, 4, w + p_th, 4, false, st);
    if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, (size_t)ng * 4, st);
    if (e != hipSuccess) break;
    GemmArgs gf{};
    gf.A = (const u16*)(w + p_q16); gf.lda = dim; gf.W = x->rows; gf.ldw = dim;
    gf.M = (int)ng; gf.N = (int)x->n; gf.K = dim;
    gf.rscale = (const float*)(w + p_qi); gf.cscale = x->inv;
    gf.theta = (const float*)(w + p_th); gf.theta_ld = 1;
    gf.cnt = cnt; gf.cand_s = (float*)(w + p_cs); gf.cand_i = (int64_t*)(w + p_ci); gf.cap = (int)cap_max;
    gf.base = x->offset; gf.m_fastest = 1;
    gf.cbound = inv_keys_of(x, st);
    // these queries' lists overflowed: appends dominate this pass, where gemm_kernel's 256 x 256
    // FILTER epilogue beats G2's (near-duplicate leg 73.7 k vs 66.0 k QPS,
    // profiles/r04_v7_neardup_ab.txt)
    static const int ocfg = getenv("CLM_GEMM_CFG") ? -1 : 1;
    if ((e = gemm_cfg(false, EPI_FILTER, ocfg, gf, st)) != hipSuccess) break;
    if ((e = rescore_wide((const int64_t*)(w + p_ci), cnt, cap_max, (const float*)(w + p_q32),
                          (const double*)(w + p_qn), dim, xrows, !x->rows32, x->offset, ng, k, (float*)(w + p_ps),
                          (int64_t*)(w + p_pi), st)) != hipSuccess) break;
    if ((e = topk_merge((const float*)(w + p_ps), (const int64_t*)(w + p_pi), ng, (int)nch, k, k, (float*)(w + p_s),
                        (int64_t*)(w + p_i), st)) != hipSuccess) break;
    hcnt.resize(ng);
    if ((e = hipMemcpyAsync(hcnt.data(), cnt, (size_t)ng * 4, hipMemcpyDeviceToHost, st)) != hipSuccess) break;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
    // scatter the complete lists' results; a list past its capacity goes to the exact scan
    std::vector<int64_t> done;
    std::vector<int64_t> rows_ok;
    for (int64_t j = 0; j < ng; ++j) {
      if (hcnt[j] > cap_max) full.push_back(qs[g0 + j]);
      else { done.push_back(qs[g0 + j]); rows_ok.push_back(j); }
    }
    if (done.size() == (size_t)ng) {
      e = gather_rows(w + p_s, (int64_t)k * 4, gx, ng, (int64_t)k * 4, osc, (int64_t)k * 4, true, st);
      if (e == hipSuccess) e = gather_rows(w + p_i, (int64_t)k * 8, gx, ng, (int64_t)k * 8, oix, (int64_t)k * 8, true, st);
    } else {
      for (size_t j = 0; j < done.size() && e == hipSuccess; ++j) {
        e = hipMemcpyAsync(osc + done[j] * k, (float*)(w + p_s) + rows_ok[j] * k, (size_t)k * 4,
                           hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess)
          e = hipMemcpyAsync(oix + done[j] * k, (int64_t*)(w + p_i) + rows_ok[j] * k, (size_t)k * 8,
                             hipMemcpyDeviceToDevice, st);
      }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);   // gx is rewritten by the next group
  }
  (void)hipStreamSynchronize(st);
  if (r) return r;
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("overflow (wide): ") + hipGetErrorString(e));
  return CLM_OK;
}

// Candidate lists that overflowed CAND_CAP (queries `overflow`, first-pass counts `ocount`): rebuilt
// whole by a second filter pass (overflow_wide) or redone by the exact scan (search_bounded,
// search_small). th: every query's filter threshold.
static int finish_overflow(clm_index* x, const std::vector<int64_t>& overflow, const std::vector<int64_t>& ocount,
                           const u16* q16, const float* qinv, const float* q32, const double* qn, const float* th,
                           int k, float* osc, int64_t* oix, hipStream_t st) {
  const int dim = (int)x->dim;
  int r;
  // Candidate lists beyond CAND_CAP (near-duplicate rows inside the window). Lists of up to
  // (SORT_MAX / k) chunks are rebuilt whole by a second filter pass over just those queries and
  // re-scored chunk-wise (overflow_wide); longer ones are redone by the exact scan, all of them in
  // ONE scan (the index is streamed once per query block of search_scan, not once per query).
  x->search_stats[2] += (int64_t)overflow.size();
  std::vector<int64_t> wide, wcount, full;
  for (size_t j = 0; j < overflow.size(); ++j) {
    // headroom over the first pass's count: a different tile shape may round a score differently
    const int64_t cap2 = ocount[j] + ocount[j] / 8 + 256;
    if ((cap2 + RESCORE_WIDE_CHUNK - 1) / RESCORE_WIDE_CHUNK * k <= 8192) {
      wide.push_back(overflow[j]);
      wcount.push_back(cap2);
    } else {
      full.push_back(overflow[j]);
    }
  }
  if (!wide.empty() && (r = overflow_wide(x, wide, wcount, q16, qinv, q32, qn, th, k, osc, oix, full, st))) return r;
  if (full.empty()) return CLM_OK;
  const int64_t no = (int64_t)full.size();
  size_t o2 = 0;
  auto take2 = [&](size_t bytes) { size_t o = o2; o2 = round_up(o2 + bytes, 256); return o; };
  const size_t p_x = take2((size_t)no * 8), p_q = take2((size_t)no * dim * 4), p_n = take2((size_t)no * 8),
               p_s = take2((size_t)no * k * 4), p_i = take2((size_t)no * k * 8);
  if ((r = grow(&x->ws4, &x->ws4_bytes, o2))) return r;   // overflow_wide is done with it (it drains its stream)
  uint8_t* wo = (uint8_t*)x->ws4;
  int64_t* gx = (int64_t*)(wo + p_x);
  float* gq = (float*)(wo + p_q);
  double* gn = (double*)(wo + p_n);
  float* gs = (float*)(wo + p_s);
  int64_t* gi = (int64_t*)(wo + p_i);
  hipError_t e = hipMemcpyAsync(gx, full.data(), (size_t)no * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = gather_rows(q32, (int64_t)dim * 4, gx, no, (int64_t)dim * 4, gq, (int64_t)dim * 4, false, st);
  if (e == hipSuccess) e = gather_rows(qn, 8, gx, no, 8, gn, 8, false, st);
  r = e == hipSuccess ? search_scan(x, true, nullptr, nullptr, gq, gn, no, k, gs, gi, st)
                      : fail(CLM_E_HIP, std::string("overflow gather: ") + hipGetErrorString(e));
  if (r == CLM_OK) e = gather_rows(gs, (int64_t)k * 4, gx, no, (int64_t)k * 4, osc, (int64_t)k * 4, true, st);
  if (r == CLM_OK && e == hipSuccess) e = gather_rows(gi, (int64_t)k * 8, gx, no, (int64_t)k * 8, oix, (int64_t)k * 8, true, st);
  (void)hipStreamSynchronize(st);
  if (r) return r;
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("overflow scatter: ") + hipGetErrorString(e));
  return CLM_OK;
}


// Bounded search (large N), per block of queries:
//  1. theta[q] <= the fp16-pass k-th best score of q:
//     sampled (k <= 256, N >= 4S): the k-th best over a strided sample of S rows -- a subset
//       of the index, so never above the true fp16-pass k-th best;
//     otherwise: the chunked fp16 scan's k-th best itself.
//  2. the EPI_FILTER GEMM streams the whole index once (M-fastest tile order: each index tile
//     is read once and shared by all query tiles) and appends every (score, row) with
//     score >= theta[q] - RESCORE_MARGIN to q's candidate list (capacity CAND_CAP): a
//     superset of the exact top-k.
//  3. rescore_select: candidates within the margin of their k-th are re-scored exactly against
//     the caller's rows, sorted (score desc, index asc), top k written.
//  Lists that overflowed CAND_CAP are redone by the full exact scan.
// $CLM_KTH_RADIX=1: the sampled thresholds through topk_rows (A/B, tests)
static const bool g_kth_radix = getenv("CLM_KTH_RADIX") && atoi(getenv("CLM_KTH_RADIX")) != 0;

static int search_bounded(clm_index* x, bool sampled, int64_t S, const u16* q16, const float* qinv,
                          const float* q32, const double* qn, int64_t nq, int k, float* osc, int64_t* oix,
                          hipStream_t st) {
  const int dim = (int)x->dim;
  const int64_t N = x->n;
  int r;
  if (sampled && (x->samp_n != N || x->samp_S != S)) {
    if (x->samp_cap < S) {
      if (x->samp) (void)hipFree(x->samp);
      if (x->samp_inv) (void)hipFree(x->samp_inv);
      x->samp = nullptr; x->samp_inv = nullptr; x->samp_cap = 0;
      if (hipMalloc(&x->samp, (size_t)S * dim * 2) != hipSuccess || hipMalloc(&x->samp_inv, (size_t)S * 4) != hipSuccess) {
        (void)hipGetLastError();
        return fail(CLM_E_OOM, "sample allocation failed");
      }
      x->samp_cap = S;
    }
    KCHK(sample_rows(x->rows, x->inv, N, dim, S, x->samp, x->samp_inv, st));
    x->samp_n = N;
    x->samp_S = S;
  }
  // query block: every block streams the whole index once through the filter GEMM, so fewer,
  // larger blocks read the index fewer times (10 M x 512 fp16 = 10 GB per pass). The sampled
  // path's block is bounded by its sample-score matrix (nqb x S fp32): at most $CLM_SEARCH_WS_MB
  // (default 8192) and at most a quarter of the free HBM.
  static const int64_t ws_mb = getenv("CLM_SEARCH_WS_MB") ? atoll(getenv("CLM_SEARCH_WS_MB")) : 8192;
  // query-block cap ($CLM_SEARCH_QB, A/B): a block's fp16 queries are re-read from L2 by every
  // index tile; with the filter GEMM on G2 tiles 2560 beats 4096 (10 k queries: 100.5 k vs 97.7 k
  // QPS, profiles/r04_v7_search_qb_ab.txt), and the blocks are balanced (a cap of 4096 gives
  // 10 k = 3392 + 3392 + 3216 instead of 4096 + 4096 + 1808)
  static const int64_t qb_cap = getenv("CLM_SEARCH_QB") ? std::max<int64_t>(64, atoll(getenv("CLM_SEARCH_QB"))) : 2560;
  // the sample-score rows' stride: S (a multiple of 256 floats, 1 KB) plus 256 B, so the score
  // GEMM's 16-row column stores do not land every row at the same power-of-two address offset
  // ($CLM_SAMPLE_PAD floats, A/B)
  static const int64_t spad = getenv("CLM_SAMPLE_PAD") ? atoll(getenv("CLM_SAMPLE_PAD")) : 64;
  const int64_t ldS = S + spad;
  int64_t nqb = std::min<int64_t>(nq, qb_cap);
  if (sampled) {
    size_t fr = 0, tot = 0;
    int64_t cap_b = ws_mb << 20;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) cap_b = std::min<int64_t>(cap_b, (int64_t)(fr / 4));
    else (void)hipGetLastError();
    nqb = std::min<int64_t>(std::min<int64_t>(nq, qb_cap), std::max<int64_t>(256, cap_b / (ldS * 4)));
  }
  {   // balance: the same number of blocks, equal sizes (multiples of 64 rows while that stays <= the cap)
    const int64_t nblk = (nq + nqb - 1) / nqb;
    const int64_t even = (nq + nblk - 1) / nblk;
    nqb = std::min<int64_t>(nqb, round_up(even, 64));
  }
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  // fp16 sample scores (rounded toward -inf: the k-th largest over them is <= the fp32 one, so
  // the thresholds only widen) where the one-pass k-th value path runs: half the bytes of the
  // phase's three passes ($CLM_SAMPLE_F32=1: fp32, A/B)
  static const bool s32_env = getenv("CLM_SAMPLE_F32") && atoi(getenv("CLM_SAMPLE_F32")) != 0;
  const bool s16 = sampled && k <= 8 && !g_kth_radix && !s32_env;
  // ... and stored as the maxima of groups of 4 sample rows (a subset of the scores: its k-th
  // largest is at most theirs, so θ stays a lower bound; 4x fewer bytes again). The dense-tile
  // estimate then counts groups, times 4 (an upper bound of the scores >= θ).
  // ($CLM_SAMPLE_GROUP=0: every score, A/B)
  static const bool grp_env = !(getenv("CLM_SAMPLE_GROUP") && atoi(getenv("CLM_SAMPLE_GROUP")) == 0);
  const bool sgrp = s16 && grp_env && S % 256 == 0;
  const int64_t Sc = sgrp ? S / 4 : S;             // stored values per sample-score row
  const int64_t ldC = sgrp ? S / 4 + 64 : ldS;     // their row stride
  const size_t o_sc = sampled ? take((size_t)nqb * ldC * (s16 ? 2 : 4)) : 0;
  const size_t o_ts = take((size_t)nqb * k * 4);
  const size_t o_ti = take((size_t)nqb * k * 8);
  const size_t o_th = take((size_t)nq * 4);   // every query's threshold (the overflow pass reuses them)
  const size_t o_cnt = take((size_t)nq * 4);   // every query's candidate count (read once, after the last block)
  const size_t o_est = take((size_t)nq * 4);
  const size_t o_cs = take((size_t)nqb * CAND_CAP * 4);
  const size_t o_ci = take((size_t)nqb * CAND_CAP * 8);
  if ((r = grow(&x->ws2, &x->ws2_bytes, off))) return r;
  uint8_t* w = (uint8_t*)x->ws2;
  float* sc = (float*)(w + o_sc);
  float* ts = (float*)(w + o_ts);
  int64_t* ti = (int64_t*)(w + o_ti);
  float* th = (float*)(w + o_th);
  int* cnt = (int*)(w + o_cnt);
  int* est = (int*)(w + o_est);
  std::vector<int> hest;
  float* cs = (float*)(w + o_cs);
  int64_t* ci = (int64_t*)(w + o_ci);
  const void* xrows = x->rows32 ? (const void*)x->rows32 : (const void*)x->rows;
  std::vector<int> hcnt;
  std::vector<int64_t> overflow, ocount;
  // Phase 1, every block: the per-query thresholds (and, sampled, the estimated candidate counts)
  // -- no host round trip between blocks
  for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
    const int64_t nb = std::min(nqb, nq - q0);
    if (sampled) {
      GemmArgs ga{};
      ga.A = q16 + q0 * dim; ga.lda = dim; ga.W = x->samp; ga.ldw = dim;
      ga.M = (int)nb; ga.N = (int)S; ga.K = dim; ga.out = sc; ga.ldo = ldC; ga.out16 = sgrp ? 2 : s16 ? 1 : 0;
      ga.rscale = qinv + q0; ga.cscale = x->samp_inv;
      if (sgrp) KCHK(gemm_cfg(false, EPI_SCORE, 1, ga, st));   // config 1 (256 x 256): the group layout's tile
      else KCHK(gemm(false, EPI_SCORE, ga, st));
      if (s16) {
        KCHK(kth_thresholds16((const u16*)sc, ldC, nb, Sc, k, RESCORE_MARGIN, th + q0, st));
        KCHK(count_ge16((const u16*)sc, ldC, nb, Sc, th + q0, est + q0, st));
      } else {
        if (k <= 8 && !g_kth_radix) {   // one streaming pass for the k-th value alone
          KCHK(kth_thresholds(sc, ldS, nb, S, k, RESCORE_MARGIN, th + q0, st));
        } else {
          KCHK(topk_rows(sc, ldS, nb, S, k, 0, ts, ti, k, st));
          KCHK(filter_thresholds(ts, k, nb, k, RESCORE_MARGIN, th + q0, st));
        }
        KCHK(count_ge(sc, ldS, nb, S, th + q0, est + q0, st));
      }
    } else {
      if ((r = search_scan(x, false, q16 + q0 * dim, qinv + q0, nullptr, nullptr, nb, k, ts, ti, st))) return r;
      KCHK(filter_thresholds(ts, k, nb, k, RESCORE_MARGIN, th + q0, st));
    }
  }
  // Filter tile per block, from the block's own data: when most of its queries' candidate windows
  // hold more than CAND_CAP rows (near-duplicate rows: the sampled count above the threshold,
  // scaled by N / S), the appends dominate the pass and gemm_kernel's 256 x 256 FILTER epilogue is
  // the faster one; otherwise G2's 256 x 192 (same candidates either way)
  if (sampled) {
    hest.resize(nq);
    HIPCHK(hipMemcpyAsync(hest.data(), est, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  HIPCHK(hipMemsetAsync(cnt, 0, (size_t)nq * 4, st));
  // Phase 2, every block: the filter pass and the exact re-score of its candidates
  for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
    const int64_t nb = std::min(nqb, nq - q0);
    bool dense = false;
    if (sampled) {
      int64_t over = 0;
      for (int64_t i = 0; i < nb; ++i) over += (double)hest[q0 + i] * (sgrp ? 4.0 : 1.0) * ((double)N / (double)S) > CAND_CAP;
      dense = 2 * over > nb;
    }
    GemmArgs gf{};
    gf.A = q16 + q0 * dim; gf.lda = dim; gf.W = x->rows; gf.ldw = dim;
    gf.M = (int)nb; gf.N = (int)N; gf.K = dim;
    gf.rscale = qinv + q0; gf.cscale = x->inv;
    gf.theta = th + q0; gf.theta_ld = 1;
    gf.cnt = cnt + q0; gf.cand_s = cs; gf.cand_i = ci; gf.cap = CAND_CAP; gf.base = x->offset;
    gf.m_fastest = 1;
    gf.cbound = inv_keys_of(x, st);
    // never clm_debug_set / $CLM_GEMM_DEBUG (those drop epilogues: the candidate lists would be
    // empty and the top-k wrong); the filter pass's own timing knob is $CLM_SEARCH_EPI_DEBUG,
    // read by tools only, whose results are discarded
    static const int search_dbg = getenv("CLM_SEARCH_EPI_DEBUG") ? (atoi(getenv("CLM_SEARCH_EPI_DEBUG")) & 3) : 0;
    gf.debug = search_dbg;
    static const bool cfg_forced = getenv("CLM_GEMM_CFG") != nullptr;
    KCHK(gemm_cfg(false, EPI_FILTER, dense && !cfg_forced ? 1 : -1, gf, st));
    x->search_stats[dense ? 5 : 4] += nb;
    KCHK(rescore_select(cs, ci, cnt + q0, CAND_CAP, q32 + q0 * dim, qn + q0, dim, xrows, !x->rows32, x->offset,
                        RESCORE_MARGIN, nb, k, osc + q0 * k, oix + q0 * k, st));
  }
  hcnt.resize(nq);
  HIPCHK(hipMemcpyAsync(hcnt.data(), cnt, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (int64_t i = 0; i < nq; ++i)
    if (hcnt[i] > CAND_CAP) {
      overflow.push_back(i);
      ocount.push_back(hcnt[i]);
    }
  x->search_stats[sampled ? 0 : 3] += nq - (int64_t)overflow.size();
  if (overflow.empty()) return CLM_OK;
  return finish_overflow(x, overflow, ocount, q16, qinv, q32, qn, th, k, osc, oix, st);
}

// Small query batches (nq <= 16) on a large index -- the reference's own pattern, one query per
// search_with_embedding call (search.py:93-99, seeker_service.py:183-186). The bounded search's
// MFMA filter pads such a batch to 256-row query tiles (>= 94 % padding) and its sampled-threshold
// phase adds a second GEMM; here the index is streamed ONCE (scan16: fp16-pass scores of every row
// into [N, ldq], ldq = nq rounded up to a power of two, + each 256-row chunk's maximum), then
//  1. th[q] = (k-th largest chunk maximum of q) - RESCORE_MARGIN: k chunks whose maxima are >= the
//     k-th largest hold k distinct rows, so it is <= the fp16-pass k-th best, a lower bound like
//     the sampled threshold (search_bounded step 1);
//  2. collect_ge appends every (score, row) >= th[q] (CAND_CAP per query; ~k + the rows within the
//     margin), 4 bytes per stored score read once;
//  3. rescore_select: exact fp64 re-score and (score desc, index asc) top k -- the same routine and
//     bits as every other path. Lists past CAND_CAP go through finish_overflow.
// Needs nchunk >= k (N >= 256 k) and the score matrix's offsets within one buffer descriptor.
// from this many rows on, a small batch takes search_small by default (below it the full exact
// scan is as fast: ~1.9 ms per query per 1 M rows at 512 dims against ~0.1 ms + launches)
constexpr int64_t SMALL_MIN_ROWS = 65536;
static bool search_small_fits(const clm_index* x, int64_t nq, int k) {
  const int64_t N = x->n, dim = x->dim;
  const int64_t nchunk = (N + 255) / 256;
  return nq >= 1 && nq <= 16 && k >= 1 && k <= 1024 && dim >= 64 && dim <= 1024 && dim % 64 == 0 && nchunk >= k &&
         (nq - 1) * nchunk * 4 + 4 <= 0x7FFFFFF0LL;
}

static int search_small(clm_index* x, const u16* q16, const float* qinv, const float* q32, const double* qn,
                        int64_t nq, int k, float* osc, int64_t* oix, hipStream_t st) {
  const int dim = (int)x->dim;
  const int64_t N = x->n;
  const int64_t nchunk = (N + 255) / 256;
  int64_t ldq = 1;   // scores per index row, a power of two >= nq
  while (ldq < nq) ldq *= 2;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t o_sc = take((size_t)N * ldq * 4);
  const size_t o_cm = take((size_t)nq * nchunk * 4);
  const size_t o_th = take((size_t)nq * 4);
  const size_t o_cnt = take((size_t)nq * 4);
  const size_t o_ts = take((size_t)nq * k * 4);
  const size_t o_ti = take((size_t)nq * k * 8);
  const size_t o_cs = take((size_t)nq * CAND_CAP * 4);
  const size_t o_ci = take((size_t)nq * CAND_CAP * 8);
  const int64_t W = scan16_waves(nchunk, dim);   // k <= 8: every wave's 8 largest chunk maxima
  const int64_t ldw = W * 8;
  const size_t o_wt = take((size_t)nq * ldw * 4);
  int r = grow(&x->ws2, &x->ws2_bytes, off);
  if (r) return r;
  uint8_t* w = (uint8_t*)x->ws2;
  float* sc = (float*)(w + o_sc);
  float* cm = (float*)(w + o_cm);
  float* th = (float*)(w + o_th);
  int* cnt = (int*)(w + o_cnt);
  Scan16Args a{};
  a.rows = x->rows; a.inv = x->inv; a.N = N; a.dim = dim;
  a.q16 = q16; a.qinv = qinv; a.nq = (int)nq;
  a.out = sc; a.ldo = ldq; a.cmax = cm; a.nchunk = nchunk;
  const bool wave_top = k <= 8 && !g_kth_radix && W * 8 >= k;
  a.wtop = wave_top ? (float*)(w + o_wt) : nullptr; a.ldw = ldw;
  KCHK(scan16(a, st));
  if (wave_top) {   // the k-th largest of the waves' top-8 lists = the k-th largest chunk maximum
    KCHK(kth_thresholds((const float*)(w + o_wt), ldw, nq, ldw, k, RESCORE_MARGIN, th, st));
  } else {
    KCHK(topk_rows(cm, nchunk, nq, nchunk, k, 0, (float*)(w + o_ts), (int64_t*)(w + o_ti), k, st));
    KCHK(filter_thresholds((const float*)(w + o_ts), k, nq, k, RESCORE_MARGIN, th, st));
  }
  HIPCHK(hipMemsetAsync(cnt, 0, (size_t)nq * 4, st));
  KCHK(collect_ge(sc, (int)ldq, (int)nq, N, th, cnt, CAND_CAP, (float*)(w + o_cs), (int64_t*)(w + o_ci), x->offset,
                  st));
  const void* xrows = x->rows32 ? (const void*)x->rows32 : (const void*)x->rows;
  KCHK(rescore_select((const float*)(w + o_cs), (const int64_t*)(w + o_ci), cnt, CAND_CAP, q32, qn, dim, xrows,
                      !x->rows32, x->offset, RESCORE_MARGIN, nq, k, osc, oix, st));
  std::vector<int> hcnt(nq);
  HIPCHK(hipMemcpyAsync(hcnt.data(), cnt, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::vector<int64_t> overflow, ocount;
  for (int64_t i = 0; i < nq; ++i)
    if (hcnt[i] > CAND_CAP) {
      overflow.push_back(i);
      ocount.push_back(hcnt[i]);
    }
  x->search_stats[6] += nq - (int64_t)overflow.size();
  if (overflow.empty()) return CLM_OK;
  return finish_overflow(x, overflow, ocount, q16, qinv, q32, qn, th, k, osc, oix, st);
}

// Top-k by EXACT cosine (the fp32-rounded fp64 cosine of the caller's query and rows), order
// (score desc, index asc). The reference ranks fp32 dot products of fp32-normalised rows
// (search.py:36,68,93,96-99), i.e. the same scores to within its own fp32 summation error.
//  * small problems (nq * N <= 2^24 dot products, or $CLM_SEARCH_FULL=1): the exact scan;
//  * otherwise (or $CLM_SEARCH_BOUNDED=1) search_bounded, sampled when the index is large
//    enough for sampling to pay ($CLM_SEARCH_EXACT=1 forces the chunked fp16 scan for step 1).
int clm_index_search(clm_index* x, const void* q, int q_dtype, int64_t nq, int k, float* out_scores,
                     int64_t* out_idx, void* stream) {
  if (!x || nq < 0 || (nq > 0 && (!q || !out_scores || !out_idx))) return fail(CLM_E_ARG, "bad argument");
  if (q_dtype != CLM_F32 && q_dtype != CLM_F16) return fail(CLM_E_ARG, "queries must be f32 or f16");
  if (k < 1) return fail(CLM_E_ARG, "k must be >= 1");
  if (k > (1 << 26)) return fail(CLM_E_ARG, "k must be <= 2^26");
  if (nq == 0) return CLM_OK;
  DeviceGuard g(x->dev);
  hipStream_t st = (hipStream_t)stream;
  const int dim = (int)x->dim;
  const int64_t N = x->n;
  const bool q_dev = is_device_ptr(q);
  const bool o_dev = is_device_ptr(out_scores) && is_device_ptr(out_idx);
  const size_t q_src_bytes = (size_t)nq * dim * (q_dtype == CLM_F32 ? 4 : 2);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t o_qsrc = q_dev ? 0 : take(q_src_bytes);
  const size_t o_q16 = take((size_t)nq * dim * 2);
  const size_t o_qinv = take((size_t)nq * 4);
  const size_t o_q32 = (q_dtype == CLM_F32 && q_dev) ? 0 : take((size_t)nq * dim * 4);
  const size_t o_qn = take((size_t)nq * 8);
  const size_t o_os = o_dev ? 0 : take((size_t)nq * k * 4);
  const size_t o_oi = o_dev ? 0 : take((size_t)nq * k * 8);
  int r = grow(&x->ws, &x->ws_bytes, off);
  if (r) return r;
  uint8_t* ws = (uint8_t*)x->ws;
  const void* qsrc = q;
  if (!q_dev) {
    HIPCHK(hipMemcpyAsync(ws + o_qsrc, q, q_src_bytes, hipMemcpyHostToDevice, st));
    qsrc = ws + o_qsrc;
  }
  u16* q16 = (u16*)(ws + o_q16);
  float* qinv = (float*)(ws + o_qinv);
  const float* q32 = (const float*)qsrc;
  if (!(q_dtype == CLM_F32 && q_dev)) {
    float* t = (float*)(ws + o_q32);
    if (q_dtype == CLM_F32) HIPCHK(hipMemcpyAsync(t, qsrc, (size_t)nq * dim * 4, hipMemcpyDeviceToDevice, st));
    else KCHK(f16_to_f32_rows((const u16*)qsrc, nq, dim, t, st));
    q32 = t;
  }
  double* qn = (double*)(ws + o_qn);
  KCHK(query_norms(q32, nq, dim, qn, st));
  // fp16 operands of the MFMA pass: queries normalised, then rounded
  KCHK(rows_to_f16(qsrc, q_dtype == CLM_F32 ? 0 : 1, nq, dim, q16, qinv, st, 2));
  float* osc = o_dev ? out_scores : (float*)(ws + o_os);
  int64_t* oix = o_dev ? out_idx : (int64_t*)(ws + o_oi);
  const char* e_full = getenv("CLM_SEARCH_FULL");
  const char* e_exact = getenv("CLM_SEARCH_EXACT");
  const char* e_bounded = getenv("CLM_SEARCH_BOUNDED");   // tests: bounded search at any size
  const bool force_bounded = e_bounded && atoi(e_bounded) && N > 0;
  // small batches on a large index: one streaming pass (search_small); $CLM_SEARCH_SMALLQ=1 takes
  // it at any size (tests), 0 never
  const char* e_small = getenv("CLM_SEARCH_SMALLQ");
  const int small_mode = e_small ? atoi(e_small) : -1;
  const bool small = small_mode != 0 && k <= 1024 && N > 0 && search_small_fits(x, nq, k) &&
                     (small_mode == 1 || (!force_bounded && !(e_full && atoi(e_full)) && !(e_exact && atoi(e_exact)) &&
                                          N >= SMALL_MIN_ROWS));
  if (small) {
    r = search_small(x, q16, qinv, q32, qn, nq, k, osc, oix, st);
  } else if (k > 1024) {
    // any k: the exact scan over whole rows (topk_rows / the candidate lists stop at 1024)
    r = search_scan_large(x, q32, qn, nq, k, osc, oix, st);
    x->search_stats[1] += nq;
  } else if ((e_full && atoi(e_full)) || N == 0 || dim > MARGIN_MAX_DIM ||
             (!force_bounded && (double)nq * (double)N <= (double)(1 << 24))) {
    r = search_scan(x, true, q16, qinv, q32, qn, nq, k, osc, oix, st);
    x->search_stats[1] += nq;
  } else {
    // sample of S rows: the k-th best of the sample ranks ~k * N / S = 256 in the index, so ~256
    // candidates per query ($CLM_SAMPLE_DIV replaces the 256: A/B only)
    static const int64_t sdiv = getenv("CLM_SAMPLE_DIV") ? std::max<int64_t>(16, atoll(getenv("CLM_SAMPLE_DIV"))) : 256;
    const int64_t S = round_up(std::max<int64_t>(8192, (int64_t)k * N / sdiv), 256);
    const bool sampled = !(e_exact && atoi(e_exact)) && k <= 256 && N >= 4 * S && S <= (1 << 18);
    r = search_bounded(x, sampled, S, q16, qinv, q32, qn, nq, k, osc, oix, st);
  }
  if (r) return r;
  if (!o_dev) {
    HIPCHK(hipMemcpyAsync(out_scores, osc, (size_t)nq * k * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(out_idx, oix, (size_t)nq * k * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    HIPCHK(hipStreamSynchronize(st));   // workspaces are reused by the next call
  }
  return CLM_OK;
}

int clm_index_stats(const clm_index* x, int64_t* filtered, int64_t* exact, int64_t* overflow) {
  if (!x) return fail(CLM_E_ARG, "null index");
  if (filtered) *filtered = x->search_stats[0];
  if (exact) *exact = x->search_stats[1] + x->search_stats[3];
  if (overflow) *overflow = x->search_stats[2];
  return CLM_OK;
}

int clm_index_stats2(const clm_index* x, int64_t* out, int n) {
  if (!x || !out || n < 0) return fail(CLM_E_ARG, "bad argument");
  const int64_t v[7] = {x->search_stats[0], x->search_stats[3], x->search_stats[1], x->search_stats[2],
                        x->search_stats[4], x->search_stats[5], x->search_stats[6]};
  for (int i = 0; i < n && i < 7; ++i) out[i] = v[i];
  return CLM_OK;
}

// similarity.cosine_similarity (similarity.py:10-33): every score exact (fp32-rounded fp64 cosine)
int clm_cosine_scores(int hip_device, const float* q, int64_t nq, const float* c, int64_t n, int dim, float* out,
                      void* stream) {
  if (nq < 0 || n < 0 || dim <= 0 || (nq * n > 0 && (!q || !c || !out)))
    return fail(CLM_E_ARG, "bad argument");
  if (nq == 0 || n == 0) return CLM_OK;
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  const bool qd = is_device_ptr(q), cd = is_device_ptr(c), od = is_device_ptr(out);
  size_t bytes = (size_t)nq * 8 + (qd ? 0 : (size_t)nq * dim * 4) + (cd ? 0 : (size_t)n * dim * 4) +
                 (od ? 0 : (size_t)nq * n * 4) + 1024;
  Scratch& scr = scratch_of_current_device();
  std::lock_guard<std::mutex> lock(scr.mu);
  if (int rg = grow(&scr.p, &scr.bytes, bytes)) return rg;
  uint8_t* w = (uint8_t*)scr.p;
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off = round_up(off + b, 256); return w + o; };
  double* qn = (double*)take((size_t)nq * 8);
  const float* qs = q;
  const float* cs = c;
  float* os = out;
  int rc = CLM_OK;
  hipError_t e = hipSuccess;
  if (!qd) { float* t = (float*)take((size_t)nq * dim * 4); e = hipMemcpyAsync(t, q, (size_t)nq * dim * 4, hipMemcpyHostToDevice, st); qs = t; }
  if (e == hipSuccess && !cd) { float* t = (float*)take((size_t)n * dim * 4); e = hipMemcpyAsync(t, c, (size_t)n * dim * 4, hipMemcpyHostToDevice, st); cs = t; }
  if (!od) os = (float*)take((size_t)nq * n * 4);
  if (e == hipSuccess) e = query_norms(qs, nq, dim, qn, st);
  if (e == hipSuccess) e = exact_scores(qs, qn, nq, cs, false, n, dim, os, n, st);
  if (e == hipSuccess && !od) e = hipMemcpyAsync(out, os, (size_t)nq * n * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  scratch_trim(scr);
  if (e != hipSuccess) rc = fail(CLM_E_HIP, std::string("cosine_scores: ") + hipGetErrorString(e));
  return rc;
}

int clm_topk_threshold(int hip_device, const float* scores, int64_t lds, int64_t nq, int64_t C, int k, float margin,
                       int method, float* th, void* stream) {
  if (nq < 0 || C < k || lds < C || k < 1 || k > (method == 0 ? 8 : 1024) || (method != 0 && method != 1))
    return fail(CLM_E_ARG, "bad threshold shape (k <= C <= lds; k <= 8 streaming, <= 1024 radix)");
  if (nq == 0) return CLM_OK;
  if (!is_device_ptr(scores) || !is_device_ptr(th)) return fail(CLM_E_ARG, "topk_threshold: device pointers");
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  if (method == 0) {
    KCHK(kth_thresholds(scores, lds, nq, C, k, margin, th, st));
    return CLM_OK;
  }
  Scratch& scr = scratch_of_current_device();
  std::lock_guard<std::mutex> lock(scr.mu);
  const size_t bs = round_up((size_t)nq * k * 4, 256);
  if (int rg = grow(&scr.p, &scr.bytes, bs + (size_t)nq * k * 8)) return rg;
  float* ts = (float*)scr.p;
  int64_t* ti = (int64_t*)((uint8_t*)scr.p + bs);
  KCHK(topk_rows(scores, lds, nq, C, k, 0, ts, ti, k, st));
  KCHK(filter_thresholds(ts, k, nq, k, margin, th, st));
  HIPCHK(hipStreamSynchronize(st));   // the scratch is reused by the next call
  scratch_trim(scr);
  return CLM_OK;
}

int clm_topk_merge(int hip_device, const float* scores, const int64_t* idx, int64_t nq, int parts, int k_in, int k,
                   float* out_scores, int64_t* out_idx, void* stream) {
  if (nq < 0 || parts <= 0 || k_in <= 0 || k <= 0 || (int64_t)parts * k_in > 0x7FFFFFFF)
    return fail(CLM_E_ARG, "bad merge shape");
  if (nq == 0) return CLM_OK;
  // one LDS sort per row (topk_merge) up to 8192 candidates and k <= 1024; beyond, topk_any
  const bool any = k > 1024 || (int64_t)parts * k_in > 8192;
  const int64_t any_rows = std::min<int64_t>(nq, 65535);
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  const bool in_d = is_device_ptr(scores) && is_device_ptr(idx);
  const bool out_d = is_device_ptr(out_scores) && is_device_ptr(out_idx);
  const size_t n_in = (size_t)nq * parts * k_in;
  uint8_t* w = nullptr;
  // every take() rounds its offset up to 256 B: size the workspace by the same rule (a flat
  // +512 slack under-allocated 4 small takes -- found by the host-sanitizer harness)
  const size_t bytes = (in_d ? 0 : round_up(n_in * 4, 256) + round_up(n_in * 8, 256)) +
                       (out_d ? 0 : round_up((size_t)nq * k * 4, 256) + round_up((size_t)nq * k * 8, 256)) +
                       (any ? round_up(topk_any_ws_bytes(any_rows, k), 256) : 0);
  Scratch& scr = scratch_of_current_device();
  std::unique_lock<std::mutex> lock(scr.mu, std::defer_lock);
  if (bytes > 0) {   // host lists: staged through the device scratch (the call drains its stream)
    lock.lock();
    if (int rg = grow(&scr.p, &scr.bytes, bytes)) return rg;
    w = (uint8_t*)scr.p;
  }
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off = round_up(off + b, 256); return w + o; };
  const float* s_in = scores;
  const int64_t* i_in = idx;
  float* s_out = out_scores;
  int64_t* i_out = out_idx;
  hipError_t e = hipSuccess;
  if (!in_d) {
    float* a = (float*)take(n_in * 4);
    int64_t* b = (int64_t*)take(n_in * 8);
    e = hipMemcpyAsync(a, scores, n_in * 4, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(b, idx, n_in * 8, hipMemcpyHostToDevice, st);
    s_in = a; i_in = b;
  }
  if (!out_d) { s_out = (float*)take((size_t)nq * k * 4); i_out = (int64_t*)take((size_t)nq * k * 8); }
  if (!any) {
    if (e == hipSuccess) e = topk_merge(s_in, i_in, nq, parts, k_in, k, s_out, i_out, st);
  } else {
    void* aws = take(topk_any_ws_bytes(any_rows, k));
    const int64_t n_row = (int64_t)parts * k_in;
    for (int64_t q0 = 0; e == hipSuccess && q0 < nq; q0 += any_rows)
      e = topk_any(s_in + q0 * n_row, n_row, i_in + q0 * n_row, n_row, std::min(any_rows, nq - q0), n_row, k, 0,
                   s_out + q0 * k, i_out + q0 * k, k, aws, st);
  }
  if (e == hipSuccess && !out_d) {
    e = hipMemcpyAsync(out_scores, s_out, (size_t)nq * k * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(out_idx, i_out, (size_t)nq * k * 8, hipMemcpyDeviceToHost, st);
  }
  if (e == hipSuccess && bytes > 0) e = hipStreamSynchronize(st);   // the scratch is free again
  if (bytes > 0) scratch_trim(scr);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("topk_merge: ") + hipGetErrorString(e));
  return CLM_OK;
}

int clm_l2_normalize(int hip_device, float* rows, int64_t n, int dim, void* stream) {
  if (n < 0 || dim <= 0 || (n > 0 && !rows)) return fail(CLM_E_ARG, "bad argument");
  if (n == 0) return CLM_OK;
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  if (is_device_ptr(rows)) {
    KCHK(l2_normalize_rows(rows, n, dim, st));
    return CLM_OK;
  }
  Scratch& scr = scratch_of_current_device();
  std::lock_guard<std::mutex> lock(scr.mu);
  if (int rg = grow(&scr.p, &scr.bytes, (size_t)n * dim * 4)) return rg;
  float* t = (float*)scr.p;
  hipError_t e = hipMemcpyAsync(t, rows, (size_t)n * dim * 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = l2_normalize_rows(t, n, dim, st);
  if (e == hipSuccess) e = hipMemcpyAsync(rows, t, (size_t)n * dim * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  scratch_trim(scr);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("l2_normalize: ") + hipGetErrorString(e));
  return CLM_OK;
}

int clm_fuse_queries(int hip_device, const float* a, float w_a, const float* b, float w_b, int64_t n,
                     int dim, float* out, void* stream) {
  if (n < 0 || dim <= 0 || (n > 0 && (!a || !out))) return fail(CLM_E_ARG, "bad argument");
  if (n == 0) return CLM_OK;
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  const bool dev = is_device_ptr(a);
  if (dev != is_device_ptr(out) || (b && dev != is_device_ptr(b)))
    return fail(CLM_E_ARG, "fuse_queries: a, b and out must all be device or all host pointers");
  if (dev) {
    KCHK(fuse_rows(a, w_a, b, w_b, n, dim, out, st));
    return CLM_OK;
  }
  const size_t bytes = (size_t)n * dim * 4;
  Scratch& scr = scratch_of_current_device();
  std::lock_guard<std::mutex> lock(scr.mu);
  if (int rg = grow(&scr.p, &scr.bytes, bytes * (b ? 2 : 1))) return rg;
  float* t = (float*)scr.p;
  float* tb = b ? t + (size_t)n * dim : nullptr;
  hipError_t e = hipMemcpyAsync(t, a, bytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && b) e = hipMemcpyAsync(tb, b, bytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = fuse_rows(t, w_a, tb, w_b, n, dim, t, st);
  if (e == hipSuccess) e = hipMemcpyAsync(out, t, bytes, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  scratch_trim(scr);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("fuse_queries: ") + hipGetErrorString(e));
  return CLM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- images ----
// Tap tables of PIL's 8-bit resampler (Pillow 12.2.0 src/libImaging/Resample.c precompute_coeffs +
// normalize_coeffs_8bpc, BICUBIC a = -0.5, support 2), the resize CLIPImageProcessor runs
// (models/clip_model.py:108-110); restated with the same double arithmetic and operation order as
// oracle/image_ref.py:coeffs. Contraction is off so no FMA can change a weight's last bit.
namespace {
#pragma clang fp contract(off)
double pil_bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// taps of output coordinates [first, first + count) of an in_size -> out_size resample:
// mins / ns [count] and fixed-point weights [count][ksize]; returns ksize
int pil_coeffs(int in_size, int out_size, int first, int count, std::vector<int32_t>& mins,
               std::vector<int32_t>& ns, std::vector<int32_t>& ks) {
  const double scale = (double)(float)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  mins.assign(count, 0);
  ns.assign(count, 0);
  ks.assign((size_t)count * ksize, 0);
  std::vector<double> w(ksize);
  for (int i = 0; i < count; ++i) {
    const int xx = first + i;
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      w[x] = pil_bicubic((x + xmin - center + 0.5) * ss);
      ww += w[x];
    }
    for (int x = 0; x < xmax; ++x) {
      const double k = ww != 0.0 ? w[x] / ww : w[x];
      ks[(size_t)i * ksize + x] = k < 0 ? (int32_t)(-0.5 + k * (1 << 22)) : (int32_t)(0.5 + k * (1 << 22));
    }
    mins[i] = xmin;
    ns[i] = xmax;
  }
  return ksize;
}
#pragma clang fp contract(on)

}  // namespace

extern "C" int clm_resize_crop(int hip_device, const uint8_t* src, const int64_t* offs, const int32_t* hw,
                               int n, int S, uint8_t* out, void* stream) {
  if (n < 0 || S <= 0 || S > 4096 || (n > 0 && (!src || !offs || !hw || !out)))
    return fail(CLM_E_ARG, "resize_crop: bad argument");
  if (n == 0) return CLM_OK;
  std::vector<ResizeDesc> desc(n);
  std::vector<int32_t> coef;
  int64_t src_bytes = 0, tmp_bytes = 0;
  int max_rows = 0;
  std::vector<int32_t> xmin, xn, xk, ymin, yn, yk;
  for (int i = 0; i < n; ++i) {
    const int H = hw[2 * i], W = hw[2 * i + 1];
    if (H < 1 || W < 1 || (int64_t)H * W > ((int64_t)1 << 28) || offs[i] < 0)
      return fail(CLM_E_ARG, "resize_crop: image " + std::to_string(i) + " has a bad size or offset");
    src_bytes = std::max(src_bytes, offs[i] + (int64_t)H * W * 3);
    // get_resize_output_image_size(default_to_square=False): short -> S, long -> int(S * long / short)
    const int shrt = std::min(H, W), lng = std::max(H, W);
    // int(S * long / short) in double as transformers does; an extreme aspect ratio (a 1 x 10^7
    // strip) would overflow int -- undefined behaviour, PIL fails on it too: refuse
    const double nl = (double)((int64_t)S * lng) / shrt;
    if (!(nl < (double)(1 << 24)))
      return fail(CLM_E_ARG, "resize_crop: image " + std::to_string(i) + " resizes to a side over 2^24 pixels");
    const int new_long = (int)nl;
    const int nh = W <= H ? new_long : S, nw = W <= H ? S : new_long;
    const int top = (nh - S) / 2, left = (nw - S) / 2;   // center_crop; nh, nw >= S
    ResizeDesc& d = desc[i];
    d.src_off = offs[i];
    d.W = W;
    d.kh = pil_coeffs(W, nw, left, S, xmin, xn, xk);
    d.kv = pil_coeffs(H, nh, top, S, ymin, yn, yk);
    int r1 = 0;
    for (int y = 0; y < S; ++y) r1 = std::max(r1, ymin[y] + yn[y]);
    d.r0 = ymin[0];
    d.rows = r1 - d.r0;
    for (int y = 0; y < S; ++y) ymin[y] -= d.r0;
    d.tmp_off = tmp_bytes;
    tmp_bytes += round_up((int64_t)d.rows * S * 3, 256);
    max_rows = std::max(max_rows, d.rows);
    d.coef_off = (int32_t)coef.size();
    if ((int64_t)coef.size() + 4 * S + (int64_t)S * (d.kh + d.kv) > INT32_MAX)
      return fail(CLM_E_ARG, "resize_crop: tap tables too large");
    coef.insert(coef.end(), xmin.begin(), xmin.end());
    coef.insert(coef.end(), xn.begin(), xn.end());
    coef.insert(coef.end(), ymin.begin(), ymin.end());
    coef.insert(coef.end(), yn.begin(), yn.end());
    coef.insert(coef.end(), xk.begin(), xk.end());
    coef.insert(coef.end(), yk.begin(), yk.end());
  }
  DeviceGuard g(hip_device);
  hipStream_t st = (hipStream_t)stream;
  const bool sd = is_device_ptr(src), od = is_device_ptr(out);
  const size_t out_bytes = (size_t)n * S * S * 3;
  const size_t b_desc = round_up(sizeof(ResizeDesc) * n, 256), b_coef = round_up(coef.size() * 4, 256);
  const size_t bytes = b_desc + b_coef + (size_t)tmp_bytes + (sd ? 0 : round_up(src_bytes, 256)) +
                       (od ? 0 : round_up(out_bytes, 256));
  Scratch& scr = scratch_of_current_device();
  std::lock_guard<std::mutex> lock(scr.mu);
  if (int rg = grow(&scr.p, &scr.bytes, bytes)) return rg;
  uint8_t* w = (uint8_t*)scr.p;
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off = round_up(off + b, 256); return w + o; };
  ResizeDesc* d_desc = (ResizeDesc*)take(sizeof(ResizeDesc) * n);
  int32_t* d_coef = (int32_t*)take(coef.size() * 4);
  uint8_t* d_tmp = take((size_t)tmp_bytes);
  const uint8_t* d_src = src;
  uint8_t* d_out = out;
  hipError_t e = hipMemcpyAsync(d_desc, desc.data(), sizeof(ResizeDesc) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_coef, coef.data(), coef.size() * 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && !sd) {
    uint8_t* t = take((size_t)src_bytes);
    e = hipMemcpyAsync(t, src, (size_t)src_bytes, hipMemcpyHostToDevice, st);
    d_src = t;
  }
  if (!od) d_out = take(out_bytes);
  if (e == hipSuccess) e = resize_crop(d_src, d_desc, n, S, max_rows, d_coef, d_tmp, d_out, st);
  if (e == hipSuccess && !od) e = hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, st);
  // the tables live in host vectors and the workspace is freed below: wait for the stream
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  scratch_trim(scr);
  if (e != hipSuccess) return fail(CLM_E_HIP, std::string("resize_crop: ") + hipGetErrorString(e));
  return CLM_OK;
}

extern "C" int clm_synth_images(int hip_device, uint64_t seed, int64_t row0, int n, int S, uint8_t* out,
                                void* stream) {
  if (n < 0 || S <= 0 || row0 < 0 || ((int64_t)S * S * 3) % 16 || (n > 0 && !out))
    return fail(CLM_E_ARG, "synth_images: bad argument (S * S * 3 must be a multiple of 16)");
  if (n == 0) return CLM_OK;
  if (!is_device_ptr(out) || ((uintptr_t)out & 15)) return fail(CLM_E_ARG, "synth_images: out must be 16-B aligned device memory");
  DeviceGuard g(hip_device);
  KCHK(synth_images(seed, row0, n, S, out, (hipStream_t)stream));
  return CLM_OK;
}
