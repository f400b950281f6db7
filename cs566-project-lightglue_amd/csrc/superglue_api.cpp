// C-ABI of the SuperGlue matcher (include/superglue_mi355x.h): schema, load-time repacking and
// folds, and the eval forward (reference gluefactory_nonfree/superglue.py:253-307) on the
// LightGlue kernels:
//   keypoint encoder + descriptors -> residual stream x (fp32 rows) and its plane image
//   per GNN layer (AttentionalPropagation, :131-139):
//     q, k, v = proj(x / source)        one fp16x3 GEMM over both images (EPI_QKV_ROT without a
//                                       cos table: head-major q fp32, k / v plane images)
//     message = softmax(q k^T / 8) v    the fp16x3 attention kernel; "cross" pairs image 0's
//                                       queries with image 1's keys / values and back
//     h = relu(BN(W1 [x; merge(m)]))    merge and the eval BatchNorm folded into W1 at load time
//     x = x + W2 h + b2                 residual GEMM (fp32 rows + plane image)
//   md = final_proj(x); cost = md0 md1^T / 16 (bf16x6, full fp32 range); Sinkhorn; mutual filter
// Reference channel order: MultiHeadedAttention views projections as [b, dim, head, n], i.e.
// channel d * 4 + h (:121-127); the q/k/v rows are gathered into head-major packed order here and
// merge's columns into the context's h * 64 + d order, so the math is unchanged.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/lightglue_mi355x.h"
#include "../../include/superglue_mi355x.h"
#include "common.h"
#include "kernels.h"
#include "train.h"

namespace lg {
int api_fail(int code, const char* msg);
}

namespace {

int fail(int code, const std::string& msg) { return lg::api_fail(code, msg.c_str()); }

#define SG_HIP(expr)                                                                                \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess) return fail(LG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

constexpr int D = 256, H = 4, HD = 64;
constexpr int kSlots = 512;
// per forward: at most 6 slots for the encoder / inputs, 4 per GNN layer, 1 for the head
static_assert(kSlots >= 8 + 4 * SG_MAX_LAYERS, "range table too small for SG_MAX_LAYERS");

struct Tensor {
  std::string name;
  int64_t numel;
};

// MLP (superglue.py:63-72) schema: conv weights / biases and BatchNorm tensors (no counters)
void add_mlp(std::vector<Tensor>& s, const std::string& p, const std::vector<int>& ch) {
  int idx = 0;
  for (size_t i = 1; i < ch.size(); ++i) {
    s.push_back({p + "." + std::to_string(idx) + ".weight", (int64_t)ch[i] * ch[i - 1]});
    s.push_back({p + "." + std::to_string(idx) + ".bias", ch[i]});
    ++idx;
    if (i < ch.size() - 1) {
      for (const char* f : {"weight", "bias", "running_mean", "running_var"})
        s.push_back({p + "." + std::to_string(idx) + "." + f, ch[i]});
      idx += 2;
    }
  }
}

std::vector<int> kenc_channels(const sg_config_t& c) {
  std::vector<int> ch = {c.use_scores ? 3 : 2};
  for (int i = 0; i < c.n_kenc; ++i) ch.push_back(c.keypoint_encoder[i]);
  ch.push_back(D);
  return ch;
}

std::vector<Tensor> make_schema(const sg_config_t& c) {
  std::vector<Tensor> s = {{"bin_score", 1}};  // the module's own parameter leads its state dict
  add_mlp(s, "kenc.encoder", kenc_channels(c));
  for (int i = 0; i < c.n_layers; ++i) {
    const std::string p = "gnn.layers." + std::to_string(i);
    s.push_back({p + ".attn.merge.weight", (int64_t)D * D});
    s.push_back({p + ".attn.merge.bias", D});
    for (int j = 0; j < 3; ++j) {
      s.push_back({p + ".attn.proj." + std::to_string(j) + ".weight", (int64_t)D * D});
      s.push_back({p + ".attn.proj." + std::to_string(j) + ".bias", D});
    }
    add_mlp(s, p + ".mlp", {2 * D, 2 * D, D});
  }
  s.push_back({"final_proj.weight", (int64_t)D * D});
  s.push_back({"final_proj.bias", D});
  return s;
}

size_t a256(size_t n) { return (n + 255) & ~size_t(255); }

struct Work {
  float *X, *Q, *ctx, *md, *cost, *Z, *fws, *sws;
  void *KP, *VP;
  _Float16 *Xp, *Cp, *Hp;
  unsigned* rtab;
  int rows_pad;
  size_t bytes;
};
Work carve(char* base, int B, int M, int N) {
  const size_t R = (size_t)B * (M + N);
  const size_t RP = (R + 255) / 256 * 256;
  size_t o = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + o : nullptr;
    o += a256(n);
    return p;
  };
  Work w{};
  w.rows_pad = (int)RP;
  w.X = (float*)take(R * D * 4);
  w.Q = (float*)take(R * D * 4);
  w.ctx = (float*)take(R * D * 4);
  w.md = (float*)take(R * D * 4);
  w.KP = take(2 * R * D * 2);
  w.VP = take(2 * R * D * 2);
  w.Xp = (_Float16*)take(2 * RP * D * 2);
  w.Cp = (_Float16*)take(2 * RP * D * 2);
  w.Hp = (_Float16*)take(2 * RP * 2 * D * 2);
  w.cost = (float*)take((size_t)B * M * N * 4);
  w.Z = (float*)take((size_t)B * (M + 1) * (N + 1) * 4);
  w.sws = (float*)take(lg::sinkhorn_workspace_floats(B, M, N) * 4);
  w.fws = (float*)take(lg::filter_workspace_floats(B, M, N) * 4);
  w.rtab = (unsigned*)take(kSlots * lg::kRangeStride * sizeof(unsigned));
  w.bytes = o;
  return w;
}

// packed q/k/v row t*256 + h*64 + j <- proj.t row dim(j)*4 + h (dim(j): rotary-pair order of the
// QKV epilogue, j < 32 -> 2j, else 2(j-32)+1); merge column h*64 + d <- d*4 + h
std::vector<int> qkv_perm() {
  std::vector<int> p(3 * D);
  auto dim = [](int j) { return j < 32 ? 2 * j : 2 * (j - 32) + 1; };
  for (int t = 0; t < 3; ++t)
    for (int h = 0; h < H; ++h)
      for (int j = 0; j < HD; ++j) p[t * D + h * HD + j] = t * D + dim(j) * H + h;
  return p;
}
std::vector<int> merge_perm() {
  std::vector<int> p(D);
  for (int h = 0; h < H; ++h)
    for (int d = 0; d < HD; ++d) p[h * HD + d] = d * H + h;
  return p;
}

}  // namespace

struct sg_handle {
  sg_config_t cfg;
  int device;
  lg::BnSync sync;                          // sg_set_collective (SyncBatchNorm across ranks)
  sg_grad_ready_fn grad_hook = nullptr;     // sg_set_grad_ready_hook
  void* grad_hook_ctx = nullptr;
  std::vector<Tensor> schema;
  std::map<std::string, int> index;
  std::vector<float*> raw;   // device copies of the loaded tensors (schema order)
  float* buf = nullptr;      // packed / folded fp32 weights
  int* perm = nullptr;       // qkv_perm [768] | merge_perm [256]
  _Float16* planes = nullptr;
  struct Mat {
    size_t off, boff;   // floats into buf
    int rows, K;
    size_t poff;        // halfs into planes
    float unscale;
    float g, bmax;      // row-L1 max, |bias| max
  };
  struct Layer {
    int type;
    Mat qkv, w1, w2;    // qkv: 768 x 256 (stats: keys / values rows below)
    float gK, bK, gV, bV;
    size_t bn1;         // raw BatchNorm of mlp.1 (folded into w1)
  };
  std::vector<Layer> layers;
  Mat fin;
  struct Enc {
    size_t wt, b;       // transposed weight [Cin][Cout], bias
    int bn;             // schema index of the BatchNorm weight (-1: last layer)
  };
  std::vector<Enc> enc;
  std::vector<int> ch;
  // the encoder's last layer as an fp16x3 GEMM with the descriptor add as its residual (its input
  // width a multiple of 32 and at least one hidden layer); otherwise the whole MLP in VALU
  bool enc_gemm = false;
  Mat enc_last{};
  float bin_score = 1.f;
  bool loaded = false;
};

// accessors for the training path (sg_train.cpp)
namespace lg {
const sg_config_t* sg_handle_config(const sg_handle* h) { return &h->cfg; }
int sg_handle_device(const sg_handle* h) { return h->device; }
const BnSync* sg_handle_sync(const sg_handle* h) { return h->sync.fn ? &h->sync : nullptr; }
void sg_handle_grad_ready(const sg_handle* h, int layer, void* stream) {
  if (h->grad_hook) h->grad_hook(h->grad_hook_ctx, layer, stream);
}
int sg_handle_weight_index(const sg_handle* h, const std::string& name) {
  auto it = h->index.find(name);
  return it == h->index.end() ? -1 : it->second;
}
}  // namespace lg

extern "C" {

int sg_create(const sg_config_t* cfg, int device, sg_handle_t** out) {
  if (!cfg || !out) return fail(LG_E_INVALID, "null argument");
  if (cfg->descriptor_dim != D) return fail(LG_E_INVALID, "descriptor_dim must be 256 (kernels are specialised)");
  if (cfg->n_layers < 0 || cfg->n_layers > SG_MAX_LAYERS) return fail(LG_E_INVALID, "n_layers out of range");
  if (cfg->n_kenc < 0 || cfg->n_kenc > SG_MAX_KENC) return fail(LG_E_INVALID, "keypoint_encoder too long");
  for (int i = 0; i < cfg->n_kenc; ++i)
    if (cfg->keypoint_encoder[i] <= 0 || cfg->keypoint_encoder[i] > 256 || cfg->keypoint_encoder[i] % 4)
      return fail(LG_E_INVALID, "keypoint_encoder widths must be multiples of 4 in [4, 256]");
  for (int i = 0; i < cfg->n_layers; ++i)
    if (cfg->layer_types[i] != 0 && cfg->layer_types[i] != 1) return fail(LG_E_INVALID, "GNN layer must be self or cross");
  if (cfg->sinkhorn_iterations < 0) return fail(LG_E_INVALID, "num_sinkhorn_iterations must be >= 0");
  SG_HIP(hipSetDevice(device));
  sg_handle* h = new sg_handle();
  h->cfg = *cfg;
  h->device = device;
  h->schema = make_schema(*cfg);
  for (size_t k = 0; k < h->schema.size(); ++k) h->index[h->schema[k].name] = (int)k;
  h->ch = kenc_channels(*cfg);
  h->enc_gemm = h->ch.size() >= 3 && h->ch[h->ch.size() - 2] % 32 == 0;
  *out = h;
  return LG_OK;
}

int sg_destroy(sg_handle_t* h) {
  if (!h) return LG_OK;
  (void)hipSetDevice(h->device);
  for (float* p : h->raw) (void)hipFree(p);
  if (h->buf) (void)hipFree(h->buf);
  if (h->perm) (void)hipFree(h->perm);
  if (h->planes) (void)hipFree(h->planes);
  delete h;
  return LG_OK;
}

int sg_weight_count(const sg_handle_t* h) { return h ? (int)h->schema.size() : 0; }
const char* sg_weight_name(const sg_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].name.c_str() : nullptr;
}
int64_t sg_weight_numel(const sg_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].numel : -1;
}

int sg_load_weights(sg_handle_t* h, int n, const char* const* names, const float* const* tensors, const int64_t* numels,
                    void* stream) {
  if (!h || n < 0 || (n && (!names || !tensors || !numels))) return fail(LG_E_INVALID, "null argument");
  SG_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  std::vector<int> seen(h->schema.size(), 0), src(h->schema.size(), -1);
  for (int i = 0; i < n; ++i) {
    auto it = h->index.find(names[i]);
    if (it == h->index.end()) return fail(LG_E_WEIGHTS, std::string("unexpected key in state_dict: ") + names[i]);
    const int k = it->second;
    if (seen[k]++) return fail(LG_E_WEIGHTS, std::string("duplicate key: ") + names[i]);
    if (numels[i] != h->schema[k].numel)
      return fail(LG_E_WEIGHTS, std::string("size mismatch for ") + names[i] + ": expected " +
                                    std::to_string(h->schema[k].numel) + " got " + std::to_string(numels[i]));
    src[k] = i;
  }
  for (size_t k = 0; k < h->schema.size(); ++k)
    if (!seen[k]) return fail(LG_E_WEIGHTS, "missing key in state_dict: " + h->schema[k].name);
  // raw device copies (BatchNorm statistics and the encoder are read from them directly)
  for (float* p : h->raw) (void)hipFree(p);
  h->raw.assign(h->schema.size(), nullptr);
  for (size_t k = 0; k < h->schema.size(); ++k) {
    SG_HIP(hipMalloc((void**)&h->raw[k], h->schema[k].numel * sizeof(float)));
    SG_HIP(hipMemcpyAsync(h->raw[k], tensors[src[k]], h->schema[k].numel * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  auto raw = [&](const std::string& name) { return h->raw[h->index.at(name)]; };

  // packed layout
  const int L = h->cfg.n_layers;
  size_t off = 0;
  auto take = [&](size_t nf) {
    const size_t o = off;
    off += (nf + 63) & ~size_t(63);
    return o;
  };
  h->enc.clear();
  for (size_t l = 0; l + 1 < h->ch.size(); ++l) {
    sg_handle::Enc e;
    e.wt = take((size_t)h->ch[l] * h->ch[l + 1]);
    e.b = take(h->ch[l + 1]);
    e.bn = l + 2 < h->ch.size() ? h->index.at("kenc.encoder." + std::to_string(3 * l + 1) + ".weight") : -1;
    h->enc.push_back(e);
  }
  h->layers.assign(L, {});
  for (int i = 0; i < L; ++i) {
    sg_handle::Layer& ly = h->layers[i];
    ly.type = h->cfg.layer_types[i];
    ly.qkv = {take(3 * D * D), take(3 * D), 3 * D, D, 0, 0.f, 0.f, 0.f};
    ly.w1 = {take(4 * D * D), take(2 * D), 2 * D, 2 * D, 0, 0.f, 0.f, 0.f};
    ly.w2 = {take(2 * D * D), take(D), D, 2 * D, 0, 0.f, 0.f, 0.f};
  }
  h->fin = {take(D * D), take(D), D, D, 0, 0.f, 0.f, 0.f};
  const int kl = h->ch[h->ch.size() - 2];
  if (h->enc_gemm) h->enc_last = {take((size_t)D * kl), take(D), D, kl, 0, 0.f, 0.f, 0.f};
  float* tmp = nullptr;
  if (h->buf) (void)hipFree(h->buf);
  h->buf = nullptr;
  SG_HIP(hipMalloc((void**)&h->buf, off * sizeof(float)));
  if (!h->perm) {
    SG_HIP(hipMalloc((void**)&h->perm, 4 * D * sizeof(int)));
    std::vector<int> p = qkv_perm(), pm = merge_perm();
    p.insert(p.end(), pm.begin(), pm.end());
    SG_HIP(hipMemcpy(h->perm, p.data(), p.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  SG_HIP(hipMallocAsync((void**)&tmp, (3 * D * D + 3 * D + 512 * 256 + 512 + D * D) * sizeof(float), st));
  float* B = h->buf;
  // keypoint encoder: transposed weights
  for (size_t l = 0; l < h->enc.size(); ++l) {
    const std::string p = "kenc.encoder." + std::to_string(3 * l);
    SG_HIP(lg::sg_transpose(raw(p + ".weight"), h->ch[l + 1], h->ch[l], B + h->enc[l].wt, st));
    SG_HIP(hipMemcpyAsync(B + h->enc[l].b, raw(p + ".bias"), h->ch[l + 1] * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  for (int i = 0; i < L; ++i) {
    sg_handle::Layer& ly = h->layers[i];
    const std::string p = "gnn.layers." + std::to_string(i);
    // q / k / v stacked [768][256] then gathered into the packed head-major order
    float* stk = tmp;
    float* stb = tmp + 3 * D * D;
    for (int j = 0; j < 3; ++j) {
      const std::string q = p + ".attn.proj." + std::to_string(j);
      SG_HIP(hipMemcpyAsync(stk + (size_t)j * D * D, raw(q + ".weight"), D * D * sizeof(float), hipMemcpyDeviceToDevice, st));
      SG_HIP(hipMemcpyAsync(stb + j * D, raw(q + ".bias"), D * sizeof(float), hipMemcpyDeviceToDevice, st));
    }
    SG_HIP(lg::gather_rows(B + ly.qkv.off, stk, h->perm, 3 * D, D, st));
    SG_HIP(lg::gather_rows(B + ly.qkv.boff, stb, h->perm, 3 * D, 1, st));
    // merge columns into context order, folded into mlp.0 (fold_out_proj: W1[:, 256:] Wm, b1 +=
    // W1[:, 256:] bm), then the eval BatchNorm of mlp.1
    float* wm = tmp + 3 * D * D + 3 * D + 512 * 256 + 512;
    SG_HIP(lg::sg_gather_cols(wm, raw(p + ".attn.merge.weight"), h->perm + 3 * D, D, D, st));
    SG_HIP(hipMemcpyAsync(B + ly.w1.off, raw(p + ".mlp.0.weight"), 4 * D * D * sizeof(float), hipMemcpyDeviceToDevice, st));
    SG_HIP(hipMemcpyAsync(B + ly.w1.boff, raw(p + ".mlp.0.bias"), 2 * D * sizeof(float), hipMemcpyDeviceToDevice, st));
    SG_HIP(lg::fold_out_proj(B + ly.w1.off, B + ly.w1.boff, wm, raw(p + ".attn.merge.bias"), tmp + 3 * D * D + 3 * D, st));
    SG_HIP(lg::sg_bn_fold(B + ly.w1.off, B + ly.w1.boff, raw(p + ".mlp.1.weight"), raw(p + ".mlp.1.bias"),
                          raw(p + ".mlp.1.running_mean"), raw(p + ".mlp.1.running_var"), 2 * D, 2 * D, st));
    SG_HIP(hipMemcpyAsync(B + ly.w2.off, raw(p + ".mlp.3.weight"), 2 * D * D * sizeof(float), hipMemcpyDeviceToDevice, st));
    SG_HIP(hipMemcpyAsync(B + ly.w2.boff, raw(p + ".mlp.3.bias"), D * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  if (h->enc_gemm) {
    const std::string p = "kenc.encoder." + std::to_string(3 * (h->ch.size() - 2));
    SG_HIP(hipMemcpyAsync(B + h->enc_last.off, raw(p + ".weight"), (size_t)D * kl * sizeof(float), hipMemcpyDeviceToDevice, st));
    SG_HIP(hipMemcpyAsync(B + h->enc_last.boff, raw(p + ".bias"), D * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  SG_HIP(hipMemcpyAsync(B + h->fin.off, raw("final_proj.weight"), D * D * sizeof(float), hipMemcpyDeviceToDevice, st));
  SG_HIP(hipMemcpyAsync(B + h->fin.boff, raw("final_proj.bias"), D * sizeof(float), hipMemcpyDeviceToDevice, st));
  SG_HIP(hipFreeAsync(tmp, st));

  // fp16x3 plane images (per-matrix power-of-two scale, max |W 2^sw| in [8, 16)) and range stats
  std::vector<sg_handle::Mat*> mats;
  for (auto& ly : h->layers) {
    mats.push_back(&ly.qkv);
    mats.push_back(&ly.w1);
    mats.push_back(&ly.w2);
  }
  mats.push_back(&h->fin);
  if (h->enc_gemm) mats.push_back(&h->enc_last);
  size_t total = 0;
  for (auto* m : mats) total += 2 * (size_t)m->rows * m->K;
  if (h->planes) (void)hipFree(h->planes);
  h->planes = nullptr;
  SG_HIP(hipMalloc((void**)&h->planes, total * sizeof(_Float16)));
  const size_t nst = mats.size() * 3 + 4 * (size_t)L + 1;
  float* dst = nullptr;
  SG_HIP(hipMallocAsync((void**)&dst, nst * sizeof(float), st));
  for (size_t i = 0; i < mats.size(); ++i) {
    SG_HIP(lg::absmax(B + mats[i]->off, (size_t)mats[i]->rows * mats[i]->K, dst + 3 * i, st));
    SG_HIP(lg::weight_range_stats(B + mats[i]->off, mats[i]->rows, mats[i]->K, B + mats[i]->boff, dst + 3 * i + 1, st));
  }
  float* ls = dst + 3 * mats.size();
  for (int i = 0; i < L; ++i) {
    const auto& q = h->layers[i].qkv;
    SG_HIP(lg::weight_range_stats(B + q.off + (size_t)D * D, D, D, B + q.boff + D, ls + 4 * i, st));
    SG_HIP(lg::weight_range_stats(B + q.off + (size_t)2 * D * D, D, D, B + q.boff + 2 * D, ls + 4 * i + 2, st));
  }
  SG_HIP(hipMemcpyAsync(ls + 4 * L, raw("bin_score"), sizeof(float), hipMemcpyDeviceToDevice, st));
  std::vector<float> hs(nst);
  SG_HIP(hipMemcpyAsync(hs.data(), dst, nst * sizeof(float), hipMemcpyDeviceToHost, st));
  SG_HIP(hipStreamSynchronize(st));
  SG_HIP(hipFreeAsync(dst, st));
  size_t poff = 0;
  for (size_t i = 0; i < mats.size(); ++i) {
    sg_handle::Mat& m = *mats[i];
    int sw = 0;
    const float mx = hs[3 * i];
    if (mx > 0.f && std::isfinite(mx)) {
      int E;
      (void)std::frexp(mx, &E);
      sw = std::min(std::max(4 - E, -100), 100);
    }
    SG_HIP(lg::split_weight_h3(B + m.off, m.rows, m.K, std::ldexp(1.f, sw), h->planes + poff, st));
    m.poff = poff;
    m.unscale = std::ldexp(1.f, -(11 + sw));
    m.g = hs[3 * i + 1];
    m.bmax = hs[3 * i + 2];
    poff += 2 * (size_t)m.rows * m.K;
  }
  for (int i = 0; i < L; ++i) {
    h->layers[i].gK = hs[3 * mats.size() + 4 * i];
    h->layers[i].bK = hs[3 * mats.size() + 4 * i + 1];
    h->layers[i].gV = hs[3 * mats.size() + 4 * i + 2];
    h->layers[i].bV = hs[3 * mats.size() + 4 * i + 3];
  }
  h->bin_score = hs[3 * mats.size() + 4 * L];
  SG_HIP(hipStreamSynchronize(st));
  h->loaded = true;
  return LG_OK;
}

int sg_workspace_bytes(const sg_handle_t* h, int32_t B, int32_t M, int32_t N, size_t* bytes) {
  if (!h || !bytes || B < 0 || M < 0 || N < 0) return fail(LG_E_INVALID, "bad argument");
  *bytes = carve(nullptr, B, M, N).bytes;
  return LG_OK;
}

int sg_forward(sg_handle_t* h, const sg_inputs_t* in, sg_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream) {
  using namespace lg;
  if (!h || !in || !out) return fail(LG_E_INVALID, "null argument");
  if (!h->loaded) return fail(LG_E_WEIGHTS, "weights not loaded");
  const int B = in->B, M = in->M, N = in->N;
  if (B <= 0 || M <= 0 || N <= 0) return fail(LG_E_INVALID, "B, M and N must be >= 1 (empty views: superglue.py:257)");
  if (!in->keypoints0 || !in->keypoints1 || !in->descriptors0 || !in->descriptors1)
    return fail(LG_E_INVALID, "missing input tensor");
  if (h->cfg.use_scores && (!in->scores0 || !in->scores1)) return fail(LG_E_INVALID, "use_scores needs keypoint_scores0/1");
  if ((!in->image_size0 && (in->image_w0 <= 0 || in->image_h0 <= 0)) || (!in->image_size1 && (in->image_w1 <= 0 || in->image_h1 <= 0)))
    return fail(LG_E_INVALID, "image_size or the image shape is required (superglue.py:78-83)");
  if (!out->matches0 || !out->matches1 || !out->matching_scores0 || !out->matching_scores1)
    return fail(LG_E_INVALID, "missing output tensor");
  const Work need = carve(nullptr, B, M, N);
  if (!workspace || workspace_bytes < need.bytes) return fail(LG_E_WORKSPACE, "workspace too small: need " + std::to_string(need.bytes));
  SG_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  Work w = carve((char*)workspace, B, M, N);
  const int R = B * (M + N), RP = w.rows_pad;
  const float* W = h->buf;
  unsigned* rt = w.rtab;
  int nslot = 0;
  auto slot = [&]() { return nslot < kSlots ? nslot++ : kSlots - 1; };
  auto ro = [&](int in0, float g0, int in1, float g1, float add, int o, int track = 0) {
    return RangeOut{rt, in0, in1, g0, g1, add, o, track, 0};
  };
  auto image = [&](_Float16* p, int K) { return PlaneRef{p, (long long)RP * K, RP}; };
  auto wplanes = [&](GemmH3Args& g, const sg_handle::Mat& m) {
    g.W = {h->planes + m.poff, (long long)m.rows * m.K, m.rows};
    g.acc_scale = m.unscale;
    g.bias = W + m.boff;
  };
  SG_HIP(hipMemsetAsync(rt, 0, kSlots * kRangeStride * sizeof(unsigned), st));

  // ---- keypoint encoder + descriptors -> x (superglue.py:266-276).  enc_gemm: the hidden layers
  // in VALU into fp32 rows, their plane image, then the last layer as an fp16x3 GEMM whose residual
  // is the descriptor rows (x = desc + W h + b, written as fp32 rows and as x's plane image)
  const int nl_all = (int)h->enc.size();
  const int nl_valu = h->enc_gemm ? nl_all - 1 : nl_all;
  const int kl = h->ch[nl_valu];
  if (h->enc_gemm) {
    SG_HIP(hipMemcpyAsync(w.X, in->descriptors0, sizeof(float) * B * M * D, hipMemcpyDeviceToDevice, st));
    SG_HIP(hipMemcpyAsync(w.X + (size_t)B * M * D, in->descriptors1, sizeof(float) * B * N * D, hipMemcpyDeviceToDevice, st));
  }
  for (int s = 0; s < 2; ++s) {
    SgEncArgs e;
    memset(&e, 0, sizeof(e));
    e.kpts = s ? in->keypoints1 : in->keypoints0;
    e.scores = h->cfg.use_scores ? (s ? in->scores1 : in->scores0) : nullptr;
    e.size = s ? in->image_size1 : in->image_size0;
    e.fw = (float)(s ? in->image_w1 : in->image_w0);
    e.fh = (float)(s ? in->image_h1 : in->image_h0);
    e.n = s ? N : M;
    e.rows = B * e.n;
    const size_t r0 = s ? (size_t)B * M : 0;
    if (h->enc_gemm) {
      e.desc = nullptr;
      e.out = w.ctx + r0 * kl;  // hidden rows [R][kl] (w.ctx is free until the first attention)
      e.ldo = kl;
    } else {
      e.desc = s ? in->descriptors1 : in->descriptors0;
      e.out = w.X + r0 * D;
      e.ldo = D;
    }
    e.nl = nl_valu;
    for (int l = 0; l <= e.nl; ++l) e.ch[l] = h->ch[l];
    for (int l = 0; l < e.nl; ++l) {
      e.layer[l].Wt = W + h->enc[l].wt;
      e.layer[l].b = W + h->enc[l].b;
      if (h->enc[l].bn >= 0) {
        e.layer[l].bn_w = h->raw[h->enc[l].bn];
        e.layer[l].bn_b = h->raw[h->enc[l].bn + 1];
        e.layer[l].bn_mean = h->raw[h->enc[l].bn + 2];
        e.layer[l].bn_var = h->raw[h->enc[l].bn + 3];
      }
    }
    SG_HIP(sg_keypoint_encoder(e, st));
  }
  int s_x = -1;
  if (h->enc_gemm) {
    const int s_d = slot(), s_hr = slot(), s_he = slot();
    s_x = slot();
    SG_HIP(range_absmax2(in->descriptors0, (size_t)B * M * D, in->descriptors1, (size_t)B * N * D, rt, s_d, st));
    SG_HIP(range_absmax(w.ctx, (size_t)R * kl, rt, s_hr, st));
    SG_HIP(rows_to_planes(w.ctx, R, kl, kl, w.Hp, RP, 0, ro(s_hr, 1.f, -1, 0.f, 0.f, s_he, 1), st));
    GemmH3Args g;
    memset(&g, 0, sizeof(g));
    g.out_scale = 1.f;
    g.A0 = image(w.Hp, kl); g.K0 = kl; g.K = kl; wplanes(g, h->enc_last);
    g.rtab = rt; g.a0_slot = s_he; g.a1_slot = -1;
    g.R = R; g.Nout = D; g.Y = w.X; g.ldy = D; g.res = w.X; g.ldr = D;
    g.Yp = w.Xp; g.yps = (long long)RP * D; g.yrows_pad = RP;
    g.ro = ro(s_d, 1.f, s_he, h->enc_last.g, h->enc_last.bmax, s_x, 1);
    SG_HIP(gemm_h3(g, EPI_STORE, st));
  } else {
    const int s_in = slot();
    s_x = slot();
    SG_HIP(range_absmax(w.X, (size_t)R * D, rt, s_in, st));
    SG_HIP(rows_to_planes(w.X, R, D, D, w.Xp, RP, 0, ro(s_in, 1.f, -1, 0.f, 0.f, s_x, 1), st));
  }

  // ---- AttentionalGNN (superglue.py:148-170)
  const size_t img1 = (size_t)B * H * M * HD;
  const long long ps = (long long)R * D;
  for (int i = 0; i < h->cfg.n_layers; ++i) {
    const sg_handle::Layer& ly = h->layers[i];
    const int s_k = slot(), s_v = slot();
    {
      HeadLayout hl;
      memset(&hl, 0, sizeof(hl));
      hl.B = B; hl.H = H; hl.M = M; hl.N = N; hl.cosb = nullptr; hl.sinb = nullptr;
      hl.q = w.Q; hl.kp = w.KP; hl.vp = w.VP; hl.pstride = ps; hl.qk_scale = 1.f;
      GemmH3Args g;
      memset(&g, 0, sizeof(g));
      g.out_scale = 1.f;
      g.A0 = image(w.Xp, D); g.K0 = D; g.K = D; wplanes(g, ly.qkv);
      g.rtab = rt; g.a0_slot = s_x; g.a1_slot = -1;
      g.ro = ro(s_x, ly.gK, -1, 0.f, ly.bK, s_k, 1);
      g.ro_v = ro(s_x, ly.gV, -1, 0.f, ly.bV, s_v, kRangeTrack | kRangeTwoSided);  // M[v] bounds the context (mlp.0's input)
      g.R = R; g.Nout = 3 * D; g.hl = hl;
      SG_HIP(gemm_h3(g, EPI_QKV_ROT, st));
    }
    {
      const void* kp1 = static_cast<const char*>(w.KP) + 2 * img1;
      const void* vp1 = static_cast<const char*>(w.VP) + 2 * img1;
      float* ctx1 = w.ctx + (size_t)B * M * D;
      AttnSet a0, a1;
      if (ly.type == 0) {  // self: layer(desc0, desc0), layer(desc1, desc1)
        a0 = {w.Q, w.KP, w.VP, ps, w.ctx, M, M, w.Cp, (long long)RP * D, RP, 0, rt, s_k, nullptr, nullptr, nullptr};
        a1 = {w.Q + img1, kp1, vp1, ps, ctx1, N, N, w.Cp, (long long)RP * D, RP, B * M, rt, s_k, nullptr, nullptr, nullptr};
      } else {  // cross: layer(desc0, desc1), layer(desc1, desc0)
        a0 = {w.Q, kp1, vp1, ps, w.ctx, M, N, w.Cp, (long long)RP * D, RP, 0, rt, s_k, nullptr, nullptr, nullptr};
        a1 = {w.Q + img1, w.KP, w.VP, ps, ctx1, N, M, w.Cp, (long long)RP * D, RP, B * M, rt, s_k, nullptr, nullptr, nullptr};
      }
      SG_HIP(attention_f32(a0, a1, B, H, 0.125f, PREC_H3, st));  // 1 / sqrt(dim = 64) (:108)
    }
    // mlp.0 with merge and BatchNorm folded, ReLU -> hidden plane image (context planes carry the
    // value planes' exponent, s_v)
    const int s_h = slot(), s_xn = slot();
    {
      GemmH3Args g;
      memset(&g, 0, sizeof(g));
      g.out_scale = 1.f;
      g.A0 = image(w.Xp, D); g.K0 = D; g.A1 = image(w.Cp, D); g.K = 2 * D; wplanes(g, ly.w1);
      g.rtab = rt; g.a0_slot = s_x; g.a1_slot = s_v;
      g.R = R; g.Nout = 2 * D; g.relu = 1;
      g.Yp = w.Hp; g.yps = (long long)RP * 2 * D; g.yrows_pad = RP;
      g.ro = ro(s_x, ly.w1.g, s_v, ly.w1.g, ly.w1.bmax, s_h, 1);
      SG_HIP(gemm_h3(g, EPI_STORE, st));
    }
    {  // mlp.3 + residual: x = x + delta (fp32 rows and plane image)
      GemmH3Args g;
      memset(&g, 0, sizeof(g));
      g.out_scale = 1.f;
      g.A0 = image(w.Hp, 2 * D); g.K0 = 2 * D; g.K = 2 * D; wplanes(g, ly.w2);
      g.rtab = rt; g.a0_slot = s_h; g.a1_slot = -1;
      g.R = R; g.Nout = D; g.Y = w.X; g.ldy = D; g.res = w.X; g.ldr = D;
      g.Yp = w.Xp; g.yps = (long long)RP * D; g.yrows_pad = RP;
      g.ro = ro(s_x, 1.f, s_h, ly.w2.g, ly.w2.bmax, s_xn, 1);
      SG_HIP(gemm_h3(g, EPI_STORE, st));
    }
    s_x = s_xn;
  }
  if (out->descriptors0)
    SG_HIP(hipMemcpyAsync(out->descriptors0, w.X, sizeof(float) * B * M * D, hipMemcpyDeviceToDevice, st));
  if (out->descriptors1)
    SG_HIP(hipMemcpyAsync(out->descriptors1, w.X + (size_t)B * M * D, sizeof(float) * B * N * D, hipMemcpyDeviceToDevice, st));

  // ---- final_proj, cost = md0 . md1 / sqrt(256) (superglue.py:278-282), Sinkhorn, filter
  {
    GemmH3Args g;
    memset(&g, 0, sizeof(g));
    g.out_scale = 1.f;
    g.A0 = image(w.Xp, D); g.K0 = D; g.K = D; wplanes(g, h->fin);
    g.rtab = rt; g.a0_slot = s_x; g.a1_slot = -1;
    g.R = R; g.Nout = D; g.Y = w.md; g.ldy = D;
    SG_HIP(gemm_h3(g, EPI_STORE, st));
  }
  float* cost = out->sinkhorn_cost ? out->sinkhorn_cost : w.cost;
  {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A0 = w.md; g.lda0 = D; g.K0 = D; g.K = D; g.sA = (long long)M * D;
    g.W = w.md + (size_t)B * M * D; g.ldw = D; g.sW = (long long)N * D;
    g.R = M; g.Nout = N; g.Y = cost; g.ldy = N; g.sY = (long long)M * N;
    g.out_scale = 1.f / 16.f;
    SG_HIP(gemm_x6(g, EPI_STORE, B, st));
  }
  float* Z = out->log_assignment ? out->log_assignment : w.Z;
  SG_HIP(log_optimal_transport(cost, h->bin_score, B, M, N, h->cfg.sinkhorn_iterations, Z, w.sws, st));
  SG_HIP(filter_from_scores(Z, B, M, N, h->cfg.filter_threshold, w.fws, out->matches0, out->matches1,
                            out->matching_scores0, out->matching_scores1, st));
  return LG_OK;
}

static int nll_loss(const float* la, int32_t B, int32_t M, int32_t N, const uint8_t* gta, const int64_t* gt0,
                    const int64_t* gt1, int32_t mode, float bal, float* out, void* ws, size_t ws_bytes, void* stream) {
  if (!la || !gta || !gt0 || !gt1 || !out || B < 0 || M < 0 || N < 0) return fail(LG_E_INVALID, "bad argument");
  if (ws && ws_bytes < sizeof(double) * lg::sg_nll_part_doubles(B, M)) return fail(LG_E_WORKSPACE, "workspace too small");
  if (mode != 0 && mode != 1) return fail(LG_E_INVALID, "mode must be 0 (SuperGlue.loss) or 1 (NLLLoss)");
  if (mode == 1 && M != N)  // losses.py:72 writes gt_matches1 == -1 into [:, -1, :m]
    return fail(LG_E_INVALID, "The expanded size of the tensor (" + std::to_string(M) +
                                  ") must match the existing size (" + std::to_string(N) + ") at non-singleton dimension 1");
  SG_HIP(lg::sg_nll_loss(la, B, M, N, gta, gt0, gt1, mode, bal, out, static_cast<double*>(ws), (hipStream_t)stream));
  return LG_OK;
}

size_t sg_collective_floats(void) { return lg::bn_sync_floats(); }

int sg_set_collective(sg_handle_t* h, sg_collective_fn fn, void* ctx, float* buf, int64_t capacity) {
  if (!h) return fail(LG_E_INVALID, "null handle");
  if (fn && (!buf || capacity < (int64_t)lg::bn_sync_floats()))
    return fail(LG_E_WORKSPACE, "collective buffer too small: need " + std::to_string(lg::bn_sync_floats()) + " floats");
  h->sync = fn ? lg::BnSync{fn, ctx, buf, capacity} : lg::BnSync{};
  return LG_OK;
}

int sg_set_grad_ready_hook(sg_handle_t* h, sg_grad_ready_fn fn, void* ctx) {
  if (!h) return fail(LG_E_INVALID, "null handle");
  h->grad_hook = fn;
  h->grad_hook_ctx = fn ? ctx : nullptr;
  return LG_OK;
}

int sg_nll_workspace_bytes(int32_t B, int32_t M, size_t* bytes) {
  if (!bytes || B < 0 || M < 0) return fail(LG_E_INVALID, "bad argument");
  *bytes = sizeof(double) * lg::sg_nll_part_doubles(B, M);
  return LG_OK;
}

int sg_nll_loss(const float* la, int32_t B, int32_t M, int32_t N, const uint8_t* gta, const int64_t* gt0, const int64_t* gt1,
                int32_t mode, float bal, float* out, void* stream) {
  return nll_loss(la, B, M, N, gta, gt0, gt1, mode, bal, out, nullptr, 0, stream);
}

int sg_nll_loss_ws(const float* la, int32_t B, int32_t M, int32_t N, const uint8_t* gta, const int64_t* gt0,
                   const int64_t* gt1, int32_t mode, float bal, float* out, void* workspace, size_t workspace_bytes,
                   void* stream) {
  if (!workspace) return fail(LG_E_WORKSPACE, "missing workspace");
  return nll_loss(la, B, M, N, gta, gt0, gt1, mode, bal, out, workspace, workspace_bytes, stream);
}

}  // extern "C"
