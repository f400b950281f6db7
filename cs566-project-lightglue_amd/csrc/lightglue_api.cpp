// C-ABI of liblightglue_mi355x.so: handle, weight repacking and the LightGlue eval forward
// orchestration (reference gluefactory/models/matchers/lightglue.py:444-579).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/lightglue_mi355x.h"
#include "kernels.h"

// two-image launches of the input preparation / final matchability (round 6 A/B switches)
#ifndef LG_MERGE_PE
#define LG_MERGE_PE 1
#endif
#ifndef LG_MERGE_R2P
#define LG_MERGE_R2P 1
#endif
#ifndef LG_MERGE_GEMV
#define LG_MERGE_GEMV 1
#endif
#include "common.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define LG_HIP(expr)                                                                                \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      return fail(LG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));                     \
  } while (0)

struct Tensor {
  std::string name;
  std::vector<int64_t> shape;
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

// Same order as lightglue_amd.weights.state_dict_schema (lightglue.py:367-398).
std::vector<Tensor> make_schema(const lg_config_t& c) {
  const int64_t d = c.descriptor_dim, din = c.input_dim, L = c.n_layers;
  const int64_t hd = d / c.num_heads, m_in = 2 + 2 * (c.add_scale_ori ? 1 : 0);
  std::vector<Tensor> s;
  auto add = [&](const std::string& n, std::vector<int64_t> sh) { s.push_back({n, sh}); };
  auto ffn = [&](const std::string& p) {
    add(p + ".ffn.0.weight", {2 * d, 2 * d});
    add(p + ".ffn.0.bias", {2 * d});
    add(p + ".ffn.1.weight", {2 * d});
    add(p + ".ffn.1.bias", {2 * d});
    add(p + ".ffn.3.weight", {d, 2 * d});
    add(p + ".ffn.3.bias", {d});
  };
  if (din != d) {
    add("input_proj.weight", {d, din});
    add("input_proj.bias", {d});
  }
  add("posenc.Wr.weight", {hd / 2, m_in});
  add("posenc.condition_modulation.weight", {hd / 2, 1});
  add("posenc.condition_modulation.bias", {hd / 2});
  for (int64_t i = 0; i < L; ++i) {
    const std::string sp = "transformers." + std::to_string(i) + ".self_attn";
    add(sp + ".Wqkv.weight", {3 * d, d});
    add(sp + ".Wqkv.bias", {3 * d});
    add(sp + ".out_proj.weight", {d, d});
    add(sp + ".out_proj.bias", {d});
    ffn(sp);
    const std::string cp = "transformers." + std::to_string(i) + ".cross_attn";
    add(cp + ".to_qk.weight", {d, d});
    add(cp + ".to_qk.bias", {d});
    add(cp + ".to_v.weight", {d, d});
    add(cp + ".to_v.bias", {d});
    add(cp + ".to_out.weight", {d, d});
    add(cp + ".to_out.bias", {d});
    ffn(cp);
  }
  for (int64_t i = 0; i < L; ++i) {
    const std::string a = "log_assignment." + std::to_string(i);
    add(a + ".matchability.weight", {1, d});
    add(a + ".matchability.bias", {1});
    add(a + ".final_proj.weight", {d, d});
    add(a + ".final_proj.bias", {d});
  }
  for (int64_t i = 0; i + 1 < L; ++i) {
    const std::string t = "token_confidence." + std::to_string(i) + ".token.0";
    add(t + ".weight", {1, d});
    add(t + ".bias", {1});
  }
  return s;
}

constexpr int D = 256;
// range-table slots one forward uses at most: 3 for the inputs, 5 per block (4 with out_proj
// folded), 1 per pruned layer, 1 for the assignment head's md image
int range_slots(int n_layers) { return 8 + 11 * n_layers; }

// Packed per-layer weights (offsets in floats into one device buffer).
struct BlockW {
  size_t Wqkv, bqkv, Wo, bo, W1, b1, g, be, W2, b2;
};
struct LayerW {
  BlockW self, cross;
  size_t Wf, bf, wm, bm, wt, bt;
};

size_t align64(size_t n) { return (n + 63) & ~size_t(63); }

}  // namespace

namespace lg {
// the other C-ABI families of this library (superpoint_api.cpp) report through lg_last_error()
int api_fail(int code, const char* msg) {
  g_err = msg;
  return code;
}
}  // namespace lg

struct lg_handle {
  lg_config_t cfg;
  int device;
  lg_grad_ready_fn grad_hook = nullptr;  // lg_set_grad_ready_hook (data-parallel training)
  void* grad_hook_ctx = nullptr;
  std::vector<Tensor> schema;
  std::map<std::string, int> index;
  // where each schema tensor goes: destination offset (floats) and how (0 copy, 1 gather rows
  // through perm[0,768) (Wqkv), 2 gather through perm[768,1024) (to_qk / to_v))
  std::vector<size_t> dst;
  std::vector<int> gkind;
  std::vector<LayerW> layers;
  size_t Wr, Wc, bc, Wi, bi, total;
  float* wbuf = nullptr;
  int* perm = nullptr;  // head_perm() [1024]
  // fp16x3 plane images of every GEMM weight matrix (PREC_H3), keyed by the fp32 offset
  struct Planes {
    size_t off;         // halfs into wplanes
    long long pstride;  // rows * K
    int rows;
    float unscale;      // 2^-(11+sw)
  };
  std::map<size_t, Planes> planes;
  _Float16* wplanes = nullptr;
  // run-time range bounds (kernels.h RangeOut), per layer and block: row-L1 maxima and bias
  // maxima of the matrices whose outputs become plane images, and the LayerNorm output bound
  struct BlockGain {
    float gK, bK, gV, bV;  // key / value rows of Wqkv (self: rotary x1.5) or to_qk (x scale^0.5) / to_v
    float hb;              // |GELU(LN(.))| <= hb
    float g2, b2;          // ffn.3
    float go, bo;          // out_proj / to_out (unfolded path only)
  };
  std::vector<BlockGain> gains;  // [layer * 2 + block]
  float gi = 0.f, bi_max = 0.f;  // input_proj
  std::vector<float> gf, bf_max;  // per layer: final_proj row-L1 max / |bias| max (md range bound)
  bool loaded = false;
  bool pass_started = false;  // forward_pass got past argument checks (work was enqueued)
  // fold out_proj / to_out into ffn.0 at load time (env LG_FOLD_OUT_PROJ=0 disables)
  bool fold = true;
  // ffn.3 walks its tiles back to front (the LN GEMM's newest output first; LG_FFN3_REVERSE=0|1)
  int ffn3_reverse = 1;
  // profiling (lg_profile_enable / lg_profile_read)
  struct Rec {
    hipEvent_t a, b;
    int kind;
    double flops, bytes;
    // pruned forwards: the per-pair counts at launch time (a stream-ordered copy into snap), from
    // which lg_profile_read recomputes the launch's algorithmic flops over the LIVE rows only
    int snap = -1;  // offset (ints) into snap: cnt[2B], then sel[B] when has_sel
    int B = 0, sel_eq = 0, mode = 0;  // mode 1: self attention, 2: cross attention, 3: GEMM
    bool has_sel = false;
    double unit = 0.0;  // self/cross: 64 * heads; GEMM: 2 * K * Nout
  };
  bool prof_on = false;
  unsigned prof_mask = 0;  // bit k: kernel family k is timed
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  int* snap = nullptr;
  size_t snap_cap = 0, snap_used = 0;
  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  int prof_begin(int kind, hipStream_t st) {
    if (!prof_on || !(prof_mask & (1u << kind))) return -1;
    Rec r{ev(), ev(), kind, 0.0, 0.0};
    (void)hipEventRecord(r.a, st);
    recs.push_back(r);
    return (int)recs.size() - 1;
  }
  void prof_end(int idx, double flops, double bytes, hipStream_t st) {
    if (idx < 0) return;
    recs[idx].flops = flops;
    recs[idx].bytes = bytes;
    (void)hipEventRecord(recs[idx].b, st);
  }
  // attach the live-row counts of a pruned forward to record idx (no-op outside profiling)
  void prof_counts(int idx, int mode, double unit, const int* cnt, const int* sel, int sel_eq, int B, hipStream_t st) {
    if (idx < 0 || !cnt || !snap) return;
    const size_t need = 3 * (size_t)B;
    if (snap_used + need > snap_cap) return;  // out of snapshot space: the capacity flops stay
    Rec& r = recs[idx];
    r.snap = (int)snap_used;
    r.B = B;
    r.mode = mode;
    r.unit = unit;
    r.sel_eq = sel_eq;
    r.has_sel = sel != nullptr;
    (void)hipMemcpyAsync(snap + snap_used, cnt, 2 * B * sizeof(int), hipMemcpyDeviceToDevice, st);
    if (sel) (void)hipMemcpyAsync(snap + snap_used + 2 * B, sel, B * sizeof(int), hipMemcpyDeviceToDevice, st);
    snap_used += need;
  }
};

namespace {

// Packed projection row order c' = t*256 + h*64 + j with j < 32 -> dim 2j, j >= 32 -> dim
// 2(j-32)+1: lane l32 of a 64-wide GEMM wave tile then holds the natural-order dim pair
// (2*l32, 2*l32+1) -- the rotary partners -- so the epilogue stores pairs (gemm.hip).
//   perm[0, 768):    Wqkv, reference layout row = h*192 + dim*3 + t (lightglue.py:185)
//   perm[768, 1024): to_qk / to_v, reference layout row = h*64 + dim (lightglue.py:226)
constexpr int kPermCross = 3 * D;
std::vector<int> head_perm(int H) {
  std::vector<int> p(4 * D);
  auto dim = [](int j) { return j < 32 ? 2 * j : 2 * (j - 32) + 1; };
  for (int t = 0; t < 3; ++t)
    for (int h = 0; h < H; ++h)
      for (int j = 0; j < 64; ++j) p[t * D + h * 64 + j] = h * 192 + dim(j) * 3 + t;
  for (int h = 0; h < H; ++h)
    for (int j = 0; j < 64; ++j) p[kPermCross + h * 64 + j] = h * 64 + dim(j);
  return p;
}

void plan_layout(lg_handle* h) {
  size_t off = 0;
  auto take = [&](size_t n) {
    size_t o = off;
    off += align64(n);
    return o;
  };
  const int L = h->cfg.n_layers;
  const int m_in = 2 + 2 * (h->cfg.add_scale_ori ? 1 : 0);
  h->layers.resize(L);
  h->Wr = take(32 * m_in);
  h->Wc = take(32);
  h->bc = take(32);
  h->Wi = take((size_t)D * h->cfg.input_dim);
  h->bi = take(D);
  for (int i = 0; i < L; ++i) {
    for (int b = 0; b < 2; ++b) {
      BlockW& w = b == 0 ? h->layers[i].self : h->layers[i].cross;
      const int nq = b == 0 ? 3 * D : 2 * D;
      w.Wqkv = take((size_t)nq * D);
      w.bqkv = take(nq);
      w.Wo = take((size_t)D * D);
      w.bo = take(D);
      w.W1 = take((size_t)2 * D * 2 * D);
      w.b1 = take(2 * D);
      w.g = take(2 * D);
      w.be = take(2 * D);
      w.W2 = take((size_t)D * 2 * D);
      w.b2 = take(D);
    }
    h->layers[i].Wf = take((size_t)D * D);
    h->layers[i].bf = take(D);
    h->layers[i].wm = take(D);
    h->layers[i].bm = take(1);
    h->layers[i].wt = take(D);
    h->layers[i].bt = take(1);
  }
  h->total = off;

  // destination of each schema tensor (projection weights are gathered through head_perm)
  h->dst.assign(h->schema.size(), SIZE_MAX);
  h->gkind.assign(h->schema.size(), 0);
  for (size_t k = 0; k < h->schema.size(); ++k) {
    const std::string& n = h->schema[k].name;
    size_t o = SIZE_MAX;
    if (n == "posenc.Wr.weight") o = h->Wr;
    else if (n == "posenc.condition_modulation.weight") o = h->Wc;
    else if (n == "posenc.condition_modulation.bias") o = h->bc;
    else if (n == "input_proj.weight") o = h->Wi;
    else if (n == "input_proj.bias") o = h->bi;
    else {
      int li = -1;
      char rest[160] = {0};
      if (sscanf(n.c_str(), "transformers.%d.%159s", &li, rest) == 2) {
        const std::string r = rest;
        LayerW& lw = h->layers[li];
        const bool self = r.rfind("self_attn.", 0) == 0;
        BlockW& w = self ? lw.self : lw.cross;
        const std::string f = r.substr(r.find('.') + 1);
        if (f == "Wqkv.weight") { o = w.Wqkv; h->gkind[k] = 1; }
        else if (f == "Wqkv.bias") { o = w.bqkv; h->gkind[k] = 1; }
        else if (f == "to_qk.weight") { o = w.Wqkv; h->gkind[k] = 2; }
        else if (f == "to_qk.bias") { o = w.bqkv; h->gkind[k] = 2; }
        else if (f == "to_v.weight") { o = w.Wqkv + (size_t)D * D; h->gkind[k] = 2; }
        else if (f == "to_v.bias") { o = w.bqkv + D; h->gkind[k] = 2; }
        else if (f == "out_proj.weight" || f == "to_out.weight") o = w.Wo;
        else if (f == "out_proj.bias" || f == "to_out.bias") o = w.bo;
        else if (f == "ffn.0.weight") o = w.W1;
        else if (f == "ffn.0.bias") o = w.b1;
        else if (f == "ffn.1.weight") o = w.g;
        else if (f == "ffn.1.bias") o = w.be;
        else if (f == "ffn.3.weight") o = w.W2;
        else if (f == "ffn.3.bias") o = w.b2;
      } else if (sscanf(n.c_str(), "log_assignment.%d.%159s", &li, rest) == 2) {
        const std::string r = rest;
        LayerW& lw = h->layers[li];
        if (r == "final_proj.weight") o = lw.Wf;
        else if (r == "final_proj.bias") o = lw.bf;
        else if (r == "matchability.weight") o = lw.wm;
        else if (r == "matchability.bias") o = lw.bm;
      } else if (sscanf(n.c_str(), "token_confidence.%d.%159s", &li, rest) == 2) {
        const std::string r = rest;
        if (r == "token.0.weight") o = h->layers[li].wt;
        else if (r == "token.0.bias") o = h->layers[li].bt;
      }
    }
    h->dst[k] = o;
  }
}

// ------------------------------------------------------------------ forward workspace
struct Work {
  float *X, *X2, *cosb, *sinb, *cos2, *sin2, *size, *Q, *ctx, *msg, *H1, *md, *z, *tok, *sim, *aws;
  void *KP, *VP;  // operand planes of keys (qk) and values: 3 bf16 (X6) / 2 fp16 (H3) x R x 256
  // PREC_H3 plane images (common.h), rows_pad rows: x, context, message (unfolded out_proj),
  // FFN hidden, input descriptors (input_dim != 256)
  _Float16 *Xp, *Cp, *Mp, *Hp, *Dp;
  _Float16* mdp;  // md = final_proj(x) / 4 as a plane image (rows_pad + 256 rows) for the fused assignment
  float* Dst;
  int rows_pad;
  size_t R;
  int *flags, *pos, *ind, *indb, *cnt, *cntb, *act, *stop;  // pruning / early stop (SegLayout)
  unsigned* rtab;  // PREC_H3 range table (kernels.h RangeOut), nslots slots
  int nslots;
  int64_t *m0c, *m1c;
  float *s0c, *s1c;
  float* apart;  // attention key-split partials (small batches)
  size_t apart_floats;
  size_t bytes;
};

Work carve(char* base, int B, int M, int N, bool prune, int din, int n_layers) {
  const size_t R = (size_t)B * (M + N);
  const size_t RP = (R + 255) / 256 * 256;
  Work w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~size_t(255);
    return p;
  };
  auto tf = [&](size_t n) { return reinterpret_cast<float*>(take(n * sizeof(float))); };
  auto ti = [&](size_t n) { return reinterpret_cast<int*>(take(n * sizeof(int))); };
  auto th = [&](size_t n) { return reinterpret_cast<_Float16*>(take(n * sizeof(_Float16))); };
  w.X = tf(R * D);
  w.cosb = tf(R * 32);
  w.sinb = tf(R * 32);
  w.size = tf(4 * (size_t)B);
  w.R = R;
  w.rows_pad = (int)RP;
  w.Q = tf(R * D);
  w.KP = take(3 * R * D * 2);
  w.VP = take(3 * R * D * 2);
  w.ctx = tf(R * D);
  w.msg = tf(R * D);
  w.H1 = tf(R * 2 * D);
  w.Xp = th(2 * RP * D);
  w.Cp = th(2 * RP * D);
  w.Mp = th(2 * RP * D);
  w.Hp = th(2 * RP * 2 * D);
  w.Dp = din != D ? th(2 * RP * din) : nullptr;
  w.Dst = din != D ? tf(R * din) : nullptr;  // staging for 16-byte-unaligned input descriptors
  w.md = tf(R * D);
  w.mdp = th(2 * (RP + 256) * D);
  w.z = tf(R);
  w.tok = tf(R);
  w.sim = tf((size_t)B * M * N);
  w.aws = tf(lg::assign_workspace_floats(B, M, N) + 64 + lg::sim_h3_workspace_floats(B, M, N));
  w.apart_floats = lg::attention_split_floats(B, D / 64, std::max(M, N), std::max(M, N));
  w.apart = w.apart_floats ? tf(w.apart_floats) : nullptr;
  w.nslots = range_slots(n_layers);
  w.rtab = reinterpret_cast<unsigned*>(ti((size_t)w.nslots * lg::kRangeStride));
  if (prune) {
    w.X2 = tf(R * D);
    w.cos2 = tf(R * 32);
    w.sin2 = tf(R * 32);
    w.flags = ti(R);
    w.pos = ti(R);
    w.ind = ti(R);
    w.indb = ti(R);
    w.cnt = ti(2 * (size_t)B);
    w.cntb = ti(2 * (size_t)B);
    w.act = ti(B);
    w.stop = ti(B);
    w.m0c = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * B * M));
    w.m1c = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * B * N));
    w.s0c = tf((size_t)B * M);
    w.s1c = tf((size_t)B * N);
  }
  w.bytes = off;
  return w;
}

bool prune_enabled(const lg_config_t& c) { return c.width_confidence > 0.f || c.depth_confidence > 0.f; }

lg::GemmArgs gemm_base() {
  lg::GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.out_scale = 1.f;
  return a;
}

lg::GemmH3Args gemm_h3_base() {
  lg::GemmH3Args a;
  memset(&a, 0, sizeof(a));
  a.out_scale = 1.f;
  return a;
}

float confidence_threshold(int i, int L) {  // lightglue.py:581-584
  double t = 0.8 + 0.1 * std::exp(-4.0 * i / L);
  return (float)std::min(1.0, std::max(0.0, t));  // compared in fp32 like torch
}

}  // namespace

extern "C" {

int lg_abi_version(void) { return LG_ABI_VERSION; }
const char* lg_last_error(void) { return g_err.c_str(); }

int lg_create(const lg_config_t* cfg, int device, lg_handle_t** out) {
  if (!cfg || !out) return fail(LG_E_INVALID, "null argument");
  if (cfg->descriptor_dim != D) return fail(LG_E_INVALID, "descriptor_dim must be 256 (kernels are specialised)");
  if (cfg->num_heads <= 0 || cfg->descriptor_dim / cfg->num_heads != 64 || cfg->descriptor_dim % cfg->num_heads)
    return fail(LG_E_INVALID, "head_dim must be 64 (descriptor_dim / num_heads)");
  if (cfg->n_layers < 1) return fail(LG_E_INVALID, "n_layers must be >= 1");
  if (cfg->input_dim <= 0 || cfg->input_dim % 32) return fail(LG_E_INVALID, "input_dim must be a positive multiple of 32");
  LG_HIP(hipSetDevice(device));
  lg_handle* h = new lg_handle();
  h->cfg = *cfg;
  h->device = device;
  if (const char* f = getenv("LG_FOLD_OUT_PROJ")) h->fold = atoi(f) != 0;
  if (const char* f = getenv("LG_FFN3_REVERSE")) h->ffn3_reverse = atoi(f) != 0;
  h->schema = make_schema(*cfg);
  for (size_t k = 0; k < h->schema.size(); ++k) h->index[h->schema[k].name] = (int)k;
  plan_layout(h);
  for (size_t k = 0; k < h->schema.size(); ++k)
    if (h->dst[k] == SIZE_MAX) {
      std::string n = h->schema[k].name;
      delete h;
      return fail(LG_E_WEIGHTS, "internal: unplaced schema tensor " + n);
    }
  hipError_t e = hipMalloc(&h->wbuf, h->total * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&h->perm, 4 * D * sizeof(int));
  if (e == hipSuccess) {
    auto p = head_perm(cfg->num_heads);
    e = hipMemcpy(h->perm, p.data(), p.size() * sizeof(int), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemset(h->wbuf, 0, h->total * sizeof(float));
  if (e != hipSuccess) {
    if (h->wbuf) (void)hipFree(h->wbuf);
    if (h->perm) (void)hipFree(h->perm);
    delete h;
    return fail(LG_E_HIP, std::string("allocation: ") + hipGetErrorString(e));
  }
  *out = h;
  return LG_OK;
}

int lg_destroy(lg_handle_t* h) {
  if (!h) return LG_OK;
  (void)hipSetDevice(h->device);
  if (h->wbuf) (void)hipFree(h->wbuf);
  if (h->perm) (void)hipFree(h->perm);
  if (h->wplanes) (void)hipFree(h->wplanes);
  if (h->snap) (void)hipFree(h->snap);
  for (auto& r : h->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : h->pool) (void)hipEventDestroy(e);
  delete h;
  return LG_OK;
}

int lg_set_grad_ready_hook(lg_handle_t* h, lg_grad_ready_fn fn, void* ctx) {
  if (!h) return fail(LG_E_INVALID, "null handle");
  h->grad_hook = fn;
  h->grad_hook_ctx = fn ? ctx : nullptr;
  return LG_OK;
}
}  // extern "C"

// accessors for the training entry points (lightglue_train.cpp)
namespace lg {
const lg_config_t* handle_config(const lg_handle* h) { return &h->cfg; }
int handle_device(const lg_handle* h) { return h->device; }
void handle_grad_ready(const lg_handle* h, int layer, void* stream) {
  if (h->grad_hook) h->grad_hook(h->grad_hook_ctx, layer, stream);
}
int handle_weight_index(const lg_handle* h, const std::string& name) {
  auto it = h->index.find(name);
  return it == h->index.end() ? -1 : it->second;
}
}  // namespace lg

extern "C" {

int lg_weight_count(const lg_handle_t* h) { return h ? (int)h->schema.size() : 0; }
const char* lg_weight_name(const lg_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].name.c_str() : nullptr;
}
int64_t lg_weight_numel(const lg_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].numel() : -1;
}

int lg_load_weights(lg_handle_t* h, int n, const char* const* names, const float* const* tensors, const int64_t* numels,
                    void* stream) {
  if (!h || n < 0 || (n && (!names || !tensors || !numels))) return fail(LG_E_INVALID, "null argument");
  LG_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  std::vector<int> seen(h->schema.size(), 0);
  for (int i = 0; i < n; ++i) {
    auto it = h->index.find(names[i]);
    if (it == h->index.end()) return fail(LG_E_WEIGHTS, std::string("unexpected key in state_dict: ") + names[i]);
    const int k = it->second;
    if (seen[k]++) return fail(LG_E_WEIGHTS, std::string("duplicate key: ") + names[i]);
    if (numels[i] != h->schema[k].numel())
      return fail(LG_E_WEIGHTS, std::string("size mismatch for ") + names[i] + ": expected " +
                                    std::to_string(h->schema[k].numel()) + " got " + std::to_string(numels[i]));
  }
  for (size_t k = 0; k < h->schema.size(); ++k)
    if (!seen[k]) return fail(LG_E_WEIGHTS, "missing key in state_dict: " + h->schema[k].name);
  for (int i = 0; i < n; ++i) {
    const int k = h->index[names[i]];
    const std::string& name = h->schema[k].name;
    if (h->gkind[k] != 0) {
      const bool is_w = name.size() > 6 && name.compare(name.size() - 6, 6, "weight") == 0;
      const int rows = h->gkind[k] == 1 ? 3 * D : D;
      const int* perm = h->perm + (h->gkind[k] == 1 ? 0 : kPermCross);
      hipError_t e = lg::gather_rows(h->wbuf + h->dst[k], tensors[i], perm, rows, is_w ? D : 1, st);
      if (e != hipSuccess) return fail(LG_E_HIP, std::string("gather ") + name + ": " + hipGetErrorString(e));
    } else {
      LG_HIP(hipMemcpyAsync(h->wbuf + h->dst[k], tensors[i], numels[i] * sizeof(float), hipMemcpyDeviceToDevice, st));
    }
  }
  if (h->fold) {
    float* tmp = nullptr;
    LG_HIP(hipMallocAsync((void**)&tmp, (512 * 256 + 512) * sizeof(float), st));
    for (auto& lw : h->layers)
      for (int b = 0; b < 2; ++b) {
        const BlockW& w = b == 0 ? lw.self : lw.cross;
        hipError_t e = lg::fold_out_proj(h->wbuf + w.W1, h->wbuf + w.b1, h->wbuf + w.Wo, h->wbuf + w.bo, tmp, st);
        if (e != hipSuccess) return fail(LG_E_HIP, std::string("fold_out_proj: ") + hipGetErrorString(e));
      }
    LG_HIP(hipFreeAsync(tmp, st));
  }
  // fp16x3 plane images (common.h) of every GEMM weight matrix, scaled per matrix by 2^sw so
  // that max|W 2^sw| lies in [8, 16) (gemm_h3.hip forms the third piece, h * 2^11, in registers)
  {
    struct Mat { size_t off; int rows, K; };
    std::vector<Mat> mats;
    if (h->cfg.input_dim != D) mats.push_back({h->Wi, D, h->cfg.input_dim});
    for (auto& lw : h->layers) {
      for (int b = 0; b < 2; ++b) {
        const BlockW& w = b == 0 ? lw.self : lw.cross;
        mats.push_back({w.Wqkv, b == 0 ? 3 * D : 2 * D, D});
        if (!h->fold) mats.push_back({w.Wo, D, D});
        mats.push_back({w.W1, 2 * D, 2 * D});
        mats.push_back({w.W2, D, 2 * D});
      }
      mats.push_back({lw.Wf, D, D});
    }
    size_t total = 0;
    for (auto& m : mats) total += 2 * (size_t)m.rows * m.K;
    if (h->wplanes) (void)hipFree(h->wplanes);
    h->wplanes = nullptr;
    h->planes.clear();
    LG_HIP(hipMalloc((void**)&h->wplanes, total * sizeof(_Float16)));
    float* dmax = nullptr;
    LG_HIP(hipMallocAsync((void**)&dmax, mats.size() * sizeof(float), st));
    for (size_t i = 0; i < mats.size(); ++i)
      LG_HIP(lg::absmax(h->wbuf + mats[i].off, (size_t)mats[i].rows * mats[i].K, dmax + i, st));
    std::vector<float> mx(mats.size());
    LG_HIP(hipMemcpyAsync(mx.data(), dmax, mats.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    LG_HIP(hipStreamSynchronize(st));
    LG_HIP(hipFreeAsync(dmax, st));
    size_t off = 0;
    for (size_t i = 0; i < mats.size(); ++i) {
      int sw = 0;
      if (mx[i] > 0.f && std::isfinite(mx[i])) {
        int E;
        (void)std::frexp(mx[i], &E);  // max = m 2^E, m in [0.5, 1)
        sw = std::min(std::max(4 - E, -100), 100);
      }
      const size_t n = (size_t)mats[i].rows * mats[i].K;
      LG_HIP(lg::split_weight_h3(h->wbuf + mats[i].off, mats[i].rows, mats[i].K, std::ldexp(1.f, sw), h->wplanes + off, st));
      h->planes[mats[i].off] = {off, (long long)n, mats[i].rows, std::ldexp(1.f, -(11 + sw))};
      off += 2 * n;
    }
  }
  // range-bound statistics (one read-back at load time)
  {
    const int L = h->cfg.n_layers;
    const int per = 2 * 4 + 1;  // per block: K, V, W2, Wo stats (2 floats each) + LN bound
    const int nf = L * 2 * per + 2;
    float* dst = nullptr;
    LG_HIP(hipMallocAsync((void**)&dst, nf * sizeof(float), st));
    const float* W = h->wbuf;
    for (int i = 0; i < L; ++i)
      for (int b = 0; b < 2; ++b) {
        const BlockW& w = b == 0 ? h->layers[i].self : h->layers[i].cross;
        float* o = dst + (i * 2 + b) * per;
        const size_t k0 = b == 0 ? (size_t)D : 0, v0 = b == 0 ? 2 * (size_t)D : (size_t)D;
        LG_HIP(lg::weight_range_stats(W + w.Wqkv + k0 * D, D, D, W + w.bqkv + k0, o + 0, st));
        LG_HIP(lg::weight_range_stats(W + w.Wqkv + v0 * D, D, D, W + w.bqkv + v0, o + 2, st));
        LG_HIP(lg::weight_range_stats(W + w.W2, D, 2 * D, W + w.b2, o + 4, st));
        LG_HIP(lg::weight_range_stats(W + w.Wo, D, D, W + w.bo, o + 6, st));
        LG_HIP(lg::layernorm_bound(W + w.g, W + w.be, 2 * D, o + 8, st));
      }
    if (h->cfg.input_dim != D) LG_HIP(lg::weight_range_stats(W + h->Wi, D, h->cfg.input_dim, W + h->bi, dst + nf - 2, st));
    else LG_HIP(hipMemsetAsync(dst + nf - 2, 0, 2 * sizeof(float), st));
    std::vector<float> hs(nf);
    LG_HIP(hipMemcpyAsync(hs.data(), dst, nf * sizeof(float), hipMemcpyDeviceToHost, st));
    LG_HIP(hipStreamSynchronize(st));
    LG_HIP(hipFreeAsync(dst, st));
    h->gains.assign((size_t)L * 2, {});
    const float qk_scale = std::sqrt(1.f / std::sqrt(64.f));
    for (int i = 0; i < L * 2; ++i) {
      const float* o = hs.data() + i * per;
      // self keys are rotated: |k cos - k' sin| <= sqrt(2) max(|k|, |k'|) < 1.5 max
      const float kf = (i % 2 == 0) ? 1.5f : qk_scale;
      h->gains[i] = {o[0] * kf, o[1] * kf, o[2], o[3], o[8], o[4], o[5], o[6], o[7]};
    }
    h->gi = hs[nf - 2];
    h->bi_max = hs[nf - 1];
    // final_proj of every layer (the md plane image of the fused assignment)
    float* fst = nullptr;
    LG_HIP(hipMallocAsync((void**)&fst, 2 * L * sizeof(float), st));
    for (int i = 0; i < L; ++i)
      LG_HIP(lg::weight_range_stats(W + h->layers[i].Wf, D, D, W + h->layers[i].bf, fst + 2 * i, st));
    std::vector<float> fs(2 * L);
    LG_HIP(hipMemcpyAsync(fs.data(), fst, 2 * L * sizeof(float), hipMemcpyDeviceToHost, st));
    LG_HIP(hipStreamSynchronize(st));
    LG_HIP(hipFreeAsync(fst, st));
    h->gf.resize(L);
    h->bf_max.resize(L);
    for (int i = 0; i < L; ++i) {
      h->gf[i] = fs[2 * i];
      h->bf_max[i] = fs[2 * i + 1];
    }
  }
  h->loaded = true;
  return LG_OK;
}

int lg_workspace_bytes(const lg_handle_t* h, int32_t B, int32_t M, int32_t N, size_t* bytes) {
  if (!h || !bytes || B < 0 || M < 0 || N < 0) return fail(LG_E_INVALID, "bad argument");
  *bytes = carve(nullptr, B, M, N, prune_enabled(h->cfg), h->cfg.input_dim, h->cfg.n_layers).bytes;
  return LG_OK;
}

// One full eval forward in operand format `prec` (lg::PREC_H3 / PREC_X6).
static int forward_pass(lg_handle_t* h, const lg_inputs_t* in, lg_outputs_t* out, void* workspace,
                        size_t workspace_bytes, void* stream, int prec) {
  using namespace lg;
  if (!h || !in || !out) return fail(LG_E_INVALID, "null argument");
  if (!h->loaded) return fail(LG_E_WEIGHTS, "weights not loaded");
  h->pass_started = false;
  const lg_config_t& c = h->cfg;
  const int B = in->B, M0 = in->M, N0 = in->N, H = c.num_heads, L = c.n_layers;
  if (B <= 0) return fail(LG_E_INVALID, "batch must be >= 1");
  if (M0 <= 0 || N0 <= 0)
    return fail(LG_E_INVALID, "max(): Expected reduction dim to have non-zero size (empty keypoint set)");
  if (!in->keypoints0 || !in->keypoints1 || !in->descriptors0 || !in->descriptors1)
    return fail(LG_E_INVALID, "missing input tensor");
  if (c.add_scale_ori && (!in->scales0 || !in->oris0 || !in->scales1 || !in->oris1))
    return fail(LG_E_INVALID, "add_scale_ori requires scales0/1 and oris0/1");
  if (!out->matches0 || !out->matches1 || !out->matching_scores0 || !out->matching_scores1)
    return fail(LG_E_INVALID, "missing output tensor");
  // training-mode gating (lightglue.py:502-503): no early stop, no pruning
  const bool gated = (in->flags & LG_FWD_TRAINING_GATE) != 0;
  const bool do_stop = !gated && c.depth_confidence > 0.f, do_prune = !gated && c.width_confidence > 0.f;
  if ((out->layer_descriptors0 || out->layer_descriptors1) && (do_stop || do_prune))
    return fail(LG_E_INVALID, "layer_descriptors need early stop and pruning off (training-mode outputs)");
  if (do_prune && (!out->prune0 || !out->prune1)) return fail(LG_E_INVALID, "prune0/prune1 outputs required with pruning");
  const Work need = carve(nullptr, B, M0, N0, prune_enabled(c), c.input_dim, c.n_layers);
  const bool din_a16 = ((uintptr_t)in->descriptors0 % 16 == 0) && ((uintptr_t)in->descriptors1 % 16 == 0);
  if (!workspace || workspace_bytes < need.bytes)
    return fail(LG_E_WORKSPACE, "workspace too small: need " + std::to_string(need.bytes));
  LG_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  Work w = carve((char*)workspace, B, M0, N0, prune_enabled(c), c.input_dim, c.n_layers);
  const float* Wb = h->wbuf;
  int M = M0, N = N0;
  const int RP = w.rows_pad;
  // launch wrappers that feed lg_profile_* (algorithmic flops / bytes per launch)
  auto gemm = [&](const GemmArgs& g, int epi, int batch) -> hipError_t {
    const int p = h->prof_begin(LG_KERNEL_GEMM, st);
    const hipError_t e = gemm_x6(g, epi, batch, st);
    const double R = g.R, K = g.K, O = g.Nout;
    h->prof_end(p, 2.0 * R * K * O * batch, 4.0 * (R * K + O * K + R * O) * batch, st);
    return e;
  };
  auto gemmh = [&](const GemmH3Args& g, int epi) -> hipError_t {
    const int p = h->prof_begin(LG_KERNEL_GEMM, st);
    const hipError_t e = gemm_h3(g, epi, st);
    const double R = g.R, K = g.K, O = g.Nout;
    h->prof_end(p, 2.0 * R * K * O, 4.0 * (R * K + O * K + R * O), st);
    if (g.rm.cnt) h->prof_counts(p, 3, 2.0 * K * O, g.rm.cnt, g.rm.sel, g.rm.sel_eq, B, st);
    return e;
  };
  // fp16x3 plane image of a packed weight matrix (by its fp32 offset) / of a workspace tensor
  auto wplanes = [&](GemmH3Args& g, size_t off) {
    const auto& pl = h->planes.at(off);
    g.W = {h->wplanes + pl.off, pl.pstride, pl.rows};
    g.acc_scale = pl.unscale;
  };
  auto image = [&](_Float16* p, int K) { return PlaneRef{p, (long long)RP * K, RP}; };
  auto attn = [&](const AttnSet& a0, const AttnSet& a1, float scale, bool cross, bool q_planes) -> hipError_t {
    const int p = h->prof_begin(LG_KERNEL_ATTENTION, st);
    const hipError_t e = attention_f32(a0, a1, B, H, scale, prec, st, w.apart, w.apart_floats, q_planes);
    // self: 2 matmuls per image (QK^T, PV); cross: one shared sim + two PV (lightglue.py:236-242)
    const double hd = 64.0 * H * B;
    const double fl = cross ? 6.0 * a0.Nq * a0.Nk * hd : 4.0 * hd * ((double)a0.Nq * a0.Nk + (double)a1.Nq * a1.Nk);
    const double by = 4.0 * 256.0 * B * 4.0 * (a0.Nq + a1.Nq);  // q, k, v read + o written, per row
    h->prof_end(p, fl, by, st);
    if (a0.nq_cnt) h->prof_counts(p, cross ? 2 : 1, 64.0 * H, a0.nq_cnt, a0.act, 1, B, st);
    return e;
  };
  auto assign = [&](const AssignArgs& a) -> hipError_t {
    const int p = h->prof_begin(LG_KERNEL_ASSIGN, st);
    const hipError_t e = assign_and_filter(a, st);
    const double mn = (double)a.B * a.M * a.N;
    h->prof_end(p, 0.0, 4.0 * (mn + (a.la ? (double)a.B * (a.M + 1) * (a.N + 1) : 0.0)), st);
    return e;
  };

  // ---- run-time range table (PREC_H3): every plane image written below picks its power-of-two
  // scale on the device from the maxima of its inputs (kernels.h RangeOut), so the fp16 range
  // cannot be exceeded and nothing is read back -- the forward stays asynchronous
  unsigned* rt = prec == PREC_H3 ? w.rtab : nullptr;
  int nslot = 0;
  // a slot is never shared: an exhausted table is an internal error (range_slots() undercounts),
  // reported after the pass instead of silently aliasing two tensors' exponents
  bool slots_overflow = false;
  auto slot = [&]() {
    if (nslot < w.nslots) return nslot++;
    slots_overflow = true;
    return w.nslots - 1;
  };
  auto ro = [&](int in0, float g0, int in1, float g1, float add, int out, int track = 0) {
    return RangeOut{rt, in0, in1, g0, g1, add, out, track};
  };
  if (prec == PREC_H3) LG_HIP(hipMemsetAsync(w.rtab, 0, (size_t)w.nslots * lg::kRangeStride * sizeof(unsigned), st));
  h->pass_started = true;
  int s_x = -1;  // slot of the current residual-stream plane image Xp
  // set when w.X was not initialised from the descriptors: layer 0's self-block ffn.3 reads its
  // residual rows from here (image 0 rows, then image 1 rows)
  const float* res_in0 = nullptr;
  const float* res_in1 = nullptr;
  // ---- input projection (lightglue.py:370-373,486-487); H3 also builds x's plane image
  if (c.input_dim != D) {
    if (prec == PREC_H3) {
      const int din = c.input_dim;
      const float* d0 = in->descriptors0;
      const float* d1 = in->descriptors1;
      if (!din_a16) {  // rows_to_planes reads 16-byte vectors: stage unaligned inputs first
        LG_HIP(hipMemcpyAsync(w.Dst, d0, sizeof(float) * B * M * din, hipMemcpyDeviceToDevice, st));
        LG_HIP(hipMemcpyAsync(w.Dst + (size_t)B * M * din, d1, sizeof(float) * B * N * din, hipMemcpyDeviceToDevice, st));
        d0 = w.Dst;
        d1 = w.Dst + (size_t)B * M * din;
      }
      const int s_in = slot(), s_d = slot();
      s_x = slot();
      LG_HIP(range_absmax2(d0, (size_t)B * M * din, d1, (size_t)B * N * din, rt, s_in, st));
      LG_HIP(rows_to_planes(d0, B * M, din, din, w.Dp, RP, 0, ro(s_in, 1.f, -1, 0.f, 0.f, s_d), st));
      LG_HIP(rows_to_planes(d1, B * N, din, din, w.Dp, RP, B * M, ro(s_in, 1.f, -1, 0.f, 0.f, s_d), st));
      GemmH3Args g = gemm_h3_base();
      g.A0 = image(w.Dp, din); g.K0 = din; g.K = din; wplanes(g, h->Wi); g.rtab = rt; g.a0_slot = s_d;
      g.bias = Wb + h->bi; g.R = B * (M + N); g.Nout = D; g.Y = w.X; g.ldy = D;
      g.Yp = w.Xp; g.yps = (long long)RP * D; g.yrows_pad = RP; g.ro = ro(s_d, h->gi, -1, 0.f, h->bi_max, s_x, 1);
      LG_HIP(gemmh(g, EPI_STORE));
    } else {
      GemmArgs g = gemm_base();
      g.W = Wb + h->Wi; g.ldw = c.input_dim; g.K = c.input_dim; g.K0 = c.input_dim;
      g.bias = Wb + h->bi; g.ldy = D; g.Nout = D;
      g.A0 = in->descriptors0; g.lda0 = c.input_dim; g.R = B * M; g.Y = w.X;
      LG_HIP(gemm(g, EPI_STORE, 1));
      g.A0 = in->descriptors1; g.R = B * N; g.Y = w.X + (size_t)B * M * D;
      LG_HIP(gemm(g, EPI_STORE, 1));
    }
  } else {
    const int s_in = prec == PREC_H3 ? slot() : -1;
    s_x = prec == PREC_H3 ? slot() : -1;
    if (prec == PREC_H3) {
      LG_HIP(range_absmax2(in->descriptors0, (size_t)B * M * D, in->descriptors1, (size_t)B * N * D, rt, s_in, st));
    }
    if (prec == PREC_H3 && din_a16 && L > 0) {
      // the plane image from one read of the descriptors; the fp32 residual stream w.X is first
      // written by layer 0's self-block ffn.3, which reads its residual from the descriptors
      // themselves (res_in) -- no copy; with pruning / early stop every row of layer 0 is live
#if LG_MERGE_R2P
      LG_HIP(rows_to_planes2(in->descriptors0, B * M, in->descriptors1, B * N, D, D, w.Xp, RP, 0,
                             ro(s_in, 1.f, -1, 0.f, 0.f, s_x, 1), st));
#else
      LG_HIP(rows_to_planes(in->descriptors0, B * M, D, D, w.Xp, RP, 0, ro(s_in, 1.f, -1, 0.f, 0.f, s_x, 1), st));
      LG_HIP(rows_to_planes(in->descriptors1, B * N, D, D, w.Xp, RP, B * M, ro(s_in, 1.f, -1, 0.f, 0.f, s_x, 1), st));
#endif
      res_in0 = in->descriptors0;
      res_in1 = in->descriptors1;
    } else {
      LG_HIP(hipMemcpyAsync(w.X, in->descriptors0, sizeof(float) * B * M * D, hipMemcpyDeviceToDevice, st));
      LG_HIP(hipMemcpyAsync(w.X + (size_t)B * M * D, in->descriptors1, sizeof(float) * B * N * D, hipMemcpyDeviceToDevice, st));
      if (prec == PREC_H3) LG_HIP(rows_to_planes(w.X, B * (M + N), D, D, w.Xp, RP, 0, ro(s_in, 1.f, -1, 0.f, 0.f, s_x, 1), st));
    }
  }

  // ---- keypoint normalisation + positional encoding (lightglue.py:455-456,490-494)
  {
    const float* s0 = in->image_size0;
    const float* s1 = in->image_size1;
    if (!s0) { LG_HIP(kpt_extent(in->keypoints0, B, M, w.size, st)); s0 = w.size; }
    if (!s1) { LG_HIP(kpt_extent(in->keypoints1, B, N, w.size + 2 * B, st)); s1 = w.size + 2 * B; }
    PEArgs p;
    p.Wr = Wb + h->Wr; p.Wc = Wb + h->Wc; p.bc = Wb + h->bc; p.m_in = c.add_scale_ori ? 4 : 2; p.B = B;
    p.kpts = in->keypoints0; p.size = s0; p.scales = in->scales0; p.oris = in->oris0; p.n = M;
    p.cosb = w.cosb; p.sinb = w.sinb;
    PEArgs p1 = p;
    p1.kpts = in->keypoints1; p1.size = s1; p1.scales = in->scales1; p1.oris = in->oris1; p1.n = N;
    p1.cosb = w.cosb + (size_t)B * M * 32; p1.sinb = w.sinb + (size_t)B * M * 32;
#if LG_MERGE_PE
    LG_HIP(positional_encoding2(p, p1, st));
#else
    LG_HIP(positional_encoding(p, st));
    LG_HIP(positional_encoding(p1, st));
#endif
  }

  // ---- early stop / point pruning for any batch size, counts on the device (kernels.h
  // SegLayout): each (image, pair) keeps a fixed slot whose kept points are a compacted prefix;
  // GEMMs skip dead rows, the attention reads per-pair counts, a stopped pair is frozen
  const bool seg = do_stop || do_prune;
  const SegLayout SL{B, M0, N0};
  int* cnt = w.cnt;
  int* cntb = w.cntb;
  int* ind = w.ind;
  int* indb = w.indb;
  RowMask live{};  // cnt == null outside pruning: every row live
  if (seg) {
    LG_HIP(prune_init(SL, cnt, w.act, w.stop, L, ind, st));
    live = RowMask{cnt, w.act, 1, SL};
  }
  if (out->prune0) LG_HIP(fill_i64(out->prune0, do_prune ? 1 : L, (size_t)B * M0, st));
  if (out->prune1) LG_HIP(fill_i64(out->prune1, do_prune ? 1 : L, (size_t)B * N0, st));

  const float thr_w = (float)(1.0 - c.width_confidence);  // python-float arithmetic, then fp32 compare
  const int R = B * (M + N);
  // the last layer's ffn.3 writes the final descriptors straight into ref_descriptors0/1 (no copy)
  // when every pair runs every layer and nothing reads the fp32 stream after it
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool direct_out = prec == PREC_H3 && !seg && !do_stop && !do_prune && out->ref_descriptors0 &&
                          out->ref_descriptors1 && a16(out->ref_descriptors0) && a16(out->ref_descriptors1) &&
                          !out->layer_descriptors0 && !out->layer_descriptors1;
  for (int i = 0; i < L; ++i) {
    const LayerW& lw = h->layers[i];
    for (int blk = 0; blk < 2; ++blk) {
      const BlockW& bw = blk == 0 ? lw.self : lw.cross;
      // QKV projection with fused rotary (self) / scale (cross) and head-major scatter
      HeadLayout hl;
      hl.B = B; hl.H = H; hl.M = M; hl.N = N; hl.cosb = w.cosb; hl.sinb = w.sinb;
      // the cross block's qk goes out only as planes in fp16x3 (the attention reads its queries
      // from them: attention_f32's q_planes); self q and every bf16x6 query stay fp32 rows
      const bool q_planes = prec == PREC_H3 && blk == 1;
      hl.q = q_planes ? nullptr : w.Q; hl.kp = w.KP; hl.vp = w.VP; hl.pstride = (long long)w.R * D;
      hl.qk_scale = std::sqrt(1.f / std::sqrt(64.f));  // scale**0.5 (lightglue.py:235)
      const int epi_qkv = blk == 0 ? EPI_QKV_ROT : EPI_CROSS_QKV;
      const lg_handle::BlockGain& gn = h->gains[(size_t)i * 2 + blk];
      const int s_k = slot(), s_v = slot();
      if (prec == PREC_H3) {
        GemmH3Args g = gemm_h3_base();
        g.A0 = image(w.Xp, D); g.K0 = D; g.K = D; wplanes(g, bw.Wqkv); g.bias = Wb + bw.bqkv;
        g.rtab = rt; g.a0_slot = s_x; g.rm = live;
        g.ro = ro(s_x, gn.gK, -1, 0.f, gn.bK, s_k, 1);  // M[k]: the attention's exact-softmax test
        g.ro_v = ro(s_x, gn.gV, -1, 0.f, gn.bV, s_v, kRangeTwoSided | (h->fold ? 0 : kRangeTrack));
        g.R = R; g.Nout = blk == 0 ? 3 * D : 2 * D; g.hl = hl;
        LG_HIP(gemmh(g, epi_qkv));
      } else {
        GemmArgs g = gemm_base();
        g.A0 = w.X; g.lda0 = D; g.K0 = D; g.K = D; g.W = Wb + bw.Wqkv; g.ldw = D; g.bias = Wb + bw.bqkv;
        g.R = R; g.Nout = blk == 0 ? 3 * D : 2 * D; g.hl = hl; g.rm = live;
        LG_HIP(gemm(g, epi_qkv, 1));
      }
      const size_t img1 = (size_t)B * H * M * 64;
      const long long ps = (long long)w.R * D;
      AttnSet a0, a1;
      // planes are 2-byte elements in both formats (bf16 / fp16)
      const void* kp1 = static_cast<const char*>(w.KP) + 2 * img1;
      const void* vp1 = static_cast<const char*>(w.VP) + 2 * img1;
      float* ctx1 = w.ctx + (size_t)B * M * D;
      // per-pair counts of a pruned batch: image 0 = cnt[0..B), image 1 = cnt[B..2B)
      const int* c0 = seg ? cnt : nullptr;
      const int* c1 = seg ? cnt + B : nullptr;
      const int* act = seg ? w.act : nullptr;
      if (blk == 0) {  // self: q/k/v of the same image, scale 1/sqrt(64) (SDPA default)
        a0 = {w.Q, w.KP, w.VP, ps, w.ctx, M, M, w.Cp, (long long)RP * D, RP, 0, rt, s_k, c0, c0, act};
        a1 = {w.Q + img1, kp1, vp1, ps, ctx1, N, N, w.Cp, (long long)RP * D, RP, B * M, rt, s_k, c1, c1, act};
      } else {  // cross: qk as planes in w.KP (fp16x3: also the queries; bf16x6: fp32 in w.Q), v planes in w.VP
        a0 = {w.Q, kp1, vp1, ps, w.ctx, M, N, w.Cp, (long long)RP * D, RP, 0, rt, s_k, c0, c1, act};
        a1 = {w.Q + img1, w.KP, w.VP, ps, ctx1, N, M, w.Cp, (long long)RP * D, RP, B * M, rt, s_k, c1, c0, act};
        if (q_planes) {  // the queries are the qk planes (the key planes of the other direction)
          a0.q = w.KP;
          a1.q = kp1;
        }
      }
      LG_HIP(attn(a0, a1, blk == 0 ? 0.125f : 1.0f, blk == 1, q_planes));
      if (prec == PREC_H3) {
        // out projection (skipped when folded into ffn.0 at load time: ffn.0 then reads ctx)
        // the context planes carry the value planes' exponent (attention.hip)
        int s_msg = s_v;
        if (!h->fold) {
          s_msg = slot();
          GemmH3Args g = gemm_h3_base();
          g.A0 = image(w.Cp, D); g.K0 = D; g.K = D; wplanes(g, bw.Wo); g.bias = Wb + bw.bo;
          g.rtab = rt; g.a0_slot = s_v; g.ro = ro(s_v, gn.go, -1, 0.f, gn.bo, s_msg); g.rm = live;
          g.R = R; g.Nout = D; g.Yp = w.Mp; g.yps = (long long)RP * D; g.yrows_pad = RP;
          LG_HIP(gemmh(g, EPI_STORE));
        }
        // FFN: Linear(cat[x, msg]) -> LN -> GELU (one kernel: the activations leave only as the
        // plane image ffn.3 consumes) -> Linear + residual (x also as plane image)
        GemmH3Args g = gemm_h3_base();
        g.A0 = image(w.Xp, D); g.K0 = D; g.A1 = image(h->fold ? w.Cp : w.Mp, D); g.K = 2 * D;
        wplanes(g, bw.W1); g.bias = Wb + bw.b1; g.R = R; g.Nout = 2 * D;
        g.rtab = rt; g.a0_slot = s_x; g.a1_slot = s_msg; g.rm = live;
        const int s_h = slot();
        const RangeOut ro_h = ro(-1, 0.f, -1, 0.f, gn.hb, s_h);
        if (gemm_h3_ln_split(R)) {  // small R: 64x64-tile GEMM into H1, then the LN + GELU row kernel
          g.Y = w.H1; g.ldy = 2 * D;
          LG_HIP(gemmh(g, EPI_STORE));
          LG_HIP(layernorm_gelu_512(w.H1, Wb + bw.g, Wb + bw.be, R, w.Hp, RP, ro_h, st));
        } else {
          g.Yp = w.Hp; g.yps = (long long)RP * 2 * D; g.yrows_pad = RP; g.ln_g = Wb + bw.g; g.ln_b = Wb + bw.be;
          g.ro = ro_h;
          LG_HIP(gemmh(g, EPI_LN_GELU));
        }
        const int s_xn = slot();
        g = gemm_h3_base();
        g.A0 = image(w.Hp, 2 * D); g.K0 = 2 * D; g.K = 2 * D; wplanes(g, bw.W2); g.bias = Wb + bw.b2;
        g.rtab = rt; g.a0_slot = s_h; g.rm = live;  // frozen / dead rows keep their residual stream
        g.R = R; g.Nout = D; g.Y = w.X; g.ldy = D; g.res = w.X; g.ldr = D;
        if (res_in0) {  // the first ffn.3: the residual is the input descriptors (never copied into w.X)
          g.res = res_in0;
          g.res2 = res_in1;
          g.res2_row0 = B * M;
          res_in0 = res_in1 = nullptr;
        }
        g.reverse = h->ffn3_reverse;  // read the hidden planes the LN GEMM wrote last first
        if (direct_out && i == L - 1 && blk == 1) {  // the final descriptors straight into the outputs
          g.Y = out->ref_descriptors0;
          g.Y2 = out->ref_descriptors1;
          g.y2_row0 = B * M;
        }
        g.Yp = w.Xp; g.yps = (long long)RP * D; g.yrows_pad = RP;
        g.ro = ro(s_x, 1.f, -1, 0.f, gn.g2 * gn.hb + gn.b2, s_xn, 1);  // |x + ffn(..)| <= M_x + |W2|_1 hb + |b2|
        LG_HIP(gemmh(g, EPI_STORE));
        s_x = s_xn;
      } else {
        if (!h->fold) {
          GemmArgs g = gemm_base();
          g.A0 = w.ctx; g.lda0 = D; g.K0 = D; g.K = D; g.W = Wb + bw.Wo; g.ldw = D; g.bias = Wb + bw.bo;
          g.R = R; g.Nout = D; g.Y = w.msg; g.ldy = D; g.rm = live;
          LG_HIP(gemm(g, EPI_STORE, 1));
        }
        GemmArgs g = gemm_base();
        g.A0 = w.X; g.lda0 = D; g.K0 = D; g.A1 = h->fold ? w.ctx : w.msg; g.lda1 = D; g.K = 2 * D;
        g.W = Wb + bw.W1; g.ldw = 2 * D; g.bias = Wb + bw.b1; g.R = R; g.Nout = 2 * D; g.Y = w.H1; g.ldy = 2 * D;
        g.rm = live;
        LG_HIP(gemm(g, EPI_STORE, 1));
        LG_HIP(layernorm_gelu_512(w.H1, Wb + bw.g, Wb + bw.be, R, nullptr, 0, range_none(), st));
        g = gemm_base();
        g.A0 = w.H1; g.lda0 = 2 * D; g.K0 = 2 * D; g.K = 2 * D; g.W = Wb + bw.W2; g.ldw = 2 * D; g.bias = Wb + bw.b2;
        g.R = R; g.Nout = D; g.Y = w.X; g.ldy = D; g.res = w.X; g.ldr = D; g.rm = live;
        LG_HIP(gemm(g, EPI_STORE, 1));
      }
    }
    // training-mode outputs: every layer's descriptors (lightglue.py:521-524)
    for (int s2 = 0; s2 < 2; ++s2) {
      float* dst = s2 == 0 ? out->layer_descriptors0 : out->layer_descriptors1;
      if (!dst) continue;
      const int n = s2 == 0 ? M : N;
      const size_t row = sizeof(float) * (size_t)n * D;
      LG_HIP(hipMemcpy2DAsync(reinterpret_cast<char*>(dst) + row * i, row * L, w.X + (s2 == 0 ? 0 : (size_t)B * M * D),
                              row, row, B, hipMemcpyDeviceToDevice, st));
    }
    if (i == L - 1) break;

    // ---- early stop (lightglue.py:527-531, check_if_stop :595-606; thresholds per :581-584),
    // decided per pair on the device
    const float thr_c = confidence_threshold(i, L);
    if (do_stop) {
      LG_HIP(gemv_256(w.X, Wb + lw.wt, Wb + lw.bt, w.tok, R, 1, st));
      LG_HIP(stop_decide(w.tok, cnt, w.act, w.stop, SL, thr_c, (float)c.depth_confidence, i, st));
    }
    // ---- width pruning (lightglue.py:532-547, get_pruning_mask :586-593), compaction inside each
    // pair's slot; a pair that stopped at this layer keeps every point (the reference breaks first)
    if (do_prune) {
      LG_HIP(gemv_256(w.X, Wb + lw.wm, Wb + lw.bm, w.z, R, 0, st));
      LG_HIP(prune_scan(w.z, do_stop ? w.tok : nullptr, cnt, cntb, w.act, w.flags, w.pos, SL, thr_w, thr_c, st));
      LG_HIP(compact_seg(w.X, w.X2, D, w.flags, w.pos, cnt, SL, st));
      LG_HIP(compact_seg(w.cosb, w.cos2, 32, w.flags, w.pos, cnt, SL, st));
      LG_HIP(compact_seg(w.sinb, w.sin2, 32, w.flags, w.pos, cnt, SL, st));
      LG_HIP(compact_ind_seg(ind, indb, out->prune0, out->prune1, w.flags, w.pos, cnt, w.act, SL, st));
      std::swap(w.X, w.X2);
      std::swap(w.cosb, w.cos2);
      std::swap(w.sinb, w.sin2);
      std::swap(ind, indb);
      std::swap(cnt, cntb);
      live = RowMask{cnt, w.act, 1, SL};
      if (prec == PREC_H3) {
        const int s_c = slot();
        const RowMask kept{cnt, nullptr, 0, SL};  // every kept row (frozen pairs too)
        LG_HIP(rows_to_planes(w.X, R, D, D, w.Xp, RP, 0, ro(s_x, 1.f, -1, 0.f, 0.f, s_c, 1), st, nullptr, &kept));
        s_x = s_c;
      }
    }
  }
  out->precision_used = prec;
  if (slots_overflow) return fail(LG_E_INTERNAL, "range table exhausted (internal: range_slots undercounts)");

  // ---- assignment head of each pair's last executed layer (lightglue.py:549-551,
  // MatchAssignment :306-315): one final_proj / matchability launch per layer a pair may have
  // stopped at (rows of the other pairs are masked out)
  // fused assignment (assign_h3.hip): the similarity is recomputed from md's plane image, held
  // to |md| <= 16 (the "y" side of the fp16x3 product), instead of a bf16x6 GEMM into w.sim
  // a caller that wants the similarity (lg_outputs_t.similarity) gets it from the materialised
  // bf16x6 GEMM, written straight into its buffer
  const bool fused_sim = prec == PREC_H3 && !seg && sim_h3_supported(M, N) && !out->similarity;
  float* simbuf = out->similarity ? out->similarity : w.sim;
  const int md_rows_pad = RP + 256;
  const int s_md = fused_sim ? slot() : -1;
  auto head = [&](int li, const RowMask& m) -> int {
    const LayerW& la = h->layers[li];
    if (prec == PREC_H3) {
      GemmH3Args g = gemm_h3_base();
      g.A0 = image(w.Xp, D); g.K0 = D; g.K = D; wplanes(g, la.Wf); g.bias = Wb + la.bf;
      g.rtab = rt; g.a0_slot = s_x; g.rm = m;
      g.R = R; g.Nout = D; g.Y = w.md; g.ldy = D; g.out_scale = 0.25f;  // / d**0.25
      if (fused_sim) {
        g.Y = nullptr;
        g.Yp = w.mdp; g.yps = (long long)md_rows_pad * D; g.yrows_pad = md_rows_pad;
        g.ro = RangeOut{rt, s_x, -1, 0.25f * h->gf[li], 0.f, 0.25f * h->bf_max[li], s_md, 0, 11};
      }
      LG_HIP(gemmh(g, EPI_STORE));
    } else {
      GemmArgs g = gemm_base();
      g.A0 = w.X; g.lda0 = D; g.K0 = D; g.K = D; g.W = Wb + la.Wf; g.ldw = D; g.bias = Wb + la.bf;
      g.R = R; g.Nout = D; g.Y = w.md; g.ldy = D; g.out_scale = 0.25f; g.rm = m;  // / d**0.25
      LG_HIP(gemm(g, EPI_STORE, 1));
    }
    if (direct_out) {  // the final fp32 descriptors live in the outputs (every row live)
#if LG_MERGE_GEMV
      LG_HIP(gemv_256_masked2(out->ref_descriptors0, B * M, out->ref_descriptors1, B * N, Wb + la.wm, Wb + la.bm, w.z, m,
                              st));
#else
      LG_HIP(gemv_256_masked(out->ref_descriptors0, Wb + la.wm, Wb + la.bm, w.z, B * M, m, st));
      LG_HIP(gemv_256_masked(out->ref_descriptors1, Wb + la.wm, Wb + la.bm, w.z + (size_t)B * M, B * N, m, st));
#endif
    } else {
      LG_HIP(gemv_256_masked(w.X, Wb + la.wm, Wb + la.bm, w.z, R, m, st));
    }
    return LG_OK;
  };
  if (do_stop) {
    for (int li = 0; li < L; ++li) {
      const int rc = head(li, RowMask{cnt, w.stop, li, SL});
      if (rc != LG_OK) return rc;
    }
  } else {
    const int rc = head(L - 1, seg ? RowMask{cnt, nullptr, 0, SL} : RowMask{});
    if (rc != LG_OK) return rc;
  }
  if (!fused_sim) {
    // similarity: both operands are run-time values -> bf16x6 (full fp32 range); per pair over
    // the slot capacities (the assignment bounds everything by the kept counts)
    GemmArgs g = gemm_base();
    g.A0 = w.md; g.lda0 = D; g.K0 = D; g.K = D; g.sA = (long long)M * D;
    g.W = w.md + (size_t)B * M * D; g.ldw = D; g.sW = (long long)N * D;
    g.R = M; g.Nout = N; g.Y = simbuf; g.ldy = N; g.sY = (long long)M * N;
    LG_HIP(gemm(g, EPI_STORE, B));
  }
  if (rt && getenv("LG_DEBUG_RANGE")) {  // diagnostic: the range table of this forward
    std::vector<unsigned> tab((size_t)nslot * lg::kRangeStride);
    LG_HIP(hipMemcpyAsync(tab.data(), rt, tab.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    LG_HIP(hipStreamSynchronize(st));
    for (int k = 0; k < nslot; ++k) {
      float m = 0.f;
      for (int j = 0; j < lg::kRangeShards; ++j) {
        float v;
        memcpy(&v, &tab[(size_t)k * lg::kRangeStride + j], 4);
        m = std::max(m, v);
      }
      fprintf(stderr, "range slot %d: max %.4g exp %d\n", k, m, (int)tab[(size_t)k * lg::kRangeStride + lg::kRangeShards]);
    }
  }
  if (slots_overflow) return fail(LG_E_INTERNAL, "range table exhausted (internal: range_slots undercounts)");
  AssignArgs aa;
  memset(&aa, 0, sizeof(aa));
  aa.sim = simbuf; aa.z0 = w.z; aa.z1 = w.z + (size_t)B * M; aa.la = out->log_assignment; aa.ws = w.aws;
  aa.B = B; aa.M = M; aa.N = N; aa.th = (float)c.filter_threshold;
  if (seg) {  // per-pair kept counts; la holds pair b's [M_b+1][N_b+1] block at the capacity strides
    aa.Mb = cnt;
    aa.Nb = cnt + B;
  }
  if (do_prune) {
    aa.m0 = w.m0c; aa.m1 = w.m1c; aa.s0 = w.s0c; aa.s1 = w.s1c;
    LG_HIP(assign(aa));
    LG_HIP(remap_seg(w.m0c, w.m1c, w.s0c, w.s1c, ind, cnt, SL, out->matches0, out->matches1, out->matching_scores0,
                     out->matching_scores1, st));
  } else {
    aa.m0 = out->matches0; aa.m1 = out->matches1; aa.s0 = out->matching_scores0; aa.s1 = out->matching_scores1;
    if (fused_sim) {
      const int p = h->prof_begin(LG_KERNEL_ASSIGN, st);
      LG_HIP(assign_and_filter_h3(aa, PlaneRef{w.mdp, (long long)md_rows_pad * D, md_rows_pad}, rt, s_md, st));
      // two similarity GEMMs; HBM: the la write (the similarity is never stored)
      h->prof_end(p, 2.0 * 2.0 * B * M * N * D, aa.la ? 4.0 * B * (M + 1) * (N + 1) : 0.0, st);
    } else {
      LG_HIP(assign(aa));
    }
  }
  if (out->ref_descriptors0 && !direct_out)
    LG_HIP(hipMemcpyAsync(out->ref_descriptors0, w.X, sizeof(float) * B * M * D, hipMemcpyDeviceToDevice, st));
  if (out->ref_descriptors1 && !direct_out)
    LG_HIP(hipMemcpyAsync(out->ref_descriptors1, w.X + (size_t)B * M * D, sizeof(float) * B * N * D,
                          hipMemcpyDeviceToDevice, st));
  // kept counts and stop layers: on the device for the caller, and (one read-back, the only
  // synchronisation of a pruning forward) as host outs
  out->stop_layer = L - 1;
  out->kept0 = M;
  out->kept1 = N;
  if (seg) {
    if (out->kept) LG_HIP(hipMemcpyAsync(out->kept, cnt, 2 * B * sizeof(int), hipMemcpyDeviceToDevice, st));
    if (out->stop) LG_HIP(hipMemcpyAsync(out->stop, w.stop, B * sizeof(int), hipMemcpyDeviceToDevice, st));
    std::vector<int> hc(3 * (size_t)B);
    LG_HIP(hipMemcpyAsync(hc.data(), cnt, 2 * B * sizeof(int), hipMemcpyDeviceToHost, st));
    LG_HIP(hipMemcpyAsync(hc.data() + 2 * B, w.stop, B * sizeof(int), hipMemcpyDeviceToHost, st));
    LG_HIP(hipStreamSynchronize(st));
    out->kept0 = hc[0];
    out->kept1 = hc[B];
    out->stop_layer = hc[2 * B];
    for (int k = 0; k < 2 * B; ++k)
      if (hc[k] == 0)  // the reference's filter_matches fails on the empty set the same way
        return fail(LG_E_INVALID, "max(): Expected reduction dim to have non-zero size (all keypoints pruned)");
  }
  return LG_OK;
}

int lg_forward(lg_handle_t* h, const lg_inputs_t* in, lg_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream) {
  if (!h || !in || !out) return fail(LG_E_INVALID, "null argument");
  // fp16x3 needs no guard or rerun: run-time operands are range-scaled on the device
  return forward_pass(h, in, out, workspace, workspace_bytes, stream,
                      h->cfg.precision == LG_PREC_X6 ? lg::PREC_X6 : lg::PREC_H3);
}

// ---- MatchAssignment of one layer on caller descriptors (lightglue.py:306-315 + :284-296); the
// training loss evaluates it on every layer's descriptors (:614-620).  Not a hot path: bf16x6
// GEMMs straight from the fp32 rows (no plane images, no range table), the materialised similarity
// and the unfused assignment kernels of the pruning path.
namespace {
struct HeadWork {
  float *md, *z, *sim, *aws, *s0, *s1;
  int64_t *m0, *m1;
  size_t bytes;
};
HeadWork carve_head(char* base, int B, int M, int N) {
  HeadWork w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~size_t(255);
    return p;
  };
  const size_t R = (size_t)B * (M + N);
  w.md = reinterpret_cast<float*>(take(R * D * 4));
  w.z = reinterpret_cast<float*>(take(R * 4));
  w.sim = reinterpret_cast<float*>(take((size_t)B * M * N * 4));
  w.aws = reinterpret_cast<float*>(take((lg::assign_workspace_floats(B, M, N) + 64) * 4));
  w.s0 = reinterpret_cast<float*>(take((size_t)B * M * 4));
  w.s1 = reinterpret_cast<float*>(take((size_t)B * N * 4));
  w.m0 = reinterpret_cast<int64_t*>(take((size_t)B * M * 8));
  w.m1 = reinterpret_cast<int64_t*>(take((size_t)B * N * 8));
  w.bytes = off;
  return w;
}
}  // namespace

int lg_assignment_workspace_bytes(const lg_handle_t* h, int32_t B, int32_t M, int32_t N, size_t* bytes) {
  if (!h || !bytes || B < 0 || M < 0 || N < 0) return fail(LG_E_INVALID, "bad argument");
  *bytes = carve_head(nullptr, B, M, N).bytes;
  return LG_OK;
}

int lg_assignment_head(lg_handle_t* h, int32_t layer, const float* desc0, const float* desc1, int32_t B, int32_t M,
                       int32_t N, float* log_assignment, float* similarity, float* token_logits0, float* token_logits1,
                       void* workspace, size_t workspace_bytes, void* stream) {
  using namespace lg;
  if (!h || !desc0 || !desc1 || !log_assignment) return fail(LG_E_INVALID, "null argument");
  if (!h->loaded) return fail(LG_E_WEIGHTS, "weights not loaded");
  const int L = h->cfg.n_layers;
  if (layer < 0) layer += L;  // python-style index: -1 = the last layer's head
  if (layer < 0 || layer >= L) return fail(LG_E_INVALID, "layer index out of range");
  if ((token_logits0 || token_logits1) && layer >= L - 1)
    return fail(LG_E_INVALID, "token_confidence exists for layers 0..n_layers-2 only (lightglue.py:395-397)");
  if (B <= 0) return fail(LG_E_INVALID, "batch must be >= 1");
  if (M <= 0 || N <= 0) return fail(LG_E_INVALID, "max(): Expected reduction dim to have non-zero size (empty keypoint set)");
  const HeadWork need = carve_head(nullptr, B, M, N);
  if (!workspace || workspace_bytes < need.bytes) return fail(LG_E_WORKSPACE, "workspace too small: need " + std::to_string(need.bytes));
  LG_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  HeadWork w = carve_head((char*)workspace, B, M, N);
  const float* Wb = h->wbuf;
  const LayerW& lw = h->layers[layer];
  float* sim = similarity ? similarity : w.sim;
  // md = final_proj(desc) / d**0.25 (:308-310), per image
  for (int s2 = 0; s2 < 2; ++s2) {
    GemmArgs g = gemm_base();
    g.A0 = s2 == 0 ? desc0 : desc1; g.lda0 = D; g.K0 = D; g.K = D; g.W = Wb + lw.Wf; g.ldw = D; g.bias = Wb + lw.bf;
    g.R = B * (s2 == 0 ? M : N); g.Nout = D; g.Y = w.md + (s2 == 0 ? 0 : (size_t)B * M * D); g.ldy = D;
    g.out_scale = 0.25f;
    LG_HIP(gemm_x6(g, EPI_STORE, 1, st));
  }
  // matchability logits z (:314) and, for the loss, the token-confidence logits (:109-110)
  LG_HIP(gemv_256(desc0, Wb + lw.wm, Wb + lw.bm, w.z, B * M, 0, st));
  LG_HIP(gemv_256(desc1, Wb + lw.wm, Wb + lw.bm, w.z + (size_t)B * M, B * N, 0, st));
  if (token_logits0) LG_HIP(gemv_256(desc0, Wb + lw.wt, Wb + lw.bt, token_logits0, B * M, 0, st));
  if (token_logits1) LG_HIP(gemv_256(desc1, Wb + lw.wt, Wb + lw.bt, token_logits1, B * N, 0, st));
  // sim = md0 md1^T (:311), per pair
  {
    GemmArgs g = gemm_base();
    g.A0 = w.md; g.lda0 = D; g.K0 = D; g.K = D; g.sA = (long long)M * D;
    g.W = w.md + (size_t)B * M * D; g.ldw = D; g.sW = (long long)N * D;
    g.R = M; g.Nout = N; g.Y = sim; g.ldy = N; g.sY = (long long)M * N;
    LG_HIP(gemm_x6(g, EPI_STORE, B, st));
  }
  // sigmoid_log_double_softmax (:284-296); the filter outputs go to scratch
  AssignArgs aa;
  memset(&aa, 0, sizeof(aa));
  aa.sim = sim; aa.z0 = w.z; aa.z1 = w.z + (size_t)B * M; aa.la = log_assignment; aa.ws = w.aws;
  aa.B = B; aa.M = M; aa.N = N; aa.th = (float)h->cfg.filter_threshold;
  aa.m0 = w.m0; aa.m1 = w.m1; aa.s0 = w.s0; aa.s1 = w.s1;
  LG_HIP(assign_and_filter(aa, st));
  return LG_OK;
}

int lg_profile_enable(lg_handle_t* h, int enable) {
  if (!h) return fail(LG_E_INVALID, "null handle");
  for (auto& r : h->recs) {
    h->pool.push_back(r.a);
    h->pool.push_back(r.b);
  }
  h->recs.clear();
  h->snap_used = 0;
  h->prof_on = enable != 0;
  if (h->prof_on && !h->snap) {  // live-count snapshots of pruned forwards (lg_profile_read)
    LG_HIP(hipSetDevice(h->device));
    LG_HIP(hipMalloc((void**)&h->snap, (1u << 20) * sizeof(int)));
    h->snap_cap = 1u << 20;
  }
  // 1 = every family; otherwise bit (k + 1) selects family k (LG_PROFILE_ONLY(k))
  h->prof_mask = enable == 1 ? ~0u : ((unsigned)enable >> 1);
  return LG_OK;
}

int lg_profile_read(lg_handle_t* h, int kernel, double* total_ms, int64_t* launches, double* flops, double* bytes) {
  if (!h || kernel < 0 || kernel >= LG_KERNEL_COUNT) return fail(LG_E_INVALID, "bad argument");
  double ms = 0.0, fl = 0.0, by = 0.0;
  int64_t n = 0;
  std::vector<int> snap;
  // the snapshot copies (prof_counts) are queued after their record's end event, on whatever
  // stream the forward ran: wait for the device before reading them (profiling reads only)
  for (auto& r : h->recs)
    if (r.snap >= 0) {
      LG_HIP(hipSetDevice(h->device));
      LG_HIP(hipDeviceSynchronize());
      break;
    }
  for (auto& r : h->recs) {
    if (r.kind != kernel) continue;
    LG_HIP(hipEventSynchronize(r.b));
    float t = 0.f;
    LG_HIP(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    double f = r.flops;
    if (r.snap >= 0) {  // pruned forward: flops over the live rows / kept points at launch time
      if (snap.empty()) {
        snap.resize(h->snap_used);
        LG_HIP(hipMemcpy(snap.data(), h->snap, h->snap_used * sizeof(int), hipMemcpyDeviceToHost));
      }
      const int* c = snap.data() + r.snap;
      const int* sel = r.has_sel ? c + 2 * r.B : nullptr;
      f = 0.0;
      for (int b = 0; b < r.B; ++b) {
        if (sel && sel[b] != r.sel_eq) continue;
        const double c0 = c[b], c1 = c[r.B + b];
        if (r.mode == 1) f += 4.0 * r.unit * (c0 * c0 + c1 * c1);
        else if (r.mode == 2) f += 6.0 * r.unit * c0 * c1;
        else f += r.unit * (c0 + c1);
      }
    }
    fl += f;
    by += r.bytes;
    ++n;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = n;
  if (flops) *flops = fl;
  if (bytes) *bytes = by;
  return LG_OK;
}

int lg_filter_workspace_bytes(int32_t B, int32_t M, int32_t N, size_t* bytes) {
  if (!bytes) return fail(LG_E_INVALID, "null argument");
  *bytes = lg::filter_workspace_floats(B, M, N) * sizeof(float);
  return LG_OK;
}

int lg_filter_matches(const float* scores, int32_t B, int32_t M, int32_t N, double threshold, int64_t* m0, int64_t* m1,
                      float* s0, float* s1, void* workspace, size_t workspace_bytes, void* stream) {
  if (!scores || !m0 || !m1 || !s0 || !s1) return fail(LG_E_INVALID, "null argument");
  if (B <= 0 || M <= 0 || N <= 0) return fail(LG_E_INVALID, "max(): Expected reduction dim to have non-zero size");
  if (!workspace || workspace_bytes < lg::filter_workspace_floats(B, M, N) * sizeof(float))
    return fail(LG_E_WORKSPACE, "workspace too small");
  LG_HIP(lg::filter_from_scores(scores, B, M, N, (float)threshold, (float*)workspace, m0, m1, s0, s1, (hipStream_t)stream));
  return LG_OK;
}

int lg_sinkhorn_workspace_bytes(int32_t B, int32_t M, int32_t N, size_t* bytes) {
  if (!bytes) return fail(LG_E_INVALID, "null argument");
  *bytes = lg::sinkhorn_workspace_floats(B, M, N) * sizeof(float);
  return LG_OK;
}

int lg_log_optimal_transport(const float* scores, float alpha, int32_t B, int32_t M, int32_t N, int32_t iters, float* Z,
                             void* workspace, size_t workspace_bytes, void* stream) {
  if (!scores || !Z) return fail(LG_E_INVALID, "null argument");
  if (B < 0 || M < 0 || N < 0 || iters < 0) return fail(LG_E_INVALID, "bad shape");
  if (!workspace || workspace_bytes < lg::sinkhorn_workspace_floats(B, M, N) * sizeof(float))
    return fail(LG_E_WORKSPACE, "workspace too small");
  LG_HIP(lg::log_optimal_transport(scores, alpha, B, M, N, iters, Z, (float*)workspace, (hipStream_t)stream));
  return LG_OK;
}

namespace {
size_t attention_ws(int B, int H, int Nq, int Nk, size_t& kv_off, size_t& img_off, int& rp, size_t* part_off = nullptr) {
  const size_t n = (size_t)B * H * Nk * 64;
  rp = (int)(((size_t)B * Nq + 255) / 256 * 256);
  kv_off = 4 * 32 * 4;  // [range table (4 slots) | k planes (3 max) | v planes | ctx image | key-split partials]
  img_off = kv_off + 2 * 3 * n * 2;
  const size_t po = img_off + (size_t)2 * rp * 256 * 2;
  if (part_off) *part_off = po;
  return po + lg::attention_split_floats(B, H, Nq, Nk) * sizeof(float);
}
}  // namespace

int lg_attention_workspace_bytes(int32_t B, int32_t H, int32_t Nq, int32_t Nk, size_t* bytes) {
  if (!bytes || B < 0 || H <= 0 || Nq < 0 || Nk < 0) return fail(LG_E_INVALID, "bad argument");
  size_t kv, img;
  int rp;
  *bytes = attention_ws(B, H, Nq, Nk, kv, img, rp);
  return LG_OK;
}

int lg_attention(const float* q, const float* k, const float* v, int32_t B, int32_t H, int32_t Nq, int32_t Nk,
                 float scale, int32_t precision, float* ctx, void* workspace, size_t workspace_bytes, void* stream) {
  if (!q || !k || !v || !ctx) return fail(LG_E_INVALID, "null argument");
  if (H * 64 != 256 || B < 0 || Nq < 0 || Nk <= 0) return fail(LG_E_INVALID, "bad shape (H * 64 must be 256, Nk > 0)");
  size_t kv_off, img_off, part_off;
  int rp;
  const size_t need = attention_ws(B, H, Nq, Nk, kv_off, img_off, rp, &part_off);
  if (!workspace || workspace_bytes < need) return fail(LG_E_WORKSPACE, "workspace too small");
  if (B == 0 || Nq == 0) return LG_OK;
  hipStream_t st = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  unsigned* rtab = reinterpret_cast<unsigned*>(ws);  // slots 0/1: max|k|, max|v|; 2/3: k, v planes
  const size_t n = (size_t)B * H * Nk * 64;
  const int prec = precision == LG_PREC_X6 ? lg::PREC_X6 : lg::PREC_H3;
  const int np = prec == lg::PREC_X6 ? 3 : 2;
  void* kp = ws + kv_off;
  void* vp = ws + kv_off + np * n * 2;
  _Float16* img = reinterpret_cast<_Float16*>(ws + img_off);
  const bool h3 = prec == lg::PREC_H3;
  LG_HIP(hipMemsetAsync(rtab, 0, 4 * lg::kRangeStride * sizeof(unsigned), st));
  if (h3) {
    LG_HIP(lg::range_absmax(k, n, rtab, 0, st));
    LG_HIP(lg::range_absmax(v, n, rtab, 1, st));
  }
  LG_HIP(lg::split_planes(k, n, kp, prec, lg::RangeOut{h3 ? rtab : nullptr, 0, -1, 1.f, 0.f, 0.f, 2, 1}, st));
  LG_HIP(lg::split_planes(v, n, vp, prec, lg::RangeOut{h3 ? rtab : nullptr, 1, -1, 1.f, 0.f, 0.f, 3, lg::kRangeTrack | lg::kRangeTwoSided}, st,
                          true));
  // one set; the second set is empty (Nq = 0: its workgroups exit at once)
  const lg::AttnSet s0{q, kp, vp, (long long)n, ctx, Nq, Nk, img, (long long)rp * 256, rp, 0, h3 ? rtab : nullptr, 2};
  lg::AttnSet s1 = s0;
  s1.Nq = 0;
  LG_HIP(lg::attention_f32(s0, s1, B, H, scale, prec, st, reinterpret_cast<float*>(ws + part_off),
                           lg::attention_split_floats(B, H, Nq, Nk)));
  if (h3) LG_HIP(lg::image_to_rows(img, (long long)rp * 256, rp, 256, ctx, B * Nq, rtab, 3, st));
  LG_HIP(hipStreamSynchronize(st));
  return LG_OK;
}

}  // extern "C"
