// C-ABI of the SuperPoint extractor (include/superpoint_mi355x.h): handle, weight repacking and
// the eval forward orchestration (reference gluefactory_nonfree/superpoint.py:202-350).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/lightglue_mi355x.h"
#include "../../include/superpoint_mi355x.h"
#include "common.h"
#include "kernels.h"

namespace lg {
int api_fail(int code, const char* msg);
}

namespace {

int fail(int code, const std::string& msg) { return lg::api_fail(code, msg.c_str()); }

#define SP_HIP(expr)                                                                                \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess) return fail(LG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
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

// superpoint.py:179-196, registration order (lightglue_amd.sp_weights.superpoint_schema)
std::vector<Tensor> make_schema(const sp_config_t& c) {
  struct L { const char* n; int ci, co, k; };
  std::vector<L> ls = {{"conv1a", 1, 64, 3},    {"conv1b", 64, 64, 3},   {"conv2a", 64, 64, 3},
                       {"conv2b", 64, 64, 3},   {"conv3a", 64, 128, 3},  {"conv3b", 128, 128, 3},
                       {"conv4a", 128, 128, 3}, {"conv4b", 128, 128, 3}};
  if (c.has_detector) {
    ls.push_back({"convPa", 128, 256, 3});
    ls.push_back({"convPb", 256, 65, 1});
  }
  if (c.has_descriptor) {
    ls.push_back({"convDa", 128, 256, 3});
    ls.push_back({"convDb", 256, c.descriptor_dim, 1});
  }
  std::vector<Tensor> s;
  for (auto& l : ls) {
    s.push_back({std::string(l.n) + ".weight", {l.co, l.ci, l.k, l.k}});
    s.push_back({std::string(l.n) + ".bias", {l.co}});
  }
  return s;
}

constexpr int kSlots = 16;
size_t a256(size_t n) { return (n + 255) & ~size_t(255); }
int rows_pad_for(long long R) { return (int)(((R + 1) + 255) / 256 * 256); }  // >= R + 1: a zero row

// A GEMM weight matrix: fp32 repacked [rows][K] in gbuf, its fp16x3 plane image, range stats
struct Mat {
  size_t off = 0;    // floats into gbuf
  int rows = 0, K = 0;
  size_t poff = 0;   // halfs into planes
  float unscale = 1.f;
  size_t boff = 0;   // bias (floats into gbuf)
  float g = 0.f, bmax = 0.f;
};

struct Shape {
  int B, C, H, W, H2, W2, H3, W3, Hc, Wc, Hs, Ws, cap;
  long long R1, R2, R3, Rc;
};
Shape make_shape(int B, int C, int H, int W, int cap) {
  Shape s{B, C, H, W, H / 2, W / 2, H / 4, W / 4, H / 8, W / 8, 0, 0, cap, 0, 0, 0, 0};
  s.H3 = s.H2 / 2;
  s.W3 = s.W2 / 2;
  s.Hc = s.H3 / 2;
  s.Wc = s.W3 / 2;
  s.Hs = 8 * s.Hc;
  s.Ws = 8 * s.Wc;
  s.R1 = (long long)B * H * W;
  s.R2 = (long long)B * s.H2 * s.W2;
  s.R3 = (long long)B * s.H3 * s.W3;
  s.Rc = (long long)B * s.Hc * s.Wc;
  return s;
}

struct Work {
  unsigned* rtab;
  _Float16 *bx, *by;                 // ping-pong plane images
  float *logits, *scores, *desc, *ss, *kp;
  unsigned char *mask, *sup;
  unsigned* key;
  int *idx, *blk, *cnt, *sel;
  size_t bytes;
};
Work carve(char* base, const Shape& s, int Nh) {
  size_t o = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + o : nullptr;
    o += a256(n);
    return p;
  };
  Work w{};
  const auto pl = [](long long R, int K) { return (size_t)2 * rows_pad_for(R) * K * sizeof(_Float16); };
  const size_t bx = std::max({pl(s.R1, 64), pl(s.R2, 64), pl(s.R3, 128), pl(s.Rc, 128), pl(s.Rc, Nh)});
  const size_t by = std::max({pl(s.R2, 64), pl(s.R3, 64), pl(s.Rc, 128)});
  const size_t map = (size_t)s.B * s.Hs * s.Ws;
  w.rtab = (unsigned*)take(kSlots * lg::kRangeStride * sizeof(unsigned));
  w.bx = (_Float16*)take(bx);
  w.by = (_Float16*)take(by);
  w.logits = (float*)take((size_t)s.Rc * 256 * sizeof(float));
  w.desc = (float*)take((size_t)s.Rc * 256 * sizeof(float));
  w.scores = (float*)take(map * sizeof(float));
  w.ss = (float*)take(map * sizeof(float));
  w.mask = (unsigned char*)take(map);
  w.sup = (unsigned char*)take(map);
  w.key = (unsigned*)take(map * sizeof(unsigned));
  w.idx = (int*)take(map * sizeof(int));
  w.blk = (int*)take((size_t)s.B * lg::sp_cand_blocks(s.Hs) * sizeof(int));
  w.cnt = (int*)take((size_t)s.B * sizeof(int));
  w.sel = (int*)take((size_t)s.B * s.cap * sizeof(int));
  w.kp = (float*)take((size_t)s.B * s.cap * 2 * sizeof(float));
  w.bytes = o;
  return w;
}

}  // namespace

struct sp_handle {
  sp_config_t cfg;
  int device;
  std::vector<Tensor> schema;
  std::map<std::string, int> index;
  std::vector<size_t> woff;  // fp32 offsets of the loaded tensors in wbuf
  float* wbuf = nullptr;
  float* gbuf = nullptr;     // repacked GEMM matrices + biases
  _Float16* planes = nullptr;
  Mat enc[7];                // conv1b .. conv4b
  Mat heads, pb, db;         // [convPa | convDa], convPb (rows padded to 256), convDb
  float g1a = 0.f, b1a = 0.f;
  bool loaded = false;
  Shape last{};
  bool have_last = false;
};

static int layer_index(const sp_handle* h, const std::string& name) {
  auto it = h->index.find(name);
  return it == h->index.end() ? -1 : it->second;
}

extern "C" {

int sp_create(const sp_config_t* cfg, int device, sp_handle_t** out) {
  if (!cfg || !out) return fail(LG_E_INVALID, "null argument");
  if (cfg->descriptor_dim != 256) return fail(LG_E_INVALID, "descriptor_dim must be 256");
  if (cfg->nms_radius < 0 || cfg->nms_radius > 8) return fail(LG_E_INVALID, "nms_radius must be in [0, 8]");
  if (cfg->refinement_radius < 0 || cfg->remove_borders < 0) return fail(LG_E_INVALID, "negative radius / border");
  int n = 0;
  SP_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(LG_E_INVALID, "bad device");
  SP_HIP(hipSetDevice(device));
  auto* h = new sp_handle();
  h->cfg = *cfg;
  h->device = device;
  h->schema = make_schema(*cfg);
  size_t off = 0;
  for (size_t i = 0; i < h->schema.size(); ++i) {
    h->index[h->schema[i].name] = (int)i;
    h->woff.push_back(off);
    off += (size_t)h->schema[i].numel();
  }
  hipError_t e = hipMalloc((void**)&h->wbuf, off * sizeof(float));
  if (e != hipSuccess) {
    delete h;
    return fail(LG_E_HIP, std::string("hipMalloc weights: ") + hipGetErrorString(e));
  }
  *out = h;
  return LG_OK;
}

int sp_destroy(sp_handle_t* h) {
  if (!h) return LG_OK;
  (void)hipSetDevice(h->device);
  (void)hipFree(h->wbuf);
  (void)hipFree(h->gbuf);
  (void)hipFree(h->planes);
  delete h;
  return LG_OK;
}

int sp_weight_count(const sp_handle_t* h) { return h ? (int)h->schema.size() : 0; }
const char* sp_weight_name(const sp_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].name.c_str() : nullptr;
}
int64_t sp_weight_numel(const sp_handle_t* h, int i) {
  return (h && i >= 0 && i < (int)h->schema.size()) ? h->schema[i].numel() : -1;
}

int sp_load_weights(sp_handle_t* h, int n, const char* const* names, const float* const* tensors, const int64_t* numels,
                    void* stream) {
  if (!h || n < 0 || (n && (!names || !tensors || !numels))) return fail(LG_E_INVALID, "null argument");
  SP_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  std::vector<int> seen(h->schema.size(), 0);
  for (int i = 0; i < n; ++i) {
    const int k = layer_index(h, names[i]);
    if (k < 0) return fail(LG_E_WEIGHTS, std::string("unexpected key in state_dict: ") + names[i]);
    if (seen[k]++) return fail(LG_E_WEIGHTS, std::string("duplicate key: ") + names[i]);
    if (numels[i] != h->schema[k].numel())
      return fail(LG_E_WEIGHTS, std::string("size mismatch for ") + names[i] + ": expected " +
                                    std::to_string(h->schema[k].numel()) + " got " + std::to_string(numels[i]));
  }
  for (size_t k = 0; k < h->schema.size(); ++k)
    if (!seen[k]) return fail(LG_E_WEIGHTS, "missing key in state_dict: " + h->schema[k].name);
  for (int i = 0; i < n; ++i)
    SP_HIP(hipMemcpyAsync(h->wbuf + h->woff[layer_index(h, names[i])], tensors[i], numels[i] * sizeof(float),
                          hipMemcpyDeviceToDevice, st));
  auto W = [&](const char* nm) { return h->wbuf + h->woff[layer_index(h, std::string(nm) + ".weight")]; };
  auto Bi = [&](const char* nm) { return h->wbuf + h->woff[layer_index(h, std::string(nm) + ".bias")]; };

  // repacked GEMM matrices: [Cout][9 Cin] for 3x3 (k = (3 ky + kx) Cin + ci), [Cout][Cin] for 1x1
  const char* encn[7] = {"conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b"};
  const int enc_ci[7] = {64, 64, 64, 64, 128, 128, 128}, enc_co[7] = {64, 64, 64, 128, 128, 128, 128};
  const bool det = h->cfg.has_detector, des = h->cfg.has_descriptor;
  const int Nh = 256 * ((det ? 1 : 0) + (des ? 1 : 0));
  size_t off = 0;
  auto place = [&](Mat& m, int rows, int K) {
    m.rows = rows;
    m.K = K;
    m.off = off;
    off += (size_t)rows * K;
    m.boff = off;
    off += rows;
  };
  for (int i = 0; i < 7; ++i) place(h->enc[i], enc_co[i], 9 * enc_ci[i]);
  if (Nh) place(h->heads, Nh, 9 * 128);
  if (det) place(h->pb, 256, 256);
  if (des) place(h->db, 256, 256);
  (void)hipFree(h->gbuf);
  (void)hipFree(h->planes);
  h->gbuf = nullptr;
  h->planes = nullptr;
  SP_HIP(hipMalloc((void**)&h->gbuf, off * sizeof(float)));
  SP_HIP(hipMemsetAsync(h->gbuf, 0, off * sizeof(float), st));
  float* G = h->gbuf;
  for (int i = 0; i < 7; ++i) {
    SP_HIP(lg::sp_repack_conv(W(encn[i]), enc_co[i], enc_ci[i], 3, G + h->enc[i].off, st));
    SP_HIP(hipMemcpyAsync(G + h->enc[i].boff, Bi(encn[i]), enc_co[i] * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  int hr = 0;
  if (det) {
    SP_HIP(lg::sp_repack_conv(W("convPa"), 256, 128, 3, G + h->heads.off, st));
    SP_HIP(hipMemcpyAsync(G + h->heads.boff, Bi("convPa"), 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
    hr = 256;
    SP_HIP(hipMemcpyAsync(G + h->pb.off, W("convPb"), 65 * 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
    SP_HIP(hipMemcpyAsync(G + h->pb.boff, Bi("convPb"), 65 * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  if (des) {
    SP_HIP(lg::sp_repack_conv(W("convDa"), 256, 128, 3, G + h->heads.off + (size_t)hr * 9 * 128, st));
    SP_HIP(hipMemcpyAsync(G + h->heads.boff + hr, Bi("convDa"), 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
    SP_HIP(hipMemcpyAsync(G + h->db.off, W("convDb"), 256 * 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
    SP_HIP(hipMemcpyAsync(G + h->db.boff, Bi("convDb"), 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  std::vector<Mat*> mats;
  for (auto& m : h->enc) mats.push_back(&m);
  if (Nh) mats.push_back(&h->heads);
  if (det) mats.push_back(&h->pb);
  if (des) mats.push_back(&h->db);
  // per matrix: absmax (plane scale 2^sw, max |W 2^sw| in [8, 16)), max row L1 and max |bias|
  // (range bounds, kernels.h RangeOut); conv1a: row L1 / bias max of its [64][9] weight
  const int nf = (int)mats.size() * 3 + 2;
  float* dst = nullptr;
  SP_HIP(hipMallocAsync((void**)&dst, nf * sizeof(float), st));
  for (size_t i = 0; i < mats.size(); ++i) {
    SP_HIP(lg::absmax(G + mats[i]->off, (size_t)mats[i]->rows * mats[i]->K, dst + 3 * i, st));
    SP_HIP(lg::weight_range_stats(G + mats[i]->off, mats[i]->rows, mats[i]->K, G + mats[i]->boff, dst + 3 * i + 1, st));
  }
  SP_HIP(lg::weight_range_stats(W("conv1a"), 64, 9, Bi("conv1a"), dst + nf - 2, st));
  std::vector<float> hs(nf);
  SP_HIP(hipMemcpyAsync(hs.data(), dst, nf * sizeof(float), hipMemcpyDeviceToHost, st));
  SP_HIP(hipStreamSynchronize(st));
  SP_HIP(hipFreeAsync(dst, st));
  size_t ptotal = 0;
  for (auto* m : mats) ptotal += 2 * (size_t)m->rows * m->K;
  SP_HIP(hipMalloc((void**)&h->planes, ptotal * sizeof(_Float16)));
  size_t po = 0;
  for (size_t i = 0; i < mats.size(); ++i) {
    Mat& m = *mats[i];
    int sw = 0;
    if (hs[3 * i] > 0.f && std::isfinite(hs[3 * i])) {
      int E;
      (void)std::frexp(hs[3 * i], &E);
      sw = std::min(std::max(4 - E, -100), 100);
    }
    SP_HIP(lg::split_weight_h3(G + m.off, m.rows, m.K, std::ldexp(1.f, sw), h->planes + po, st));
    m.poff = po;
    m.unscale = std::ldexp(1.f, -(11 + sw));
    m.g = hs[3 * i + 1];
    m.bmax = hs[3 * i + 2];
    po += 2 * (size_t)m.rows * m.K;
  }
  h->g1a = hs[nf - 2];
  h->b1a = hs[nf - 1];
  h->loaded = true;
  return LG_OK;
}

int sp_workspace_bytes(const sp_handle_t* h, int32_t B, int32_t C, int32_t H, int32_t W, int32_t capacity, size_t* bytes) {
  if (!h || !bytes || B < 0 || H < 0 || W < 0 || capacity < 0) return fail(LG_E_INVALID, "bad argument");
  const int Nh = 256 * ((h->cfg.has_detector ? 1 : 0) + (h->cfg.has_descriptor ? 1 : 0));
  *bytes = carve(nullptr, make_shape(B, C, H, W, capacity), std::max(Nh, 256)).bytes;
  return LG_OK;
}

int sp_forward(sp_handle_t* h, const sp_inputs_t* in, sp_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream) {
  if (!h || !in || !out) return fail(LG_E_INVALID, "null argument");
  if (!h->loaded) return fail(LG_E_WEIGHTS, "weights not loaded");
  const sp_config_t& c = h->cfg;
  if (in->B <= 0 || (in->C != 1 && in->C != 3) || !in->image) return fail(LG_E_INVALID, "image must be [B, 1 or 3, H, W]");
  const Shape s = make_shape(in->B, in->C, in->H, in->W, out->capacity);
  if (s.Hc < 1 || s.Wc < 1) return fail(LG_E_INVALID, "image smaller than 8 x 8");
  const bool sparse = in->sparse != 0;
  if (sparse && !(c.has_detector && c.has_descriptor))
    return fail(LG_E_INVALID, "sparse outputs need the detector and the descriptor (superpoint.py:239)");
  if (sparse && (!out->keypoints || !out->keypoint_scores || !out->counts))
    return fail(LG_E_INVALID, "sparse outputs: keypoints, keypoint_scores and counts are required");
  if (sparse && in->max_keypoints > lg::kSpSelectMax)
    return fail(LG_E_INVALID, "max_keypoints above " + std::to_string(lg::kSpSelectMax));
  if (sparse && in->max_keypoints > 0 && out->capacity < in->max_keypoints)
    return fail(LG_E_INVALID, "capacity below max_keypoints");
  if (sparse && in->max_keypoints <= 0 && out->capacity < s.Hs * s.Ws)
    return fail(LG_E_INVALID, "capacity must hold every candidate (8Hc * 8Wc) when max_keypoints <= 0");
  if (s.R1 + 1 >= (1LL << 26)) return fail(LG_E_INVALID, "B * H * W too large for one forward (< 2^26 pixels)");
  const int Nh = 256 * ((c.has_detector ? 1 : 0) + (c.has_descriptor ? 1 : 0));
  const Work w = carve((char*)workspace, s, std::max(Nh, 256));
  if (!workspace || workspace_bytes < w.bytes)
    return fail(LG_E_WORKSPACE, "workspace too small: need " + std::to_string(w.bytes) + " bytes");
  SP_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const int B = s.B;

  SP_HIP(hipMemsetAsync(w.rtab, 0, kSlots * lg::kRangeStride * sizeof(unsigned), st));
  SP_HIP(lg::range_absmax(in->image, (size_t)B * s.C * s.H * s.W, w.rtab, 0, st));
  auto ro = [&](int in_slot, float g, float add, int out_slot) {
    return lg::RangeOut{w.rtab, in_slot, -1, g, 0.f, add, out_slot, 1};
  };
  // gray weights sum to 1: |gray| <= max |image|
  const float* W1a = h->wbuf + h->woff[layer_index(h, "conv1a.weight")];
  const float* B1a = h->wbuf + h->woff[layer_index(h, "conv1a.bias")];
  const int rp1 = rows_pad_for(s.R1);
  SP_HIP(lg::sp_conv1a(in->image, B, s.C, s.H, s.W, W1a, B1a, w.bx, rp1, ro(0, h->g1a, h->b1a, 1), st));

  // encoder: (input image, its rows, K, spatial H x W, pool?) -> output
  struct Step { _Float16* x; _Float16* y; int H, W, Cin, Cout; bool pool; };
  const Step steps[7] = {{w.bx, w.by, s.H, s.W, 64, 64, true},       {w.by, w.bx, s.H2, s.W2, 64, 64, false},
                         {w.bx, w.by, s.H2, s.W2, 64, 64, true},     {w.by, w.bx, s.H3, s.W3, 64, 128, false},
                         {w.bx, w.by, s.H3, s.W3, 128, 128, true},   {w.by, w.bx, s.Hc, s.Wc, 128, 128, false},
                         {w.bx, w.by, s.Hc, s.Wc, 128, 128, false}};
  auto conv = [&](const Step& t, const Mat& m, int x_slot, int y_slot) -> int {
    const long long rin = (long long)B * t.H * t.W;
    const int rpx = rows_pad_for(rin);
    const long long rout = t.pool ? (long long)B * (t.H / 2) * (t.W / 2) : rin;
    const int rpy = rows_pad_for(rout);
    SP_HIP(lg::sp_zero_rows(t.x, (long long)rpx * t.Cin, rpx, t.Cin, (int)rin, st));
    lg::ConvH3Args a{};
    a.X = {t.x, (long long)rpx * t.Cin, rpx};
    a.B = B;
    a.H = t.H;
    a.W = t.W;
    a.Cin = t.Cin;
    a.Cout = t.Cout;
    a.Wt = {h->planes + m.poff, (long long)m.rows * m.K, m.rows};
    a.acc_scale = m.unscale;
    a.bias = h->gbuf + m.boff;
    a.Y = t.y;
    a.yps = (long long)rpy * t.Cout;
    a.yrows_pad = rpy;
    a.rtab = w.rtab;
    a.x_slot = x_slot;
    a.ro = ro(x_slot, m.g, m.bmax, y_slot);
    a.pool = t.pool;
    SP_HIP(lg::sp_conv3x3(a, st));
    return LG_OK;
  };
  for (int i = 0; i < 7; ++i)
    if (int r = conv(steps[i], h->enc[i], 1 + i, 2 + i)) return r;  // slots 1..8
  const int rpc = rows_pad_for(s.Rc);
  if (Nh) {
    const Step hs{w.by, w.bx, s.Hc, s.Wc, 128, Nh, false};
    if (int r = conv(hs, h->heads, 8, 9)) return r;  // slot 9: [Pa | Da] after ReLU
  }
  auto head1x1 = [&](const Mat& m, int kb0, float* y) -> int {
    lg::GemmH3Args a{};
    a.A0 = {w.bx + (size_t)kb0 * rpc * lg::kKB, (long long)rpc * Nh, rpc};
    a.K0 = a.K = 256;
    a.W = {h->planes + m.poff, (long long)m.rows * m.K, m.rows};
    a.R = (int)s.Rc;
    a.Nout = 256;
    a.acc_scale = m.unscale;
    a.out_scale = 1.f;
    a.bias = h->gbuf + m.boff;
    a.Y = y;
    a.ldy = 256;
    a.rtab = w.rtab;
    a.a0_slot = 9;
    a.a1_slot = -1;
    a.ro = lg::range_none();
    a.ro_v = lg::range_none();
    SP_HIP(lg::gemm_h3(a, lg::EPI_STORE, st));
    return LG_OK;
  };
  float* scores = out->dense_scores ? out->dense_scores : w.scores;
  if (c.has_detector) {
    if (int r = head1x1(h->pb, 0, w.logits)) return r;
    SP_HIP(lg::sp_detector_scores(w.logits, 256, B, s.Hc, s.Wc, scores, st));
  }
  if (c.has_descriptor) {
    if (int r = head1x1(h->db, c.has_detector ? 8 : 0, w.desc)) return r;
    SP_HIP(lg::sp_desc_normalize(w.desc, (int)s.Rc, w.desc, st));
    if (out->dense_descriptors)
      SP_HIP(hipMemcpyAsync(out->dense_descriptors, w.desc, (size_t)s.Rc * 256 * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  h->last = s;
  h->have_last = true;
  if (sparse) {
    SP_HIP(lg::sp_nms(scores, B, s.Hs, s.Ws, c.nms_radius, w.mask, w.sup, w.ss, st));
    SP_HIP(lg::sp_candidates(scores, w.mask, B, s.Hs, s.Ws, c.remove_borders, in->image_size, c.detection_threshold, w.key,
                             w.idx, w.blk, w.cnt, st));
    const int k = in->max_keypoints;
    SP_HIP(lg::sp_select(w.key, w.idx, w.cnt, B, s.Hs * s.Ws, k, w.sel, out->keypoint_scores, s.cap, out->counts, st));
    SP_HIP(lg::sp_keypoints(w.sel, out->counts, B, s.cap, s.Hs, s.Ws, scores, c.refinement_radius, w.kp, st));
    SP_HIP(lg::sp_sample(w.kp, out->counts, B, s.cap, w.desc, s.Hc, s.Wc, c.legacy_sampling, out->descriptors, out->keypoints,
                         st));
    if (out->host_counts) {
      SP_HIP(hipMemcpyAsync(out->host_counts, out->counts, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
      SP_HIP(hipStreamSynchronize(st));
    }
  }
  return LG_OK;
}

int sp_sample_descriptors(sp_handle_t* h, const float* keypoints, const int32_t* counts, int32_t B, int32_t capacity,
                          float* descriptors, void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !keypoints || !counts || !descriptors || !workspace) return fail(LG_E_INVALID, "null argument");
  if (!h->have_last || B != h->last.B) return fail(LG_E_INVALID, "no sp_forward of this batch on the handle");
  const int Nh = 256 * ((h->cfg.has_detector ? 1 : 0) + (h->cfg.has_descriptor ? 1 : 0));
  const Work w = carve((char*)workspace, h->last, std::max(Nh, 256));
  if (workspace_bytes < w.bytes) return fail(LG_E_WORKSPACE, "workspace too small");
  SP_HIP(hipSetDevice(h->device));
  SP_HIP(lg::sp_sample(keypoints, counts, B, capacity, w.desc, h->last.Hc, h->last.Wc, h->cfg.legacy_sampling, descriptors,
                       nullptr, (hipStream_t)stream));
  return LG_OK;
}

}  // extern "C"
