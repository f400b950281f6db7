// Host-visible launch wrappers for the gfx950 kernels (internal to liblightglue_mi355x.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lg {

enum EpiKind {
  EPI_STORE = 0,
  EPI_QKV_ROT = 1,
  EPI_CROSS_QKV = 2,
  EPI_PROBE = 3,    // benchmarking only
  EPI_LN_GELU = 4,  // gemm_h3 only: Yp = plane image of GELU(LayerNorm(acc + bias)), Nout = 512
};

// Operand formats of the fp32-accurate matrix-core arithmetic (common.h):
//   PREC_H3  fp16x3 -- 3 fp16 MFMAs per product; run-time operands are written as plane images
//            scaled by a per-tensor power of two chosen on the device (RangeOut below), so the
//            fp16 range cannot be exceeded and no host check is needed
//   PREC_X6  bf16x6 -- 6 bf16 MFMAs per product; full fp32 range
enum Prec { PREC_H3 = 0, PREC_X6 = 1 };

// ---- Point pruning and early stop for any batch size (lightglue.py:527-562,586-606) --------
// The row space keeps a fixed slot per (image, pair): segment s < B is image 0 of pair s (rows
// s*M0 ..), segment s >= B is image 1 of pair s-B (rows B*M0 + (s-B)*N0 ..).  A segment's kept
// points are a prefix of its slot (cnt[s] of them), compacted in place layer by layer; a pair that
// stopped early is frozen (act[pair] = 0).  Every count lives on the device: no host sync.
struct SegLayout {
  int B, M0, N0;
};
__host__ __device__ inline int seg_base(const SegLayout& L, int s) { return s < L.B ? s * L.M0 : L.B * L.M0 + (s - L.B) * L.N0; }
__host__ __device__ inline int seg_len(const SegLayout& L, int s) { return s < L.B ? L.M0 : L.N0; }
__host__ __device__ inline int seg_of_row(const SegLayout& L, int r, int& local) {
  if (r < L.B * L.M0) {
    const int s = r / L.M0;
    local = r - s * L.M0;
    return s;
  }
  const int r2 = r - L.B * L.M0, p = r2 / L.N0;
  local = r2 - p * L.N0;
  return L.B + p;
}
// Which rows of a GEMM are live: local < cnt[segment] and (sel == null or sel[pair] == sel_eq).
// cnt == null: every row.  Dead rows are neither stored nor tracked; a tile of dead rows exits.
struct RowMask {
  const int* cnt;
  const int* sel;
  int sel_eq;
  SegLayout L;
};
__host__ __device__ inline bool row_live(const RowMask& m, int r) {
  if (!m.cnt) return true;
  int local;
  const int s = seg_of_row(m.L, r, local);
  if (local >= m.cnt[s]) return false;
  return !m.sel || m.sel[s < m.L.B ? s : s - m.L.B] == m.sel_eq;
}
// Run-time range scaling of fp16x3 plane images.  A forward keeps a small table
// in its workspace, zeroed at the start; slot s holds (common.h: sharded layout)
//   M[s]: max |x| over the values written (float bits; atomicMax of non-negative floats), kept
//         only where a later bound needs it (track = 1: the residual stream)
//   E[s]: the exponent the planes were written with -- they hold x * 2^-E[s]
// A producer chooses E before writing from an upper bound of what it will write,
//   bound = g0 * M[in0] + g1 * M[in1] + add     (in0/in1: slots of its inputs, -1 = unused;
//                                                g0/g1/add: weight row-L1 norms and bias maxima)
// E = 0 while bound <= 2^15 (the plane image is then exactly the unscaled one), else the smallest
// E with bound * 2^-E <= 2^15.  Consumers fold 2^E into a scale they apply anyway (the GEMM
// epilogue's accumulator scale, the attention's softmax scale).  Every workgroup of a producer
// derives the same E from the same table entries; a null tab disables scaling (E = 0).
struct RangeOut {
  unsigned* tab;
  int in0, in1;
  float g0, g1, add;
  int out;
  int track;          // kRangeTrack: record M[out] (only the residual stream's images need it; E is
                      // always kept); kRangeTwoSided: E may be negative -- small tensors are scaled
                      // UP to the limit too (value planes, whose low piece is stored unscaled)
  int lshift;         // the bound is held to 2^(15 - lshift): 11 for images used as the "y" operand
                      // of an fp16x3 product (|y| <= 16, so y_h * 2^11 stays finite)
};
constexpr int kRangeTrack = 1, kRangeTwoSided = 2;
inline RangeOut range_none() { return RangeOut{nullptr, -1, -1, 0.f, 0.f, 0.f, 0, 0}; }

// Head-major destinations [set][b][h][n][64] for the QKV epilogues; set 0 = image 0 (B*M rows),
// set 1 = image 1 (B*N rows), rows in GEMM order (image 0 rows first).  All in natural dim order.
//   q   fp32 queries (self) / qk (cross)
//   kp  keys as operand planes (plane p at kp + p*pstride): k (self) / qk (cross)
//       PREC_X6: three bf16 planes (h, m, l);  PREC_H3: two fp16 planes (h, l * 2^11)
//   vp  values, same planes; PREC_H3: (h, l) with the low piece NOT scaled (split2h_v: the
//       attention's P V product then needs no unscaled copy of P's high piece)
struct HeadLayout {
  float* q;
  void* kp;
  void* vp;
  long long pstride;  // elements between planes (= B*(M+N)*H*64)
  int B, H, M, N;
  const float* cosb;  // [rows][32] rotary cos table, by GEMM row
  const float* sinb;
  float qk_scale;
};

struct GemmArgs {
  const float* A0;  // [R][lda0], columns [0, K0)
  int lda0, K0;
  const float* A1;  // [R][lda1], columns [K0, K) (nullable: K0 == K)
  int lda1;
  const float* W;   // [Nout][ldw] (PyTorch Linear layout), k contiguous
  int ldw, K;
  const float* bias;  // [Nout] or null
  const float* res;   // residual [R][ldr] or null (EPI_STORE): Y = res + (acc + bias) * out_scale
  int ldr;
  float* Y;
  int ldy;
  float out_scale;
  int R, Nout;
  long long sA, sA1, sW, sY;  // per-blockIdx.z strides (floats)
  HeadLayout hl;
  RowMask rm;                 // live rows (batched pruning; cnt == null: all)
};

// bf16x6 GEMM on fp32 operands (gemm.hip): the PREC_X6 linears and the similarity GEMM.
hipError_t gemm_x6(const GemmArgs& a, int epi, int batch, hipStream_t st);

// fp16x3 "linear" GEMM on plane images (common.h, gemm_h3.hip):
//   Y = epilogue(A . W^T * acc_scale + bias), A = [A0 | A1] plane images, W = plane image of
//   W * 2^sw (acc_scale = 2^-(11+sw)).  R rows (image rows_pad >= R, multiple of 256),
//   Nout a multiple of 256, K0 and K multiples of 32.
struct PlaneRef {
  const _Float16* p;  // plane 0; plane 1 at p + ps
  long long ps;       // elements between the two planes (= rows_pad * K)
  int rows_pad;
};
struct GemmH3Args {
  PlaneRef A0, A1;  // A1 used for k >= K0 (nullable p when K0 == K)
  int K0, K;
  PlaneRef W;       // rows_pad = Nout
  int R, Nout;
  float acc_scale, out_scale;
  const float* bias;  // [Nout] or null
  const float* res;   // EPI_STORE: Y = res + (...) (nullable), row stride ldr
  int ldr;
  const float* res2;  // EPI_STORE (nullable): rows >= res2_row0 read their residual at res2 + (row - res2_row0) * ldr
  int res2_row0;
  float* Y;           // EPI_STORE fp32 output (nullable), row stride ldy
  int ldy;
  float* Y2;          // EPI_STORE (nullable): rows >= y2_row0 go to Y2 + (row - y2_row0) * ldy instead
  int y2_row0;
  int stream;         // set by gemm_h3: operands too big for the caches take the non-temporal hints
  int reverse;        // walk each XCD's tile range from its end (read what the previous kernel wrote last first)
  _Float16* Yp;       // EPI_STORE: also write Y as a plane image (nullable), with its rows_pad
  long long yps;
  int yrows_pad;
  const unsigned* rtab;  // range table of the A plane images (nullable: both exponents 0)
  int a0_slot, a1_slot;  // their slots (-1: exponent 0)
  RangeOut ro;        // Yp / EPI_LN_GELU planes (EPI_QKV_*: the key planes)
  RangeOut ro_v;      // EPI_QKV_*: the value planes
  RowMask rm;         // live rows (batched pruning; cnt == null: all)
  const float* ln_g;  // EPI_LN_GELU: LayerNorm weight / bias [Nout]
  const float* ln_b;
  HeadLayout hl;      // EPI_QKV_ROT / EPI_CROSS_QKV (EPI_QKV_ROT with hl.cosb null: no rotary)
  int relu;           // EPI_STORE: max(., 0) after bias / scale / residual
};
hipError_t gemm_h3(const GemmH3Args& a, int epi, hipStream_t st);
// fp32 rows [R][K] (row stride ld) -> rows row0 .. row0+R-1 of a plane image (rows_pad), with
// the fp16-range guard; xcopy (optional) also receives the fp32 rows, row stride K
hipError_t rows_to_planes(const float* x, int R, int K, int ld, _Float16* planes, int rows_pad, int row0,
                          const RangeOut& ro, hipStream_t st, float* xcopy = nullptr, const RowMask* rm = nullptr);
// two row sources (r0 rows of x0, then r1 rows of x1) in one launch, no copy / mask
hipError_t rows_to_planes2(const float* x0, int r0, const float* x1, int r1, int K, int ld, _Float16* planes,
                           int rows_pad, int row0, const RangeOut& ro, hipStream_t st);
// max |x| over n floats, atomicMax'ed into slot `slot` of a range table (M only)
hipError_t range_absmax(const float* x, size_t n, unsigned* tab, int slot, hipStream_t st);
// the same over two arrays in one launch (x1 may be null when n1 == 0)
hipError_t range_absmax2(const float* x0, size_t n0, const float* x1, size_t n1, unsigned* tab, int slot,
                         hipStream_t st);

// Attention over head-major Q/K/V ([set][b][h][n][64]); O written row-major into ctx
// [rows][256] at column h*64 (rows in GEMM order).  Two "sets" per launch (blockIdx.z).
struct AttnSet {
  // [B][H][Nq][64] fp32 rows; with attention_f32(..., q_planes) (PREC_H3) instead a plane image
  // [planes][B][H][Nq][64] (plane stride pstride) holding q * 2^-E[k_slot] -- the cross block's
  // qk, whose planes the key side needs anyway, so the QKV GEMM stores it once (the pieces the
  // attention forms from them are the ones it forms from the fp32 rows)
  const void* q;
  const void* kp;    // [planes][B][H][Nk][64] (plane stride pstride): 3 bf16 (X6) / 2 fp16 (H3)
  const void* vp;    // [planes][B][H][Nk][64]
  long long pstride;
  float* o;          // ctx + row_base*256 (PREC_X6)
  int Nq, Nk;
  _Float16* op;      // PREC_H3: ctx plane image (K = 256), rows of this set start at o_row0
  long long ops;
  int o_rows_pad, o_row0;
  // PREC_H3 range exponents (RangeOut): the key planes hold k * 2^-E[k_slot] (folded into the
  // softmax scale); the value planes v * 2^-E[v_slot], so the context planes come out as
  // ctx * 2^-E[v_slot] and their consumer reads v_slot.  Null rtab: exponents 0.
  const unsigned* rtab;
  int k_slot;
  // batched pruning (nullable): per-pair query / key counts (Nq, Nk above are then the layout
  // capacities) and the pairs still running (0 = stopped early: nothing computed or written)
  const int* nq_cnt;
  const int* nk_cnt;
  const int* act;
};
// part / part_floats (optional): scratch for the key-split partials of small batches
// (attention_split_floats(B, H, max Nq, max Nk) floats; without it the launch does not split)
// q_planes (PREC_H3): both sets' q point at plane images with the key planes' exponent (k_slot)
hipError_t attention_f32(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, int prec, hipStream_t st,
                         float* part = nullptr, size_t part_floats = 0, bool q_planes = false);
size_t attention_split_floats(int B, int H, int nq, int nk);

// Positional encoding: normalised keypoints -> cos/sin tables [rows][32].
struct PEArgs {
  const float* kpts;   // [B][n][2]
  const float* size;   // [B][2] or null
  const float* scales; // [B][n] or null
  const float* oris;   // [B][n] or null
  const float* Wr;     // [32][m_in]
  const float* Wc;     // [32]
  const float* bc;     // [32]
  float* cosb;         // [B*n][32]
  float* sinb;
  int B, n, m_in;
};
hipError_t positional_encoding(const PEArgs& a, hipStream_t st);
// both images in one launch
hipError_t positional_encoding2(const PEArgs& a0, const PEArgs& a1, hipStream_t st);
// size = 1 + max - min of each pair's keypoints (normalize_keypoints fallback, lightglue.py:25-26)
hipError_t kpt_extent(const float* kpts, int B, int n, float* size_out, hipStream_t st);

// In place (planes == null, PREC_X6) or into a plane image of K = 512 (PREC_H3).
bool gemm_h3_ln_split(int R);
hipError_t layernorm_gelu_512(float* x, const float* g, const float* b, int rows, _Float16* planes, int rows_pad,
                              const RangeOut& ro, hipStream_t st);
// y[r] = dot(x[r,:256], w) + b ; optional sigmoid
hipError_t gemv_256(const float* x, const float* w, const float* b, float* y, int rows, int sigmoid, hipStream_t st);
// rows of x0 then rows of x1 into y (no sigmoid), one launch
hipError_t gemv_256_masked2(const float* x0, int r0, const float* x1, int r1, const float* w, const float* b, float* y,
                            const RowMask& m, hipStream_t st);

// Dual-softmax assignment + mutual filter (lightglue.py:284-296, 321-337).
struct AssignArgs {
  const float* sim;  // [B][M][N]
  const float* z0;   // [B*M] matchability logits
  const float* z1;   // [B*N]
  float* la;         // [B][M+1][N+1] or null
  float* ws;         // scratch
  int B, M, N;       // M, N: the layout capacities when Mb / Nb are given
  float th;
  int64_t* m0; int64_t* m1; float* s0; float* s1;
  const int* Mb;      // per-pair kept counts (batched pruning; null: M, N for every pair); la
  const int* Nb;      // then holds pair b's [Mb+1][Nb+1] block with the capacity strides
};
size_t assign_workspace_floats(int B, int M, int N);
hipError_t assign_and_filter(const AssignArgs& a, hipStream_t st);
// The same with the similarity recomputed inside two fp16x3 GEMM passes instead of materialised
// (assign_h3.hip): P = plane image of md (rows: image 0 rows of pair b at b*M, image 1 rows at
// B*M + b*N; |md| <= 16 after its range exponent E[slot]), rows_pad >= B*(M+N) + 256, M and N
// multiples of 16, no per-pair counts.  a.sim is not read; a.ws needs assign_workspace_floats +
// sim_h3_workspace_floats.
struct SimH3Args {
  PlaneRef P;
  const unsigned* rtab;
  int slot;
  int B, M, N;
  float2* rowp;                       // stats pass: [B][M][ntn] (max, sum) per column tile
  float* pmax; float* psum;           //             [B][ntm][N] per row tile
  const float* rmax; const float* rlog; const float* ls0;  // la pass inputs [B*M]
  const float* cmax; const float* clog; const float* ls1;  //               [B*N]
  float* la;                          // [B][M+1][N+1] or null
  float* rbest; int* rbi;             // la pass: [B][M][ntn] row argmax per column tile
  float* pv; int* pi;                 //          [B][ntm][N] column argmax per row tile
};
bool sim_h3_supported(int M, int N);
size_t sim_h3_workspace_floats(int B, int M, int N);
hipError_t sim_h3_pass(const SimH3Args& a, int mode, hipStream_t st);
hipError_t sim_row_stats(const SimH3Args& a, hipStream_t st);
hipError_t sim_row_arg(const SimH3Args& a, const float* z0, float* max0, int* arg0, hipStream_t st);
hipError_t assign_and_filter_h3(const AssignArgs& a, const PlaneRef& md, const unsigned* rtab, int slot, hipStream_t st);
// filter_matches on an existing [B][M+1][N+1] log-assignment.
hipError_t filter_from_scores(const float* scores, int B, int M, int N, float th, float* ws, int64_t* m0, int64_t* m1,
                              float* s0, float* s1, hipStream_t st);
size_t filter_workspace_floats(int B, int M, int N);

// Load-time fold of out_proj/to_out into ffn.0 (W1 [512][512], b1 [512], Wo [256][256], bo [256]);
// tmp holds 512*256 + 512 floats.
hipError_t fold_out_proj(float* W1, float* b1, const float* Wo, const float* bo, float* tmp, hipStream_t st);

// fp16x3 weight planes (PREC_H3): absmax of n floats -> *out (one block), then the plane image
// of W [rows][K] * scale (rows_pad = rows).
hipError_t absmax(const float* src, size_t n, float* out, hipStream_t st);
hipError_t split_weight_h3(const float* src, int rows, int K, float scale, _Float16* planes, hipStream_t st);

// lg_attention (kernel-level checks): fp32 [n] -> operand planes of `prec` (plane stride n; PREC_H3
// range-scaled by ro), and a plane image (K columns) -> fp32 rows, times 2^E[slot] of tab.
// values: PREC_H3 value planes (low piece unscaled, HeadLayout.vp)
hipError_t split_planes(const float* x, size_t n, void* planes, int prec, const RangeOut& ro, hipStream_t st,
                        bool values = false);
hipError_t image_to_rows(const _Float16* planes, long long ps, int rows_pad, int K, float* out, int rows,
                         const unsigned* tab, int slot, hipStream_t st);
// Load-time weight statistics for the range bounds: out[0] = max over rows of sum_k |W[r,k]|,
// out[1] = max |bias| (bias may be null), over rows [0, rows) of W [rows][K]; and the LayerNorm
// output bound max_k |g_k| sqrt(n - 1) + |b_k|.
hipError_t weight_range_stats(const float* W, int rows, int K, const float* bias, float* out, hipStream_t st);
hipError_t layernorm_bound(const float* g, const float* b, int n, float* out, hipStream_t st);

// Weight repacking: dst[r,:] = src[idx[r],:] (row length `cols`).
hipError_t gather_rows(float* dst, const float* src, const int* idx, int rows, int cols, hipStream_t st);

// ---- Point pruning and early stop for any batch size: layout and masks above (RowMask) -----
// initial state: cnt = slot sizes, act = 1, stop = L-1, ind = 0, 1, 2, .. per segment
hipError_t prune_init(const SegLayout& L, int* cnt, int* act, int* stop, int n_layers, int* ind, hipStream_t st);
// early stop (check_if_stop :595-606, thresholds :581-584): per running pair, ratio =
// 1 - #(token < thr over its kept points) / (M0 + N0); ratio > depth_conf stops it at `layer`
hipError_t stop_decide(const float* token, const int* cnt, int* act, int* stop, const SegLayout& L, float thr,
                       float depth_conf, int layer, hipStream_t st);
// keep flags + in-segment exclusive scan (get_pruning_mask :586-593): running pairs keep
// sigmoid(z) > width_thr or (token && token <= conf_thr); frozen pairs keep every point
hipError_t prune_scan(const float* zmatch, const float* token, const int* cnt_in, int* cnt_out, const int* act,
                      int* flags, int* pos, const SegLayout& L, float width_thr, float conf_thr, hipStream_t st);
// move kept rows (cols floats each) to their compacted position of the same segment
hipError_t compact_seg(const float* src, float* dst, int cols, const int* flags, const int* pos, const int* cnt_in,
                       const SegLayout& L, hipStream_t st);
// compacted original indices; prune[ind] += 1 for the kept points of running pairs (:540,546)
hipError_t compact_ind_seg(const int* ind, int* ind_out, int64_t* prune0, int64_t* prune1, const int* flags,
                           const int* pos, const int* cnt_in, const int* act, const SegLayout& L, hipStream_t st);
hipError_t fill_i64(int64_t* p, int64_t v, size_t n, hipStream_t st);
// scatter the per-pair compact matches back to full size (lightglue.py:553-562); m0c.. have the
// capacity strides (M0 per pair), the outputs are [B][M0] / [B][N0]
hipError_t remap_seg(const int64_t* m0c, const int64_t* m1c, const float* s0c, const float* s1c, const int* ind,
                     const int* cnt, const SegLayout& L, int64_t* m0, int64_t* m1, float* s0, float* s1, hipStream_t st);
// y[r] = dot(x[r], w) + b for the live rows of a mask (the per-pair assignment heads)
hipError_t gemv_256_masked(const float* x, const float* w, const float* b, float* y, int rows, const RowMask& m,
                           hipStream_t st);

// Sinkhorn (superglue.py:173-201).
size_t sinkhorn_workspace_floats(int B, int M, int N);
hipError_t log_optimal_transport(const float* scores, float alpha, int B, int M, int N, int iters, float* Z, float* ws,
                                 hipStream_t st);

// ---- SuperPoint extractor (gluefactory_nonfree/superpoint.py, superpoint.hip) --------------
// Feature maps are NHWC plane images: rows = pixels (n, y, x) in row-major order, K = channels.
// An image that feeds a 3x3 convolution keeps rows [R, rows_pad) zero (sp_zero_rows): the
// implicit GEMM reads its last row for every tap that falls outside the image.
//
// gray (RGB: 0.299 r + 0.587 g + 0.114 b) + conv1a (1 -> 64, 3x3, pad 1) + bias + ReLU -> planes
hipError_t sp_conv1a(const float* image, int B, int C, int H, int W, const float* w, const float* bias, _Float16* Y,
                     int yrows_pad, const RangeOut& ro, hipStream_t st);
// 3x3 convolution (pad 1) as an implicit fp16x3 GEMM + bias + ReLU (+ 2x2 max-pool, floor):
//   Y = planes of relu(conv(X) + bias) [B*H*W rows] or of its pool [B*(H/2)*(W/2) rows]
struct ConvH3Args {
  PlaneRef X;            // input image, rows B*H*W, K = Cin, rows_pad > B*H*W (zero tail)
  int B, H, W, Cin, Cout;
  PlaneRef Wt;           // [Cout][9*Cin] weight planes, k = (3*ky + kx)*Cin + ci (rows_pad = Cout)
  float acc_scale;       // 2^-(11+sw)
  const float* bias;     // [Cout]
  _Float16* Y;           // output planes (K = Cout)
  long long yps;
  int yrows_pad;
  const unsigned* rtab;  // range table: X holds x * 2^-E[x_slot]
  int x_slot;
  RangeOut ro;           // Y
  int pool;
};
hipError_t sp_conv3x3(const ConvH3Args& a, hipStream_t st);
hipError_t sp_zero_rows(_Float16* planes, long long ps, int rows_pad, int K, int R, hipStream_t st);
// conv weight [Cout][Cin][k][k] -> dst [Cout][k*k*Cin] (column (k*ky + kx)*Cin + ci)
hipError_t sp_repack_conv(const float* w, int Cout, int Cin, int ksize, float* dst, hipStream_t st);
// detector head: 65 logits per cell (row stride ld) -> softmax without the dustbin, unfolded:
// scores[b][8y + dy][8x + dx] = p[8 dy + dx] (superpoint.py:224-230)
hipError_t sp_detector_scores(const float* logits, int ld, int B, int Hc, int Wc, float* scores, hipStream_t st);
// dense descriptors: rows of 256 -> x / max(|x|, 1e-12) (in place allowed)
hipError_t sp_desc_normalize(const float* x, int rows, float* y, hipStream_t st);
// simple_nms (superpoint.py:60-80) on [B][Hs][Ws]; mask / sup bytes, ss floats (scratch)
hipError_t sp_nms(const float* scores, int B, int Hs, int Ws, int radius, unsigned char* mask, unsigned char* sup,
                  float* ss, hipStream_t st);
// candidates: nms(scores) with borders at -1 (superpoint.py:244-254) > threshold, per image in
// row-major order -> key (orderable score bits) / pixel index; cnt[b] = their number.
// image_size: [B][2] (w, h) or null.  blk: scratch ints, B * sp_cand_blocks(Hs)
int sp_cand_blocks(int Hs);
hipError_t sp_candidates(const float* scores, const unsigned char* mask, int B, int Hs, int Ws, int border,
                         const float* image_size, float thr, unsigned* key, int* idx, int* blk, int* cnt, hipStream_t st);
// per image: the k best candidates by score, sorted (torch.topk, superpoint.py:83-87; ties -> lower
// pixel index first), or all of them in row-major order when k <= 0 or there are not more than k.
// Writes sel_idx [B][cap] (pixel index), sel_score [B][cap], n[b]; k <= kSpSelectMax
constexpr int kSpSelectMax = 16384;
hipError_t sp_select(const unsigned* key, const int* idx, const int* cnt, int B, int cand_cap, int k, int* sel_idx,
                     float* sel_score, int cap, int* n, hipStream_t st);
// keypoints (x, y) [B][cap][2] from pixel indices; radius > 0: soft-argmax refinement on the dense
// scores (superpoint.py:97-113)
hipError_t sp_keypoints(const int* sel_idx, const int* n, int B, int cap, int Hs, int Ws, const float* dense,
                        int radius, float* kpts, hipStream_t st);
// bilinear descriptor sampling at (x, y) keypoints + L2 normalisation (superpoint.py:117-149);
// desc NHWC [B][Hc][Wc][256]; out [B][cap][256]; kpts_out (nullable) = kpts + 0.5
hipError_t sp_sample(const float* kpts, const int* n, int B, int cap, const float* desc, int Hc, int Wc, int legacy,
                     float* out, float* kpts_out, hipStream_t st);


// ---- SuperGlue (gluefactory_nonfree/superglue.py, superglue.hip) ---------------------------
constexpr int kSgMaxEnc = 8;
struct SgEncLayer {
  const float* Wt;  // [Cin][Cout] (transposed Conv1d weight)
  const float* b;
  const float *bn_w, *bn_b, *bn_mean, *bn_var;  // eval BatchNorm (all layers but the last)
};
// The first nl layers of the keypoint MLP for rows r of one image set (rows = B * n): out[r] =
// (desc[r] +) layers(x_n, y_n(, score)), row stride ldo; keypoints normalised by size[b] (w, h) or
// (fw, fh) (superglue.py:75-86).  Widths multiples of 4, at most 256.  A layer with bn_w set is
// followed by its BatchNorm and ReLU.
struct SgEncArgs {
  const float* kpts;
  const float* scores;  // null without use_scores
  const float* size;
  float fw, fh;
  const float* desc;    // null: out = the last layer's output alone
  float* out;
  int ldo;
  int rows, n, nl;
  int ch[kSgMaxEnc + 1];
  SgEncLayer layer[kSgMaxEnc];
};
hipError_t sg_keypoint_encoder(const SgEncArgs& a, hipStream_t st);
hipError_t sg_transpose(const float* src, int rows, int cols, float* dst, hipStream_t st);
hipError_t sg_gather_cols(float* dst, const float* src, const int* idx, int rows, int cols, hipStream_t st);
hipError_t sg_bn_fold(float* W, float* b, const float* g, const float* be, const float* mean, const float* var, int rows,
                      int cols, hipStream_t st);
// part: sg_nll_part_doubles(B, M) fp64 partials (caller workspace); nullptr = a stream-ordered
// allocation freed before returning (also on the error paths)
size_t sg_nll_part_doubles(int B, int M);
hipError_t sg_nll_loss(const float* la, int B, int M, int N, const uint8_t* gta, const int64_t* gt0, const int64_t* gt1,
                       int mode, float balancing, float* out, double* part, hipStream_t st);

}  // namespace lg
