#include <algorithm>
// Bandwidth-bound kernels of the LightGlue hot path (gfx950): positional encoding, fused
// LayerNorm+GELU, 256-wide GEMVs (matchability / token confidence), weight repacking and the
// point-pruning compaction.  One wave per row wherever a row reduction is needed.
#include "common.h"
#include "kernels.h"

namespace lg {

// ----------------------------------------------------------------------------------------
// normalize_keypoints (lightglue.py:21-33) + ConditionalLearnableFourierPositionalEncoding
// (lightglue.py:63-77).  The op order mirrors torch-CPU exactly (probed in the build
// container): Wr(x) = fma chain starting from x0*w0 (MKL sgemm, K = 2), the condition
// Linear(1,32) is a separate multiply and add, then `projected + condition` is a separate add.
// With the reference's default init the condition term reaches |2000|, so a single rounding
// difference moves the phase by ~1e-4 rad; mirroring the order keeps the phases bit-exact.
// ----------------------------------------------------------------------------------------
__global__ void kpt_extent_kernel(const float* kpts, int n, float* size_out) {
  // size = 1 + max - min over the pair's keypoints (lightglue.py:25-26); one block per pair.
  const int b = blockIdx.x;
  float mx[2] = {-INFINITY, -INFINITY}, mn[2] = {INFINITY, INFINITY};
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float v = kpts[((size_t)b * n + i) * 2 + c];
      mx[c] = fmaxf(mx[c], v);
      mn[c] = fminf(mn[c], v);
    }
  }
  __shared__ float red[4][256];
  red[0][threadIdx.x] = mx[0]; red[1][threadIdx.x] = mx[1];
  red[2][threadIdx.x] = mn[0]; red[3][threadIdx.x] = mn[1];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][threadIdx.x + s]);
      red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + s]);
      red[2][threadIdx.x] = fminf(red[2][threadIdx.x], red[2][threadIdx.x + s]);
      red[3][threadIdx.x] = fminf(red[3][threadIdx.x], red[3][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 2) size_out[b * 2 + threadIdx.x] = add_rn(1.f, sub_rn(red[threadIdx.x][0], red[2 + threadIdx.x][0]));
}

__global__ void pe_kernel(PEArgs a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;  // (point, freq)
  const int f = gid & 31;
  const int pt = gid >> 5;
  if (pt >= a.B * a.n) return;
  const int b = pt / a.n;
  const float w = a.size[b * 2 + 0], h = a.size[b * 2 + 1];
  const float scale = div_rn(fmaxf(w, h), 2.f);
  float x[4];
  x[0] = div_rn(sub_rn(a.kpts[(size_t)pt * 2 + 0], div_rn(w, 2.f)), scale);
  x[1] = div_rn(sub_rn(a.kpts[(size_t)pt * 2 + 1], div_rn(h, 2.f)), scale);
  if (a.m_in == 4) {
    x[2] = a.scales[pt];
    x[3] = a.oris[pt];
  }
  const float* wr = a.Wr + f * a.m_in;
  float p = mul_rn(x[0], wr[0]);
  for (int k = 1; k < a.m_in; ++k) p = __fmaf_rn(x[k], wr[k], p);
  const float cond = add_rn(mul_rn((float)a.n, a.Wc[f]), a.bc[f]);  // relu(n) = n
  p = add_rn(p, cond);
  a.cosb[(size_t)pt * kFreq + f] = cosf(p);
  a.sinb[(size_t)pt * kFreq + f] = sinf(p);
}

hipError_t positional_encoding(const PEArgs& a0, hipStream_t st) {
  if (a0.B * a0.n == 0) return hipSuccess;
  const int threads = a0.B * a0.n * 32;
  hipLaunchKernelGGL(pe_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, a0);
  return hipGetLastError();
}

// both images in one launch (blockIdx.y selects the image; the values are pe_kernel's)
__global__ void pe2_kernel(PEArgs a0, PEArgs a1) {
  const PEArgs& a = blockIdx.y == 0 ? a0 : a1;
  if ((int)blockIdx.x * (int)blockDim.x >= a.B * a.n * 32) return;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int f = gid & 31;
  const int pt = gid >> 5;
  if (pt >= a.B * a.n) return;
  const int b = pt / a.n;
  const float w = a.size[b * 2 + 0], h = a.size[b * 2 + 1];
  const float scale = div_rn(fmaxf(w, h), 2.f);
  float x[4];
  x[0] = div_rn(sub_rn(a.kpts[(size_t)pt * 2 + 0], div_rn(w, 2.f)), scale);
  x[1] = div_rn(sub_rn(a.kpts[(size_t)pt * 2 + 1], div_rn(h, 2.f)), scale);
  if (a.m_in == 4) {
    x[2] = a.scales[pt];
    x[3] = a.oris[pt];
  }
  const float* wr = a.Wr + f * a.m_in;
  float p = mul_rn(x[0], wr[0]);
  for (int k = 1; k < a.m_in; ++k) p = __fmaf_rn(x[k], wr[k], p);
  const float cond = add_rn(mul_rn((float)a.n, a.Wc[f]), a.bc[f]);  // relu(n) = n
  p = add_rn(p, cond);
  a.cosb[(size_t)pt * kFreq + f] = cosf(p);
  a.sinb[(size_t)pt * kFreq + f] = sinf(p);
}

hipError_t positional_encoding2(const PEArgs& a0, const PEArgs& a1, hipStream_t st) {
  const int t = std::max(a0.B * a0.n, a1.B * a1.n) * 32;
  if (t == 0) return hipSuccess;
  hipLaunchKernelGGL(pe2_kernel, dim3((t + 255) / 256, 2), dim3(256), 0, st, a0, a1);
  return hipGetLastError();
}

hipError_t kpt_extent(const float* kpts, int B, int n, float* size_out, hipStream_t st) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(kpt_extent_kernel, dim3(B), dim3(256), 0, st, kpts, n, size_out);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// ffn.1 LayerNorm(512, eps 1e-5) + ffn.2 GELU(erf) (lightglue.py:171-176), in place.
// One wave per row: lane holds columns [4l, 4l+4) and [256+4l, 256+4l+4).
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ln_gelu_kernel(float* x, const float* g, const float* bta, int rows,
                                                      _Float16* planes, int rows_pad, RangeOut ro) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int eo = planes ? range_exponent(ro) : 0;
  const float so = ldexpf(1.f, -eo);
  float wmax = 0.f;
  if (row < rows) {
    float* xr = x + (size_t)row * 512;
    f32x4 v0 = *reinterpret_cast<f32x4*>(xr + lane * 4);
    f32x4 v1 = *reinterpret_cast<f32x4*>(xr + 256 + lane * 4);
    float s = (v0[0] + v0[1]) + (v0[2] + v0[3]) + (v1[0] + v1[1]) + (v1[2] + v1[3]);
    const float mean = wave_sum(s) * (1.f / 512.f);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d0 = v0[i] - mean, d1 = v1[i] - mean;
      q += d0 * d0 + d1 * d1;
    }
    const float var = wave_sum(q) * (1.f / 512.f);
    const float rstd = 1.f / sqrtf(var + 1e-5f);
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(g + lane * 4), g1 = *reinterpret_cast<const f32x4*>(g + 256 + lane * 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(bta + lane * 4), b1 = *reinterpret_cast<const f32x4*>(bta + 256 + lane * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float y0 = (v0[i] - mean) * rstd * g0[i] + b0[i];
      float y1 = (v1[i] - mean) * rstd * g1[i] + b1[i];
      const f32x2_ z = gelu_erf2(f32x2_{y0, y1});  // packed: the same values as gelu_erf
      v0[i] = z.x;
      v1[i] = z.y;
    }
    if (!planes) {
      *reinterpret_cast<f32x4*>(xr + lane * 4) = v0;
      *reinterpret_cast<f32x4*>(xr + 256 + lane * 4) = v1;
    } else {
      // plane image (K = 512): 4 consecutive columns = 8 bytes per plane
      const size_t ps = (size_t)rows_pad * 512;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const f32x4 v = hf ? v1 : v0;
        f16x4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wmax = fmaxf(wmax, fabsf(v[e]));
          _Float16 a, b;
          split2h(v[e] * so, a, b);
          h[e] = a;
          l[e] = b;
        }
        const size_t off = plane_off(row, hf * 256 + lane * 4, rows_pad);
        *reinterpret_cast<f16x4*>(planes + off) = h;
        *reinterpret_cast<f16x4*>(planes + ps + off) = l;
      }
    }
  }
  if (planes) range_commit(ro, wmax, eo);
}

hipError_t layernorm_gelu_512(float* x, const float* g, const float* b, int rows, _Float16* planes, int rows_pad,
                              const RangeOut& ro, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(ln_gelu_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, g, b, rows, planes, rows_pad, ro);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// Linear(256 -> 1) (+ sigmoid): MatchAssignment.matchability (lightglue.py:303,312-313,318)
// and TokenConfidence.token (:99,104-106).  One wave per row.
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gemv256_kernel(const float* x, const float* w, const float* b, float* y, int rows,
                                                      int sigmoid, RowMask rm) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows || !row_live(rm, row)) return;
  const f32x4 xv = *reinterpret_cast<const f32x4*>(x + (size_t)row * kDim + lane * 4);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w + lane * 4);
  float s = xv[0] * wv[0] + xv[1] * wv[1] + xv[2] * wv[2] + xv[3] * wv[3];
  s = wave_sum(s);
  if (lane == 0) {
    float v = s + b[0];
    if (sigmoid) v = 1.f / (1.f + expf(-v));
    y[row] = v;
  }
}

hipError_t gemv_256(const float* x, const float* w, const float* b, float* y, int rows, int sigmoid, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(gemv256_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, y, rows, sigmoid, RowMask{});
  return hipGetLastError();
}

hipError_t gemv_256_masked(const float* x, const float* w, const float* b, float* y, int rows, const RowMask& m,
                           hipStream_t st) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(gemv256_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, y, rows, 0, m);
  return hipGetLastError();
}

// the same over two row sources in one launch: rows [0, r0) of x0, then rows [0, r1) of x1 into
// y[0 .. r0 + r1); each source's rows are tested against rm with their own index (as two calls)
__global__ __launch_bounds__(256) void gemv256_2_kernel(const float* x0, int r0, const float* x1, int r1, const float* w,
                                                        const float* b, float* y, RowMask rm) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= r0 + r1) return;
  const bool second = row >= r0;
  const int sr = second ? row - r0 : row;
  if (!row_live(rm, sr)) return;
  const float* x = (second ? x1 : x0) + (size_t)sr * kDim;
  const f32x4 xv = *reinterpret_cast<const f32x4*>(x + lane * 4);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w + lane * 4);
  float s = xv[0] * wv[0] + xv[1] * wv[1] + xv[2] * wv[2] + xv[3] * wv[3];
  s = wave_sum(s);
  if (lane == 0) y[row] = s + b[0];
}

hipError_t gemv_256_masked2(const float* x0, int r0, const float* x1, int r1, const float* w, const float* b, float* y,
                            const RowMask& m, hipStream_t st) {
  if (r0 + r1 == 0) return hipSuccess;
  hipLaunchKernelGGL(gemv256_2_kernel, dim3((r0 + r1 + 3) / 4), dim3(256), 0, st, x0, r0, x1, r1, w, b, y, m);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// Load-time fold of out_proj into ffn.0 (lightglue.py:172,190-191):
//   ffn0([x, Wo c + bo]) = W1[:, :256] x + (W1[:, 256:] Wo) c + (b1 + W1[:, 256:] bo)
// The folded block and bias are accumulated in fp64 and rounded once to fp32.
// ----------------------------------------------------------------------------------------
__global__ void fold_out_proj_kernel(const float* W1, const float* b1, const float* Wo, const float* bo, float* Wf,
                                     float* bf) {
  const int r = blockIdx.x;  // 0..511 (ffn.0 output row)
  const int c = threadIdx.x; // 0..255 (context column)
  const float* w1r = W1 + (size_t)r * 512 + 256;
  double s = 0.0;
  for (int k = 0; k < 256; ++k) s += (double)w1r[k] * (double)Wo[(size_t)k * 256 + c];
  Wf[(size_t)r * 256 + c] = (float)s;
  if (c == 0) {
    double t = (double)b1[r];
    for (int k = 0; k < 256; ++k) t += (double)w1r[k] * (double)bo[k];
    bf[r] = (float)t;
  }
}

hipError_t fold_out_proj(float* W1, float* b1, const float* Wo, const float* bo, float* tmp, hipStream_t st) {
  // tmp: 512*256 + 512 floats
  hipLaunchKernelGGL(fold_out_proj_kernel, dim3(512), dim3(256), 0, st, W1, b1, Wo, bo, tmp, tmp + 512 * 256);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipMemcpy2DAsync(W1 + 256, 512 * sizeof(float), tmp, 256 * sizeof(float), 256 * sizeof(float), 512,
                       hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(b1, tmp + 512 * 256, 512 * sizeof(float), hipMemcpyDeviceToDevice, st);
}

// ----------------------------------------------------------------------------------------
// weight repacking
// ----------------------------------------------------------------------------------------
// absmax over n floats -> *out (one block of 1024 threads; load time only)
__global__ __launch_bounds__(1024) void absmax_kernel(const float* src, size_t n, float* out) {
  __shared__ float red[16];
  float m = 0.f;
  for (size_t i = threadIdx.x; i < n; i += 1024) m = fmaxf(m, fabsf(src[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t = fmaxf(t, red[w]);
    *out = t;
  }
}

hipError_t absmax(const float* src, size_t n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(absmax_kernel, dim3(1), dim3(1024), 0, st, src, n, out);
  return hipGetLastError();
}

// fp16x3 weight plane image (common.h) of W [rows][K] * scale (a power of two, so that
// max|W * scale| < 16 and the h * 2^11 piece the GEMM forms in registers stays finite).
__global__ void split_weight_h3_kernel(const float* src, int rows, int K, float scale, _Float16* planes) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)rows * K) return;
  const int r = (int)(i / K), k = (int)(i % K);
  _Float16 h, l;
  split2h(src[i] * scale, h, l);
  const size_t off = plane_off(r, k, rows);
  planes[off] = h;
  planes[(size_t)rows * K + off] = l;
}

hipError_t split_weight_h3(const float* src, int rows, int K, float scale, _Float16* planes, hipStream_t st) {
  const size_t n = (size_t)rows * K;
  if (n == 0) return hipSuccess;
  if (K % kKB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(split_weight_h3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, rows, K, scale,
                     planes);
  return hipGetLastError();
}

__global__ void gather_rows_kernel(float* dst, const float* src, const int* idx, int rows, int cols) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i % cols);
  dst[i] = src[(size_t)idx[r] * cols + c];
}

hipError_t gather_rows(float* dst, const float* src, const int* idx, int rows, int cols, hipStream_t st) {
  const size_t n = (size_t)rows * cols;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, src, idx, rows, cols);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// Point pruning (lightglue.py:532-547, get_pruning_mask :586-593) and early stop
// (check_if_stop :595-606) for any batch size: fixed per-(image, pair) segments, device counts
// (kernels.h SegLayout).
// ----------------------------------------------------------------------------------------
__global__ void prune_init_kernel(SegLayout L, int* cnt, int* act, int* stop, int n_layers, int* ind) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int R = L.B * (L.M0 + L.N0);
  if (t < R) {
    int local;
    (void)seg_of_row(L, t, local);
    ind[t] = local;
  }
  if (t < 2 * L.B) cnt[t] = seg_len(L, t);
  if (t < L.B) {
    act[t] = 1;
    stop[t] = n_layers - 1;
  }
}

hipError_t prune_init(const SegLayout& L, int* cnt, int* act, int* stop, int n_layers, int* ind, hipStream_t st) {
  const int R = L.B * (L.M0 + L.N0);
  hipLaunchKernelGGL(prune_init_kernel, dim3((R + 255) / 256), dim3(256), 0, st, L, cnt, act, stop, n_layers, ind);
  return hipGetLastError();
}

// one workgroup per pair
__global__ __launch_bounds__(256) void stop_decide_kernel(const float* token, const int* cnt, int* act, int* stop,
                                                          SegLayout L, float thr, float depth_conf, int layer) {
  __shared__ int red[4];
  const int b = blockIdx.x;
  if (!act[b]) return;
  int below = 0;
  for (int sgi = 0; sgi < 2; ++sgi) {
    const int s = sgi == 0 ? b : L.B + b;
    const int base = seg_base(L, s), n = cnt[s];
    for (int i = threadIdx.x; i < n; i += 256) below += token[base + i] < thr ? 1 : 0;
  }
  for (int o = 32; o >= 1; o >>= 1) below += __shfl_xor(below, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = below;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int c = red[0] + red[1] + red[2] + red[3];
    // 1.0 - (confidences < threshold).float().sum() / num_points, num_points = m + n (:602-605)
    const float ratio = 1.0f - (float)c / (float)(L.M0 + L.N0);
    if (ratio > depth_conf) {
      act[b] = 0;
      stop[b] = layer;
    }
  }
}

hipError_t stop_decide(const float* token, const int* cnt, int* act, int* stop, const SegLayout& L, float thr,
                       float depth_conf, int layer, hipStream_t st) {
  hipLaunchKernelGGL(stop_decide_kernel, dim3(L.B), dim3(256), 0, st, token, cnt, act, stop, L, thr, depth_conf, layer);
  return hipGetLastError();
}

// one workgroup per segment: keep flags and their exclusive scan (chunks of 1024 with a carry)
__global__ __launch_bounds__(1024) void prune_scan_kernel(const float* zmatch, const float* token, const int* cnt_in,
                                                          int* cnt_out, const int* act, int* flags, int* pos, SegLayout L,
                                                          float width_thr, float conf_thr) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int s = blockIdx.x;
  const int pair = s < L.B ? s : s - L.B;
  const int base = seg_base(L, s), n = cnt_in[s];
  const bool running = act[pair] != 0;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    bool keep = false;
    if (i < n) {
      keep = true;
      if (running) {
        const float prob = 1.f / (1.f + expf(-zmatch[base + i]));  // sigmoid(matchability)
        keep = prob > width_thr;
        if (token) keep = keep || (token[base + i] <= conf_thr);  // low confidence: never pruned
      }
    }
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int off = carry;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    if (i < n) {
      flags[base + i] = keep ? 1 : 0;
      pos[base + i] = off + before;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      carry += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) cnt_out[s] = carry;
}

hipError_t prune_scan(const float* zmatch, const float* token, const int* cnt_in, int* cnt_out, const int* act,
                      int* flags, int* pos, const SegLayout& L, float width_thr, float conf_thr, hipStream_t st) {
  hipLaunchKernelGGL(prune_scan_kernel, dim3(2 * L.B), dim3(1024), 0, st, zmatch, token, cnt_in, cnt_out, act, flags, pos,
                     L, width_thr, conf_thr);
  return hipGetLastError();
}

// four floats per thread (cols % 4 == 0)
__global__ void compact_seg_kernel(const float* src, float* dst, int cols, const int* flags, const int* pos,
                                   const int* cnt_in, SegLayout L) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = cols / 4;
  const int r = (int)(t / q), c = (int)(t % q) * 4;
  if (r >= L.B * (L.M0 + L.N0)) return;
  int local;
  const int s = seg_of_row(L, r, local);
  if (local >= cnt_in[s] || !flags[r]) return;
  const int to = seg_base(L, s) + pos[r];
  *reinterpret_cast<f32x4*>(dst + (size_t)to * cols + c) = *reinterpret_cast<const f32x4*>(src + (size_t)r * cols + c);
}

hipError_t compact_seg(const float* src, float* dst, int cols, const int* flags, const int* pos, const int* cnt_in,
                       const SegLayout& L, hipStream_t st) {
  if (cols % 4) return hipErrorInvalidValue;
  const size_t n = (size_t)L.B * (L.M0 + L.N0) * (cols / 4);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(compact_seg_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst, cols, flags, pos,
                     cnt_in, L);
  return hipGetLastError();
}

__global__ void compact_ind_seg_kernel(const int* ind, int* ind_out, int64_t* prune0, int64_t* prune1, const int* flags,
                                       const int* pos, const int* cnt_in, const int* act, SegLayout L) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= L.B * (L.M0 + L.N0)) return;
  int local;
  const int s = seg_of_row(L, r, local);
  if (local >= cnt_in[s] || !flags[r]) return;
  const int base = seg_base(L, s), orig = ind[r];
  ind_out[base + pos[r]] = orig;
  const int pair = s < L.B ? s : s - L.B;
  if (act[pair]) {  // prune0[:, ind0] += 1 after the selection (lightglue.py:540,546)
    int64_t* pr = s < L.B ? prune0 + (size_t)pair * L.M0 : prune1 + (size_t)pair * L.N0;
    if (pr) pr[orig] += 1;
  }
}

hipError_t compact_ind_seg(const int* ind, int* ind_out, int64_t* prune0, int64_t* prune1, const int* flags,
                           const int* pos, const int* cnt_in, const int* act, const SegLayout& L, hipStream_t st) {
  const int R = L.B * (L.M0 + L.N0);
  if (R == 0) return hipSuccess;
  hipLaunchKernelGGL(compact_ind_seg_kernel, dim3((R + 255) / 256), dim3(256), 0, st, ind, ind_out, prune0, prune1, flags,
                     pos, cnt_in, act, L);
  return hipGetLastError();
}

__global__ void fill_i64_kernel(int64_t* p, int64_t v, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
hipError_t fill_i64(int64_t* p, int64_t v, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_i64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, v, n);
  return hipGetLastError();
}

// Scatter compact matches back to full size (lightglue.py:553-562): one thread per output slot
// of the full [B][M0] / [B][N0] arrays is initialised (-1 / 0) by remap_init; then one thread per
// kept point writes its match through the index arrays
__global__ void remap_init_kernel(int64_t* m0, int64_t* m1, float* s0, float* s1, SegLayout L) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < L.B * L.M0) {
    m0[t] = -1;
    s0[t] = 0.f;
  } else if (t < L.B * (L.M0 + L.N0)) {
    m1[t - L.B * L.M0] = -1;
    s1[t - L.B * L.M0] = 0.f;
  }
}
__global__ void remap_seg_kernel(const int64_t* m0c, const int64_t* m1c, const float* s0c, const float* s1c, const int* ind,
                                 const int* cnt, SegLayout L, int64_t* m0, int64_t* m1, float* s0, float* s1) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= L.B * (L.M0 + L.N0)) return;
  int local;
  const int s = seg_of_row(L, r, local);
  if (local >= cnt[s]) return;
  if (s < L.B) {  // image 0, pair s: compact match -> image-1 original index
    const int b = s;
    const int64_t j = m0c[(size_t)b * L.M0 + local];
    const int* ind1 = ind + seg_base(L, L.B + b);
    m0[(size_t)b * L.M0 + ind[r]] = j == -1 ? -1 : (int64_t)ind1[j];
    s0[(size_t)b * L.M0 + ind[r]] = s0c[(size_t)b * L.M0 + local];
  } else {
    const int b = s - L.B;
    const int64_t j = m1c[(size_t)b * L.N0 + local];
    const int* ind0 = ind + seg_base(L, b);
    m1[(size_t)b * L.N0 + ind[r]] = j == -1 ? -1 : (int64_t)ind0[j];
    s1[(size_t)b * L.N0 + ind[r]] = s1c[(size_t)b * L.N0 + local];
  }
}

hipError_t remap_seg(const int64_t* m0c, const int64_t* m1c, const float* s0c, const float* s1c, const int* ind,
                     const int* cnt, const SegLayout& L, int64_t* m0, int64_t* m1, float* s0, float* s1, hipStream_t st) {
  const int R = L.B * (L.M0 + L.N0);
  if (R == 0) return hipSuccess;
  hipLaunchKernelGGL(remap_init_kernel, dim3((R + 255) / 256), dim3(256), 0, st, m0, m1, s0, s1, L);
  hipLaunchKernelGGL(remap_seg_kernel, dim3((R + 255) / 256), dim3(256), 0, st, m0c, m1c, s0c, s1c, ind, cnt, L, m0, m1,
                     s0, s1);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// Kernel-check helpers (lg_attention): fp32 -> operand planes, plane image -> fp32 rows.
// ----------------------------------------------------------------------------------------
__global__ void split_planes_kernel(const float* x, size_t n, void* planes, int prec, RangeOut ro, bool values) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int eo = prec == PREC_H3 ? range_exponent(ro) : 0;
  float wmax = 0.f;
  if (i < n) {
    const float v = x[i];
    if (prec == PREC_H3) {
      _Float16 h, l;
      if (values) split2h_v(ldexpf(v, -eo), h, l);  // value planes (kernels.h HeadLayout)
      else split2h(ldexpf(v, -eo), h, l);
      wmax = fabsf(v);
      static_cast<_Float16*>(planes)[i] = h;
      static_cast<_Float16*>(planes)[n + i] = l;
    } else {
      __bf16 h, m, l;
      split3(v, h, m, l);
      static_cast<__bf16*>(planes)[i] = h;
      static_cast<__bf16*>(planes)[n + i] = m;
      static_cast<__bf16*>(planes)[2 * n + i] = l;
    }
  }
  if (prec == PREC_H3) range_commit(ro, wmax, eo);
}

hipError_t split_planes(const float* x, size_t n, void* planes, int prec, const RangeOut& ro, hipStream_t st, bool values) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, planes, prec, ro, values);
  return hipGetLastError();
}

__global__ void image_to_rows_kernel(const _Float16* p, long long ps, int rows_pad, int K, float* out, int rows,
                                     const unsigned* tab, int slot) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)rows * K) return;
  const int r = (int)(i / K), c = (int)(i % K);
  const size_t off = plane_off(r, c, rows_pad);
  out[i] = ldexpf((float)p[off] + (float)p[ps + off] * (1.f / kLoScale), range_slot_exp(tab, slot));
}

hipError_t image_to_rows(const _Float16* planes, long long ps, int rows_pad, int K, float* out, int rows,
                         const unsigned* tab, int slot, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const size_t n = (size_t)rows * K;
  hipLaunchKernelGGL(image_to_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, planes, ps, rows_pad, K,
                     out, rows, tab, slot);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// Load-time weight statistics for the run-time range bounds (kernels.h RangeOut)
// ----------------------------------------------------------------------------------------
// out[0] = max_r sum_k |W[r,k]|, out[1] = max |bias| (one block; load time only)
__global__ __launch_bounds__(1024) void weight_range_stats_kernel(const float* W, int rows, int K, const float* bias,
                                                                 float* out) {
  __shared__ float red[2][16];
  float l1max = 0.f, bmax = 0.f;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int r = wave; r < rows; r += 16) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += fabsf(W[(size_t)r * K + k]);
    l1max = fmaxf(l1max, wave_sum(s));
  }
  if (bias)
    for (int r = threadIdx.x; r < rows; r += 1024) bmax = fmaxf(bmax, fabsf(bias[r]));
  bmax = wave_max(bmax);
  if (lane == 0) {
    red[0][wave] = l1max;
    red[1][wave] = bmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < 16; ++w) {
      a = fmaxf(a, red[0][w]);
      b = fmaxf(b, red[1][w]);
    }
    out[0] = a;
    out[1] = b;
  }
}

hipError_t weight_range_stats(const float* W, int rows, int K, const float* bias, float* out, hipStream_t st) {
  hipLaunchKernelGGL(weight_range_stats_kernel, dim3(1), dim3(1024), 0, st, W, rows, K, bias, out);
  return hipGetLastError();
}

// LayerNorm output bound: |(x - mean) / std| <= sqrt(n - 1) for any row, so
// |LN(x)_k| <= |g_k| sqrt(n - 1) + |b_k|; GELU(y) <= |y| (and > -0.17)
__global__ void layernorm_bound_kernel(const float* g, const float* b, int n, float* out) {
  float m = 0.f;
  for (int k = threadIdx.x; k < n; k += 64) m = fmaxf(m, fabsf(g[k]) * sqrtf((float)(n - 1)) + fabsf(b[k]));
  m = wave_max(m);
  if (threadIdx.x == 0) *out = m;
}

hipError_t layernorm_bound(const float* g, const float* b, int n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(layernorm_bound_kernel, dim3(1), dim3(64), 0, st, g, b, n, out);
  return hipGetLastError();
}

}  // namespace lg
