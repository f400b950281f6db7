// Dual-softmax assignment and mutual-nearest-neighbour filter (gfx950).
//
//   sigmoid_log_double_softmax  lightglue.py:284-296
//     la[i,j] = (sim-rmax_i-rlog_i) + (sim-cmax_j-clog_j) + (logsig(z0_i) + logsig(z1_j))
//     la[i,N] = logsig(-z0_i), la[M,j] = logsig(-z1_j), la[M,N] = 0
//   filter_matches              lightglue.py:321-337 (== superglue.py:288-298)
//
// All passes stream the [B,M,N] similarity (HBM/Infinity-Cache bound, no MFMA):
//   row stats   one wave per row (max, then sum of exp(x - max); 16-byte loads)
//   col stats   256 columns x a 64-row chunk per workgroup, one read: running (max, sum) per
//               column -> per-chunk partials, combined in chunk order
//   row pass    one wave per row: the la value, written once, and the row argmax
//   col argmax  per-chunk partial (value, first index) -> combine
//   filter      one thread per keypoint
// Ties resolve to the smallest index, as torch-CPU max(dim) does.
#include "common.h"
#include "kernels.h"

namespace lg {

constexpr int CCH = 64;  // rows per column-chunk

struct Stats {
  float* rmax; float* rlog;   // [B*M]
  float* cmax; float* clog;   // [B*N]
  float* ls0; float* ls1;     // logsigmoid(z0), logsigmoid(z1)
  float* pv; int* pi;         // column partials [B][nch][N]
  float* max0; int* arg0;     // row best value / index [B*M]
  float* max1; int* arg1;     // col best [B*N]
};

// Score provider: either computed from sim + stats (fused la construction) or read from an
// existing [B][M+1][N+1] log-assignment.
template <bool FROM_LA>
__device__ __forceinline__ float score_at(const float* src, const Stats& st, int b, int i, int j, int M, int N) {
  if constexpr (FROM_LA) {
    return src[((size_t)b * (M + 1) + i) * (N + 1) + j];
  } else {
    const float x = src[((size_t)b * M + i) * N + j];
    const int ri = b * M + i, cj = b * N + j;
    const float s0 = (x - st.rmax[ri]) - st.rlog[ri];
    const float s1 = (x - st.cmax[cj]) - st.clog[cj];
    return (s0 + s1) + (st.ls0[ri] + st.ls1[cj]);
  }
}

__global__ __launch_bounds__(256) void row_stats_kernel(const float* sim, int rows, int N, float* rmax, float* rlog) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* x = sim + (size_t)row * N;
  float m = -INFINITY, s = 0.f;
  if ((N & 3) == 0) {  // 16-byte loads (the second pass re-reads the 8 KiB row from cache)
    for (int j = 4 * lane; j < N; j += 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
      m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    }
    m = wave_max(m);
    for (int j = 4 * lane; j < N; j += 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
      s += (expf(v[0] - m) + expf(v[1] - m)) + (expf(v[2] - m) + expf(v[3] - m));
    }
  } else {
    for (int j = lane; j < N; j += 64) m = fmaxf(m, x[j]);
    m = wave_max(m);
    for (int j = lane; j < N; j += 64) s += expf(x[j] - m);
  }
  s = wave_sum(s);
  if (lane == 0) { rmax[row] = m; rlog[row] = logf(s); }
}

// Column statistics of one 64-row chunk in a single read: running (max, sum of exp(x - max))
// per column, rescaled when the max rises (rare after the first rows).
__global__ __launch_bounds__(256) void col_stats_partial_kernel(const float* sim, int M, int N, float* pmax,
                                                                float* psum) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y, b = blockIdx.z;
  const int nch = gridDim.y;
  if (j >= N) return;
  const int i0 = ch * CCH, i1 = min(M, i0 + CCH);
  const float* x = sim + (size_t)b * M * N + j;
  float m = -INFINITY, acc = 0.f;
  for (int i = i0; i < i1; ++i) {
    const float v = x[(size_t)i * N];
    if (v > m) {
      acc = acc * expf(m - v) + 1.f;
      m = v;
    } else {
      acc += expf(v - m);
    }
  }
  pmax[((size_t)b * nch + ch) * N + j] = m;
  psum[((size_t)b * nch + ch) * N + j] = acc;
}

// combine the chunk partials in chunk order: cmax = max_c m_c, clog = log(sum_c s_c exp(m_c - cmax))
__global__ void col_stats_combine_kernel(const float* pmax, const float* psum, int nch, int N, int BN, float* cmax,
                                         float* clog) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BN) return;
  const int b = t / N, j = t - b * N;
  const float* pm = pmax + (size_t)b * nch * N + j;
  const float* pv = psum + (size_t)b * nch * N + j;
  float m = -INFINITY;
  for (int c = 0; c < nch; ++c) m = fmaxf(m, pm[(size_t)c * N]);
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += pv[(size_t)c * N] * expf(pm[(size_t)c * N] - m);
  cmax[t] = m;
  clog[t] = logf(s);
}

__global__ void logsig_kernel(const float* z, float* ls, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ls[i] = log_sigmoid(z[i]);
}

// One wave per row: la row write (optional) + row max / first argmax of the inner block.
template <bool FROM_LA>
__global__ __launch_bounds__(256) void row_pass_kernel(const float* src, Stats st, const float* z0, float* la, int B, int M,
                                                       int N) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B * M) return;
  const int b = row / M, i = row - b * M;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  float* lr = la ? la + ((size_t)b * (M + 1) + i) * (N + 1) : nullptr;
  for (int j = lane; j < N; j += 64) {
    const float v = score_at<FROM_LA>(src, st, b, i, j, M, N);
    if (lr) lr[j] = v;
    if (bi == 0x7fffffff || v > best) { best = v; bi = j; }
  }
  // wave arg-max, ties -> smaller index
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) {
    st.max0[row] = best;
    st.arg0[row] = bi;
    if (lr) lr[N] = log_sigmoid(-z0[row]);
  }
}

__global__ void la_last_row_kernel(const float* z1, float* la, int B, int M, int N) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * (N + 1)) return;
  const int b = t / (N + 1), j = t - b * (N + 1);
  la[((size_t)b * (M + 1) + M) * (N + 1) + j] = j < N ? log_sigmoid(-z1[b * N + j]) : 0.f;
}

template <bool FROM_LA>
__global__ __launch_bounds__(256) void col_arg_partial_kernel(const float* src, Stats st, int M, int N) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y, b = blockIdx.z, nch = gridDim.y;
  if (j >= N) return;
  const int i0 = ch * CCH, i1 = min(M, i0 + CCH);
  float best = -INFINITY;
  int bi = i0;
  for (int i = i0; i < i1; ++i) {
    const float v = score_at<FROM_LA>(src, st, b, i, j, M, N);
    if (v > best) { best = v; bi = i; }
  }
  st.pv[((size_t)b * nch + ch) * N + j] = best;
  st.pi[((size_t)b * nch + ch) * N + j] = bi;
}

__global__ void col_arg_combine_kernel(Stats st, int nch, int N, int BN) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BN) return;
  const int b = t / N, j = t - b * N;
  float best = st.pv[(size_t)b * nch * N + j];
  int bi = st.pi[(size_t)b * nch * N + j];
  for (int c = 1; c < nch; ++c) {
    const float v = st.pv[((size_t)b * nch + c) * N + j];
    if (v > best) { best = v; bi = st.pi[((size_t)b * nch + c) * N + j]; }
  }
  st.max1[t] = best;
  st.arg1[t] = bi;
}

// filter_matches: mutual check, exp(max0), threshold, -1 for invalid.
__global__ void filter_kernel(Stats st, int B, int M, int N, float th, int64_t* m0, int64_t* m1, float* s0, float* s1) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < B * M) {
    const int b = t / M, i = t - b * M;
    const int j = st.arg0[t];
    const bool mutual = st.arg1[b * N + j] == i;
    const float sc = mutual ? expf(st.max0[t]) : 0.f;
    const bool valid = mutual && sc > th;
    m0[t] = valid ? (int64_t)j : -1;
    s0[t] = sc;
  } else if (t < B * M + B * N) {
    const int u = t - B * M;
    const int b = u / N, j = u - b * N;
    const int i = st.arg1[u];
    const bool mutual = st.arg0[b * M + i] == j;  // then row i is mutual too
    const float sc = mutual ? expf(st.max0[b * M + i]) : 0.f;
    const bool valid = mutual && sc > th;         // valid0[m1[j]] (lightglue.py:334)
    m1[u] = valid ? (int64_t)i : -1;
    s1[u] = sc;
  }
}

static Stats carve(float* ws, int B, int M, int N) {
  const int nch = (M + CCH - 1) / CCH;
  Stats s;
  float* p = ws;
  auto take = [&](size_t n) { float* r = p; p += (n + 63) & ~size_t(63); return r; };
  s.rmax = take((size_t)B * M); s.rlog = take((size_t)B * M);
  s.cmax = take((size_t)B * N); s.clog = take((size_t)B * N);
  s.ls0 = take((size_t)B * M); s.ls1 = take((size_t)B * N);
  s.pv = take((size_t)B * nch * N); s.pi = reinterpret_cast<int*>(take((size_t)B * nch * N));
  s.max0 = take((size_t)B * M); s.arg0 = reinterpret_cast<int*>(take((size_t)B * M));
  s.max1 = take((size_t)B * N); s.arg1 = reinterpret_cast<int*>(take((size_t)B * N));
  return s;
}

size_t assign_workspace_floats(int B, int M, int N) {
  const size_t nch = (M + CCH - 1) / CCH;
  auto r = [](size_t n) { return (n + 63) & ~size_t(63); };
  return 5 * r((size_t)B * M) + 5 * r((size_t)B * N) + 2 * r((size_t)B * nch * N) + 64;
}
size_t filter_workspace_floats(int B, int M, int N) { return assign_workspace_floats(B, M, N); }

template <bool FROM_LA>
static hipError_t argmax_and_filter(const float* src, const Stats& s, const float* z0, float* la, int B, int M, int N,
                                    float th, int64_t* m0, int64_t* m1, float* s0, float* s1, hipStream_t st) {
  const int nch = (M + CCH - 1) / CCH;
  hipLaunchKernelGGL((row_pass_kernel<FROM_LA>), dim3((B * M + 3) / 4), dim3(256), 0, st, src, s, z0, la, B, M, N);
  hipLaunchKernelGGL((col_arg_partial_kernel<FROM_LA>), dim3((N + 255) / 256, nch, B), dim3(256), 0, st, src, s, M, N);
  hipLaunchKernelGGL(col_arg_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s, nch, N, B * N);
  hipLaunchKernelGGL(filter_kernel, dim3((B * (M + N) + 255) / 256), dim3(256), 0, st, s, B, M, N, th, m0, m1, s0, s1);
  return hipGetLastError();
}

hipError_t assign_and_filter(const AssignArgs& a, hipStream_t st) {
  const int B = a.B, M = a.M, N = a.N;
  if (B * M == 0 || B * N == 0) return hipErrorInvalidValue;
  const Stats s = carve(a.ws, B, M, N);
  const int nch = (M + CCH - 1) / CCH;
  hipLaunchKernelGGL(row_stats_kernel, dim3((B * M + 3) / 4), dim3(256), 0, st, a.sim, B * M, N, s.rmax, s.rlog);
  const dim3 cg((N + 255) / 256, nch, B);
  float* psum = reinterpret_cast<float*>(s.pi);  // the argmax index partials are not live yet
  hipLaunchKernelGGL(col_stats_partial_kernel, cg, dim3(256), 0, st, a.sim, M, N, s.pv, psum);
  hipLaunchKernelGGL(col_stats_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s.pv, psum, nch, N, B * N,
                     s.cmax, s.clog);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * M + 255) / 256), dim3(256), 0, st, a.z0, s.ls0, B * M);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, a.z1, s.ls1, B * N);
  if (a.la) hipLaunchKernelGGL(la_last_row_kernel, dim3((B * (N + 1) + 255) / 256), dim3(256), 0, st, a.z1, a.la, B, M, N);
  return argmax_and_filter<false>(a.sim, s, a.z0, a.la, B, M, N, a.th, a.m0, a.m1, a.s0, a.s1, st);
}

hipError_t filter_from_scores(const float* scores, int B, int M, int N, float th, float* ws, int64_t* m0, int64_t* m1,
                              float* s0, float* s1, hipStream_t st) {
  if (B * M == 0 || B * N == 0) return hipErrorInvalidValue;
  const Stats s = carve(ws, B, M, N);
  return argmax_and_filter<true>(scores, s, nullptr, nullptr, B, M, N, th, m0, m1, s0, s1, st);
}

}  // namespace lg
