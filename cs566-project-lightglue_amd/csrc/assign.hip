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
#include <cstdlib>
#include <cstring>

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

// Mb / Nb (nullable): per-pair kept counts of a pruned batch; M, N are then the layout capacities
__global__ __launch_bounds__(256) void row_stats_kernel(const float* sim, int B, int M, int N, const int* Mb, const int* Nb,
                                                        float* rmax, float* rlog) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B * M) return;
  const int b = row / M;
  if (Mb && row - b * M >= Mb[b]) return;
  const int ne = Nb ? Nb[b] : N;
  const float* x = sim + (size_t)row * N;
  float m = -INFINITY, s = 0.f;
  if (((N | ne) & 3) == 0) {  // 16-byte loads (the second pass re-reads the 8 KiB row from cache)
    for (int j = 4 * lane; j < ne; j += 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
      m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    }
    m = wave_max(m);
    for (int j = 4 * lane; j < ne; j += 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
      s += (expf(v[0] - m) + expf(v[1] - m)) + (expf(v[2] - m) + expf(v[3] - m));
    }
  } else {
    for (int j = lane; j < ne; j += 64) m = fmaxf(m, x[j]);
    m = wave_max(m);
    for (int j = lane; j < ne; j += 64) s += expf(x[j] - m);
  }
  s = wave_sum(s);
  if (lane == 0) { rmax[row] = m; rlog[row] = logf(s); }
}

// Column statistics of one 64-row chunk in a single read: running (max, sum of exp(x - max))
// per column, rescaled when the max rises (rare after the first rows).
__global__ __launch_bounds__(256) void col_stats_partial_kernel(const float* sim, int M, int N, const int* Mb,
                                                                const int* Nb, float* pmax, float* psum) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y, b = blockIdx.z;
  const int nch = gridDim.y;
  if (j >= (Nb ? Nb[b] : N)) return;
  const int i0 = ch * CCH, i1 = min(Mb ? Mb[b] : M, i0 + CCH);
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
__global__ void col_stats_combine_kernel(const float* pmax, const float* psum, int nch, int N, int BN, const int* Nb,
                                         float* cmax, float* clog) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BN) return;
  const int b = t / N, j = t - b * N;
  if (Nb && j >= Nb[b]) return;
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
                                                       int N, const int* Mb, const int* Nb) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B * M) return;
  const int b = row / M, i = row - b * M;
  if (Mb && i >= Mb[b]) return;
  const int ne = Nb ? Nb[b] : N;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  float* lr = la ? la + ((size_t)b * (M + 1) + i) * (N + 1) : nullptr;
  for (int j = lane; j < ne; j += 64) {
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
    if (lr) lr[ne] = log_sigmoid(-z0[row]);
  }
}

__global__ void la_last_row_kernel(const float* z1, float* la, int B, int M, int N, const int* Mb, const int* Nb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * (N + 1)) return;
  const int b = t / (N + 1), j = t - b * (N + 1);
  const int me = Mb ? Mb[b] : M, ne = Nb ? Nb[b] : N;
  if (j > ne) return;
  la[((size_t)b * (M + 1) + me) * (N + 1) + j] = j < ne ? log_sigmoid(-z1[b * N + j]) : 0.f;
}

template <bool FROM_LA>
__global__ __launch_bounds__(256) void col_arg_partial_kernel(const float* src, Stats st, int M, int N, const int* Mb,
                                                              const int* Nb) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y, b = blockIdx.z, nch = gridDim.y;
  if (j >= (Nb ? Nb[b] : N)) return;
  const int i0 = ch * CCH, i1 = min(Mb ? Mb[b] : M, i0 + CCH);
  float best = -INFINITY;
  int bi = i0;
  for (int i = i0; i < i1; ++i) {
    const float v = score_at<FROM_LA>(src, st, b, i, j, M, N);
    if (v > best) { best = v; bi = i; }
  }
  st.pv[((size_t)b * nch + ch) * N + j] = best;
  st.pi[((size_t)b * nch + ch) * N + j] = bi;
}

__global__ void col_arg_combine_kernel(Stats st, int nch, int N, int BN, const int* Nb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BN) return;
  const int b = t / N, j = t - b * N;
  if (Nb && j >= Nb[b]) return;
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
__global__ void filter_kernel(Stats st, int B, int M, int N, float th, int64_t* m0, int64_t* m1, float* s0, float* s1,
                              const int* Mb, const int* Nb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < B * M) {
    const int b = t / M, i = t - b * M;
    if (Mb && i >= Mb[b]) return;
    const int j = st.arg0[t];
    const bool mutual = st.arg1[b * N + j] == i;
    const float sc = mutual ? expf(st.max0[t]) : 0.f;
    const bool valid = mutual && sc > th;
    m0[t] = valid ? (int64_t)j : -1;
    s0[t] = sc;
  } else if (t < B * M + B * N) {
    const int u = t - B * M;
    const int b = u / N, j = u - b * N;
    if (Nb && j >= Nb[b]) return;
    const int i = st.arg1[u];
    const bool mutual = st.arg0[b * M + i] == j;  // then row i is mutual too
    const float sc = mutual ? expf(st.max0[b * M + i]) : 0.f;
    const bool valid = mutual && sc > th;         // valid0[m1[j]] (lightglue.py:334)
    m1[u] = valid ? (int64_t)i : -1;
    s1[u] = sc;
  }
}


// ------------------------------------------------------------------ fused passes (N % 4 == 0,
// N <= 2048: the main path).  A workgroup of 8 waves owns one 64-row chunk of one pair (wave w:
// rows 8w .. 8w+7 of the chunk), so its column partials have exactly the [B][nch][N] layout the
// combine kernels above read.
//   stats pass: ONE read of sim for both softmax directions -- a wave holds a row in registers
//     (row max, then sum of exp(x - max): row_stats_kernel's formula) and folds it into running
//     (max, sum) column pairs; the 8 waves merge through LDS (col_stats_combine finishes)
//   la pass:    ONE read of sim for the la write, the row argmax and the column argmax partials
//     (running first-index best per column, merged across waves in row order)
// The old path (row_stats + col_stats_partial, row_pass + col_arg_partial: four reads) serves
// other N.
namespace {
constexpr int kAsW = 8;          // waves per workgroup (CCH / kAsW = 8 rows each)
constexpr int kAsMaxN = 2048;

__device__ __forceinline__ void lse_merge_pair(float& am, float& as, float bm, float bs) {
  const float m = fmaxf(am, bm);
  const float ea = am == m ? 1.f : expf(am - m);
  const float eb = bm == m ? 1.f : expf(bm - m);
  as = as * ea + bs * eb;
  am = m;
}
}  // namespace

template <int K4>
__global__ __launch_bounds__(kAsW * 64) void stats_fused_kernel(const float* __restrict__ sim, int M, int N, float* rmax,
                                                                float* rlog, float* pmax, float* psum) {
  __shared__ float2 mb[kAsW / 2][kAsMaxN];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ch = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  float cm[K4][4], cs[K4][4];
#pragma unroll
  for (int k = 0; k < K4; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) cm[k][e] = -INFINITY, cs[k][e] = 0.f;
  const int r0 = ch * CCH + wave * (CCH / kAsW);
  const int r1 = min(M, r0 + CCH / kAsW);
  auto c_ok = [&](int k, int e) { return 256 * k + 4 * lane + e < N; };
#pragma unroll 1
  for (int i = r0; i < r1; ++i) {
    const char* row = reinterpret_cast<const char*>(sim + ((size_t)b * M + i) * N);
    f32x4 x[K4];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int c = 256 * k + 4 * lane;
      x[k] = c < N ? *reinterpret_cast<const f32x4*>(row + 1024 * k + (uint32_t)(16 * lane))
                   : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      m = fmaxf(m, fmaxf(fmaxf(x[k][0], x[k][1]), fmaxf(x[k][2], x[k][3])));
    }
    m = wave_max_dpp(m);
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < K4; ++k) sum += (expf(x[k][0] - m) + expf(x[k][1] - m)) + (expf(x[k][2] - m) + expf(x[k][3] - m));
    sum = wave_sum_dpp(sum);
    if (lane == 0) {
      rmax[(size_t)b * M + i] = m;
      rlog[(size_t)b * M + i] = logf(sum);
    }
#pragma unroll
    for (int k = 0; k < K4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // running (max, sum) with one exponential: e^-|v - max|
        const float v = x[k][e];
        const float d = v - cm[k][e];
        const float t = expf(-fabsf(d));
        if (d > 0.f) {
          cs[k][e] = fmaf(cs[k][e], t, 1.f);
          cm[k][e] = v;
        } else if (c_ok(k, e)) {
          cs[k][e] += t;
        }
      }
  }
#pragma unroll
  for (int half = kAsW / 2; half >= 1; half >>= 1) {
    if (wave >= half && wave < 2 * half) {
#pragma unroll
      for (int k = 0; k < K4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 256 * k + 4 * lane + e;
          if (c < N) mb[wave - half][c] = make_float2(cm[k][e], cs[k][e]);
        }
    }
    __syncthreads();
    if (wave < half) {
#pragma unroll
      for (int k = 0; k < K4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 256 * k + 4 * lane + e;
          if (c < N) {
            const float2 o = mb[wave][c];
            lse_merge_pair(cm[k][e], cs[k][e], o.x, o.y);
          }
        }
    }
    __syncthreads();
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < K4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 256 * k + 4 * lane + e;
        if (c < N) {
          pmax[((size_t)b * nch + ch) * N + c] = cm[k][e];
          psum[((size_t)b * nch + ch) * N + c] = cs[k][e];
        }
      }
  }
}

// la row write + row argmax + column argmax partials; lane columns 256 k + 4 lane + e (16-byte
// sim loads and LDS column-stat reads; the la rows are N+1 long, so their stores stay scalar)
template <int K4>
__global__ __launch_bounds__(kAsW * 64) void la_fused_kernel(const float* __restrict__ sim, Stats st,
                                                             const float* __restrict__ z0, float* la, int M, int N) {
  __shared__ __attribute__((aligned(16))) float cst[3][kAsMaxN];  // cmax, clog, ls1 of this pair
  __shared__ float mbv[kAsW / 2][kAsMaxN];
  __shared__ int mbi[kAsW / 2][kAsMaxN];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ch = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  for (int j = tid; j < N; j += kAsW * 64) {
    cst[0][j] = st.cmax[(size_t)b * N + j];
    cst[1][j] = st.clog[(size_t)b * N + j];
    cst[2][j] = st.ls1[(size_t)b * N + j];
  }
  __syncthreads();
  const int r0 = ch * CCH + wave * (CCH / kAsW);
  const int r1 = min(M, r0 + CCH / kAsW);
  float cb[K4][4];  // col_arg_partial_kernel's scan: best = -inf, index = first row, strict >
  int ci[K4][4];
#pragma unroll
  for (int k = 0; k < K4; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[k][e] = -INFINITY, ci[k][e] = r0;
#pragma unroll 1
  for (int i = r0; i < r1; ++i) {
    const int ri = b * M + i;
    const float rm = st.rmax[ri], rl = st.rlog[ri], l0 = st.ls0[ri];
    const char* row = reinterpret_cast<const char*>(sim + (size_t)ri * N);
    float* lr = la ? la + ((size_t)b * (M + 1) + i) * (N + 1) : nullptr;
    f32x4 xv[K4];
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int c = 256 * k + 4 * lane;
      xv[k] = c < N ? *reinterpret_cast<const f32x4*>(row + 1024 * k + (uint32_t)(16 * lane)) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int c = 256 * k + 4 * lane;
      if (c < N) {
        const f32x4 cmx = *reinterpret_cast<const f32x4*>(&cst[0][c]);
        const f32x4 clg = *reinterpret_cast<const f32x4*>(&cst[1][c]);
        const f32x4 l1 = *reinterpret_cast<const f32x4*>(&cst[2][c]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // score_at<false>: same operations in the same order
          const float s0 = (xv[k][e] - rm) - rl;
          const float s1 = (xv[k][e] - cmx[e]) - clg[e];
          const float v = (s0 + s1) + (l0 + l1[e]);
          if (lr) lr[c + e] = v;
          if (bi == 0x7fffffff || v > best) { best = v; bi = c + e; }
          if (v > cb[k][e]) { cb[k][e] = v; ci[k][e] = i; }
        }
      }
    }
    wave_argmax_dpp(best, bi);
    if (lane == 0) {
      st.max0[ri] = best;
      st.arg0[ri] = bi;
      if (lr) lr[N] = log_sigmoid(-z0[ri]);
    }
  }
  // merge waves (wave w + half holds later rows: it wins only with a strictly greater value)
#pragma unroll
  for (int half = kAsW / 2; half >= 1; half >>= 1) {
    if (wave >= half && wave < 2 * half) {
#pragma unroll
      for (int k = 0; k < K4; ++k) {
        const int c = 256 * k + 4 * lane;
        if (c < N) {
          *reinterpret_cast<f32x4*>(&mbv[wave - half][c]) = f32x4{cb[k][0], cb[k][1], cb[k][2], cb[k][3]};
          *reinterpret_cast<int4*>(&mbi[wave - half][c]) = make_int4(ci[k][0], ci[k][1], ci[k][2], ci[k][3]);
        }
      }
    }
    __syncthreads();
    if (wave < half) {
#pragma unroll
      for (int k = 0; k < K4; ++k) {
        const int c = 256 * k + 4 * lane;
        if (c < N) {
          const f32x4 ov = *reinterpret_cast<const f32x4*>(&mbv[wave][c]);
          const int4 oi = *reinterpret_cast<const int4*>(&mbi[wave][c]);
          const int oa[4] = {oi.x, oi.y, oi.z, oi.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ov[e] > cb[k][e]) { cb[k][e] = ov[e]; ci[k][e] = oa[e]; }
        }
      }
    }
    __syncthreads();
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int c = 256 * k + 4 * lane;
      if (c < N) {
        *reinterpret_cast<f32x4*>(st.pv + ((size_t)b * nch + ch) * N + c) = f32x4{cb[k][0], cb[k][1], cb[k][2], cb[k][3]};
        *reinterpret_cast<int4*>(st.pi + ((size_t)b * nch + ch) * N + c) = make_int4(ci[k][0], ci[k][1], ci[k][2], ci[k][3]);
      }
    }
  }
}

template <int K4>
static void launch_assign_fused(const AssignArgs& a, const Stats& s, int nch, float* psum, hipStream_t st) {
  const dim3 grid(nch, a.B), block(kAsW * 64);
  hipLaunchKernelGGL((stats_fused_kernel<K4>), grid, block, 0, st, a.sim, a.M, a.N, s.rmax, s.rlog, s.pv, psum);
}
template <int T>
static void launch_la_fused(const AssignArgs& a, const Stats& s, int nch, hipStream_t st) {
  const dim3 grid(nch, a.B), block(kAsW * 64);
  hipLaunchKernelGGL((la_fused_kernel<T>), grid, block, 0, st, a.sim, s, a.z0, a.la, a.M, a.N);
}

#ifndef LG_ASSIGN_FUSED
#define LG_ASSIGN_FUSED 1
#endif

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
                                    float th, int64_t* m0, int64_t* m1, float* s0, float* s1, hipStream_t st,
                                    const int* Mb = nullptr, const int* Nb = nullptr) {
  const int nch = (M + CCH - 1) / CCH;
  hipLaunchKernelGGL((row_pass_kernel<FROM_LA>), dim3((B * M + 3) / 4), dim3(256), 0, st, src, s, z0, la, B, M, N, Mb, Nb);
  hipLaunchKernelGGL((col_arg_partial_kernel<FROM_LA>), dim3((N + 255) / 256, nch, B), dim3(256), 0, st, src, s, M, N, Mb,
                     Nb);
  hipLaunchKernelGGL(col_arg_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s, nch, N, B * N, Nb);
  hipLaunchKernelGGL(filter_kernel, dim3((B * (M + N) + 255) / 256), dim3(256), 0, st, s, B, M, N, th, m0, m1, s0, s1, Mb,
                     Nb);
  return hipGetLastError();
}

hipError_t assign_and_filter(const AssignArgs& a, hipStream_t st) {
  const int B = a.B, M = a.M, N = a.N;
  if (B * M == 0 || B * N == 0) return hipErrorInvalidValue;
  const Stats s = carve(a.ws, B, M, N);
  const int nch = (M + CCH - 1) / CCH;
  float* psum = reinterpret_cast<float*>(s.pi);  // the argmax index partials are not live yet
  // per-pair counts (pruned batches) take the four-read kernels, which bound every loop by them
  const bool fused = LG_ASSIGN_FUSED && !a.Mb && N % 4 == 0 && N <= kAsMaxN && !getenv("LG_ASSIGN_UNFUSED");
  if (fused) {
    const int k4 = (N + 255) / 256;
    if (k4 <= 1) launch_assign_fused<1>(a, s, nch, psum, st);
    else if (k4 <= 2) launch_assign_fused<2>(a, s, nch, psum, st);
    else if (k4 <= 4) launch_assign_fused<4>(a, s, nch, psum, st);
    else launch_assign_fused<8>(a, s, nch, psum, st);
  } else {
    hipLaunchKernelGGL(row_stats_kernel, dim3((B * M + 3) / 4), dim3(256), 0, st, a.sim, B, M, N, a.Mb, a.Nb, s.rmax,
                       s.rlog);
    const dim3 cg((N + 255) / 256, nch, B);
    hipLaunchKernelGGL(col_stats_partial_kernel, cg, dim3(256), 0, st, a.sim, M, N, a.Mb, a.Nb, s.pv, psum);
  }
  hipLaunchKernelGGL(col_stats_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s.pv, psum, nch, N, B * N,
                     a.Nb, s.cmax, s.clog);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * M + 255) / 256), dim3(256), 0, st, a.z0, s.ls0, B * M);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, a.z1, s.ls1, B * N);
  if (a.la)
    hipLaunchKernelGGL(la_last_row_kernel, dim3((B * (N + 1) + 255) / 256), dim3(256), 0, st, a.z1, a.la, B, M, N, a.Mb,
                       a.Nb);
  if (fused) {
    const int k4 = (N + 255) / 256;
    if (k4 <= 1) launch_la_fused<1>(a, s, nch, st);
    else if (k4 <= 2) launch_la_fused<2>(a, s, nch, st);
    else if (k4 <= 4) launch_la_fused<4>(a, s, nch, st);
    else launch_la_fused<8>(a, s, nch, st);
    hipLaunchKernelGGL(col_arg_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s, nch, N, B * N, nullptr);
    hipLaunchKernelGGL(filter_kernel, dim3((B * (M + N) + 255) / 256), dim3(256), 0, st, s, B, M, N, a.th, a.m0, a.m1,
                       a.s0, a.s1, nullptr, nullptr);
    return hipGetLastError();
  }
  return argmax_and_filter<false>(a.sim, s, a.z0, a.la, B, M, N, a.th, a.m0, a.m1, a.s0, a.s1, st, a.Mb, a.Nb);
}

// similarity recomputed in two fp16x3 GEMM passes (assign_h3.hip) instead of materialised
hipError_t assign_and_filter_h3(const AssignArgs& a, const PlaneRef& md, const unsigned* rtab, int slot, hipStream_t st) {
  const int B = a.B, M = a.M, N = a.N;
  if (B * M == 0 || B * N == 0 || a.Mb || !sim_h3_supported(M, N)) return hipErrorInvalidValue;
  const Stats s = carve(a.ws, B, M, N);
  const int ntm = (M + 255) / 256;
  float* extra = a.ws + ((assign_workspace_floats(B, M, N) + 63) & ~size_t(63));
  SimH3Args g;
  memset(&g, 0, sizeof(g));
  g.P = md;
  g.rtab = rtab;
  g.slot = slot;
  g.B = B;
  g.M = M;
  g.N = N;
  g.rowp = reinterpret_cast<float2*>(extra);
  g.pmax = s.pv;
  g.psum = reinterpret_cast<float*>(s.pi);  // the argmax index partials are not live yet
  hipError_t e = sim_h3_pass(g, 0, st);
  if (e != hipSuccess) return e;
  g.rmax = s.rmax;
  g.rlog = s.rlog;
  if ((e = sim_row_stats(g, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(col_stats_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s.pv, g.psum, ntm, N, B * N,
                     nullptr, s.cmax, s.clog);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * M + 255) / 256), dim3(256), 0, st, a.z0, s.ls0, B * M);
  hipLaunchKernelGGL(logsig_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, a.z1, s.ls1, B * N);
  if (a.la)
    hipLaunchKernelGGL(la_last_row_kernel, dim3((B * (N + 1) + 255) / 256), dim3(256), 0, st, a.z1, a.la, B, M, N, nullptr,
                       nullptr);
  g.ls0 = s.ls0;
  g.cmax = s.cmax;
  g.clog = s.clog;
  g.ls1 = s.ls1;
  g.la = a.la;
  g.rbest = extra;
  g.rbi = reinterpret_cast<int*>(extra + (size_t)B * M * ((N + 255) / 256));
  g.pv = s.pv;
  g.pi = s.pi;
  if ((e = sim_h3_pass(g, 1, st)) != hipSuccess) return e;
  if ((e = sim_row_arg(g, a.z0, s.max0, s.arg0, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(col_arg_combine_kernel, dim3((B * N + 255) / 256), dim3(256), 0, st, s, ntm, N, B * N, nullptr);
  hipLaunchKernelGGL(filter_kernel, dim3((B * (M + N) + 255) / 256), dim3(256), 0, st, s, B, M, N, a.th, a.m0, a.m1, a.s0,
                     a.s1, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t filter_from_scores(const float* scores, int B, int M, int N, float th, float* ws, int64_t* m0, int64_t* m1,
                              float* s0, float* s1, hipStream_t st) {
  if (B * M == 0 || B * N == 0) return hipErrorInvalidValue;
  const Stats s = carve(ws, B, M, N);
  return argmax_and_filter<true>(scores, s, nullptr, nullptr, B, M, N, th, m0, m1, s0, s1, st);
}

}  // namespace lg
