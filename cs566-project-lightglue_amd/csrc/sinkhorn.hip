// Log-domain Sinkhorn with a dustbin (gfx950) — superglue.py:173-201 log_optimal_transport.
//
//   Zc = [[scores, alpha], [alpha, alpha]]            [B, M+1, N+1]
//   log_mu = [-log(M+N)] * M ++ [log N - log(M+N)],  log_nu likewise with M
//   iters x { u = log_mu - LSE_j(Zc + v);  v = log_nu - LSE_i(Zc + u) }
//   out = Zc + u + v + log(M+N)
//
// Both half-steps are row reductions: the u-step walks rows of `scores`, the v-step walks rows
// of a transposed copy made once (tiled LDS transpose), so every pass is a coalesced stream.
// One wave per row; the two-pass max-then-sum LSE mirrors torch.logsumexp's formulation.
// HBM/Infinity-Cache bound: per iteration 2 x B*M*N*4 bytes are read.
#include "common.h"
#include "kernels.h"

namespace lg {

__global__ __launch_bounds__(256) void transpose_kernel(const float* src, float* dst, int M, int N) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const float* s = src + (size_t)b * M * N;
  float* d = dst + (size_t)b * M * N;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int i = i0 + r, j = j0 + tx;
    if (i < M && j < N) tile[r][tx] = s[(size_t)i * N + j];
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int j = j0 + r, i = i0 + tx;
    if (i < M && j < N) d[(size_t)j * M + i] = tile[tx][r];
  }
}

// One Sinkhorn half-step over `rows`+1 rows of length `cols`+1 (last row / column = dustbin).
// src: [B][rows][cols] real scores; other: the opposite potential [B][cols+1]; out: [B][rows+1].
__global__ __launch_bounds__(256) void lse_step_kernel(const float* src, const float* other, float* out, int B, int rows,
                                                       int cols, float alpha, float lm_in, float lm_bin) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= B * (rows + 1)) return;
  const int b = r / (rows + 1), i = r - b * (rows + 1);
  const float* o = other + (size_t)b * (cols + 1);
  const float* x = src + ((size_t)b * rows + i) * cols;
  const bool bin_row = i == rows;
  float m = -INFINITY;
  for (int j = lane; j <= cols; j += 64) {
    const float z = (bin_row || j == cols) ? alpha : x[j];
    m = fmaxf(m, z + o[j]);
  }
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j <= cols; j += 64) {
    const float z = (bin_row || j == cols) ? alpha : x[j];
    s += expf((z + o[j]) - m);
  }
  s = wave_sum(s);
  if (lane == 0) {
    const float lse = (m == -INFINITY) ? m : m + logf(s);
    out[r] = (bin_row ? lm_bin : lm_in) - lse;
  }
}

__global__ void sinkhorn_out_kernel(const float* scores, const float* u, const float* v, float* Z, int B, int M, int N,
                                    float alpha, float norm) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t per = (size_t)(M + 1) * (N + 1);
  if (t >= (size_t)B * per) return;
  const int b = (int)(t / per);
  const int rem = (int)(t - (size_t)b * per);
  const int i = rem / (N + 1), j = rem - i * (N + 1);
  const float z = (i < M && j < N) ? scores[((size_t)b * M + i) * N + j] : alpha;
  Z[t] = ((z + u[b * (M + 1) + i]) + v[b * (N + 1) + j]) - norm;
}

size_t sinkhorn_workspace_floats(int B, int M, int N) {
  return (size_t)B * M * N + (size_t)B * (M + 1) + (size_t)B * (N + 1) + 256;
}

hipError_t log_optimal_transport(const float* scores, float alpha, int B, int M, int N, int iters, float* Z, float* ws,
                                 hipStream_t st) {
  if (B == 0) return hipSuccess;
  float* sT = ws;
  float* u = sT + (size_t)B * M * N;
  float* v = u + (size_t)B * (M + 1) + 64;
  hipError_t e;
  if ((e = hipMemsetAsync(u, 0, sizeof(float) * B * (M + 1), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(v, 0, sizeof(float) * B * (N + 1), st)) != hipSuccess) return e;
  if (M > 0 && N > 0)
    hipLaunchKernelGGL(transpose_kernel, dim3((N + 63) / 64, (M + 63) / 64, B), dim3(256), 0, st, scores, sT, M, N);
  // log_mu / log_nu (superglue.py:194-197), computed in fp32 like the reference
  const float ms = (float)M, ns = (float)N;
  const float norm = -logf(ms + ns);
  const float mu_bin = logf(ns) + norm, nu_bin = logf(ms) + norm;
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(lse_step_kernel, dim3((B * (M + 1) + 3) / 4), dim3(256), 0, st, scores, v, u, B, M, N, alpha, norm,
                       mu_bin);
    hipLaunchKernelGGL(lse_step_kernel, dim3((B * (N + 1) + 3) / 4), dim3(256), 0, st, sT, u, v, B, N, M, alpha, norm,
                       nu_bin);
  }
  const size_t tot = (size_t)B * (M + 1) * (N + 1);
  hipLaunchKernelGGL(sinkhorn_out_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, scores, u, v, Z, B, M, N,
                     alpha, norm);
  return hipGetLastError();
}

}  // namespace lg
