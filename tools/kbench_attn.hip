// Micro-benchmark of attention variants (tools only; not shipped).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench_attn.hip -o tools/kbench_attn && tools/kbench_attn [N]
// Self-attention shape of the bench (B=32 pairs, 4 heads, N keys, 2 sets), random q/k in
// [-2, 2), v in [-1, 1); each variant is checked against an fp64 reference on set 0.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cs566-project-lightglue_amd/csrc/attention.hip"

using namespace lg;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill(float* p, size_t n, unsigned seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
    p[i] = (((x & 0xffffff) / 16777216.0f) * 2.f - 1.f) * scale;
  }
}

__global__ void planes_x6(const float* x, __bf16* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    __bf16 h, m, l;
    split3(x[i], h, m, l);
    p[i] = h; p[n + i] = m; p[2 * n + i] = l;
  }
}
__global__ void planes_h3(const float* x, _Float16* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    _Float16 h, l;
    split2h(x[i], h, l);
    p[i] = h; p[n + i] = l;
  }
}

// naive reference: one thread per (bh, query), double accumulation
__global__ void ref_attn(const float* Q, const float* K, const float* V, float* O, int BH, int H, int N, float scale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BH * N) return;
  const int bh = t / N, q = t % N;
  const float* qp = Q + ((size_t)bh * N + q) * 64;
  double m = -1e300;
  for (int k = 0; k < N; ++k) {
    double s = 0;
    for (int d = 0; d < 64; ++d) s += (double)qp[d] * K[((size_t)bh * N + k) * 64 + d];
    m = fmax(m, s * scale);
  }
  double l = 0, o[64] = {0};
  for (int k = 0; k < N; ++k) {
    double s = 0;
    for (int d = 0; d < 64; ++d) s += (double)qp[d] * K[((size_t)bh * N + k) * 64 + d];
    const double p = exp(s * scale - m);
    l += p;
    for (int d = 0; d < 64; ++d) o[d] += p * V[((size_t)bh * N + k) * 64 + d];
  }
  const int b = bh / H, h = bh % H;
  for (int d = 0; d < 64; ++d) O[((size_t)b * N + q) * 256 + h * 64 + d] = (float)(o[d] / l);
}

template <class F>
void run(const char* name, F launch, int B, int H, const AttnSet& a0, const AttnSet& a1, float* Oref, float* O, size_t on) {
  CK(hipMemset(O, 0, on * 4));
  CK(launch());
  CK(hipDeviceSynchronize());
  std::vector<float> x(on), y(on);
  CK(hipMemcpy(x.data(), O, on * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), Oref, on * 4, hipMemcpyDeviceToHost));
  double md = 0;
  for (size_t i = 0; i < on; ++i) md = fmax(md, fabs((double)x[i] - y[i]));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int it = 10;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < it; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= it;
  const double fl = 4.0 * 64.0 * H * B * ((double)a0.Nq * a0.Nk + (double)a1.Nq * a1.Nk);
  printf("%-26s %8.1f us  %6.1f TF/s (fp32-eq)  maxdiff(set0 vs fp64) %.2e\n", name, ms * 1e3, fl / ms / 1e9, md);
}

int main(int argc, char** argv) {
  const int B = 32, H = 4, N = argc > 1 ? atoi(argv[1]) : 2048;
  const size_t n = (size_t)B * H * N * 64;
  float *Q, *K, *V, *O, *Oref;
  void *KP, *VP, *KH, *VH;
  CK(hipMalloc(&Q, 2 * n * 4)); CK(hipMalloc(&K, 2 * n * 4)); CK(hipMalloc(&V, 2 * n * 4));
  CK(hipMalloc(&KP, 3 * 2 * n * 2)); CK(hipMalloc(&VP, 3 * 2 * n * 2));
  CK(hipMalloc(&KH, 2 * 2 * n * 2)); CK(hipMalloc(&VH, 2 * 2 * n * 2));
  CK(hipMalloc(&O, 2 * n * 4)); CK(hipMalloc(&Oref, 2 * n * 4));
  fill<<<(2 * n + 255) / 256, 256>>>(Q, 2 * n, 1, 2.f);
  fill<<<(2 * n + 255) / 256, 256>>>(K, 2 * n, 2, 2.f);
  fill<<<(2 * n + 255) / 256, 256>>>(V, 2 * n, 3, 1.f);
  planes_x6<<<(2 * n + 255) / 256, 256>>>(K, (__bf16*)KP, 2 * n);
  planes_x6<<<(2 * n + 255) / 256, 256>>>(V, (__bf16*)VP, 2 * n);
  planes_h3<<<(2 * n + 255) / 256, 256>>>(K, (_Float16*)KH, 2 * n);
  planes_h3<<<(2 * n + 255) / 256, 256>>>(V, (_Float16*)VH, 2 * n);
  const float scale = 0.125f;
  ref_attn<<<(B * H * N + 127) / 128, 128>>>(Q, K, V, Oref, B * H, H, N, scale);
  CK(hipDeviceSynchronize());
  const long long ps = 2 * (long long)n;
  AttnSet x0{Q, KP, VP, ps, O, N, N}, x1{Q + n, (__bf16*)KP + n, (__bf16*)VP + n, ps, O + (size_t)B * N * 256, N, N};
  AttnSet h0{Q, KH, VH, ps, O, N, N}, h1{Q + n, (_Float16*)KH + n, (_Float16*)VH + n, ps, O + (size_t)B * N * 256, N, N};
  const size_t on = (size_t)B * N * 256;  // compare set 0
  run("x6   w8 kt64", [&] { return attention_x6_launch<8, 64>(x0, x1, B, H, scale, 0); }, B, H, x0, x1, Oref, O, on);
  run("h3   w8 kt64", [&] { return attention_h3_launch<8, 64>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3v2 w8 kt64 occ2", [&] { return attention_h3v2_launch<8, 64, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3v2 DIAG1 no softmax", [&] { return attention_h3v2_launch<8, 64, 2, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3v2 DIAG1 occ4", [&] { return attention_h3v2_launch<8, 64, 4, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3v2 DIAG1 w4 occ4", [&] { return attention_h3v2_launch<4, 64, 4, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3v2 DIAG1 w8 kt32 occ4", [&] { return attention_h3v2_launch<8, 32, 4, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  return 0;
}
