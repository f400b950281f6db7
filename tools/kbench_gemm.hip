// Micro-benchmark of GEMM tilings (tools only; not shipped).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cs566-project-lightglue_amd/csrc tools/kbench_gemm.hip -o /tmp/kb && /tmp/kb
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../cs566-project-lightglue_amd/csrc/gemm.hip"

using namespace lg;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct Shape { int R, K, N; const char* name; };

template <int BM, int BN, int BK, int WM, int WN, int EPI = EPI_STORE>
double run(const Shape& s, float* A, float* W, float* bias, float* Y, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.A0 = A; a.lda0 = s.K; a.K0 = s.K; a.K = s.K; a.W = W; a.ldw = s.K; a.bias = bias; a.out_scale = 1.f;
  a.R = s.R; a.Nout = s.N; a.Y = Y; a.ldy = s.N;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK((launch<BM, BN, BK, WM, WN, EPI>(a, 1, 0)));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK((launch<BM, BN, BK, WM, WN, EPI>(a, 1, 0)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

__global__ void fill(float* p, size_t n, unsigned seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
    p[i] = ((x & 0xffffff) / 16777216.0f) * 2.f - 1.f;
  }
}

float maxdiff(const float* a, const float* b, size_t n) {
  std::vector<float> x(n), y(n);
  hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost);
  float m = 0;
  for (size_t i = 0; i < n; ++i) m = fmaxf(m, fabsf(x[i] - y[i]));
  return m;
}

int main() {
  const Shape shapes[] = {{131072, 256, 768, "qkv"}, {131072, 512, 512, "ffn1"}, {131072, 512, 256, "ffn2"}, {131072, 256, 256, "outp"}};
  for (const Shape& s : shapes) {
    float *A, *W, *bias, *Y0, *Y;
    CK(hipMalloc(&A, (size_t)s.R * s.K * 4)); CK(hipMalloc(&W, (size_t)s.N * s.K * 4));
    CK(hipMalloc(&bias, s.N * 4)); CK(hipMalloc(&Y0, (size_t)s.R * s.N * 4)); CK(hipMalloc(&Y, (size_t)s.R * s.N * 4));
    fill<<<(s.R * (size_t)s.K + 255) / 256, 256>>>(A, (size_t)s.R * s.K, 1);
    fill<<<(s.N * (size_t)s.K + 255) / 256, 256>>>(W, (size_t)s.N * s.K, 2);
    fill<<<(s.N + 255) / 256, 256>>>(bias, s.N, 3);
    const double fl = 2.0 * s.R * s.K * s.N;
    auto rep = [&](const char* name, double ms) {
      printf("%-5s %-28s %8.1f us %7.1f TF/s  maxdiff %.2e\n", s.name, name, ms * 1e3, fl / ms / 1e9, maxdiff(Y0, Y, (size_t)s.R * s.N));
    };
    const int it = 20;
    double ms = run<256, 128, 16, 64, 64>(s, A, W, bias, Y0, it); rep("256x128x16 w64x64 (8w)", ms);
    ms = run<256, 128, 16, 64, 64, EPI_PROBE>(s, A, W, bias, Y, it); rep("  same, no store", ms);
    ms = run<128, 256, 32, 64, 64>(s, A, W, bias, Y, it); rep("128x256x32 w64x64 (8w)", ms);
    ms = run<128, 256, 32, 64, 64, EPI_PROBE>(s, A, W, bias, Y, it); rep("  same, no store", ms);
    ms = run<128, 128, 32, 64, 64>(s, A, W, bias, Y, it); rep("128x128x32 w64x64 (4w)", ms);
    ms = run<128, 128, 32, 64, 64, EPI_PROBE>(s, A, W, bias, Y, it); rep("  same, no store", ms);
    ms = run<128, 128, 16, 64, 64>(s, A, W, bias, Y, it); rep("128x128x16 w64x64 (4w)", ms);
    ms = run<128, 128, 16, 64, 64, EPI_PROBE>(s, A, W, bias, Y, it); rep("  same, no store", ms);
    ms = run<256, 256, 16, 64, 64>(s, A, W, bias, Y, it); rep("256x256x16 w64x64 (16w)", ms);
    ms = run<256, 256, 16, 64, 64, EPI_PROBE>(s, A, W, bias, Y, it); rep("  same, no store", ms);
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(bias)); CK(hipFree(Y0)); CK(hipFree(Y));
  }
  return 0;
}
