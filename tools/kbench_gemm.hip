// Micro-benchmark of GEMM tilings / arithmetic modes (tools only; not shipped).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cs566-project-lightglue_amd/csrc tools/kbench_gemm.hip -o /tmp/kb && /tmp/kb
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../cs566-project-lightglue_amd/csrc/gemm.hip"
#include "../cs566-project-lightglue_amd/csrc/elementwise.hip"
#include "../cs566-project-lightglue_amd/csrc/gemm_h3.hip"
#include "gemm_persist.hip"
#include "gemm_defer.hip"

using namespace lg;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct Shape { int R, K, N; const char* name; };

__global__ void empty_kernel() {}

static _Float16* g_planes = nullptr;  // plane image of W * 2^sw
static _Float16* g_aplanes = nullptr; // plane image of A
static float g_unscale = 1.f;

template <int BM, int NS, int EPI = EPI_STORE, int BN = 256, int WN = 64, int KS = 1>
double run_h3(const Shape& s, float* bias, float* Y, int iters, bool planes_out, _Float16* Yp, int stagger = 0) {
  GemmH3Args a;
  memset(&a, 0, sizeof(a));
  (void)stagger;  // start-stagger experiment (round 2): removed from the kernel, no gain
  a.A0 = {g_aplanes, (long long)s.R * s.K, s.R}; a.K0 = s.K; a.K = s.K;
  a.W = {g_planes, (long long)s.N * s.K, s.N}; a.R = s.R; a.Nout = s.N;
  a.acc_scale = g_unscale; a.out_scale = 1.f; a.bias = bias; a.Y = Y; a.ldy = s.N;
  if (planes_out) { a.Yp = Yp; a.yps = (long long)s.R * s.N; a.yrows_pad = s.R; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK((gemm_h3_launch<BM, NS, BN, WN, KS>(a, EPI, 0)));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK((gemm_h3_launch<BM, NS, BN, WN, KS>(a, EPI, 0)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

double run_h3p(const Shape& s, float* bias, float* Y, int iters, _Float16* Yp, int grid) {
  GemmH3Args a;
  memset(&a, 0, sizeof(a));
  a.A0 = {g_aplanes, (long long)s.R * s.K, s.R}; a.K0 = s.K; a.K = s.K;
  a.W = {g_planes, (long long)s.N * s.K, s.N}; a.R = s.R; a.Nout = s.N;
  a.acc_scale = g_unscale; a.out_scale = 1.f; a.bias = bias; a.Y = Y; a.ldy = s.N;
  a.Yp = Yp; a.yps = (long long)s.R * s.N; a.yrows_pad = s.R;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(gemm_h3p(a, 0, grid));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(gemm_h3p(a, 0, grid));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int NK, int DIAG = 0>
double run_h3d(const Shape& s, float* bias, float* Y, int iters, int grid) {
  GemmH3Args a;
  memset(&a, 0, sizeof(a));
  a.A0 = {g_aplanes, (long long)s.R * s.K, s.R}; a.K0 = s.K; a.K = s.K;
  a.W = {g_planes, (long long)s.N * s.K, s.N}; a.R = s.R; a.Nout = s.N;
  a.acc_scale = g_unscale; a.out_scale = 1.f; a.bias = bias; a.Y = Y; a.ldy = s.N;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK((gemm_h3d<NK, DIAG>(a, 0, grid)));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK((gemm_h3d<NK, DIAG>(a, 0, grid)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int WN, int EPI = EPI_LN_GELU, int BM = 128>
double run_ln(const Shape& s, float* bias, float* gam, float* bet, _Float16* Yp, int iters, int stagger = 0) {
  GemmH3Args a;
  memset(&a, 0, sizeof(a));
  (void)stagger;  // start-stagger experiment (round 2): removed from the kernel, no gain
  a.A0 = {g_aplanes, (long long)s.R * s.K, s.R}; a.K0 = s.K; a.K = s.K;
  a.W = {g_planes, (long long)s.N * s.K, s.N}; a.R = s.R; a.Nout = s.N;
  a.acc_scale = g_unscale; a.out_scale = 1.f; a.bias = bias; a.ln_g = gam; a.ln_b = bet;
  a.Yp = Yp; a.yps = (long long)s.R * s.N; a.yrows_pad = s.R;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto launch = [&]() {
    if (EPI == EPI_LN_GELU) return gemm_h3_ln_launch<WN, BM>(a, 0);
    hipLaunchKernelGGL((gemm_h3_kernel<EPI_PROBE, BM, 2, 512, WN>), dim3((a.R + BM - 1) / BM), dim3((BM / 64) * (512 / WN) * 64), 0, 0, a);
    return hipGetLastError();
  };
  CK(launch());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int MODE, int BM, int BN, int BK, int WM, int WN, int EPI = EPI_STORE>
double run(const Shape& s, float* A, float* W, float* bias, float* Y, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.A0 = A; a.lda0 = s.K; a.K0 = s.K; a.K = s.K; a.W = W; a.ldw = s.K; a.bias = bias; a.out_scale = 1.f;
  a.R = s.R; a.Nout = s.N; a.Y = Y; a.ldy = s.N;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK((launch<MODE, BM, BN, BK, WM, WN, EPI>(a, 1, 0)));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK((launch<MODE, BM, BN, BK, WM, WN, EPI>(a, 1, 0)));
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

// fp64 reference for the first `rows` rows; also sum |a*b| for relative errors
__global__ void ref64(const float* A, const float* W, const float* bias, double* Y, double* S, int rows, int K, int N) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * N) return;
  const int r = t / N, c = t % N;
  double s = bias[c], a = 0;
  for (int k = 0; k < K; ++k) { const double p = (double)A[(size_t)r * K + k] * W[(size_t)c * K + k]; s += p; a += fabs(p); }
  Y[t] = s; S[t] = a;
}

int main() {
  const Shape big_shapes[] = {{131072, 32, 768, "k32"}, {131072, 256, 768, "qkv"}, {131072, 512, 512, "ffn1"},
                              {131072, 512, 256, "ffn2"}, {131072, 256, 256, "outp"}};
  // KB_SMALL: the B = 1, N = 1024 forward's GEMMs (R = 2048 rows), small-tile launch shapes
  const Shape small_shapes[] = {{2048, 256, 768, "qkv"}, {2048, 512, 512, "ffn1"}, {2048, 512, 256, "ffn2"},
                                {2048, 256, 512, "xqk"}};
  const bool small = getenv("KB_SMALL") != nullptr;
  if (small) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    empty_kernel<<<256, 256>>>();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 100; ++i) empty_kernel<<<256, 256>>>();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("empty kernel, 256 x 256 threads: %.2f us per launch\n", ms * 10.f);
  }
  std::vector<Shape> shapes;
  if (small) shapes.assign(std::begin(small_shapes), std::end(small_shapes));
  else shapes.assign(std::begin(big_shapes), std::end(big_shapes));
  const int RR = 512;  // rows checked against fp64
  for (const Shape& s : shapes) {
    float *A, *W, *bias, *Y;
    double *Yr, *Sr;
    CK(hipMalloc(&A, (size_t)s.R * s.K * 4)); CK(hipMalloc(&W, (size_t)s.N * s.K * 4));
    CK(hipMalloc(&bias, s.N * 4)); CK(hipMalloc(&Y, (size_t)s.R * s.N * 4));
    CK(hipMalloc(&Yr, (size_t)RR * s.N * 8)); CK(hipMalloc(&Sr, (size_t)RR * s.N * 8));
    fill<<<(s.R * (size_t)s.K + 255) / 256, 256>>>(A, (size_t)s.R * s.K, 1);
    fill<<<(s.N * (size_t)s.K + 255) / 256, 256>>>(W, (size_t)s.N * s.K, 2);
    fill<<<(s.N + 255) / 256, 256>>>(bias, s.N, 3);
    ref64<<<(RR * s.N + 255) / 256, 256>>>(A, W, bias, Yr, Sr, RR, s.K, s.N);
    CK(hipMalloc(&g_planes, (size_t)2 * s.N * s.K * 2));
    CK(hipMalloc(&g_aplanes, (size_t)2 * s.R * s.K * 2));
    // fill() draws from [-1, 1): max|W| < 1 -> scale 2^3 puts max|W 2^sw| in [4, 8) (< 16)
    CK(split_weight_h3(W, s.N, s.K, 8.f, g_planes, 0));
    CK(rows_to_planes(A, s.R, s.K, s.K, g_aplanes, s.R, 0, range_none(), 0));
    g_unscale = ldexpf(1.f, -(11 + 3));
    _Float16* Yp;
    CK(hipMalloc(&Yp, (size_t)2 * s.R * s.N * 2));
    CK(hipDeviceSynchronize());
    std::vector<double> yr((size_t)RR * s.N), sr((size_t)RR * s.N);
    CK(hipMemcpy(yr.data(), Yr, yr.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sr.data(), Sr, sr.size() * 8, hipMemcpyDeviceToHost));
    const double fl = 2.0 * s.R * s.K * s.N;
    auto rep = [&](const char* name, double ms, bool check) {
      double mx = 0, mean = 0;
      if (check) {
        std::vector<float> y((size_t)RR * s.N);
        CK(hipMemcpy(y.data(), Y, y.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < y.size(); ++i) { const double e = fabs(y[i] - yr[i]) / sr[i]; mx = fmax(mx, e); mean += e; }
        mean /= y.size();
      }
      printf("%-5s %-30s %8.1f us %7.1f TF/s  rel.err mean %.2e max %.2e\n", s.name, name, ms * 1e3, fl / ms / 1e9, mean, mx);
    };
    const int it = 20;
    double ms;
    const bool only_stagger = getenv("KB_STAGGER") != nullptr;
    if (getenv("KB_PERSIST")) {  // persistent overlapped-epilogue prototype (tools/gemm_persist.hip)
      if (s.K < 256) continue;
      ms = run_h3<256, 2>(s, bias, Y, it, true, Yp); rep("h3  256x256 + planes", ms, true);
      for (int grid : {256, 512}) {
        char nm[64];
        snprintf(nm, sizeof(nm), "h3p persistent + planes, grid %d", grid);
        CK(hipMemset(Y, 0, (size_t)s.R * s.N * 4));
        ms = run_h3p(s, bias, Y, it, Yp, grid); rep(nm, ms, true);
      }
      continue;
    }
    if (getenv("KB_DEFER")) {  // deferred-store persistent prototype (tools/gemm_defer.hip), fp32 out
      if (s.K < 256) continue;
      ms = run_h3<256, 2, EPI_PROBE>(s, bias, Y, it, false, Yp); rep("256x256 k-loop only", ms, false);
      CK(hipMemset(Y, 0, (size_t)s.R * s.N * 4));
      ms = run_h3<256, 2>(s, bias, Y, it, false, Yp); rep("256x256 + fp32 out", ms, true);
      CK(hipMemset(Y, 0, (size_t)s.R * s.N * 4));
      ms = s.K == 256 ? run_h3d<8>(s, bias, Y, it, 256) : run_h3d<16>(s, bias, Y, it, 256);
      rep("defer 256x128 + fp32 (deferred)", ms, true);
      ms = s.K == 256 ? run_h3d<8, 1>(s, bias, Y, it, 256) : run_h3d<16, 1>(s, bias, Y, it, 256);
      rep("defer 256x128 k-loop only", ms, false);
      CK(hipMemset(Y, 0, (size_t)s.R * s.N * 4));
      ms = s.K == 256 ? run_h3d<8, 2>(s, bias, Y, it, 256) : run_h3d<16, 2>(s, bias, Y, it, 256);
      rep("defer 256x128 + fp32 (stores at tile end)", ms, true);
      continue;
    }
    if (getenv("KB_CHAIN")) {
      // VERDICT r4 item 1(b), costing a chained ffn.3 -> next QKV kernel on 128-row panels (A of the
      // QKV phase resident in LDS): the 128 x 256 tile (8 waves) against the production 256 x 256
      // tile.  Build with -DLG_GEMM_DIAG=32 to drop the A copies (the QKV phase's A from LDS).
      if (s.K < 256) continue;
      ms = run_h3<256, 2, EPI_PROBE>(s, bias, Y, it, false, Yp); rep("256x256 k-loop only", ms, false);
      ms = run_h3<256, 2>(s, bias, Y, it, false, Yp); rep("256x256 + fp32 out", ms, !LG_GEMM_DIAG);
      ms = run_h3<256, 2>(s, bias, Y, it, true, Yp); rep("256x256 + fp32 + planes", ms, !LG_GEMM_DIAG);
      ms = run_h3<128, 2, EPI_PROBE, 256>(s, bias, Y, it, false, Yp); rep("128x256 8w k-loop only", ms, false);
      ms = run_h3<128, 2, EPI_STORE, 256>(s, bias, Y, it, false, Yp); rep("128x256 8w + fp32 out", ms, !LG_GEMM_DIAG);
      ms = run_h3<128, 2, EPI_STORE, 256>(s, bias, Y, it, true, Yp); rep("128x256 8w + fp32 + planes", ms, !LG_GEMM_DIAG);
      ms = run_h3<128, 3, EPI_PROBE, 256>(s, bias, Y, it, false, Yp); rep("128x256 8w 3 stages k-loop only", ms, false);
      ms = run_h3<128, 3, EPI_STORE, 256>(s, bias, Y, it, false, Yp); rep("128x256 8w 3 stages + fp32", ms, !LG_GEMM_DIAG);
      continue;
    }
    if (getenv("KB_LN64")) {  // LN GEMM at 64-row vs 128-row tiles (k-loop and full)
      if (s.N != 512) continue;
      float *gam, *bet;
      CK(hipMalloc(&gam, s.N * 4)); CK(hipMalloc(&bet, s.N * 4));
      fill<<<(s.N + 255) / 256, 256>>>(gam, s.N, 4);
      fill<<<(s.N + 255) / 256, 256>>>(bet, s.N, 5);
      ms = run_ln<64, EPI_PROBE, 128>(s, bias, nullptr, nullptr, Yp, it); rep("h3  128x512, no epilogue", ms, false);
      ms = run_ln<64, EPI_LN_GELU, 128>(s, bias, gam, bet, Yp, it); rep("h3  LN+GELU 128x512", ms, false);
      ms = run_ln<64, EPI_PROBE, 64>(s, bias, nullptr, nullptr, Yp, it); rep("h3  64x512, no epilogue", ms, false);
      ms = run_ln<64, EPI_LN_GELU, 64>(s, bias, gam, bet, Yp, it); rep("h3  LN+GELU 64x512", ms, false);
      CK(hipFree(gam)); CK(hipFree(bet));
      continue;
    }
    if (getenv("KB_LN")) {  // LN epilogue probes (build with -DLG_LN_PROBE=0/1/2/3)
      if (s.N != 512) continue;
      ms = run_ln<64, EPI_PROBE>(s, bias, nullptr, nullptr, Yp, it); rep("h3  128x512 x2, no epilogue", ms, false);
      float *gam, *bet;
      CK(hipMalloc(&gam, s.N * 4)); CK(hipMalloc(&bet, s.N * 4));
      fill<<<(s.N + 255) / 256, 256>>>(gam, s.N, 4);
      fill<<<(s.N + 255) / 256, 256>>>(bet, s.N, 5);
      ms = run_ln<64>(s, bias, gam, bet, Yp, it); rep("h3  LN+GELU 128x512", ms, false);
      CK(hipFree(gam)); CK(hipFree(bet));
      continue;
    }
    if (small) {  // latency decomposition (build with -DLG_GEMM_DIAG=0 / 2 no copies / 4 no waits)
      ms = run_h3<64, 2, EPI_STORE, 64, 64, 4>(s, bias, Y, it, false, Yp); rep("64x64 ks4, fp32 out", ms, !LG_GEMM_DIAG);
      ms = run_h3<64, 2, EPI_STORE, 64, 64, 4>(s, bias, Y, it, true, Yp); rep("64x64 ks4, fp32 + planes", ms, !LG_GEMM_DIAG);
      ms = run_h3<64, 2, EPI_PROBE, 64, 64, 4>(s, bias, Y, it, false, Yp); rep("64x64 ks4, no epilogue", ms, false);
      ms = run_h3<64, 4, EPI_STORE, 64, 64, 2>(s, bias, Y, it, false, Yp); rep("64x64 ks2, fp32 out", ms, !LG_GEMM_DIAG);
      ms = run_h3<64, 4, EPI_STORE, 64, 64, 1>(s, bias, Y, it, false, Yp); rep("64x64 ks1, fp32 out", ms, !LG_GEMM_DIAG);
      continue;
    }
    if (getenv("KB_QUICK")) {  // k-loop probes (build with -DLG_GEMM_DIAG=0/1/2)
      if (s.K < 256) continue;
      ms = run_h3<256, 2, EPI_PROBE>(s, bias, Y, it, false, Yp); rep("h3  256x256x32 x2, no epilogue", ms, false);
      ms = run_h3<256, 2>(s, bias, Y, it, true, Yp); rep("h3  256x256 + planes", ms, !LG_GEMM_DIAG);
      continue;
    }
    if (!only_stagger) {
    ms = run<MODE_X6, 256, 256, 16, 64, 64>(s, A, W, bias, Y, it); rep("x6  256x256x16 (16w)", ms, true);
    ms = run_h3<256, 2>(s, bias, Y, it, false, Yp); rep("h3  256x256x32 x2", ms, true);
    ms = run_h3<256, 2, EPI_PROBE>(s, bias, Y, it, false, Yp); rep("h3  256x256x32 x2, no epilogue", ms, false);
    ms = run_h3<128, 2, EPI_STORE, 128>(s, bias, Y, it, true, Yp); rep("h3  128x128 x2 + planes out", ms, true);
    }
    for (int stg : {0}) {
      char nm[64];
      snprintf(nm, sizeof(nm), "h3  256x256 + planes, stagger %d", stg);
      ms = run_h3<256, 2>(s, bias, Y, it, true, Yp, stg); rep(nm, ms, true);
    }
    if (s.N == 512) {
      ms = run_ln<64, EPI_PROBE>(s, bias, nullptr, nullptr, Yp, it); rep("h3  128x512 x2, no epilogue", ms, false);
      float *gam, *bet;
      CK(hipMalloc(&gam, s.N * 4)); CK(hipMalloc(&bet, s.N * 4));
      fill<<<(s.N + 255) / 256, 256>>>(gam, s.N, 4);
      fill<<<(s.N + 255) / 256, 256>>>(bet, s.N, 5);
      for (int stg : {0}) {
        char nm[64];
        snprintf(nm, sizeof(nm), "h3  LN+GELU 128x512, stagger %d", stg);
        ms = run_ln<64>(s, bias, gam, bet, Yp, it, stg); rep(nm, ms, false);
      }

      CK(hipFree(gam)); CK(hipFree(bet));
    }
    CK(hipFree(Yp)); CK(hipFree(g_aplanes));
    CK(hipFree(g_planes));
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(bias)); CK(hipFree(Y)); CK(hipFree(Yr)); CK(hipFree(Sr));
  }
  return 0;
}
