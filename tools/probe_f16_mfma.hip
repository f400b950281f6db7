// Probe (tools only): does v_mfma_f32_32x32x16_f16 keep fp16 subnormal A/B inputs, and how
// exactly does it sum its 16 products?  Decides the fp16x3 operand format.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_f16_mfma.hip -o /tmp/pf && /tmp/pf
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

// A [32][16] row-major, B [16][32] row-major (k, col), C [32][32]; one wave.
__global__ void mfma_once(const _Float16* A, const _Float16* B, const float* Cin, float* C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r * 16 + 8 * h + j];
    b[j] = B[(8 * h + j) * 32 + r];
  }
  f32x16 c;
  for (int i = 0; i < 16; ++i) c[i] = Cin[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

__global__ void cvt(const float* x, unsigned short* y, int n) {
  int i = threadIdx.x;
  if (i < n) {
    _Float16 v = (_Float16)x[i];
    y[i] = __builtin_bit_cast(unsigned short, v);
  }
}

static float h2f(_Float16 v) { return (float)v; }

int main() {
  _Float16 *dA, *dB;
  float *dC, *dCin;
  CK(hipMalloc(&dA, 32 * 16 * 2));
  CK(hipMalloc(&dB, 16 * 32 * 2));
  CK(hipMalloc(&dC, 32 * 32 * 4));
  CK(hipMalloc(&dCin, 32 * 32 * 4));
  std::vector<_Float16> A(32 * 16), B(16 * 32);
  std::vector<float> C(32 * 32), Cin(32 * 32, 0.f);
  auto run = [&]() {
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dCin, Cin.data(), Cin.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mfma_once, dim3(1), dim3(64), 0, 0, dA, dB, dCin, dC);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
  };
  // 1. subnormal A input times 1
  for (auto& v : A) v = 0;
  for (auto& v : B) v = 0;
  A[0] = (_Float16)ldexpf(1.f, -20);  // fp16 subnormal
  B[0] = (_Float16)1.f;
  A[1 * 16 + 0] = (_Float16)ldexpf(1.f, -24);  // smallest subnormal
  A[2 * 16 + 0] = (_Float16)ldexpf(3.f, -16);  // subnormal 3*2^-16
  run();
  printf("subnormal A: got %.6e (want %.6e), %.6e (want %.6e), %.6e (want %.6e)\n", C[0], ldexp(1.0, -20), C[32],
         ldexp(1.0, -24), C[64], ldexp(3.0, -16));
  // 2. subnormal B input times normal A
  for (auto& v : A) v = 0;
  for (auto& v : B) v = 0;
  A[0] = (_Float16)ldexpf(1.f, -10);
  B[0] = (_Float16)ldexpf(1.f, -22);
  run();
  printf("subnormal B: got %.6e (want %.6e)\n", C[0], ldexp(1.0, -32));
  // 3. internal accumulation: big + tiny terms, and C input
  for (auto& v : A) v = 0;
  for (auto& v : B) v = 0;
  for (int k = 0; k < 16; ++k) {
    A[k] = (_Float16)(k == 0 ? 2048.f : ldexpf(1.f, -14));
    B[k * 32] = (_Float16)(k == 0 ? 2048.f : ldexpf(1.f, -10));
  }
  Cin[0] = 0.f;
  run();
  const double exact = 2048.0 * 2048.0 + 15 * ldexp(1.0, -24);
  printf("accumulate 2^22 + 15*2^-24: got %.17g exact %.17g fp32(exact) %.17g\n", C[0], exact, (double)(float)exact);
  // 4. random accuracy vs fp64
  std::mt19937 g(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  double worst = 0, mean = 0;
  int cnt = 0;
  for (int trial = 0; trial < 200; ++trial) {
    for (auto& v : A) v = (_Float16)(U(g) * ldexpf(1.f, (int)(U(g) * 8)));
    for (auto& v : B) v = (_Float16)(U(g) * ldexpf(1.f, (int)(U(g) * 8)));
    for (auto& v : Cin) v = U(g) * 4.f;
    run();
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double s = Cin[i * 32 + j], sa = fabs(s);
        for (int k = 0; k < 16; ++k) {
          const double p = (double)h2f(A[i * 16 + k]) * (double)h2f(B[k * 32 + j]);
          s += p;
          sa += fabs(p);
        }
        const double e = fabs(C[i * 32 + j] - s) / sa;
        worst = fmax(worst, e);
        mean += e;
        ++cnt;
      }
  }
  printf("random: max rel err %.3e  mean %.3e (per sum|terms|; fp32 ulp/2 = %.3e)\n", worst, mean / cnt,
         ldexp(1.0, -24));
  // 5. f32 -> f16 conversion of subnormals
  float xs[4] = {ldexpf(1.f, -20), ldexpf(1.f, -24), ldexpf(1.f, -26), 70000.f};
  float* dx;
  unsigned short* dy;
  CK(hipMalloc(&dx, 16));
  CK(hipMalloc(&dy, 8));
  CK(hipMemcpy(dx, xs, 16, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(cvt, dim3(1), dim3(64), 0, 0, dx, dy, 4);
  unsigned short ys[4];
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ys, dy, 8, hipMemcpyDeviceToHost));
  printf("cvt f32->f16: 2^-20 -> 0x%04x (want 0x0010), 2^-24 -> 0x%04x (want 0x0001), 2^-26 -> 0x%04x, 70000 -> 0x%04x\n",
         ys[0], ys[1], ys[2], ys[3]);
  return 0;
}
