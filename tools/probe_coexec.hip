// Probe: do MFMAs of one wave and VALU work of its SIMD partner execute concurrently?
// 8-wave workgroups (2 waves per SIMD), one workgroup per CU.  mode 0: waves 0-3 MFMA only;
// mode 1: waves 4-7 VALU only; mode 2: both at once; mode 3: every wave does both, interleaved;
// mode 4: waves 0-3 MFMA with LDS-read operands; mode 5: mode 4 + waves 4-7 VALU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_coexec.hip -o tools/probe_coexec
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(512, 2) void probe(float* out, int iters, float seed) {
  __shared__ float pad[40 * 1024];  // one workgroup per CU
  for (int i = threadIdx.x; i < 40 * 1024; i += 512) pad[i] = seed * (i & 63);
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool do_mfma = MODE == 3 || (MODE != 1 && wave < 4);
  const bool do_valu = MODE == 3 || ((MODE == 1 || MODE == 2 || MODE == 5) && wave >= 4);
  const bool lds_ops = MODE >= 4;
  f16x8* lp = reinterpret_cast<f16x8*>(pad) + (threadIdx.x & 255);
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(seed * (e + 1)); b[e] = (_Float16)(seed - e); }
  f32x16 c0 = {0.f}, c1 = {0.f};
  float x[16];
  for (int e = 0; e < 16; ++e) x[e] = seed * (threadIdx.x + e);
  for (int it = 0; it < iters; ++it) {
    if (do_mfma && !lds_ops) {
#pragma unroll
      for (int k = 0; k < 24; ++k) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
      }
    }
    if (do_mfma && lds_ops) {  // one 16-byte LDS read per MFMA, issued 4 MFMAs ahead
      f16x8 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = lp[k * 256];
#pragma unroll
      for (int k = 0; k < 48; ++k) {
        const f16x8 x = r[k & 3];
        if (k + 4 < 48) r[k & 3] = lp[((k + 4) & 7) * 256];
        if (k & 1) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, a, c1, 0, 0, 0);
        else c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, b, c0, 0, 0, 0);
      }
    }
    if (do_valu) {
#pragma unroll
      for (int k = 0; k < 24; ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) x[e] = __builtin_amdgcn_exp2f(fmaf(x[e], 0.999f, -0.5f)) * 0.5f;
    }
  }
  float t = 0.f;
  for (int e = 0; e < 16; ++e) t += c0[e] + c1[e] + x[e];
  if (t == 1234.5f) out[threadIdx.x] = t + pad[threadIdx.x];
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  const int iters = 200, blocks = 256 * 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"MFMA only (waves 0-3)", "VALU only (waves 4-7)", "both, split by wave", "both, every wave",
                         "MFMA+LDS reads (waves 0-3)", "MFMA+LDS reads || VALU"};
  for (int mode = 0; mode < 6; ++mode) {
    auto launch = [&]() {
      switch (mode) {
        case 0: hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
        case 1: hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
        case 2: hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
        case 4: hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
        case 5: hipLaunchKernelGGL(probe<5>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
        default: hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.001f); break;
      }
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.1f us\n", names[mode], ms * 1e3 / 5);
  }
  return 0;
}
