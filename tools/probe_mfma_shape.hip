// Probe: fp16 MFMA throughput of v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 on random
// operands (the clock the chip holds depends on data and shape, MI355X_MICROARCH.md DVFS item 7).
// Same flops per wave in both: 32x32x16 = 2 x 16x16x32.  8 waves per workgroup, 4 independent
// accumulators per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_mfma_shape.hip -o tools/probe_mfma_shape
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ inline f16x8 rnd8(unsigned s) {
  f16x8 v;
  for (int e = 0; e < 8; ++e) {
    s = s * 1664525u + 1013904223u;
    v[e] = (_Float16)(((s >> 8) & 0xffff) / 65536.f - 0.5f);
  }
  return v;
}

template <int SHAPE>
__global__ __launch_bounds__(512) void probe(float* out, int iters) {
  const unsigned seed = blockIdx.x * 512 + threadIdx.x;
  const f16x8 a0 = rnd8(seed), a1 = rnd8(seed + 7), b0 = rnd8(seed + 13), b1 = rnd8(seed + 29);
  float t = 0.f;
  if (SHAPE == 32) {
    f32x16 c[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k & 1 ? a1 : a0, k & 2 ? b1 : b0, c[k], 0, 0, 0);
    }
    for (int k = 0; k < 4; ++k)
      for (int e = 0; e < 16; ++e) t += c[k][e];
  } else {
    f32x4 c[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k & 1 ? a1 : a0, k & 2 ? b1 : b0, c[k], 0, 0, 0);
    }
    for (int k = 0; k < 8; ++k)
      for (int e = 0; e < 4; ++e) t += c[k][e];
  }
  if (t == 1234.5f) out[threadIdx.x] = t;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096);
  const int iters = 4000, blocks = 256 * 4;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (int shape : {32, 16}) {
      auto launch = [&]() {
        if (shape == 32) hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(512), 0, 0, out, iters);
        else hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(512), 0, 0, out, iters);
      };
      launch();
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int r = 0; r < 3; ++r) launch();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 3;
      const double flops = 2.0 * 32 * 32 * 16 * 4 * (double)iters * 8 * blocks;  // per launch
      printf("%s: %8.1f us  %7.1f TF/s fp16\n", shape == 32 ? "32x32x16" : "16x16x32", ms * 1e3, flops / ms / 1e9);
    }
  return 0;
}
