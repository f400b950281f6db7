// Shared device helpers for the gfx950 kernels (wave64, f32-input MFMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lg {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;
constexpr int kDim = 256;      // descriptor_dim the kernels are specialised for
constexpr int kHeadDim = 64;   // descriptor_dim / num_heads
constexpr int kFreq = 32;      // Fourier frequencies = head_dim / 2

// 32x32x2 f32 MFMA: lane l supplies A[l&31][l>>5], B[l>>5][l&31]; accumulator register r of
// lane l holds C[row32(r, l>>5)][l&31].
__device__ __forceinline__ int row32(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Exact (IEEE, non-contracted) elementwise ops: used where the reference's torch-CPU op order
// is mirrored bit-for-bit (positional encoding, keypoint normalisation, rotary).
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float sub_rn(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float div_rn(float a, float b) { return __fdiv_rn(a, b); }

__device__ __forceinline__ float log_sigmoid(float x) {
  // logsigmoid(x) = min(x,0) - log1p(exp(-|x|))  (torch's CPU formulation)
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}

}  // namespace lg
