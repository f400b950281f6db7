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

// ---- bf16x6: fp32-accurate products on bf16 matrix cores --------------------------------
// x = h + m + l exactly up to 2^-27 |x| (three round-to-nearest bf16 pieces); a*b is then the
// sum of the six piece products of weight >= 2^-18, each exact in the fp32 accumulator.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;  // exact
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);   // exact subtraction, rounded once
}

// acc += a * b with a = a0+a1+a2, b = b0+b1+b2 (smallest terms first)
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                          const bf16x8& b1, const bf16x8& b2, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ float log_sigmoid(float x) {
  // logsigmoid(x) = min(x,0) - log1p(exp(-|x|))  (torch's CPU formulation)
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}

}  // namespace lg
