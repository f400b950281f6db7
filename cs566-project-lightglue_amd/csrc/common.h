// Shared device helpers for the gfx950 kernels (wave64; fp32-accurate products on the
// bf16 / fp16 matrix cores).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lg {

typedef float f32x2 __attribute__((ext_vector_type(2)));
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
// op(v, v of lane ^ 32) for a commutative op, through v_permlane32_swap (no LDS round trip:
// a ds_bpermute would queue behind the other waves' LDS reads).  Both halves get bitwise the
// same result (same operands, same order).
__device__ __forceinline__ float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// wave-wide max / sum without an LDS round trip: DPP within 16 lanes (quad xor 1, xor 2,
// half-row mirror, row mirror), then v_permlane16_swap / v_permlane32_swap across rows; every
// lane ends with bitwise the same value
template <int C>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), C, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max_xor32(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return sum_xor32(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}

// wave-wide (max value, smallest index among the maxima) with the same DPP / permlane steps
template <int C>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false);
}
__device__ __forceinline__ void argmax_merge(float& best, int& bi, float ov, int oi) {
  if (ov > best || (ov == best && oi < bi)) {
    best = ov;
    bi = oi;
  }
}
__device__ __forceinline__ void wave_argmax_dpp(float& best, int& bi) {
  argmax_merge(best, bi, dppf<0xB1>(best), dppi<0xB1>(bi));
  argmax_merge(best, bi, dppf<0x4E>(best), dppi<0x4E>(bi));
  argmax_merge(best, bi, dppf<0x141>(best), dppi<0x141>(bi));
  argmax_merge(best, bi, dppf<0x140>(best), dppi<0x140>(bi));
  {
    const auto v = __builtin_amdgcn_permlane16_swap(__float_as_uint(best), __float_as_uint(best), false, false);
    const auto i = __builtin_amdgcn_permlane16_swap((unsigned)bi, (unsigned)bi, false, false);
    float b0 = __uint_as_float(v[0]);
    int i0 = (int)i[0];
    argmax_merge(b0, i0, __uint_as_float(v[1]), (int)i[1]);
    best = b0;
    bi = i0;
  }
  {
    const auto v = __builtin_amdgcn_permlane32_swap(__float_as_uint(best), __float_as_uint(best), false, false);
    const auto i = __builtin_amdgcn_permlane32_swap((unsigned)bi, (unsigned)bi, false, false);
    float b0 = __uint_as_float(v[0]);
    int i0 = (int)i[0];
    argmax_merge(b0, i0, __uint_as_float(v[1]), (int)i[1]);
    best = b0;
    bi = i0;
  }
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

// ---- fp16x3: fp32-accurate products on fp16 matrix cores (half the MFMAs of bf16x6) ------
// x = h + l * 2^-11 with h = fp16(x) and l = fp16((x - h) * 2^11): the low piece is stored
// pre-scaled so it stays a normal fp16 number; together they carry 22 significant bits
// (probed on gfx950: v_mfma_f32_32x32x16_f16 keeps fp16 subnormal A/B inputs, products are exact
// in the fp32 accumulator; tools/probe_f16_mfma.hip).  For a product the "y" side additionally
// supplies h * 2^11 (exact: |h| <= 16 * 2^11 by construction), so that all three terms land in
// ONE accumulator at the common scale 2^11:
//   2^11 * (x . y) ~= x_h . (y_h 2^11) + x_h . y_l + x_l . y_h        (x_l y_l ~ 2^-22 dropped)
// Operand ranges: |x| <= 2^15 (run-time values are written scaled by a per-tensor power of two
// chosen on the device, RangeOut in kernels.h); y is scaled so |y| < 16 (weights:
// per matrix at load time; queries: per row; P <= 8).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr float kLoScale = 2048.f;    // 2^11
constexpr float kF16Max = 65504.f;    // largest finite fp16

#ifndef LG_NT_STORES
#define LG_NT_STORES 0  // measured: GEMM epilogues +0.17 ms per forward with non-temporal stores, la pass +-0
#endif
// store of a streamed output (non-temporal when LG_NT_STORES)
template <class T>
__device__ __forceinline__ void st_stream(T* p, const T& v) {
#if LG_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

__device__ __forceinline__ void split2h(float x, _Float16& h, _Float16& l) {
  h = (_Float16)x;
  l = (_Float16)((x - (float)h) * kLoScale);  // x - h is exact
}
// split2h / split2h_v of 8 values v[e] * so, two per step: h = cvt_pk(y0, y1), and the low piece
// as ONE v_fma_mix per value -- l = fp16(h * (-lsc) + v * (so * lsc)), lsc = 2^11 (split2h) or 1
// (split2h_v): y * lsc - h * lsc is exact in fp32 before its single rounding, so the pieces equal
// split2h's (the compiler's form of split2h takes 7 VALU per pair, this one 5)
template <bool V = false>
__device__ __forceinline__ void split2h_x8(const float (&v)[8], float so, f16x8& h, f16x8& l) {
  typedef _Float16 f16x2_s __attribute__((ext_vector_type(2)));
  const float lsc = V ? 1.f : kLoScale, nl = -lsc, sl = so * lsc;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float y0 = v[2 * p] * so, y1 = v[2 * p + 1] * so;
    const f16x2_s hp = {(_Float16)y0, (_Float16)y1};
    unsigned lo;
    asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hp), "s"(nl), "v"(v[2 * p] * sl));
    asm("v_fma_mixhi_f16 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hp), "s"(nl), "v"(v[2 * p + 1] * sl));
    const f16x2_s lp = __builtin_bit_cast(f16x2_s, lo);
    h[2 * p] = hp[0];
    h[2 * p + 1] = hp[1];
    l[2 * p] = lp[0];
    l[2 * p + 1] = lp[1];
  }
}
// value planes (PREC_H3 V): the low piece at its own scale, x = h + l.  Small residuals become
// fp16 subnormals (absolute error <= 2^-25 in plane units); the value planes' range exponent is
// two-sided (kRangeTwoSided), so a plane's largest values sit near 2^15 and that error stays
// ~2^-40 of them
__device__ __forceinline__ void split2h_v(float x, _Float16& h, _Float16& l) {
  h = (_Float16)x;
  l = (_Float16)(x - (float)h);
}

__device__ __forceinline__ f32x16 mfma16(const f16x8& a, const f16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// the same with v_mfma_f32_16x16x32_f16: lane l supplies A[l & 15][8 (l >> 4) + j] and
// B[8 (l >> 4) + j][l & 15]; accumulator register r of lane l holds C[4 (l >> 4) + r][l & 15]
typedef float f32x4_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4_ mfma_h3_16(const f16x8& xh, const f16x8& xl, const f16x8& yhs, const f16x8& yl,
                                             const f16x8& yh, f32x4_ c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, yh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, yl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, yhs, c, 0, 0, 0);
  return c;
}

// acc += 2^11 * (x . y), x = (xh, xl), y = (yhs = yh * 2^11, yl, yh); smallest terms first
__device__ __forceinline__ f32x16 mfma_h3(const f16x8& xh, const f16x8& xl, const f16x8& yhs, const f16x8& yl,
                                          const f16x8& yh, f32x16 c) {
  c = mfma16(xl, yh, c);
  c = mfma16(xh, yl, c);
  c = mfma16(xh, yhs, c);
  return c;
}

// ---- fp16x3 operand images in HBM ("plane images") ----------------------------------------
// A [rows][K] fp32 matrix that feeds the fp16x3 GEMM (gemm_h3.hip) is stored as its two fp16
// pieces, k-blocked and pre-swizzled exactly like the GEMM's LDS tile, so that a k-tile of a row
// tile is one contiguous block per plane and the GEMM stages it with plain LDS-DMA copies:
//   [plane 0 (h) | plane 1 (l * 2^11)][K / 32 kblocks][rows_pad][32]
// i.e. 64-byte rows of four 16-byte chunks; chunk c (k = 8c..8c+7 of the kblock) of row r is
// stored at chunk c ^ plane_swz(r): the swizzle under which the GEMM's 16x16x32 fragment reads
// (lane l: row l & 15 of a 16-row block, chunk l >> 4) hit all 16 slots of a 256-byte bank line
// in every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...): with
// k = (r >> 2) & 3, plane_swz = sigma(k), sigma = (0, 2, 3, 1).  rows_pad is a multiple of 256.
constexpr int kKB = 32;  // k-block (columns per plane row)
__device__ __forceinline__ int plane_swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }
// element offset of (row, k) inside one plane of an image with `rows_pad` rows
__device__ __forceinline__ size_t plane_off(int row, int k, int rows_pad) {
  return ((size_t)(k >> 5) * rows_pad + row) * kKB + ((((k >> 3) & 3) ^ plane_swz(row)) << 3) + (k & 7);
}

// ---- run-time range scaling of plane images (kernels.h RangeOut) ----------------------------
// Table layout: slot s occupies kRangeStride words -- M as kRangeShards shards (a writing
// workgroup updates shard blockIdx.x % kRangeShards, so thousands of workgroups do not serialise
// on one address; M = max over the shards), then E.
constexpr int kRangeShards = 16, kRangeStride = 32;
constexpr float kRangeLimit = 32768.f;  // 2^15: half the fp16 range, so rounding cannot reach inf
__device__ __forceinline__ float range_max(const unsigned* tab, int s) {
  const unsigned* p = tab + s * kRangeStride;
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < kRangeShards; ++i) m = fmaxf(m, __uint_as_float(p[i]));
  return m;
}
template <class RO>
__device__ __forceinline__ int range_exponent(const RO& r) {
  if (!r.tab) return 0;
  float b = r.add;
  if (r.in0 >= 0) b += r.g0 * range_max(r.tab, r.in0);
  if (r.in1 >= 0) b += r.g1 * range_max(r.tab, r.in1);
  const float lim = ldexpf(kRangeLimit, -r.lshift);
  if (!(b <= 3.0e38f)) return 0;  // non-finite data
  if (r.track & 2) {  // kernels.h kRangeTwoSided
    if (!(b > 0.f)) return 0;
    int E;
    (void)frexpf(b / lim, &E);  // 2^(E-1) < b / lim <= 2^E: the bound lands in (lim / 2, lim]
    return max(E, -64);
  }
  if (!(b > lim)) return 0;  // in range
  int E;
  (void)frexpf(b / lim, &E);  // b / lim = m 2^E, m in [0.5, 1)  ->  2^E >= it
  return E;
}
__device__ __forceinline__ int range_slot_exp(const unsigned* tab, int slot) {
  return (tab && slot >= 0) ? (int)tab[slot * kRangeStride + kRangeShards] : 0;
}
// Block-wide max of |x| written -> one atomicMax into this workgroup's shard of M[out], and
// E[out] (stored only when not the table's initial 0; every writer stores the same value).
// Called by every thread of the workgroup (it contains a barrier).
// range_commit_lds reuses 16 floats of the caller's LDS (kernels that declare all of it) and
// first waits for every wave to be done with it.
template <class RO>
__device__ __forceinline__ void range_commit_lds(const RO& r, float lane_max, int e, float* red, int nwaves = -1) {
  if (!r.tab) return;
  if (!(r.track & 1)) {  // kernels.h kRangeTrack clear: E only, no reduction, no barrier
    if (e != 0 && (threadIdx.x & 63) == 0) r.tab[r.out * kRangeStride + kRangeShards] = (unsigned)e;
    return;
  }
  const float m = wave_max_dpp(lane_max);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = 0.f;
    const int nw = nwaves > 0 ? nwaves : (int)(blockDim.x >> 6);  // waves still running
    for (int w = 0; w < nw; ++w) mm = fmaxf(mm, red[w]);
    unsigned* slot = r.tab + r.out * kRangeStride;
    if (mm > 0.f) atomicMax(slot + (blockIdx.x % kRangeShards), __float_as_uint(mm));
    if (e != 0) slot[kRangeShards] = (unsigned)e;
  }
}
template <class RO>
__device__ __forceinline__ void range_commit(const RO& r, float lane_max, int e) {
  __shared__ float range_red[16];
  range_commit_lds(r, lane_max, e, range_red);
}

// ---- LDS-DMA ------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) char lds_char;
// one global_load_lds_dwordx4: lane i copies the 16 bytes at base + voff (base wave-uniform,
// in SGPRs; voff per lane) to LDS byte address lds + 16 i (lds wave-uniform).  Inline asm: the
// compiler neither counts it nor orders LDS reads behind it -- callers wait for it with an
// explicit vmcnt + barrier.
__device__ __forceinline__ void dma16(const void* base, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(lds)
               : "memory");
}

// dma16 from code the compiler cannot prove wave-uniform (e.g. inside a lambda called from another
// lambda): the base and the LDS address are made scalar explicitly (they are uniform by construction)
__device__ __forceinline__ void dma16_u(const void* base, uint32_t voff, uint32_t lds) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  dma16(reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo), voff, __builtin_amdgcn_readfirstlane(lds));
}

// the same copy with the non-temporal hint (operands streamed exactly once)
__device__ __forceinline__ void dma16_nt(const void* base, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(lds)
               : "memory");
}

__device__ __forceinline__ float log_sigmoid(float x) {
  // logsigmoid(x) = min(x,0) - log1p(exp(-|x|))  (torch's CPU formulation)
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}

// GELU(y) = y Phi(y) (nn.GELU(), erf form) without erff's branches: Phi(-|y|) = erfc(|y| / sqrt2) / 2
// from the Chebyshev fit of erfc (Numerical Recipes' erfcc, fractional error < 1.2e-7 for all
// arguments), y Phi(y) = y - y Phi(-y) for y >= 0.  Measured over every fp32 y in [-14, 14]:
// |error| <= 2.4e-7 against fp64 (0.5 y (1 + erff(y / sqrt2)) itself: 4.5e-7).  ~15 VALU ops,
// a third of erff's divergent two-branch polynomial -- the LN epilogue's GELU pass was 40 us of
// the ffn.0 GEMM's 269 (tools/kbench_gemm.hip, LG_LN_PROBE).
__device__ __forceinline__ float gelu_erf(float y) {
  const float z = fabsf(y) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float h = 0.5f * t * __builtin_amdgcn_exp2f((p - z * z) * 1.4426950408889634f);
  return y >= 0.f ? fmaf(-y, h, y) : y * h;
}
// the same for two values with packed fp32 arithmetic (v_pk_fma_f32 / v_pk_mul_f32: two lanes per
// issue, each lane the scalar form's operation sequence, so the results are bit-identical); for
// epilogues with no MFMA beside them (MI355X_MICROARCH.md: packed fp32 only loses beside MFMAs)
typedef float f32x2_ __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_ gelu_erf2(f32x2_ y) {
  const f32x2_ z = __builtin_elementwise_abs(y) * 0.70710678118654752f;
  const f32x2_ u = __builtin_elementwise_fma(f32x2_{0.5f, 0.5f}, z, f32x2_{1.f, 1.f});
  const f32x2_ t = {__builtin_amdgcn_rcpf(u.x), __builtin_amdgcn_rcpf(u.y)};
  auto fm = [&](f32x2_ p, float c) { return __builtin_elementwise_fma(p, t, f32x2_{c, c}); };
  f32x2_ p = {0.17087277f, 0.17087277f};
  p = fm(p, -0.82215223f);
  p = fm(p, 1.48851587f);
  p = fm(p, -1.13520398f);
  p = fm(p, 0.27886807f);
  p = fm(p, -0.18628806f);
  p = fm(p, 0.09678418f);
  p = fm(p, 0.37409196f);
  p = fm(p, 1.00002368f);
  p = fm(p, -1.26551223f);
  const f32x2_ w = (p - z * z) * 1.4426950408889634f;
  const f32x2_ h = 0.5f * t * f32x2_{__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2_ pos = __builtin_elementwise_fma(-y, h, y), neg = y * h;
  return f32x2_{y.x >= 0.f ? pos.x : neg.x, y.y >= 0.f ? pos.y : neg.y};
}

}  // namespace lg
