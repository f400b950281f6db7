// Prototype (tools/kbench_gemm.hip only, KB_DEFER): a persistent fp16x3 GEMM whose epilogue stores
// are deferred into the NEXT tile's k-loop, so that a CU's output stores run under its MFMAs
// instead of after them.  The question it answers: does hiding the epilogue behind the k-loop of
// the following tile pay, when the tile has to shrink to 256 x 128 (8 waves, 2 per SIMD) for the
// second accumulator set to fit the register file?
//
//  * one 512-thread workgroup per CU walks tiles it*G + blockIdx.x (XCD-remapped like gemm_h3);
//    the k-tiles of consecutive tiles form ONE LDS-DMA stream over NSTAGE stages (the next tile's
//    first k-tiles are copied under the current tile's last ones);
//  * products with the MFMA operands swapped (W fragments as the A operand): the accumulator of a
//    lane holds 4 CONSECUTIVE output columns of one row, stored as one 16-byte store;
//  * after a tile's last k-tile its accumulators become the pending output (scale + bias) and the
//    next tile's k-loop issues 16 / NK of those stores per k-tile, AFTER that k-tile's copies, so
//    each copy wait counts the younger stores out exactly (s_waitcnt vmcnt retires in order).
#pragma once
#include "../cs566-project-lightglue_amd/csrc/common.h"
#include "../cs566-project-lightglue_amd/csrc/kernels.h"

namespace lg {
namespace defer {

__device__ __forceinline__ f32x4_ mfma_h3_16t(const f16x8& xh, const f16x8& xl, const f16x8& yhs, const f16x8& yl,
                                              const f16x8& yh, f32x4_ c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(yh, xl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(yl, xh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(yhs, xh, c, 0, 0, 0);
  return c;
}

template <int N>
__device__ __forceinline__ void wvm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int remap(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  return xcd * base + (xcd < extra ? xcd : extra) + local;
}

}  // namespace defer

// DIAG: 0 deferred stores, 1 no stores at all (k-loop + conversion only), 2 each tile's stores
// issued right after it (a classic epilogue inside the persistent loop)
template <int NSTAGE, int NK, int DIAG = 0>
__global__ __launch_bounds__(512, 1) void gemm_h3d_kernel(GemmH3Args g) {
  using namespace defer;
  constexpr int BM = 256, BN = 128, BK = 32, NW = 8;
  constexpr int APT = BM * BK * 2, WPT = BN * BK * 2;
  constexpr int STAGE = 2 * APT + 2 * WPT;
  constexpr int PIECES = STAGE / 1024, PPW = PIECES / NW;
  constexpr int SPK = 16 / NK;  // pending stores per k-tile per wave
  static_assert(NSTAGE == 3, "the wait counts below are written for three stages");
  static_assert(16 % NK == 0 && PIECES % NW == 0, "shape");
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE];
  // the bias vector, read once: a global load inside the loop would wait (vmcnt is in order) for
  // every store and copy issued before it
  __shared__ float bias_s[2048];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 64;
  const int num_n = g.Nout / BN, total = (g.R / BM) * num_n;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= total) return;
  const int ntile = (total - (int)blockIdx.x + G - 1) / G;
  const int TK = ntile * NK;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem);
  const uint32_t voff = lane * 16;
  const float accs = g.acc_scale;
  for (int c = tid; c < g.Nout; c += 512) bias_s[c] = g.bias ? g.bias[c] : 0.f;
  __syncthreads();

  auto issue = [&](int gk) __attribute__((always_inline)) {
    const int it = gk / NK, kt = gk - it * NK;
    const int t = remap(it * G + (int)blockIdx.x, total);
    const int tm = t / num_n;
    const int m0 = tm * BM, n0 = (t - tm * num_n) * BN;
    const uint32_t dst = lds0 + (uint32_t)((gk % NSTAGE) * STAGE);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      if (q < 2 * (APT / 1024)) {
        const int pl = q / (APT / 1024), pc = q % (APT / 1024);
        const char* src = reinterpret_cast<const char*>(g.A0.p + pl * g.A0.ps + ((size_t)kt * g.A0.rows_pad + m0) * BK) + pc * 1024;
        dma16_nt(src, voff, dst + q * 1024);
      } else {
        const int qw = q - 2 * (APT / 1024);
        const int pl = qw / (WPT / 1024), pc = qw % (WPT / 1024);
        const char* src = reinterpret_cast<const char*>(g.W.p + pl * g.W.ps + ((size_t)kt * g.W.rows_pad + n0) * BK) + pc * 1024;
        dma16(src, voff, dst + q * 1024);
      }
    }
  };

  auto frag = [&](const char* st, int t0, int r, int c) {
    return *reinterpret_cast<const f16x8*>(st + t0 + r * (BK * 2) + ((c ^ plane_swz(r)) << 4));
  };
  f32x4 acc[4][4];  // [16-column block j][16-row block i]: lane holds columns 4 (lane >> 4) + r of row lane & 15
  f32x4 pend[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = pend[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int stage) __attribute__((always_inline)) {
    const char* st = smem + stage * STAGE;
    const int c = lane >> 4, r16 = lane & 15;
    f16x8 ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm0 + i * 16 + r16;
      ah[i] = frag(st, 0, r, c);
      al[i] = frag(st, APT, r, c);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn0 + j * 16 + r16;
      const f16x8 wh = frag(st, 2 * APT, r, c);
      const f16x8 wl = frag(st, 2 * APT + WPT, r, c);
      const f16x8 whs = wh * (_Float16)kLoScale;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = mfma_h3_16t(ah[i], al[i], whs, wl, wh, acc[j][i]);
    }
  };
  int pm0 = 0, pn0 = 0;
  auto store_one = [&](int q) __attribute__((always_inline)) {
    const int j = q >> 2, i = q & 3;
    const int row = pm0 + wm0 + 16 * i + (lane & 15);
    const int col = pn0 + wn0 + 16 * j + 4 * (lane >> 4);
    *reinterpret_cast<f32x4*>(g.Y + (size_t)row * g.ldy + col) = pend[j][i];
  };

  issue(0);
  if (TK > 1) issue(1);
  for (int it = 0; it < ntile; ++it) {
    const int t = remap(it * G + (int)blockIdx.x, total);
    const int tm = t / num_n;
    const int m0 = tm * BM, n0 = (t - tm * num_n) * BN;
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      const int gk = it * NK + kt;
      // younger than copy gk: the stores of k-tiles gk-2, gk-1 (pending from the previous tile) and copy gk+1
      const bool cn = gk + 1 < TK;
      const int ns = DIAG ? 0 : (gk - 1 >= NK ? 1 : 0) + (gk - 2 >= NK ? 1 : 0);
      if (cn) {
        if (ns == 2) wvm<PPW + 2 * SPK>();
        else if (ns == 1) wvm<PPW + SPK>();
        else wvm<PPW>();
      } else {
        if (ns == 2) wvm<2 * SPK>();
        else if (ns == 1) wvm<SPK>();
        else wvm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (gk + 2 < TK) issue(gk + 2);
      if (DIAG == 0 && it > 0) {
#pragma unroll
        for (int s = 0; s < SPK; ++s) store_one(kt * SPK + s);
      }
      compute(gk % NSTAGE);
    }
    // the tile's result becomes the pending output: stored under the next tile's k-loop
    f32x4 bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = *reinterpret_cast<const f32x4*>(bias_s + n0 + wn0 + 16 * j + 4 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) pend[j][i][r] = fmaf(acc[j][i][r], accs, bj[j][r]);
        acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    pm0 = m0;
    pn0 = n0;
    if (DIAG == 2) {
#pragma unroll
      for (int q = 0; q < 16; ++q) store_one(q);
      wvm<0>();  // the wait counts above assume no stores in flight
    }
    if (DIAG == 1) {  // keep every product live
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) t += (pend[j][i][0] + pend[j][i][1]) + (pend[j][i][2] + pend[j][i][3]);
      if (t == 1234.5f) g.Y[tid] = t;
    }
  }
  if (DIAG == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) store_one(q);
  }
}

// grid = one workgroup per CU (or fewer when there are fewer tiles)
template <int NK, int DIAG = 0>
hipError_t gemm_h3d(const GemmH3Args& a, hipStream_t st, int grid) {
  const int total = (a.R / 256) * (a.Nout / 128);
  hipLaunchKernelGGL((gemm_h3d_kernel<3, NK, DIAG>), dim3(grid < total ? grid : total), dim3(512), 0, st, a);
  return hipGetLastError();
}

}  // namespace lg
