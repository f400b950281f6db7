// fp32-accurate "linear" GEMM on gfx950 matrix cores, with fused epilogues.
//
//   Y[r, c] = epilogue( sum_k A[r, k] * W[c, k] + bias[c] )
//
// Replaces every nn.Linear on the LightGlue hot path (reference lightglue.py):
//   SelfBlock.Wqkv        :168,184   -> EPI_QKV_ROT  (+ rotary :36-43,187-188, head-major scatter :185-186)
//   SelfBlock.out_proj    :170,190   -> folded into ffn.0 at load time (or EPI_STORE)
//   CrossBlock.to_qk/to_v :203-204,223-228,235 -> EPI_CROSS_QKV (one GEMM, 512 outputs, qk * scale^0.5)
//   CrossBlock.to_out     :205,246   -> folded into ffn.0 at load time (or EPI_STORE)
//   ffn.0 on cat([x,msg]) :172,191,247-248 -> EPI_STORE with a two-source A (the cat is never built)
//   ffn.3 + residual      :175,191   -> EPI_STORE with res (x + ffn(...))
//   MatchAssignment.final_proj / d^.25 :304,308-310 -> EPI_STORE with out_scale 0.25
//   MatchAssignment einsum bmd,bnd->bmn :311 -> EPI_STORE, batched over pairs (blockIdx.z)
//
// Two arithmetic modes, both fp32-accurate:
//  * MODE_F32: v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain).  K is permuted inside each k-tile
//    (MFMA step s, lane half h uses k = h*BK/2 + s) so a lane's operands for 4 consecutive steps
//    are one 16-byte LDS read.
//  * MODE_X6: "bf16x6" on v_mfma_f32_32x32x16_bf16.  Each fp32 operand is split exactly into
//    three bf16 pieces x = x0 + x1 + x2 (round-to-nearest each; residual <= 2^-27 |x|) when the
//    k-tile is staged into LDS, and the product is accumulated as the six terms whose weight is
//    >= 2^-18 (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0, small terms first).  Every term is an
//    exact bf16*bf16 product summed in fp32, so the result is as accurate as the fp32 chain
//    (simulated: mean relative error 5e-9 vs 2e-8 for fp32 FMA, K = 256) at 6 x 32 cycles per
//    32x32x16 block instead of 8 x 64.
// Tiling: BM x BN block tile, BK-deep k-tiles, one wave per WM x WN sub-tile of 32x32 MFMA
// tiles; LDS rows padded so every 16-lane ds_read_b128 group hits 16 distinct 4-bank slots;
// register-staged double buffer (one barrier per k-tile); blockIdx -> tile through a bijective
// XCD remap so the column tiles of one row panel run on one XCD and share its L2.
#include "common.h"
#include "kernels.h"

namespace lg {

enum GemmMode { MODE_F32 = 0, MODE_X6 = 1 };

__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  return xcd * base + (xcd < extra ? xcd : extra) + local;
}

// Row -> head-major base offset for the two-image row space: rows [0, B*M) are image 0, then
// image 1; destination [set][b][h][n][64].  Returns the offset of head 0; heads are `stride` apart.
__device__ __forceinline__ void head_row_base(const HeadLayout& hl, int row, int& base, int& stride) {
  if (row < hl.B * hl.M) {
    const int b = row / hl.M, n = row - b * hl.M;
    base = (b * hl.H * hl.M + n) * kHeadDim;
    stride = hl.M * kHeadDim;
  } else {
    const int r2 = row - hl.B * hl.M;
    const int b = r2 / hl.N, n = r2 - b * hl.N;
    base = hl.B * hl.H * hl.M * kHeadDim + (b * hl.H * hl.N + n) * kHeadDim;
    stride = hl.N * kHeadDim;
  }
}

template <int MODE, int BM, int BN, int BK>
struct GemmSmem {
  static constexpr int LDF = BK + 4;  // fp32 row stride (floats)
  // bf16x6 planes: unpadded BK-element rows of 16-byte chunks, chunk index XOR-swizzled by
  // swz(row) so that both the ds_write_b128 staging groups and the ds_read_b128 fragment
  // groups ({0-3,12-15,20-27} rows) hit distinct banks.
  static constexpr size_t bytes =
      MODE == MODE_F32 ? 2 * (size_t)(BM + BN) * LDF * 4 : 2 * 3 * (size_t)(BM + BN) * BK * 2;
};

template <int BK>
__device__ __forceinline__ int chunk_swz(int row) {
  static_assert(BK == 16 || BK == 32, "bf16x6 tiles are 16 or 32 deep");
  return BK == 16 ? (row >> 3) & 1 : (row >> 2) & 3;
}

template <int MODE, int BM, int BN, int BK, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void gemm_kernel(GemmArgs args) {
  constexpr int NWN = BN / WN;
  constexpr int NT = 64 * (BM / WM) * NWN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int C4 = BK / 4;              // float4 chunks per row of a k-tile
  constexpr int A_LD = BM * C4 / NT;      // float4 loads per thread per k-tile
  constexpr int B_LD = BN * C4 / NT;
  using SM = GemmSmem<MODE, BM, BN, BK>;
  static_assert(MODE != MODE_F32 || (BM * C4 % NT == 0 && BN * C4 % NT == 0), "tile/threads mismatch");
  static_assert(MODE == MODE_F32 || BK % 16 == 0, "bf16x6 needs BK % 16 == 0");

  __shared__ __attribute__((aligned(16))) char smem[SM::bytes];
  __shared__ int rowinfo[EPI == EPI_STORE || EPI == EPI_PROBE ? 1 : 2 * BM];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5;
  const int wm0 = (wave / NWN) * WM, wn0 = (wave % NWN) * WN;

  const int num_m = (args.R + BM - 1) / BM;
  const int num_n = (args.Nout + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, num_m * num_n);
  const int tm_blk = tile / num_n, tn_blk = tile - tm_blk * num_n;
  const int m0 = tm_blk * BM, n0 = tn_blk * BN;
  const size_t z = blockIdx.z;

  const float* A0 = args.A0 + z * args.sA;
  const float* A1 = args.A1 ? args.A1 + z * args.sA1 : nullptr;
  const float* W = args.W + z * args.sW;

  if constexpr (EPI == EPI_QKV_ROT || EPI == EPI_CROSS_QKV) {
    for (int r = tid; r < BM; r += NT) {
      int base = 0, stride = 0;
      if (m0 + r < args.R) head_row_base(args.hl, m0 + r, base, stride);
      rowinfo[2 * r] = base;
      rowinfo[2 * r + 1] = stride;
    }
  }

  // bf16x6 staging items: 8 consecutive k of one row (A rows first, then W rows)
  constexpr int NCH = BK / 8;
  constexpr int X6_ITEMS = MODE == MODE_X6 ? (BM + BN) * NCH / NT : 1;
  static_assert(MODE == MODE_F32 || (BM + BN) * NCH % NT == 0, "bf16x6 staging/threads mismatch");
  f32x4 rx[X6_ITEMS][2];
  f32x4 ra[A_LD], rb[B_LD];
  auto gload = [&](int kt) {
    if constexpr (MODE == MODE_X6) {
      const int k0 = kt * BK;
      const float* src;
      int ld, kk;
      if (k0 < args.K0) { src = A0; ld = args.lda0; kk = k0; }
      else { src = A1; ld = args.lda1; kk = k0 - args.K0; }
#pragma unroll
      for (int i = 0; i < X6_ITEMS; ++i) {
        const int q = tid + i * NT;
        const float* p;
        if (q < BM * NCH) {
          int row = m0 + q / NCH;
          row = row < args.R ? row : args.R - 1;
          p = src + (size_t)row * ld + kk + (q % NCH) * 8;
        } else {
          const int qb = q - BM * NCH;
          int col = n0 + qb / NCH;
          col = col < args.Nout ? col : args.Nout - 1;
          p = W + (size_t)col * args.ldw + k0 + (qb % NCH) * 8;
        }
        rx[i][0] = *reinterpret_cast<const f32x4*>(p);
        rx[i][1] = *reinterpret_cast<const f32x4*>(p + 4);
      }
      return;
    }
    const int k0 = kt * BK;
    const float* src;
    int ld, kk;
    if (k0 < args.K0) { src = A0; ld = args.lda0; kk = k0; }
    else { src = A1; ld = args.lda1; kk = k0 - args.K0; }
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int q = tid + i * NT;
      const int r = q / C4, c4 = q % C4;
      int row = m0 + r;
      row = row < args.R ? row : args.R - 1;
      ra[i] = *reinterpret_cast<const f32x4*>(src + (size_t)row * ld + kk + c4 * 4);
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int q = tid + i * NT;
      const int r = q / C4, c4 = q % C4;
      int col = n0 + r;
      col = col < args.Nout ? col : args.Nout - 1;
      rb[i] = *reinterpret_cast<const f32x4*>(W + (size_t)col * args.ldw + k0 + c4 * 4);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{0.f};

  // ---------------------------------------------------------------- stage / compute per mode
  auto sstore = [&](int buf) {
    if constexpr (MODE == MODE_F32) {
      float* As = reinterpret_cast<float*>(smem) + (size_t)buf * (BM + BN) * SM::LDF;
      float* Bs = As + BM * SM::LDF;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const int q = tid + i * NT;
        *reinterpret_cast<f32x4*>(&As[(q / C4) * SM::LDF + (q % C4) * 4]) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < B_LD; ++i) {
        const int q = tid + i * NT;
        *reinterpret_cast<f32x4*>(&Bs[(q / C4) * SM::LDF + (q % C4) * 4]) = rb[i];
      }
    } else {
      // three bf16 planes per operand: plane p of A at [p][BM][BK], of W at [p][BN][BK]
      __bf16* As = reinterpret_cast<__bf16*>(smem) + (size_t)buf * 3 * (BM + BN) * BK;
      __bf16* Bs = As + 3 * BM * BK;
#pragma unroll
      for (int i = 0; i < X6_ITEMS; ++i) {
        const int q = tid + i * NT;
        const bool isA = q < BM * NCH;
        const int qq = isA ? q : q - BM * NCH;
        const int r = qq / NCH, c = qq % NCH;
        __bf16* base = isA ? As : Bs;
        const int rows = isA ? BM : BN;
        bf16x8 h, m, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          __bf16 a, b, cc;
          split3(rx[i][e >> 2][e & 3], a, b, cc);
          h[e] = a; m[e] = b; l[e] = cc;
        }
        const int off = r * BK + ((c ^ chunk_swz<BK>(r)) * 8);
        *reinterpret_cast<bf16x8*>(base + off) = h;
        *reinterpret_cast<bf16x8*>(base + rows * BK + off) = m;
        *reinterpret_cast<bf16x8*>(base + 2 * rows * BK + off) = l;
      }
    }
  };
  auto compute = [&](int buf) {
    if constexpr (MODE == MODE_F32) {
      constexpr int HK = BK / 2;
      const float* as = reinterpret_cast<const float*>(smem) + (size_t)buf * (BM + BN) * SM::LDF;
      const float* bs = as + BM * SM::LDF;
#pragma unroll
      for (int s4 = 0; s4 < HK / 4; ++s4) {
        f32x4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const f32x4*>(as + (wm0 + i * 32 + l32) * SM::LDF + half * HK + s4 * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const f32x4*>(bs + (wn0 + j * 32 + l32) * SM::LDF + half * HK + s4 * 4);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(a[i][kk], b[j][kk], acc[i][j]);
      }
    } else {
      const __bf16* as = reinterpret_cast<const __bf16*>(smem) + (size_t)buf * 3 * (BM + BN) * BK;
      const __bf16* bs = as + 3 * BM * BK;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 a[TM][3], b[TN][3];
        const int c = 2 * s + half;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int r = wm0 + i * 32 + l32;
            a[i][p] = *reinterpret_cast<const bf16x8*>(as + (p * BM + r) * BK + (c ^ chunk_swz<BK>(r)) * 8);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int r = wn0 + j * 32 + l32;
            b[j][p] = *reinterpret_cast<const bf16x8*>(bs + (p * BN + r) * BK + (c ^ chunk_swz<BK>(r)) * 8);
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma_x6(a[i][0], a[i][1], a[i][2], b[j][0], b[j][1], b[j][2], acc[i][j]);
      }
    }
  };

  const int nk = args.K / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    compute(cur);
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ------------------------------------------------------------------ epilogues
  float* Y = args.Y ? args.Y + z * args.sY : nullptr;
  if constexpr (EPI == EPI_PROBE) {
    // timing probe (tools/kbench_gemm.hip): keeps the accumulators live, stores nothing
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    if (s == 1234.5678f) Y[tid] = s;
  } else if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn0 + j * 32 + l32;
      if (col >= args.Nout) continue;
      const float bj = args.bias ? args.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + i * 32 + row32(r, half);
          if (row >= args.R) continue;
          float v = (acc[i][j][r] + bj) * args.out_scale;
          if (args.res) v = args.res[(size_t)row * args.ldr + col] + v;
          Y[(size_t)row * args.ldy + col] = v;
        }
    }
  } else {
    // Head-major scatter.  WN == 64 and n0 + wn0 is a multiple of 64, so the wave owns one
    // (type t, head) block.  The packed weight rows (lightglue_api.cpp: head_perm) put dims
    // 2*l32 (tile 0) and 2*l32+1 (tile 1) of the head in lane l32, so every store is a
    // natural-order pair and the rotary partners meet in one lane.
    //   self  (EPI_QKV_ROT):   t0 -> q fp32 (rotary), t1 -> k bf16 planes (rotary), t2 -> v planes
    //   cross (EPI_CROSS_QKV): t0 -> qk fp32 * scale^0.5 and qk planes,             t1 -> v planes
    static_assert(WN == 64 && TN == 2, "head epilogues need 64-wide wave tiles");
    const HeadLayout& hl = args.hl;
    const int cbase = n0 + wn0;
    const int t = cbase / kDim, head = (cbase % kDim) / kHeadDim;
    const bool rot = EPI == EPI_QKV_ROT && t < 2;
    const bool to_q = t == 0;
    const bool to_kp = EPI == EPI_QKV_ROT ? t == 1 : t == 0;
    const bool to_vp = EPI == EPI_QKV_ROT ? t == 2 : t == 1;
    const float sc = (EPI == EPI_CROSS_QKV && t == 0) ? hl.qk_scale : 1.f;
    const float be = args.bias[cbase + l32], bo = args.bias[cbase + 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm0 + i * 32 + row32(r, half);
        const int row = m0 + lr;
        if (row >= args.R) continue;
        const size_t off = (size_t)rowinfo[2 * lr] + (size_t)head * rowinfo[2 * lr + 1] + 2 * l32;
        float xe = acc[i][0][r] + be;  // dim 2*l32   (even)
        float xo = acc[i][1][r] + bo;  // dim 2*l32+1 (odd)
        if (rot) {
          // t*cos + rotate_half(t)*sin, rotate_half(x)[2i] = -x[2i+1], [2i+1] = x[2i]
          const float c = hl.cosb[(size_t)row * kFreq + l32];
          const float s = hl.sinb[(size_t)row * kFreq + l32];
          const float e2 = add_rn(mul_rn(xe, c), mul_rn(-xo, s));
          const float o2 = add_rn(mul_rn(xo, c), mul_rn(xe, s));
          xe = e2;
          xo = o2;
        }
        xe *= sc;
        xo *= sc;
        if (to_q) *reinterpret_cast<float2*>(hl.q + off) = make_float2(xe, xo);
        if (to_kp || to_vp) {
          __bf16* base = to_kp ? hl.kp : hl.vp;
          __bf16 eh, em, el, oh, om, ol;
          split3(xe, eh, em, el);
          split3(xo, oh, om, ol);
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<bf16x2*>(base + off) = bf16x2{eh, oh};
          *reinterpret_cast<bf16x2*>(base + hl.pstride + off) = bf16x2{em, om};
          *reinterpret_cast<bf16x2*>(base + 2 * hl.pstride + off) = bf16x2{el, ol};
        }
      }
  }
}

template <int MODE, int BM, int BN, int BK, int WM, int WN, int EPI>
static hipError_t launch(const GemmArgs& a, int batch, hipStream_t st) {
  const int nt = 64 * (BM / WM) * (BN / WN);
  const int blocks = ((a.R + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
  if (blocks == 0 || batch == 0) return hipSuccess;
  if (a.K % BK != 0 || (a.A1 && a.K0 % BK != 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, BK, WM, WN, EPI>), dim3(blocks, 1, batch), dim3(nt), 0, st, a);
  return hipGetLastError();
}

#ifndef LG_GEMM_CONFIG
// MODE, BM, BN, BK, WM, WN: chosen by tools/kbench_gemm.hip on MI355X (K = 256/512 shapes of
// this model, R = 131072 rows).
// bf16x6 at 256x256x16 with 16 waves of 64x64 ran 173-198 TF/s on the four Linear shapes
// (fp32 MFMA 256x128x16: 95-120 TF/s) with a lower error vs fp64 (mean 1.4e-8 vs 1.7e-8).
#define LG_GEMM_CONFIG MODE_X6, 256, 256, 16, 64, 64
#endif

hipError_t gemm_f32(const GemmArgs& a, int epi, int batch, hipStream_t st) {
  switch (epi) {
    case EPI_STORE:
      return launch<LG_GEMM_CONFIG, EPI_STORE>(a, batch, st);
    case EPI_QKV_ROT:
      return launch<LG_GEMM_CONFIG, EPI_QKV_ROT>(a, batch, st);
    case EPI_CROSS_QKV:
      return launch<LG_GEMM_CONFIG, EPI_CROSS_QKV>(a, batch, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace lg
