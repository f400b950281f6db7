// Flash-style fp32 attention on gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
//   O = softmax(Q K^T * scale) V      per (set, pair, head); never materialises the N x N scores.
//
// Replaces (reference lightglue.py):
//   Attention.forward / F.scaled_dot_product_attention  :139-149  (self, scale 1/sqrt(64))
//   CrossBlock sim / softmax / einsum                    :235-242  (cross, scale 1: the
//     s^0.5 factors are applied to qk in the GEMM epilogue).  attn10 = softmax over the
//     transposed sim is computed as a second set with Q/K swapped: m1 = softmax_i(sim)^T v0
//     equals attention(q = qk1, k = qk0, v = v0), the same identity the reference's flash path
//     uses (:229-233).
//
// Structure: a workgroup of WAVES waves owns 32*WAVES queries of one (set, pair, head); each
// wave 32 queries.  K/V stream through LDS in KT-key tiles (register-staged, double-buffered).
// S^T = K Q^T is computed with the KEY on the MFMA row and the QUERY on the lane, so each lane
// holds the scores of one query: the softmax row reduction is in-register plus one exchange
// with lane^32, and the probability accumulator is directly the B operand of O^T = V^T P^T
// (no LDS round trip for P).  Q lives in registers (32 floats per lane).
// Work items (set, pair*head, query block) are walked through an XCD-aware remap so that the
// query blocks sharing one K/V run on the same XCD (L2).
#include "common.h"
#include "kernels.h"

namespace lg {

constexpr int KS = kHeadDim + 4;  // LDS row stride (floats): conflict-free ds_read_b128 rows

__device__ __forceinline__ int xcd_chunk(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  return xcd * base + (xcd < extra ? xcd : extra) + local;
}

template <int WAVES, int KT>
__global__ __launch_bounds__(64 * WAVES) void attention_f32_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                    float scale_log2e) {
  constexpr int NT = 64 * WAVES;
  constexpr int QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;                 // 32-key sub-tiles per tile
  constexpr int LD = KT * 16 / NT;              // float4 loads per thread per tile (each of K, V)
  __shared__ float Ks[2][KT * KS];
  __shared__ float Vs[2][KT * KS];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;                   // set * (B*H) + bh
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const float* K = S.k + (size_t)bh * Nk * kHeadDim;
  const float* V = S.v + (size_t)bh * Nk * kHeadDim;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5;

  // Q operand for the 32 MFMA steps: step s covers dims {s, 32+s}; lane half h supplies dim 32h+s.
  const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
  float qreg[32];
  {
    const f32x4* qp = reinterpret_cast<const f32x4*>(Q + (size_t)qrow * kHeadDim + half * 32);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 v = qp[i];
      qreg[4 * i + 0] = v[0]; qreg[4 * i + 1] = v[1]; qreg[4 * i + 2] = v[2]; qreg[4 * i + 3] = v[3];
    }
  }

  f32x4 rk[LD], rv[LD];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int q = tid + i * NT;
      const int r = q >> 4, c4 = q & 15;
      const int key = min(t0 + r, Nk - 1);
      rk[i] = *reinterpret_cast<const f32x4*>(K + (size_t)key * kHeadDim + c4 * 4);
      rv[i] = *reinterpret_cast<const f32x4*>(V + (size_t)key * kHeadDim + c4 * 4);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int q = tid + i * NT;
      const int r = q >> 4, c4 = q & 15;
      *reinterpret_cast<f32x4*>(&Ks[buf][r * KS + c4 * 4]) = rk[i];
      *reinterpret_cast<f32x4*>(&Vs[buf][r * KS + c4 * 4]) = rv[i];
    }
  };

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};  // O^T tiles: dims [0,32) and [32,64), query on lane
  float m_run = -INFINITY;  // running max of raw scores (both halves agree)
  float l_run = 0.f;        // per-lane partial row sum (halves combined at the end)

  const int ntiles = (Nk + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    if (t + 1 < ntiles) gload(t0 + KT);
    const float* ks = &Ks[cur][0];
    const float* vs = &Vs[cur][0];

    // ---- S^T = K Q^T for NSUB 32-key sub-tiles
    f32x16 sc[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      sc[u] = f32x16{0.f};
      const float* kr = ks + (u * 32 + l32) * KS + half * 32;
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) {
        const f32x4 kv = *reinterpret_cast<const f32x4*>(kr + s4 * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[u] = mfma32(kv[j], qreg[s4 * 4 + j], sc[u]);
      }
    }
    // ---- mask keys beyond Nk (last tile only), online softmax
    if (t0 + KT > Nk) {
#pragma unroll
      for (int u = 0; u < NSUB; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[u][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * scale_log2e);
    m_run = m_new;
    const float mb = m_new * scale_log2e;
    float psum = 0.f;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[u][r], scale_log2e, -mb));
        sc[u][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }

    // ---- O^T += V^T P^T : step (u, r) consumes key u*32 + row32(r, half) for this lane half
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* vr = vs + (u * 32 + row32(r, half)) * KS + l32;
        o0 = mfma32(vr[0], sc[u][r], o0);
        o1 = mfma32(vr[32], sc[u][r], o1);
      }

    if (t + 1 < ntiles) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- finalise: combine the two lane halves' row sums, normalise, store rows of O.
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_tot;
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    float* orow = S.o + ((size_t)b * Nq + q) * kDim + head * kHeadDim;
    // register r holds dim row32(r, half) (+32 for o1): r = 4g + e -> dim 8g + 4*half + e
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 a = {o0[4 * g] * inv, o0[4 * g + 1] * inv, o0[4 * g + 2] * inv, o0[4 * g + 3] * inv};
      f32x4 c = {o1[4 * g] * inv, o1[4 * g + 1] * inv, o1[4 * g + 2] * inv, o1[4 * g + 3] * inv};
      *reinterpret_cast<f32x4*>(orow + 8 * g + 4 * half) = a;
      *reinterpret_cast<f32x4*>(orow + 32 + 8 * g + 4 * half) = c;
    }
  }
}

template <int WAVES, int KT>
static hipError_t attention_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_f32_kernel<WAVES, KT>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

#ifndef LG_ATTN_CONFIG
// WAVES, KT: 8 waves (256 queries) per workgroup, 64-key tiles (tools/kbench_attn.hip).
#define LG_ATTN_CONFIG 8, 64
#endif

hipError_t attention_f32(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  return attention_launch<LG_ATTN_CONFIG>(s0, s1, B, H, scale, st);
}

}  // namespace lg
