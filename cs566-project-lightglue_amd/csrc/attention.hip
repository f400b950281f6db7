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

// ----------------------------------------------------------------------------------------
// bf16x6 variant (fp32-accurate, see common.h): the same dataflow on v_mfma_f32_32x32x16_bf16.
//  * Q pieces live in registers (3 x 4 k-steps x bf16x8 per lane).
//  * K and V are split into three bf16 planes while they are staged into LDS; V is staged
//    transposed ([dim][key]) so the PV A-operand is two 8-byte reads per plane.
//  * The S^T accumulator is split per 8 registers into the B operand of O^T += V^T P^T (the
//    accumulator-as-operand k order: register 8s+j of lane half h is key 16s + 8(j>>2) + 4h + (j&3)).
// Plane row strides: K 72 bf16 (36 dwords: conflict-free ds_read_b128 groups), V^T 68 bf16
// (34 dwords: the 32 lanes of each ds_read_b64 half cover all 64 banks).
// ----------------------------------------------------------------------------------------
template <int WAVES, int KT>
__global__ __launch_bounds__(64 * WAVES) void attention_x6_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                   float scale_log2e) {
  constexpr int NT = 64 * WAVES;
  constexpr int QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  constexpr int KLD = kHeadDim + 8;  // bf16
  constexpr int VLD = KT + 4;        // bf16 (KT = 64 -> 68)
  constexpr int LDK = KT * 16 / NT;  // float4 K loads per thread per tile
  constexpr int LDV = KT * 16 / NT;  // 4-key x 1-dim V groups per thread per tile
  static_assert(KT * 16 % NT == 0, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) __bf16 Ks[2][3][KT * KLD];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[2][3][kHeadDim * VLD];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
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

  // Q^T B operand: k-step s, lane half h holds dims 16s + 8h + j (j = 0..7) of its query.
  const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
  bf16x8 qp[3][4];
  {
    const float* qr = Q + (size_t)qrow * kHeadDim + half * 8;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(qr + 16 * s);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(qr + 16 * s + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 h, m, l;
        split3(e < 4 ? x0[e] : x1[e - 4], h, m, l);
        qp[0][s][e] = h; qp[1][s][e] = m; qp[2][s][e] = l;
      }
    }
  }

  f32x4 rk[LDK];
  float rv[LDV][4];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDK; ++i) {
      const int q = tid + i * NT;
      const int r = q >> 4, c4 = q & 15;
      const int key = min(t0 + r, Nk - 1);
      rk[i] = *reinterpret_cast<const f32x4*>(K + (size_t)key * kHeadDim + c4 * 4);
    }
#pragma unroll
    for (int i = 0; i < LDV; ++i) {
      const int q = tid + i * NT;
      const int kg = q >> 6, d = q & 63;  // lanes walk dims: coalesced 256-B rows
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int key = min(t0 + 4 * kg + e, Nk - 1);
        rv[i][e] = V[(size_t)key * kHeadDim + d];
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDK; ++i) {
      const int q = tid + i * NT;
      const int r = q >> 4, c4 = q & 15;
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 a, bb, c;
        split3(rk[i][e], a, bb, c);
        h[e] = a; m[e] = bb; l[e] = c;
      }
      *reinterpret_cast<bf16x4*>(&Ks[buf][0][r * KLD + c4 * 4]) = h;
      *reinterpret_cast<bf16x4*>(&Ks[buf][1][r * KLD + c4 * 4]) = m;
      *reinterpret_cast<bf16x4*>(&Ks[buf][2][r * KLD + c4 * 4]) = l;
    }
#pragma unroll
    for (int i = 0; i < LDV; ++i) {
      const int q = tid + i * NT;
      const int kg = q >> 6, d = q & 63;
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 a, bb, c;
        split3(rv[i][e], a, bb, c);
        h[e] = a; m[e] = bb; l[e] = c;
      }
      *reinterpret_cast<bf16x4*>(&Vs[buf][0][d * VLD + 4 * kg]) = h;
      *reinterpret_cast<bf16x4*>(&Vs[buf][1][d * VLD + 4 * kg]) = m;
      *reinterpret_cast<bf16x4*>(&Vs[buf][2][d * VLD + 4 * kg]) = l;
    }
  };

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};  // O^T tiles: dims [0,32) and [32,64), query on lane
  float m_run = -INFINITY;
  float l_run = 0.f;

  const int ntiles = (Nk + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    if (t + 1 < ntiles) gload(t0 + KT);

    // ---- S^T = K Q^T
    f32x16 sc[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      sc[u] = f32x16{0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int off = (u * 32 + l32) * KLD + 16 * s + 8 * half;
        const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(&Ks[cur][0][off]);
        const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(&Ks[cur][1][off]);
        const bf16x8 k2 = *reinterpret_cast<const bf16x8*>(&Ks[cur][2][off]);
        sc[u] = mfma_x6(k0, k1, k2, qp[0][s], qp[1][s], qp[2][s], sc[u]);
      }
    }
    // ---- mask (last tile), online softmax
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

    // ---- O^T += V^T P^T, 16 keys per MFMA step
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 p0, p1, p2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 a, bb, c;
          split3(sc[u][8 * s + j], a, bb, c);
          p0[j] = a; p1[j] = bb; p2[j] = c;
        }
        const int ka = u * 32 + 16 * s + 4 * half;  // keys ka..ka+3 and ka+8..ka+11
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          bf16x8 v[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const __bf16* vr = &Vs[cur][p][(dt * 32 + l32) * VLD];
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(vr + ka);
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(vr + ka + 8);
            v[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          if (dt == 0) o0 = mfma_x6(v[0], v[1], v[2], p0, p1, p2, o0);
          else o1 = mfma_x6(v[0], v[1], v[2], p0, p1, p2, o1);
        }
      }

    if (t + 1 < ntiles) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_tot;
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    float* orow = S.o + ((size_t)b * Nq + q) * kDim + head * kHeadDim;
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
static hipError_t attention_x6_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_x6_kernel<WAVES, KT>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
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

#ifndef LG_ATTN_X6
#define LG_ATTN_X6 1
#endif

hipError_t attention_f32(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  if (LG_ATTN_X6) return attention_x6_launch<LG_ATTN_CONFIG>(s0, s1, B, H, scale, st);
  return attention_launch<LG_ATTN_CONFIG>(s0, s1, B, H, scale, st);
}

}  // namespace lg
