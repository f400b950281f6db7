// Flash-style fp32-accurate attention on gfx950 matrix cores: fp16x3 (PREC_H3, default) and
// bf16x6 (PREC_X6) operand formats, see common.h.
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
// wave 32 queries.  K and V arrive already split into three bf16 planes (written by the QKV
// GEMM epilogue) and stream through LDS in KT-key tiles (register-staged, double-buffered).
//  * S^T = K Q^T puts the KEY on the MFMA row and the QUERY on the lane, so each lane holds
//    the scores of one query: the softmax row reduction is in-register plus one exchange with
//    lane^32.  Q pieces live in registers (3 x 4 k-steps x bf16x8 per lane).
//  * The S^T accumulator, split per 8 registers, is directly the B operand of O^T += V^T P^T
//    (register 8s+j of lane half h is key 16s + 8(j>>2) + 4h + (j&3)); the matching V^T
//    A-operand is read from the row-major V tile with ds_read_b64_tr_b16 (4 keys x 16 dims
//    per 16-lane group, delivered dim-on-lane).
//  * LDS images: K planes [key][72] (36-dword rows: the 16 lanes of each ds_read_b128 group hit
//    16 distinct 4-bank slots); V planes [key][64] with the two 32-dim halves swapped on rows
//    whose key bit 1 is set (each transposed read's 4 rows x 64 B then cover all 64 banks).
// Work items (set, pair*head, query block) are walked through an XCD-aware remap so that the
// query blocks sharing one K/V run on the same XCD (L2).
#include <type_traits>

#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"

namespace lg {

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_chunk(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  return xcd * base + (xcd < extra ? xcd : extra) + local;
}
#ifndef LG_ATTN_CTX_NT
// context planes with the non-temporal hint: -0.1 ms per forward while the attention walked its
// items front to back; with the reversed walk the LN GEMM reads the newest context first and
// cached stores win (three same-box pairs: 1312 vs 1301 pairs/s)
#define LG_ATTN_CTX_NT 0
#endif
// common-form lazy softmax reference (log2 units of the score accumulator, e = 2^acc): a query is
// re-referenced when a score tile's max passes LG_ATTN_RAISE, to put that max at LG_ATTN_REF
// (e <= 2^LG_ATTN_RAISE < 65504 keeps every e an fp16 for the P split)
#ifndef LG_ATTN_RAISE
#define LG_ATTN_RAISE 14
#endif
#ifndef LG_ATTN_REF
#define LG_ATTN_REF 11
#endif
static_assert(LG_ATTN_RAISE <= 15, "e = 2^acc <= 2^LG_ATTN_RAISE must stay a finite fp16 for the P split");
static_assert(LG_ATTN_REF < LG_ATTN_RAISE, "the re-reference target must lie below the raise threshold");
#ifndef LG_ATTN_REVERSE
#define LG_ATTN_REVERSE 1  // configs[2] three same-box pairs: 1326 vs 1321 pairs/s, attention -0.6 %
#endif
// the same chunks, each XCD walking its chunk from the end: the QKV GEMM wrote every XCD's rows
// front to back, so the newest q/k/v (the ones still in the Infinity Cache) come first
__device__ __forceinline__ int xcd_chunk_rev(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  const int cnt = base + (xcd < extra ? 1 : 0);
  return xcd * base + (xcd < extra ? xcd : extra) + (cnt - 1 - local);
}

__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

template <int WAVES, int KT>
__global__ __launch_bounds__(64 * WAVES) void attention_x6_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                   float scale_log2e) {
  constexpr int NT = 64 * WAVES;
  constexpr int QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  constexpr int KLD = kHeadDim + 8;       // K plane row stride (bf16)
  constexpr int CH = 3 * KT * 8;          // 16-byte chunks per tile per tensor (3 planes x KT rows x 8)
  constexpr int LDC = CH / NT;            // chunks per thread per tensor
  static_assert(CH % NT == 0, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) __bf16 Ks[2][3][KT * KLD];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[2][3][KT * kHeadDim];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  // S.Nq / S.Nk are the layout capacities; per-pair counts (batched pruning) bound the loops
  const int NqS = S.Nq, NkS = S.Nk, pb = bh / H;
  if (S.act && !S.act[pb]) return;
  const int Nq = S.nq_cnt ? S.nq_cnt[pb] : NqS, Nk = S.nk_cnt ? S.nk_cnt[pb] : NkS;
  if (q_blk >= Nq || Nk <= 0) return;
  const float* Q = static_cast<const float*>(S.q) + (size_t)bh * NqS * kHeadDim;
  const __bf16* Kp = static_cast<const __bf16*>(S.kp) + (size_t)bh * NkS * kHeadDim;
  const __bf16* Vp = static_cast<const __bf16*>(S.vp) + (size_t)bh * NkS * kHeadDim;
  const long long ps = S.pstride;
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

  // tile staging: chunk c -> plane c / (KT*8), row (c / 8) % KT, 8-dim column block c % 8
  bf16x8 rk[LDC], rv[LDC];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      const size_t src = (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8;
      rk[i] = *reinterpret_cast<const bf16x8*>(Kp + src);
      rv[i] = *reinterpret_cast<const bf16x8*>(Vp + src);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<bf16x8*>(&Ks[buf][p][r * KLD + cb * 8]) = rk[i];
      *reinterpret_cast<bf16x8*>(&Vs[buf][p][r * kHeadDim + ((cb ^ (((r >> 1) & 1) << 2)) * 8)]) = rv[i];
    }
  };

  // per-lane constants of the transposed V reads: 16-lane group g = lane >> 4 covers dims
  // (g & 1) * 16 .. +15 of lane half h = g >> 1; lane 4q+p of the group addresses row q, dims 4p..4p+3
  const int tq = (lane & 15) >> 2, tp = lane & 3, tdim = ((lane >> 4) & 1) * 16 + 4 * tp;

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
    tmax = max_xor32(tmax);
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * scale_log2e);
    m_run = m_new;
    // (s - m) first: exact for the keys that matter, whatever the logits' magnitude (the fused
    // fma(s, c, -m c) loses absolute accuracy once m c is beyond 2^24)
    float psum = 0.f;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f((sc[u][r] - m_new) * scale_log2e);
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
        // keys of element j: ka + j (j < 4), ka + 8 + (j - 4) (j >= 4); transposed-read row = ka + tq
        const int ka = u * 32 + 16 * s + 4 * half;
        const int r0 = ka + tq, r1 = ka + 8 + tq;  // r0, r1 share bit 1 (ka % 4 == 0)
        const int sw = ((r0 >> 1) & 1) << 5;       // half swap, in dims
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = (dt * 32 + tdim) ^ sw;
          bf16x8 v[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const bf16x4 lo = tr_read(&Vs[cur][p][r0 * kHeadDim + dcol]);
            const bf16x4 hi = tr_read(&Vs[cur][p][r1 * kHeadDim + dcol]);
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

  const float l_tot = sum_xor32(l_run);
  const float inv = 1.f / l_tot;
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    float* orow = S.o + ((size_t)b * NqS + q) * kDim + head * kHeadDim;
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
// fp16x3 attention (PREC_H3, common.h): the bf16x6 tiling above with half the MFMAs.
//  * K arrives as two fp16 planes (h, l*2^11), V as (h, l) (split2h_v, two-sided range exponent)
//    from the QKV GEMM epilogue.
//  * Each query row is scaled by 2^e (per lane: the query sits on the lane) so that
//    max|q 2^e| lies in [8, 16); its pieces (h*2^11, l, h) stay in registers.  The S^T
//    accumulator then holds 2^(11+e) q.k, and the per-lane factor scale*log2(e)*2^-(11+e)
//    folds into the fma that feeds exp2 -- the softmax costs nothing extra.
//  * Lazy max: a query's softmax reference is raised only when a tile would push its
//    probabilities above 2^3 (p <= 8 keeps p_h * 2^11 inside fp16); otherwise the O / l rescale
//    is skipped for the whole wave (ballot) -- after the first tiles it almost always is.
//  * P is split in-register with fp16 arithmetic: p_h = fp16(p), p_h 2^11 by an fp16 multiply
//    (exact), p_l = fp16(p 2^11 - p_h 2^11) in one mixed-precision fma (exact before its
//    rounding); O accumulates 2^11 * P V and the 2^-11 folds into the final 1/l.
//  * Tree reductions for the tile max / sum; per-lane LDS offsets hoisted out of the loop.
//  * The context is written straight into the plane image that ffn.0 consumes (common.h).
// (These numerics are shared by the production attention_h3g_kernel below; the first kernel
// built on them, attention_h3_kernel, now lives in tools/attn_h3_legacy.hip.)
// ----------------------------------------------------------------------------------------
// 8 consecutive dims of a query row (element offset off from q, the head's [Nq][64] block):
// fp32 rows or (QP) a plane image (plane stride ps), whose h + l 2^-11 is exact in fp32 (22 significant
// bits), times 2^E of its range slot (qsc) -- the values the fp32 rows would hold
template <bool QP>
__device__ __forceinline__ void load_q8(const void* q, long long ps, size_t off, float qsc, f32x4& a, f32x4& b) {
  if constexpr (QP) {
    const _Float16* qp = static_cast<const _Float16*>(q) + off;
    const f16x8 h = *reinterpret_cast<const f16x8*>(qp);
    const f16x8 l = *reinterpret_cast<const f16x8*>(qp + ps);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = ((float)h[e] + (float)l[e] * (1.f / kLoScale)) * qsc;
      b[e] = ((float)h[e + 4] + (float)l[e + 4] * (1.f / kLoScale)) * qsc;
    }
  } else {
    const float* qf = static_cast<const float*>(q) + off;
    a = *reinterpret_cast<const f32x4*>(qf);
    b = *reinterpret_cast<const f32x4*>(qf + 4);
  }
}

__device__ __forceinline__ f16x4 tr_read_h(const _Float16* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(f16x4, v);
}



// ----------------------------------------------------------------------------------------
// fp16x3 attention (PREC_H3; attention_h3f/h3g kernels): 8 waves x 32 queries, 64-key
// K/V softmax steps, tiles double-buffered in LDS, lazy softmax reference, context
// straight into ffn.0's plane image, all products on v_mfma_f32_16x16x32_f16 (16 x 16 tiles run
// at ~1.15x the rate of 32 x 32 tiles on random data, tools/probe_mfma_shape.hip):
//   S^T[key][query] = K Q^T:  A = K tile (16 keys x 32 dims, lane: key l&15, dims 8(l>>4)..),
//                             B = Q^T (lane: query l&15, dims 8(l>>4)..), two k-steps per head.
//     Accumulator: lane l holds query l&15, keys 4(l>>4) + r (r < 4) of each 16-key tile.
//   O^T[dim][query] += V^T P^T over 32-key steps p: B = P^T with k index 8g+j <-> key
//     32p + 16(j>>2) + 4g + (j&3) (g = l>>4) -- exactly the S^T registers the lane already holds;
//     A = V^T, lane: dim l&15 of a 16-dim tile, the same 8 keys, two ds_read_b64_tr_b16.
//   Per-query reductions run over the 4 lanes sharing l&15 via v_permlane{16,32}_swap.
// LDS: rows of 64 halves (128 B); K 16-byte chunk c of row r at c ^ ((r >> 1) & 7), V chunk c at
// c ^ 2((r >> 1) & 3) -- conflict-free for the b128 fragment reads and the transposed reads.
// Softmax VALU trimmed to what the MFMA gaps can hide (the earlier h3/h3m loops issued ~13 VALU
// per score; tools/attn_experiments.hip keeps them):
//   * the tile body is instantiated per LDS buffer (static ds_read offsets) and per masking mode
//     (only the ragged last tile compares key indices);
//   * P is produced pre-scaled: e = exp2(s c - (m c - 11)) = p 2^11 is exactly the "yhs" MFMA
//     operand (hs = fp16(e) = fp16(p) 2^11 for p >= 2^-14), the low piece e - hs is formed and
//     rounded to fp16 by one v_fma_mix{lo,hi}_f16 per score, and yh = hs 2^-11 is one packed
//     fp16 multiply per two scores; l accumulates e (2^11 l), folded into the final scale;
//   * the tile max is a v_max3 tree per lane; the cross-lane reduction and the reference raise
//     run only when some lane's max could need a raise (ballot), so the common tile has no
//     cross-lane step between the score MFMAs and the exponentials.
// ----------------------------------------------------------------------------------------
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// (e0 - hs[0], e1 - hs[1]) rounded to fp16, one instruction per element (both differences are
// exact in fp32: hs = fp16(e))
__device__ __forceinline__ f16x2 lo_pair(float e0, float e1, f16x2 hs) {
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(e0), "v"(hs));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(e1), "v"(hs));
  return __builtin_bit_cast(f16x2, l);
}
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
// the common form's score max tree: llvm.maximum (v_maximum3_f32 on gfx950) takes the MFMA results
// as they are, where fmaxf's maxnum first quiets each operand it cannot prove canonical (a
// v_max_f32 x, x); the two differ only on NaN, which the exponentials propagate either way
__device__ __forceinline__ float max2m(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float max3m(float a, float b, float c) { return max2m(max2m(a, b), c); }
// op over the 4 lanes l, l^16, l^32, l^48 through v_permlane{16,32}_swap (no LDS round trip)
__device__ __forceinline__ float max_x16_32(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max_xor32(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
__device__ __forceinline__ float sum_x16_32(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return sum_xor32(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}


// attention_h3g_kernel: the production kernel of the design above.  K/V tiles are staged by
// LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write; the swizzle is applied by
// the per-lane source offsets), SUBS 64-key softmax steps per LDS tile, i.e. per barrier
// (SUBS = 2: 2 x 64 KiB of LDS), and PRIO raises the second-dispatched half of the waves to
// s_setprio 1 once.  tools/kbench_attn.hip: 862 us vs 907-918 us for the register-staged
// attention_h3f_kernel (tools/attn_experiments.hip) at the bench shape.
// SPLIT (small batches): the keys of a work item are cut into nsplit ranges of lsplit keys, one
// workgroup each; instead of the context the workgroup writes its unnormalised partial (O, the
// softmax reference m, the 2^11-scaled sum l and the query's exponent factor c) and
// attn_split_combine_kernel merges the ranges.
template <int SUBS, int PRIO, int WAVES = 8, bool SPLIT = false, bool QP = false>
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 ? 2 : 1) void attention_h3g_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                float scale_log2e, float* part = nullptr,
                                                                int nsplit = 1, int lsplit = 0) {
  constexpr int QB = 32 * WAVES;
  constexpr int KT = 64;                   // keys per sub-tile (one softmax step)
  constexpr int LT = KT * SUBS;            // keys per LDS tile (one barrier)
  constexpr int NKT = KT / 16;
  constexpr int PL = LT * kHeadDim;        // one plane of an LDS tile (elements)
  constexpr int PIECES = 4 * LT / 8;       // 1 KiB LDS-DMA pieces per tile (K h/l, V h/l; 8 rows each)
  constexpr int PPW = PIECES / WAVES;
  static_assert(PIECES % WAVES == 0, "pieces per wave");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * PL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 2 * PL];

  int item = LG_ATTN_REVERSE ? xcd_chunk_rev(blockIdx.x, gridDim.x) : xcd_chunk(blockIdx.x, gridDim.x);
  int split = 0;
  if constexpr (SPLIT) {
    split = item % nsplit;
    item /= nsplit;
  }
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  // S.Nq / S.Nk are the layout capacities; per-pair counts (batched pruning) bound the loops
  const int NqS = S.Nq, NkS = S.Nk, pb = bh / H;
  const int nqs = max(s0.Nq, s1.Nq);  // query stride of the split partials
  if (S.act && !S.act[pb]) return;
  const int Nq = S.nq_cnt ? S.nq_cnt[pb] : NqS;
  int Nk = S.nk_cnt ? S.nk_cnt[pb] : NkS;
  const int k0 = SPLIT ? split * lsplit : 0;
  if constexpr (SPLIT) Nk = min(lsplit, Nk - k0);
  if (q_blk >= Nq) return;
  if (Nk <= 0) {
    if constexpr (SPLIT) {  // an empty key range: a partial that weighs nothing
      for (int q = q_blk + (int)threadIdx.x; q < min(q_blk + QB, Nq); q += 64 * WAVES) {
        const size_t rec = (((size_t)split * 2 + set) * B * H + bh) * nqs + q;
        *reinterpret_cast<f32x4*>(part + (size_t)nsplit * 2 * B * H * nqs * kHeadDim + rec * 4) = f32x4{-INFINITY, 0.f, 1.f, 0.f};
      }
    }
    return;
  }
  const void* Q = QP ? static_cast<const void*>(static_cast<const _Float16*>(S.q) + (size_t)bh * NqS * kHeadDim)
                    : static_cast<const void*>(static_cast<const float*>(S.q) + (size_t)bh * NqS * kHeadDim);
  const float qsc = QP ? ldexpf(1.f, range_slot_exp(S.rtab, S.k_slot)) : 1.f;  // QP: queries from planes
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + ((size_t)bh * NkS + k0) * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + ((size_t)bh * NkS + k0) * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;

  f16x8 qh[2][2], qhs[2][2], ql[2][2];
  float c_lane[2];
  const int ek = range_slot_exp(S.rtab, S.k_slot);  // key planes hold k * 2^-ek (RangeOut)
  // Query pieces, two forms (mfma_h3_16 computes x_l yh + x_h yl + x_h yhs, the key planes being
  // x_h = fp16(k 2^-ek) and x_l = its residual * 2^11):
  //  * common form: y = q scale log2(e) 2^ek split UNSCALED -- yhs = y_h, yl = fp16(y - y_h),
  //    yh = y_h 2^-11 -- so the score accumulator IS the exponent argument in log2 units; each
  //    tile's first MFMA takes C = 11 - m (m the query's softmax reference), so e = p 2^11 =
  //    exp2(accumulator) with no VALU between the MFMA and the exponential.  Small components'
  //    low pieces go subnormal: absolute error <= 2^-25 per component in log2-logit units per unit
  //    of k, below the fp32 reference's own rounding of logits of order 10.
  //  * exact form (extreme or tiny data, wave-uniform): |scale q.k log2 e| <= 64 max|q_row| max|k|
  //    scale log2 e beyond 2^21, or a row's max|y| outside [2^-4, 2^14]: each row scaled by 2^ex into [8, 16), pieces
  //    (h 2^11, l 2^11, h), the accumulator holds 2^(11+ex) q.k, and the exponent argument is
  //    formed as (s - m) c + 11 in VALU with the per-lane factor c.
  const float kmax = S.rtab ? range_max(S.rtab, S.k_slot) : INFINITY;
  const float ysc = ldexpf(scale_log2e, ek);
  bool big = false;
  f32x4 xq[2][2][2];
  int exq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qrow = min(q_blk + wave * 32 + qt * 16 + r16, Nq - 1);
    const size_t qr = (size_t)qrow * kHeadDim + 8 * g;
    float mx = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      load_q8<QP>(Q, S.pstride, qr + 32 * ks, qsc, xq[qt][ks][0], xq[qt][ks][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(xq[qt][ks][0][e]), fabsf(xq[qt][ks][1][e])));
    }
    mx = max_x16_32(mx);
    // common form only for rows whose largest y is in [2^-4, 2^14]: the subnormal low pieces'
    // error (<= 2^-25 sum|x|) then stays under 2^-21 of the row's logit scale (max|y| sum|x|)
    big |= !(64.f * mx * kmax * scale_log2e <= 2097152.f) || !(mx * ysc <= 16384.f) || !(mx * ysc >= 0.0625f);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    exq[qt] = ex;
  }
  const bool exact = __builtin_amdgcn_readfirstlane((int)(__ballot(big) != 0ull)) != 0;  // wave-uniform
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    c_lane[qt] = exact ? ldexpf(scale_log2e, ek - (11 + exq[qt])) : 1.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = xq[qt][ks][e >> 2][e & 3];
        _Float16 h, l;
        if (exact) {
          split2h(ldexpf(xv, exq[qt]), h, l);
          qh[qt][ks][e] = h;
          ql[qt][ks][e] = l;
          qhs[qt][ks][e] = h * (_Float16)kLoScale;
        } else {
          const float y = xv * ysc;
          h = (_Float16)y;
          l = (_Float16)(y - (float)h);  // exact difference, rounded (subnormal when tiny)
          qhs[qt][ks][e] = h;
          ql[qt][ks][e] = l;
          qh[qt][ks][e] = (_Float16)((float)h * (1.f / kLoScale));
        }
      }
  }
  // LDS-DMA staging of one LDS tile (keys t0 .. t0+LT-1) into buffer buf: piece q (wave-uniform)
  // = 8 rows of one plane of K (q < PIECES/2) or V; lane i fills LDS slot (row i>>3, chunk i&7)
  // with the source chunk that the swizzle puts there (rows past Nk repeat row Nk-1)
  const uint32_t ks_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)Ks);
  const uint32_t vs_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)Vs);
  auto issue = [&](int t0, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      const bool isv = q >= PIECES / 2;
      const int qq = isv ? q - PIECES / 2 : q;
      const int pl = qq / (LT / 8), r = (qq % (LT / 8)) * 8 + (lane >> 3), cs = lane & 7;
      const int c = isv ? cs ^ (((r >> 1) & 3) << 1) : cs ^ ((r >> 1) & 7);
      const _Float16* base = (isv ? Vp : Kp) + (size_t)pl * ps + (size_t)t0 * kHeadDim;
      const uint32_t voff = (uint32_t)((min(t0 + r, Nk - 1) - t0) * kHeadDim + c * 8) * 2u;
      const uint32_t dst = (isv ? vs_lds : ks_lds) + (uint32_t)(((buf * 2 + pl) * PL + (qq % (LT / 8)) * 8 * kHeadDim) * 2);
      dma16_u(base, voff, dst);
    }
  };
  // the same staging for a tile with no row past Nk (every tile but the ragged last one): the
  // per-lane source offsets do not depend on t0 and are computed once here, so a full tile's
  // pieces cost no VALU (the clamp above was ~16 VALU per 64-key step, ~7 % of the loop's VALU)
  uint32_t voff_full[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = wave * PPW + i;
    const bool isv = q >= PIECES / 2;
    const int qq = isv ? q - PIECES / 2 : q;
    const int r = (qq % (LT / 8)) * 8 + (lane >> 3), cs = lane & 7;
    const int c = isv ? cs ^ (((r >> 1) & 3) << 1) : cs ^ ((r >> 1) & 7);
    voff_full[i] = (uint32_t)(r * kHeadDim + c * 8) * 2u;
  }
  auto issue_full = [&](int t0, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      const bool isv = q >= PIECES / 2;
      const int qq = isv ? q - PIECES / 2 : q;
      const int pl = qq / (LT / 8);
      const _Float16* base = (isv ? Vp : Kp) + (size_t)pl * ps + (size_t)t0 * kHeadDim;
      const uint32_t dst = (isv ? vs_lds : ks_lds) + (uint32_t)(((buf * 2 + pl) * PL + (qq % (LT / 8)) * 8 * kHeadDim) * 2);
      dma16_u(base, voff_full[i], dst);
    }
  };

  const int kswz = (r16 >> 1) & 7;
  const int vq = (lane & 15) >> 2, vp4 = lane & 3;
  const int vrow = 4 * g + vq;
  const int vswz = ((vrow >> 1) & 3) << 1;
  int kcol[2], vcol[4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kcol[ks] = ((4 * ks + g) ^ kswz) << 3;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) vcol[dt] = ((2 * dt + (vp4 >> 1)) ^ vswz) << 3;

  f32x4 o[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt][0] = o[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // softmax reference per query: exact form in accumulator units (m_use = -inf forces the first
  // raise); common form in log2 units, starting at 0 with the first step always re-referencing
  float m_use[2] = {exact ? -INFINITY : 0.f, exact ? -INFINITY : 0.f};
  float l_run[2] = {0.f, 0.f};
  // exact form: raise test (lmax - m_use) c > 3 as one compare against m_use + 3 / c
  float thr[2] = {-INFINITY, -INFINITY};
  const float inv3c[2] = {3.f / c_lane[0], 3.f / c_lane[1]};
  // common form: C operand of each score tile's first MFMA, 11 - m_use (so the accumulator holds
  // s - m + 11 = log2(p 2^11)); raise when it exceeds LG_ATTN_RAISE, re-referencing the query so
  // that its largest accumulator becomes LG_ATTN_REF
  f32x4 cm[2] = {f32x4{11.f, 11.f, 11.f, 11.f}, f32x4{11.f, 11.f, 11.f, 11.f}};
  bool first = true;  // wave-uniform: the first 64-key step sets every query's reference

  // one 64-key softmax step over LDS rows off .. off+63 of the current buffer (off: element
  // offset buf*2*PL + sub*KT*kHeadDim, a compile-time constant in the main loop)
  // mid(): called between the exponentials and the P split / PV MFMAs -- the LDS-DMA pieces of the
  // next tile are issued there, in the step's VALU-only stretch, where a piece costs a fraction of
  // its issue price among the score MFMAs (MI355X_MICROARCH.md, LDS-DMA piece issue cost)
  // nmode: 0 none, 1 issue_full(nt0, nbuf), 2 issue(nt0, nbuf) -- the next tile's staging
  auto body = [&](auto OFFc, auto MASKc, auto EXc, int t0, int nmode, int nt0, int nbuf) __attribute__((always_inline)) {
    const int off = OFFc;
    constexpr bool MASK = decltype(MASKc)::value;
    constexpr bool EXACT = decltype(EXc)::value;
    // from the __shared__ arrays themselves (not captured pointers), so the reads stay ds_read
    const _Float16* Kc = Ks + r16 * kHeadDim + off;
    const _Float16* Vc = Vs + vrow * kHeadDim + 4 * (vp4 & 1) + off;

    f16x8 kf[NKT][2][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int off = kt * 16 * kHeadDim + kcol[ks];
        kf[kt][ks][0] = *reinterpret_cast<const f16x8*>(Kc + off);
        kf[kt][ks][1] = *reinterpret_cast<const f16x8*>(Kc + PL + off);
      }
    asm volatile("" ::: "memory");
    f32x4 sc[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 a = EXACT ? f32x4{0.f, 0.f, 0.f, 0.f} : cm[qt];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a = mfma_h3_16(kf[kt][ks][0], kf[kt][ks][1], qhs[qt][ks], ql[qt][ks], qh[qt][ks], a);
        sc[kt][qt] = a;
      }
    f16x8 vf[NKT / 2][4][2];
#pragma unroll
    for (int p = 0; p < NKT / 2; ++p)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const f16x4 lo = tr_read_h(Vc + pl * PL + (32 * p) * kHeadDim + vcol[dt]);
          const f16x4 hi = tr_read_h(Vc + pl * PL + (32 * p + 16) * kHeadDim + vcol[dt]);
          vf[p][dt][pl] = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      if constexpr (MASK) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t0 + 16 * kt + 4 * g + r >= Nk) sc[kt][qt][r] = -INFINITY;
      }
      float lmax;
      if constexpr (EXACT) {
        const float m0 = max3f(sc[0][qt][0], sc[0][qt][1], sc[0][qt][2]);
        const float m1 = max3f(sc[0][qt][3], sc[1][qt][0], sc[1][qt][1]);
        const float m2 = max3f(sc[1][qt][2], sc[1][qt][3], sc[2][qt][0]);
        const float m3 = max3f(sc[2][qt][1], sc[2][qt][2], sc[2][qt][3]);
        const float m4 = max3f(sc[3][qt][0], sc[3][qt][1], sc[3][qt][2]);
        lmax = fmaxf(max3f(m0, m1, m2), max3f(m3, m4, sc[3][qt][3]));
      } else {
        const float m0 = max3m(sc[0][qt][0], sc[0][qt][1], sc[0][qt][2]);
        const float m1 = max3m(sc[0][qt][3], sc[1][qt][0], sc[1][qt][1]);
        const float m2 = max3m(sc[1][qt][2], sc[1][qt][3], sc[2][qt][0]);
        const float m3 = max3m(sc[2][qt][1], sc[2][qt][2], sc[2][qt][3]);
        const float m4 = max3m(sc[3][qt][0], sc[3][qt][1], sc[3][qt][2]);
        lmax = max2m(max3m(m0, m1, m2), max3m(m3, m4, sc[3][qt][3]));
      }
      // the lane-local max decides whether any query can need a raise; only then are the four
      // lanes of each query reduced (the raise itself is per query, exactly as in h3/h3m)
      if constexpr (EXACT) {
        if (__ballot(lmax > thr[qt]) != 0ull) {
          const float tmax = max_x16_32(lmax);
          const bool need = (tmax - m_use[qt]) * c_lane[qt] > 3.f;
          const float m_new = need ? tmax : m_use[qt];
          const float alpha = __builtin_amdgcn_exp2f((m_use[qt] - m_new) * c_lane[qt]);
          m_use[qt] = m_new;
          thr[qt] = m_new + inv3c[qt];
          l_run[qt] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[dt][qt][r] *= alpha;
        }
      } else {
        // accumulators hold s - m + 11: re-reference a query whose tile max passes LG_ATTN_RAISE
        // (and every query on the first step) by d = tmax - LG_ATTN_REF, shifting this step's
        // accumulators, C and the running sums (nothing to rescale on the first step)
        if (first || __ballot(lmax > (float)LG_ATTN_RAISE) != 0ull) {
          const float tmax = max_x16_32(lmax);
          const float d = (first || tmax > (float)LG_ATTN_RAISE) && tmax > -INFINITY ? tmax - (float)LG_ATTN_REF : 0.f;
          m_use[qt] += d;
#pragma unroll
          for (int r = 0; r < 4; ++r) cm[qt][r] -= d;
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[kt][qt][r] -= d;
          if (!first) {
            const float alpha = __builtin_amdgcn_exp2f(-d);
            l_run[qt] *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
              for (int r = 0; r < 4; ++r) o[dt][qt][r] *= alpha;
          }
        }
      }
      // e = p 2^11; the partial sums start from the first sub-tile's values (0 + e costs an add)
      float ps4[4];
      if constexpr (!EXACT) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __builtin_amdgcn_exp2f(sc[kt][qt][r]);
            sc[kt][qt][r] = e;
            ps4[r] = kt == 0 ? e : ps4[r] + e;
          }
      } else {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][qt][r] - m_use[qt], c_lane[qt], 11.f));
            sc[kt][qt][r] = e;
            ps4[r] = kt == 0 ? e : ps4[r] + e;
          }
      }
      l_run[qt] += (ps4[0] + ps4[1]) + (ps4[2] + ps4[3]);
    }
    if constexpr (!EXACT) first = false;
    if (nmode == 1) issue_full(__builtin_amdgcn_readfirstlane(nt0), __builtin_amdgcn_readfirstlane(nbuf));
    else if (nmode == 2) issue(__builtin_amdgcn_readfirstlane(nt0), __builtin_amdgcn_readfirstlane(nbuf));
#pragma unroll
    for (int p = 0; p < NKT / 2; ++p)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        // P pieces at scale 2^11: phs = fp16(e), pl = fp16(e - phs); the value planes' low piece is
        // unscaled (split2h_v), so v_h phs + v_h pl + v_l phs = 2^11 (v_h p_h + v_h p_l + v_l p_h)
        f16x8 phs, pl;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float e0 = sc[2 * p + (j >> 2)][qt][j & 3];
          const float e1 = sc[2 * p + (j >> 2)][qt][(j & 3) + 1];
          const f16x2 hs = {(_Float16)e0, (_Float16)e1};
          const f16x2 lo = lo_pair(e0, e1, hs);
          phs[j] = hs[0]; phs[j + 1] = hs[1];
          pl[j] = lo[0]; pl[j + 1] = lo[1];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][qt] = mfma_h3_16(vf[p][dt][0], vf[p][dt][1], phs, pl, phs, o[dt][qt]);
      }
  };

  using NoMask = std::integral_constant<bool, false>;
  using Mask = std::integral_constant<bool, true>;
  const int nlt = (Nk + LT - 1) / LT;
  const int nfull = Nk / LT;  // LDS tiles without a ragged end
  using IC0 = std::integral_constant<int, 0>;
  using IC1 = std::integral_constant<int, KT * kHeadDim>;
  using IC2 = std::integral_constant<int, 2 * PL>;
  using IC3 = std::integral_constant<int, 2 * PL + KT * kHeadDim>;
  static_assert(SUBS == 1 || SUBS == 2, "sub-tiles per LDS tile");
  // static priority for the second-dispatched half (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (PRIO && wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // the tile loop in two copies (normal / exact exponent arguments): the choice is one uniform
  // branch here, none inside the loop, so the common copy keeps its schedule (a macro, not a
  // lambda: a closure around `issue` would leave its uniform operands in VGPRs)
#define LG_ATTN_TILES(EXc)                                                          \
  {                                                                                 \
    int t = 0;                                                                      \
    for (; t + 2 <= nfull; t += 2) {                                                \
      /* buffer 1 released by the barrier; t+1 < nfull */                           \
      body(IC0{}, NoMask{}, EXc, t * LT, 1, (t + 1) * LT, 1);                       \
      if constexpr (SUBS == 2) body(IC1{}, NoMask{}, EXc, t * LT + KT, 0, 0, 0);    \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
      body(IC2{}, NoMask{}, EXc, (t + 1) * LT, t + 2 < nfull ? 1 : (t + 2 < nlt ? 2 : 0), (t + 2) * LT, 0); \
      if constexpr (SUBS == 2) body(IC3{}, NoMask{}, EXc, (t + 1) * LT + KT, 0, 0, 0); \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
    }                                                                               \
    for (; t < nlt; ++t) { /* at most two LDS tiles: masked steps, runtime buffer */ \
      const int buf = t & 1;                                                        \
      if (t + 1 < nlt) issue((t + 1) * LT, buf ^ 1);                                \
      for (int sub = 0; sub < SUBS; ++sub) {                                        \
        const int s0 = t * LT + sub * KT;                                           \
        if (s0 < Nk) body(buf * 2 * PL + sub * KT * kHeadDim, Mask{}, EXc, s0, 0, 0, 0); \
      }                                                                             \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
    }                                                                               \
  }
  if (exact) LG_ATTN_TILES((std::integral_constant<bool, true>{}))
  else LG_ATTN_TILES((std::integral_constant<bool, false>{}))
#undef LG_ATTN_TILES

  if constexpr (SPLIT) {
    // partial record of (split, set, b, h, query): O [64] (lane: dims 16 dt + 4 g ..), then
    // (m, l, c) -- the combine weighs the split by exp2((m - max m) c), as the in-loop rescale does
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float l_tot = sum_x16_32(l_run[qt]);
      const int q = q_blk + wave * 32 + qt * 16 + r16;
      if (q < Nq) {
        const size_t rec = (((size_t)split * 2 + set) * B * H + bh) * nqs + q;
        float* po = part + rec * kHeadDim;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(po + 16 * dt + 4 * g) = o[dt][qt];
        if (g == 0)
          *reinterpret_cast<f32x4*>(part + (size_t)nsplit * 2 * B * H * nqs * kHeadDim + rec * 4) =
              f32x4{m_use[qt], l_tot, c_lane[qt], 0.f};
      }
    }
    return;
  }
  // context rows into the plane image: o = 2^11 sum(v p) (the MFMA scale), l_run = 2^11 sum(p),
  // so 1 / l_run is the old 2^-11 / l exactly; v arrived as v * 2^-E[v] and the context leaves
  // as ctx * 2^-E[v] (its consumer reads the value slot)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l_tot = sum_x16_32(l_run[qt]);
    const float inv = 1.f / l_tot;
    const int q = q_blk + wave * 32 + qt * 16 + r16;
    if (q < Nq) {
      const int orow = S.o_row0 + b * NqS + q;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        f16x4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 a, c;
          split2h(o[dt][qt][e] * inv, a, c);
          h[e] = a;
          l[e] = c;
        }
        const size_t off = plane_off(orow, head * kHeadDim + 16 * dt + 4 * g, S.o_rows_pad);
#if LG_ATTN_CTX_NT
        __builtin_nontemporal_store(h, reinterpret_cast<f16x4*>(S.op + off));
        __builtin_nontemporal_store(l, reinterpret_cast<f16x4*>(S.op + S.ops + off));
#else
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
#endif
      }
    }
  }
}

// merges the NS partials of every (set, b, h, query) into the context plane image: one thread per
// 8 dims of a query, every load issued before the first use, the splits summed in order
template <int NS>
__global__ __launch_bounds__(256) void attn_split_combine_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqs, const float* part) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = (int)(t & 7);
  size_t r = t >> 3;
  const int q = (int)(r % nqs);
  r /= nqs;
  const int bh = (int)(r % ((size_t)B * H));
  const int set = (int)(r / ((size_t)B * H));
  if (set >= 2) return;
  const AttnSet& S = set == 0 ? s0 : s1;
  const int head = bh % H, b = bh / H;
  if (q >= (S.nq_cnt ? S.nq_cnt[b] : S.Nq) || (S.act && !S.act[b])) return;  // rows the kernel skipped
  const size_t nrec = (size_t)2 * B * H * nqs;
  const size_t rec0 = ((size_t)set * B * H + bh) * nqs + q;
  const float* ml = part + (size_t)NS * nrec * kHeadDim;
  f32x4 v[NS], a[NS], c[NS];
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) {
    const size_t rec = (size_t)sp * nrec + rec0;
    v[sp] = *reinterpret_cast<const f32x4*>(ml + rec * 4);
    a[sp] = *reinterpret_cast<const f32x4*>(part + rec * kHeadDim + 8 * chunk);
    c[sp] = *reinterpret_cast<const f32x4*>(part + rec * kHeadDim + 8 * chunk + 4);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int sp = 0; sp < NS; ++sp)
    if (v[sp][1] > 0.f) mx = fmaxf(mx, v[sp][0]);
  float l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) {
    if (!(v[sp][1] > 0.f)) continue;  // an empty key range
    const float w = __builtin_amdgcn_exp2f((v[sp][0] - mx) * v[sp][2]);
    l = fmaf(v[sp][1], w, l);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = fmaf(a[sp][e], w, o[e]);
      o[4 + e] = fmaf(c[sp][e], w, o[4 + e]);
    }
  }
  const float inv = 1.f / l;
  const int orow = S.o_row0 + b * S.Nq + q;
  f16x8 h, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    _Float16 x, y;
    split2h(o[e] * inv, x, y);
    h[e] = x;
    lo[e] = y;
  }
  const size_t off = plane_off(orow, head * kHeadDim + 8 * chunk, S.o_rows_pad);
  *reinterpret_cast<f16x8*>(S.op + off) = h;
  *reinterpret_cast<f16x8*>(S.op + S.ops + off) = lo;
}

template <int SUBS, int PRIO = 0, int WAVES = 8>
static hipError_t attention_h3g_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st,
                                       bool qp, float* part = nullptr, int nsplit = 1) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  if (nsplit > 1 && part) {
    constexpr int LT = 64 * SUBS;  // keys per LDS tile
    const int nk = s0.Nk > s1.Nk ? s0.Nk : s1.Nk;
    const int lsplit = ((nk + nsplit - 1) / nsplit + LT - 1) / LT * LT;
    if (qp)
      hipLaunchKernelGGL((attention_h3g_kernel<SUBS, PRIO, WAVES, true, true>), dim3(items * nsplit), dim3(64 * WAVES), 0, st,
                         s0, s1, B, H, nqb, scale * 1.4426950408889634f, part, nsplit, lsplit);
    else
      hipLaunchKernelGGL((attention_h3g_kernel<SUBS, PRIO, WAVES, true>), dim3(items * nsplit), dim3(64 * WAVES), 0, st, s0,
                         s1, B, H, nqb, scale * 1.4426950408889634f, part, nsplit, lsplit);
    const size_t threads = (size_t)2 * B * H * nq * 8;
    const dim3 cg((unsigned)((threads + 255) / 256)), cb(256);
    switch (nsplit) {
      case 2: hipLaunchKernelGGL(attn_split_combine_kernel<2>, cg, cb, 0, st, s0, s1, B, H, nq, (const float*)part); break;
      case 4: hipLaunchKernelGGL(attn_split_combine_kernel<4>, cg, cb, 0, st, s0, s1, B, H, nq, (const float*)part); break;
      default: hipLaunchKernelGGL(attn_split_combine_kernel<8>, cg, cb, 0, st, s0, s1, B, H, nq, (const float*)part); break;
    }
    return hipGetLastError();
  }
  if (qp)
    hipLaunchKernelGGL((attention_h3g_kernel<SUBS, PRIO, WAVES, false, true>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B,
                       H, nqb, scale * 1.4426950408889634f);
  else
    hipLaunchKernelGGL((attention_h3g_kernel<SUBS, PRIO, WAVES>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                       scale * 1.4426950408889634f);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// attention_h3m_kernel: attention_h3g_kernel's pipeline (LDS-DMA K/V staging, pre-scaled P with
// fma_mix low pieces, ballot-gated lazy reference, exact-exponent loop copy) on
// v_mfma_f32_32x32x16_f16.  Why: the 16x16x32 MFMA holds the SIMD's VALU issue for 8 of its 16
// cycles, the 32x32x16 one for 8 of its 32 (MI355X_MICROARCH.md, per-instruction constants).  The
// h3g body issues ~180 VALU per 96 MFMAs per wave, so two waves on a SIMD need ~2 x (96 x 8 + ~820)
// issue cycles against 2 x 96 x 16 MFMA cycles -- issue-bound with no room for the partner's
// softmax; with 48 32x32 MFMAs the same work needs 2 x (48 x 8 + ~820) issue cycles against
// 2 x 1536 MFMA cycles.  Layouts (the register-level mapping of tools/attn_h3_legacy.hip):
//   S^T[key][query] = K Q^T: A = K (lane: key l&31 of a 32-key sub-tile, dims 16ks + 8(l>>5)..),
//     B = Q^T (lane: query l&31, the same dims), four k-steps per head;
//     accumulator register r of lane l: query l&31, key row32(r, l>>5).
//   O^T[dim][query] += V^T P^T over 16-key steps: B = P^T = S^T registers 8s..8s+7 (keys
//     ka + j / ka + 8 + j - 4, ka = 16s + 4(l>>5)); A = V^T from two ds_read_b64_tr_b16 per
//     plane and 32-dim tile (rows ka + (l&15)>>2, +8).
//   Per-query reductions: in-lane over 32 scores, then lane ^ 32 (v_permlane32_swap).
// LDS: K as in h3g (16-byte chunk c of row r at c ^ ((r >> 1) & 7): the 32x32 fragment reads hit
// 16 distinct slots per lane group too); V rows with the two 32-dim halves swapped where key bit 1
// is set (each transposed read's 4 rows then cover all 64 banks).
template <int SUBS, int PRIO, int WAVES = 8, bool QP = false>
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 ? 2 : 1) void attention_h3m_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                float scale_log2e) {
  constexpr int QB = 32 * WAVES;
  constexpr int KT = 64;                   // keys per softmax step
  constexpr int LT = KT * SUBS;            // keys per LDS tile (one barrier)
  constexpr int PL = LT * kHeadDim;        // one plane of an LDS tile (elements)
  constexpr int PIECES = 4 * LT / 8;       // 1 KiB LDS-DMA pieces per tile (K h/l, V h/l; 8 rows each)
  constexpr int PPW = PIECES / WAVES;
  static_assert(PIECES % WAVES == 0, "pieces per wave");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * PL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 2 * PL];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  // S.Nq / S.Nk are the layout capacities; per-pair counts (batched pruning) bound the loops
  const int NqS = S.Nq, NkS = S.Nk, pb = bh / H;
  if (S.act && !S.act[pb]) return;
  const int Nq = S.nq_cnt ? S.nq_cnt[pb] : NqS, Nk = S.nk_cnt ? S.nk_cnt[pb] : NkS;
  if (q_blk >= Nq || Nk <= 0) return;
  const void* Q = QP ? static_cast<const void*>(static_cast<const _Float16*>(S.q) + (size_t)bh * NqS * kHeadDim)
                    : static_cast<const void*>(static_cast<const float*>(S.q) + (size_t)bh * NqS * kHeadDim);
  const float qsc = QP ? ldexpf(1.f, range_slot_exp(S.rtab, S.k_slot)) : 1.f;  // QP: queries from planes
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * NkS * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * NkS * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, half = lane >> 5;

  // queries: lane = query l32 of the wave's 32, dims 16ks + 8 half + j, scaled per row by 2^ex
  // so that the row max lies in [8, 16) (the per-lane factor folds into the exp argument)
  const int ek = range_slot_exp(S.rtab, S.k_slot);  // key planes hold k * 2^-ek (RangeOut)
  const float kmax = S.rtab ? range_max(S.rtab, S.k_slot) : INFINITY;
  f16x8 qh[4], qhs[4], ql[4];
  float c_lane;
  bool big;
  {
    const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
    const size_t qr = (size_t)qrow * kHeadDim + 8 * half;
    f32x4 x[4][2];
    float mx = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      load_q8<QP>(Q, S.pstride, qr + 16 * ks, qsc, x[ks][0], x[ks][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[ks][0][e]), fabsf(x[ks][1][e])));
    }
    mx = max_xor32(mx);
    big = !(64.f * mx * kmax * scale_log2e <= 2097152.f);  // see attention_h3g_kernel
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane = ldexpf(scale_log2e, ek - (11 + ex));
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[ks][e >> 2][e & 3], ex), h, l);
        qh[ks][e] = h;
        ql[ks][e] = l;
        qhs[ks][e] = h * (_Float16)kLoScale;
      }
  }
  const bool exact = __builtin_amdgcn_readfirstlane((int)(__ballot(big) != 0ull)) != 0;  // wave-uniform

  // LDS-DMA staging of one LDS tile (keys t0 .. t0+LT-1) into buffer buf, as in h3g, with the V
  // half-swap swizzle (chunk cs of row r at cs ^ 4 ((r >> 1) & 1))
  const uint32_t ks_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)Ks);
  const uint32_t vs_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)Vs);
  auto issue = [&](int t0, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      const bool isv = q >= PIECES / 2;
      const int qq = isv ? q - PIECES / 2 : q;
      const int pl = qq / (LT / 8), r = (qq % (LT / 8)) * 8 + (lane >> 3), cs = lane & 7;
      const int c = isv ? cs ^ (((r >> 1) & 1) << 2) : cs ^ ((r >> 1) & 7);
      const _Float16* base = (isv ? Vp : Kp) + (size_t)pl * ps + (size_t)t0 * kHeadDim;
      const uint32_t voff = (uint32_t)((min(t0 + r, Nk - 1) - t0) * kHeadDim + c * 8) * 2u;
      const uint32_t dst = (isv ? vs_lds : ks_lds) + (uint32_t)(((buf * 2 + pl) * PL + (qq % (LT / 8)) * 8 * kHeadDim) * 2);
      dma16(base, voff, dst);
    }
  };
  // full tiles: t0-independent per-lane source offsets, computed once (as attention_h3g_kernel)
  uint32_t voff_full[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = wave * PPW + i;
    const bool isv = q >= PIECES / 2;
    const int qq = isv ? q - PIECES / 2 : q;
    const int r = (qq % (LT / 8)) * 8 + (lane >> 3), cs = lane & 7;
    const int c = isv ? cs ^ (((r >> 1) & 1) << 2) : cs ^ ((r >> 1) & 7);
    voff_full[i] = (uint32_t)(r * kHeadDim + c * 8) * 2u;
  }
  auto issue_full = [&](int t0, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      const bool isv = q >= PIECES / 2;
      const int qq = isv ? q - PIECES / 2 : q;
      const int pl = qq / (LT / 8);
      const _Float16* base = (isv ? Vp : Kp) + (size_t)pl * ps + (size_t)t0 * kHeadDim;
      const uint32_t dst = (isv ? vs_lds : ks_lds) + (uint32_t)(((buf * 2 + pl) * PL + (qq % (LT / 8)) * 8 * kHeadDim) * 2);
      dma16(base, voff_full[i], dst);
    }
  };

  // per-lane LDS offsets: K fragment row l32, chunk 2ks + half (swizzled); transposed V reads:
  // 16-lane group covers dims 16 ((lane >> 4) & 1) + 4 (lane & 3) of lane half `half`, rows
  // ka + ((lane & 15) >> 2) (+8)
  int kcol[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) kcol[ks] = l32 * kHeadDim + (((2 * ks + half) ^ ((l32 >> 1) & 7)) << 3);
  const int tq = (lane & 15) >> 2, tdim = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  const int vsw = ((tq >> 1) & 1) << 5;
  const int voff0 = (4 * half + tq) * kHeadDim + (tdim ^ vsw);
  const int voff1 = (4 * half + tq) * kHeadDim + ((32 + tdim) ^ vsw);

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};  // O^T (x 2^11): dims [0,32) and [32,64)
  float m_use = -INFINITY;
  float l_run = 0.f;
  float thr = -INFINITY;  // raise test (lmax - m_use) c > 3 as one compare, kept with m_use
  const float inv3c = 3.f / c_lane;

  auto body = [&](auto OFFc, auto MASKc, auto EXc, int t0) __attribute__((always_inline)) {
    const int off = OFFc;
    constexpr bool MASK = decltype(MASKc)::value;
    constexpr bool EXACT = decltype(EXc)::value;
    f16x8 kf[2][4][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int o = off + u * 32 * kHeadDim + kcol[ks];
        kf[u][ks][0] = *reinterpret_cast<const f16x8*>(Ks + o);
        kf[u][ks][1] = *reinterpret_cast<const f16x8*>(Ks + PL + o);
      }
    asm volatile("" ::: "memory");
    f32x16 sc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sc[u] = f32x16{0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sc[u] = mfma_h3(kf[u][ks][0], kf[u][ks][1], qhs[ks], ql[ks], qh[ks], sc[u]);
    }
    f16x8 vf[2][2][2][2];  // [u][s][dim tile][plane]
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int vr = off + (u * 32 + 16 * ss) * kHeadDim;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4 a0 = tr_read_h(Vs + p * PL + vr + voff0);
          const f16x4 a1 = tr_read_h(Vs + p * PL + vr + 8 * kHeadDim + voff0);
          const f16x4 b0 = tr_read_h(Vs + p * PL + vr + voff1);
          const f16x4 b1 = tr_read_h(Vs + p * PL + vr + 8 * kHeadDim + voff1);
          vf[u][ss][0][p] = f16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          vf[u][ss][1][p] = f16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        }
      }
    asm volatile("" ::: "memory");
    if constexpr (MASK) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
    }
    float mt[11];
#pragma unroll
    for (int i = 0; i < 10; ++i) mt[i] = max3f(sc[(3 * i) >> 4][(3 * i) & 15], sc[(3 * i + 1) >> 4][(3 * i + 1) & 15],
                                               sc[(3 * i + 2) >> 4][(3 * i + 2) & 15]);
    mt[10] = fmaxf(sc[1][14], sc[1][15]);
    const float lmax = fmaxf(max3f(max3f(mt[0], mt[1], mt[2]), max3f(mt[3], mt[4], mt[5]), max3f(mt[6], mt[7], mt[8])),
                             fmaxf(mt[9], mt[10]));
    if (__ballot(lmax > thr) != 0ull) {
      const float tmax = max_xor32(lmax);
      const bool need = (tmax - m_use) * c_lane > 3.f;
      const float m_new = need ? tmax : m_use;
      const float alpha = __builtin_amdgcn_exp2f((m_use - m_new) * c_lane);
      m_use = m_new;
      thr = m_new + inv3c;
      l_run *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
    }
    // e = p 2^11
    float ps8[8];
    if constexpr (!EXACT) {
      const float mb = fmaf(m_use, c_lane, -11.f);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[u][r], c_lane, -mb));
          sc[u][r] = e;
          ps8[r & 7] = u == 0 && r < 8 ? e : ps8[r & 7] + e;
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[u][r] - m_use, c_lane, 11.f));
          sc[u][r] = e;
          ps8[r & 7] = u == 0 && r < 8 ? e : ps8[r & 7] + e;
        }
    }
    l_run += ((ps8[0] + ps8[1]) + (ps8[2] + ps8[3])) + ((ps8[4] + ps8[5]) + (ps8[6] + ps8[7]));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        f16x8 phs, pl;  // as in attention_h3g_kernel: unscaled value low piece, no p_h copy
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float e0 = sc[u][8 * ss + j], e1 = sc[u][8 * ss + j + 1];
          const f16x2 hs = {(_Float16)e0, (_Float16)e1};
          const f16x2 lo = lo_pair(e0, e1, hs);
          phs[j] = hs[0]; phs[j + 1] = hs[1];
          pl[j] = lo[0]; pl[j + 1] = lo[1];
        }
        o0 = mfma_h3(vf[u][ss][0][0], vf[u][ss][0][1], phs, pl, phs, o0);
        o1 = mfma_h3(vf[u][ss][1][0], vf[u][ss][1][1], phs, pl, phs, o1);
      }
  };

  using NoMask = std::integral_constant<bool, false>;
  using Mask = std::integral_constant<bool, true>;
  const int nlt = (Nk + LT - 1) / LT;
  const int nfull = Nk / LT;
  using IC0 = std::integral_constant<int, 0>;
  using IC1 = std::integral_constant<int, KT * kHeadDim>;
  using IC2 = std::integral_constant<int, 2 * PL>;
  using IC3 = std::integral_constant<int, 2 * PL + KT * kHeadDim>;
  static_assert(SUBS == 1 || SUBS == 2, "sub-tiles per LDS tile");
  if (PRIO && wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#define LG_ATTN_TILES(EXc)                                                          \
  {                                                                                 \
    int t = 0;                                                                      \
    for (; t + 2 <= nfull; t += 2) {                                                \
      issue_full((t + 1) * LT, 1); /* t + 1 < nfull */                              \
      body(IC0{}, NoMask{}, EXc, t * LT);                                           \
      if constexpr (SUBS == 2) body(IC1{}, NoMask{}, EXc, t * LT + KT);             \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
      if (t + 2 < nfull) issue_full((t + 2) * LT, 0);                               \
      else if (t + 2 < nlt) issue((t + 2) * LT, 0);                                 \
      body(IC2{}, NoMask{}, EXc, (t + 1) * LT);                                     \
      if constexpr (SUBS == 2) body(IC3{}, NoMask{}, EXc, (t + 1) * LT + KT);       \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
    }                                                                               \
    for (; t < nlt; ++t) {                                                          \
      const int buf = t & 1;                                                        \
      if (t + 1 < nlt) issue((t + 1) * LT, buf ^ 1);                                \
      for (int sub = 0; sub < SUBS; ++sub) {                                        \
        const int s0_ = t * LT + sub * KT;                                          \
        if (s0_ < Nk) body(buf * 2 * PL + sub * KT * kHeadDim, Mask{}, EXc, s0_);   \
      }                                                                             \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
      __syncthreads();                                                              \
    }                                                                               \
  }
  if (exact) LG_ATTN_TILES((std::integral_constant<bool, true>{}))
  else LG_ATTN_TILES((std::integral_constant<bool, false>{}))
#undef LG_ATTN_TILES

  // context row into the plane image: register r = 4g + e holds dim 8g + 4 half + e (+32 for o1);
  // o = 2^11 sum(p v), l_run = 2^11 sum(p) -> ctx * 2^-E[v] (RangeOut, as h3g)
  const float l_tot = sum_xor32(l_run);
  const float inv = 1.f / l_tot;
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    const int orow = S.o_row0 + b * NqS + q;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f16x4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 a, c;
          split2h((hf ? o1 : o0)[4 * g + e] * inv, a, c);
          h[e] = a;
          l[e] = c;
        }
        const size_t off = plane_off(orow, head * kHeadDim + hf * 32 + 8 * g + 4 * half, S.o_rows_pad);
#if LG_ATTN_CTX_NT
        __builtin_nontemporal_store(h, reinterpret_cast<f16x4*>(S.op + off));
        __builtin_nontemporal_store(l, reinterpret_cast<f16x4*>(S.op + S.ops + off));
#else
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
#endif
      }
  }
}

template <int SUBS, int PRIO = 0, int WAVES = 8>
static hipError_t attention_h3m_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st,
                                       bool qp) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  if (qp)
    hipLaunchKernelGGL((attention_h3m_kernel<SUBS, PRIO, WAVES, true>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                       scale * 1.4426950408889634f);
  else
    hipLaunchKernelGGL((attention_h3m_kernel<SUBS, PRIO, WAVES>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                       scale * 1.4426950408889634f);
  return hipGetLastError();
}

// fp16x3 kernel choice: LG_ATTN_KERNEL=h3g (16x16x32 MFMAs, default) | h3m (32x32x16 MFMAs).
// Measured equal at the bench shape (profiles/r02/pmc_ab: h3m takes 6 % fewer cycles per launch
// but the chip holds a 7 % lower clock under it -- 1.84 vs 1.97 GHz, MFMA busy 0.54 vs 0.51), so
// the saving returns as clock (MI355X_MICROARCH.md, DVFS give-back); h3g stays the default.
static bool attention_use_h3m() {
  const char* e = getenv("LG_ATTN_KERNEL");
  return e && !strcmp(e, "h3m");
}

// Query block size: 8 waves (256 queries) per workgroup is the throughput shape; when that gives
// fewer work items than CUs (B = 1, pruned sets) 4 waves per workgroup spread the queries over
// twice the CUs (each workgroup still streams all keys).  LG_ATTN_WAVES=8|4|2 forces one.
static int attention_waves(int B, int H, int nq) {
  if (const char* e = getenv("LG_ATTN_WAVES")) {
    const int w = atoi(e);
    if (w == 8 || w == 4 || w == 2) return w;
  }
  // 4 waves measured best below one item per CU (B = 1, N = 1024: 32.9 us vs 42.7 (8) / 38.1 (2));
  // 2 is kept for LG_ATTN_WAVES only
  return (long long)((nq + 255) / 256) * B * H * 2 >= 256 ? 8 : 4;
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

#ifndef LG_ATTN_CONFIG
// WAVES, KT: 8 waves (256 queries) per workgroup, 64-key tiles (tools/kbench_attn.hip).
#define LG_ATTN_CONFIG 8, 64
#endif

// Key splits for small batches (4-wave h3g items only): while the work items leave most CUs idle,
// double the splits (at least 256 keys each, at most 512 workgroups).  B = 1, N = 1024 (64 items):
// 4 splits 1.48 ms per forward vs 1.55 (2), 1.67 (8, one LDS tile each) and 1.68 (unsplit).
// LG_ATTN_SPLIT=1|2|4|8 overrides.
int attention_nsplit(int B, int H, int nq, int nk) {
  if (attention_use_h3m() || attention_waves(B, H, nq) != 4) return 1;
  const long long items = (long long)((nq + 127) / 128) * B * H * 2;
  int ns = 1;
  if (const char* e = getenv("LG_ATTN_SPLIT")) {
    ns = atoi(e);
    return ns == 2 || ns == 4 || ns == 8 ? ns : 1;
  }
  while (ns < 8 && items * ns * 2 <= 512 && nk / (ns * 2) >= 256) ns *= 2;
  return ns;
}
size_t attention_split_floats(int B, int H, int nq, int nk) {
  const int ns = attention_nsplit(B, H, nq, nk);
  return ns > 1 ? (size_t)ns * 2 * B * H * nq * (kHeadDim + 4) : 0;
}

hipError_t attention_f32(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, int prec, hipStream_t st,
                         float* part, size_t part_floats, bool q_planes) {
  if (prec == PREC_H3) {
    if (!s0.op || !s1.op || !s0.q || !s1.q) return hipErrorInvalidValue;
    const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
    if (attention_use_h3m()) {
      switch (attention_waves(B, H, nq)) {
        case 2: return attention_h3m_launch<2, 1, 2>(s0, s1, B, H, scale, st, q_planes);
        case 4: return attention_h3m_launch<2, 1, 4>(s0, s1, B, H, scale, st, q_planes);
        default: return attention_h3m_launch<2, 1, 8>(s0, s1, B, H, scale, st, q_planes);
      }
    }
    switch (attention_waves(B, H, nq)) {
      case 2: return attention_h3g_launch<2, 1, 2>(s0, s1, B, H, scale, st, q_planes);
      case 4: {
        const int nk = s0.Nk > s1.Nk ? s0.Nk : s1.Nk;
        const int ns = attention_nsplit(B, H, nq, nk);
        const bool fits = part && part_floats >= attention_split_floats(B, H, nq, nk);
        return attention_h3g_launch<2, 1, 4>(s0, s1, B, H, scale, st, q_planes, fits ? part : nullptr, fits ? ns : 1);
      }
      default: return attention_h3g_launch<2, 1, 8>(s0, s1, B, H, scale, st, q_planes);
    }
  }
  if (q_planes || !s0.q || !s1.q) return hipErrorInvalidValue;  // bf16x6 reads fp32 queries
  return attention_x6_launch<LG_ATTN_CONFIG>(s0, s1, B, H, scale, st);
}

}  // namespace lg
