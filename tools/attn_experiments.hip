// Attention schedules that were measured and NOT adopted (tools only; built by
// tools/kbench_attn.hip, never by the library).  Both compute exactly what attention_h3_kernel
// computes (same operands and numerics) and pass the same fp64 check; on MI355X at the bench
// shape (B=32, H=4, N=2048, two sets) they ran at 1040-1070 us vs 960-1000 us for
// attention_h3_kernel (DESIGN.md §5 "attention schedules tried"):
//   attention_h3p_kernel  -- software-pipelined: S(t+1) MFMAs interleaved with the exp/sum of
//                            S(t) in one basic block (sched_group_barrier)
//   attention_h3pp_kernel -- ping-pong: wave groups 0-3 / 4-7 one phase apart, MFMA phase of one
//                            wave beside the softmax phase of its SIMD partner, LDS-DMA staging
//                            with three K slots.  Co-execution itself works (tools/probe_coexec:
//                            MFMA || VALU of the partner overlap almost fully), but the MFMA phase
//                            roughly doubles once its LDS fragment reads run beside the partner's
//                            softmax, so the phases do not shorten.
#pragma once
#include <type_traits>

#include "../cs566-project-lightglue_amd/csrc/attention.hip"
#include "attn_h3_legacy.hip"

namespace lg {

// ----------------------------------------------------------------------------------------
// fp16x3 attention, software-pipelined (PREC_H3): same operands and numerics as
// attention_h3_kernel, but each wave overlaps the score MFMAs of tile t+1 with the exp/sum of
// tile t (independent work in one basic block, interleaved by sched_group_barrier), instead of
// alternating MFMA-only and VALU-only phases in lock-step with its SIMD partner.  K and V sit in
// separate two-slot LDS rings, K one tile ahead of V.
// ----------------------------------------------------------------------------------------
template <int WAVES, int KT, int OCC>
__global__ __launch_bounds__(64 * WAVES, OCC) void attention_h3p_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                         float scale_log2e) {
  constexpr int NT = 64 * WAVES;
  constexpr int QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  constexpr int KLD = kHeadDim + 8;
  constexpr int CH = 2 * KT * 8;
  constexpr int LDC = CH / NT;
  constexpr int KPL = KT * KLD, VPL = KT * kHeadDim;
  static_assert(CH % NT == 0, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * KPL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 2 * VPL];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * Nk * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * Nk * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5;

  const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
  f16x8 qh[4], qhs[4], ql[4];
  float c_lane;
  {
    const float* qr = Q + (size_t)qrow * kHeadDim + half * 8;
    f32x4 x[4][2];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s][0] = *reinterpret_cast<const f32x4*>(qr + 16 * s);
      x[s][1] = *reinterpret_cast<const f32x4*>(qr + 16 * s + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[s][0][e]), fabsf(x[s][1][e])));
    }
    mx = max_xor32(mx);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane = ldexpf(scale_log2e, -(11 + ex));
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[s][e >> 2][e & 3], ex), h, l);
        qh[s][e] = h;
        ql[s][e] = l;
        qhs[s][e] = h * (_Float16)kLoScale;
      }
  }

  f32x4 rk[LDC], rv[LDC];
  auto gload_k = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      rk[i] = *reinterpret_cast<const f32x4*>(Kp + (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8);
    }
  };
  auto gload_v = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      rv[i] = *reinterpret_cast<const f32x4*>(Vp + (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8);
    }
  };
  auto sstore_k = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<f32x4*>(&Ks[(buf * 2 + p) * KPL + r * KLD + cb * 8]) = rk[i];
    }
  };
  auto sstore_v = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<f32x4*>(&Vs[(buf * 2 + p) * VPL + r * kHeadDim + ((cb ^ (((r >> 1) & 1) << 2)) * 8)]) = rv[i];
    }
  };

  const int tq = (lane & 15) >> 2, tp = lane & 3, tdim = ((lane >> 4) & 1) * 16 + 4 * tp;
  const int sw = ((tq >> 1) & 1) << 5;
  const int koff = l32 * KLD + 8 * half;
  const int voff0 = (4 * half + tq) * kHeadDim + (tdim ^ sw);
  const int voff1 = (4 * half + tq) * kHeadDim + ((32 + tdim) ^ sw);

  // S^T of the K tile in ring slot buf (x 2^(11+e)); K fragments read up front
  auto scores = [&](int buf, f32x16 (&out)[NSUB]) {
    const _Float16* Kc = Ks + buf * 2 * KPL + koff;
    f16x8 kf[NSUB][4][2];
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[u][s][0] = *reinterpret_cast<const f16x8*>(Kc + u * 32 * KLD + 16 * s);
        kf[u][s][1] = *reinterpret_cast<const f16x8*>(Kc + KPL + u * 32 * KLD + 16 * s);
      }
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      out[u] = f32x16{0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) out[u] = mfma_h3(kf[u][s][0], kf[u][s][1], qhs[s], ql[s], qh[s], out[u]);
    }
  };

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};
  float m_use = -INFINITY;
  float l_run = 0.f;

  const int ntiles = (Nk + KT - 1) / KT;
  gload_k(0);
  gload_v(0);
  sstore_k(0);
  sstore_v(0);
  __syncthreads();
  if (ntiles > 1) gload_k(KT);
  f32x16 sc[NSUB];
  scores(0, sc);
  if (ntiles > 1) sstore_k(1);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    if (t + 2 < ntiles) gload_k(t0 + 2 * KT);  // -> K slot t&1 (K(t) was consumed in iteration t-1)
    if (t + 1 < ntiles) gload_v(t0 + KT);      // -> V slot (t+1)&1

    // ---- mask, tile max, lazy reference raise on S(t)
    if (t0 + KT > Nk) {
#pragma unroll
      for (int u = 0; u < NSUB; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
    }
    float mr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float m = sc[0][r];
#pragma unroll
      for (int u = 1; u < NSUB; ++u) m = fmaxf(m, sc[u][r]);
      mr[r] = m;
    }
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int r = 0; r < w; ++r) mr[r] = fmaxf(mr[r], mr[r + w]);
    const float tmax = max_xor32(mr[0]);
    const bool need = (tmax - m_use) * c_lane > 3.f;
    if (__ballot(need) != 0ull) {
      const float m_new = need ? tmax : m_use;
      const float alpha = __builtin_amdgcn_exp2f((m_use - m_new) * c_lane);
      m_use = m_new;
      l_run *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    const float mb = m_use * c_lane;

    // ---- [S(t+1) MFMAs] || [exp / sum of S(t)] -- one basic block, interleaved
    f32x16 sn[NSUB];
    scores((t + 1) & 1, sn);  // last iteration: a stale slot, result unused
    float ps8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ps8[i] = 0.f;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[u][r], c_lane, -mb));
        sc[u][r] = p;
        ps8[(u * 16 + r) & 7] += p;
      }
    __builtin_amdgcn_sched_group_barrier(0x100, 8 * NSUB, 0);  // K fragment reads first
#pragma unroll
    for (int i = 0; i < 12 * NSUB; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then four VALU
    }
    l_run += ((ps8[0] + ps8[1]) + (ps8[2] + ps8[3])) + ((ps8[4] + ps8[5]) + (ps8[6] + ps8[7]));

    // ---- O^T += V(t)^T P(t)^T (x 2^11)
    const _Float16* Vc = Vs + (t & 1) * 2 * VPL;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int vr = (u * 32 + 16 * s) * kHeadDim;
        f16x8 v[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4 a0 = tr_read_h(Vc + p * VPL + vr + voff0);
          const f16x4 a1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff0);
          const f16x4 b0 = tr_read_h(Vc + p * VPL + vr + voff1);
          const f16x4 b1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff1);
          v[0][p] = f16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          v[1][p] = f16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        }
        f16x8 ph, phs, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = sc[u][8 * s + j];
          const _Float16 h = (_Float16)p;
          const _Float16 hs = h * (_Float16)kLoScale;
          ph[j] = h;
          phs[j] = hs;
          pl[j] = (_Float16)fmaf(p, kLoScale, -(float)hs);
        }
        o0 = mfma_h3(v[0][0], v[0][1], phs, pl, ph, o0);
        o1 = mfma_h3(v[1][0], v[1][1], phs, pl, ph, o1);
      }

    if (t + 2 < ntiles) sstore_k(t & 1);
    if (t + 1 < ntiles) sstore_v((t + 1) & 1);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NSUB; ++u) sc[u] = sn[u];
  }

  const float l_tot = sum_xor32(l_run);
  const float inv = ldexpf(1.f / l_tot, -11);
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    const int orow = S.o_row0 + b * Nq + q;
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
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
      }
  }
}

template <int WAVES, int KT, int OCC>
static hipError_t attention_h3p_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3p_kernel<WAVES, KT, OCC>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// fp16x3 attention, ping-pong (PREC_H3): same operands and numerics as attention_h3_kernel.
// One 8-wave workgroup per CU, so waves w and w+4 share a SIMD.  The per-tile work of a wave is
// split into an MFMA phase M(j) = [O += P(j-1) V(j-1); S(j) = K(j) Q^T] and a VALU phase
// V(j) = [mask / max / lazy rescale / exp / sum / fp16 split of S(j) -> P(j)], and the two wave
// groups (waves 0-3, 4-7) run the same sequence M(0) V(0) M(1) ... one phase apart between
// workgroup barriers: while one wave of a SIMD issues MFMAs, its partner issues the softmax VALU
// work, so the SIMD's matrix core and vector ALU run concurrently instead of in turn.  For that
// the M phase is kept (nearly) free of VALU work -- the partner's VALU stream has priority and
// would starve it: the fp16 pieces of P (h, h 2^11, l) and of q are formed outside it, and the
// LDS-DMA addresses are per-lane constants plus a wave-uniform base.
// Staging: K(j) in K slot j%3, V(j) in V slot j&1, copied HBM -> LDS by LDS-DMA (no registers),
// both issued from VALU phases (an LDS-DMA issue inside an MFMA phase costs the MFMA stream):
// group 0 copies K(j+2) during its V(j) (slot (j+2)%3 last held K(j-1), read by group 1 in phase
// 2j-1), group 1 copies V(j+1) during its V(j) (slot (j+1)&1 last held V(j-1), read by group 1's
// own M(j)).  Each copy is waited for by its issuing wave at the end of the following phase.
// LAG / PRIO / DIAG are tools/kbench_attn.hip experiments; the library uses the defaults.
// DIAG bits (timing only): 1 no softmax, 2 no MFMAs, 4 no LDS fragment reads, 8 no LDS-DMA
// copies, 16 s_memtime stamps of the waves of workgroup 0 into S.o, 32 empty VALU phase,
// 64 no phase barriers.
// ----------------------------------------------------------------------------------------
template <int KT, int LAG = 1, int PRIO = 1, int DIAG = 0>
__global__ __launch_bounds__(512, 2) void attention_h3pp_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                 float scale_log2e) {
  constexpr int WAVES = 8, QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  static_assert(NSUB == 2, "phase_m stages two 32-key sub-tiles");
  constexpr int PL = KT * kHeadDim;                    // one plane of a tile (elements), 128-byte rows
  constexpr int DMA_PER_WAVE = 2 * PL * 2 / 1024 / 4;  // 1 KiB LDS-DMA pieces per wave per tile
  static_assert(DMA_PER_WAVE * 4 * 1024 == 2 * PL * 2, "tile / wave group mismatch");
  // [K slots 0-2 | V slots 0-1], each [plane h | plane l][KT][64] fp16, 16-byte
  // chunks swizzled within a row: K chunk c of row r at c ^ ((r >> 1) & 7) (each ds_read_b128
  // lane group {0-3,12-15,20-27}, ... then covers all 16 slots of the 256-byte bank line),
  // V chunk c at c ^ 4*((r >> 1) & 1) (the transposed-read layout of attention_h3_kernel)
  __shared__ __attribute__((aligned(1024))) _Float16 smem[10 * PL];
  _Float16* const Ks = smem;
  _Float16* const Vs = smem + 6 * PL;

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * Nk * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * Nk * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int l32 = lane & 31, half = lane >> 5;

  // query pieces (x 2^ex per lane, see attention_h3_kernel): h, h 2^11, l
  const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
  f16x8 qh[4], qhs[4], ql[4];
  float c_lane;
  {
    const float* qr = Q + (size_t)qrow * kHeadDim + half * 8;
    f32x4 x[4][2];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s][0] = *reinterpret_cast<const f32x4*>(qr + 16 * s);
      x[s][1] = *reinterpret_cast<const f32x4*>(qr + 16 * s + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[s][0][e]), fabsf(x[s][1][e])));
    }
    mx = max_xor32(mx);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane = ldexpf(scale_log2e, -(11 + ex));
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[s][e >> 2][e & 3], ex), h, l);
        qh[s][e] = h;
        ql[s][e] = l;
        qhs[s][e] = h * (_Float16)kLoScale;
      }
  }

  // ---- staging by LDS-DMA: group 0 copies K tiles, group 1 V tiles.  A tile is 2 planes x KT
  // rows of 128 bytes; wave w of the group copies the 1 KiB pieces (8 rows each)
  // DMA_PER_WAVE*(w&3) + i.  Lane i of a piece fills row i/8 at chunk position i%8 and reads
  // source chunk (i%8) ^ swizzle(row).  Per lane the source offset within the piece is a
  // constant (dvo); the tile / piece offset goes into the wave-uniform base.
  const _Float16* const Gsrc = grp == 0 ? Kp : Vp;
  const uint32_t lds_grp =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)(grp == 0 ? Ks : Vs));
  const int lrow = lane >> 3, cpos = lane & 7;
  uint32_t dvo[DMA_PER_WAVE];
#pragma unroll
  for (int i = 0; i < DMA_PER_WAVE; ++i) {
    const int rg = ((wave & 3) * DMA_PER_WAVE + i) % (KT / 8);
    // row r = 8 rg + lrow: K swizzle (r >> 1) & 7, V swizzle 4 ((r >> 1) & 1)
    const int gswz = grp == 0 ? (((rg & 1) << 2) | (lrow >> 1)) : ((lrow >> 1) & 1) << 2;
    dvo[i] = (uint32_t)((lrow * kHeadDim + (cpos ^ gswz) * 8) * 2);
  }
  auto dma_tile = [&](int t0, int buf) {
    if constexpr (DIAG & 8) return;
    const bool tail = t0 + KT > Nk;  // last tile of a ragged Nk: clamp rows to Nk - 1
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const int piece = (wave & 3) * DMA_PER_WAVE + i;  // wave-uniform
      const int p = piece / (KT / 8), rg = piece % (KT / 8);
      const uint32_t lds = lds_grp + (uint32_t)((buf * 2 + p) * PL * 2 + rg * 1024);
      if (!tail) {
        dma16(Gsrc + p * ps + (size_t)(t0 + rg * 8) * kHeadDim, dvo[i], lds);
      } else {
        const uint32_t voff = dvo[i] + (uint32_t)((min(t0 + rg * 8 + lrow, Nk - 1) - lrow) * kHeadDim * 2);
        dma16(Gsrc + p * ps, voff, lds);
      }
    }
  };

  // per-lane LDS fragment offsets (see attention_h3_kernel for the transposed V reads)
  const int tq = (lane & 15) >> 2, tdim = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  const int vsw = ((tq >> 1) & 1) << 5;
  const int voff0 = (4 * half + tq) * kHeadDim + (tdim ^ vsw);
  const int voff1 = (4 * half + tq) * kHeadDim + ((32 + tdim) ^ vsw);
  // K fragment (row l32, chunk 2s + half) of a 32-row block, swizzled: koff0 ^ 16 s
  const int koff0 = l32 * kHeadDim + ((half ^ ((l32 >> 1) & 7)) * 8);

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};
  float m_use = -INFINITY;
  float l_run = 0.f;
  f32x16 sc[NSUB];                                // S(j): produced in M(j), consumed in V(j)
  f16x8 pph[NSUB][2], phs[NSUB][2], ppl[NSUB][2];  // P(j) pieces: V(j) -> M(j+1)
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    sc[u] = f32x16{0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) pph[u][s] = phs[u][s] = ppl[u][s] = f16x8{0};
  }

  // M(j) = [O += P(j-1) V(j-1) (PV: j > 0);  S(j) = K(j) Q^T (QK: j < ntiles)].  Its LDS reads
  // are staged one step ahead of the MFMAs that consume them (sched_barrier fences), so that at
  // most two fragment groups (64 VGPRs) are live.
  auto phase_m = [&](int j, auto pv_c, auto qk_c) {
    constexpr bool PV = decltype(pv_c)::value, QK = decltype(qk_c)::value;
    const _Float16* Vc = Vs + ((j - 1) & 1) * 2 * PL;
    const _Float16* Kc = Ks + (j % 3) * 2 * PL;
    f16x8 vf[NSUB][2][2][2];  // [u][s][dim tile][plane]
    f16x8 kf[NSUB][4][2];     // [u][s][plane]
    auto read_v = [&](int u) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr ((DIAG & 4) != 0) {
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            vf[u][s][0][p] = qh[2 * s + p];
            vf[u][s][1][p] = ql[2 * s + p];
          }
          continue;
        }
        const int vr = (u * 32 + 16 * s) * kHeadDim;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4 a0 = tr_read_h(Vc + p * PL + vr + voff0);
          const f16x4 a1 = tr_read_h(Vc + p * PL + vr + 8 * kHeadDim + voff0);
          const f16x4 b0 = tr_read_h(Vc + p * PL + vr + voff1);
          const f16x4 b1 = tr_read_h(Vc + p * PL + vr + 8 * kHeadDim + voff1);
          vf[u][s][0][p] = f16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          vf[u][s][1][p] = f16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        }
      }
    };
    auto read_k = [&](int u) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr ((DIAG & 4) != 0) {
          kf[u][s][0] = qh[s];
          kf[u][s][1] = ql[s];
          continue;
        }
        const int ko = koff0 ^ (16 * s);
        kf[u][s][0] = *reinterpret_cast<const f16x8*>(Kc + u * 32 * kHeadDim + ko);
        kf[u][s][1] = *reinterpret_cast<const f16x8*>(Kc + PL + u * 32 * kHeadDim + ko);
      }
    };
    auto pv_mfma = [&](int u) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const auto& v = vf[u][s];
        if constexpr ((DIAG & 2) != 0) {
          o0[s] += (float)v[0][0][1] + (float)v[0][1][2] + (float)phs[u][s][3] + (float)ppl[u][s][4];
          o1[s] += (float)v[1][0][1] + (float)v[1][1][2] + (float)pph[u][s][5];
        } else {
          o0 = mfma_h3(v[0][0], v[0][1], phs[u][s], ppl[u][s], pph[u][s], o0);
          o1 = mfma_h3(v[1][0], v[1][1], phs[u][s], ppl[u][s], pph[u][s], o1);
        }
      }
    };
    auto qk_mfma = [&](int u) {
      sc[u] = f32x16{0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr ((DIAG & 2) != 0)
          sc[u][s] += (float)kf[u][s][0][0] + (float)kf[u][s][1][1] + (float)qhs[s][2];
        else
          sc[u] = mfma_h3(kf[u][s][0], kf[u][s][1], qhs[s], ql[s], qh[s], sc[u]);
      }
    };
    auto fence = []() { __builtin_amdgcn_sched_barrier(0); };
    // [V0 K0] PV0 [V1] QK0 [K1] PV1 QK1: each read group is issued one 12-MFMA step before its use
    if constexpr (PV) read_v(0);
    if constexpr (QK) read_k(0);
    fence();
    if constexpr (PV) pv_mfma(0);
    fence();
    if constexpr (PV) read_v(1);
    fence();
    if constexpr (QK) qk_mfma(0);
    fence();
    if constexpr (QK) read_k(1);
    fence();
    if constexpr (PV) pv_mfma(1);
    fence();
    if constexpr (QK) qk_mfma(1);
  };

  // V(j) = softmax of S(j) -> P(j) pieces
  auto phase_v = [&](int j) {
    if constexpr ((DIAG & 32) != 0) return;
    if constexpr ((DIAG & 1) != 0) {
#pragma unroll
      for (int u = 0; u < NSUB; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) pph[u][s][e] = phs[u][s][e] = ppl[u][s][e] = (_Float16)sc[u][8 * s + e];
      l_run += 1.f;
      return;
    }
    const int t0 = j * KT;
    if (t0 + KT > Nk) {  // mask keys past the end (last tile only)
#pragma unroll
      for (int u = 0; u < NSUB; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
    }
    float mr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) mr[r] = fmaxf(sc[0][r], sc[1][r]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int r = 0; r < w; ++r) mr[r] = fmaxf(mr[r], mr[r + w]);
    const float tmax = max_xor32(mr[0]);
    const bool need = (tmax - m_use) * c_lane > 3.f;
    if (__ballot(need) != 0ull) {
      // O holds tiles < j here (P(j-1) V(j-1) was added in M(j)): the rescale covers all of it
      const float m_new = need ? tmax : m_use;
      const float alpha = __builtin_amdgcn_exp2f((m_use - m_new) * c_lane);
      m_use = m_new;
      l_run *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    const float mb = m_use * c_lane;
    float ps8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ps8[i] = 0.f;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[u][8 * s + e], c_lane, -mb));
          ps8[e] += p;
          const _Float16 h = (_Float16)p;
          const _Float16 hs = h * (_Float16)kLoScale;  // exact (p <= 8)
          pph[u][s][e] = h;
          phs[u][s][e] = hs;
          ppl[u][s][e] = (_Float16)fmaf(p, kLoScale, -(float)hs);
        }
    l_run += ((ps8[0] + ps8[1]) + (ps8[2] + ps8[3])) + ((ps8[4] + ps8[5]) + (ps8[6] + ps8[7]));
  };

  auto barrier = []() {
    if constexpr ((DIAG & 64) != 0) return;  // timing only: no phase barriers
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto wait_dma = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  const int ntiles = (Nk + KT - 1) / KT;
  // prologue: K(0), K(1) (group 0) and V(0) (group 1)
  dma_tile(0, 0);
  if (grp == 0 && ntiles > 1) dma_tile(KT, 1);
  wait_dma();
  __syncthreads();
  // the later-dispatched half loses VALU arbitration to its SIMD partner by default
  if (PRIO == 1 && grp == 1) __builtin_amdgcn_s_setprio(1);

  // Both groups run M(0) V(0) M(1) ... V(nt-1) M(nt), one phase per barrier; group 1 starts one
  // barrier late (LAG) and group 0 ends with an idle phase, so the barrier counts match.
  const std::true_type yes{};
  const std::false_type no{};
  // timing build: stamps kept in LDS (a global store per stamp would perturb the vmcnt waits)
  constexpr int NSTAMP = (DIAG & 16) ? 160 : 1;
  __shared__ unsigned long long stamps[8][NSTAMP];
  int nst = 0;
  auto stamp = [&]() {
    if constexpr ((DIAG & 16) != 0) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (lane == 0 && nst < NSTAMP) stamps[wave][nst] = t;
      ++nst;
    }
  };
  if (LAG && grp == 1) barrier();
  for (int j = 0; j < ntiles; ++j) {
    stamp();
    if (PRIO == 2) __builtin_amdgcn_s_setprio(1);  // the MFMA wave wins issue arbitration
    if (j == 0)
      phase_m(j, no, yes);
    else
      phase_m(j, yes, yes);
    if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    stamp();
    if (grp == 1) wait_dma();
    barrier();
    stamp();
    const bool issue = grp == 0 ? j + 2 < ntiles : j + 1 < ntiles;
    if (issue) {
      if (grp == 0)
        dma_tile((j + 2) * KT, (j + 2) % 3);
      else
        dma_tile((j + 1) * KT, (j + 1) & 1);
    }
    phase_v(j);
    stamp();
    if (grp == 0) {  // K(j+1), issued in V(j-1), must have landed; K(j+2) may stay in flight
      if (issue)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_WAVE) : "memory");
      else
        wait_dma();
    }
    barrier();
  }
  phase_m(ntiles, yes, no);
  barrier();
  if (LAG && grp == 0) barrier();
  if (PRIO == 1 && grp == 1) __builtin_amdgcn_s_setprio(0);
  if constexpr ((DIAG & 16) != 0) {
    if (blockIdx.x == 0 && lane == 0)
      for (int k = 0; k < min(nst, NSTAMP); ++k) reinterpret_cast<unsigned long long*>(S.o)[wave * 4096 + k] = stamps[wave][k];
  }

  const float l_tot = sum_xor32(l_run);
  const float inv = ldexpf(1.f / l_tot, -11);
  const int qq = q_blk + wave * 32 + l32;
  if (qq < Nq) {
    const int orow = S.o_row0 + b * Nq + qq;
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
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
      }
  }
}

template <int KT, int LAG = 1, int PRIO = 1, int DIAG = 0>
static hipError_t attention_h3pp_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 256;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3pp_kernel<KT, LAG, PRIO, DIAG>), dim3(items), dim3(512), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// fp16x3 attention, staggered groups (PREC_H3): same operands, numerics and LDS layout as
// attention_h3_kernel, one workgroup barrier per 64-key tile.  Waves 0-3 run each tile as
// [QK(t) MFMAs][softmax(t) VALU][PV(t) MFMAs]; waves 4-7 (their SIMD partners) defer the PV by
// one tile: [PV(t-1) MFMAs][QK(t) MFMAs][softmax(t) VALU].  Between the barriers the partners'
// MFMA and VALU blocks then line up against each other for two thirds of the tile (the softmax
// of one beside the MFMAs of the other) instead of running in lock-step.  The late group keeps
// P(t-1) in its score registers across the barrier and reads V(t-1) while V(t+1) is being
// staged, hence three V slots.
// ----------------------------------------------------------------------------------------
template <int KT>
__global__ __launch_bounds__(512, 2) void attention_h3s_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                float scale_log2e) {
  constexpr int WAVES = 8, NT = 64 * WAVES, QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  constexpr int KLD = kHeadDim + 8;       // K plane row stride (fp16)
  constexpr int CH = 2 * KT * 8;          // 16-byte chunks per tile per tensor
  constexpr int LDC = CH / NT;            // chunks per thread per tensor
  constexpr int KPL = KT * KLD, VPL = KT * kHeadDim;
  static_assert(CH % NT == 0, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * KPL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[3 * 2 * VPL];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * Nk * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * Nk * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool late = wave >= 4;
  const int l32 = lane & 31, half = lane >> 5;

  const int qrow = min(q_blk + wave * 32 + l32, Nq - 1);
  f16x8 qh[4], ql[4];  // q_h * 2^11 is re-formed per tile (the wave is at the VGPR limit)
  float c_lane;
  {
    const float* qr = Q + (size_t)qrow * kHeadDim + half * 8;
    f32x4 x[4][2];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s][0] = *reinterpret_cast<const f32x4*>(qr + 16 * s);
      x[s][1] = *reinterpret_cast<const f32x4*>(qr + 16 * s + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[s][0][e]), fabsf(x[s][1][e])));
    }
    mx = max_xor32(mx);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane = ldexpf(scale_log2e, -(11 + ex));
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[s][e >> 2][e & 3], ex), h, l);
        qh[s][e] = h;
        ql[s][e] = l;
      }
  }

  f32x4 rk[LDC], rv[LDC];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      const size_t src = (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8;
      rk[i] = *reinterpret_cast<const f32x4*>(Kp + src);
      rv[i] = *reinterpret_cast<const f32x4*>(Vp + src);
    }
  };
  auto sstore = [&](int kbuf, int vbuf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<f32x4*>(&Ks[(kbuf * 2 + p) * KPL + r * KLD + cb * 8]) = rk[i];
      *reinterpret_cast<f32x4*>(&Vs[(vbuf * 2 + p) * VPL + r * kHeadDim + ((cb ^ (((r >> 1) & 1) << 2)) * 8)]) = rv[i];
    }
  };

  const int tq = (lane & 15) >> 2, tp = lane & 3, tdim = ((lane >> 4) & 1) * 16 + 4 * tp;
  const int sw = ((tq >> 1) & 1) << 5;
  const int koff = l32 * KLD + 8 * half;
  const int voff0 = (4 * half + tq) * kHeadDim + (tdim ^ sw);
  const int voff1 = (4 * half + tq) * kHeadDim + ((32 + tdim) ^ sw);

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};
  float m_use = -INFINITY;
  float l_run = 0.f;
  f32x16 sc[NSUB];  // S(t), then P(t) in place (the late group carries P(t-1) across the barrier)

  // S^T = K Q^T (x 2^(11+e)) for the K tile in slot kbuf
  auto qk = [&](int kbuf) {
    const _Float16* Kc = Ks + kbuf * 2 * KPL + koff;
    f16x8 kf[NSUB][4][2];
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int off = u * 32 * KLD + 16 * s;
        kf[u][s][0] = *reinterpret_cast<const f16x8*>(Kc + off);
        kf[u][s][1] = *reinterpret_cast<const f16x8*>(Kc + KPL + off);
      }
    _Float16 two11 = (_Float16)kLoScale;
    asm volatile("" : "+v"(two11));  // keeps q_h * 2^11 from being hoisted out of the loop
    f16x8 qhs[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qhs[s] = qh[s] * two11;
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      sc[u] = f32x16{0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) sc[u] = mfma_h3(kf[u][s][0], kf[u][s][1], qhs[s], ql[s], qh[s], sc[u]);
    }
  };
  // mask / tile max / lazy reference raise / exp / sum: S(t) -> P(t) in sc
  auto softmax = [&](int t0) {
    if (t0 + KT > Nk) {
#pragma unroll
      for (int u = 0; u < NSUB; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
    }
    float mr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float m = sc[0][r];
#pragma unroll
      for (int u = 1; u < NSUB; ++u) m = fmaxf(m, sc[u][r]);
      mr[r] = m;
    }
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int r = 0; r < w; ++r) mr[r] = fmaxf(mr[r], mr[r + w]);
    const float tmax = max_xor32(mr[0]);
    const bool need = (tmax - m_use) * c_lane > 3.f;
    if (__ballot(need) != 0ull) {
      // O holds every tile before t here (both groups): the rescale covers all of it
      const float m_new = need ? tmax : m_use;
      const float alpha = __builtin_amdgcn_exp2f((m_use - m_new) * c_lane);
      m_use = m_new;
      l_run *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    const float mb = m_use * c_lane;
    float ps8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ps8[i] = 0.f;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[u][r], c_lane, -mb));
        sc[u][r] = p;
        ps8[(u * 16 + r) & 7] += p;
      }
    l_run += ((ps8[0] + ps8[1]) + (ps8[2] + ps8[3])) + ((ps8[4] + ps8[5]) + (ps8[6] + ps8[7]));
  };
  // O^T += V^T P^T (x 2^11) for the V tile in slot vbuf, P in sc
  auto pv = [&](int vbuf) {
    const _Float16* Vc = Vs + vbuf * 2 * VPL;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int vr = (u * 32 + 16 * s) * kHeadDim;
        f16x8 v[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4 a0 = tr_read_h(Vc + p * VPL + vr + voff0);
          const f16x4 a1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff0);
          const f16x4 b0 = tr_read_h(Vc + p * VPL + vr + voff1);
          const f16x4 b1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff1);
          v[0][p] = f16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          v[1][p] = f16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        }
        f16x8 ph, phs, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = sc[u][8 * s + j];
          const _Float16 h = (_Float16)p;
          const _Float16 hs = h * (_Float16)kLoScale;
          ph[j] = h;
          phs[j] = hs;
          pl[j] = (_Float16)fmaf(p, kLoScale, -(float)hs);
        }
        o0 = mfma_h3(v[0][0], v[0][1], phs, pl, ph, o0);
        o1 = mfma_h3(v[1][0], v[1][1], phs, pl, ph, o1);
      }
  };

  const int ntiles = (Nk + KT - 1) / KT;
  gload(0);
  sstore(0, 0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    if (t + 1 < ntiles) gload(t0 + KT);
    if (!late) {
      qk(t & 1);
      softmax(t0);
      pv(t % 3);
    } else {
      if (t > 0) pv((t + 2) % 3);  // PV(t-1): V(t-1) in slot (t-1) % 3
      qk(t & 1);
      softmax(t0);
    }
    if (t + 1 < ntiles) sstore((t + 1) & 1, (t + 1) % 3);
    __syncthreads();
  }
  if (late) pv((ntiles + 2) % 3);

  const float l_tot = sum_xor32(l_run);
  const float inv = ldexpf(1.f / l_tot, -11);  // 2^-11 exact: same rounding as (o 2^-11) / l
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    const int orow = S.o_row0 + b * Nq + q;
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
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
      }
  }
}

template <int KT>
static hipError_t attention_h3s_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 256;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3s_kernel<KT>), dim3(items), dim3(512), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// attention_h3m16_kernel -- measured, superseded by attention_h3f_kernel (same MFMA data flow,
// leaner softmax).  fp16x3 attention on v_mfma_f32_16x16x32_f16: the schedule of attention_h3_kernel
// (8 waves x 32 queries, 64-key tiles double-buffered in LDS, one barrier per tile, lazy softmax
// reference, context straight into ffn.0's plane image) with 16 x 16 MFMA tiles, which the chip
// runs at a higher sustained rate than 32 x 32 tiles on random data (tools/probe_mfma_shape.hip).
//   S^T[key][query] = K Q^T:  A = K tile (16 keys x 32 dims, lane: key l&15, dims 8(l>>4)..),
//                             B = Q^T (lane: query l&15, dims 8(l>>4)..), two k-steps per head.
//     Accumulator: lane l holds query l&15, keys 4(l>>4) + r (r < 4) of each 16-key tile.
//   O^T[dim][query] += V^T P^T over 32-key steps p: B = P^T with k index 8g+j <-> key
//     32p + 16(j>>2) + 4g + (j&3) (g = l>>4) -- exactly the S^T registers the lane already holds;
//     A = V^T, lane: dim l&15 of a 16-dim tile, the same 8 keys, two ds_read_b64_tr_b16 (4 keys
//     x 16 dims each per 16-lane group).
//   Per-query reductions (max, sum, q range) run over the 4 lanes sharing l&15 (xor 16, xor 32).
// LDS: rows of 64 halves (128 B); K 16-byte chunk c of row r at c ^ ((r >> 1) & 7), V chunk c at
// c ^ 2((r >> 1) & 3) -- conflict-free for the b128 fragment reads and the transposed reads.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ float max_xor16_32(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return max_xor32(v);
}
__device__ __forceinline__ float sum_xor16_32(float v) {
  v += __shfl_xor(v, 16, 64);
  return sum_xor32(v);
}

template <int KT>
__global__ __launch_bounds__(512, 2) void attention_h3m16_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                float scale_log2e) {
  constexpr int WAVES = 8, NT = 64 * WAVES, QB = 32 * WAVES;
  constexpr int NKT = KT / 16;             // 16-key tiles per tile
  constexpr int CH = 2 * KT * 8;           // 16-byte chunks per tile per tensor
  constexpr int LDC = CH / NT;
  constexpr int PL = KT * kHeadDim;        // one plane of a tile (elements)
  static_assert(CH % NT == 0 && KT % 32 == 0, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * PL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 2 * PL];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * Nk * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * Nk * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;

  // Q^T B operand: query qt*16 + r16 of the wave, k-step ks: dims 32 ks + 8 g + j, scaled per
  // query by 2^ex (row max over the 4 lanes sharing the query in [8, 16))
  f16x8 qh[2][2], qhs[2][2], ql[2][2];
  float c_lane[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qrow = min(q_blk + wave * 32 + qt * 16 + r16, Nq - 1);
    const float* qr = Q + (size_t)qrow * kHeadDim + 8 * g;
    f32x4 x[2][2];
    float mx = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      x[ks][0] = *reinterpret_cast<const f32x4*>(qr + 32 * ks);
      x[ks][1] = *reinterpret_cast<const f32x4*>(qr + 32 * ks + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[ks][0][e]), fabsf(x[ks][1][e])));
    }
    mx = max_xor16_32(mx);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane[qt] = ldexpf(scale_log2e, -(11 + ex));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[ks][e >> 2][e & 3], ex), h, l);
        qh[qt][ks][e] = h;
        ql[qt][ks][e] = l;
        qhs[qt][ks][e] = h * (_Float16)kLoScale;
      }
  }

  // tile staging through registers: chunk c -> plane c / (KT*8), row (c / 8) % KT, chunk c % 8
  f32x4 rk[LDC], rv[LDC];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      const size_t src = (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8;
      rk[i] = *reinterpret_cast<const f32x4*>(Kp + src);
      rv[i] = *reinterpret_cast<const f32x4*>(Vp + src);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<f32x4*>(&Ks[(buf * 2 + p) * PL + r * kHeadDim + ((cb ^ ((r >> 1) & 7)) * 8)]) = rk[i];
      *reinterpret_cast<f32x4*>(&Vs[(buf * 2 + p) * PL + r * kHeadDim + ((cb ^ (((r >> 1) & 3) << 1)) * 8)]) = rv[i];
    }
  };

  // per-lane LDS offsets (elements).  K fragment (key kt*16 + r16, chunk 4 ks + g), swizzle of row
  // r16 (kt*16 does not change (r >> 1) & 7).  V transposed read: the 16-lane group g reads rows
  // (keys) 32p + 16h + 4g + q (q = (lane & 15) >> 2) at dims 16 dt + 4 (lane & 3); row bits (r>>1)&3
  // = (2g + (q >> 1)) & 3.
  const int kswz = (r16 >> 1) & 7;
  const int koff = r16 * kHeadDim;
  const int vq = (lane & 15) >> 2, vp4 = lane & 3;
  const int vrow = 4 * g + vq;
  const int vswz = ((vrow >> 1) & 3) << 1;

  f32x4 o[4][2];  // O^T tiles (x 2^11): [dim tile dt][query tile qt]
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt][0] = o[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_use[2] = {-INFINITY, -INFINITY};
  float l_run[2] = {0.f, 0.f};

  const int ntiles = (Nk + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    const _Float16* Kc = Ks + cur * 2 * PL;
    const _Float16* Vc = Vs + cur * 2 * PL;

    // ---- S^T = K Q^T
    f16x8 kf[NKT][2][2];  // [key tile][k-step][plane]
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int off = kt * 16 * kHeadDim + koff + (((4 * ks + g) ^ kswz) << 3);
        kf[kt][ks][0] = *reinterpret_cast<const f16x8*>(Kc + off);
        kf[kt][ks][1] = *reinterpret_cast<const f16x8*>(Kc + PL + off);
      }
    asm volatile("" ::: "memory");
    if (t + 1 < ntiles) gload(t0 + KT);
    f32x4 sc[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a = mfma_h3_16(kf[kt][ks][0], kf[kt][ks][1], qhs[qt][ks], ql[qt][ks], qh[qt][ks], a);
        sc[kt][qt] = a;
      }
    // ---- V^T fragments of the tile: [32-key step p][dim tile dt][plane] (8 keys per lane)
    f16x8 vf[NKT / 2][4][2];
#pragma unroll
    for (int p = 0; p < NKT / 2; ++p)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          // rows 32p + vrow and 32p + 16 + vrow; dims 16 dt + 4 vp4 -> chunk 2dt + (vp4 >> 1), 8-byte half vp4 & 1
          const int col = ((((2 * dt + (vp4 >> 1)) ^ vswz) << 3) + 4 * (vp4 & 1));
          const f16x4 lo = tr_read_h(Vc + pl * PL + (32 * p + vrow) * kHeadDim + col);
          const f16x4 hi = tr_read_h(Vc + pl * PL + (32 * p + 16 + vrow) * kHeadDim + col);
          vf[p][dt][pl] = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
    asm volatile("" ::: "memory");
    // ---- softmax per query tile: keys t0 + 16 kt + 4 g + r
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      if (t0 + KT > Nk) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t0 + 16 * kt + 4 * g + r >= Nk) sc[kt][qt][r] = -INFINITY;
      }
      float mr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float m = sc[0][qt][r];
#pragma unroll
        for (int kt = 1; kt < NKT; ++kt) m = fmaxf(m, sc[kt][qt][r]);
        mr[r] = m;
      }
      const float tmax = max_xor16_32(fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3])));
      const bool need = (tmax - m_use[qt]) * c_lane[qt] > 3.f;
      if (__ballot(need) != 0ull) {
        const float m_new = need ? tmax : m_use[qt];
        const float alpha = __builtin_amdgcn_exp2f((m_use[qt] - m_new) * c_lane[qt]);
        m_use[qt] = m_new;
        l_run[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dt][qt][r] *= alpha;
      }
      const float mb = m_use[qt] * c_lane[qt];
      float ps4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kt][qt][r], c_lane[qt], -mb));
          sc[kt][qt][r] = pv;
          ps4[r] += pv;
        }
      l_run[qt] += (ps4[0] + ps4[1]) + (ps4[2] + ps4[3]);
    }
    // ---- O^T += V^T P^T (x 2^11), 32 keys per step
#pragma unroll
    for (int p = 0; p < NKT / 2; ++p)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f16x8 ph, phs, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float pv = sc[2 * p + (j >> 2)][qt][j & 3];
          const _Float16 h = (_Float16)pv;
          const _Float16 hs = h * (_Float16)kLoScale;
          ph[j] = h;
          phs[j] = hs;
          pl[j] = (_Float16)fmaf(pv, kLoScale, -(float)hs);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][qt] = mfma_h3_16(vf[p][dt][0], vf[p][dt][1], phs, pl, ph, o[dt][qt]);
      }

    if (t + 1 < ntiles) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // context rows into the plane image (K = 256): lane holds dims 16 dt + 4 g + r of query qt*16+r16
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l_tot = sum_xor16_32(l_run[qt]);
    const float inv = ldexpf(1.f / l_tot, -11);
    const int q = q_blk + wave * 32 + qt * 16 + r16;
    if (q < Nq) {
      const int orow = S.o_row0 + b * Nq + q;
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
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
      }
    }
  }
}

template <int KT>
static hipError_t attention_h3m16_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 256;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3m16_kernel<KT>), dim3(items), dim3(512), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

// attention_h3f_kernel -- measured, superseded by attention_h3g_kernel: the same math with K/V
// staged through registers (global_load -> ds_write) and one 64-key tile per barrier.
template <int KT>
__global__ __launch_bounds__(512, 2) void attention_h3f_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                float scale_log2e) {
  constexpr int WAVES = 8, NT = 64 * WAVES, QB = 32 * WAVES;
  constexpr int NKT = KT / 16;
  constexpr int CH = 2 * KT * 8;
  constexpr int LDC = CH / NT;
  constexpr int PL = KT * kHeadDim;
  static_assert(CH % NT == 0 && KT == 64, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * 2 * PL];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 2 * PL];

  const int item = xcd_chunk(blockIdx.x, gridDim.x);
  const int qb = item % nqb;
  const int sbh = item / nqb;
  const int set = sbh / (B * H), bh = sbh - set * (B * H);
  const AttnSet& S = set == 0 ? s0 : s1;
  const int q_blk = qb * QB;
  if (q_blk >= S.Nq) return;
  const int Nq = S.Nq, Nk = S.Nk;
  const float* Q = S.q + (size_t)bh * Nq * kHeadDim;
  const _Float16* Kp = static_cast<const _Float16*>(S.kp) + (size_t)bh * Nk * kHeadDim;
  const _Float16* Vp = static_cast<const _Float16*>(S.vp) + (size_t)bh * Nk * kHeadDim;
  const long long ps = S.pstride;
  const int head = bh % H;
  const int b = bh / H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;

  f16x8 qh[2][2], qhs[2][2], ql[2][2];
  float c_lane[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qrow = min(q_blk + wave * 32 + qt * 16 + r16, Nq - 1);
    const float* qr = Q + (size_t)qrow * kHeadDim + 8 * g;
    f32x4 x[2][2];
    float mx = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      x[ks][0] = *reinterpret_cast<const f32x4*>(qr + 32 * ks);
      x[ks][1] = *reinterpret_cast<const f32x4*>(qr + 32 * ks + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(x[ks][0][e]), fabsf(x[ks][1][e])));
    }
    mx = max_x16_32(mx);
    int ex = 0;
    if (mx > 0.f && mx <= 3.0e38f) {
      int E;
      (void)frexpf(mx, &E);
      ex = min(max(4 - E, -100), 100);
    }
    c_lane[qt] = ldexpf(scale_log2e, -(11 + ex));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split2h(ldexpf(x[ks][e >> 2][e & 3], ex), h, l);
        qh[qt][ks][e] = h;
        ql[qt][ks][e] = l;
        qhs[qt][ks][e] = h * (_Float16)kLoScale;
      }
  }

  f32x4 rk[LDC], rv[LDC];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      const size_t src = (size_t)p * ps + (size_t)min(t0 + r, Nk - 1) * kHeadDim + cb * 8;
      rk[i] = *reinterpret_cast<const f32x4*>(Kp + src);
      rv[i] = *reinterpret_cast<const f32x4*>(Vp + src);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LDC; ++i) {
      const int c = tid + i * NT;
      const int p = c / (KT * 8), r = (c / 8) % KT, cb = c % 8;
      *reinterpret_cast<f32x4*>(&Ks[(buf * 2 + p) * PL + r * kHeadDim + ((cb ^ ((r >> 1) & 7)) * 8)]) = rk[i];
      *reinterpret_cast<f32x4*>(&Vs[(buf * 2 + p) * PL + r * kHeadDim + ((cb ^ (((r >> 1) & 3) << 1)) * 8)]) = rv[i];
    }
  };

  const int kswz = (r16 >> 1) & 7;
  const int vq = (lane & 15) >> 2, vp4 = lane & 3;
  const int vrow = 4 * g + vq;
  const int vswz = ((vrow >> 1) & 3) << 1;
  // per-lane LDS bases; everything else in a tile's reads is a compile-time offset
  const _Float16* kbase = Ks + r16 * kHeadDim;
  const _Float16* vbase = Vs + vrow * kHeadDim + 4 * (vp4 & 1);
  int kcol[2], vcol[4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kcol[ks] = ((4 * ks + g) ^ kswz) << 3;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) vcol[dt] = ((2 * dt + (vp4 >> 1)) ^ vswz) << 3;

  f32x4 o[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt][0] = o[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_use[2] = {-INFINITY, -INFINITY};
  float l_run[2] = {0.f, 0.f};
  const int ntiles = (Nk + KT - 1) / KT;

  auto body = [&](auto BUFc, auto MASKc, int t) {
    constexpr int buf = decltype(BUFc)::value;
    constexpr bool MASK = decltype(MASKc)::value;
    const int t0 = t * KT;
    const _Float16* Kc = kbase + buf * 2 * PL;
    const _Float16* Vc = vbase + buf * 2 * PL;

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
    if (t + 1 < ntiles) gload(t0 + KT);
    f32x4 sc[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
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
      const float m0 = max3f(sc[0][qt][0], sc[0][qt][1], sc[0][qt][2]);
      const float m1 = max3f(sc[0][qt][3], sc[1][qt][0], sc[1][qt][1]);
      const float m2 = max3f(sc[1][qt][2], sc[1][qt][3], sc[2][qt][0]);
      const float m3 = max3f(sc[2][qt][1], sc[2][qt][2], sc[2][qt][3]);
      const float m4 = max3f(sc[3][qt][0], sc[3][qt][1], sc[3][qt][2]);
      const float lmax = fmaxf(max3f(m0, m1, m2), max3f(m3, m4, sc[3][qt][3]));
      // the lane-local max decides whether any query can need a raise; only then are the four
      // lanes of each query reduced (the raise itself is per query, exactly as in h3/h3m16)
      if (__ballot((lmax - m_use[qt]) * c_lane[qt] > 3.f) != 0ull) {
        const float tmax = max_x16_32(lmax);
        const bool need = (tmax - m_use[qt]) * c_lane[qt] > 3.f;
        const float m_new = need ? tmax : m_use[qt];
        const float alpha = __builtin_amdgcn_exp2f((m_use[qt] - m_new) * c_lane[qt]);
        m_use[qt] = m_new;
        l_run[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dt][qt][r] *= alpha;
      }
      // e = p 2^11
      const float mb = fmaf(m_use[qt], c_lane[qt], -11.f);
      float ps4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][qt][r], c_lane[qt], -mb));
          sc[kt][qt][r] = e;
          ps4[r] += e;
        }
      l_run[qt] += (ps4[0] + ps4[1]) + (ps4[2] + ps4[3]);
    }
#pragma unroll
    for (int p = 0; p < NKT / 2; ++p)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f16x8 ph, phs, pl;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float e0 = sc[2 * p + (j >> 2)][qt][j & 3];
          const float e1 = sc[2 * p + (j >> 2)][qt][(j & 3) + 1];
          const f16x2 hs = {(_Float16)e0, (_Float16)e1};
          const f16x2 h = hs * (f16x2){(_Float16)(1.f / kLoScale), (_Float16)(1.f / kLoScale)};
          const f16x2 lo = lo_pair(e0, e1, hs);
          phs[j] = hs[0]; phs[j + 1] = hs[1];
          ph[j] = h[0]; ph[j + 1] = h[1];
          pl[j] = lo[0]; pl[j + 1] = lo[1];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][qt] = mfma_h3_16(vf[p][dt][0], vf[p][dt][1], phs, pl, ph, o[dt][qt]);
      }

    if (t + 1 < ntiles) sstore(buf ^ 1);
    __syncthreads();
  };

  gload(0);
  sstore(0);
  __syncthreads();
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using NoMask = std::integral_constant<bool, false>;
  using Mask = std::integral_constant<bool, true>;
  const int nfull = Nk / KT;
  int t = 0;
  for (; t + 2 <= nfull; t += 2) {
    body(B0{}, NoMask{}, t);
    body(B1{}, NoMask{}, t + 1);
  }
  if (t < nfull) {
    body(B0{}, NoMask{}, t);
    if (t + 1 < ntiles) body(B1{}, Mask{}, t + 1);
  } else if (t < ntiles) {
    body(B0{}, Mask{}, t);
  }

  // context rows into the plane image: o = 2^11 sum(v p) (the MFMA scale), l_run = 2^11 sum(p),
  // so 1 / l_run is the old 2^-11 / l exactly
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l_tot = sum_x16_32(l_run[qt]);
    const float inv = 1.f / l_tot;
    const int q = q_blk + wave * 32 + qt * 16 + r16;
    if (q < Nq) {
      const int orow = S.o_row0 + b * Nq + q;
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
        *reinterpret_cast<f16x4*>(S.op + off) = h;
        *reinterpret_cast<f16x4*>(S.op + S.ops + off) = l;
      }
    }
  }
}

template <int KT>
static hipError_t attention_h3f_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 256;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3f_kernel<KT>), dim3(items), dim3(512), 0, st, s0, s1, B, H, nqb,
                     scale * 1.4426950408889634f);
  return hipGetLastError();
}

}  // namespace lg
