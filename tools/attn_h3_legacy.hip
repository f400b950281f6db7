// attention_h3_kernel: the first fp16x3 attention (register-staged K/V tiles, 32x32 MFMAs),
// superseded in the library by attention_h3g_kernel (attention.hip) and kept here for
// tools/kbench_attn.hip comparisons and tools/attn_experiments.hip.  Included after attention.hip.
// DIAG: 1 = no softmax VALU, 2 = no MFMAs, 3 = MFMAs alone (no LDS, staging or barriers) -- to
// split the loop's time.
namespace lg {
template <int WAVES, int KT, int OCC, int DIAG = 0>
__global__ __launch_bounds__(64 * WAVES, OCC) void attention_h3_kernel(AttnSet s0, AttnSet s1, int B, int H, int nqb,
                                                                        float scale_log2e) {
  constexpr int NT = 64 * WAVES;
  constexpr int QB = 32 * WAVES;
  constexpr int NSUB = KT / 32;
  constexpr int KLD = kHeadDim + 8;       // K plane row stride (fp16)
  constexpr int CH = 2 * KT * 8;          // 16-byte chunks per tile per tensor (2 planes x KT rows x 8)
  constexpr int LDC = CH / NT;            // chunks per thread per tensor
  constexpr int KPL = KT * KLD, VPL = KT * kHeadDim;  // plane sizes (elements)
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

  // Q^T B operand: k-step s, lane half h holds dims 16s + 8h + j (j = 0..7) of its query,
  // scaled by 2^ex so that the row max lies in [8, 16).
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
      (void)frexpf(mx, &E);  // mx = m 2^E, m in [0.5, 1)
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

  // tile staging: chunk c -> plane c / (KT*8), row (c / 8) % KT, 8-dim column block c % 8
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
      *reinterpret_cast<f32x4*>(&Ks[(buf * 2 + p) * KPL + r * KLD + cb * 8]) = rk[i];
      *reinterpret_cast<f32x4*>(&Vs[(buf * 2 + p) * VPL + r * kHeadDim + ((cb ^ (((r >> 1) & 1) << 2)) * 8)]) = rv[i];
    }
  };

  // per-lane LDS offsets: K fragment row l32, dims 8*half..; transposed V reads: 16-lane group
  // g = lane >> 4 covers dims (g & 1) * 16 + 4p of lane half h = g >> 1, rows ka + tq (+8)
  const int tq = (lane & 15) >> 2, tp = lane & 3, tdim = ((lane >> 4) & 1) * 16 + 4 * tp;
  const int sw = ((tq >> 1) & 1) << 5;  // V half swap of rows with key bit 1 set (ka % 4 == 0)
  const int koff = l32 * KLD + 8 * half;
  const int voff0 = (4 * half + tq) * kHeadDim + (tdim ^ sw);
  const int voff1 = (4 * half + tq) * kHeadDim + ((32 + tdim) ^ sw);

  f32x16 o0 = f32x16{0.f}, o1 = f32x16{0.f};  // O^T tiles (x 2^11): dims [0,32) and [32,64)
  float m_use = -INFINITY;                    // softmax reference (raw score units), raised lazily
  float l_run = 0.f;

  const int ntiles = (Nk + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const int t0 = t * KT;
    const _Float16* Kc = Ks + cur * 2 * KPL + koff;
    const _Float16* Vc = Vs + cur * 2 * VPL;

    // ---- S^T = K Q^T (x 2^(11+e)).  All K fragments of the tile are read up front (64 VGPRs),
    // so the MFMAs wait on the first read only instead of one LDS round trip per k-step.
    f16x8 kf[NSUB][4][2];
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int off = u * 32 * KLD + 16 * s;
        if constexpr (DIAG == 3) {
          kf[u][s][0] = qh[s];
          kf[u][s][0][u] = (_Float16)(float)t;  // keep the MFMAs inside the loop
          kf[u][s][1] = ql[s];
        } else {
          kf[u][s][0] = *reinterpret_cast<const f16x8*>(Kc + off);
          kf[u][s][1] = *reinterpret_cast<const f16x8*>(Kc + KPL + off);
        }
      }
    asm volatile("" ::: "memory");
    if (DIAG != 3 && t + 1 < ntiles) gload(t0 + KT);
    f32x16 sc[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      sc[u] = f32x16{0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr (DIAG == 2) {
          sc[u][s] += (float)kf[u][s][0][0] + (float)kf[u][s][1][1];
        } else {
          sc[u] = mfma_h3(kf[u][s][0], kf[u][s][1], qhs[s], ql[s], qh[s], sc[u]);
        }
      }
    }
    // ---- V^T fragments of the tile (transposed reads), issued before the softmax so their
    // latency hides behind it: key rows ka + tq (+8), ka = u*32 + 16s + 4*half
    f16x8 vf[NSUB][2][2][2];  // [u][s][dim tile][plane]
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int vr = (u * 32 + 16 * s) * kHeadDim;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          if constexpr (DIAG == 3) {
            vf[u][s][0][p] = qhs[s];
            vf[u][s][1][p] = ql[s + 2 * p];
            continue;
          }
          const f16x4 a0 = tr_read_h(Vc + p * VPL + vr + voff0);
          const f16x4 a1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff0);
          const f16x4 b0 = tr_read_h(Vc + p * VPL + vr + voff1);
          const f16x4 b1 = tr_read_h(Vc + p * VPL + vr + 8 * kHeadDim + voff1);
          vf[u][s][0][p] = f16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          vf[u][s][1][p] = f16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        }
      }
    asm volatile("" ::: "memory");
    if constexpr (DIAG != 1 && DIAG != 3) {
      if (t0 + KT > Nk) {  // mask keys past the end (last tile only)
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (t0 + u * 32 + row32(r, half) >= Nk) sc[u][r] = -INFINITY;
      }
      // ---- tile max (tree), lazy reference raise
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
    }

    // ---- O^T += V^T P^T (x 2^11), 16 keys per MFMA step
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 ph, phs, pl;
        if constexpr (DIAG == 1 || DIAG == 3) {
#pragma unroll
          for (int j = 0; j < 8; ++j) ph[j] = phs[j] = pl[j] = (_Float16)sc[u][8 * s + j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float p = sc[u][8 * s + j];
            const _Float16 h = (_Float16)p;
            const _Float16 hs = h * (_Float16)kLoScale;
            ph[j] = h;
            phs[j] = hs;
            pl[j] = (_Float16)fmaf(p, kLoScale, -(float)hs);
          }
        }
        // keys of element j: ka + j (j < 4), ka + 8 + (j - 4) (j >= 4), ka = u*32 + 16s + 4*half
        const auto& v = vf[u][s];
        if constexpr (DIAG == 2) {
          o0[s] += (float)v[0][0][1] + (float)v[0][1][2] + (float)ph[3] + (float)pl[4] + (float)phs[5];
          o1[s] += (float)v[1][0][1] + (float)v[1][1][2];
        } else {
          o0 = mfma_h3(v[0][0], v[0][1], phs, pl, ph, o0);
          o1 = mfma_h3(v[1][0], v[1][1], phs, pl, ph, o1);
        }
      }

    if constexpr (DIAG != 3) {
      if (t + 1 < ntiles) sstore(cur ^ 1);
      __syncthreads();
    }
    cur ^= 1;
  }

  const float l_tot = sum_xor32(l_run);
  const float inv = ldexpf(1.f / l_tot, -11);  // 2^-11 exact: same rounding as (o 2^-11) / l
  const int q = q_blk + wave * 32 + l32;
  if (q < Nq) {
    // context row into the plane image (K = 256): register r = 4g + e holds dim 8g + 4*half + e
    // (+32 for o1); 4 consecutive dims = 8 bytes per plane.  |o| <= max|v| <= 65504 (v checked).
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

template <int WAVES, int KT, int OCC, int DIAG = 0>
static hipError_t attention_h3_launch(const AttnSet& s0, const AttnSet& s1, int B, int H, float scale, hipStream_t st) {
  constexpr int QB = 32 * WAVES;
  const int nq = s0.Nq > s1.Nq ? s0.Nq : s1.Nq;
  if (nq == 0 || B == 0) return hipSuccess;
  if (s0.Nk <= 0 || s1.Nk <= 0) return hipErrorInvalidValue;
  const int nqb = (nq + QB - 1) / QB;
  const int items = nqb * B * H * 2;
  hipLaunchKernelGGL((attention_h3_kernel<WAVES, KT, OCC, DIAG>), dim3(items), dim3(64 * WAVES), 0, st, s0, s1, B, H,
                     nqb, scale * 1.4426950408889634f);
  return hipGetLastError();
}

}  // namespace lg
