// Prototype, measured and NOT adopted (profiles/r02/kbench_gemm_persistent.txt: 6-27 % slower than
// gemm_h3_kernel; tools only, built by tools/kbench_gemm.hip): persistent 256 x 256 fp16x3 GEMM whose
// epilogue stores drain under the next tile's k-loop.
//
// gemm_h3_kernel runs one tile per workgroup: every CU finishes its k-loop, then stores its tile,
// all CUs at once (phase-locked), with the matrix cores idle through the store phase.  Here a
// workgroup loops over tiles; the first k-tile of tile t+1 is copied into the idle stage while
// tile t's last k-tile is multiplied, and tile t's epilogue transposes through a small per-wave
// LDS window (2 KiB: 8 rows x 64 columns) beside the two stages, so the stages stay free.  The
// next tile's first wait counts only the copy that precedes the epilogue's stores (vmcnt retires
// in order); the second k-tile's wait is the first to cover the stores, one k-tile later.
// EPI_STORE with Y (fp32) and/or Yp (planes), bias, out_scale; no residual, no row mask.
#pragma once
#include "../cs566-project-lightglue_amd/csrc/common.h"
#include "../cs566-project-lightglue_amd/csrc/kernels.h"

namespace lg {

template <int N>
__device__ __forceinline__ void pwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(1024) void gemm_h3p_kernel(GemmH3Args g) {
  constexpr int BM = 256, BN = 256, BK = kKB, NW = 16, WGN = 4;
  constexpr int APT = BM * BK * 2, WPT = BN * BK * 2;
  constexpr int STAGE_BYTES = 2 * APT + 2 * WPT;  // 64 KiB
  constexpr int PPW = STAGE_BYTES / 1024 / NW;     // 4
  constexpr int WIN = 8 * 64 * 4;                  // per-wave epilogue window (bytes)
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES + NW * WIN];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WGN) * 64, wn0 = (wave % WGN) * 64;
  const int num_m = (g.R + BM - 1) / BM, num_n = g.Nout / BN, T = num_m * num_n;
  const int nk = g.K / BK;
  const float accs = g.acc_scale;
  const int eo = g.Yp ? range_exponent(g.ro) : 0;
  const float so = ldexpf(1.f, -eo);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem);
  const uint32_t voff = lane * 16;
  auto coords = [&](int it, int& m0, int& n0) {
    // workgroup b takes b, b + G, ...: with G a multiple of 8 every tile of a workgroup stays on
    // its XCD, and the remap gives each XCD a contiguous tile range (row panels share an L2)
    const int xcd = it & 7, local = it >> 3, base = T >> 3, extra = T & 7;
    const int tile = xcd * base + (xcd < extra ? xcd : extra) + local;
    m0 = (tile / num_n) * BM;
    n0 = (tile % num_n) * BN;
  };
  auto issue = [&](int m0, int n0, int kt, int stage) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      const char* src;
      if (q < 2 * (APT / 1024)) {
        const int pl = q / (APT / 1024), pc = q % (APT / 1024);
        src = reinterpret_cast<const char*>(g.A0.p + pl * g.A0.ps + ((size_t)kt * g.A0.rows_pad + m0) * BK) + pc * 1024;
      } else {
        const int qw = q - 2 * (APT / 1024);
        const int pl = qw / (WPT / 1024), pc = qw % (WPT / 1024);
        src = reinterpret_cast<const char*>(g.W.p + pl * g.W.ps + ((size_t)kt * g.W.rows_pad + n0) * BK) + pc * 1024;
      }
      dma16(src, voff, lds0 + stage * STAGE_BYTES + q * 1024);
    }
  };
  auto frag = [&](const char* st, int t0, int r, int c) {
    return *reinterpret_cast<const f16x8*>(st + t0 + r * (BK * 2) + ((c ^ plane_swz(r)) << 4));
  };
  f32x4 acc[4][4];
  auto compute = [&](int stage) {
    const char* st = smem + stage * STAGE_BYTES;
    const int c = lane >> 4, r16 = lane & 15;
    f16x8 ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = frag(st, 0, wm0 + i * 16 + r16, c);
      al[i] = frag(st, APT, wm0 + i * 16 + r16, c);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn0 + j * 16 + r16;
      const f16x8 wh = frag(st, 2 * APT, r, c);
      const f16x8 wl = frag(st, 2 * APT + WPT, r, c);
      const f16x8 whs = wh * (_Float16)kLoScale;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = mfma_h3_16(ah[i], al[i], whs, wl, wh, acc[i][j]);
    }
  };

  int it = blockIdx.x;
  if (it >= T) return;
  int m0, n0;
  coords(it, m0, n0);
  const int c4 = (lane & 7) * 4, cq = (lane & 7) * 8;
  const bool fp32_pass = g.Y != nullptr;
  auto load_bias = [&](int n0_, f32x4& b0, f32x4& b1) {
    b0 = b1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (g.bias) {
      const int ca = fp32_pass ? c4 : cq, cb = fp32_pass ? 32 + c4 : cq + 4;
      b0 = *reinterpret_cast<const f32x4*>(g.bias + n0_ + wn0 + ca);
      b1 = *reinterpret_cast<const f32x4*>(g.bias + n0_ + wn0 + cb);
    }
  };
  f32x4 b0, b1;
  load_bias(n0, b0, b1);
  issue(m0, n0, 0, 0);
  int gk = 0;         // k-tiles multiplied so far (stage parity)
  int pend = -1;      // vm instructions issued by this wave after the pending prefetch (-1: none)
  float wmax = 0.f;
  float* ep = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES + wave * WIN);
  for (;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int it_next = it + (int)gridDim.x;
    int mn = 0, nn = 0;
    if (it_next < T) coords(it_next, mn, nn);
    f32x4 nb0 = b0, nb1 = b1;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt == 0 && pend == 32) pwait_vm<32>();  // the prefetch, not the previous tile's stores
      else pwait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 1 < nk) {
        issue(m0, n0, kt + 1, (gk + 1) & 1);
      } else if (it_next < T) {
        issue(mn, nn, 0, (gk + 1) & 1);  // the next tile's first k-tile, ahead of this epilogue
        load_bias(nn, nb0, nb1);
      }
      compute(gk & 1);
      ++gk;
    }
    // epilogue: 8 passes of 8 rows (rows 16 i + 4 h2 + r of the wave tile, h2 = pass & 1 selects
    // the lane half (lane >> 5) that owns them) through the wave's window
    const bool full = m0 + BM <= g.R;
    int nvm = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int i = p >> 1, h = p & 1;
      if ((lane >> 5) == h) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = ((lane >> 4) & 1) * 4 + r, c = j * 16 + (lane & 15);
            ep[rr * 64 + (c ^ ((rr & 1) << 2))] = acc[i][j][r];
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int rr = lane >> 3;
      const int row = m0 + wm0 + 16 * i + 8 * h + rr;
      const int sw = (rr & 1) << 2;
      float* pa = ep + rr * 64 + ((fp32_pass ? c4 : cq) ^ sw);
      float* pb = ep + rr * 64 + ((fp32_pass ? 32 + c4 : cq + 4) ^ sw);
      f32x4 v0 = *reinterpret_cast<const f32x4*>(pa), v1 = *reinterpret_cast<const f32x4*>(pb);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] = fmaf(v0[e], accs, b0[e]) * g.out_scale;
        v1[e] = fmaf(v1[e], accs, b1[e]) * g.out_scale;
      }
      if (fp32_pass) {
        if (row < g.R) {
          float* yp = g.Y + (size_t)row * g.ldy + n0 + wn0 + c4;
          *reinterpret_cast<f32x4*>(yp) = v0;
          *reinterpret_cast<f32x4*>(yp + 32) = v1;
        }
        nvm += 2;
        if (g.Yp) {
          *reinterpret_cast<f32x4*>(pa) = v0;
          *reinterpret_cast<f32x4*>(pb) = v1;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
          v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
        }
      }
      if (g.Yp) {
        f16x8 hh, ll;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = e < 4 ? v0[e] : v1[e - 4];
          wmax = fmaxf(wmax, fabsf(v));
          _Float16 a, c;
          split2h(v * so, a, c);
          hh[e] = a;
          ll[e] = c;
        }
        if (row < g.R) {
          const size_t off = plane_off(row, n0 + wn0 + cq, g.yrows_pad);
          *reinterpret_cast<f16x8*>(g.Yp + off) = hh;
          *reinterpret_cast<f16x8*>(g.Yp + g.yps + off) = ll;
        }
        nvm += 2;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // window reads done before the next pass
    }
    // exact store count only when every row group issued its stores (full tile, both outputs)
    pend = (full && fp32_pass && g.Yp && nvm == 32) ? 32 : 0;
    if (it_next >= T) break;
    it = it_next;
    m0 = mn;
    n0 = nn;
    b0 = nb0;
    b1 = nb1;
  }
  if (g.Yp) range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem));
}

hipError_t gemm_h3p(const GemmH3Args& a, hipStream_t st, int grid) {
  if (a.Nout % 256 || a.K % kKB || a.K0 != a.K || a.rm.cnt || a.res || a.relu) return hipErrorInvalidValue;
  const int T = ((a.R + 255) / 256) * (a.Nout / 256);
  const int g = std::min(grid, T) & ~7 ? std::min(grid, T) & ~7 : std::min(grid, T);
  hipLaunchKernelGGL(gemm_h3p_kernel, dim3(g), dim3(1024), 0, st, a);
  return hipGetLastError();
}

}  // namespace lg
