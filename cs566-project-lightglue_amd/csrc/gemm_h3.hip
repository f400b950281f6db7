// fp16x3 "linear" GEMM on plane images (PREC_H3), gfx950 LDS-DMA pipeline.
//
//   Y[r, c] = epilogue( (sum_k A[r, k] * W[c, k]) + bias[c] )      fp32-accurate (common.h)
//
// Replaces every nn.Linear of the LightGlue forward (reference lightglue.py) in the default
// operand format:
//   SelfBlock.Wqkv        :168,184   -> EPI_QKV_ROT  (+ rotary :36-43,187-188, head-major scatter :185-186)
//   CrossBlock.to_qk/to_v :203-204,223-228,235 -> EPI_CROSS_QKV (one GEMM, 512 outputs, qk * scale^0.5)
//   ffn.0 on cat([x,msg]) :172,191,247-248 -> EPI_STORE, A = [x | ctx] (the cat is never built;
//                                            out_proj / to_out folded in at load time)
//   ffn.3 + residual      :175,191   -> EPI_STORE with res, writing x in fp32 AND as a plane image
//   MatchAssignment.final_proj / d^.25 :304,308-310 -> EPI_STORE, out_scale 0.25
//   input_proj            :370-373,486-487 -> EPI_STORE (fp32 + plane image)
//
// Operands: A and W arrive as plane images -- the two fp16 pieces of the fp32 matrix, k-blocked
// by 32 and chunk-swizzled exactly like the LDS tile (common.h).  The producers write them (the
// previous GEMM's epilogue, the attention epilogue, the LayerNorm+GELU kernel; W at load time,
// pre-scaled by 2^sw), so this kernel does no conversion: every k-tile is four contiguous
// blocks (A h, A l, W h, W l) copied HBM/L2 -> LDS by global_load_lds_dwordx4 (1 KiB per
// wave-instruction, uniform base in SGPRs) into a ring of LDS stages, NSTAGE-1 k-tiles in
// flight.  The third piece of W (h * 2^11) is formed in registers (one packed fp16 multiply per
// fragment register), and the product is accumulated as three fp16 MFMAs per 32x32x16 block
// (common.h mfma_h3).
// Tile: BM x 256 x 32, BM/16 waves as (BM/64) x 4 of 64 x 64 (2 x 2 MFMA tiles each); at
// BM = 256, two 64 KiB stages fill 128 KiB of LDS, one workgroup per CU (tools/kbench_gemm.hip:
// 256 x 256 x 32 beat 128 x 256 at two workgroups per CU and every k-tile of 16 with 2-4
// stages).  blockIdx -> tile through a bijective XCD remap so the column tiles of one row panel
// share an XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace lg {

namespace {
constexpr int TB = 256;  // column tile; rows_pad granule

__device__ __forceinline__ int xcd_remap_h3(int id, int n, bool rev = false) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  const int cnt = base + (xcd < extra ? 1 : 0);
  return xcd * base + (xcd < extra ? xcd : extra) + (rev ? cnt - 1 - local : local);
}

__device__ __forceinline__ void head_row_base_h3(const HeadLayout& hl, int row, int& base, int& stride) {
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
}  // namespace

#ifndef LG_LN_PROBE
#define LG_LN_PROBE 0  // timing probes of the LN epilogue (tools/kbench_gemm.hip only): 1 no GELU, 2 no stores
#endif
#ifndef LG_GEMM_DIAG
// timing probes of the k-loop (tools/kbench_gemm.hip only; results are wrong under 1, 2, 4):
// 1 every tile reads one of 8 row panels (L2-resident A), 2 no k-tile copies, 4 no vmcnt waits,
// 8 the copies issued by the first NW/4 waves only, 16 A pieces only, 32 W pieces only,
// 64 only the first NSTAGE k-tiles copied (later ones re-read them: realistic operands, no copy stream)
#define LG_GEMM_DIAG 0
#endif
#ifndef LG_GEMM_A_NT
// non-temporal A-operand copies (and residual reads) for operands of at least LG_NT_MIN_MB
// (gemm_h3): streamed once, they should not displace the weights and the attention's q/k/v in the
// Infinity Cache.  configs[2], same box: 1235 -> 1277 pairs/s for the single-column-tile GEMMs,
// +0.5 % more for QKV and cross QKV as well (three pairs, attention -0.7 %).  Ungated (every size)
// it cost the cache-resident SuperGlue / small-batch forwards
#define LG_GEMM_A_NT 1
#endif
#ifndef LG_GEMM_RES_NT
// non-temporal stores of the fp32 residual stream (ffn.3 with its residual): next read one layer
// later, after ~1.5 GB of other traffic; configs[2] +0.4 % same box (1263 -> 1268 pairs/s)
#define LG_GEMM_RES_NT 1
#endif
#ifndef LG_GEMM_SETPRIO
#define LG_GEMM_SETPRIO 0
#endif
#ifndef LG_GEMM_MF16
// MFMA shape: 1 = v_mfma_f32_16x16x32_f16 (one instruction per 32-k tile; on random operands the
// chip sustains ~1.2x the flop rate of the 32x32x16 shape, tools/probe_mfma_shape.hip),
// 0 = v_mfma_f32_32x32x16_f16
#define LG_GEMM_MF16 1
#endif

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// BN x BM tile of (BM/64) x (BN/WN) waves, each 64 x WN (2 x WN/32 MFMA tiles of 32 x 32).
// KS > 1 (single-wave tiles only): KS waves split the k-tiles of one tile, each with its own LDS
// ring and no barriers in the k-loop; the partial accumulators meet in LDS and wave 0 adds them
// in wave order and runs the epilogue alone (small row counts: KS times the waves in flight per
// tile, at the cost of a different rounding order from the KS = 1 kernels).
template <int EPI, int BM, int NSTAGE, int BN = TB, int WN = 64, int KS = 1>
__global__ __launch_bounds__((BM / 64) * (BN / WN) * 64 * KS) void gemm_h3_kernel(GemmH3Args g) {
  constexpr int WGN = BN / WN;               // waves along N
  constexpr int NW = (BM / 64) * WGN;        // waves of the tile (per k-split group)
  static_assert(KS == 1 || NW == 1, "split-k: single-wave tiles");
  constexpr int NJ = WN / 32;                // 32-column MFMA tiles per wave
  constexpr int BK = kKB;                    // k-tile = one k-block of the plane images (32)
  constexpr int APT = BM * BK * 2;           // one A plane tile (bytes)
  constexpr int WPT = BN * BK * 2;           // one W plane tile
  constexpr int STAGE_BYTES = 2 * APT + 2 * WPT;
  constexpr int PIECES = STAGE_BYTES / 1024; // 1 KiB LDS-DMA pieces per stage
  constexpr int PPW = PIECES / NW;
  static_assert(PIECES % NW == 0, "pieces per wave");
  constexpr int RING = NSTAGE * STAGE_BYTES;  // one k-split group's stages
  static_assert(KS == 1 || RING >= 64 * 64 * 4, "split-k: a partial accumulator fits the ring");
  __shared__ __attribute__((aligned(1024))) char smem[KS * RING];
  constexpr bool kQkv = EPI == EPI_QKV_ROT || EPI == EPI_CROSS_QKV;
  __shared__ int rowinfo[kQkv ? 2 * BM : 1];  // QKV epilogues: head-major base / stride per tile row

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ks = KS > 1 ? wave_all : 0;    // k-split group
  const int wave = KS > 1 ? 0 : wave_all;  // wave within the tile
  const int l32 = lane & 31, half = lane >> 5;
  const int wm0 = (wave / WGN) * 64, wn0 = (wave % WGN) * WN;

  // run-time range exponents of the A plane images (RangeOut): A0 holds a0 * 2^-e0, A1 a1 * 2^-e1
  const int e0 = range_slot_exp(g.rtab, g.a0_slot);
  const int e1 = g.K0 < g.K ? range_slot_exp(g.rtab, g.a1_slot) : e0;
  const float accs = ldexpf(g.acc_scale, e1);  // after the k-loop the accumulator holds 2^-e1 units
  // exponents of the planes this launch writes, read here so the loads are long done by the
  // epilogue (QKV: waves of a workgroup share one output type -- a 256-column tile is one of q/k/v)
  const int eo_main = range_exponent(g.ro);
  const int eo_v = (EPI == EPI_QKV_ROT || EPI == EPI_CROSS_QKV) ? range_exponent(g.ro_v) : 0;

  const int num_m = (g.R + BM - 1) / BM, num_n = g.Nout / BN;
  const int tile = xcd_remap_h3(blockIdx.x, num_m * num_n, g.reverse != 0);
  const int tm = tile / num_n, tn = tile - tm * num_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = g.K / BK, nk0 = g.K0 / BK;
  if (g.rm.cnt) {  // batched pruning: a tile without a live row does nothing (flag in the idle LDS)
    volatile int* fl = reinterpret_cast<volatile int*>(smem);
    if (threadIdx.x == 0) *fl = 0;
    __syncthreads();
    if (threadIdx.x < BM && m0 + (int)threadIdx.x < g.R && row_live(g.rm, m0 + threadIdx.x)) *fl = 1;
    __syncthreads();
    const bool any = *fl != 0;
    __syncthreads();  // read before the first LDS-DMA stage lands on it
    if (!any) return;
  }

  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem) + ks * RING;

  // k-tile kt of a plane image is one contiguous block per plane (the tile's rows of k-block kt),
  // already in the LDS tile's swizzled layout: staging is a straight copy.  The stage is cut into
  // 1 KiB pieces [A h | A l | W h | W l]; wave w copies pieces PPW*w .. PPW*w + PPW-1.
  const uint32_t voff = lane * 16;
  auto issue = [&](int kt, int stage) {
#if LG_GEMM_DIAG & 2
    return;
#endif
#if LG_GEMM_DIAG & 64
    if (kt >= NSTAGE) return;  // real data in every stage, later k-tiles re-read it (same MFMA power)
#endif
#if LG_GEMM_DIAG & 8
    constexpr int IW = NW / 4 > 0 ? NW / 4 : 1;  // issuing waves
    if (wave >= IW) return;
#pragma unroll
    for (int i = 0; i < PIECES / IW; ++i) {
      const int q = wave * (PIECES / IW) + i;
#else
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;  // wave-uniform
#endif
      const char* src;
#if LG_GEMM_DIAG & 16
      if (q >= 2 * (APT / 1024)) continue;  // A pieces only
#endif
#if LG_GEMM_DIAG & 32
      if (q < 2 * (APT / 1024)) continue;   // W pieces only
#endif
      if (q < 2 * (APT / 1024)) {
        const int pl = q / (APT / 1024), pc = q % (APT / 1024);
        const bool first = kt < nk0;
        const PlaneRef& A = first ? g.A0 : g.A1;
        const int kb = first ? kt : kt - nk0;
#if LG_GEMM_DIAG & 1
        const int am0 = m0 & 2047;
#else
        const int am0 = m0;
#endif
        src = reinterpret_cast<const char*>(A.p + pl * A.ps + ((size_t)kb * A.rows_pad + am0) * BK) + pc * 1024;
      } else {
        const int qw = q - 2 * (APT / 1024);
        const int pl = qw / (WPT / 1024), pc = qw % (WPT / 1024);
        src = reinterpret_cast<const char*>(g.W.p + pl * g.W.ps + ((size_t)kt * g.W.rows_pad + n0) * BK) + pc * 1024;
      }
#if LG_GEMM_A_NT
      // A too big to stay cached: its row panels are read by the column tiles of one XCD within
      // microseconds (L2) and never again -- stream them past the Infinity Cache
      if (g.stream && q < 2 * (APT / 1024))
        dma16_nt(src, voff, lds0 + stage * STAGE_BYTES + q * 1024);
      else
#endif
        dma16(src, voff, lds0 + stage * STAGE_BYTES + q * 1024);
    }
  };

  // wave tile 64 x WN as TI x TJ MFMA tiles of TR accumulator registers
  constexpr bool kMF16 = LG_GEMM_MF16 != 0;
  constexpr int TI = kMF16 ? 4 : 2, TJ = kMF16 ? WN / 16 : NJ, TR = kMF16 ? 4 : 16;
  using AccT = typename std::conditional<kMF16, f32x4, f32x16>::type;
  AccT acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = AccT{0.f};
  // visit(i, fn): every accumulator element of the wave tile's row pass i (rows 32i .. 32i+31),
  // as acc = fn(local row rr in [0,32), local column c in [0,WN), acc)
  auto visit = [&](int i, auto fn) {
    if constexpr (kMF16) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[2 * i + a][j][r] = fn(a * 16 + (lane >> 4) * 4 + r, j * 16 + (lane & 15), acc[2 * i + a][j][r]);
    } else {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = fn(row32(r, half), j * 32 + l32, acc[i][j][r]);
    }
  };

  // fragment (row r, 16-byte k-chunk c) of the plane tile at byte offset t0 of a stage
  auto frag = [&](const char* st, int t0, int r, int c) {
    return *reinterpret_cast<const f16x8*>(st + t0 + r * (BK * 2) + ((c ^ plane_swz(r)) << 4));
  };
  auto compute = [&](int stage) {
    const char* st = smem + ks * RING + stage * STAGE_BYTES;
    if constexpr (kMF16) {
      // lane: row (lane & 15) of each 16-row block, k chunk lane >> 4 (k = 8c .. 8c+7)
      const int c = lane >> 4, r16 = lane & 15;
      f16x8 ah[TI], al[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm0 + i * 16 + r16;
        ah[i] = frag(st, 0, r, c);
        al[i] = frag(st, APT, r, c);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn0 + j * 16 + r16;
        const f16x8 wh = frag(st, 2 * APT, r, c);
        const f16x8 wl = frag(st, 2 * APT + WPT, r, c);
        const f16x8 whs = wh * (_Float16)kLoScale;  // exact: |W_h| < 16
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma_h3_16(ah[i], al[i], whs, wl, wh, acc[i][j]);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = 2 * s + half;
      f16x8 ah[2], al[2], wh[NJ], wl[NJ], whs[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm0 + i * 32 + l32;
        ah[i] = frag(st, 0, r, c);
        al[i] = frag(st, APT, r, c);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wn0 + j * 32 + l32;
        wh[j] = frag(st, 2 * APT, r, c);
        wl[j] = frag(st, 2 * APT + WPT, r, c);
        whs[j] = wh[j] * (_Float16)kLoScale;  // exact: |W_h| < 16
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if constexpr (!kMF16) acc[i][j] = mfma_h3(ah[i], al[i], whs[j], wl[j], wh[j], acc[i][j]);
    }
  };

  // ring of NSTAGE stages, NSTAGE-1 k-tiles in flight; one barrier per k-tile: wait for my
  // copies of tile kt -> barrier (everyone's copies landed AND everyone is done reading stage
  // (kt-1) % NSTAGE) -> refill that stage with tile kt+NSTAGE-1 -> multiply tile kt
  // k-tiles kb .. ke-1 (the whole range unless split-k)
  const int kb = KS > 1 ? (ks * nk) / KS : 0, ke = KS > 1 ? ((ks + 1) * nk) / KS : nk;
  auto scale_acc = [&](float f) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < TR; ++r) acc[i][j][r] *= f;
  };
#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p)
    if (kb + p < ke) issue(kb + p, p);
  for (int kt = kb; kt < ke; ++kt) {
    const int ahead = min(NSTAGE - 2, ke - 1 - kt);  // my k-tiles in flight beyond kt
#if LG_GEMM_DIAG & 8
    wait_vm<0>();
#elif !(LG_GEMM_DIAG & 4)
    if (NSTAGE >= 4 && ahead >= 2) wait_vm<2 * PPW>();
    else if (NSTAGE >= 3 && ahead >= 1) wait_vm<PPW>();
    else wait_vm<0>();
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (KS == 1) __builtin_amdgcn_s_barrier();  // split-k groups are single waves
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < ke) issue(kt + NSTAGE - 1, (kt - kb + NSTAGE - 1) % NSTAGE);
    if (kt == nk0 && e0 != e1) scale_acc(ldexpf(1.f, e0 - e1));  // A0 -> A1 units (exact; rare)
#if LG_GEMM_SETPRIO
    __builtin_amdgcn_s_setprio(1);  // keeps the MFMA cluster between the barriers (guide T5)
#endif
    compute((kt - kb) % NSTAGE);
#if LG_GEMM_SETPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
  if (KS > 1 && ke <= nk0 && e0 != e1) scale_acc(ldexpf(1.f, e0 - e1));  // a partial of A0 k-tiles only
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // waves running the epilogue: split-k tiles give each group 16 rows of the tile (4 groups, 16 x 16
  // MFMA tiles) or 32 (2 groups); otherwise a wave runs both 32-row passes of its own tile
  constexpr int EW = KS > 1 ? (kMF16 && KS >= 4 ? 4 : 2) : NW;
  if constexpr (KS > 1) {
    // every group leaves its partial accumulator in the upper half of its (idle) ring, lane-major
    // (conflict-free); the lower half becomes its transpose buffer.  Each epilogue group then adds
    // up the partials of its own rows in group order, p0 + p1 + p2 + ..., the same order for every
    // row whichever group stores it; groups beyond EW leave (s_barrier waits only for surviving waves)
    static_assert(TI * TJ * TR == 64, "single-wave 64 x 64 tile");
    static_assert(RING >= 2 * 64 * 64 * 4, "split-k: partial + transpose buffer fit the ring");
    auto part = [&](int q) { return reinterpret_cast<float*>(smem + q * RING + RING / 2); };
    {
      float* pp = part(ks);
      int x = 0;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < TR; ++r, ++x) pp[x * 64 + lane] = acc[i][j][r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ks >= EW) return;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      if (EW == 4 ? i != ks : (i * 2 / TI) != ks) continue;  // MFMA row tiles this group stores
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < TR; ++r) {
          const int x = (i * TJ + j) * TR + r;
          float v = part(0)[x * 64 + lane];
#pragma unroll
          for (int q = 1; q < KS; ++q) v += part(q)[x * 64 + lane];
          acc[i][j][r] = v;
        }
    }
  }
  float* const ep_buf = KS > 1 ? reinterpret_cast<float*>(smem + ks * RING) : reinterpret_cast<float*>(smem) + wave * (32 * 64);
  // this wave's 32-row passes, and within a pass its 8-row store groups k (rows 8k .. 8k+7)
  auto my_pass = [&](int i) { return KS == 1 || (EW == 4 ? i == (ks >> 1) : i == ks); };
  auto my_rows = [&](int k) { return KS == 1 || EW != 4 || (k >> 1) == (ks & 1); };

  // ------------------------------------------------------------------ epilogues
  float wmax = 0.f;  // max |x| this lane wrote into planes (RangeOut tracking)
  if constexpr (EPI == EPI_PROBE) {
    // timing probe (tools/kbench_gemm.hip): keeps the accumulators live, stores nothing
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < TR; ++r) t += acc[i][j][r];
    if (t == 1234.5678f) g.Y[tid] = t;
  } else if constexpr (EPI == EPI_LN_GELU) {
    // ffn.0 + ffn.1 LayerNorm(512, eps 1e-5) + ffn.2 GELU(erf) (lightglue.py:171-176), fused: the
    // workgroup holds complete rows (BN = 512), so the row statistics are reduced in LDS (free
    // after the k-loop) and the activations leave only as the plane image ffn.3 consumes.
    static_assert(BN == 512 && (BM == 128 || BM == 64) && WN == 64, "LN epilogue tile");
    constexpr int NT = NW * 64;
    constexpr int PARTS = NT / BM;            // threads per row in the table reduction
    constexpr int LC = kMF16 ? 16 : 32;       // lanes sharing a row within a wave
    constexpr int RS = WGN * LC + 4;          // row stride of the partial-sum table (floats)
    constexpr int PW = WGN * LC / PARTS;      // partials summed per thread
    static_assert(PW % 4 == 0, "table reduction");
    constexpr int SCRATCH = NSTAGE * STAGE_BYTES / 4;  // floats
    // LDS (free after the k-loop): [partial table | ... | mean | rstd]; the per-wave transpose
    // buffers of the final stage overlay the table once the statistics are done
    float* red = reinterpret_cast<float*>(smem);           // [BM][RS] per-lane partials
    float* mean_s = red + SCRATCH - 2 * BM;                // [BM]
    float* rstd_s = mean_s + BM;                           // [BM]
    float* ep = red + wave * (32 * 64);                    // per-wave transpose buffer
    static_assert(BM * RS + 2 * BM <= SCRATCH && NW * 32 * 64 + 2 * BM <= SCRATCH, "epilogue scratch");
    // per-lane columns: j * LC + (lane % LC) of the wave tile
    const int lcol = kMF16 ? (lane & 15) : l32;
    float bj_[TJ], gj[TJ], bj[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn0 + j * LC + lcol;
      bj_[j] = g.bias ? g.bias[col] : 0.f;
      gj[j] = g.ln_g[col];
      bj[j] = g.ln_b[col];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      visit(i, [&](int, int c, float v) { return fmaf(v, accs, bj_[c / LC]); });
    // row sum of f(v) over the 512 columns: lane partials over its TJ columns -> table ->
    // PARTS threads per row -> shuffle
    auto row_total = [&](auto f, float* out) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < TR; ++r) {
          const int lr = wm0 + (kMF16 ? i * 16 + (lane >> 4) * 4 + r : i * 32 + row32(r, half));
          float p = 0.f;
#pragma unroll
          for (int j = 0; j < TJ; ++j) p += f(acc[i][j][r], lr);
          red[lr * RS + (wave % WGN) * LC + lcol] = p;
        }
      __syncthreads();
      const int row = tid / PARTS, part = tid % PARTS;
      const f32x4* src = reinterpret_cast<const f32x4*>(red + row * RS + part * PW);
      float s4 = 0.f;
#pragma unroll
      for (int q = 0; q < PW / 4; ++q) {
        const f32x4 v = src[q];
        s4 += (v[0] + v[1]) + (v[2] + v[3]);
      }
#pragma unroll
      for (int o = 1; o < PARTS; o <<= 1) s4 += __shfl_xor(s4, o, 64);
      if (part == 0) out[row] = s4;
      __syncthreads();
    };
    row_total([](float v, int) { return v; }, mean_s);
    if (tid < BM) mean_s[tid] *= (1.f / 512.f);
    __syncthreads();
    row_total([&](float v, int lr) { const float d = v - mean_s[lr]; return d * d; }, rstd_s);
    if (tid < BM) rstd_s[tid] = 1.f / sqrtf(rstd_s[tid] * (1.f / 512.f) + 1e-5f);
    __syncthreads();
    // normalise + GELU, then 16-byte plane-image stores through the per-wave transpose buffer
    const int cq = (lane & 7) * 8;
    const int eo = eo_main;
    const float so = ldexpf(1.f, -eo);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      constexpr int jh = 0;  // WN == 64: one 64-column pass per row pass
      if constexpr (kMF16 && !(LG_LN_PROBE & 1)) {
        // rows 4 (lane >> 4) + r, r = 0..3, of each 16-row block, column 16 j + (lane & 15): the
        // normalisation and GELU run on row pairs (r, r + 1) with packed fp32 arithmetic
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int rp = 0; rp < 4; rp += 2) {
            const int rr0 = a * 16 + (lane >> 4) * 4 + rp, lr0 = wm0 + i * 32 + rr0;
            const f32x2_ m2 = {mean_s[lr0], mean_s[lr0 + 1]}, s2 = {rstd_s[lr0], rstd_s[lr0 + 1]};
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
              const int c = j * 16 + (lane & 15);
              const f32x2_ v2 = {acc[2 * i + a][j][rp], acc[2 * i + a][j][rp + 1]};
              const f32x2_ z2 = gelu_erf2((v2 - m2) * s2 * gj[j] + bj[j]);
              ep[rr0 * 64 + (c ^ ((rr0 & 1) << 2))] = z2.x;
              ep[(rr0 + 1) * 64 + (c ^ (((rr0 + 1) & 1) << 2))] = z2.y;
            }
          }
      } else {
        visit(i, [&](int rr, int c, float v) {
          const int lr = wm0 + i * 32 + rr;
          const float y = (v - mean_s[lr]) * rstd_s[lr] * gj[c / LC] + bj[c / LC];
#if LG_LN_PROBE & 1
          ep[rr * 64 + (c ^ ((rr & 1) << 2))] = y;
#else
          ep[rr * 64 + (c ^ ((rr & 1) << 2))] = gelu_erf(y);
#endif
          return v;
        });
      }
      {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!my_rows(k)) continue;
          const int rr = (lane >> 3) + 8 * k;
          const int row = m0 + wm0 + i * 32 + rr;
          const int sw = (rr & 1) << 2;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
          if (!(LG_LN_PROBE & 2) && row < g.R && row_live(g.rm, row)) {
            f16x8 h, l;
            float vv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              vv[e] = e < 4 ? v0[e] : v1[e - 4];
              wmax = fmaxf(wmax, fabsf(vv[e]));
            }
            split2h_x8(vv, so, h, l);
            const size_t off = plane_off(row, n0 + wn0 + jh * 64 + cq, g.yrows_pad);
            st_stream(reinterpret_cast<f16x8*>(g.Yp + off), h);
            st_stream(reinterpret_cast<f16x8*>(g.Yp + g.yps + off), l);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass writes
      }
    }
    range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem), NW);
  } else if constexpr (EPI == EPI_STORE) {
    static_assert(WN == 64, "EPI_STORE tile");
    // Transposed through LDS (free after the k-loop; 8 KiB per wave per 32-row pass), LDS element
    // (r, c) of a pass at r*64 + (c ^ 4*(r&1)) (conflict-free ds_write_b32 rows, ds_read_b128 groups).
    // fp32 rows (Y, residual) are read and written as full 128-byte lines per 8 lanes: a lane owns
    // columns 4(lane&7) .. +3 and 32 + 4(lane&7) .. +3 (a 16-byte access at a 32-byte stride would
    // write half lines, which measured 2x the cost per byte); the finished values go back into the
    // LDS slots they came from and the plane pass re-reads them as 8 consecutive columns (one
    // 16-byte fp16 chunk per plane: consecutive rows of a k-block are contiguous).
    static_assert(KS > 1 || NW * 32 * 64 * 4 <= NSTAGE * STAGE_BYTES, "epilogue scratch");
    float* ep = ep_buf;
    const int cq = (lane & 7) * 8;  // plane pass: the lane's 8 columns (in the wave tile)
    const int c4 = (lane & 7) * 4;  // fp32 pass: columns c4 .. c4+3 and 32 + c4 ..
    const int eo = g.Yp ? eo_main : 0;
    const float so = ldexpf(1.f, -eo);
    const bool fp32_pass = g.Y || g.res || !g.Yp;
    f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
    if (g.bias) {
      const int ca = fp32_pass ? c4 : cq, cb = fp32_pass ? 32 + c4 : cq + 4;
      b0 = *reinterpret_cast<const f32x4*>(g.bias + n0 + wn0 + ca);
      b1 = *reinterpret_cast<const f32x4*>(g.bias + n0 + wn0 + cb);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (!my_pass(i)) continue;
      visit(i, [&](int rr, int c, float v) {
        ep[rr * 64 + (c ^ ((rr & 1) << 2))] = v;
        return v;
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (fp32_pass) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!my_rows(k)) continue;
          const int rr = (lane >> 3) + 8 * k;
          const int row = m0 + wm0 + i * 32 + rr;
          const int sw = (rr & 1) << 2;
          float* pa = ep + rr * 64 + (c4 ^ sw);
          float* pb = ep + rr * 64 + ((32 + c4) ^ sw);
          f32x4 v0 = *reinterpret_cast<const f32x4*>(pa);
          f32x4 v1 = *reinterpret_cast<const f32x4*>(pb);
          if (row < g.R && row_live(g.rm, row)) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v0[e] = fmaf(v0[e], accs, b0[e]) * g.out_scale;
              v1[e] = fmaf(v1[e], accs, b1[e]) * g.out_scale;
            }
            if (g.res) {
              const float* rp = (g.res2 && row >= g.res2_row0 ? g.res2 + (size_t)(row - g.res2_row0) * g.ldr
                                                              : g.res + (size_t)row * g.ldr) + n0 + wn0 + c4;
              f32x4 r0, r1;
              if (LG_GEMM_A_NT && g.stream) {
                r0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(rp));
                r1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(rp + 32));
              } else {
                r0 = *reinterpret_cast<const f32x4*>(rp);
                r1 = *reinterpret_cast<const f32x4*>(rp + 32);
              }
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v0[e] = r0[e] + v0[e];
                v1[e] = r1[e] + v1[e];
              }
            }
            if (g.relu)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v0[e] = fmaxf(v0[e], 0.f);
                v1[e] = fmaxf(v1[e], 0.f);
              }
            if (g.Y) {
              float* yp = (g.Y2 && row >= g.y2_row0 ? g.Y2 + (size_t)(row - g.y2_row0) * g.ldy : g.Y + (size_t)row * g.ldy) +
                          n0 + wn0 + c4;
#if LG_GEMM_RES_NT
              if (g.res && g.stream) {  // the residual stream: next read a layer later
                __builtin_nontemporal_store(v0, reinterpret_cast<f32x4*>(yp));
                __builtin_nontemporal_store(v1, reinterpret_cast<f32x4*>(yp + 32));
              } else
#endif
              {
                st_stream(reinterpret_cast<f32x4*>(yp), v0);
                st_stream(reinterpret_cast<f32x4*>(yp + 32), v1);
              }
            }
            if (g.Yp) {
              *reinterpret_cast<f32x4*>(pa) = v0;
              *reinterpret_cast<f32x4*>(pb) = v1;
            }
          }
        }
        if (g.Yp) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (g.Yp) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!my_rows(k)) continue;
          const int rr = (lane >> 3) + 8 * k;
          const int row = m0 + wm0 + i * 32 + rr;
          const int sw = (rr & 1) << 2;
          f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
          f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
          if (row < g.R && row_live(g.rm, row)) {
            if (!fp32_pass) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v0[e] = fmaf(v0[e], accs, b0[e]) * g.out_scale;
                v1[e] = fmaf(v1[e], accs, b1[e]) * g.out_scale;
                if (g.relu) {
                  v0[e] = fmaxf(v0[e], 0.f);
                  v1[e] = fmaxf(v1[e], 0.f);
                }
              }
            }
            f16x8 h, l;
            float vv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              vv[e] = e < 4 ? v0[e] : v1[e - 4];
              wmax = fmaxf(wmax, fabsf(vv[e]));
            }
            split2h_x8(vv, so, h, l);
            const size_t off = plane_off(row, n0 + wn0 + cq, g.yrows_pad);
            st_stream(reinterpret_cast<f16x8*>(g.Yp + off), h);
            st_stream(reinterpret_cast<f16x8*>(g.Yp + g.yps + off), l);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass writes
    }
    if (g.Yp) range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem), EW);
  } else {
    static_assert(WN == 64, "QKV epilogue tile");
    // Head-major scatter through the same LDS transpose as EPI_STORE.  The wave's 64 columns are
    // one (type t, head) block; GEMM column c holds dim 2c (c < 32) or 2(c - 32) + 1 (c >= 32) (the
    // load-time Wqkv row order puts rotary partners in one lane of the MFMA tile).  Written into
    // LDS at their natural dim, each lane then owns whole rotary pairs of one row.
    //   self  (EPI_QKV_ROT):   t0 -> q fp32 (rotary), t1 -> k planes (rotary), t2 -> v planes
    //   cross (EPI_CROSS_QKV): t0 -> qk planes * scale^0.5 (+ fp32 rows when hl.q is set), t1 -> v planes
    //   (the attention reads the cross queries from the qk planes: attention_f32's q_planes)
    const HeadLayout& hl = g.hl;
    for (int r = tid; r < BM; r += BM * 4) {
      int base = 0, stride = 0;
      if (m0 + r < g.R) head_row_base_h3(hl, m0 + r, base, stride);
      rowinfo[2 * r] = base;
      rowinfo[2 * r + 1] = stride;
    }
    __syncthreads();
    const int cbase = n0 + wn0;
    const int t = cbase / kDim, head = (cbase % kDim) / kHeadDim;
    const bool rot = EPI == EPI_QKV_ROT && t < 2 && hl.cosb;  // no cos table: plain q/k/v (SuperGlue)
    const bool to_q = t == 0 && hl.q;
    const bool to_kp = EPI == EPI_QKV_ROT ? t == 1 : t == 0;
    const bool to_vp = EPI == EPI_QKV_ROT ? t == 2 : t == 1;
    const float sc = (EPI == EPI_CROSS_QKV && t == 0) ? hl.qk_scale : 1.f;
    const int eo = to_kp ? eo_main : to_vp ? eo_v : 0;
    const float so = ldexpf(1.f, -eo);
    float* ep = ep_buf;
    // fp32 rows (q, qk) go out as full 128-byte lines per 8 lanes (lane dims c4 .. c4+3 and
    // 32 + c4 ..: two rotary pairs each); plane rows as one 16-byte chunk per lane (dims d0 ..
    // d0+7).  qk (cross) needs both: the fp32 pass puts its finished values back into LDS and the
    // plane pass re-reads them.
    const bool qpass = to_q, ppass = to_kp || to_vp;
    const int d0 = (lane & 7) * 8, c4 = (lane & 7) * 4;
    auto dimA = [&](int e) { return e < 4 ? c4 + e : 32 + c4 + (e - 4); };
    float bA[8], bB[8];  // bias in dim order: dim d <- GEMM column (d & 1) * 32 + d / 2
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bA[e] = qpass ? g.bias[cbase + (dimA(e) & 1) * 32 + (dimA(e) >> 1)] : 0.f;
      bB[e] = ppass && !qpass ? g.bias[cbase + ((d0 + e) & 1) * 32 + ((d0 + e) >> 1)] : 0.f;
    }
    // t*cos + rotate_half(t)*sin, rotate_half(x)[2p] = -x[2p+1], [2p+1] = x[2p]; freq p = dim / 2
    auto rotate = [&](float* x, const float* cs, const float* sn) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float xe = x[2 * p], xo = x[2 * p + 1];
        x[2 * p] = add_rn(mul_rn(xe, cs[p]), mul_rn(-xo, sn[p]));
        x[2 * p + 1] = add_rn(mul_rn(xo, cs[p]), mul_rn(xe, sn[p]));
      }
    };
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (!my_pass(i)) continue;
      visit(i, [&](int rr, int c, float v) {
        const int dim = c < 32 ? 2 * c : 2 * (c - 32) + 1;
        ep[rr * 64 + (dim ^ ((rr & 1) << 2))] = v;
        return v;
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (qpass) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!my_rows(k)) continue;
          const int rr = (lane >> 3) + 8 * k;
          const int lr = wm0 + i * 32 + rr;
          const int row = m0 + lr;
          const int sw = (rr & 1) << 2;
          float* pa = ep + rr * 64 + (c4 ^ sw);
          float* pb = ep + rr * 64 + ((32 + c4) ^ sw);
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(pa);
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(pb);
          if (row >= g.R || !row_live(g.rm, row)) continue;
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = fmaf(e < 4 ? v0[e] : v1[e - 4], accs, bA[e]);
          if (rot) {
            const float* cr = hl.cosb + (size_t)row * kFreq;
            const float* sr = hl.sinb + (size_t)row * kFreq;
            const f32x2 ca = *reinterpret_cast<const f32x2*>(cr + c4 / 2), cb = *reinterpret_cast<const f32x2*>(cr + 16 + c4 / 2);
            const f32x2 sa = *reinterpret_cast<const f32x2*>(sr + c4 / 2), sb = *reinterpret_cast<const f32x2*>(sr + 16 + c4 / 2);
            const float cs[4] = {ca[0], ca[1], cb[0], cb[1]}, sn[4] = {sa[0], sa[1], sb[0], sb[1]};
            rotate(x, cs, sn);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] *= sc;
          const size_t off = (size_t)rowinfo[2 * lr] + (size_t)head * rowinfo[2 * lr + 1] + c4;
          st_stream(reinterpret_cast<f32x4*>(hl.q + off), f32x4{x[0], x[1], x[2], x[3]});
          st_stream(reinterpret_cast<f32x4*>(hl.q + off + 32), f32x4{x[4], x[5], x[6], x[7]});
          if (ppass) {
            *reinterpret_cast<f32x4*>(pa) = f32x4{x[0], x[1], x[2], x[3]};
            *reinterpret_cast<f32x4*>(pb) = f32x4{x[4], x[5], x[6], x[7]};
          }
        }
        if (ppass) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (ppass) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!my_rows(k)) continue;
          const int rr = (lane >> 3) + 8 * k;
          const int lr = wm0 + i * 32 + rr;
          const int row = m0 + lr;
          const int sw = (rr & 1) << 2;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (d0 ^ sw));
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((d0 + 4) ^ sw));
          if (row >= g.R || !row_live(g.rm, row)) continue;
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = e < 4 ? v0[e] : v1[e - 4];
          if (!qpass) {
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = fmaf(x[e], accs, bB[e]);
            if (rot) {
              const f32x4 c4v = *reinterpret_cast<const f32x4*>(hl.cosb + (size_t)row * kFreq + d0 / 2);
              const f32x4 s4v = *reinterpret_cast<const f32x4*>(hl.sinb + (size_t)row * kFreq + d0 / 2);
              const float cs[4] = {c4v[0], c4v[1], c4v[2], c4v[3]}, sn[4] = {s4v[0], s4v[1], s4v[2], s4v[3]};
              rotate(x, cs, sn);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] *= sc;
          }
          const size_t off = (size_t)rowinfo[2 * lr] + (size_t)head * rowinfo[2 * lr + 1] + d0;
          _Float16* base = static_cast<_Float16*>(to_kp ? hl.kp : hl.vp);
          f16x8 h, l;
#pragma unroll
          for (int e = 0; e < 8; ++e) wmax = fmaxf(wmax, fabsf(x[e]));
          if (to_vp) split2h_x8<true>(x, so, h, l);  // value planes: unscaled low piece (kernels.h HeadLayout)
          else split2h_x8(x, so, h, l);
          st_stream(reinterpret_cast<f16x8*>(base + off), h);
          st_stream(reinterpret_cast<f16x8*>(base + hl.pstride + off), l);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass writes
    }
    if (to_kp) range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem), EW);
    else if (to_vp) range_commit_lds(g.ro_v, wmax, eo, reinterpret_cast<float*>(smem), EW);
  }
}

template <int BM, int NSTAGE, int BN = TB, int WN = 64, int KS = 1>
hipError_t gemm_h3_launch(const GemmH3Args& a, int epi, hipStream_t st) {
  const int blocks = ((a.R + BM - 1) / BM) * (a.Nout / BN);
  const dim3 grid(blocks), block((BM / 64) * (BN / WN) * 64 * KS);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_h3_kernel<EPI_STORE, BM, NSTAGE, BN, WN, KS>), grid, block, 0, st, a); break;
    case EPI_QKV_ROT: hipLaunchKernelGGL((gemm_h3_kernel<EPI_QKV_ROT, BM, NSTAGE, BN, WN, KS>), grid, block, 0, st, a); break;
    case EPI_CROSS_QKV:
      hipLaunchKernelGGL((gemm_h3_kernel<EPI_CROSS_QKV, BM, NSTAGE, BN, WN, KS>), grid, block, 0, st, a);
      break;
    case EPI_PROBE: hipLaunchKernelGGL((gemm_h3_kernel<EPI_PROBE, BM, NSTAGE, BN, WN, KS>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#ifndef LG_GEMM_LN_WN
#define LG_GEMM_LN_WN 64  // wave tile width: 64 -> 16 waves of 64 x 64, 128 -> 8 waves of 64 x 128
#endif
// ffn.0 + LayerNorm + GELU (EPI_LN_GELU): 128 x 512 tiles, two 80 KiB stages (BM = 64: 64 x 512
// tiles, two 72 KiB stages -- small row counts)
template <int WN, int BM = 128>
hipError_t gemm_h3_ln_launch(const GemmH3Args& a, hipStream_t st) {
  const dim3 grid((a.R + BM - 1) / BM), block((BM / 64) * (512 / WN) * 64);
  hipLaunchKernelGGL((gemm_h3_kernel<EPI_LN_GELU, BM, 2, 512, WN>), grid, block, 0, st, a);
  return hipGetLastError();
}

// Tile choice.  The 256 x 256 (16-wave) tile is the throughput shape; when it would leave CUs
// idle (fewer tiles than CUs) the 128 x 128 four-wave tile (two workgroups per CU) keeps the MFMA
// density while quadrupling the tile count (SuperGlue's B = 16, N = 1024 row space), and when even
// that leaves most CUs idle (B = 1 forwards, pruned token sets) the 64 x 64 single-wave tile
// spreads the work over 16x more workgroups.  LG_GEMM_TILE=big|medium|small overrides the choice
// (tests run each on the golden cases).
enum { TILE_AUTO, TILE_BIG, TILE_SMALL, TILE_MEDIUM };
static int gemm_tile_override() {
  const char* e = getenv("LG_GEMM_TILE");
  if (!e) return TILE_AUTO;
  if (!strcmp(e, "big")) return TILE_BIG;
  if (!strcmp(e, "small")) return TILE_SMALL;
  if (!strcmp(e, "medium")) return TILE_MEDIUM;
  return TILE_AUTO;
}
static bool use_small_tiles(long long big_tiles) {
  const int o = gemm_tile_override();
  return o == TILE_SMALL || (o == TILE_AUTO && big_tiles < 256);
}
static int gemm_tile_for(long long big_tiles) {
  const int o = gemm_tile_override();
  if (o != TILE_AUTO) return o;
  if (big_tiles >= 256) return TILE_BIG;
  return 4 * big_tiles >= 512 ? TILE_MEDIUM : TILE_SMALL;  // 128 x 128: two workgroups per CU
}

#ifndef LG_GEMM_H3_TILE
// BM (rows per workgroup; 4*BM threads), LDS stages -- tools/kbench_gemm.hip
#define LG_GEMM_H3_TILE 256, 2
#endif

// ffn.0 + LN + GELU at small row counts: even 64 x 512 tiles leave most CUs idle, so the caller
// runs ffn.0 as a 64 x 64-tile EPI_STORE GEMM and LayerNorm + GELU as a row kernel
// (layernorm_gelu_512, which writes the same plane image)
bool gemm_h3_ln_split(int R) { return use_small_tiles((R + 127) / 128) && gemm_tile_override() != TILE_BIG; }

// Streamed-once hints (LG_GEMM_A_NT / LG_GEMM_RES_NT) only for operands too big to stay cached:
// A at least LG_NT_MIN_MB (default 128) MiB.  Smaller working sets (SuperGlue's 32k rows, pruned
// tails) live in the 256 MiB Infinity Cache from one kernel to the next.
static size_t nt_min_bytes() {
  const char* e = getenv("LG_NT_MIN_MB");
  return (size_t)(e ? atof(e) : 128.0) << 20;
}

// QKV projections (3 / 2 column tiles per row panel, the tiles of a panel run together on one
// XCD and share A through its L2): LG_QKV_A_NT=0 reads their A with the default cache policy
static bool qkv_a_nt() {
  static const int v = [] { const char* e = getenv("LG_QKV_A_NT"); return e ? atoi(e) : 1; }();
  return v != 0;
}

hipError_t gemm_h3(const GemmH3Args& a_in, int epi, hipStream_t st) {
  GemmH3Args a = a_in;
  a.stream = LG_GEMM_A_NT && (size_t)a.R * a.K * 4 >= nt_min_bytes();
  if ((epi == EPI_QKV_ROT || epi == EPI_CROSS_QKV) && !qkv_a_nt()) a.stream = false;
  if (a.R <= 0) return hipSuccess;
  if (a.Nout % TB || a.K % kKB || a.K0 % kKB || a.K0 <= 0 || a.K0 > a.K || (a.K0 < a.K && !a.A1.p) || !a.A0.p ||
      !a.W.p || a.A0.rows_pad < ((a.R + TB - 1) / TB) * TB || (a.K0 < a.K && a.A1.rows_pad < ((a.R + TB - 1) / TB) * TB) ||
      a.W.rows_pad != a.Nout || (a.Yp && a.yrows_pad < a.R))
    return hipErrorInvalidValue;
  if (epi == EPI_LN_GELU) {
    if (a.Nout != 512 || !a.Yp || !a.ln_g || !a.ln_b || a.yrows_pad < a.R) return hipErrorInvalidValue;
    if (use_small_tiles((a.R + 127) / 128)) return gemm_h3_ln_launch<64, 64>(a, st);
    return gemm_h3_ln_launch<LG_GEMM_LN_WN>(a, st);
  }
  switch (gemm_tile_for((long long)((a.R + TB - 1) / TB) * (a.Nout / TB))) {
    case TILE_SMALL: {
      // 64 x 64 single-wave tiles (fewer than 128 big tiles: at most 2048 of them), the k-tiles
      // split over 4 waves so that each CU runs 4 waves instead of one or two.  The split does not
      // depend on the row count, so every small-tile launch of one shape rounds alike whatever
      // the batch (LG_GEMM_KSPLIT=1|2|4 overrides)
      int ksplit = 4;
      if (const char* e = getenv("LG_GEMM_KSPLIT")) ksplit = atoi(e);
      if (ksplit >= 4 && a.K >= 4 * kKB) return gemm_h3_launch<64, 2, 64, 64, 4>(a, epi, st);
      if (ksplit >= 2 && a.K >= 2 * kKB) return gemm_h3_launch<64, 4, 64, 64, 2>(a, epi, st);
      return gemm_h3_launch<64, 4, 64, 64>(a, epi, st);
    }
    case TILE_MEDIUM: return gemm_h3_launch<128, 2, 128, 64>(a, epi, st);
    default: return gemm_h3_launch<LG_GEMM_H3_TILE>(a, epi, st);
  }
}

// fp32 rows -> plane image (scaled by 2^-E, RangeOut); one thread per 8-element chunk
// (xc != nullptr: the fp32 rows are also copied to xc, row stride K -- the residual stream's
// initial value taken in the same read)
__global__ void rows_to_planes_kernel(const float* x, int R, int K, int ld, _Float16* planes, int rows_pad, int row0,
                                      RangeOut ro, float* xc, RowMask rm) {
  const int nch = K / 8;
  const int eo = range_exponent(ro);
  const float so = ldexpf(1.f, -eo);
  float wmax = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)R * nch; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / nch), c = (int)(i % nch);
    if (!row_live(rm, row0 + r)) continue;  // dead rows of a pruned batch: stale data, not tracked
    const float* p = x + (size_t)r * ld + c * 8;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(p), v1 = *reinterpret_cast<const f32x4*>(p + 4);
    if (xc) {
      float* q = xc + (size_t)r * K + c * 8;
      *reinterpret_cast<f32x4*>(q) = v0;
      *reinterpret_cast<f32x4*>(q + 4) = v1;
    }
    f16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = e < 4 ? v0[e] : v1[e - 4];
      wmax = fmaxf(wmax, fabsf(v));
      _Float16 a, b;
      split2h(v * so, a, b);
      h[e] = a;
      l[e] = b;
    }
    const size_t off = plane_off(row0 + r, c * 8, rows_pad);
    *reinterpret_cast<f16x8*>(planes + off) = h;
    *reinterpret_cast<f16x8*>(planes + (size_t)rows_pad * K + off) = l;
  }
  range_commit(ro, wmax, eo);
}

hipError_t rows_to_planes(const float* x, int R, int K, int ld, _Float16* planes, int rows_pad, int row0,
                          const RangeOut& ro, hipStream_t st, float* xcopy, const RowMask* rm) {
  if (R <= 0) return hipSuccess;
  if (K % kKB || rows_pad < row0 + R) return hipErrorInvalidValue;
  const size_t n = (size_t)R * (K / 8);
  hipLaunchKernelGGL(rows_to_planes_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 2048)), dim3(256), 0, st, x, R, K, ld, planes,
                     rows_pad, row0, ro, xcopy, rm ? *rm : RowMask{});
  return hipGetLastError();
}

// rows_to_planes of two row sources in one launch: rows row0 .. row0+r0-1 from x0, then r1 rows
// from x1 (no fp32 copy, no row mask); element for element the values of two rows_to_planes calls
__global__ void rows_to_planes2_kernel(const float* x0, int r0, const float* x1, int r1, int K, int ld,
                                       _Float16* planes, int rows_pad, int row0, RangeOut ro) {
  const int nch = K / 8;
  const int eo = range_exponent(ro);
  const float so = ldexpf(1.f, -eo);
  float wmax = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)(r0 + r1) * nch;
       i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / nch), c = (int)(i % nch);
    const float* p = (r < r0 ? x0 + (size_t)r * ld : x1 + (size_t)(r - r0) * ld) + c * 8;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(p), v1 = *reinterpret_cast<const f32x4*>(p + 4);
    f16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = e < 4 ? v0[e] : v1[e - 4];
      wmax = fmaxf(wmax, fabsf(v));
      _Float16 a, b;
      split2h(v * so, a, b);
      h[e] = a;
      l[e] = b;
    }
    const size_t off = plane_off(row0 + r, c * 8, rows_pad);
    *reinterpret_cast<f16x8*>(planes + off) = h;
    *reinterpret_cast<f16x8*>(planes + (size_t)rows_pad * K + off) = l;
  }
  range_commit(ro, wmax, eo);
}

hipError_t rows_to_planes2(const float* x0, int r0, const float* x1, int r1, int K, int ld, _Float16* planes,
                           int rows_pad, int row0, const RangeOut& ro, hipStream_t st) {
  if (r0 + r1 <= 0) return hipSuccess;
  if (K % kKB || rows_pad < row0 + r0 + r1) return hipErrorInvalidValue;
  const size_t n = (size_t)(r0 + r1) * (K / 8);
  hipLaunchKernelGGL(rows_to_planes2_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 2048)), dim3(256), 0, st,
                     x0, r0, x1, r1, K, ld, planes, rows_pad, row0, ro);
  return hipGetLastError();
}

}  // namespace lg

namespace lg {
// max |x| -> M[slot] of a range table (the inputs' bound for the first plane images)
__global__ void range_absmax_kernel(const float* x, size_t n, unsigned* tab, int slot) {
  float m = 0.f;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {  // 16-byte loads over the aligned body
    const size_t n4 = n / 4;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    for (size_t i = t0; i < n4; i += stride) {
      const f32x4 v = x4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    for (size_t i = n4 * 4 + t0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  } else {
    for (size_t i = t0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  }
  range_commit(RangeOut{tab, -1, -1, 0.f, 0.f, 0.f, slot, 1}, m, 0);
}

hipError_t range_absmax(const float* x, size_t n, unsigned* tab, int slot, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n / 4 + 255) / 256 + 1, 1024);
  hipLaunchKernelGGL(range_absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, tab, slot);
  return hipGetLastError();
}

// max |x| over two arrays (both images' descriptors) -> M[slot] in one launch, eight 16-byte loads
// in flight per thread (the one-array kernel above keeps one: 67 MB in ~30 us, 2.2 TB/s); the
// maximum is order-independent, so the slot holds the same value as two range_absmax calls
__global__ __launch_bounds__(256) void range_absmax2_kernel(const float* x0, size_t n0, const float* x1, size_t n1,
                                                            unsigned* tab, int slot) {
  float m = 0.f;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  auto am4 = [](const f32x4& v) { return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))); };
  auto body = [&](const float* x, size_t n) {
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
      const size_t n4 = n / 4;
      const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
      size_t i = t0;
      for (; i + 7 * stride < n4; i += 8 * stride) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = x4[i + u * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) m = fmaxf(m, am4(v[u]));
      }
      for (; i < n4; i += stride) m = fmaxf(m, am4(x4[i]));
      for (size_t j = n4 * 4 + t0; j < n; j += stride) m = fmaxf(m, fabsf(x[j]));
    } else {
      for (size_t j = t0; j < n; j += stride) m = fmaxf(m, fabsf(x[j]));
    }
  };
  body(x0, n0);
  body(x1, n1);
  range_commit(RangeOut{tab, -1, -1, 0.f, 0.f, 0.f, slot, 1}, m, 0);
}

hipError_t range_absmax2(const float* x0, size_t n0, const float* x1, size_t n1, unsigned* tab, int slot,
                         hipStream_t st) {
  if (n0 + n1 == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>(((n0 + n1) / 4 + 255) / 256 + 1, 1024);
  hipLaunchKernelGGL(range_absmax2_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x0, n0, x1, n1, tab, slot);
  return hipGetLastError();
}
}  // namespace lg
