// SuperPoint extractor on gfx950 (reference gluefactory_nonfree/superpoint.py, SuperPoint._forward
// :202-350 and the helpers it calls, :60-149).
//
//   image --gray+conv1a (VALU, fp32)--> planes --3x3 implicit fp16x3 GEMMs (ReLU, fused 2x2 pool)-->
//   conv4b planes --[convPa | convDa] one GEMM--> planes --1x1 GEMMs (gemm_h3)--> logits / dense
//   descriptors --softmax+unfold / L2 norm--> dense scores / NHWC descriptors
//   scores --5 separable max-pool passes (simple_nms)--> mask --borders, threshold, row-major
//   compaction--> candidates --radix select + bitonic sort (top-k)--> keypoints --bilinear
//   sampling + L2 norm--> descriptors
//
// Feature maps are NHWC plane images (common.h): a 3x3 convolution is a GEMM with K = 9 Cin whose
// A tile for tap (ky, kx) is the input image shifted by (ky-1, kx-1) -- gathered row by row by
// LDS-DMA with per-lane source addresses (taps outside the image read a zero row), so there is no
// im2col buffer.  Convolutions followed by a 2x2 max-pool enumerate their output pixels in quad
// order (the four pixels of a pooling window are consecutive GEMM rows = the four accumulator
// registers of one lane of a 16x16 MFMA tile): the pool is a max over one lane's registers and
// only the pooled map is written.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"

namespace lg {

namespace {
__device__ __forceinline__ int sp_xcd_remap(int id, int n) {
  const int xcd = id & 7, local = id >> 3;
  const int base = n >> 3, extra = n & 7;
  return xcd * base + (xcd < extra ? xcd : extra) + local;
}
template <int N>
__device__ __forceinline__ void sp_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// float -> unsigned with the same order (larger key <=> larger value)
__device__ __forceinline__ unsigned order_key(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_value(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
unsigned grid_for(long long n, int block, int cap = 8192) {
  return (unsigned)std::max<long long>(1, std::min<long long>((n + block - 1) / block, cap));
}
}  // namespace

// ---- gray + conv1a -------------------------------------------------------------------------
// superpoint.py:204-209.  Four threads per pixel (thread c of a pixel owns the 16-byte chunk c of
// both 32-channel blocks, channels 8c..8c+7 and 32+8c..32+8c+7): the 3x3 gray neighbourhood
// (zero padded) in registers -> ReLU -> fp16x3 planes.  A wave's store covers 16 consecutive
// 64-byte rows = 1 KiB contiguous (one thread per pixel with 16-byte stores at a 64-byte stride
// wrote each line in four partial pieces and ran at half the store rate).
__global__ __launch_bounds__(256) void sp_conv1a_kernel(const float* __restrict__ img, int B, int C, int H, int W,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        _Float16* Y, int yrows_pad, RangeOut ro) {
  __shared__ float wsh[64 * 9 + 64];
  for (int i = threadIdx.x; i < 64 * 9 + 64; i += blockDim.x) wsh[i] = i < 64 * 9 ? w[i] : bias[i - 64 * 9];
  __syncthreads();
  const int eo = range_exponent(ro);
  const float so = ldexpf(1.f, -eo);
  const long long yps = (long long)yrows_pad * 64;
  float wmax = 0.f;
  const long long HW = (long long)H * W, total = (long long)B * HW * 4;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long p = t >> 2;
    const int c = (int)(t & 3);
    const int n = (int)(p / HW);
    const int rem = (int)(p - (long long)n * HW);
    const int y = rem / W, x = rem - y * W;
    float g[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
      float v = 0.f;
      if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
        const size_t o = (size_t)yy * W + xx;
        if (C == 3) {  // (image * [0.299, 0.587, 0.114]).sum(1)
          const float* q = img + (size_t)n * 3 * HW + o;
          v = add_rn(add_rn(mul_rn(q[0], 0.299f), mul_rn(q[HW], 0.587f)), mul_rn(q[2 * HW], 0.114f));
        } else {
          v = img[(size_t)n * HW + o];
        }
      }
      g[k] = v;
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f16x8 h, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = kb * 32 + c * 8 + e;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) a = fmaf(wsh[co * 9 + k], g[k], a);
        const float v = fmaxf(a + wsh[64 * 9 + co], 0.f);
        wmax = fmaxf(wmax, v);
        _Float16 hh, ll;
        split2h(v * so, hh, ll);
        h[e] = hh;
        l[e] = ll;
      }
      const size_t off = plane_off((int)p, kb * 32 + c * 8, yrows_pad);
      *reinterpret_cast<f16x8*>(Y + off) = h;
      *reinterpret_cast<f16x8*>(Y + yps + off) = l;
    }
  }
  range_commit(ro, wmax, eo);
}

hipError_t sp_conv1a(const float* image, int B, int C, int H, int W, const float* w, const float* bias, _Float16* Y,
                     int yrows_pad, const RangeOut& ro, hipStream_t st) {
  if (B <= 0 || H <= 0 || W <= 0) return hipSuccess;
  if ((C != 1 && C != 3) || (long long)yrows_pad < (long long)B * H * W) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sp_conv1a_kernel, dim3(grid_for(4LL * B * H * W, 256, 8192)), dim3(256), 0, st, image, B, C,
                     H, W, w, bias, Y, yrows_pad, ro);
  return hipGetLastError();
}

// ---- 3x3 convolution as an implicit fp16x3 GEMM ---------------------------------------------
// Tile 256 (pixels) x BN (channels) x 32 (k), (BN/64)*4 waves of 64 x 64 (16x16x32 MFMAs, three
// per product as in gemm_h3.hip), NSTAGE LDS stages.  k-tile kt = (tap, 32-channel block).
// BN = 128 (8 waves, 2 per SIMD, no spills) for Cout % 128 == 0, else 64; a 256-wide tile would
// need 16 waves at 128 VGPRs and spills its gather state.
template <int BN, int NSTAGE, bool POOL>
__global__ __launch_bounds__(4 * (BN / 64) * 64) void sp_conv3x3_kernel(ConvH3Args g) {
  constexpr int BM = 256, BK = kKB;
  constexpr int WGN = BN / 64, NW = 4 * WGN;
  constexpr int APT = BM * BK * 2, WPT = BN * BK * 2;
  constexpr int STAGE_BYTES = 2 * APT + 2 * WPT;
  constexpr int PIECES = STAGE_BYTES / 1024, PPW = PIECES / NW;
  constexpr int AP = 2 * APT / 1024;  // A pieces per stage (16 rows of one plane each)
  static_assert(PIECES % NW == 0, "pieces per wave");
  static_assert(NW * 32 * 64 * 4 <= NSTAGE * STAGE_BYTES, "epilogue scratch");
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WGN) * 64, wn0 = (wave % WGN) * 64;
  const int H = g.H, W = g.W, Hp = H >> 1, Wp = W >> 1;
  const int R = POOL ? 4 * g.B * Hp * Wp : g.B * H * W;
  const int num_m = (R + BM - 1) / BM, num_n = g.Cout / BN;
  const int tile = sp_xcd_remap(blockIdx.x, num_m * num_n);
  const int tm = tile / num_n, tn = tile - tm * num_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int CB = g.Cin / BK, nk = 9 * CB;
  const float accs = ldexpf(g.acc_scale, range_slot_exp(g.rtab, g.x_slot));
  const int eo = range_exponent(g.ro);
  const int zrow = g.X.rows_pad - 1;  // a zero row (caller keeps rows >= B*H*W zero)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem);

  // output pixel of the row each of this lane's A pieces gathers, and its input row
  int py[PPW], px[PPW], pr[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = wave * PPW + i;
    py[i] = -4;
    px[i] = -4;
    pr[i] = 0;
    if (q < AP) {
      const int m = m0 + (q % 16) * 16 + (lane >> 2);
      if (m < R) {
        int n, y, x;
        if (POOL) {
          const int quad = m >> 2, sub = m & 3;
          n = quad / (Hp * Wp);
          const int rem = quad - n * Hp * Wp;
          const int yp = rem / Wp;
          y = 2 * yp + (sub >> 1);
          x = 2 * (rem - yp * Wp) + (sub & 1);
        } else {
          n = m / (H * W);
          const int rem = m - n * H * W;
          y = rem / W;
          x = rem - y * W;
        }
        py[i] = y;
        px[i] = x;
        pr[i] = (n * H + y) * W + x;
      }
    }
  }

  auto issue = [&](int kt, int stage) {
    const int tap = kt / CB, cb = kt - tap * CB;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int dr = (ky - 1) * W + (kx - 1);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;  // wave-uniform
      if (q < AP) {
        const int pl = q / 16, rr = (q % 16) * 16 + (lane >> 2);
        const int yy = py[i] + ky - 1, xx = px[i] + kx - 1;
        const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const int rs = ok ? pr[i] + dr : zrow;
        const int c = (lane & 3) ^ plane_swz(rr);  // logical chunk of LDS slot lane & 3 of row rr
        const uint32_t voff = (uint32_t)rs * 64u + (uint32_t)((c ^ plane_swz(rs)) << 4);
        const char* base = reinterpret_cast<const char*>(g.X.p + pl * g.X.ps + (size_t)cb * g.X.rows_pad * BK);
        dma16(base, voff, lds0 + stage * STAGE_BYTES + q * 1024);
      } else {
        const int qw = q - AP;
        const int pl = qw / (WPT / 1024), pc = qw % (WPT / 1024);
        const char* src = reinterpret_cast<const char*>(g.Wt.p + pl * g.Wt.ps + ((size_t)kt * g.Wt.rows_pad + n0) * BK) + pc * 1024;
        dma16(src, lane * 16, lds0 + stage * STAGE_BYTES + q * 1024);
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto frag = [&](const char* st, int t0, int r, int c) {
    return *reinterpret_cast<const f16x8*>(st + t0 + r * (BK * 2) + ((c ^ plane_swz(r)) << 4));
  };
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
      const f16x8 whs = wh * (_Float16)kLoScale;  // exact: |W_h| < 16
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = mfma_h3_16(ah[i], al[i], whs, wl, wh, acc[i][j]);
    }
  };

#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NSTAGE - 2, nk - 1 - kt);
    if (NSTAGE >= 3 && ahead >= 1) sp_wait_vm<PPW>();
    else sp_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    compute(kt % NSTAGE);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // epilogue: bias + ReLU (+ pool) -> planes, 16-byte stores through a per-wave LDS transpose
  float* ep = reinterpret_cast<float*>(smem) + wave * (32 * 64);
  const int cq = (lane & 7) * 8;
  const int col0 = n0 + wn0 + cq;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.bias + col0);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.bias + col0 + 4);
  const float so = ldexpf(1.f, -eo);
  float wmax = 0.f;
  auto store8 = [&](int row, f32x4 v0, f32x4 v1) {
    f16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = fmaxf(fmaf(e < 4 ? v0[e] : v1[e - 4], accs, e < 4 ? b0[e] : b1[e - 4]), 0.f);
      wmax = fmaxf(wmax, v);
      _Float16 a, c;
      split2h(v * so, a, c);
      h[e] = a;
      l[e] = c;
    }
    const size_t off = plane_off(row, col0, g.yrows_pad);
    *reinterpret_cast<f16x8*>(g.Y + off) = h;
    *reinterpret_cast<f16x8*>(g.Y + g.yps + off) = l;
  };
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (!POOL) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = a * 16 + (lane >> 4) * 4 + r, c = j * 16 + (lane & 15);
            ep[rr * 64 + (c ^ ((rr & 1) << 2))] = acc[2 * i + a][j][r];
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rr = (lane >> 3) + 8 * k;
        const int row = m0 + wm0 + i * 32 + rr;
        const int sw = (rr & 1) << 2;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
        if (row < R) store8(row, v0, v1);
      }
    } else {
      // the 4 registers of a lane are the 4 pixels of one pooling window: relu(max + b) ==
      // max(relu(. + b)) (monotone, and rounding is monotone)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 v = acc[2 * i + a][j];
          const int pr_ = a * 4 + (lane >> 4), c = j * 16 + (lane & 15);
          ep[pr_ * 64 + (c ^ ((pr_ & 1) << 2))] = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int rr = lane >> 3;
      const int prow = (m0 + wm0 + i * 32) / 4 + rr;
      const int sw = (rr & 1) << 2;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
      if (prow < R / 4) store8(prow, v0, v1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass writes
  }
  range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem));
}

// ---- 3x3 convolution with a halo tile per channel block (the production form) -------------
// Output tile = 16 x 16 pixels of one image (GEMM rows in quad order, as above) x BN channels.
// Per 32-channel block the (16+2) x (16+2) input halo is gathered ONCE into LDS by LDS-DMA
// (384 rows x 64 B per plane; rows past 324 and taps outside the image read the zero row) and
// the nine taps read their A fragments from it at a shifted row (halo row (py + ky) * 18 + px + kx):
// per k-step the CU loads the BN x 32 weight tile plus 1/9 of a halo, ~3x less than re-gathering
// 256 shifted rows per tap.
// Persistent: one workgroup per CU walks its tiles (each XCD a contiguous range, so the tiles in
// flight on one L2 are neighbours), and the step sequence (tile, channel block, tap) runs through
// one pipeline: weights two steps ahead (ring of 3), the next halo -- next channel block or the
// next tile's first -- issued at tap 0 into the other of two halo buffers (nine steps of lead),
// so neither a tile's start nor a block boundary waits on HBM.  Waves of 32 x 64 (8 per 64
// channels: two or four waves per SIMD hide each other's LDS reads).  Measured and not kept:
// fragments read a step ahead into a second register set (4-deep weight ring) -- the compiler
// copies the set every step and conv1b ran 10 % slower.  The epilogue transposes through
// the halo buffer just consumed.  vmcnt waits count only the loads issued after the one needed
// (the LDS-DMA loads return in order; epilogue stores can only make a wait longer).
constexpr int kHT = 16, kHH = kHT + 2, kHRows = 384;
// Halo layout in LDS: pixel (y, x) of the 18 x 18 halo at layout row halo_row(y, x) (< 360), its
// 16-byte chunk c at slot halo_pos(x, c) of that row.  Chosen so the A-fragment reads are
// conflict-free for every tap: a ds_read_b128 lane group reads 8 consecutive pixels of two
// adjacent halo rows with two chunk values, and bank slot 4 * (row mod 4) + pos = (2x + (c & 1)
// + 8 (y & 1)) mod 16 (up to a per-group constant) is distinct over those 16 -- the linear
// layout (row 18 y + x) hit 3-way conflicts.  Rows: 20 per halo row, (x >> 1) + 2 (y & 1) fixes
// the row residue; x = 16, 17 use the spare slots of rows y and y +- 1.
__device__ __forceinline__ int halo_row(int y, int x) {
  const int a = x >> 1, b = x & 1, p = y & 1;
  if (x < 16) return 20 * y + 4 * (2 * (a >> 2) + b) + ((a + 2 * p) & 3);
  return 20 * (y + (b ? (p ? -1 : 1) : 0)) + 16 + 2 * p;
}
__device__ __forceinline__ int halo_pos(int x, int c) { return (2 * (x & 1) + (c & 1)) ^ (c & 2); }
// inverse: the pixel and chunk stored at (layout row lr, slot s); false for unused slots
__device__ __forceinline__ bool halo_inv(int lr, int s, int& y, int& x, int& c) {
  if (lr >= 20 * kHH) return false;
  const int y0 = lr / 20, off = lr - 20 * y0, k = off >> 2, r = off & 3, p = y0 & 1;
  if (k < 4) {
    y = y0;
    x = 2 * (4 * (k >> 1) + ((r - 2 * p) & 3)) + (k & 1);
  } else if (r == 2 * p) {
    y = y0;
    x = 16;
  } else if (r == 2 - 2 * p) {  // x = 17 of the neighbouring row
    y = p ? y0 - 1 : y0 + 1;
    x = 17;
  } else {
    return false;
  }
  c = 2 * (((s >> 1) ^ x) & 1) + (s & 1);
  return true;
}
template <int BN, bool POOL>
__global__ __launch_bounds__(8 * (BN / 64) * 64) void sp_conv3x3_halo_kernel(ConvH3Args g) {
  constexpr int BK = kKB, WGN = BN / 64, NW = 8 * WGN, WM = 32, WMT = WM / 16;
  constexpr int HALO_PLANE = kHRows * BK * 2, HALO_BYTES = 2 * HALO_PLANE;
  constexpr int WPT = BN * BK * 2, WSTAGE = 2 * WPT, NSW = 3;
  constexpr int PH = HALO_BYTES / 1024 / NW, PW = WSTAGE / 1024 / NW;
  constexpr int EPR = NW == 8 ? 16 : 8;  // epilogue rows per pass (per-wave scratch EPR x 64 fp32)
  static_assert((HALO_BYTES / 1024) % NW == 0 && (WSTAGE / 1024) % NW == 0, "pieces per wave");
  static_assert(NW * EPR * 64 * 4 <= HALO_BYTES, "epilogue scratch");
  __shared__ __attribute__((aligned(1024))) char smem[2 * HALO_BYTES + NSW * WSTAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * 64;
  const int H = g.H, W = g.W, Hp = H >> 1, Wp = W >> 1;
  const int tiles_x = (W + kHT - 1) / kHT, tiles_y = (H + kHT - 1) / kHT;
  const int num_n = g.Cout / BN, ntiles = g.B * tiles_y * tiles_x * num_n;
  // this workgroup's tiles: t_begin + local + k * nx (workgroups go to XCDs round-robin)
  const int G = min(8, (int)gridDim.x);  // tile ranges (XCDs in use)
  const int xcd = blockIdx.x % G, local = blockIdx.x / G, nx = ((int)gridDim.x - xcd + G - 1) / G;
  const int t_begin = (int)((long long)ntiles * xcd / G), t_end = (int)((long long)ntiles * (xcd + 1) / G);
  const int T = local < t_end - t_begin ? (t_end - t_begin - local + nx - 1) / nx : 0;
  if (T == 0) return;  // workgroup-uniform
  const int CB = g.Cin / BK, nsteps = 9 * CB, S = T * nsteps, GCB = T * CB;
  const float accs = ldexpf(g.acc_scale, range_slot_exp(g.rtab, g.x_slot));
  const int eo = range_exponent(g.ro);
  const int zrow = g.X.rows_pad - 1;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem);

  struct Tile {
    int n, y0, x0, n0;
  };
  auto decode = [&](int k) {
    const int tile = t_begin + local + k * nx;
    const int tm = tile / num_n, tn = tile - tm * num_n;
    const int n = tm / (tiles_y * tiles_x), trem = tm - n * tiles_y * tiles_x;
    return Tile{n, (trem / tiles_x) * kHT, (trem % tiles_x) * kHT, tn * BN};
  };
  auto issue_halo = [&](const Tile& t, int cb, int buf) {
#pragma unroll
    for (int i = 0; i < PH; ++i) {
      const int q = wave * PH + i;  // wave-uniform piece: 16 layout rows of one plane
      const int pl = q / (kHRows / 16);
      const int lr = (q % (kHRows / 16)) * 16 + (lane >> 2);
      int hy = 0, hx = 0, c = 0;
      const bool used = halo_inv(lr, lane & 3, hy, hx, c);
      const int yy = t.y0 - 1 + hy, xx = t.x0 - 1 + hx;
      const bool ok = used && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const int rs = ok ? (t.n * H + yy) * W + xx : zrow;
      const uint32_t voff = (uint32_t)rs * 64u + (uint32_t)((c ^ plane_swz(rs)) << 4);
      const char* base = reinterpret_cast<const char*>(g.X.p + pl * g.X.ps + (size_t)cb * g.X.rows_pad * BK);
      dma16(base, voff, lds0 + buf * HALO_BYTES + q * 1024);
    }
  };
  auto issue_w = [&](int n0, int ls, int slot) {
    const int kt = (ls % 9) * CB + ls / 9;  // local step ls = (channel block ls / 9, tap ls % 9)
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int q = wave * PW + i;
      const int pl = q / (WPT / 1024), pc = q % (WPT / 1024);
      const char* src = reinterpret_cast<const char*>(g.Wt.p + pl * g.Wt.ps + ((size_t)kt * g.Wt.rows_pad + n0) * BK) + pc * 1024;
      dma16(src, lane * 16, lds0 + 2 * HALO_BYTES + slot * WSTAGE + q * 1024);
    }
  };
  // W(u) for global step u: tile k + (ls >= nsteps), local step ls
  auto issue_w_step = [&](const Tile& cur, const Tile& nxt, int ls, int u) {
    if (ls < nsteps) issue_w(cur.n0, ls, u % NSW);
    else issue_w(nxt.n0, ls - nsteps, u % NSW);
  };
  // GEMM row p of the tile (quad order) -> pixel (py, px)
  auto pix = [&](int p, int& py, int& px) {
    const int q4 = p >> 2, sub = p & 3;
    py = 2 * (q4 >> 3) + (sub >> 1);
    px = 2 * (q4 & 7) + (sub & 1);
  };
  int hpy[WMT], hpx[WMT];  // halo pixel of this lane's A rows at tap (0, 0)
#pragma unroll
  for (int i = 0; i < WMT; ++i) pix(wm0 + i * 16 + (lane & 15), hpy[i], hpx[i]);

  // one step's fragments: all twelve reads in flight, then the MFMAs (left to itself the
  // scheduler recycles fragment registers and serialises each read behind the last MFMAs)
  struct Frag {
    f16x8 ah[WMT], al[WMT], wh[4], wl[4];
  };
  auto load = [&](Frag& f, int hbuf, int tap, int wslot) {
    const char* hb = smem + hbuf * HALO_BYTES;
    const char* wb = smem + 2 * HALO_BYTES + wslot * WSTAGE;
    const int c = lane >> 4, r16 = lane & 15;
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      const int x = hpx[i] + tap % 3;
      const int o = halo_row(hpy[i] + tap / 3, x) * (BK * 2) + (halo_pos(x, c) << 4);
      f.ah[i] = *reinterpret_cast<const f16x8*>(hb + o);
      f.al[i] = *reinterpret_cast<const f16x8*>(hb + HALO_PLANE + o);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn0 + j * 16 + r16;
      const int o = r * (BK * 2) + ((c ^ plane_swz(r)) << 4);
      f.wh[j] = *reinterpret_cast<const f16x8*>(wb + o);
      f.wl[j] = *reinterpret_cast<const f16x8*>(wb + WPT + o);
    }
  };
  f32x4 acc[WMT][4];
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f16x8 whs = f.wh[j] * (_Float16)kLoScale;  // exact: |W_h| < 16
#pragma unroll
      for (int i = 0; i < WMT; ++i) acc[i][j] = mfma_h3_16(f.ah[i], f.al[i], whs, f.wl[j], f.wh[j], acc[i][j]);
    }
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  const int cq = (lane & 7) * 8;
  const float so = ldexpf(1.f, -eo);
  float wmax = 0.f;
  auto store8 = [&](int row, int col0, f32x4 v0, f32x4 v1) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.bias + col0);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.bias + col0 + 4);
    f16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = fmaxf(fmaf(e < 4 ? v0[e] : v1[e - 4], accs, e < 4 ? b0[e] : b1[e - 4]), 0.f);
      wmax = fmaxf(wmax, v);
      _Float16 a, c;
      split2h(v * so, a, c);
      h[e] = a;
      l[e] = c;
    }
    const size_t off = plane_off(row, col0, g.yrows_pad);
    *reinterpret_cast<f16x8*>(g.Y + off) = h;
    *reinterpret_cast<f16x8*>(g.Y + g.yps + off) = l;
  };

  // prologue: halo 0, weights of steps 0 and 1
  Tile cur = decode(0);
  Tile nxt = T > 1 ? decode(1) : cur;
  issue_halo(cur, 0, 0);
  issue_w(cur.n0, 0, 0);
  issue_w_step(cur, nxt, 1, 1);

  int gs = 0;
  for (int k = 0; k < T; ++k) {
#pragma unroll
    for (int i = 0; i < WMT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int cb = 0; cb < CB; ++cb) {
      const int gcb = k * CB + cb;
      const bool hnext = gcb + 1 < GCB;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap, ++gs) {
        // W(gs) complete (and with it the halo of this block, issued before it); issued after
        // it: W(gs + 1) and, at taps 1-2, the next halo (issued at tap 0)
        if ((tap == 1 || tap == 2) && hnext) sp_wait_vm<PW + PH>();
        else if (gs + 1 < S) sp_wait_vm<PW>();
        else sp_wait_vm<0>();
        barrier();
        if (gs + 2 < S) issue_w_step(cur, nxt, cb * 9 + tap + 2, gs + 2);
        if (tap == 0 && hnext) {
          if (cb + 1 < CB) issue_halo(cur, cb + 1, (gcb + 1) & 1);
          else issue_halo(nxt, 0, (gcb + 1) & 1);
        }
        Frag f;
        load(f, gcb & 1, tap, gs % NSW);
        __builtin_amdgcn_sched_barrier(0);
        mma(f);
      }
    }
    // epilogue: bias + ReLU (+ pool) -> planes through a per-wave transpose in the halo buffer
    // just consumed (every wave past its last read of it: the barrier)
    barrier();
    float* ep = reinterpret_cast<float*>(smem + ((k * CB + CB - 1) & 1) * HALO_BYTES) + wave * (EPR * 64);
    const int col0 = cur.n0 + wn0 + cq;
    if constexpr (!POOL) {
#pragma unroll
      for (int a = 0; a < WMT; ++a)
#pragma unroll
        for (int h = 0; h < 16 / EPR; ++h) {
          if ((lane >> 4) / (EPR / 4) == h)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int rr = ((lane >> 4) % (EPR / 4)) * 4 + r, c = j * 16 + (lane & 15);
                ep[rr * 64 + (c ^ ((rr & 1) << 2))] = acc[a][j][r];
              }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int kk = 0; kk < EPR / 8; ++kk) {
            const int rr = (lane >> 3) + 8 * kk;
            int py, px;
            pix(wm0 + a * 16 + h * EPR + rr, py, px);
            const int sw = (rr & 1) << 2;
            const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
            if (cur.y0 + py < H && cur.x0 + px < W) store8((cur.n * H + cur.y0 + py) * W + cur.x0 + px, col0, v0, v1);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass writes
        }
    } else {
      // the 4 registers of a lane are the 4 pixels of one pooling window: relu(max + b) ==
      // max(relu(. + b)) (monotone, and rounding is monotone); 16 quads per pass
#pragma unroll
      for (int a2 = 0; a2 < WMT / 4 + (WMT < 4); ++a2) {
#pragma unroll
        for (int a = 0; a < (WMT < 4 ? WMT : 4); ++a)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 v = acc[a2 * 4 + a][j];
            const int pr_ = a * 4 + (lane >> 4), c = j * 16 + (lane & 15);
            ep[pr_ * 64 + (c ^ ((pr_ & 1) << 2))] = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int kk = 0; kk < (WMT < 4 ? WMT : 4) / 2; ++kk) {
          const int rr = (lane >> 3) + 8 * kk;
          const int q4 = (wm0 + a2 * 64) / 4 + rr;  // quad of the tile
          const int qy = cur.y0 / 2 + (q4 >> 3), qx = cur.x0 / 2 + (q4 & 7);
          const int sw = (rr & 1) << 2;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + (cq ^ sw));
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rr * 64 + ((cq + 4) ^ sw));
          if (qy < Hp && qx < Wp) store8((cur.n * Hp + qy) * Wp + qx, col0, v0, v1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    cur = nxt;
    if (k + 2 < T) nxt = decode(k + 2);
  }
  range_commit_lds(g.ro, wmax, eo, reinterpret_cast<float*>(smem + 2 * HALO_BYTES));
}

static int sp_num_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return 256;
    return cus;
  }();
  return n;
}

template <int BN, bool POOL>
static hipError_t sp_conv3x3_halo_launch(const ConvH3Args& a, hipStream_t st) {
  const int tiles = a.B * ((a.H + kHT - 1) / kHT) * ((a.W + kHT - 1) / kHT) * (a.Cout / BN);
  const int grid = std::min(tiles, sp_num_cus());  // one workgroup per CU (LDS-limited)
  hipLaunchKernelGGL((sp_conv3x3_halo_kernel<BN, POOL>), dim3(grid), dim3(8 * (BN / 64) * 64), 0, st, a);
  return hipGetLastError();
}

template <int BN, int NS, bool POOL>
static hipError_t sp_conv3x3_launch(const ConvH3Args& a, int R, hipStream_t st) {
  const int tiles = ((R + 255) / 256) * (a.Cout / BN);
  hipLaunchKernelGGL((sp_conv3x3_kernel<BN, NS, POOL>), dim3(tiles), dim3(4 * (BN / 64) * 64), 0, st, a);
  return hipGetLastError();
}

hipError_t sp_conv3x3(const ConvH3Args& a, hipStream_t st) {
  if (a.B <= 0 || a.H <= 0 || a.W <= 0) return hipSuccess;
  const long long rin = (long long)a.B * a.H * a.W;
  const long long rout = a.pool ? (long long)a.B * (a.H / 2) * (a.W / 2) : rin;
  if (a.Cin % kKB || a.Cout % 64 || !a.X.p || !a.Wt.p || !a.Y || !a.bias || a.X.rows_pad <= rin || a.X.rows_pad % 256 ||
      a.Wt.rows_pad != a.Cout || a.yrows_pad < rout || a.X.rows_pad > (1 << 26))  // 32-bit DMA byte offsets
    return hipErrorInvalidValue;
  if (a.pool && (a.H < 2 || a.W < 2)) return hipErrorInvalidValue;
  const char* conv = getenv("LG_SP_CONV");  // read per launch (tests flip it between calls)
  const bool gather = conv && !strcmp(conv, "gather");
  if (!gather) {  // halo tiles (default); LG_SP_CONV=gather: the per-tap row gather above
    if (a.Cout % 128 == 0) return a.pool ? sp_conv3x3_halo_launch<128, true>(a, st) : sp_conv3x3_halo_launch<128, false>(a, st);
    return a.pool ? sp_conv3x3_halo_launch<64, true>(a, st) : sp_conv3x3_halo_launch<64, false>(a, st);
  }
  const int R = (int)(a.pool ? 4 * rout : rin);
  if (a.Cout % 128 == 0) return a.pool ? sp_conv3x3_launch<128, 3, true>(a, R, st) : sp_conv3x3_launch<128, 3, false>(a, R, st);
  return a.pool ? sp_conv3x3_launch<64, 3, true>(a, R, st) : sp_conv3x3_launch<64, 3, false>(a, R, st);
}

__global__ void sp_zero_rows_kernel(_Float16* planes, long long ps, int rows_pad, int nkb, int R) {
  const int tail = rows_pad - R;
  const long long total = 2LL * nkb * tail * 4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int chunk = (int)(i & 3);
    long long t = i >> 2;
    const int rr = (int)(t % tail);
    t /= tail;
    const int kb = (int)(t % nkb), pl = (int)(t / nkb);
    *reinterpret_cast<f32x4*>(planes + pl * ps + ((size_t)kb * rows_pad + R + rr) * kKB + chunk * 8) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

hipError_t sp_zero_rows(_Float16* planes, long long ps, int rows_pad, int K, int R, hipStream_t st) {
  if (R >= rows_pad) return hipSuccess;
  const long long total = 2LL * (K / kKB) * (rows_pad - R) * 4;
  hipLaunchKernelGGL(sp_zero_rows_kernel, dim3(grid_for(total, 256, 1024)), dim3(256), 0, st, planes, ps, rows_pad, K / kKB, R);
  return hipGetLastError();
}

__global__ void sp_repack_kernel(const float* w, int Cout, int Cin, int k, float* dst) {
  const int K = k * k * Cin;
  const long long total = (long long)Cout * K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / K), col = (int)(i % K);
    const int tap = col / Cin, ci = col - tap * Cin;
    dst[i] = w[((size_t)co * Cin + ci) * k * k + tap];
  }
}

hipError_t sp_repack_conv(const float* w, int Cout, int Cin, int ksize, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(sp_repack_kernel, dim3(grid_for((long long)Cout * Cin * ksize * ksize, 256, 1024)), dim3(256), 0, st, w,
                     Cout, Cin, ksize, dst);
  return hipGetLastError();
}

// ---- heads ---------------------------------------------------------------------------------
// superpoint.py:224-230: softmax over the 65 channels, dustbin dropped, cell (y, x) channel
// 8 dy + dx -> pixel (8y + dy, 8x + dx).  One thread per cell.
__global__ void sp_scores_kernel(const float* logits, int ld, int B, int Hc, int Wc, float* scores) {
  const int cells = B * Hc * Wc;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < cells; p += gridDim.x * blockDim.x) {
    const float* l = logits + (size_t)p * ld;
    float v[65];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 65; ++c) {
      v[c] = l[c];
      mx = fmaxf(mx, v[c]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 65; ++c) {
      v[c] = expf(v[c] - mx);
      s += v[c];
    }
    const int n = p / (Hc * Wc), rem = p - n * Hc * Wc, y = rem / Wc, x = rem - y * Wc;
    const int Ws = 8 * Wc;
#pragma unroll
    for (int dy = 0; dy < 8; ++dy) {
      float* o = scores + ((size_t)n * 8 * Hc + 8 * y + dy) * Ws + 8 * x;
      f32x4 a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = div_rn(v[8 * dy + e], s);
        b[e] = div_rn(v[8 * dy + 4 + e], s);
      }
      *reinterpret_cast<f32x4*>(o) = a;
      *reinterpret_cast<f32x4*>(o + 4) = b;
    }
  }
}

hipError_t sp_detector_scores(const float* logits, int ld, int B, int Hc, int Wc, float* scores, hipStream_t st) {
  const long long cells = (long long)B * Hc * Wc;
  if (cells == 0) return hipSuccess;
  hipLaunchKernelGGL(sp_scores_kernel, dim3(grid_for(cells, 256, 4096)), dim3(256), 0, st, logits, ld, B, Hc, Wc, scores);
  return hipGetLastError();
}

// F.normalize(x, p=2, dim=channels): one wave per 256-channel row, 4 channels per lane
__global__ void sp_desc_norm_kernel(const float* x, int rows, float* y) {
  const int lane = threadIdx.x & 63;
  for (long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < rows;
       row += ((long long)gridDim.x * blockDim.x) >> 6) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + row * 256 + lane * 4);
    const float s = wave_sum_dpp(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
    const float d = fmaxf(sqrtf(s), 1e-12f);
    *reinterpret_cast<f32x4*>(y + row * 256 + lane * 4) =
        f32x4{div_rn(v[0], d), div_rn(v[1], d), div_rn(v[2], d), div_rn(v[3], d)};
  }
}

hipError_t sp_desc_normalize(const float* x, int rows, float* y, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(sp_desc_norm_kernel, dim3(grid_for((long long)rows * 64, 256, 4096)), dim3(256), 0, st, x, rows, y);
  return hipGetLastError();
}

// ---- simple_nms (superpoint.py:60-80) ---------------------------------------------------------
// One pass = a (2r+1)^2 max-pool (stride 1, -inf padding: max_pool2d) of a 32 x 32 output tile
// from a halo tile in LDS (horizontal then vertical max), fused with the pass's elementwise step:
//   MODE 0: mask = s == pool(s)
//   MODE 1: sup = pool(mask) > 0;  ss = sup ? 0 : s
//   MODE 2: mask |= (ss == pool(ss)) & !sup
constexpr int kNmsTile = 32, kNmsMaxR = 8, kNmsHalo = kNmsTile + 2 * kNmsMaxR;
template <int MODE>
__global__ __launch_bounds__(256) void sp_nms_kernel(const float* s, unsigned char* mask, unsigned char* sup, float* ss,
                                                     int Hs, int Ws, int r) {
  __shared__ float tin[kNmsHalo * kNmsHalo];
  __shared__ float th[kNmsHalo * kNmsTile];
  const int b = blockIdx.z, ty0 = blockIdx.y * kNmsTile, tx0 = blockIdx.x * kNmsTile;
  const int E = kNmsTile + 2 * r;
  const size_t plane = (size_t)Hs * Ws, base = (size_t)b * plane;
  for (int i = threadIdx.x; i < E * E; i += blockDim.x) {
    const int yy = ty0 - r + i / E, xx = tx0 - r + i % E;
    float v = -INFINITY;
    if ((unsigned)yy < (unsigned)Hs && (unsigned)xx < (unsigned)Ws) {
      const size_t o = base + (size_t)yy * Ws + xx;
      v = MODE == 0 ? s[o] : MODE == 1 ? (float)mask[o] : ss[o];
    }
    tin[i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < E * kNmsTile; i += blockDim.x) {
    const int ry = i / kNmsTile, cx = i % kNmsTile;
    float m = -INFINITY;
    for (int d = 0; d <= 2 * r; ++d) m = fmaxf(m, tin[ry * E + cx + d]);
    th[i] = m;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kNmsTile * kNmsTile; i += blockDim.x) {
    const int oy = i / kNmsTile, ox = i % kNmsTile, y = ty0 + oy, x = tx0 + ox;
    if (y >= Hs || x >= Ws) continue;
    float m = -INFINITY;
    for (int d = 0; d <= 2 * r; ++d) m = fmaxf(m, th[(oy + d) * kNmsTile + ox]);
    const float c = tin[(oy + r) * E + ox + r];
    const size_t o = base + (size_t)y * Ws + x;
    if (MODE == 0) {
      mask[o] = c == m;
    } else if (MODE == 1) {
      const bool sp = m > 0.f;
      sup[o] = sp;
      ss[o] = sp ? 0.f : s[o];
    } else {
      if (c == m && !sup[o]) mask[o] = 1;
    }
  }
}

hipError_t sp_nms(const float* scores, int B, int Hs, int Ws, int radius, unsigned char* mask, unsigned char* sup,
                  float* ss, hipStream_t st) {
  if (B <= 0 || Hs <= 0 || Ws <= 0) return hipSuccess;
  if (radius < 0 || radius > kNmsMaxR) return hipErrorInvalidValue;
  const dim3 grid((Ws + kNmsTile - 1) / kNmsTile, (Hs + kNmsTile - 1) / kNmsTile, B);
  hipLaunchKernelGGL(sp_nms_kernel<0>, grid, dim3(256), 0, st, scores, mask, sup, ss, Hs, Ws, radius);
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(sp_nms_kernel<1>, grid, dim3(256), 0, st, scores, mask, sup, ss, Hs, Ws, radius);
    hipLaunchKernelGGL(sp_nms_kernel<2>, grid, dim3(256), 0, st, scores, mask, sup, ss, Hs, Ws, radius);
  }
  return hipGetLastError();
}

// ---- candidates: borders, threshold, row-major compaction ------------------------------------
constexpr int kCandRows = 4;  // score-map rows per block
int sp_cand_blocks(int Hs) { return (Hs + kCandRows - 1) / kCandRows; }

// superpoint.py:244-254 (python slice starts: a negative start counts from the end)
__device__ __forceinline__ int slice_start(int start, int n) { return start < 0 ? max(start + n, 0) : start; }
__device__ __forceinline__ float cand_value(const float* s, const unsigned char* mask, size_t o, int y, int x, int border,
                                            int y1, int x1) {
  float v = mask[o] ? s[o] : 0.f;
  if (border && (y < border || x < border || y >= y1 || x >= x1)) v = -1.f;
  return v;
}

template <bool WRITE>
__global__ __launch_bounds__(256) void sp_cand_kernel(const float* s, const unsigned char* mask, int Hs, int Ws, int border,
                                                      const float* image_size, float thr, unsigned* key, int* idx, int* blk,
                                                      int* cnt) {
  __shared__ int wtot[4];
  __shared__ int sbase;
  const int b = blockIdx.y, nblk = gridDim.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int y1 = slice_start(Hs - border, Hs), x1 = slice_start(Ws - border, Ws);
  if (image_size) {
    y1 = slice_start((int)image_size[2 * b + 1] - border, Hs);
    x1 = slice_start((int)image_size[2 * b] - border, Ws);
  }
  const size_t base = (size_t)b * Hs * Ws;
  const int p0 = blockIdx.x * kCandRows * Ws, p1 = min(Hs, (blockIdx.x + 1) * kCandRows) * Ws;
  if (!WRITE) {
    int c = 0;
    for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
      const int y = p / Ws, x = p - y * Ws;
      c += cand_value(s, mask, base + p, y, x, border, y1, x1) > thr;
    }
    c = (int)wave_sum_dpp((float)c);  // < 2^24: exact
    if (lane == 0) wtot[wv] = c;
    __syncthreads();
    if (threadIdx.x == 0) blk[b * nblk + blockIdx.x] = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    return;
  }
  // exclusive prefix of the block counts of this image
  if (threadIdx.x == 0) {
    int a = 0;
    for (int j = 0; j < (int)blockIdx.x; ++j) a += blk[b * nblk + j];
    sbase = a;
    if (blockIdx.x == nblk - 1) cnt[b] = a + blk[b * nblk + blockIdx.x];
  }
  __syncthreads();
  int run = sbase;
  unsigned* kb = key + base;
  int* ib = idx + base;
  for (int p00 = p0; p00 < p1; p00 += blockDim.x) {
    const int p = p00 + threadIdx.x;
    float v = 0.f;
    bool take = false;
    if (p < p1) {
      const int y = p / Ws, x = p - y * Ws;
      v = cand_value(s, mask, base + p, y, x, border, y1, x1);
      take = v > thr;
    }
    const unsigned long long bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) wtot[wv] = __popcll(bal);
    __syncthreads();
    int off = run;
    for (int w = 0; w < wv; ++w) off += wtot[w];
    if (take) {
      kb[off + before] = order_key(v);
      ib[off + before] = p;
    }
    run += wtot[0] + wtot[1] + wtot[2] + wtot[3];
  }
}

hipError_t sp_candidates(const float* scores, const unsigned char* mask, int B, int Hs, int Ws, int border,
                         const float* image_size, float thr, unsigned* key, int* idx, int* blk, int* cnt, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  const dim3 grid(sp_cand_blocks(Hs), B);
  hipLaunchKernelGGL(sp_cand_kernel<false>, grid, dim3(256), 0, st, scores, mask, Hs, Ws, border, image_size, thr, key, idx,
                     blk, cnt);
  hipLaunchKernelGGL(sp_cand_kernel<true>, grid, dim3(256), 0, st, scores, mask, Hs, Ws, border, image_size, thr, key, idx,
                     blk, cnt);
  return hipGetLastError();
}

// ---- top-k selection (superpoint.py:83-87,274-294) -------------------------------------------
// One 1024-thread workgroup per image.  Radix select over the 32-bit order keys (4 passes of
// 8-bit digits, LDS histograms) finds the k-th largest key T and how many keys equal to T to keep;
// an ordered block scan gathers the k winners (ties at T: lowest pixel index first) into LDS,
// a bitonic sort orders them by (score desc, index asc).
__device__ __forceinline__ int block_excl_scan(bool f, int* wtot, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long bal = __ballot(f);
  const int before = __popcll(bal & ((1ull << lane) - 1ull));
  __syncthreads();
  if (lane == 0) wtot[wv] = __popcll(bal);
  __syncthreads();
  int off = 0;
  total = 0;
  for (int w = 0; w < nw; ++w) {
    if (w < wv) off += wtot[w];
    total += wtot[w];
  }
  return off + before;
}

__global__ __launch_bounds__(1024) void sp_select_kernel(const unsigned* key, const int* idx, const int* cnt, int cand_cap,
                                                         int k, int* sel_idx, float* sel_score, int cap, int* nout) {
  __shared__ unsigned skey[kSpSelectMax];
  __shared__ int sidx[kSpSelectMax];
  __shared__ int hist[256];
  __shared__ int wtot[16];
  __shared__ int s_dig, s_need;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int c = cnt[b];
  const unsigned* K = key + (size_t)b * cand_cap;
  const int* I = idx + (size_t)b * cand_cap;
  int* so = sel_idx + (size_t)b * cap;
  float* sc = sel_score + (size_t)b * cap;
  if (k <= 0 || c <= k) {  // everything, row-major (top_k_keypoints returns them unsorted)
    const int n = min(c, cap);
    for (int t = tid; t < n; t += blockDim.x) {
      so[t] = I[t];
      sc[t] = key_value(K[t]);
    }
    if (tid == 0) nout[b] = n;
    return;
  }
  unsigned prefix = 0, pmask = 0;
  int need = k;
  for (int d = 3; d >= 0; --d) {
    for (int t = tid; t < 256; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    const int sh = 8 * d;
    for (int t = tid; t < c; t += blockDim.x) {
      const unsigned kk = K[t];
      if ((kk & pmask) == prefix) atomicAdd(&hist[(kk >> sh) & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0, dig = 255;
      for (; dig > 0; --dig) {
        if (acc + hist[dig] >= need) break;
        acc += hist[dig];
      }
      s_dig = dig;
      s_need = need - acc;
    }
    __syncthreads();
    prefix |= (unsigned)s_dig << sh;
    pmask |= 255u << sh;
    need = s_need;
    __syncthreads();
  }
  const unsigned T = prefix;
  int taken = 0, ties = 0;
  for (int b0 = 0; b0 < c; b0 += blockDim.x) {
    const int t = b0 + tid;
    const unsigned kk = t < c ? K[t] : 0u;
    const bool eq = t < c && kk == T;
    int eq_total;
    const int eq_rank = ties + block_excl_scan(eq, wtot, eq_total);
    const bool take = (t < c && kk > T) || (eq && eq_rank < need);
    int take_total;
    const int pos = taken + block_excl_scan(take, wtot, take_total);
    if (take) {
      skey[pos] = kk;
      sidx[pos] = I[t];
    }
    ties += eq_total;
    taken += take_total;
  }
  int P = 1;
  while (P < k) P <<= 1;
  for (int t = k + tid; t < P; t += blockDim.x) {
    skey[t] = 0u;
    sidx[t] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = tid; p < P / 2; p += blockDim.x) {
        const int i = 2 * stride * (p / stride) + (p % stride), j = i + stride;
        const unsigned ki = skey[i], kj = skey[j];
        const int ii = sidx[i], ij = sidx[j];
        const bool j_first = kj > ki || (kj == ki && ij < ii);  // j belongs before i
        const bool up = (i & size) == 0;                         // this run in "before" order
        if (up == j_first) {
          skey[i] = kj;
          skey[j] = ki;
          sidx[i] = ij;
          sidx[j] = ii;
        }
      }
      __syncthreads();
    }
  for (int t = tid; t < k; t += blockDim.x) {
    so[t] = sidx[t];
    sc[t] = key_value(skey[t]);
  }
  if (tid == 0) nout[b] = k;
}

hipError_t sp_select(const unsigned* key, const int* idx, const int* cnt, int B, int cand_cap, int k, int* sel_idx,
                     float* sel_score, int cap, int* n, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (k > kSpSelectMax || (k > 0 && cap < k)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sp_select_kernel, dim3(B), dim3(1024), 0, st, key, idx, cnt, cand_cap, k, sel_idx, sel_score, cap, n);
  return hipGetLastError();
}

// ---- keypoints (+ soft-argmax refinement, superpoint.py:97-113) ------------------------------
__global__ void sp_kpts_kernel(const int* sel_idx, const int* n, int B, int cap, int Hs, int Ws, const float* dense, int r,
                               float* kpts) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < (long long)B * cap;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / cap), i = (int)(t - (long long)b * cap);
    if (i >= n[b]) continue;
    const int p = sel_idx[t], y = p / Ws, x = p - y * Ws;
    float fy = (float)y, fx = (float)x;
    if (r > 0) {
      const float* d = dense + (size_t)b * Hs * Ws;
      float s = 0.f, sx = 0.f, sy = 0.f;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if ((unsigned)yy >= (unsigned)Hs || (unsigned)xx >= (unsigned)Ws) continue;
          const float v = d[(size_t)yy * Ws + xx];
          s += v;
          sx = fmaf(v, (float)dx, sx);
          sy = fmaf(v, (float)dy, sy);
        }
      fy = fy + div_rn(sy, s);
      fx = fx + div_rn(sx, s);
    }
    kpts[2 * t] = fx;
    kpts[2 * t + 1] = fy;
  }
}

hipError_t sp_keypoints(const int* sel_idx, const int* n, int B, int cap, int Hs, int Ws, const float* dense, int radius,
                        float* kpts, hipStream_t st) {
  if ((long long)B * cap == 0) return hipSuccess;
  hipLaunchKernelGGL(sp_kpts_kernel, dim3(grid_for((long long)B * cap, 256)), dim3(256), 0, st, sel_idx, n, B, cap, Hs, Ws,
                     dense, radius, kpts);
  return hipGetLastError();
}

// ---- descriptor sampling (superpoint.py:117-149) ---------------------------------------------
// grid_sample(bilinear, zero padding) in torch's CPU formulation: normalised grid g = 2 k' - 1,
// unnormalised with align_corners=True (legacy) as (g + 1) * ((W - 1) / 2), else
// (g + 1) * (W / 2) - 0.5; then F.normalize over the channels.  One wave per keypoint.
__global__ void sp_sample_kernel(const float* kpts, const int* n, int B, int cap, const float* desc, int Hc, int Wc,
                                 int legacy, float* out, float* kout) {
  const int lane = threadIdx.x & 63;
  for (long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < (long long)B * cap;
       w += ((long long)gridDim.x * blockDim.x) >> 6) {
    const int b = (int)(w / cap), i = (int)(w - (long long)b * cap);
    if (i >= n[b]) continue;
    const float x = kpts[2 * w], y = kpts[2 * w + 1];
    float gx, gy, ix, iy;
    if (legacy) {  // k - s/2 + 0.5, / (size*s - s/2 - 0.5), *2 - 1
      gx = div_rn(add_rn(sub_rn(x, 4.f), 0.5f), (float)(Wc * 8) - 4.5f);
      gy = div_rn(add_rn(sub_rn(y, 4.f), 0.5f), (float)(Hc * 8) - 4.5f);
      gx = sub_rn(mul_rn(gx, 2.f), 1.f);
      gy = sub_rn(mul_rn(gy, 2.f), 1.f);
      ix = mul_rn(add_rn(gx, 1.f), (float)(Wc - 1) * 0.5f);
      iy = mul_rn(add_rn(gy, 1.f), (float)(Hc - 1) * 0.5f);
    } else {
      gx = sub_rn(mul_rn(div_rn(x, (float)(Wc * 8)), 2.f), 1.f);
      gy = sub_rn(mul_rn(div_rn(y, (float)(Hc * 8)), 2.f), 1.f);
      ix = sub_rn(mul_rn(add_rn(gx, 1.f), (float)Wc * 0.5f), 0.5f);
      iy = sub_rn(mul_rn(add_rn(gy, 1.f), (float)Hc * 0.5f), 0.5f);
    }
    const float x0f = floorf(ix), y0f = floorf(iy);
    const int x0 = (int)x0f, y0 = (int)y0f;
    const float tx = ix - x0f, ty = iy - y0f;
    const float wts[4] = {(1.f - tx) * (1.f - ty), tx * (1.f - ty), (1.f - tx) * ty, tx * ty};
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int xx = x0 + (q & 1), yy = y0 + (q >> 1);
      if ((unsigned)xx < (unsigned)Wc && (unsigned)yy < (unsigned)Hc) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(desc + (((size_t)b * Hc + yy) * Wc + xx) * 256 + lane * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = fmaf(v[e], wts[q], acc[e]);
      }
    }
    if (out) {
      const float s = wave_sum_dpp(acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2] + acc[3] * acc[3]);
      const float d = fmaxf(sqrtf(s), 1e-12f);
      *reinterpret_cast<f32x4*>(out + w * 256 + lane * 4) =
          f32x4{div_rn(acc[0], d), div_rn(acc[1], d), div_rn(acc[2], d), div_rn(acc[3], d)};
    }
    if (kout && lane == 0) {
      kout[2 * w] = x + 0.5f;
      kout[2 * w + 1] = y + 0.5f;
    }
  }
}

hipError_t sp_sample(const float* kpts, const int* n, int B, int cap, const float* desc, int Hc, int Wc, int legacy,
                     float* out, float* kpts_out, hipStream_t st) {
  if ((long long)B * cap == 0) return hipSuccess;
  hipLaunchKernelGGL(sp_sample_kernel, dim3(grid_for((long long)B * cap * 64, 256)), dim3(256), 0, st, kpts, n, B, cap, desc,
                     Hc, Wc, legacy, out, kpts_out);
  return hipGetLastError();
}

}  // namespace lg
