// Micro-benchmark of attention variants (tools only; not shipped).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench_attn.hip -o tools/kbench_attn && tools/kbench_attn [N]
// Self-attention shape of the bench (B=32 pairs, 4 heads, N keys, 2 sets), random q/k in
// [-2, 2), v in [-1, 1); each variant is checked against an fp64 reference on set 0.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "attn_experiments.hip"

using namespace lg;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill(float* p, size_t n, unsigned seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
    p[i] = (((x & 0xffffff) / 16777216.0f) * 2.f - 1.f) * scale;
  }
}

__global__ void planes_x6(const float* x, __bf16* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    __bf16 h, m, l;
    split3(x[i], h, m, l);
    p[i] = h; p[n + i] = m; p[2 * n + i] = l;
  }
}
__global__ void planes_h3(const float* x, _Float16* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    _Float16 h, l;
    split2h(x[i], h, l);
    p[i] = h; p[n + i] = l;
  }
}

// plane image (K = 256) -> fp32 rows (h + l * 2^-11)
__global__ void planes_to_rows(const _Float16* p, long long ps, int rows_pad, float* o, int rows) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)rows * 256) return;
  const int r = (int)(i / 256), c = (int)(i % 256);
  const size_t off = plane_off(r, c, rows_pad);
  o[i] = (float)p[off] + (float)p[ps + off] * (1.f / 2048.f);
}

// naive reference: one thread per (bh, query), double accumulation
__global__ void ref_attn(const float* Q, const float* K, const float* V, float* O, int BH, int H, int N, float scale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= BH * N) return;
  const int bh = t / N, q = t % N;
  const float* qp = Q + ((size_t)bh * N + q) * 64;
  double m = -1e300;
  for (int k = 0; k < N; ++k) {
    double s = 0;
    for (int d = 0; d < 64; ++d) s += (double)qp[d] * K[((size_t)bh * N + k) * 64 + d];
    m = fmax(m, s * scale);
  }
  double l = 0, o[64] = {0};
  for (int k = 0; k < N; ++k) {
    double s = 0;
    for (int d = 0; d < 64; ++d) s += (double)qp[d] * K[((size_t)bh * N + k) * 64 + d];
    const double p = exp(s * scale - m);
    l += p;
    for (int d = 0; d < 64; ++d) o[d] += p * V[((size_t)bh * N + k) * 64 + d];
  }
  const int b = bh / H, h = bh % H;
  for (int d = 0; d < 64; ++d) O[((size_t)b * N + q) * 256 + h * 64 + d] = (float)(o[d] / l);
}

static const char* g_only = nullptr;  // KB_ONLY=<substring>: run only the matching variants

template <class F>
void run(const char* name, F launch, int B, int H, const AttnSet& a0, const AttnSet& a1, float* Oref, float* O, size_t on) {
  if (g_only && !strstr(name, g_only)) return;
  CK(hipMemset(O, 0, on * 4));
  CK(launch());
  CK(hipDeviceSynchronize());
  if (a0.op) {
    planes_to_rows<<<(on + 255) / 256, 256>>>(a0.op, a0.ops, a0.o_rows_pad, O, (int)(on / 256));
    CK(hipDeviceSynchronize());
  }
  std::vector<float> x(on), y(on);
  CK(hipMemcpy(x.data(), O, on * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), Oref, on * 4, hipMemcpyDeviceToHost));
  double md = 0;
  for (size_t i = 0; i < on; ++i) md = fmax(md, fabs((double)x[i] - y[i]));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int it = 10;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < it; ++i) CK(launch());
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= it;
  const double fl = 4.0 * 64.0 * H * B * ((double)a0.Nq * a0.Nk + (double)a1.Nq * a1.Nk);
  printf("%-26s %8.1f us  %6.1f TF/s (fp32-eq)  maxdiff(set0 vs fp64) %.2e\n", name, ms * 1e3, fl / ms / 1e9, md);
}

int main(int argc, char** argv) {
  const int B = 32, H = 4, N = argc > 1 ? atoi(argv[1]) : 2048;
  g_only = getenv("KB_ONLY");
  const size_t n = (size_t)B * H * N * 64;
  float *Q, *K, *V, *O, *Oref;
  void *KP, *VP, *KH, *VH;
  CK(hipMalloc(&Q, 2 * n * 4)); CK(hipMalloc(&K, 2 * n * 4)); CK(hipMalloc(&V, 2 * n * 4));
  CK(hipMalloc(&KP, 3 * 2 * n * 2)); CK(hipMalloc(&VP, 3 * 2 * n * 2));
  CK(hipMalloc(&KH, 2 * 2 * n * 2)); CK(hipMalloc(&VH, 2 * 2 * n * 2));
  CK(hipMalloc(&O, 2 * n * 4)); CK(hipMalloc(&Oref, 2 * n * 4));
  fill<<<(2 * n + 255) / 256, 256>>>(Q, 2 * n, 1, 2.f);
  fill<<<(2 * n + 255) / 256, 256>>>(K, 2 * n, 2, 2.f);
  fill<<<(2 * n + 255) / 256, 256>>>(V, 2 * n, 3, 1.f);
  planes_x6<<<(2 * n + 255) / 256, 256>>>(K, (__bf16*)KP, 2 * n);
  planes_x6<<<(2 * n + 255) / 256, 256>>>(V, (__bf16*)VP, 2 * n);
  planes_h3<<<(2 * n + 255) / 256, 256>>>(K, (_Float16*)KH, 2 * n);
  planes_h3<<<(2 * n + 255) / 256, 256>>>(V, (_Float16*)VH, 2 * n);
  const float scale = 0.125f;
  ref_attn<<<(B * H * N + 127) / 128, 128>>>(Q, K, V, Oref, B * H, H, N, scale);
  CK(hipDeviceSynchronize());
  const long long ps = 2 * (long long)n;
  AttnSet x0{Q, KP, VP, ps, O, N, N}, x1{Q + n, (__bf16*)KP + n, (__bf16*)VP + n, ps, O + (size_t)B * N * 256, N, N};
  const int rp = (2 * B * N + 255) / 256 * 256;
  _Float16* OP;
  CK(hipMalloc(&OP, (size_t)2 * rp * 256 * 2));
  AttnSet h0{Q, KH, VH, ps, O, N, N, OP, (long long)rp * 256, rp, 0};
  AttnSet h1{Q + n, (_Float16*)KH + n, (_Float16*)VH + n, ps, O + (size_t)B * N * 256, N, N, OP, (long long)rp * 256, rp, B * N};
  // range table of the library kernels (kernels.h RangeOut): slot 0 = keys, max |k| = 2, E = 0
  unsigned* rtab;
  CK(hipMalloc(&rtab, 4 * kRangeStride * sizeof(unsigned)));
  {
    std::vector<unsigned> t(4 * kRangeStride, 0u);
    const float two = 2.f;
    memcpy(&t[0], &two, 4);
    CK(hipMemcpy(rtab, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  }
  AttnSet l0 = h0, l1 = h1;
  l0.rtab = l1.rtab = rtab;
  l0.k_slot = l1.k_slot = 0;
  const size_t on = (size_t)B * N * 256;  // compare set 0
  run("lib h3m sub2 prio", [&] { return attention_h3m_launch<2, 1, 8>(l0, l1, B, H, scale, 0); }, B, H, l0, l1, Oref, O, on);
  run("lib h3g sub2 prio", [&] { return attention_h3g_launch<2, 1, 8>(l0, l1, B, H, scale, 0); }, B, H, l0, l1, Oref, O, on);
  run("lib h3m exact", [&] { return attention_h3m_launch<2, 1, 8>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("x6   w8 kt64", [&] { return attention_x6_launch<8, 64>(x0, x1, B, H, scale, 0); }, B, H, x0, x1, Oref, O, on);
  run("h3 w8 kt64 occ2", [&] { return attention_h3_launch<8, 64, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3s staggered", [&] { return attention_h3s_launch<64>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3m 16x16x32", [&] { return attention_h3m16_launch<64>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3f lean softmax", [&] { return attention_h3f_launch<64>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3g dma sub2", [&] { return attention_h3g_launch<2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3g dma sub1", [&] { return attention_h3g_launch<1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3g dma sub1 prio", [&] { return attention_h3g_launch<1, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3g dma sub2 prio", [&] { return attention_h3g_launch<2, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3 DIAG1 no softmax", [&] { return attention_h3_launch<8, 64, 2, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3 DIAG2 no mfma", [&] { return attention_h3_launch<8, 64, 2, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3 DIAG3 mfma only", [&] { return attention_h3_launch<8, 64, 2, 3>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3 DIAG3 occ4", [&] { return attention_h3_launch<8, 64, 4, 3>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp kt64 (ping-pong)", [&] { return attention_h3pp_launch<64>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp prio on M phase", [&] { return attention_h3pp_launch<64, 1, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp no prio", [&] { return attention_h3pp_launch<64, 1, 0>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp lag0 (lock-step)", [&] { return attention_h3pp_launch<64, 0, 0>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp no reads/copies/barriers", [&] { return attention_h3pp_launch<64, 1, 1, 64 + 8 + 4>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp no softmax", [&] { return attention_h3pp_launch<64, 1, 1, 1>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp no mfma", [&] { return attention_h3pp_launch<64, 1, 1, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3pp no LDS reads/copies", [&] { return attention_h3pp_launch<64, 1, 1, 12>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  if (!g_only) {  // per-phase timelines (s_memtime) of waves 0 (group 0) and 4 (group 1) of workgroup 0
    std::vector<unsigned long long> ts(8 * 4096);
    auto show = [&](const char* name, auto launch) {
      CK(hipMemset(O, 0, 8 * 4096 * 8));
      CK(launch());
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ts.data(), O, ts.size() * 8, hipMemcpyDeviceToHost));
      const int nt = N / 64;
      printf("%s\n", name);
      for (int g = 0; g < 8; ++g) {
        double m = 0, bm = 0, v = 0, bv = 0;
        int cnt = 0;
        for (int j = 2; j < nt - 2 && 4 * j + 4 < 160; ++j, ++cnt) {
          const unsigned long long* t = &ts[g * 4096 + 4 * j];
          m += (double)(t[1] - t[0]); bm += (double)(t[2] - t[1]); v += (double)(t[3] - t[2]); bv += (double)(t[4] - t[3]);
        }
        printf("  wave %d (ticks, mean of %d tiles): M %.0f  M-wait %.0f  V %.0f  V-wait %.0f\n", g, cnt, m / cnt, bm / cnt,
               v / cnt, bv / cnt);
      }
    };
    AttnSet t0 = h0;
    t0.o = O;
    show("stamps: full", [&] { return attention_h3pp_launch<64, 1, 1, 16>(t0, h1, B, H, scale, 0); });
    {  // raw timeline of tile 10: each wave's stamps relative to wave 0's first stamp of the tile
      const int j = 10;
      const unsigned long long base = ts[0 * 4096 + 4 * j];
      for (int w = 0; w < 8; ++w) {
        printf("  raw w%d:", w);
        for (int k = 0; k < 9; ++k) printf(" %7lld", (long long)(ts[w * 4096 + 4 * j + k] - base));
        printf("\n");
      }
    }
    show("stamps: no copies", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 8>(t0, h1, B, H, scale, 0); });
    show("stamps: no LDS reads", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: no reads/copies", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 8 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: MFMA only", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 32 + 8 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: no reads/copies, empty V", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 32 + 8 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: no reads/copies/barriers", [&] { return attention_h3pp_launch<64, 1, 1, 64 + 16 + 8 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: no reads/copies, lock-step", [&] { return attention_h3pp_launch<64, 0, 1, 16 + 8 + 4>(t0, h1, B, H, scale, 0); });
    show("stamps: full, empty V", [&] { return attention_h3pp_launch<64, 1, 1, 16 + 32>(t0, h1, B, H, scale, 0); });
  }
  run("h3p w8 kt64 occ2", [&] { return attention_h3p_launch<8, 64, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3p w4 kt64 occ2", [&] { return attention_h3p_launch<4, 64, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  run("h3 w4 kt64 occ2", [&] { return attention_h3_launch<4, 64, 2>(h0, h1, B, H, scale, 0); }, B, H, h0, h1, Oref, O, on);
  return 0;
}
