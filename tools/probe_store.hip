// Per-CU global store throughput by access shape (tools only).  One 1024-thread workgroup per CU
// (256 workgroups, like the 256x256 GEMM tiles), each writing `per_wg` bytes with
// global_store_dwordx4; a wave instruction covers SEG-byte contiguous segments (64 lanes x 16 B =
// 1 KiB split into 1024/SEG segments spaced `gap` bytes apart).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_store.hip -o tools/probe_store.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SEG>
__global__ __launch_bounds__(1024) void store_kernel(float* out, size_t per_wg, size_t row_bytes, int reps) {
  // the workgroup's region: per_wg bytes laid out as rows of row_bytes; an instruction of wave w
  // writes segments of SEG bytes in 1024/SEG consecutive rows
  constexpr int LPS = SEG / 16;  // lanes per segment
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* base = reinterpret_cast<char*>(out) + (size_t)blockIdx.x * per_wg;
  const size_t rows = per_wg / row_bytes;
  const size_t segs_per_row = row_bytes / SEG;
  const size_t total_instr = per_wg / 1024;
  f32x4 v = {1.f, 2.f, 3.f, (float)lane};
  for (int rep = 0; rep < reps; ++rep)
    for (size_t ins = wave; ins < total_instr; ins += 16) {
      // instruction ins: rows (ins / segs_per_row) * (64 / LPS) .., segment column ins % segs_per_row
      const size_t rgrp = ins / segs_per_row, scol = ins % segs_per_row;
      const size_t row = rgrp * (64 / LPS) + lane / LPS;
      if (row >= rows) continue;
      char* p = base + row * row_bytes + scol * SEG + (lane % LPS) * 16;
      *reinterpret_cast<f32x4*>(p) = v;
    }
}

static int g_wgs = 256;
template <int SEG>
float run(float* buf, size_t per_wg, size_t row_bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(store_kernel<SEG>, dim3(g_wgs), dim3(1024), 0, 0, buf, per_wg, row_bytes, 1);
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(store_kernel<SEG>, dim3(g_wgs), dim3(1024), 0, 0, buf, per_wg, row_bytes, 1);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const size_t per_wg = 2u << 20;  // 2 MiB per workgroup, 512 MiB total
  float* buf;
  if (hipMalloc(&buf, per_wg * 256) != hipSuccess) return 1;
  size_t total = per_wg * 256;
  auto rep = [&](const char* name, float ms) {
    printf("%3d WGs %-34s %8.1f us  %6.2f TB/s  %5.1f B/clk/CU at 2.2 GHz\n", g_wgs, name, ms * 1e3,
           total / (ms * 1e-3) / 1e12, total / (ms * 1e-3) / g_wgs / 2.2e9);
  };
  for (int wgs : {16, 64}) {
    g_wgs = wgs;
    total = per_wg * wgs;
    rep("1 KiB contiguous per instr", run<1024>(buf, per_wg, 1024));
    rep("8 x 128 B (rows of 1 KiB)", run<128>(buf, per_wg, 1024));
  }
  g_wgs = 256;
  total = per_wg * 256;
  rep("1 KiB contiguous per instr", run<1024>(buf, per_wg, 1024));
  rep("2 x 512 B (rows of 1 KiB)", run<512>(buf, per_wg, 1024));
  rep("4 x 256 B (rows of 1 KiB)", run<256>(buf, per_wg, 1024));
  rep("8 x 128 B (rows of 1 KiB)", run<128>(buf, per_wg, 1024));
  rep("16 x 64 B (rows of 1 KiB)", run<64>(buf, per_wg, 1024));
  rep("8 x 128 B (rows of 4 KiB)", run<128>(buf, per_wg, 4096));
  rep("4 x 256 B (rows of 4 KiB)", run<256>(buf, per_wg, 4096));
  rep("1 KiB contiguous (rows 4 KiB)", run<1024>(buf, per_wg, 4096));
  return 0;
}
