/*
 * lg_c_host.c -- a non-Python host of the C-ABI (include/lightglue_mi355x.h), in plain C99 with the
 * HIP runtime's C API for device memory.  It does what the reference's
 * LightGlue.__init__ + forward do (gluefactory/models/matchers/lightglue.py:367-430, 444-579) for
 * one batch: build the matcher from a state dict, match, write matches / scores.
 *
 *   lg_c_host <weights.bin> <inputs.bin> <outputs.bin> [filter_threshold [depth_confidence width_confidence]]
 *
 * weights.bin  "LGW1", u32 count, then per tensor: u32 name length, name bytes, i64 numel,
 *              numel float32 (the state-dict keys and PyTorch layouts, lightglue.py:367-398)
 * inputs.bin   "LGI1", i32 B, M, N, then float32 keypoints0 [B,M,2], keypoints1 [B,N,2],
 *              descriptors0 [B,M,256], descriptors1 [B,N,256], image_size0 [B,2], image_size1 [B,2]
 * outputs.bin  "LGO1", i32 B, M, N, then int64 matches0 [B,M], matches1 [B,N],
 *              float32 matching_scores0 [B,M], matching_scores1 [B,N]
 *
 * tests/test_gpu_c_host.py checks its outputs against the Python drop-in class on the same data.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lightglue_mi355x.h"

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define LG_OK_(x)                                                                    \
  do {                                                                               \
    int r_ = (x);                                                                    \
    if (r_ != LG_OK) {                                                               \
      fprintf(stderr, "%s failed (%d): %s\n", #x, r_, lg_last_error());            \
      exit(3);                                                                       \
    }                                                                                \
  } while (0)

static void read_exact(FILE* f, void* p, size_t n, const char* what) {
  if (fread(p, 1, n, f) != n) {
    fprintf(stderr, "short read: %s\n", what);
    exit(4);
  }
}

static void magic(FILE* f, const char* m) {
  char b[4];
  read_exact(f, b, 4, "magic");
  if (memcmp(b, m, 4) != 0) {
    fprintf(stderr, "bad file magic (want %.4s)\n", m);
    exit(4);
  }
}

/* host buffer of n floats from the file -> new device buffer */
static float* upload(FILE* f, size_t n, const char* what) {
  float* h = (float*)malloc(n * sizeof(float) + 1);
  float* d = NULL;
  read_exact(f, h, n * sizeof(float), what);
  HIP_OK(hipMalloc((void**)&d, n * sizeof(float) + 1));
  HIP_OK(hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice));
  free(h);
  return d;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s weights.bin inputs.bin outputs.bin [filter_threshold [depth_conf width_conf]]\n", argv[0]);
    return 1;
  }
  if (lg_abi_version() != LG_ABI_VERSION) {
    fprintf(stderr, "ABI mismatch: library %d, header %d\n", lg_abi_version(), LG_ABI_VERSION);
    return 1;
  }
  /* LightGlue.default_conf (lightglue.py:341-361) with the caller's filter_threshold and, optionally,
   * the adaptive depth / width confidences (early stop and point pruning, lightglue.py:502-540) */
  lg_config_t cfg = {256, 256, 9, 4, 0, argc > 6 ? atof(argv[5]) : -1.0, argc > 6 ? atof(argv[6]) : -1.0,
                     argc > 4 ? atof(argv[4]) : 0.0, LG_PREC_AUTO};
  lg_handle_t* h = NULL;
  LG_OK_(lg_create(&cfg, 0, &h));

  /* ---- the state dict (lg_load_weights copies and repacks; strict: every schema tensor once) */
  FILE* fw = fopen(argv[1], "rb");
  if (!fw) { perror(argv[1]); return 1; }
  magic(fw, "LGW1");
  uint32_t count = 0;
  read_exact(fw, &count, 4, "count");
  char** names = (char**)calloc(count, sizeof(char*));
  float** tensors = (float**)calloc(count, sizeof(float*));
  int64_t* numels = (int64_t*)calloc(count, sizeof(int64_t));
  for (uint32_t i = 0; i < count; ++i) {
    uint32_t len = 0;
    read_exact(fw, &len, 4, "name length");
    names[i] = (char*)calloc(len + 1, 1);
    read_exact(fw, names[i], len, "name");
    read_exact(fw, &numels[i], 8, "numel");
    tensors[i] = upload(fw, (size_t)numels[i], names[i]);
  }
  fclose(fw);
  LG_OK_(lg_load_weights(h, (int)count, (const char* const*)names, (const float* const*)tensors, numels, NULL));
  HIP_OK(hipDeviceSynchronize());  /* the sources may be freed once the stream is past the load */
  for (uint32_t i = 0; i < count; ++i) {
    HIP_OK(hipFree(tensors[i]));
    free(names[i]);
  }
  free(names);
  free(tensors);
  free(numels);

  /* ---- one batch of inputs */
  FILE* fi = fopen(argv[2], "rb");
  if (!fi) { perror(argv[2]); return 1; }
  magic(fi, "LGI1");
  int32_t shp[3];
  read_exact(fi, shp, sizeof(shp), "shape");
  const int32_t B = shp[0], M = shp[1], N = shp[2];
  lg_inputs_t in;
  memset(&in, 0, sizeof(in));
  in.B = B;
  in.M = M;
  in.N = N;
  in.keypoints0 = upload(fi, (size_t)B * M * 2, "keypoints0");
  in.keypoints1 = upload(fi, (size_t)B * N * 2, "keypoints1");
  in.descriptors0 = upload(fi, (size_t)B * M * 256, "descriptors0");
  in.descriptors1 = upload(fi, (size_t)B * N * 256, "descriptors1");
  in.image_size0 = upload(fi, (size_t)B * 2, "image_size0");
  in.image_size1 = upload(fi, (size_t)B * 2, "image_size1");
  fclose(fi);

  /* ---- outputs and workspace (caller-owned device memory) */
  lg_outputs_t out;
  memset(&out, 0, sizeof(out));
  HIP_OK(hipMalloc((void**)&out.matches0, (size_t)B * M * sizeof(int64_t)));
  HIP_OK(hipMalloc((void**)&out.matches1, (size_t)B * N * sizeof(int64_t)));
  HIP_OK(hipMalloc((void**)&out.matching_scores0, (size_t)B * M * sizeof(float)));
  HIP_OK(hipMalloc((void**)&out.matching_scores1, (size_t)B * N * sizeof(float)));
  if (cfg.width_confidence > 0) { /* point pruning reports each point's layer count */
    HIP_OK(hipMalloc((void**)&out.prune0, (size_t)B * M * sizeof(int64_t)));
    HIP_OK(hipMalloc((void**)&out.prune1, (size_t)B * N * sizeof(int64_t)));
  }
  size_t ws_bytes = 0;
  LG_OK_(lg_workspace_bytes(h, B, M, N, &ws_bytes));
  void* ws = NULL;
  HIP_OK(hipMalloc(&ws, ws_bytes));

  LG_OK_(lg_forward(h, &in, &out, ws, ws_bytes, NULL));
  HIP_OK(hipDeviceSynchronize());

  int64_t* m0 = (int64_t*)malloc((size_t)B * M * sizeof(int64_t));
  int64_t* m1 = (int64_t*)malloc((size_t)B * N * sizeof(int64_t));
  float* s0 = (float*)malloc((size_t)B * M * sizeof(float));
  float* s1 = (float*)malloc((size_t)B * N * sizeof(float));
  HIP_OK(hipMemcpy(m0, out.matches0, (size_t)B * M * sizeof(int64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(m1, out.matches1, (size_t)B * N * sizeof(int64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(s0, out.matching_scores0, (size_t)B * M * sizeof(float), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(s1, out.matching_scores1, (size_t)B * N * sizeof(float), hipMemcpyDeviceToHost));

  FILE* fo = fopen(argv[3], "wb");
  if (!fo) { perror(argv[3]); return 1; }
  fwrite("LGO1", 1, 4, fo);
  fwrite(shp, sizeof(int32_t), 3, fo);
  fwrite(m0, sizeof(int64_t), (size_t)B * M, fo);
  fwrite(m1, sizeof(int64_t), (size_t)B * N, fo);
  fwrite(s0, sizeof(float), (size_t)B * M, fo);
  fwrite(s1, sizeof(float), (size_t)B * N, fo);
  fclose(fo);

  long matched = 0;
  for (size_t i = 0; i < (size_t)B * M; ++i) matched += m0[i] > -1;
  printf("lg_c_host: B %d M %d N %d, %ld matches, stop layer %d (precision used %d)\n", B, M, N, matched,
         out.stop_layer, out.precision_used);

  free(m0); free(m1); free(s0); free(s1);
  HIP_OK(hipFree(ws));
  HIP_OK(hipFree(out.matches0)); HIP_OK(hipFree(out.matches1));
  HIP_OK(hipFree(out.matching_scores0)); HIP_OK(hipFree(out.matching_scores1));
  if (out.prune0) { HIP_OK(hipFree(out.prune0)); HIP_OK(hipFree(out.prune1)); }
  HIP_OK(hipFree((void*)in.keypoints0)); HIP_OK(hipFree((void*)in.keypoints1));
  HIP_OK(hipFree((void*)in.descriptors0)); HIP_OK(hipFree((void*)in.descriptors1));
  HIP_OK(hipFree((void*)in.image_size0)); HIP_OK(hipFree((void*)in.image_size1));
  LG_OK_(lg_destroy(h));
  return 0;
}
