/*
 * superpoint_mi355x.h — C-ABI of the MI355X-native SuperPoint extractor (gfx950 HIP kernels),
 * part of liblightglue_mi355x.so.
 *
 * The reference exposes this path as a Python plugin, not an FFI:
 *   gluefactory_nonfree/superpoint.py:152-356  class SuperPoint(BaseModel)
 *     _init(conf)           :174-200  -> sp_create + sp_load_weights
 *     _forward(data) -> dict :202-350  -> sp_workspace_bytes + sp_forward (+ sp_sample_descriptors
 *                                        for keypoints the caller adds: force_num_keypoints padding)
 * The Python drop-in (lightglue_amd.superpoint.SuperPoint) binds it with ctypes; INTEGRATION.md.
 *
 * Conventions: as lightglue_mi355x.h (caller-owned device memory, stream-ordered work, int status
 * + lg_last_error(), one handle per device, not re-entrant).  fp32 in and out; the convolutions
 * run on the fp16 matrix cores with fp32-accurate products (fp16x3).
 */
#ifndef SUPERPOINT_MI355X_H
#define SUPERPOINT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sp_handle sp_handle_t;

/* SuperPoint.default_conf (superpoint.py:153-169); training-only keys stay host-side. */
typedef struct {
  int32_t has_detector;        /* 1 */
  int32_t has_descriptor;      /* 1 */
  int32_t descriptor_dim;      /* 256 (the only value the kernels support) */
  int32_t nms_radius;          /* 4 (0..8) */
  int32_t refinement_radius;   /* 0 = off */
  int32_t remove_borders;      /* 4 (0 = off) */
  int32_t legacy_sampling;     /* 1: superpoint.py:117-133, 0: :138-149 */
  float detection_threshold;   /* 0.005, strict '>' */
} sp_config_t;

typedef struct {
  int32_t B, C, H, W;          /* C = 1 (gray) or 3 (RGB, converted with 0.299/0.587/0.114) */
  const float* image;          /* device [B,C,H,W] */
  const float* image_size;     /* device [B,2] (w,h) or NULL: border removal at the true size */
  int32_t max_keypoints;       /* k > 0: the k best per image, sorted by score (ties: lower pixel
                                * index first); <= 0: every keypoint, row-major (superpoint.py:266-294) */
  int32_t sparse;              /* 0: dense outputs only (sparse_outputs = False) */
} sp_inputs_t;

/* Shapes: Hc = floor(floor(floor(H/2)/2)/2), Wc likewise (the encoder's three floor pools);
 * the score map is [B, 8 Hc, 8 Wc]. */
typedef struct {
  float* dense_scores;         /* device [B,8Hc,8Wc] or NULL (keypoint_scores of the dense outputs) */
  float* dense_descriptors;    /* device [B,Hc,Wc,D] (NHWC) or NULL; L2-normalised per cell */
  int32_t capacity;            /* keypoint slots per image in the arrays below */
  float* keypoints;            /* device [B,capacity,2] (x,y) + 0.5 (superpoint.py:342) */
  float* keypoint_scores;      /* device [B,capacity] */
  float* descriptors;          /* device [B,capacity,D] or NULL (then sample later) */
  int32_t* counts;             /* device [B]: keypoints per image (<= capacity) */
  int32_t* host_counts;        /* host [B] or NULL: filled after one stream synchronisation */
} sp_outputs_t;

int sp_create(const sp_config_t* cfg, int device, sp_handle_t** out);
int sp_destroy(sp_handle_t* h);

/* State-dict schema (superpoint.py:179-196): conv1a..conv4b, convPa/convPb, convDa/convDb. */
int sp_weight_count(const sp_handle_t* h);
const char* sp_weight_name(const sp_handle_t* h, int index);
int64_t sp_weight_numel(const sp_handle_t* h, int index);
int sp_load_weights(sp_handle_t* h, int n, const char* const* names, const float* const* tensors,
                    const int64_t* numels, void* stream);

/* Device scratch for this image shape and keypoint capacity (bytes). */
int sp_workspace_bytes(const sp_handle_t* h, int32_t B, int32_t C, int32_t H, int32_t W, int32_t capacity,
                       size_t* bytes);

/* SuperPoint._forward in eval mode.  Asynchronous unless host_counts is given.  With sparse = 1
 * and max_keypoints <= 0 the capacity must hold every candidate (8Hc * 8Wc is always enough). */
int sp_forward(sp_handle_t* h, const sp_inputs_t* in, sp_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream);

/* Descriptors at arbitrary (x,y) keypoints [B,capacity,2] (without the +0.5) from the dense map
 * the last sp_forward on this workspace produced: bilinear + L2 norm (superpoint.py:117-149).
 * counts: device [B].  Used for force_num_keypoints padding (superpoint.py:304-317). */
int sp_sample_descriptors(sp_handle_t* h, const float* keypoints, const int32_t* counts, int32_t B, int32_t capacity,
                          float* descriptors, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SUPERPOINT_MI355X_H */
