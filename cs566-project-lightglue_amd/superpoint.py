"""MI355X-native SuperPoint extractor: drop-in for ``gluefactory_nonfree.superpoint.SuperPoint``
(reference ``superpoint.py:152-356``).

Same config keys (:153-169, plus the BaseModel keys), same ``nn.Conv2d`` parameter tree
(``conv1a .. conv4b``, ``convPa/convPb``, ``convDa/convDb``: checkpoints load unchanged with
``load_state_dict``), same ``forward(data) -> dict`` outputs (:341-350).  The forward is the HIP
path of ``liblightglue_mi355x.so`` (``include/superpoint_mi355x.h``): 3x3 convolutions as implicit
fp16x3 GEMMs with fused ReLU / 2x2 pooling, NMS, border removal, top-k selection and descriptor
sampling on the device.  No CPU fallback: CPU inputs raise.

Deliberate differences from the reference, all where it raises or cannot run here:

* the trained checkpoint is a download (:172,198-200); the module starts from PyTorch's default
  init and takes weights through ``load_state_dict`` (``strict=False`` as the reference);
* B > 1 without ``force_num_keypoints``: the reference fails at ``desc.transpose`` (``desc`` is a
  list, :330-344); here the per-image samples are stacked (identical arithmetic), which needs an
  equal keypoint count per image just like the reference's ``torch.stack`` at :319;
* top-k ties at the selection boundary keep the lower pixel index first (``torch.topk`` leaves it
  unspecified);
* ``randomize_keypoints_training`` (training only) raises NotImplementedError.
"""
import ctypes

import torch
from torch import nn

from . import _lib
from .lightglue import merge_conf
from .sp_weights import SP_DEFAULT_CONF


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class SuperPoint(nn.Module):
    default_conf = SP_DEFAULT_CONF
    required_data_keys = ["image"]
    checkpoint_url = "https://github.com/magicleap/SuperGluePretrainedNetwork/raw/master/models/weights/superpoint_v1.pth"

    def __init__(self, conf=None):
        super().__init__()
        self.conf = conf = merge_conf(self.default_conf, conf or {})
        if int(conf.descriptor_dim) != 256:
            raise ValueError("lightglue_amd.SuperPoint: descriptor_dim must be 256")
        c1, c2, c3, c4, c5 = 64, 64, 128, 128, 256  # superpoint.py:177-196
        self.relu = nn.ReLU(inplace=True)
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.conv1a = nn.Conv2d(1, c1, 3, 1, 1)
        self.conv1b = nn.Conv2d(c1, c1, 3, 1, 1)
        self.conv2a = nn.Conv2d(c1, c2, 3, 1, 1)
        self.conv2b = nn.Conv2d(c2, c2, 3, 1, 1)
        self.conv3a = nn.Conv2d(c2, c3, 3, 1, 1)
        self.conv3b = nn.Conv2d(c3, c3, 3, 1, 1)
        self.conv4a = nn.Conv2d(c3, c4, 3, 1, 1)
        self.conv4b = nn.Conv2d(c4, c4, 3, 1, 1)
        if conf.has_detector:
            self.convPa = nn.Conv2d(c4, c5, 3, 1, 1)
            self.convPb = nn.Conv2d(c5, 65, 1, 1, 0)
        if conf.has_descriptor:
            self.convDa = nn.Conv2d(c4, c5, 3, 1, 1)
            self.convDb = nn.Conv2d(c5, conf.descriptor_dim, 1, 1, 0)
        if not conf.trainable:
            for p in self.parameters():
                p.requires_grad = False
        self._handle = None
        self._handle_device = None
        self._weights_key = None
        self._ws = None

    # ------------------------------------------------------------ native handle
    def _lib_config(self):
        c = self.conf
        return _lib.SPConfig(int(bool(c.has_detector)), int(bool(c.has_descriptor)), int(c.descriptor_dim),
                             int(c.nms_radius), int(c.refinement_radius), int(c.remove_borders or 0),
                             int(bool(c.legacy_sampling)), float(c.detection_threshold))

    def _weights_signature(self):
        return tuple((id(m), n, t.data_ptr(), t._version) for m in self.modules() for n, t in m._parameters.items()
                     if t is not None)

    def _ensure_handle(self, device):
        lib = _lib.load()
        if self._handle is not None and self._handle_device != device:
            lib.sp_destroy(self._handle)
            self._handle = None
        if self._handle is None:
            h = ctypes.c_void_p()
            cfg = self._lib_config()
            _lib.check(lib.sp_create(ctypes.byref(cfg), device.index or 0, ctypes.byref(h)), "sp_create")
            self._handle, self._handle_device, self._weights_key = h, device, None
        key = self._weights_signature()
        if key != self._weights_key:
            sd = self.state_dict(keep_vars=True)
            names = list(sd)
            ts = []
            for n in names:
                t = sd[n].detach()
                if t.device != device or t.dtype != torch.float32:
                    raise RuntimeError(f"lightglue_amd.SuperPoint: parameter {n} is {t.dtype} on {t.device}; "
                                       f"move the module to {device} in fp32")
                ts.append(t.contiguous())
            arr_n = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
            arr_p = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
            arr_k = (ctypes.c_int64 * len(ts))(*[t.numel() for t in ts])
            stream = torch.cuda.current_stream(device).cuda_stream
            _lib.check(lib.sp_load_weights(self._handle, len(ts), arr_n, arr_p, arr_k, ctypes.c_void_p(stream)),
                       "sp_load_weights")
            torch.cuda.current_stream(device).synchronize()
            self._weights_key = key
        return lib

    def reload_weights(self):
        self._weights_key = None

    def _apply(self, fn, *args, **kwargs):
        self._weights_key = None
        return super()._apply(fn, *args, **kwargs)

    def __del__(self):
        try:
            if self._handle is not None and _lib._lib is not None:
                _lib._lib.sp_destroy(self._handle)
        except Exception:
            pass

    def _workspace(self, lib, device, B, C, H, W, cap):
        nb = ctypes.c_size_t()
        _lib.check(lib.sp_workspace_bytes(self._handle, B, C, H, W, cap, ctypes.byref(nb)), "sp_workspace_bytes")
        if self._ws is None or self._ws.numel() < nb.value or self._ws.device != device:
            self._ws = torch.empty(nb.value, dtype=torch.uint8, device=device)
        return self._ws, nb.value

    # ------------------------------------------------------------ forward (superpoint.py:202-350)
    def forward(self, data: dict) -> dict:
        for k in self.required_data_keys:
            assert k in data, f"Missing key {k} in data"
        c = self.conf
        image = data["image"]
        if not image.is_cuda:
            raise RuntimeError("lightglue_amd.SuperPoint runs on a HIP device; inputs are on the CPU")
        if image.dim() != 4 or image.shape[1] not in (1, 3):
            raise ValueError(f"image must be [B, 1 or 3, H, W], got {tuple(image.shape)}")
        device = image.device
        image = image.float().contiguous()
        B, C, H, W = image.shape
        Hc, Wc = H // 2 // 2 // 2, W // 2 // 2 // 2
        Hs, Ws = 8 * Hc, 8 * Wc
        sparse = bool(c.sparse_outputs)
        if sparse:
            assert c.has_detector and c.has_descriptor
        max_kps = int(c.max_num_keypoints)
        if not self.training and c.max_num_keypoints_val is not None:
            max_kps = int(c.max_num_keypoints_val)
        if self.training and c.randomize_keypoints_training and sparse and max_kps > 0:
            raise NotImplementedError("randomize_keypoints_training (torch.multinomial sampling) is training-only")
        cap = (max_kps if max_kps > 0 else Hs * Ws) if sparse else 0
        lib = self._ensure_handle(device)
        ws, nb = self._workspace(lib, device, B, C, H, W, cap)
        isz = data.get("image_size")
        isz = None if isz is None or not sparse else isz.to(device=device, dtype=torch.float32).contiguous()
        dense_scores = torch.empty((B, Hs, Ws), device=device) if c.has_detector else None
        dense_desc = torch.empty((B, Hc, Wc, 256), device=device) if c.has_descriptor else None
        kpts = scores = desc = counts = None
        host_counts = (ctypes.c_int32 * B)()
        if sparse:
            kpts = torch.empty((B, cap, 2), device=device)
            scores = torch.empty((B, cap), device=device)
            desc = torch.empty((B, cap, 256), device=device) if max_kps > 0 else None
            counts = torch.empty((B,), dtype=torch.int32, device=device)
        inp = _lib.SPInputs(B, C, H, W, _ptr(image), _ptr(isz), max_kps, int(sparse))
        out = _lib.SPOutputs(_ptr(dense_scores), _ptr(dense_desc), cap, _ptr(kpts), _ptr(scores), _ptr(desc),
                             _ptr(counts), ctypes.cast(host_counts, ctypes.c_void_p) if sparse else None)
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        _lib.check(lib.sp_forward(self._handle, ctypes.byref(inp), ctypes.byref(out), _ptr(ws), nb, stream), "sp_forward")
        pred = {}
        if dense_scores is not None:
            pred["keypoint_scores"] = dense_scores
        if dense_desc is not None:
            pred["descriptors"] = dense_desc.permute(0, 3, 1, 2)  # [B, D, Hc, Wc] view of the NHWC map
        if not sparse:
            return pred
        n = list(host_counts)
        n_max = max(n)
        if c.force_num_keypoints:
            kp = kpts[:, :max(n_max, max_kps)] - 0.5  # back to the sampling frame (+0.5 is exact)
            kp, sc = self._pad(kp, scores, n, max_kps, data, image)
            if desc is None or kp.shape[1] > cap:
                desc = torch.empty((B, kp.shape[1], 256), device=device)
            full = torch.full((B,), kp.shape[1], dtype=torch.int32, device=device)
            kp = kp.contiguous()
            _lib.check(lib.sp_sample_descriptors(self._handle, _ptr(kp), _ptr(full), B, kp.shape[1], _ptr(desc), _ptr(ws),
                                                 nb, stream), "sp_sample_descriptors")
            out_pred = {"keypoints": kp + 0.5, "keypoint_scores": sc, "descriptors": desc[:, :kp.shape[1]]}
        else:
            if len(set(n)) != 1:
                raise RuntimeError(f"stack expects each tensor to be equal size, but got keypoint counts {n} "
                                   "(superpoint.py:319; set max_num_keypoints or force_num_keypoints)")
            k = n[0]
            if desc is None:  # every keypoint kept: sample now that the count is known
                desc = torch.empty((B, k, 256), device=device)
                cnt = torch.full((B,), k, dtype=torch.int32, device=device)
                kp = (kpts[:, :k] - 0.5).contiguous()
                _lib.check(lib.sp_sample_descriptors(self._handle, _ptr(kp), _ptr(cnt), B, k, _ptr(desc), _ptr(ws), nb,
                                                     stream), "sp_sample_descriptors")
            out_pred = {"keypoints": kpts[:, :k], "keypoint_scores": scores[:, :k], "descriptors": desc[:, :k]}
        if c.dense_outputs:
            out_pred["dense_descriptors"] = pred["descriptors"]
        return out_pred

    def _pad(self, kp, scores, n, length, data, image):
        """pad_and_stack(mode="random_c") / (mode="zeros") of superpoint.py:304-317
        (models/utils/misc.py:19-70): uniform keypoints within each coordinate's [min, max] of the
        real ones (or the bounds when an image has none), zero scores.  torch's RNG, as the
        reference."""
        B = kp.shape[0]
        isz = data.get("image_size", torch.tensor(image.shape[-2:]))
        hi = float(isz.min().item())
        kps, scs = [], []
        for b in range(B):
            x, s = kp[b, :n[b]], scores[b, :n[b]]
            d = x.shape[0]
            assert d <= length
            if d < length:
                cols = []
                for i in range(2):
                    lo_i, hi_i = (x[:, i].min(), x[:, i].max()) if d > 0 else (0, hi)
                    cols.append(torch.empty(length - d, 1, device=kp.device).uniform_(float(lo_i), float(hi_i)))
                x = torch.cat([x, torch.cat(cols, -1)], 0)
                s = torch.cat([s, torch.zeros(length - d, device=kp.device)], 0)
            kps.append(x)
            scs.append(s)
        return torch.stack(kps, 0), torch.stack(scs, 0)

    def loss(self, pred, data):
        raise NotImplementedError

    def metrics(self, pred, data):
        raise NotImplementedError
