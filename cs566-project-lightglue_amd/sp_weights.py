"""SuperPoint state-dict schema, default config and deterministic recipes.

Schema: the ``nn.Conv2d`` modules that ``gluefactory_nonfree.superpoint.SuperPoint`` registers, in
registration order (reference ``superpoint.py:174-196``): the shared encoder ``conv1a .. conv4b``,
the detector head ``convPa`` / ``convPb`` (when ``has_detector``) and the descriptor head
``convDa`` / ``convDb`` (when ``has_descriptor``).

Recipes (tests, smoke and bench only; the product never calls them): the trained weights are a
network download (``superpoint.py:172,199``) and unavailable here, so

* :func:`superpoint_state_dict` draws He-scaled normal weights and small biases from a NumPy PCG64
  stream (the encoder then keeps O(1) activations through its ten convolutions), and
* :func:`synthetic_images` draws smooth images in [0, 1] (sums of random Gaussian blobs and
  sinusoids), so the detector sees structure rather than white noise.
"""
from collections import OrderedDict

import numpy as np

SP_DEFAULT_CONF = {  # superpoint.py:153-169 (+ the BaseModel keys, base_model.py:54-59)
    "name": None,
    "trainable": True,
    "freeze_batch_normalization": False,
    "timeit": False,
    "has_detector": True,
    "has_descriptor": True,
    "descriptor_dim": 256,
    "sparse_outputs": True,
    "dense_outputs": False,
    "nms_radius": 4,
    "refinement_radius": 0,
    "detection_threshold": 0.005,
    "max_num_keypoints": -1,
    "max_num_keypoints_val": None,
    "force_num_keypoints": False,
    "randomize_keypoints_training": False,
    "remove_borders": 4,
    "legacy_sampling": True,
}

_ENCODER = [("conv1a", 1, 64), ("conv1b", 64, 64), ("conv2a", 64, 64), ("conv2b", 64, 64),
            ("conv3a", 64, 128), ("conv3b", 128, 128), ("conv4a", 128, 128), ("conv4b", 128, 128)]


def superpoint_schema(conf=None):
    """[(name, shape)] in registration order (superpoint.py:179-196)."""
    c = dict(SP_DEFAULT_CONF, **(conf or {}))
    layers = [(n, ci, co, 3) for n, ci, co in _ENCODER]
    if c["has_detector"]:
        layers += [("convPa", 128, 256, 3), ("convPb", 256, 65, 1)]
    if c["has_descriptor"]:
        layers += [("convDa", 128, 256, 3), ("convDb", 256, int(c["descriptor_dim"]), 1)]
    out = []
    for n, ci, co, k in layers:
        out += [(f"{n}.weight", (co, ci, k, k)), (f"{n}.bias", (co,))]
    return out


def superpoint_state_dict(conf=None, seed=0, bias_scale=0.05):
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for name, shape in superpoint_schema(conf):
        if name.endswith(".weight"):
            fan = shape[1] * shape[2] * shape[3]
            v = rng.standard_normal(shape) * np.sqrt(2.0 / fan)
        else:
            v = rng.standard_normal(shape) * bias_scale
        sd[name] = v.astype(np.float32)
    return sd


def synthetic_images(B, C, H, W, seed=0, blobs=24):
    """[B, C, H, W] float32 in [0, 1]: Gaussian blobs + two sinusoids + a little noise."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    out = np.empty((B, C, H, W), np.float64)
    for b in range(B):
        for c in range(C):
            img = np.zeros((H, W))
            for _ in range(blobs):
                cy, cx = rng.random() * H, rng.random() * W
                s = 2.0 + rng.random() * 0.08 * max(H, W)
                img += (rng.random() * 2 - 1) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
            f = rng.random(4) * 0.3
            img += 0.3 * np.sin(f[0] * xx + f[1] * yy) * np.cos(f[2] * xx - f[3] * yy)
            img += rng.standard_normal((H, W)) * 0.02
            img -= img.min()
            out[b, c] = img / max(img.max(), 1e-9)
    return out.astype(np.float32)
