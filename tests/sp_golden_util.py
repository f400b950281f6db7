"""SuperPoint golden fixtures (tests/golden/sp_*.npz, tests/golden/make_superpoint_golden.py):
regenerate a case's inputs and weights from its recipe and load its reference outputs."""
import glob
import hashlib
import json
import os

import numpy as np

from lightglue_amd.sp_weights import superpoint_state_dict, synthetic_images

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sp_case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "sp_*.npz")))


def sha(arrs):
    h = hashlib.sha256()
    for k in sorted(arrs):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrs[k]).tobytes())
    return h.hexdigest()


def sp_load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    g = {k: z[k] for k in z.files if k != "meta_json"}
    g["meta"] = json.loads(str(z["meta_json"]))
    return g


def sp_case_inputs(meta):
    """(conf, state dict, data) of a case; data["image_size"] only when the case has one."""
    conf = dict(meta["conf"])
    sd = superpoint_state_dict(conf, seed=meta["w_seed"])
    image = synthetic_images(meta["B"], meta["C"], meta["H"], meta["W"], seed=meta["img_seed"])
    data = {"image": image}
    if meta["image_size"] is not None:
        data["image_size"] = np.asarray(meta["image_size"], np.float32)
    return conf, sd, data
