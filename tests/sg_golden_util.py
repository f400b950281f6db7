"""SuperGlue golden fixtures (tests/golden/sg_*.npz, tests/golden/make_superglue_golden.py):
regenerate a case's inputs, ground truth and weights from its recipe and load its reference
outputs."""
import glob
import json
import os
import sys

import numpy as np

from lightglue_amd.sg_weights import superglue_state_dict
from sp_golden_util import sha  # noqa: F401  (same hashing as the generator)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from make_superglue_golden import case_inputs, ground_truth  # noqa: E402


def sg_case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "sg_*.npz")))


def sg_load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    g = {k: z[k] for k in z.files if k != "meta_json"}
    g["meta"] = json.loads(str(z["meta_json"]))
    return g


def sg_case(meta):
    """(conf, state dict, data, ground truth) of a case.  data: the recipe inputs plus
    ``image_size`` or ``image_hw`` (the image-shape fallback)."""
    conf = dict(meta["conf"])
    sd = superglue_state_dict(conf, seed=meta["w_seed"])
    data = case_inputs(meta["B"], meta["M"], meta["N"], conf, meta["image_size"], meta["seed"])
    if meta["image_size"] is None:
        data["image_hw"] = tuple(meta["image_hw"])
    return conf, sd, data, ground_truth(meta["B"], meta["M"], meta["N"], meta["seed"])
