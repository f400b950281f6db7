"""Generate the metric golden vectors from the reference's own functions:

* tests/golden/metric_auc.json: error lists and the AUCs of ``cal_error_auc``
  (gluefactory/utils/tools.py:137-149);
* tests/golden/metric_corner_error.json: homography pairs, image sizes and the errors of
  ``homography_corner_error`` (gluefactory/geometry/homography.py:336-342).

Run in the build container (the reference is at /root/reference; it is not needed at test time):
    python tests/golden/make_metric_golden.py
tools.py imports only the standard library, numpy and torch, so it is loaded by file path;
geometry/homography.py (numpy, torch and its sibling geometry/utils.py) is imported through
synthetic ``gluefactory`` / ``gluefactory.geometry`` package objects whose ``__path__`` points
into the reference, so the training-stack ``__init__`` files are skipped (as in make_golden.py).
"""
import importlib
import importlib.util
import json
import os
import sys
import types
import warnings

import numpy as np
import torch

REF = "/root/reference/gluefactory/utils/tools.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metric_auc.json")
OUT_CORNER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metric_corner_error.json")


def corner_error_cases():
    for name, path in [("gluefactory", "gluefactory"), ("gluefactory.geometry", "gluefactory/geometry")]:
        m = types.ModuleType(name)
        m.__path__ = [os.path.join("/root/reference", path)]
        sys.modules.setdefault(name, m)
    hom = importlib.import_module("gluefactory.geometry.homography")
    g = torch.Generator().manual_seed(0)
    cases = []
    for i, dtype in enumerate([torch.float64] * 4 + [torch.float32] * 2):
        T_gt = torch.eye(3, dtype=torch.float64) + 0.2 * torch.randn(3, 3, generator=g, dtype=torch.float64) * torch.tensor(
            [[1, 1, 100], [1, 1, 100], [1e-3, 1e-3, 0]], dtype=torch.float64)
        T = T_gt + (0.01 * i) * torch.randn(3, 3, generator=g, dtype=torch.float64) * torch.tensor(
            [[1, 1, 50], [1, 1, 50], [1e-4, 1e-4, 0]], dtype=torch.float64)
        if i == 3:  # batched: [2,3,3] homographies, one image size
            T, T_gt = torch.stack([T, T_gt]), torch.stack([T_gt, T])
        size = torch.tensor([640.0 + 32 * i, 480.0 - 16 * i], dtype=torch.float64)
        err = hom.homography_corner_error(T.to(dtype), T_gt.to(dtype), size.to(dtype))
        cases.append({"T": T.tolist(), "T_gt": T_gt.tolist(), "image_size": size.tolist(),
                      "dtype": str(dtype).replace("torch.", ""), "error": err.double().reshape(-1).tolist()})
    with open(OUT_CORNER, "w") as f:
        json.dump({"cases": cases}, f, indent=1)
    print("wrote", OUT_CORNER)


def main():
    spec = importlib.util.spec_from_file_location("ref_tools", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(0)
    cases = {
        "uniform_0_8": rng.uniform(0, 8, 200).tolist(),
        "lognormal": np.exp(rng.normal(0.5, 1.0, 117)).tolist(),
        "with_inf": rng.uniform(0, 4, 50).tolist() + [float("inf")] * 5,
        "ties_and_exact_thresholds": [0.5, 1.0, 1.0, 3.0, 3.0, 4.9, 5.0, 5.0, 7.0],
        "single": [2.5],
    }
    out = {"thresholds": [1, 3, 5], "cases": {}}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # np.trapz deprecation inside the reference
        for name, errs in cases.items():
            aucs = mod.cal_error_auc(np.array(errs), [1, 3, 5])
            out["cases"][name] = {"errors": errs, "auc": [float(a) for a in aucs]}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)
    corner_error_cases()


if __name__ == "__main__":
    main()
