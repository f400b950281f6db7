"""Generate tests/golden/metric_auc.json: error lists and the AUCs the reference's own
``cal_error_auc`` (gluefactory/utils/tools.py:137-149) gives for them.

Run in the build container (the reference is at /root/reference; it is not needed at test time):
    python tests/golden/make_metric_golden.py
tools.py imports only the standard library, numpy and torch, so it is loaded by file path.
"""
import importlib.util
import json
import os
import warnings

import numpy as np

REF = "/root/reference/gluefactory/utils/tools.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metric_auc.json")


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


if __name__ == "__main__":
    main()
