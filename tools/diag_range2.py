import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import lgamd  # noqa
from lightglue_amd import LightGlue
from lightglue_amd.weights import synthetic_pair, synthetic_state_dict
os.environ["LG_DEBUG_RANGE"] = "1"
conf = {"filter_threshold": 0.1, "n_layers": 2}
sd = synthetic_state_dict(conf, seed=0)
m = LightGlue(conf).cuda()
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
data = synthetic_pair(B=1, M=128, N=120, seed=2)
data["descriptors0"] = data["descriptors0"] * np.float32(2e5)
g = {k: torch.from_numpy(v).cuda() for k, v in data.items() if not k.startswith("image_size")}
g["view0"] = {"image_size": torch.from_numpy(data["image_size0"]).cuda()}
g["view1"] = {"image_size": torch.from_numpy(data["image_size1"]).cuda()}
with torch.no_grad():
    a = m(g)  # training mode: every layer
for i in range(2):
    d = a["ref_descriptors0"][0, i]
    print("layer", i, "nan", int(torch.isnan(d).sum()), "max", float(d[~torch.isnan(d)].abs().max()), flush=True)
