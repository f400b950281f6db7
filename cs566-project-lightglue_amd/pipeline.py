"""Callers on either side of the matcher: the two-view pipeline and the
model registry that resolve the matcher by name.

* :func:`get_model` — name -> model class, like ``gluefactory.models.get_model``
  (``models/__init__.py:7-30``): ``"matchers.lightglue"`` (and ``"lightglue"``) resolve to the HIP
  :class:`~lightglue_amd.lightglue.LightGlue` (the reference module's ``__main_model__``,
  ``lightglue.py:666``); ``"matchers.lightglue_pretrained_MINE"`` to the wrapper below;
  ``"two_view_pipeline"`` to :class:`TwoViewPipeline`.  Other components (extractors, filters,
  solvers) are supplied by the caller through :func:`register_model`.
* :class:`LightGluePreTrainedMINE` — the reference's BaseModel wrapper
  (``matchers/lightglue_pretrained_MINE.py:8-36``): builds the matcher from its config and forwards
  ``data`` unchanged.
* :class:`TwoViewPipeline` — ``models/two_view_pipeline.py:21-97``: extractor per view (or the
  view's ``cache`` when ``allow_no_extract``), then matcher / filter / solver, each called on the
  merged dict ``{**data, **pred}`` and its outputs merged into ``pred``.

Plain host-side plumbing: no arithmetic happens here; the matcher's forward is the HIP path.
"""
from torch import nn

from .lightglue import LightGlue, merge_conf

BASE_DEFAULT_CONF = {  # models/base_model.py:54-59
    "name": None,
    "trainable": True,
    "freeze_batch_normalization": False,
    "timeit": False,
}


class BaseModel(nn.Module):
    """The reference's BaseModel contract (``models/base_model.py:40-114``): class-level
    ``default_conf`` merged under the given config, ``required_data_keys`` checked recursively
    before ``_forward``; ``trainable: False`` freezes the parameters."""

    default_conf = {}
    required_data_keys = []

    def __init__(self, conf):
        super().__init__()
        self.conf = conf = merge_conf(BASE_DEFAULT_CONF, self.default_conf, conf)
        self.required_data_keys = list(self.required_data_keys)
        self._init(conf)
        if not conf.trainable:
            for p in self.parameters():
                p.requires_grad = False

    def _init(self, conf):
        raise NotImplementedError

    def _forward(self, data):
        raise NotImplementedError

    def forward(self, data):
        def check(expected, given):  # base_model.py:107-112
            for key in expected:
                assert key in given, f"Missing key {key} in data"
                if isinstance(expected, dict):
                    check(expected[key], given[key])

        check(self.required_data_keys, data)
        return self._forward(data)

    def loss(self, pred, data):
        raise NotImplementedError("training is out of scope for the MI355X matcher (SURVEY.md §2)")


class LightGluePreTrainedMINE(BaseModel):
    """matchers/lightglue_pretrained_MINE.py:8-36."""

    default_conf = {"features": "superpoint", **LightGlue.default_conf}
    required_data_keys = ["view0", "keypoints0", "descriptors0", "view1", "keypoints1", "descriptors1"]

    def _init(self, conf):
        self.net = LightGlue(dict(conf))

    def _forward(self, data):
        return self.net(data)


class TwoViewPipeline(BaseModel):
    """models/two_view_pipeline.py:21-97 (the eval path; ground-truth and loss are training-side)."""

    default_conf = {
        "extractor": {"name": None, "trainable": False},
        "matcher": {"name": None},
        "filter": {"name": None},
        "solver": {"name": None},
        "ground_truth": {"name": None},
        "allow_no_extract": False,
        "run_gt_in_forward": False,
    }
    required_data_keys = ["view0", "view1"]
    components = ["extractor", "matcher", "filter", "solver", "ground_truth"]

    def _init(self, conf):  # :44-60
        for k in self.components:
            if conf[k].name:
                setattr(self, k, get_model(conf[k].name)(dict(conf[k])))

    def extract_view(self, data, i):  # :62-77
        data_i = data[f"view{i}"]
        pred_i = data_i.get("cache", {})
        skip_extract = len(pred_i) > 0 and self.conf.allow_no_extract
        if self.conf.extractor.name and not skip_extract:
            pred_i = {**pred_i, **self.extractor(data_i)}
        elif self.conf.extractor.name and not self.conf.allow_no_extract:
            pred_i = {**pred_i, **self.extractor({**data_i, **pred_i})}
        return pred_i

    def _forward(self, data):  # :79-97
        pred0 = self.extract_view(data, "0")
        pred1 = self.extract_view(data, "1")
        pred = {**{k + "0": v for k, v in pred0.items()}, **{k + "1": v for k, v in pred1.items()}}
        for k in ("matcher", "filter", "solver"):
            if self.conf[k].name:
                pred = {**pred, **getattr(self, k)({**data, **pred})}
        if self.conf.ground_truth.name and self.conf.run_gt_in_forward:
            gt_pred = self.ground_truth({**data, **pred})
            pred.update({f"gt_{k}": v for k, v in gt_pred.items()})
        return pred


def _superpoint():
    from .superpoint import SuperPoint

    return SuperPoint


def _superglue():
    from .superglue import SuperGlue

    return SuperGlue


_REGISTRY = {
    "lightglue": LightGlue,
    "matchers.lightglue": LightGlue,
    "lightglue_pretrained_MINE": LightGluePreTrainedMINE,
    "matchers.lightglue_pretrained_MINE": LightGluePreTrainedMINE,
    "two_view_pipeline": TwoViewPipeline,
    # the extractor (gluefactory_nonfree/superpoint.py), resolved lazily
    "gluefactory_nonfree.superpoint": _superpoint,
    "extractors.superpoint": _superpoint,
    "superpoint": _superpoint,
    # the SuperGlue matcher (gluefactory_nonfree/superglue.py), resolved lazily
    "gluefactory_nonfree.superglue": _superglue,
    "superglue": _superglue,
}


def register_model(name, cls):
    """Make ``cls`` resolvable by :func:`get_model` (extractors, filters, solvers, ground truth)."""
    _REGISTRY[name] = cls


def get_model(name):
    """models/__init__.py:7-30: the name as given, or with the ``matchers.`` / ``extractors.``
    prefix the reference also tries (backward compatibility)."""
    for path in (name, f"matchers.{name}", f"extractors.{name}"):
        if path in _REGISTRY:
            obj = _REGISTRY[path]
            return obj() if obj in (_superpoint, _superglue) else obj
    paths = [name, f"gluefactory.models.{name}", f"gluefactory.models.extractors.{name}",
             f"gluefactory.models.matchers.{name}"]
    raise RuntimeError(f'Model {name} not found in any of [{" ".join(paths)}]')
