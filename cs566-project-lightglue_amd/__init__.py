"""MI355X-native LightGlue matcher (gfx950 HIP kernels behind a C-ABI library).

Drop-in for ``gluefactory.models.matchers.lightglue.LightGlue``: same config keys, same
state-dict schema, same ``forward(data) -> dict`` contract.  Import through ``lgamd`` (the
directory name is not an identifier)::

    import lgamd
    from lightglue_amd import LightGlue
"""
from .weights import DEFAULT_CONF, state_dict_schema, synthetic_pair, synthetic_state_dict  # noqa: F401


def __getattr__(name):
    # Lazy: importing the package must not require torch-ROCm or the HIP library.
    if name in ("LightGlue", "__main_model__"):
        from .lightglue import LightGlue

        return LightGlue
    if name == "SuperPoint":
        from .superpoint import SuperPoint

        return SuperPoint
    if name in ("SuperGlue", "NLLLoss"):
        from . import superglue

        return getattr(superglue, name)
    if name in ("log_optimal_transport", "filter_matches"):
        from . import assignment

        return getattr(assignment, name)
    raise AttributeError(name)
