"""CPU oracle for the LightGlue matcher hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker (or, for the bench, as the timed CPU baseline).  The
product path (``cs566-project-lightglue_amd/``) never imports it and fails loudly when its HIP
library is missing.

Pinning: ``tests/golden/make_golden.py`` runs the real reference
(``/root/reference/gluefactory/models/matchers/lightglue.py`` and
``gluefactory_nonfree/superglue.py``) in the build container and commits its outputs under
``tests/golden/``; ``tests/test_oracle_golden.py`` checks this restatement against them.
"""
from .lightglue_ref import (  # noqa: F401
    confidence_threshold,
    filter_matches,
    lightglue_forward,
    log_optimal_transport,
    normalize_keypoints,
    positional_encoding,
    sigmoid_log_double_softmax,
)
