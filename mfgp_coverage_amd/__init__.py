"""mfgp_coverage_amd -- MI355X-native GP posterior engine for the coverage-control loop
of MSU-dcypherlab/mfgp-coverage.

``from mfgp_coverage_amd.gaussian_process import SFGP, MFGP`` is the drop-in for
the reference's ``from gaussian_process import MFGP, SFGP`` (simulator.py:25).
The compute path is libmfgp_hip.so (HIP for gfx950, C ABI in include/mfgp_hip.h).
"""
from ._lib import context, set_deferred_appends, set_device  # noqa: F401
from .gaussian_process import MFGP, SFGP, DiagCov  # noqa: F401

__all__ = ["SFGP", "MFGP", "DiagCov", "context", "set_device", "set_deferred_appends"]
