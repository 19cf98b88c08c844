"""cf2sim -- MI355X-native batched CrazyFlie hover environments (drop-in for the hover envs of
phoenix_drone_simulation, the package of Hu-Hanyang/disturbance-CrazyFile-simulation).

* ``BatchedCrazyflieEnv``: N envs per GPU, one fused HIP kernel per env-step (vec_env.py).
* ``make(id)``: single-env gym-style adapter with the reference's ids, spaces and 4-tuple API.
* ``cf2sim.physics``: the reference's physics plugin classes (``PybulletPhysicsWithAdversary``, ...,
  ``HipBatchedPhysics``) over the HIP physics kernel, for ``getattr(module, physics)`` lookups.
"""
from .config import (ENV_SPECS, OUT_OF_SCOPE_IDS, REFERENCE_IDS, CF2Config, build_config,  # noqa: F401
                     spec_for_id)

__all__ = ["ENV_SPECS", "REFERENCE_IDS", "OUT_OF_SCOPE_IDS", "CF2Config", "build_config", "spec_for_id",
           "BatchedCrazyflieEnv", "make", "registry"]


def __getattr__(name):   # lazy: importing the package must not require torch / a GPU
    if name == "BatchedCrazyflieEnv":
        from .vec_env import BatchedCrazyflieEnv
        return BatchedCrazyflieEnv
    if name in ("make", "registry"):
        from . import registration
        return getattr(registration, name)
    raise AttributeError(name)
