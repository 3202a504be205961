"""MI355X-native IR->RGB colorization GAN train step.

Drop-in for the hot path of yavuzmurattas/Infrared-Colorization-with-ResNet-
Generator-and-PatchGAN (Code/ir_colorization.py): the Config / generator /
discriminator / loss API and the generator checkpoint layout are kept; the
compute runs on hand-written gfx950 HIP kernels (libirgan.so, C ABI in
include/irgan.h).  Import with importlib (the directory name is not an
identifier)::

    irc = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd")
    cfg = irc.Config(); model = irc.IRColorizationModel(cfg)
"""
from . import _lib, ops  # noqa: F401

try:  # the public API pulls in the engine; keep ops importable on its own
    from .ir_colorization import *  # noqa: F401,F403
    from .ir_colorization import __all__ as _api_all
except ImportError as _e:  # pragma: no cover - only while the API module is absent
    if "ir_colorization" not in str(_e):
        raise
    _api_all = []

__all__ = ["_lib", "ops"] + list(_api_all)

from . import inference  # noqa: E402,F401  -- batched test-mode path
from . import data  # noqa: E402,F401  -- KAIST pipeline, device resize
from . import evaluation  # noqa: E402,F401  -- run_test, metrics CSV, Top-K
