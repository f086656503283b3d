"""capk — MI355X (gfx950) compute backend for image captioning.

Drop-in for the reference's plugin surface (thromel/Image-Captioning-ML-Project):
``capk.models.encoders.build_encoder``, ``capk.models.decoders.build_decoder``,
``capk.models.captioning_model.ImageCaptioningModel``, ``capk.train.CombinedLoss``,
``capk.config`` — computing on hand-written HIP kernels in ``libcapk.so``.
"""
import torch

from . import _lib, ops  # noqa: F401
from .models.common import set_precision
from .params import attach

__version__ = "0.1.0"


def prepare(model, device="cuda", precision="bf16"):
    """Move `model` to the GPU, re-home its parameters into the flat ParamStore and
    select the kernel precision ('bf16' throughput path, 'fp32' parity path, 'fp8' =
    bf16 with the large forward Linear / Conv1D products on e4m3 scaled MFMA -- config 5)."""
    _lib.load()
    model.to(device)
    store = attach(model, device)
    set_precision(model, "bf16" if precision == "fp8" else precision)
    if precision == "fp8":
        ops.FP8.enable(store)
    elif ops.FP8.enabled:
        ops.FP8.disable()
    return store
