"""Native library loading and backend selection.

Rule: an op on a GPU tensor runs the hand-written HIP kernel from ``_native/libpcmp_hip.so``
and raises loudly if that library is missing or failed to load (no silent eager fallback);
an op on a CPU tensor runs the PyTorch reference implementation in :mod:`pcmp.ops.ref`
(CPU plumbing config + numerics tests).  ``PCMP_KERNELS=torch`` (or
:func:`set_backend`) forces the reference path on GPU too — used only for A/B parity runs.
"""
from __future__ import annotations

import os
import pathlib
import threading

import torch

_PKG = pathlib.Path(__file__).resolve().parent.parent
# PCMP_LIB: load another build of the library (same-box A/B of compile-time variants, tools/build_variant.py)
LIB_PATH = pathlib.Path(os.environ["PCMP_LIB"]) if os.environ.get("PCMP_LIB") else _PKG / "_native" / "libpcmp_hip.so"

_lock = threading.Lock()
_loaded = False
_load_error: str | None = None
_backend = os.environ.get("PCMP_KERNELS", "hip").lower()
_compute_dtype: torch.dtype | None = None   # None: bf16 on the GPU, fp32 on the CPU


def load(build_if_missing: bool = False) -> bool:
    """Load the native op library into ``torch.ops.pcmp``.  Returns True on success."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not LIB_PATH.exists() and build_if_missing:
            from .. import _build
            _build.build(verbose=False)
        if not LIB_PATH.exists():
            _load_error = f"{LIB_PATH} not built (run __graft_entry__.build() or pcmp._build.build())"
            return False
        try:
            torch.ops.load_library(str(LIB_PATH))
            _loaded = True
            _load_error = None
        except Exception as e:  # pragma: no cover - depends on the environment
            _load_error = f"failed to load {LIB_PATH}: {e}"
        if _loaded:
            _apply_env_knobs()
        return _loaded


def _apply_env_knobs() -> None:
    """``PCMP_KNOBS="name=value,..."``: kernel-variant knobs (torch.ops.pcmp.set_knob) for whole-
    program A/B runs; the defaults are the measured-best variants."""
    spec = os.environ.get("PCMP_KNOBS", "")
    for item in filter(None, (t.strip() for t in spec.split(","))):
        name, _, val = item.partition("=")
        torch.ops.pcmp.set_knob(name.strip(), int(val))


def available() -> bool:
    return load()


def load_error() -> str | None:
    return _load_error


def set_backend(name: str) -> None:
    """'hip' (default) or 'torch' (reference ops on every device)."""
    global _backend
    assert name in ("hip", "torch"), name
    _backend = name


def backend() -> str:
    return _backend


def set_precision(name: str) -> None:
    """``--dtype``: 'bf16' (default; bf16 storage with fp32 accumulation) or 'fp32' (the
    reference's precision, SURVEY §0.1 / §5.6: another_neural_net.py:95-115 and nb :655-702 run
    fp32 everywhere).  Both stay on the HIP kernels: fp32 activations select the fp32 kernels of
    ``csrc/f32.hip`` (convolutions / Linear on v_mfma_f32_16x16x4_f32, BatchNorm, pooling, dropout,
    losses) and ``csrc/text_f32.hip`` (LayerNorm, attention, GELU / tanh, embedding, masked mean,
    the BiLSTM recurrence, Linear+GELU): no op falls back to PyTorch (``kernels.FP32_REF_OPS`` is
    empty)."""
    global _compute_dtype
    assert name in ("bf16", "fp32"), name
    _compute_dtype = torch.float32 if name == "fp32" else None


def precision() -> str:
    return "fp32" if _compute_dtype == torch.float32 else "bf16"


def default_compute_dtype(device: torch.device) -> torch.dtype:
    """Activation dtype of a model on ``device`` unless the model was given one explicitly."""
    if _compute_dtype is not None:
        return _compute_dtype
    return torch.bfloat16 if device.type == "cuda" else torch.float32


def use_native(t: torch.Tensor) -> bool:
    """True if ops on ``t`` must run the HIP kernels.  Raises if they are required but absent."""
    if not t.is_cuda or _backend == "torch":
        return False
    if not load():
        raise RuntimeError(
            "pcmp: GPU tensor given but the native HIP library is unavailable: "
            f"{_load_error}.  Refusing to fall back silently (set PCMP_KERNELS=torch to use the "
            "PyTorch reference path deliberately).")
    return True


def ops():
    load()
    return torch.ops.pcmp
