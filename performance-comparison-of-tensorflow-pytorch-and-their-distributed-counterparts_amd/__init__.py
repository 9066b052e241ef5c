"""pcmp: MI355X-native training / inference benchmark framework (see README.md).

Process-level HIP runtime settings are applied here, at import, because the HIP runtime reads them
once when it initialises (the first device query), before any pcmp or torch.cuda call:

* ``GPU_MAX_HW_QUEUES`` (at least 8 here; HIP's own default, and the value the GPU pool exports, is
  4): every HIP stream is bound to a hardware queue when it is created, round-robin over this many.
  A pcmp training process uses the compute stream, the WGRAD/downsample side stream, the DDP comm
  stream and RCCL's streams; with 4 queues the side stream landed on the compute stream's queue
  once the RCCL streams existed, which serialises WGRAD behind DGRAD and RCCL's ring kernels behind
  backward (measured: ResNet-50 22.2 -> 24.9 ms/step with the RCCL path active, all step kernels on
  one queue in the rocprofv3 trace, ``profiles/r2_ddp_force_queues.txt``).  A smaller inherited
  value is raised to 8 (a larger one is kept); ``PCMP_HW_QUEUES=<n>`` pins the count exactly.
"""
import os as _os
import sys as _sys

MIN_HW_QUEUES = 8


def ensure_hw_queues(environ=_os.environ) -> int:
    """Set ``GPU_MAX_HW_QUEUES`` for this process (must run before the HIP runtime initialises)."""
    pin = environ.get("PCMP_HW_QUEUES", "").strip()
    if pin:
        try:
            n = min(32, max(1, int(pin)))
        except ValueError:
            n = MIN_HW_QUEUES
    else:
        try:
            cur = int(environ.get("GPU_MAX_HW_QUEUES", "0"))
        except ValueError:
            cur = 0
        n = min(32, max(cur, MIN_HW_QUEUES))
        if cur and n != cur and environ.get("PCMP_QUIET") != "1":
            # the override is deliberate (see above) but never silent
            print(f"[pcmp] GPU_MAX_HW_QUEUES {cur} -> {n} (compute + side + comm + RCCL streams; "
                  f"PCMP_HW_QUEUES=<n> pins it)", file=_sys.stderr)
    environ["GPU_MAX_HW_QUEUES"] = str(n)
    return n


def _hip_already_initialised() -> bool:
    torch = _sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:
        return False


if _hip_already_initialised():
    import warnings as _w
    _w.warn("pcmp imported after the HIP runtime initialised: GPU_MAX_HW_QUEUES can no longer take effect "
            "for this process (import pcmp before any torch.cuda call)", RuntimeWarning)
ensure_hw_queues()
