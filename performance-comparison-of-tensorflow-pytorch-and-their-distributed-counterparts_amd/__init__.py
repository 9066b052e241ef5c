"""pcmp: MI355X-native training / inference benchmark framework (see README.md).

Process-level HIP runtime settings are applied here, at import, because the HIP runtime reads them
once when it initialises (the first device query), before any pcmp or torch.cuda call:

* ``GPU_MAX_HW_QUEUES`` (default 8 here, HIP's own default is 4): every HIP stream is bound to a
  hardware queue when it is created, round-robin over this many.  A pcmp training process uses
  the compute stream, the WGRAD/downsample side stream, the DDP comm stream and RCCL's streams;
  with 4 queues the side stream landed on the compute stream's queue once the RCCL streams
  existed, which serialises WGRAD behind DGRAD and RCCL's ring kernels behind backward (measured:
  ResNet-50 22.3 -> 25.3 ms/step with the forced RCCL path, all step kernels on one queue in the
  rocprofv3 trace, ``profiles/r2_ddp_force_queues.txt``).  An explicit setting is kept.
"""
import os as _os

_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
