"""Device assembly of one csrc/*.hip file for gfx950 with the build's own flags (for spill checks and
instruction audits): python tools/device_asm.py bn.hip > /tmp/bn.s"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcmp import _build  # noqa: E402

inc, _, abi = _build._torch_paths()
src = _build.CSRC / sys.argv[1]
cmd = [_build.HIPCC, f"--offload-arch={_build.ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast",
       *_build._common_flags(inc, abi), "-x", "hip", "--offload-device-only", "-S", str(src), "-o", "-"]
sys.exit(subprocess.run(cmd).returncode)
