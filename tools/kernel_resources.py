"""Print VGPR / SGPR / scratch / occupancy of every kernel in a csrc/*.hip file (compile-time report).

Usage: python tools/kernel_resources.py igemm [filter]
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp._build as b  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "igemm"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
inc, _, abi = b._torch_paths()
src = b.CSRC / f"{name}.hip"
cmd = [b.HIPCC, f"--offload-arch={b.ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast", *b._common_flags(inc, abi),
       "-x", "hip", "-c", str(src), "-o", "/tmp/_kr.o", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]
r = subprocess.run(cmd, capture_output=True, text=True)
cur = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s*(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]|TotalSGPRs): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
    else:
        cur[k.split()[0]] = v
    if k.startswith("LDS") and flt in cur["name"]:
        print(f"vgpr={cur.get('VGPRs'):>4} agpr={cur.get('AGPRs'):>4} sgpr={cur.get('TotalSGPRs'):>4} "
              f"scratch={cur.get('ScratchSize'):>4} occ={cur.get('Occupancy'):>2}  {cur['name']}")
if r.returncode:
    print(r.stderr[-3000:])
