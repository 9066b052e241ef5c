"""RCCL (backend ``nccl``) data-parallel path on ONE GPU: the process group is initialised at
world size 1 and every gradient bucket's all-reduce is forced through RCCL from the DDP comm
stream (``PCMP_DDP_FORCE`` / ``bench.py --ddp-force``).  The round-end 8-GPU scaling run goes
through exactly this code with peers."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _why(r):
    """The first error lines of a failed child (a c10d watchdog abort ends in a long frame dump)."""
    lines = [ln for ln in r.stderr.splitlines() if ("rror" in ln or "WARN" in ln) and "frame #" not in ln]
    return "\n".join(lines[:12]) + "\n...\n" + r.stderr[-1500:]


def _env():
    return dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
                LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_forced_rccl_ddp_matches_local(gpu, grad_dtype):
    code = ("import json,pcmp; from pcmp.parallel.selftest import rccl_force_check; "
            f"print('RESULT', json.dumps(rccl_force_check('resnet18', '{grad_dtype}')))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_env())
    assert r.returncode == 0, _why(r)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["backend"] == "nccl"
    assert res["nbuckets"] >= 3, res
    assert res["ok_grad"], res
    assert res["ok_param"], res


def test_bench_ddp_force_rccl(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "2", "--batch-size", "32", "--ddp-force",
           "--grad-dtype", "bf16", "--infer-images", "20"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=_env())
    assert r.returncode == 0, _why(r)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["config"]["ddp_force"] is True and rec["config"]["grad_allreduce_dtype"] == "bf16"
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert 0 < rec["inference_p50_ms"] < 50
