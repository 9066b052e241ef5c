"""Shared CLI plumbing for the entry points (SURVEY §5.6 config/flag system).

Every reference constant becomes a flag whose default is the reference value;
``--preset`` selects the BASELINE.json configs; ``--local_rank`` (legacy launcher) and
``LOCAL_RANK`` (torchrun) are both honoured; ``--synthetic`` (default) vs ``--data-dir``.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os

PRESETS = {
    # BASELINE.json configs
    "mlp-cpu": dict(model="mlp", device="cpu", epochs=1, batch_size=64),
    "resnet18-1gpu": dict(model="resnet18", full_train=True, epochs=1, batch_size=256),
    "resnet50-ddp8": dict(model="resnet50", full_train=True, epochs=1, batch_size=256),
    "resnet50-tl-infer": dict(model="resnet50", epochs=1, batch_size=64, num_images=1000),
    "bilstm-ddp8": dict(model="bilstm", epochs=3, batch_size=32),
    "bert-distr": dict(model="bert", epochs=3, batch_size=32),
}


def common_parser(desc):
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--local_rank", "--local-rank", type=int, default=None)
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None)
    ap.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto")
    ap.add_argument("--synthetic", action="store_true", default=True)
    ap.add_argument("--data-dir", default=None, help="real dataset path (overrides --synthetic)")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--kernels", choices=["hip", "torch"], default="hip",
                    help="torch = PyTorch reference ops (parity runs only)")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="compute precision of the HIP kernels: bf16 (default) or fp32, the reference's "
                         "precision (fp32 kernels of csrc/f32.hip)")
    ap.add_argument("--weights", default=None,
                    help="pretrained weights (torchvision ResNet/VGG or HF BERT state_dict; .pth/.pt loaded with "
                         "torch.load(weights_only=True), or .safetensors) -- the reference's pretrained backbones")
    ap.add_argument("--weights-vgg", default=None, help="pretrained VGG16 weights where a script runs both families")
    ap.add_argument("--json", default=None, help="append a JSON metrics record to this file")
    ap.add_argument("--profile", default=None,
                    help="torch.profiler chrome trace path (per-rank suffix .rankN under DDP)")
    ap.add_argument("--reference-compat", action="store_true",
                    help="reproduce the reference's printed-value quirks (SURVEY §0.2)")
    ap.add_argument("--verbose", action="store_true", help="per-step prints (reference behaviour)")
    ap.add_argument("--watchdog", type=float, default=0.0, help="hang watchdog timeout (s), 0=off")
    return ap


def apply_preset(args, defaults: dict):
    d = dict(defaults)
    if args.preset:
        d.update(PRESETS[args.preset])
    for k, v in d.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    return args


def setup(args):
    import torch

    import pcmp  # noqa: F401
    from ..ops import _lib
    from ..parallel import launch
    from ..utils.misc import seed_everything
    _lib.set_backend(args.kernels)
    _lib.set_precision(getattr(args, "dtype", "bf16"))
    use_gpu = torch.cuda.is_available() if args.device == "auto" else args.device == "cuda"
    env = launch.init(args.local_rank, use_gpu=use_gpu)
    seed_everything(args.seed + (0 if args.kernels else 0))
    return env


@contextlib.contextmanager
def run_context(args, env):
    """Operational wrappers every entry point runs its work under: ``--watchdog S`` (hang
    detector, kicked by the engine loops; aborts the rank under DDP so the job does not hang) and
    ``--profile PATH`` (torch.profiler Chrome trace with ROCm kernel activity)."""
    from ..utils.misc import Watchdog, chrome_trace
    with contextlib.ExitStack() as stack:
        if getattr(args, "watchdog", 0) and args.watchdog > 0:
            stack.enter_context(Watchdog(args.watchdog, abort=bool(getattr(env, "distributed", False))))
        path = getattr(args, "profile", None)
        if path and getattr(env, "world_size", 1) > 1:
            path = f"{path}.rank{env.rank}"
        stack.enter_context(chrome_trace(path))
        yield


def read_state_dict(path: str) -> dict:
    """A state_dict from ``path`` through loaders that execute nothing from the file: safetensors,
    or ``torch.load(weights_only=True)``.  A checkpoint written by :mod:`pcmp.utils.checkpoint`
    (``{"model": state_dict, ...}``) is unwrapped."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    import torch
    obj = torch.load(path, map_location="cpu", weights_only=True)
    for key in ("state_dict", "model"):
        if isinstance(obj, dict) and isinstance(obj.get(key), dict):
            obj = obj[key]
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: not a state_dict")
    return obj


def load_pretrained(model, path: str | None, load_head: bool | None = None):
    """``--weights PATH``: load pretrained weights into a framework model (ResNet / VGG16:
    torchvision layout; BERT: HF layout).  No-op without a path.  Returns the model."""
    if not path:
        return model
    sd = read_state_dict(path)
    if hasattr(model, "load_torchvision"):
        if load_head is None:
            model.load_torchvision(sd)
        else:
            model.load_torchvision(sd, load_head=load_head)
    elif hasattr(model, "load_hf"):
        model.load_hf(sd)
    else:
        raise ValueError(f"--weights: {type(model).__name__} has no pretrained-weight loader")
    from ..utils.report import rprint
    rprint(f"[pcmp] loaded pretrained weights from {path}")
    return model


def write_json(args, record):
    from ..utils.report import emit_json, is_main
    emit_json(record)
    if args.json and is_main():
        with open(args.json, "a") as f:
            f.write(json.dumps(record, default=float) + "\n")


def env_info():
    return {"world_size": int(os.environ.get("WORLD_SIZE", "1")), "rank": int(os.environ.get("RANK", "0"))}
