"""Checkpoint / resume of a training run.

The reference keeps no checkpoint code: its state is the Flux parameter tree of ``Model``
(``Flux.params(model)``, scripts/script.jl:84) plus the ``ADAM`` state the external training loop
holds (scripts/script.jl:85, src/simple_depth.jl:16,42).  Here that state is the flat parameter
vector in ``param_table`` order (conv weights as cross-correlation [cout][cin][kh][kw], as the
library stores them; the Julia shim flips them at its boundary) and the ADAM
moments / step count.  The file is safetensors: loading it executes nothing from the file.
"""
from __future__ import annotations

import hashlib
import json
from typing import Optional

from .model import ADAM, Model

_FORMAT = "md2hip-checkpoint-1"


def _table_digest(model: Model) -> str:
    h = hashlib.sha256()
    for name, shape, off in model.table:
        h.update(f"{name}:{','.join(map(str, shape))}:{off};".encode())
    return h.hexdigest()


def _model_meta(model: Model) -> dict:
    return {"arch": model.encoder.depth, "in_channels": model.encoder.in_channels,
            "scale_levels": list(model.depth_decoder.scale_levels), "numel": model.numel,
            "table_sha256": _table_digest(model)}


def save_checkpoint(path: str, model: Model, opt: Optional[ADAM] = None, extra: Optional[dict] = None):
    """Write ``model.flat`` (and ``opt``'s moments / step / hyper-parameters) to ``path``."""
    from safetensors.torch import save_file
    tensors = {"params": model.flat.detach().float().cpu().contiguous()}
    meta = {"format": _FORMAT, "model": _model_meta(model), "extra": extra or {}}
    if opt is not None:
        meta["adam"] = {"t": opt.t, "eta": opt.eta, "beta": list(opt.beta), "eps": opt.eps}
        if opt.m is not None:
            tensors["adam.m"] = opt.m.detach().float().cpu().contiguous()
            tensors["adam.v"] = opt.v.detach().float().cpu().contiguous()
    save_file(tensors, path, metadata={"md2hip": json.dumps(meta)})


def load_checkpoint(path: str, model: Model, opt: Optional[ADAM] = None) -> dict:
    """Restore ``model`` (and ``opt``) from ``path``; returns the stored ``extra`` dict.
    Raises ValueError when the file was written for a different architecture / parameter layout."""
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        raw = (f.metadata() or {}).get("md2hip")
        if raw is None:
            raise ValueError(f"{path}: not an md2hip checkpoint")
        meta = json.loads(raw)
        if meta.get("format") != _FORMAT:
            raise ValueError(f"{path}: unknown checkpoint format {meta.get('format')!r}")
        want = _model_meta(model)
        if meta["model"] != want:
            raise ValueError(f"{path}: checkpoint model {meta['model']} does not match {want}")
        params = f.get_tensor("params")
        keys = set(f.keys())
        m = f.get_tensor("adam.m") if "adam.m" in keys else None
        v = f.get_tensor("adam.v") if "adam.v" in keys else None
    if params.numel() != model.numel:
        raise ValueError(f"{path}: {params.numel()} parameters, model has {model.numel}")
    model.load_flat(params)
    if opt is not None:
        a = meta.get("adam")
        if a is None:
            raise ValueError(f"{path}: no optimiser state stored")
        opt.t, opt.eta, opt.beta, opt.eps = a["t"], a["eta"], tuple(a["beta"]), a["eps"]
        if m is not None:
            opt.m = m.to(model.device, model.flat.dtype)
            opt.v = v.to(model.device, model.flat.dtype)
        else:
            opt.m = opt.v = None
    return meta.get("extra", {})
