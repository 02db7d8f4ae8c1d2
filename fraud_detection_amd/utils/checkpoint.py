"""Training checkpoints for resume (SURVEY.md §5.4 "native checkpoint for resume").

A checkpoint is one safetensors file: tensors (solver state, trees so far, ...) plus a JSON
metadata blob (step counters, RNG counters, data-shard cursor, config signature).  Files are
written to a temporary name and renamed, so a crash mid-write never leaves a torn checkpoint;
``CheckpointManager`` keeps the newest ``keep`` of them.  Loading uses safetensors only (no
pickle), so a checkpoint from an untrusted source cannot execute code.

Under data parallelism only rank 0 writes (all ranks hold identical solver state after the
all-reduces); every rank loads the same file from shared storage on resume.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import re
import tempfile

import numpy as np
import torch
from safetensors.torch import load_file, save_file

_META_KEY = "fdx_meta"


def _to_cpu_tensors(tensors: dict) -> dict:
    out = {}
    for k, v in tensors.items():
        t = torch.from_numpy(np.ascontiguousarray(v)) if isinstance(v, np.ndarray) else v
        out[k] = t.detach().to("cpu").contiguous()
    return out


def save_checkpoint(path: str, tensors: dict, meta: dict) -> str:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".ckpt_", dir=d)
    os.close(fd)
    try:
        save_file(_to_cpu_tensors(tensors), tmp, metadata={_META_KEY: json.dumps(meta, default=float)})
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return path


def load_checkpoint(path: str) -> tuple[dict, dict]:
    from safetensors import safe_open

    with safe_open(path, framework="pt") as f:
        meta = json.loads((f.metadata() or {}).get(_META_KEY, "{}"))
    return load_file(path), meta


def config_signature(**items) -> str:
    """Stable hash of everything that must match for a resume to be valid."""
    blob = json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in sorted(items.items())},
                      sort_keys=True, default=str)
    return hashlib.sha256(blob.encode()).hexdigest()[:16]


class CheckpointManager:
    """Numbered checkpoints ``<prefix>-<step>.safetensors`` in ``directory``."""

    def __init__(self, directory: str, prefix: str = "ckpt", keep: int = 2, rank: int = 0):
        self.dir, self.prefix, self.keep, self.rank = directory, prefix, max(1, keep), rank

    def _files(self):
        pat = re.compile(rf"{re.escape(self.prefix)}-(\d+)\.safetensors$")
        out = []
        for f in glob.glob(os.path.join(self.dir, f"{self.prefix}-*.safetensors")):
            m = pat.search(os.path.basename(f))
            if m:
                out.append((int(m.group(1)), f))
        return sorted(out)

    def save(self, step: int, tensors: dict, meta: dict) -> str | None:
        if self.rank != 0:
            return None
        path = os.path.join(self.dir, f"{self.prefix}-{int(step)}.safetensors")
        save_checkpoint(path, tensors, {**meta, "step": int(step)})
        for _, f in self._files()[: -self.keep]:
            os.remove(f)
        return path

    def latest(self, signature: str | None = None):
        """(tensors, meta) of the newest checkpoint whose signature matches, else None."""
        for _, f in reversed(self._files()):
            try:
                tensors, meta = load_checkpoint(f)
            except Exception:  # noqa: BLE001 - unreadable file: try the previous one
                continue
            if signature is None or meta.get("signature") == signature:
                return tensors, meta
        return None
