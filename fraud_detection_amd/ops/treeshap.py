"""K7b interventional TreeSHAP device wrapper (csrc/kernels/treeshap.hip): exact SHAP values of a
tree ensemble's margin (log-odds) against a background set, one workgroup per explanation."""
from __future__ import annotations

import numpy as np
import torch

from .kernelshap import _check_x, _outputs
from .native import native, ptr, stream_of


def _device_design(expl, dev):
    key = (str(dev),)
    if expl._dev_cache is not None and expl._dev_cache[0] == key:
        return expl._dev_cache[1]
    from .scaler import stats_from_numpy

    ens = expl.ens
    t = {
        "feat": torch.from_numpy(np.ascontiguousarray(ens.feat, np.int32)).to(dev),
        "thr": torch.from_numpy(np.ascontiguousarray(ens.thr, np.float32)).to(dev),
        "leaf": torch.from_numpy(np.ascontiguousarray(ens.leaf, np.float32)).to(dev),
        "bw": torch.from_numpy(np.ascontiguousarray(expl.bw).view(np.int32)).to(dev),
        "stats": stats_from_numpy(expl.mean, expl.scale, device=dev),
    }
    expl._dev_cache = (key, t)
    return t


def treeshap(X: torch.Tensor, expl, sync: bool = True, out=None):
    """X [E, d] RAW fp32 on device (standardized on device with the model's scaler) -> (phi [E, d],
    margin(x) [E], f0): phi sums to margin(x) - f0, f0 = mean background margin.  Numpy if
    ``sync`` else device tensors (``out``: preallocated (phi, fx, f0) device tensors)."""
    _check_x(X, expl.d)
    m = native()
    dev = X.device
    t = _device_design(expl, dev)
    from .scaler import scale_cast

    E = X.shape[0]
    Xs = scale_cast(X, t["stats"], out_dtype="f32")  # [E, 32]
    phi, fx, f0 = _outputs(E, expl.d, dev, out)
    ens = expl.ens
    m.treeshap(ptr(Xs), Xs.stride(0), E, expl.d, ptr(t["feat"]), ptr(t["thr"]), ptr(t["leaf"]), ens.n_trees,
               ens.depth, float(ens.base_margin), ptr(t["bw"]), expl.bw.shape[1], expl.B.shape[0], float(expl.f0),
               ptr(phi), ptr(fx), ptr(f0), stream_of(X))
    if not sync:
        return phi, fx, f0
    return phi.cpu().numpy().astype(np.float64), fx.cpu().numpy().astype(np.float64), float(expl.f0)
