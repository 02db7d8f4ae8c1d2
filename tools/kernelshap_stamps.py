#!/usr/bin/env python3
"""Phase timing of the KernelSHAP kernel (kernelshap.hip) from s_memtime stamps of each
explanation's workgroup: U build -> coalition GEMM + link -> f0/f(x) -> link transform -> WLS
projection A y -> write-out.  Also the dispatch span of the stamped batch.

    python tools/kernelshap_stamps.py [--expl 1000] [--link identity]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["U fragments (hi/lo bf16)", "coalition MFMA + link (wave 0)", "barrier + f0 / f(x)",
          "y = link(f) - f0", "WLS projection A y", "phi write-out"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--expl", type=int, default=1000)
    ap.add_argument("--link", default="identity")
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.explainers import KernelExplainer
    from fraud_detection_amd.ops.kernelshap import kernelshap

    dev = torch.device("cuda", 0)
    X, _ = separable(max(a.expl, 100), seed=1)
    Xr = X.numpy().astype(np.float64)  # standardized-space weights folded onto raw features
    w = np.r_[np.random.default_rng(0).normal(0, 0.4, 30) / Xr.std(0), 0.0, 0.0]
    ke = KernelExplainer(w, float(-3.0 - w[:30] @ Xr.mean(0)), X[:100].numpy(), link=a.link, device="cuda")
    Xe = X[: a.expl].contiguous().to(dev)
    st = torch.zeros((a.expl, 8), dtype=torch.int64, device=dev)
    for _ in range(3):
        kernelshap(Xe, ke, sync=False, stamps=st)
    torch.cuda.synchronize()
    t = st.cpu().numpy().astype(np.int64)
    d = np.diff(t[:, :7], axis=1)
    med = np.median(d, 0)
    print(f"kernelshap_kernel phases ({a.expl} explanations, link={a.link}; s_memtime ticks, median per workgroup; "
          f"total {med.sum():.0f})")
    for name, v in zip(PHASES, med):
        print(f"  {name:34s} {v:9.0f}")
    span = t[:, 6].max() - t[:, 0].min()
    print(f"  dispatch span (first start -> last end): {span} ticks; workgroup lifetime median {np.median(t[:,6]-t[:,0]):.0f}")


if __name__ == "__main__":
    main()
