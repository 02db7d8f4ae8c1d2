#!/usr/bin/env python3
"""Minimal driver for PMC runs of the MFMA kernels: the bench's minority k-NN self-search
(13.6k x 13.6k, k = 5), and one 1k-explanation KernelSHAP batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.explainers import KernelExplainer
    from fraud_detection_amd.ops import knn as K
    from fraud_detection_amd.ops import scaler as S
    from fraud_detection_amd.ops.kernelshap import kernelshap

    dev = torch.device("cuda", 0)
    X, y = separable(8_000_000, seed=1, device=dev)
    st = S.scaler_fit(X)
    idx = S.compact_indices(y, 1)
    xmin = S.scale_cast(X, st, labels=y, out_dtype="f32", idx=idx)
    a = np.r_[np.random.default_rng(0).normal(0, 0.2, 30), 0.0, 0.0]
    ke = KernelExplainer(a, -3.0, X[:100].cpu().numpy(), device="cuda")
    Xe = X[:1000].contiguous()
    for _ in range(reps):
        K.knn_topk(xmin, xmin, 5, 0)
        kernelshap(Xe, ke, sync=False)
    torch.cuda.synchronize()
    print("mfma_probe done", tuple(xmin.shape))


if __name__ == "__main__":
    main()
