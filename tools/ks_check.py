import sys, time, json
sys.path.insert(0, "/root/repo") if False else None
import os; sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
from fraud_detection_amd.models.explainers import KernelExplainer, kernelshap_throughput
from fraud_detection_amd.ops.kernelshap import kernelshap
dev = torch.device("cuda", 0)
X, y = separable(2_000_000, seed=1000, device=dev)
res = DevicePipeline(TrainConfig(seed=42)).fit(X, y)
print("bench helper:", kernelshap_throughput(res, dev, None))
a, c, b = res.folded()
Xb, _ = separable(100, seed=91); Xe, _ = separable(1000, seed=92)
ke = KernelExplainer(a, b, Xb.numpy(), device="cuda")
Xd = Xe.to(dev)
z = (Xe.double().numpy() @ a[:30] + b); zb = Xb.double().numpy() @ a[:30] + b
print("logit range x", z.min(), z.max(), "bg", zb.min(), zb.max(), "|a|", np.abs(a[:30]).max())
for reps in (5, 50):
    for _ in range(10): kernelshap(Xd, ke, sync=False)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(reps): kernelshap(Xd, ke, sync=False)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / reps
    print(reps, "us", dt * 1e6, "values/s", 30000 / dt)
