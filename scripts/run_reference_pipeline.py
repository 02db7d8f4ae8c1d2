#!/usr/bin/env python3
"""Run the reference's script chain end to end in a scratch working directory and collect its
plots (reference plots/*.png, produced by eda.py, evaluate_model.py and explain_model.py):

    scripts/generate_synthetic_data.py --separable -> eda.py -> preprocess.py -> train_model.py
    -> evaluate_model.py -> explain_model.py [--kernel]

On a GPU box every numeric step runs on the device kernels (scaler, SMOTE k-NN, Newton fit,
predict, exact AUC, LinearSHAP / KernelSHAP).  The data are credit_card-shaped synthetic rows
(Kaggle size: 284,807 rows, 0.17% fraud) -- the reference's own plots are of the Kaggle file,
which is not available here.

    python scripts/run_reference_pipeline.py --out plots [--rows 284807] [--kernel]
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="plots")
    ap.add_argument("--rows", type=int, default=284_807)
    ap.add_argument("--kernel", action="store_true", help="also run KernelSHAP (explain_model.py --kernel)")
    a = ap.parse_args()
    out = os.path.abspath(a.out)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT, MPLBACKEND="Agg")
    log = {}
    with tempfile.TemporaryDirectory(prefix="fdx_pipeline_") as wd:
        steps = [
            ["scripts/generate_synthetic_data.py", "--separable", "--rows", str(a.rows)],
            ["eda.py"],
            ["preprocess.py"],
            ["train_model.py"],
            ["evaluate_model.py"],
            ["explain_model.py"],
        ]
        if a.kernel:
            steps.append(["explain_model.py", "--kernel", "--rows", "1000"])
        for st in steps:
            t0 = time.perf_counter()
            r = subprocess.run([sys.executable, os.path.join(ROOT, st[0])] + st[1:], cwd=wd, env=env,
                               capture_output=True, text=True, timeout=1200)
            dt = time.perf_counter() - t0
            name = " ".join(st)
            log[name] = {"rc": r.returncode, "seconds": round(dt, 2), "stdout_tail": r.stdout[-1500:]}
            print(f"[pipeline] {name}: rc={r.returncode} {dt:.1f}s", flush=True)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                break
        for f in glob.glob(os.path.join(wd, "plots", "*.png")):
            shutil.copy(f, out)
        with open(os.path.join(out, "pipeline_run.json"), "w") as f:
            json.dump(log, f, indent=1)
    return 0 if all(v["rc"] == 0 for v in log.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
