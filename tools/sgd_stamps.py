#!/usr/bin/env python3
"""Per-step phase timing of the persistent SGD launch (logreg.hip sgd_persist_kernel) from
wall_clock64 stamps (100 MHz) at every block's pass end, barrier exit and update end, at the bench
shape (8M raw training rows -> 16M post-SMOTE rows, virtual SMOTE), plus whole-fit event timings of
the persistent launch against the per-step launches.

    python tools/sgd_stamps.py [--rows 8000000] [--storage bf16] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8_000_000)
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--cfgs", default="", help="comma list of lams:pf lab configurations, one process each")
    a = ap.parse_args()
    if a.cfgs:
        import subprocess
        allres = {}
        for c in a.cfgs.split(","):
            env = dict(os.environ, FDX_SGD_PERSIST_CFG=c.replace(":", ","))
            tag = c.replace(":", "_")
            out = (a.json or "/tmp/sgd") + f".{tag}.json"
            r = subprocess.run([sys.executable, "-u", __file__, "--rows", str(a.rows), "--storage", a.storage,
                                "--reps", str(a.reps), "--json", out], env=env)
            if r.returncode != 0:
                sys.exit(r.returncode)
            with open(out) as f:
                allres[c] = json.load(f)
        if a.json:
            with open(a.json, "w") as f:
                json.dump(allres, f, indent=1)
        return
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.ops import logreg as L

    dev = torch.device("cuda", 0)
    X, y = separable(a.rows, seed=11, device=dev)
    pipe = DevicePipeline(TrainConfig(solver="sgd", storage=a.storage))
    res = pipe.fit(X, y)
    res.fit.as_fit_info()
    rows = pipe._buf[: res.n_rows]
    v = pipe._virtual
    aff = res.scaler.aff
    ws = L.LRWorkspace(dev)
    cfg = pipe.cfg  # the pipeline's schedule (sub-sampled first epoch, per-epoch minibatch counts, ...)
    kw = dict(virtual=v, affine=aff, workspace=ws, lr=cfg.sgd_lr, momentum=cfg.sgd_momentum, epochs=cfg.sgd_epochs,
              batches=cfg.sgd_batches, subsample=cfg.sgd_subsample, extra_epochs=cfg.sgd_extra_epochs,
              avg_from=cfg.sgd_avg_from, epoch_batches=cfg.sgd_epoch_batches)
    out = {"rows": a.rows, "storage": a.storage, "post_smote_rows": res.n_train_rows,
           "cfg": os.environ.get("FDX_SGD_PERSIST_CFG", "default")}
    print("cfg", out["cfg"], flush=True)

    def timed(**k):
        ts = []
        for r in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f = L.sgd_fit(rows, **kw, **k)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1))
        info = f.as_fit_info()
        return float(np.median(ts)), info

    for name, k in [("persistent", dict(persistent=True)), ("per_step", dict(persistent=False)),
                    ("persistent_serpentine", dict(persistent=True, serpentine=True))]:
        ms, info = timed(**k)
        out[name] = {"fit_ms": ms, "converged": info.converged, "grad_max": info.grad_max, "obj": info.objective}
        print(f"{name:24s} {ms * 1e3:8.1f} us  converged={info.converged} gmax={info.grad_max:.2e}", flush=True)

    steps = int(sum(cfg.sgd_epoch_batches)) + cfg.sgd_batches * cfg.sgd_extra_epochs  # room for every step
    blocks = L.native().sgd_persist_blocks(ws.sgd_blocks)
    nrow = 3 + 8  # logreg.hip kStampRows: pass end, barrier exit, update end, 8 waves' pass ends
    stamps = torch.zeros(steps * nrow * blocks, dtype=torch.int64, device=dev)
    ran = L.sgd_fit(rows, persistent=True, _stamps=stamps, **kw).as_fit_info().n_iter
    torch.cuda.synchronize()
    t = stamps.cpu().numpy().astype(np.int64).reshape(steps, nrow, blocks) * 10  # ns
    t0 = t[0, 0].min()
    rows_out = []
    for k in range(min(steps, ran)):
        pe, be, ue = t[k, 0], t[k, 1], t[k, 2]
        we = t[k, 3:]  # [8][blocks] each wave's pass end
        start = t[k - 1, 2] if k else None
        pas = (pe - start) if start is not None else None
        wp = (we - start[None, :]) if start is not None else None
        rows_out.append({
            "step": k,
            "pass_us_med": float(np.median(pas)) / 1e3 if pas is not None else None,
            "pass_us_max": float(np.max(pas)) / 1e3 if pas is not None else None,
            "wave_pass_us_p10": float(np.percentile(wp, 10)) / 1e3 if wp is not None else None,
            "wave_pass_us_med": float(np.median(wp)) / 1e3 if wp is not None else None,
            "wave_pass_us_p90": float(np.percentile(wp, 90)) / 1e3 if wp is not None else None,
            "block_epilogue_us": float(np.median(pe - we.max(0))) / 1e3,
            "arrival_skew_us": float(pe.max() - np.median(pe)) / 1e3,
            "barrier_wake_us": float(np.median(be) - pe.max()) / 1e3,
            "update_us": float(np.median(ue - be)) / 1e3,
            "step_end_us": float(ue.max() - t0) / 1e3,
        })
    print(f"{'step':>4} {'wave p10':>9} {'wave med':>9} {'wave p90':>9} {'epilog':>7} {'pass med':>9} "
          f"{'pass max':>9} {'skew':>7} {'wake':>7} {'update':>7} {'end':>8}")
    nan = float("nan")
    for r in rows_out:
        v = [r[k] if r[k] is not None else nan for k in ("wave_pass_us_p10", "wave_pass_us_med", "wave_pass_us_p90")]
        pm = r["pass_us_med"]
        px = r["pass_us_max"]
        print(f"{r['step']:4d} {v[0]:9.1f} {v[1]:9.1f} {v[2]:9.1f} {r['block_epilogue_us']:7.1f} "
              f"{pm if pm is not None else nan:9.1f} {px if px is not None else nan:9.1f} "
              f"{r['arrival_skew_us']:7.1f} {r['barrier_wake_us']:7.1f} {r['update_us']:7.1f} {r['step_end_us']:8.1f}")
    out["steps"] = rows_out
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
