"""Training entry point behind train_model.py (reference call stack: SURVEY.md §3.1).

    read CSV (native reader) -> stratified 80/20 split (rs=42)
    -> StratifiedKFold(5, shuffle, rs=42): per fold the device pipeline (scaler on the fold's
       train rows -> SMOTE k-NN + generation -> fit) and the fold's validation AUC
    -> final pipeline on the whole train split -> exact test AUC
    -> artifacts in the reference layout (models/logistic_model.joblib, scaler.joblib,
       columns.joblib, feature_names.json; for the GBDT family models/xgb_model.joblib -- a
       GBDTClassifier, the reference's joblib contract -- plus models/xgb_model.json, the
       pickle-free copy serving loads)
    -> MLflow run (params model_type / scale_pos_weight / cv_folds, metrics test_auc /
       cv_auc_mean / cv_auc_std, sklearn model with signature + input example, scaler artifact),
       registration when test_auc >= MLFLOW_AUC_THRESHOLD and the serving alias set to
       MLFLOW_MODEL_STAGE.  Tracking failures never fail training (train_model.py:165-166).
"""
from __future__ import annotations

import json
import logging
import os
import tempfile
import time

import numpy as np
import torch

from .compat import mlflow_compat as mlf
from .compat.sklearn_export import LinearArtifacts, make_logistic, save_artifacts
from .config import Settings
from .data.io import missing_report, read_table, stratified_folds, stratified_split
from .models.pipeline import DevicePipeline, TrainConfig, evaluate
from .obs import tracing
from .obs.metrics import train_metrics
from .runtime.hbm import observe_hbm

logger = logging.getLogger("train")

DEVICE_SPLIT_ROWS = 2_000_000
FOLD_PARALLEL_ROWS = 8_000_000


def _device(name: str) -> torch.device:
    if name == "auto":
        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(name)


def _shard(idx: np.ndarray, comm) -> np.ndarray:
    """This rank's rows of an index set (strided, so every shard keeps the class mix)."""
    if comm is None:
        return idx
    return idx[comm.rank::comm.world_size]


def run(settings: Settings | None = None, model_type: str = "logistic", cv_folds: int = 5, model_dir: str = "models",
        verbose: bool = True, cfg: TrainConfig | None = None, comm=None) -> dict:
    """Single process, or data parallel when ``comm`` spans several ranks (torchrun: one rank per
    GPU).  Every rank reads the table and derives the same split; each fits on its strided shard
    with RCCL all-reduced statistics, so all ranks hold the same model; rank 0 writes artifacts."""
    s = settings or Settings.load()
    comm = comm if (comm is not None and comm.world_size > 1) else None
    lead = comm is None or comm.rank == 0
    say = print if (verbose and lead) else (lambda *a, **k: None)
    dev = _device(s.device)
    if comm is not None and dev.type == "cuda":
        dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.time()
    say("Loading dataset...")
    X, y, names = read_table(s.data_csv)
    if y is None:
        raise ValueError(f"{s.data_csv} has no 'Class' column")
    say("Checking missing values...")
    miss = missing_report(X, names)
    say({k: v for k, v in miss.items() if v} or "no missing values")
    if any(miss.values()):
        raise ValueError("missing feature values; impute before training")
    say("Splitting dataset (Train 80% / Test 20%)...")
    mode = s.split
    if mode == "auto":  # the sklearn split is a host argsort: past a few million rows use K3
        mode = "device" if dev.type == "cuda" and X.shape[0] >= DEVICE_SPLIT_ROWS else "sklearn"
    if mode == "device":
        from .ops import split as SP

        Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)  # one upload, then on-device gathers
        codes = SP.assign(yd, 0.2, cv_folds if cv_folds and cv_folds > 1 else 0, 42)
        tr, te, dev_folds = SP.split_indices(codes, cv_folds if cv_folds and cv_folds > 1 else 0)
        take = lambda idx: (Xd.index_select(0, idx), yd.index_select(0, idx))  # noqa: E731
        pos = int(yd.index_select(0, tr).sum())
        neg = int(tr.shape[0]) - pos
    elif mode == "sklearn":
        tr, te = stratified_split(y, 0.2, 42)
        take = lambda idx: (torch.from_numpy(X[idx]).to(dev), torch.from_numpy(y[idx]).to(dev))  # noqa: E731
        neg, pos = int((y[tr] == 0).sum()), int((y[tr] == 1).sum())
    else:
        raise ValueError("split must be sklearn | device | auto")
    Xtr, ytr = take(_shard(tr, comm))
    Xte, yte = take(_shard(te, comm))
    scale_pos_weight = neg / pos if pos > 0 else 1.0
    say(f" Class balance before SMOTE -> [{neg} {pos}]")
    cfg = cfg or TrainConfig(solver=s.solver, storage=s.dtype, seed=s.seed, k_neighbors=s.smote_k)
    if model_type not in ("logistic", "gbdt"):
        raise ValueError("model_type must be 'logistic' or 'gbdt'")
    cv_scores = []
    from dataclasses import asdict

    ck_dir = s.checkpoint_dir or None
    progress = _Progress(ck_dir, lead, signature=None if ck_dir is None else _job_signature(
        s, model_type, cv_folds, mode, asdict(cfg), X.shape, comm))
    if progress.folds:
        say(f" Resuming: {len(progress.folds)} completed fold(s) from {progress.path}")
    res_cv = None
    cv_engine = None
    if cv_folds and cv_folds > 1 and pos >= cv_folds:
        say(f" Performing Stratified K-Fold Cross-Validation ({cv_folds} folds) with SMOTE inside each fold...")
        if mode == "device":
            folds = dev_folds
            # the device jobs run on the K3 codes of this split (the per-fold path's folds)
            job_codes = codes.index_select(0, tr) if comm is None else None
        else:
            sk = stratified_folds(y[tr], cv_folds, 42)
            folds = [(tr[a], tr[b]) for a, b in sk]
            # sklearn's StratifiedKFold(5, shuffle, 42) membership (train_model.py:49,58) for the
            # device jobs too: their fold AUCs are on the reference's folds
            job_codes = None
            if comm is None:
                from .models.cv import fold_codes_from_splits

                job_codes = fold_codes_from_splits(sk, len(tr))
        cv_mode = s.cv_parallel
        if cv_mode == "auto":  # small folds are latency-bound under DP: give each rank whole folds
            cv_mode = "fold" if comm is not None and len(tr) < FOLD_PARALLEL_ROWS else "dp"
        if _device_cv_ok(model_type, cfg, dev, comm, progress, Xtr):
            # models/cv.DeviceCV: the reference's semantics (ONE scaler on the training split,
            # SMOTE inside every fold) on one fold-sorted device table, final fit included
            from .models.cv import DeviceCV

            t_fit = time.perf_counter()
            with tracing.span("train.cv_job", model=model_type), tracing.roctx_range("train.cv_job"):
                cvr = DeviceCV(cfg, cv_folds, seed=42).run(Xtr, ytr, fold_codes=job_codes)
            cv_scores, res_cv, cv_engine = cvr.fold_aucs, cvr.final, "device"
            for k, auc in enumerate(cv_scores):
                progress.record(k, auc)
        elif _device_gbdt_cv_ok(model_type, cfg, dev, comm, progress):
            # models/gbdt_cv.DeviceGBDTCV: one binned fold-sorted table, fold k fits around its own
            # block (row hole, no copy), its margins are the validation scores; final fit included
            from .models.gbdt_cv import DeviceGBDTCV

            t_fit = time.perf_counter()
            with tracing.span("train.cv_job", model=model_type), tracing.roctx_range("train.cv_job"):
                cvr = DeviceGBDTCV(cfg, n_folds=cv_folds, seed=42).run(Xtr, ytr, fold_codes=job_codes)
            cv_scores, res_cv, cv_engine = cvr.fold_aucs, cvr.final, "device"
            for k, auc in enumerate(cv_scores):
                progress.record(k, auc)
        else:
            cv_scores = _cross_validate(model_type, cfg, folds, take, comm, cv_mode, progress)
            cv_engine = f"per_fold:{cv_mode}"
        for k, auc in enumerate(cv_scores):
            say(f"  Fold {k + 1} AUC: {auc:.4f}")
        say(f" CV AUC Mean: {np.mean(cv_scores):.4f} (+/- {np.std(cv_scores) * 2:.4f})")
    say(f" Training final {model_type} model with SMOTE on the full training set...")
    if res_cv is None:
        t_fit = time.perf_counter()
        with tracing.span("train.final_fit", model=model_type), tracing.roctx_range("train.final_fit"):
            res = _fit(model_type, cfg, Xtr, ytr, comm,
                       checkpoint=None if ck_dir is None else os.path.join(ck_dir, f"final_{model_type}"))
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
    else:
        res = res_cv  # fitted inside the CV job (t_fit: the whole job)
    t_fit = time.perf_counter() - t_fit
    tm = train_metrics()
    tm.rows_per_second.set(float(res.n_train_rows) * (comm.world_size if comm else 1) / max(t_fit, 1e-9))
    observe_hbm(dev)
    if model_type == "gbdt":  # the weight the trees were fit with (post-SMOTE balance by default)
        scale_pos_weight = float(res.scale_pos_weight)
    if model_type == "logistic":
        ev = evaluate(res, Xte, yte, comm)
        auc = ev["auc"]
        say(f" Class balance after SMOTE -> [{res.n_rows - res.n_minority} {res.n_minority + res.n_synthetic}]"
            + (f" (rank 0 of {comm.world_size})" if comm else ""))
    else:
        ev = res.evaluate(Xte, yte, comm)
        auc = ev["auc"]
    say(f"Test AUC: {auc:.4f}")
    if not lead:
        comm.barrier()
        return {"test_auc": float(auc), "cv_scores": cv_scores, "rank": comm.rank}
    paths = _save(model_type, res, names, model_dir, cfg)
    # KernelSHAP background (shap.sample of the training rows) for the async XAI worker
    from .serve.engine import sample_background, save_background

    paths["background"] = save_background(sample_background(Xtr[: 1 << 20].cpu().numpy(), s.kernelshap_background,
                                                            s.seed), model_dir)
    say(f" Model and scaler saved to /{model_dir}")
    summary = {"test_auc": float(auc), "cv_auc_mean": float(np.mean(cv_scores)) if cv_scores else None,
               "cv_auc_std": float(np.std(cv_scores)) if cv_scores else None, "cv_scores": cv_scores,
               "scale_pos_weight": scale_pos_weight, "paths": paths, "device": str(dev), "eval": ev,
               "seconds": round(time.time() - t0, 3), "registered_version": None}
    try:
        summary["registered_version"] = _track(s, model_type, res, summary, paths, Xte, names, say)
    except Exception as e:  # noqa: BLE001 - tracking is best effort (reference train_model.py:165-166)
        say(f" MLflow Tracking Failed (likely connection error): {e}")
    summary["split"] = mode
    summary["cv_engine"] = cv_engine
    summary["resumed_folds"] = sorted(progress.resumed)
    if comm is not None:
        summary["world_size"] = comm.world_size
        comm.barrier()
    return summary


class _Progress:
    """Job-level resume: completed CV folds are recorded in
    ``<checkpoint_dir>/train_progress.json`` (atomic rename, rank 0 writes), so a job restarted
    after a crash or a lost rank (``torchrun --max-restarts``) skips them; the final GBDT fit
    resumes from its tree checkpoints.  A record is used only if the job signature (data file,
    model, folds, split, training config, world size) matches."""

    def __init__(self, directory, lead: bool, signature):
        self.path = os.path.join(directory, "train_progress.json") if directory else None
        self.lead, self.sig = lead, signature
        self.folds: dict = {}
        if self.path and os.path.exists(self.path):
            with open(self.path) as f:
                d = json.load(f)
            if d.get("signature") == signature:
                self.folds = {int(k): float(v) for k, v in d.get("folds", {}).items()}
        self.resumed = set(self.folds)

    def record(self, k: int, auc: float):
        self.folds[k] = float(auc)
        if self.path and self.lead:
            os.makedirs(os.path.dirname(self.path), exist_ok=True)
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"signature": self.sig, "folds": self.folds}, f)
            os.replace(tmp, self.path)
        fault = os.getenv("FDX_FAULT", "")
        if fault.startswith("train_crash_after_fold=") and len(self.folds) == int(fault.split("=", 1)[1]):
            logger.error("FDX_FAULT: simulated crash after %d fold(s)", len(self.folds))
            os._exit(17)  # hard exit, like a killed rank: no cleanup, no flush


def _job_signature(s, model_type, cv_folds, split_mode, cfg: dict, shape, comm) -> str:
    from .utils.checkpoint import config_signature

    st = os.stat(s.data_csv)
    return config_signature(data=os.path.abspath(s.data_csv), size=st.st_size, mtime=int(st.st_mtime),
                            shape=list(shape), model=model_type, folds=cv_folds, split=split_mode, cfg=cfg,
                            world=1 if comm is None else comm.world_size)


def _cross_validate(model_type, cfg, folds, take, comm, mode: str, progress: _Progress | None = None) -> list:
    """K12 per-fold orchestration (train_model.py:58-85).  The table is resident (device split:
    on the GPU), so each fold is an on-device gather, never a host copy.
      dp   -- every fold is fitted data-parallel over all ranks (large folds);
      fold -- fold k runs whole on rank k % world (no collectives inside a fit), and the fold AUCs
              are exchanged once at the end: the fold-parallel mode of SURVEY.md §2.4.
    Folds already in ``progress`` (a resumed job) are not recomputed."""
    progress = progress or _Progress(None, True, None)
    if comm is None or mode == "dp":
        for k, (ftr, fva) in enumerate(folds):
            if k in progress.folds:
                continue
            res = _fit(model_type, cfg, *take(_shard(ftr, comm)), comm)
            progress.record(k, _score(model_type, res, *take(_shard(fva, comm)), comm))
        return [progress.folds[k] for k in range(len(folds))]
    if mode != "fold":
        raise ValueError("cv_parallel must be dp | fold | auto")
    mine = {}
    for k in range(comm.rank, len(folds), comm.world_size):
        if k in progress.folds:
            continue
        ftr, fva = folds[k]
        res = _fit(model_type, cfg, *take(ftr), None)
        mine[k] = _score(model_type, res, *take(fva), None)
    for part in comm.all_gather_object(mine):
        for k, auc in sorted(part.items()):
            progress.record(k, auc)
    return [progress.folds[k] for k in range(len(folds))]


def _device_cv_ok(model_type, cfg, dev, comm, progress, Xtr) -> bool:
    """The device CV job (models/cv.py) runs the logistic family on one GPU, from scratch (a
    resumed job keeps the per-fold path), with virtual SMOTE (bf16 Newton or SGD in either row
    format) and an even feature count (its gathered scaler pass reads 8-byte row pieces)."""
    if os.environ.get("FDX_CV_ENGINE", "auto") == "per_fold":
        return False
    virt = cfg.solver == "sgd" or (cfg.solver == "newton" and cfg.storage == "bf16")
    return (model_type == "logistic" and dev.type == "cuda" and comm is None and not progress.folds
            and cfg.smote and cfg.virtual_smote and cfg.fold_scaler and virt and Xtr.shape[1] % 2 == 0
            and Xtr.is_contiguous())


def _device_gbdt_cv_ok(model_type, cfg, dev, comm, progress) -> bool:
    """The device GBDT CV job (models/gbdt_cv.py) runs on one GPU, from scratch (a resumed job
    keeps the per-fold path), with SMOTE inside the folds (the reference's semantics)."""
    if os.environ.get("FDX_CV_ENGINE", "auto") == "per_fold":
        return False
    return model_type == "gbdt" and dev.type == "cuda" and comm is None and not progress.folds and cfg.smote


def _fit(model_type, cfg, X, y, comm=None, checkpoint: str | None = None):
    if model_type == "logistic":
        return DevicePipeline(cfg, comm).fit(X, y)
    from .models.gbdt import GBDTPipeline

    return GBDTPipeline(cfg, comm=comm, checkpoint_dir=checkpoint).fit(X, y)


def _score(model_type, res, X, y, comm=None) -> float:
    if model_type == "logistic":
        return float(evaluate(res, X, y, comm)["auc"])
    return float(res.evaluate(X, y, comm)["auc"])


def _save(model_type, res, names, model_dir, cfg) -> dict:
    mean, var, scale = res.scaler.numpy()
    if model_type == "logistic":
        art = LinearArtifacts(coef=res.coef, intercept=res.intercept, mean=mean, var=var, scale=scale,
                              n_samples_seen=int(res.scaler.n), feature_names=names, n_iter=res.fit.n_iter, C=cfg.C)
        return save_artifacts(art, model_dir)
    return res.save(model_dir, names)


def _track(s: Settings, model_type, res, summary, paths, Xte, names, say):
    mlf.set_tracking_uri(s.mlflow_tracking_uri)
    mlf.set_experiment(s.mlflow_experiment)
    version = None
    with mlf.start_run() as run:
        mlf.log_param("model_type", "LogisticRegression" if model_type == "logistic" else "GBDT")
        mlf.log_param("scale_pos_weight", summary["scale_pos_weight"])
        mlf.log_param("cv_folds", len(summary["cv_scores"]) or 0)
        mlf.log_param("device", summary["device"])
        mlf.log_metric("test_auc", summary["test_auc"])
        if summary["cv_auc_mean"] is not None:
            mlf.log_metric("cv_auc_mean", summary["cv_auc_mean"])
            mlf.log_metric("cv_auc_std", summary["cv_auc_std"])
        sample = Xte[:5].cpu().numpy().astype(np.float64)
        if model_type == "logistic":
            model = make_logistic(res.coef, res.intercept, res.fit.n_iter)
            sc = (sample - res.scaler.numpy()[0]) / res.scaler.numpy()[2]
            sig = mlf.infer_signature(sc, model.predict_proba(sc)[:, 1])
            extra = {"scaler.joblib": paths["scaler"], "feature_names.json": paths["feature_names"]}
            if paths.get("background"):
                extra["shap_background.npy"] = paths["background"]
            uri = mlf.log_sklearn_model(model, "model", signature=sig, input_example=sc[:1], extra_files=extra)
        else:
            uri = res.log_model(mlf, paths)
        mlf.log_artifact(paths["scaler"])
        say(f" Logged run to MLflow experiment '{s.mlflow_experiment}' with input signature and examples")
        if summary["test_auc"] >= s.mlflow_auc_threshold:
            version = mlf.register_model(uri, s.mlflow_model_name)
            mlf.set_registered_model_alias(s.mlflow_model_name, s.mlflow_model_stage, version)
            say(f" Registered model version {version} (AUC {summary['test_auc']:.4f} >= {s.mlflow_auc_threshold}) "
                f"as models:/{s.mlflow_model_name}@{s.mlflow_model_stage}")
        else:
            say(f"i Model not registered (AUC {summary['test_auc']:.4f} < {s.mlflow_auc_threshold})")
        summary["run_id"] = run.info.run_id
    return version


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="Train the fraud model on MI355X (train_model.py)")
    ap.add_argument("--model", default=os.getenv("FDX_MODEL_TYPE", "logistic"), choices=["logistic", "gbdt"])
    ap.add_argument("--cv-folds", type=int, default=5)
    ap.add_argument("--model-dir", default="models")
    ap.add_argument("--json", default=None, help="write the run summary here")
    ap.add_argument("--checkpoint-dir", default=None,
                    help="resume directory: completed CV folds + GBDT tree checkpoints (FDX_CHECKPOINT_DIR)")
    ap.add_argument("--split", default=None, choices=["auto", "sklearn", "device"],
                    help="sklearn: reference-identical split; device: K3 kernel (default auto: device >= 2M rows on GPU)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    comm = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # torchrun: one rank per GPU, RCCL (gloo on CPU)
        from .parallel.comm import Communicator

        dev = None
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            dev = torch.device("cuda", torch.cuda.current_device())
        comm = Communicator(device=dev)
    try:
        over = {k: v for k, v in (("split", a.split), ("checkpoint_dir", a.checkpoint_dir)) if v}
        st = Settings.load(**over)
        out = run(st, model_type=a.model, cv_folds=a.cv_folds, model_dir=a.model_dir, comm=comm)
    finally:
        if comm is not None:
            comm.close()
    if comm is not None and comm.rank != 0:
        return 0
    if a.json:
        with open(a.json, "w") as f:
            json.dump({k: v for k, v in out.items() if k != "eval"} | {"eval": out["eval"]}, f, indent=1, default=str)
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())


def tempdir() -> str:  # helper for scripts/tests
    return tempfile.mkdtemp(prefix="fdx_train_")
