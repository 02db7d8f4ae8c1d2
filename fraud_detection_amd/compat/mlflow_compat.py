"""MLflow-compatible experiment tracking and model registry.

Reference usage (train_model.py:117-166, api/app.py:28-46, scripts/validate_auc.py:14-29):
set_tracking_uri / set_experiment / start_run / log_param / log_metric / log_artifact /
sklearn log_model (signature + input example) / register_model when AUC >= threshold, and the
API serving ``models:/<name>@<alias>`` (alias "production") with a joblib fallback.

If the real ``mlflow`` package is importable (and FDX_USE_MLFLOW != 0) every call goes to it.
Otherwise this module writes the MLflow FileStore on-disk layout itself
(``mlruns/<exp_id>/<run_id>/{meta.yaml, params/, metrics/, tags/, artifacts/}`` and the
registry under ``mlruns/models/<name>/``), so the runs are readable by a real MLflow UI later,
and it adds what the reference never did: setting the serving alias after registration
(SURVEY.md App. D item 9), so ``models:/name@production`` actually resolves.
Remote ``http(s)://`` tracking servers need the real mlflow; without it they raise
``TrackingUnavailable`` (the reference's callers already treat tracking as best-effort).
"""
from __future__ import annotations

import contextlib
import json
import os
import pickle
import shutil
import time
import uuid

import yaml

try:  # pragma: no cover - mlflow is not installed in this image
    if os.getenv("FDX_USE_MLFLOW", "1") == "1":
        import mlflow as _real_mlflow  # type: ignore
    else:
        _real_mlflow = None
except Exception:  # noqa: BLE001
    _real_mlflow = None


class TrackingUnavailable(RuntimeError):
    pass


def _now_ms() -> int:
    return int(time.time() * 1000)


def _root_from_uri(uri: str | None) -> str:
    uri = uri or os.getenv("MLFLOW_TRACKING_URI", "file:./mlruns")
    if uri.startswith("file:"):
        p = uri[len("file:"):]
        if p.startswith("//"):
            p = p[2:]
        return os.path.abspath(p)
    if uri.startswith(("http://", "https://", "databricks")):
        raise TrackingUnavailable(f"tracking server {uri} needs the mlflow package (not installed)")
    return os.path.abspath(uri)


def _write_yaml(path: str, d: dict):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(d, f, sort_keys=True)


def _read_yaml(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


class Run:
    def __init__(self, store: "FileStore", exp_id: str, run_id: str):
        self.store, self.exp_id, self.run_id = store, exp_id, run_id
        self.dir = os.path.join(store.root, exp_id, run_id)
        self.info = type("RunInfo", (), {"run_id": run_id, "experiment_id": exp_id})()

    @property
    def artifact_dir(self) -> str:
        return os.path.join(self.dir, "artifacts")

    def log_param(self, key, value):
        p = os.path.join(self.dir, "params", str(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(str(value))

    def log_metric(self, key, value, step: int = 0):
        p = os.path.join(self.dir, "metrics", str(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "a") as f:
            f.write(f"{_now_ms()} {float(value)} {int(step)}\n")

    def set_tag(self, key, value):
        p = os.path.join(self.dir, "tags", str(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(str(value))

    def log_artifact(self, local_path: str, artifact_path: str | None = None):
        dst = os.path.join(self.artifact_dir, artifact_path or "")
        os.makedirs(dst, exist_ok=True)
        shutil.copy2(local_path, os.path.join(dst, os.path.basename(local_path)))

    def log_sklearn_model(self, model, artifact_path: str = "model", signature=None, input_example=None,
                          extra_files: dict | None = None):
        d = os.path.join(self.artifact_dir, artifact_path)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "model.pkl"), "wb") as f:
            pickle.dump(model, f)
        import sklearn

        mlmodel = {
            "artifact_path": artifact_path,
            "flavors": {
                "python_function": {"loader_module": "mlflow.sklearn", "model_path": "model.pkl",
                                    "predict_fn": "predict", "python_version": "3.10"},
                "sklearn": {"code": None, "pickled_model": "model.pkl", "serialization_format": "pickle",
                            "sklearn_version": sklearn.__version__},
            },
            "model_uuid": uuid.uuid4().hex,
            "run_id": self.run_id,
            "utc_time_created": time.strftime("%Y-%m-%d %H:%M:%S", time.gmtime()),
            "written_by": "fraud_detection_amd",
        }
        if signature is not None:
            mlmodel["signature"] = signature
        _write_yaml(os.path.join(d, "MLmodel"), mlmodel)
        if input_example is not None:
            with open(os.path.join(d, "input_example.json"), "w") as f:
                json.dump({"data": [list(map(float, r)) for r in input_example]}, f)
        for name, src in (extra_files or {}).items():
            shutil.copy2(src, os.path.join(d, name))
        return f"runs:/{self.run_id}/{artifact_path}"

    def log_files_model(self, files: dict, artifact_path: str = "model", flavor: str = "fdx_gbdt",
                        flavor_conf: dict | None = None, signature=None) -> str:
        """A model stored as plain files (no pickle), e.g. the JSON tree ensemble."""
        d = os.path.join(self.artifact_dir, artifact_path)
        os.makedirs(d, exist_ok=True)
        for name, src in files.items():
            shutil.copy2(src, os.path.join(d, name))
        mlmodel = {"artifact_path": artifact_path, "flavors": {flavor: dict(flavor_conf or {})},
                   "model_uuid": uuid.uuid4().hex, "run_id": self.run_id,
                   "utc_time_created": time.strftime("%Y-%m-%d %H:%M:%S", time.gmtime()),
                   "written_by": "fraud_detection_amd"}
        if signature is not None:
            mlmodel["signature"] = signature
        _write_yaml(os.path.join(d, "MLmodel"), mlmodel)
        return f"runs:/{self.run_id}/{artifact_path}"

    def end(self, status: str = "FINISHED"):
        meta = os.path.join(self.dir, "meta.yaml")
        m = _read_yaml(meta)
        m["end_time"] = _now_ms()
        m["status"] = {"FINISHED": 3, "FAILED": 4, "KILLED": 5}.get(status, 3)
        _write_yaml(meta, m)


class FileStore:
    def __init__(self, tracking_uri: str | None = None):
        self.root = _root_from_uri(tracking_uri)

    # ---- experiments ----
    def get_or_create_experiment(self, name: str) -> str:
        os.makedirs(self.root, exist_ok=True)
        for e in os.listdir(self.root):
            mp = os.path.join(self.root, e, "meta.yaml")
            if e.isdigit() and os.path.exists(mp) and _read_yaml(mp).get("name") == name:
                return e
        ids = [int(e) for e in os.listdir(self.root) if e.isdigit()]
        eid = str(max(ids) + 1 if ids else 0)
        _write_yaml(os.path.join(self.root, eid, "meta.yaml"), {
            "artifact_location": f"file://{os.path.join(self.root, eid)}", "experiment_id": eid,
            "lifecycle_stage": "active", "name": name, "creation_time": _now_ms(), "last_update_time": _now_ms()})
        return eid

    def create_run(self, exp_id: str, run_name: str | None = None) -> Run:
        rid = uuid.uuid4().hex
        d = os.path.join(self.root, exp_id, rid)
        _write_yaml(os.path.join(d, "meta.yaml"), {
            "artifact_uri": f"file://{os.path.join(d, 'artifacts')}", "end_time": None, "entry_point_name": "",
            "experiment_id": exp_id, "lifecycle_stage": "active", "run_id": rid, "run_uuid": rid,
            "run_name": run_name or rid[:8], "source_name": "", "source_type": 4, "source_version": "",
            "start_time": _now_ms(), "status": 1, "tags": [], "user_id": os.getenv("USER", "fdx")})
        return Run(self, exp_id, rid)

    def find_run(self, run_id: str) -> Run:
        for e in os.listdir(self.root):
            if os.path.isdir(os.path.join(self.root, e, run_id)):
                return Run(self, e, run_id)
        raise KeyError(run_id)

    def read_run(self, run_id: str) -> dict:
        r = self.find_run(run_id)
        out = {"params": {}, "metrics": {}, "tags": {}}
        for kind in out:
            d = os.path.join(r.dir, kind)
            if os.path.isdir(d):
                for k in os.listdir(d):
                    with open(os.path.join(d, k)) as f:
                        txt = f.read()
                    out[kind][k] = float(txt.strip().splitlines()[-1].split()[1]) if kind == "metrics" else txt
        return out

    # ---- registry ----
    def _model_dir(self, name: str) -> str:
        return os.path.join(self.root, "models", name)

    def register_model(self, source_uri: str, name: str) -> int:
        md = self._model_dir(name)
        if not os.path.exists(os.path.join(md, "meta.yaml")):
            _write_yaml(os.path.join(md, "meta.yaml"), {"name": name, "creation_timestamp": _now_ms(),
                                                        "last_updated_timestamp": _now_ms(), "description": ""})
        versions = [int(v.split("-")[1]) for v in os.listdir(md) if v.startswith("version-")]
        ver = max(versions) + 1 if versions else 1
        run_id = source_uri.split("/")[1] if source_uri.startswith("runs:/") else None
        _write_yaml(os.path.join(md, f"version-{ver}", "meta.yaml"), {
            "name": name, "version": ver, "source": source_uri, "run_id": run_id, "status": "READY",
            "current_stage": "None", "creation_timestamp": _now_ms(), "last_updated_timestamp": _now_ms()})
        return ver

    def set_alias(self, name: str, alias: str, version: int):
        p = os.path.join(self._model_dir(name), "aliases", alias)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(str(int(version)))

    def get_version_by_alias(self, name: str, alias: str) -> int:
        p = os.path.join(self._model_dir(name), "aliases", alias)
        if not os.path.exists(p):
            raise KeyError(f"models:/{name}@{alias} has no version")
        with open(p) as f:
            return int(f.read().strip())

    def latest_version(self, name: str) -> int:
        md = self._model_dir(name)
        vs = [int(v.split("-")[1]) for v in os.listdir(md) if v.startswith("version-")] if os.path.isdir(md) else []
        if not vs:
            raise KeyError(f"no versions of {name}")
        return max(vs)

    def resolve_model_dir(self, model_uri: str) -> str:
        """models:/name@alias | models:/name/<version> | runs:/<run_id>/<path> -> local directory."""
        if model_uri.startswith("models:/"):
            rest = model_uri[len("models:/"):]
            if "@" in rest:
                name, alias = rest.split("@", 1)
                ver = self.get_version_by_alias(name, alias)
            else:
                name, _, v = rest.partition("/")
                ver = self.latest_version(name) if v in ("", "latest") else int(v)
            meta = _read_yaml(os.path.join(self._model_dir(name), f"version-{ver}", "meta.yaml"))
            model_uri = meta["source"]
        if model_uri.startswith("runs:/"):
            _, run_id, path = model_uri.split("/", 2)
            return os.path.join(self.find_run(run_id).artifact_dir, path)
        return model_uri


# ---------------------------------------------------------------------------------------------
# module-level API mirroring the mlflow calls the reference makes
# ---------------------------------------------------------------------------------------------
_state = {"uri": None, "experiment": None, "run": None}


def set_tracking_uri(uri: str):
    if _real_mlflow is not None:  # pragma: no cover
        return _real_mlflow.set_tracking_uri(uri)
    _state["uri"] = uri


def _store() -> FileStore:
    return FileStore(_state["uri"])


def set_experiment(name: str):
    if _real_mlflow is not None:  # pragma: no cover
        return _real_mlflow.set_experiment(name)
    _state["experiment"] = _store().get_or_create_experiment(name)


@contextlib.contextmanager
def start_run(run_name: str | None = None):
    if _real_mlflow is not None:  # pragma: no cover
        with _real_mlflow.start_run(run_name=run_name) as r:
            yield r
        return
    st = _store()
    if _state["experiment"] is None:
        _state["experiment"] = st.get_or_create_experiment(os.getenv("MLFLOW_EXPERIMENT", "Default"))
    run = st.create_run(_state["experiment"], run_name)
    _state["run"] = run
    try:
        yield run
        run.end("FINISHED")
    except BaseException:
        run.end("FAILED")
        raise
    finally:
        _state["last_run"] = run
        _state["run"] = None


def _active() -> Run:
    if _state["run"] is None:
        raise RuntimeError("no active run")
    return _state["run"]


def log_param(k, v):
    return _real_mlflow.log_param(k, v) if _real_mlflow else _active().log_param(k, v)


def log_metric(k, v, step: int = 0):
    return _real_mlflow.log_metric(k, v, step=step) if _real_mlflow else _active().log_metric(k, v, step)


def set_tag(k, v):
    return _real_mlflow.set_tag(k, v) if _real_mlflow else _active().set_tag(k, v)


def log_artifact(path: str, artifact_path: str | None = None):
    return _real_mlflow.log_artifact(path, artifact_path) if _real_mlflow else _active().log_artifact(path, artifact_path)


def log_sklearn_model(model, artifact_path="model", signature=None, input_example=None, extra_files=None):
    if _real_mlflow is not None:  # pragma: no cover
        import mlflow.sklearn  # type: ignore

        return mlflow.sklearn.log_model(model, artifact_path, signature=signature, input_example=input_example)
    return _active().log_sklearn_model(model, artifact_path, signature, input_example, extra_files)


def log_files_model(files: dict, artifact_path: str = "model", flavor: str = "fdx_gbdt", flavor_conf: dict | None = None,
                    signature=None) -> str:
    if _real_mlflow is not None:  # pragma: no cover
        for src in files.values():
            _real_mlflow.log_artifact(src, artifact_path)
        return f"runs:/{_real_mlflow.active_run().info.run_id}/{artifact_path}"
    return _active().log_files_model(files, artifact_path, flavor, flavor_conf, signature)


def last_run_id() -> str | None:
    r = _state.get("last_run") or _state.get("run")
    return r.run_id if r else None


def register_model(model_uri: str, name: str) -> int:
    if _real_mlflow is not None:  # pragma: no cover
        return int(_real_mlflow.register_model(model_uri, name).version)
    return _store().register_model(model_uri, name)


def set_registered_model_alias(name: str, alias: str, version: int):
    if _real_mlflow is not None:  # pragma: no cover
        from mlflow.tracking import MlflowClient  # type: ignore

        return MlflowClient().set_registered_model_alias(name, alias, str(version))
    _store().set_alias(name, alias, version)


def resolve_model_dir(model_uri: str, tracking_uri: str | None = None) -> str:
    return FileStore(tracking_uri or _state["uri"]).resolve_model_dir(model_uri)


def infer_signature(X, y) -> dict:
    import numpy as np

    X = np.asarray(X)
    cols = [{"type": "tensor", "tensor-spec": {"dtype": str(X.dtype), "shape": [-1, int(X.shape[1])]}}]
    outs = [{"type": "tensor", "tensor-spec": {"dtype": str(np.asarray(y).dtype), "shape": [-1]}}]
    return {"inputs": json.dumps(cols), "outputs": json.dumps(outs)}


def load_sklearn_model(model_uri: str, tracking_uri: str | None = None):
    """Load a model this framework logged (pickle of an sklearn estimator).  Only directories
    carrying our MLmodel marker are unpickled; anything else is refused."""
    d = resolve_model_dir(model_uri, tracking_uri)
    ml = _read_yaml(os.path.join(d, "MLmodel"))
    if ml.get("written_by") != "fraud_detection_amd":
        raise TrackingUnavailable(f"{model_uri}: not written by this framework; refusing to unpickle")
    with open(os.path.join(d, "model.pkl"), "rb") as f:
        return pickle.load(f)
