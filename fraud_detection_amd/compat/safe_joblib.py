"""Read sklearn/joblib artifacts WITHOUT executing anything from the file.

The reference ships pickled sklearn objects (models/logistic_model.joblib, scaler.joblib,
columns.joblib).  Unpickling them normally would run whatever callables the
file names.  This decoder walks the pickle with a restricted unpickler:

* every global the stream references is mapped to an inert stub class (allow-listed names
  only; anything else -> ``UnsafeArtifactError``), so REDUCE/BUILD only ever construct stubs
  that record their arguments/state;
* numpy dtypes and scalars are rebuilt through ``np.dtype`` / ``np.frombuffer`` from the bytes;
* joblib's out-of-band array payload (NumpyArrayWrapper: alignment padding, then raw bytes, or
  a nested pickle for object arrays) is read directly from the file stream.

The result is plain data: ``decode(path)`` returns a ``Stub`` whose ``.state`` dict holds the
estimator's fitted attributes as numpy arrays / Python scalars.
"""
from __future__ import annotations

import io
import pickle

import numpy as np

_ALLOWED_MODULE_PREFIXES = ("sklearn.", "numpy", "joblib.", "builtins", "copyreg", "_codecs")


class UnsafeArtifactError(RuntimeError):
    pass


class Stub:
    """Inert placeholder for any allow-listed class."""

    qualname = "?"

    def __init__(self, *args, **kwargs):
        self.args = args
        self.state = {}

    def __setstate__(self, state):
        self.state = state

    def __repr__(self):
        return f"<Stub {self.qualname} {sorted(self.state) if isinstance(self.state, dict) else type(self.state)}>"


class _ArrayWrapper(Stub):
    qualname = "joblib.NumpyArrayWrapper"


def _dtype_ctor(*args):
    return np.dtype(args[0])


def _scalar_ctor(dtype, payload=None):
    if payload is None:
        return dtype.type(0)
    if isinstance(payload, str):
        payload = payload.encode("latin-1")
    return np.frombuffer(payload, dtype=dtype)[0]


def _encode(s, enc="latin-1"):  # _codecs.encode used by protocol-2 bytes
    return s.encode(enc)


class _SafeUnpickler(pickle._Unpickler):  # pure-python unpickler: BUILD is overridable
    def __init__(self, fh):
        super().__init__(fh)
        self._fh = fh

    def find_class(self, module, name):
        if not module.startswith(_ALLOWED_MODULE_PREFIXES):
            raise UnsafeArtifactError(f"refusing global {module}.{name}")
        if name == "NumpyArrayWrapper":
            return _ArrayWrapper
        if name == "dtype":
            return _dtype_ctor
        if name == "scalar":
            return _scalar_ctor
        if module == "_codecs" and name == "encode":
            return _encode
        if module == "builtins" and name in ("list", "dict", "tuple", "set", "frozenset", "object"):
            return {"list": list, "dict": dict, "tuple": tuple, "set": set, "frozenset": frozenset,
                    "object": Stub}[name]
        if module.startswith("builtins"):
            raise UnsafeArtifactError(f"refusing builtin {name}")
        return type(name, (Stub,), {"qualname": f"{module}.{name}"})

    def _load_build(self):
        state = self.stack.pop()
        inst = self.stack[-1]
        if isinstance(inst, _ArrayWrapper):
            inst.__setstate__(state)
            self.stack[-1] = self._read_array(state)
        elif isinstance(inst, np.dtype):
            inst.__setstate__(state)
        elif isinstance(inst, Stub):
            inst.__setstate__(state)
        else:
            raise UnsafeArtifactError(f"BUILD on unexpected object {type(inst)}")

    def _read_array(self, st):
        dtype = st["dtype"]
        shape = tuple(st["shape"])
        if dtype.hasobject:
            nested = _SafeUnpickler(self._fh).load()
            data = nested.state[-1] if isinstance(nested, Stub) and isinstance(nested.state, tuple) else nested
            return np.array(list(data), dtype=object).reshape(shape)
        if st.get("numpy_array_alignment_bytes") is not None:
            pad = self._fh.read(1)[0]
            self._fh.read(pad)
        count = int(np.prod(shape)) if shape else 1
        raw = self._fh.read(count * dtype.itemsize)
        arr = np.frombuffer(raw, dtype=dtype).copy()
        order = st.get("order", "C")
        return arr.reshape(shape, order="F" if order == "F" else "C")

    dispatch = dict(pickle._Unpickler.dispatch)
    dispatch[pickle.BUILD[0]] = _load_build


def decode(path_or_bytes) -> object:
    if isinstance(path_or_bytes, (bytes, bytearray)):
        fh = io.BytesIO(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            fh = io.BytesIO(f.read())
    head = fh.read(2)
    fh.seek(0)
    if head[:1] in (b"\x1f", b"x") or head == b"ZF":
        raise UnsafeArtifactError("compressed joblib artifacts are not supported by the safe decoder")
    return _SafeUnpickler(fh).load()


def decode_logistic(path) -> dict:
    st = decode(path).state
    return {"coef": np.asarray(st["coef_"], dtype=np.float64), "intercept": np.asarray(st["intercept_"], np.float64),
            "classes": np.asarray(st["classes_"]), "n_iter": np.asarray(st.get("n_iter_", [0])),
            "C": float(st.get("C", 1.0)), "penalty": st.get("penalty", "l2"), "solver": st.get("solver", "lbfgs"),
            "max_iter": int(st.get("max_iter", 100)), "tol": float(st.get("tol", 1e-4)),
            "sklearn_version": st.get("_sklearn_version")}


def decode_scaler(path) -> dict:
    st = decode(path).state
    out = {k: np.asarray(st[k]) for k in ("mean_", "var_", "scale_") if k in st}
    out["n_samples_seen"] = int(np.asarray(st.get("n_samples_seen_", 0)))
    if "feature_names_in_" in st:
        out["feature_names"] = [str(s) for s in st["feature_names_in_"]]
    out["sklearn_version"] = st.get("_sklearn_version")
    return out


def decode_list(path) -> list:
    obj = decode(path)
    if isinstance(obj, list):
        return [str(x) for x in obj]
    raise UnsafeArtifactError("artifact is not a plain list")
