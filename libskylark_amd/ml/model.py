"""Trained-model containers with JSON persistence (reference ``ml/model.hpp:50-1255``).

Three model kinds, same JSON schema as the reference (``skylark_object_type``
``model:linear-on-features`` / ``model:kernel`` / ``model:feature_expansion``),
so model files written by either implementation load in the other:

* :class:`HilbertModel` — linear on concatenated random-feature blocks
  (BlockADMM output).  Prediction scales block j by ``sqrt(s_j / d)`` when
  ``scale_maps`` (the reference's convention, kept for file compatibility).
* :class:`KernelModel` — training points + dual coefficients; prediction is
  ``k(X_test, X_train) A``.  The file stores only the data location, as in
  the reference; loading re-reads it (LIBSVM).
* :class:`FeatureExpansionModel` — feature transforms + weights; prediction
  scales transform i by ``sqrt(S_i / total_features)``.

Classification models decode by arg-max (``rcoding`` maps column -> label;
a single-output Hilbert model predicts ``sign``).

Numbers are written as JSON numbers; reading accepts boost's all-strings
ptree encoding too.  Coefficient matrices are the reference's ``El::Print``
text (rows on lines, space separated) at full double precision.
"""
from __future__ import annotations

import json
import math

import torch

from .. import __version__
from ..sketch import ROWWISE, deserialize_sketch
from .kernels import kernel_from_dict


def _b(v) -> bool:
    if isinstance(v, str):
        return v.strip().lower() in ("1", "true", "yes")
    return bool(v)


def matrix_to_text(M: torch.Tensor) -> str:
    M = M.detach().to(torch.float64).cpu()
    return "".join(" ".join(repr(float(x)) for x in row) + "\n" for row in M.tolist())


def matrix_from_text(s: str, rows: int, cols: int) -> torch.Tensor:
    out = torch.zeros(rows, cols, dtype=torch.float64)
    lines = [ln for ln in s.split("\n") if ln.strip()]
    for i in range(min(rows, len(lines))):
        toks = lines[i].split()
        for j in range(min(cols, len(toks))):
            out[i, j] = float(toks[j])
    return out


def _read_json(fname: str) -> dict:
    with open(fname) as f:
        lines = f.readlines()
    body = "".join(ln for ln in lines if not ln.startswith("#"))
    return json.loads(body)


def _save(obj, fname: str, header: str = ""):
    with open(fname, "w") as f:
        f.write(header)
        json.dump(obj.to_dict(), f, indent=1)
        f.write("\n")


def _rcoding_to_dict(rc):
    return {str(i): v for i, v in enumerate(rc)}


def _rcoding_from_dict(d, k):
    out = []
    for i in range(k):
        v = d[str(i)]
        if isinstance(v, str):
            f = float(v)
            v = int(f) if f.is_integer() else f
        out.append(v)
    return out


def _decode_max(DV: torch.Tensor, rcoding=None):
    if DV.shape[1] == 1:
        return torch.where(DV[:, 0] >= 0, 1.0, -1.0).to(torch.float64)
    idx = DV.argmax(dim=1)
    if rcoding is None:
        return idx.to(torch.float64)
    lut = torch.tensor([float(v) for v in rcoding], dtype=torch.float64, device=DV.device)
    return lut[idx]


class HilbertModel:
    """Linear model on random features (reference ``hilbert_model_t`` ``:50-275``)."""

    object_type = "model:linear-on-features"

    def __init__(self, maps, scale_maps: bool, num_features: int, num_outputs: int, regression: bool,
                 coef: torch.Tensor | None = None, input_size: int | None = None):
        self.maps = list(maps)
        self.scale_maps = bool(scale_maps)
        self.regression = bool(regression)
        self.coef = coef if coef is not None else torch.zeros(num_features, num_outputs, dtype=torch.float64)
        self.starts, nf = [], 0
        for S in self.maps:
            self.starts.append(nf)
            nf += S.get_S()
        self.input_size = input_size if input_size is not None else (
            num_features if not self.maps else self.maps[0].get_N())

    def get_coef(self):
        return self.coef

    def get_output_size(self):
        return self.coef.shape[1]

    def get_input_size(self):
        return self.input_size

    def is_regression(self):
        return self.regression

    def decision_function(self, X: torch.Tensor) -> torch.Tensor:
        """n x k decision values for examples as ROWS of X (n x d)."""
        X = X.to_dense() if X.layout != torch.strided else X
        W = self.coef.to(X.device)
        if not self.maps:
            return X.to(W.dtype) @ W
        d = X.shape[1]
        DV = torch.zeros(X.shape[0], W.shape[1], dtype=W.dtype, device=X.device)
        for S, st in zip(self.maps, self.starts):
            sj = S.get_S()
            Z = S.apply(X, dim=ROWWISE).to(W.dtype)
            if self.scale_maps:
                Z = Z * math.sqrt(sj / d)
            DV += Z @ W[st:st + sj]
        return DV

    def predict(self, X: torch.Tensor):
        """Returns ``(labels_or_values, decision_values)``."""
        DV = self.decision_function(X)
        if self.regression:
            return DV, DV
        return _decode_max(DV), DV

    def to_dict(self) -> dict:
        return {
            "skylark_object_type": self.object_type, "skylark_version": __version__,
            "num_features": int(self.coef.shape[0]), "num_outputs": int(self.coef.shape[1]),
            "input_size": int(self.input_size), "regression": self.regression,
            "feature_mapping": {"number_maps": len(self.maps), "scale_maps": self.scale_maps,
                                "maps": {str(i): S.to_dict() for i, S in enumerate(self.maps)}},
            "coef_matrix": matrix_to_text(self.coef),
        }

    to_ptree = to_dict

    @classmethod
    def from_dict(cls, pt: dict) -> "HilbertModel":
        nf, no = int(pt["num_features"]), int(pt["num_outputs"])
        fm = pt["feature_mapping"]
        nmaps = int(fm["number_maps"])
        maps = [deserialize_sketch(fm["maps"][str(i)]) for i in range(nmaps)] if nmaps else []
        coef = matrix_from_text(pt["coef_matrix"], nf, no)
        return cls(maps, _b(fm["scale_maps"]), nf, no, _b(pt["regression"]), coef, int(pt["input_size"]))

    def save(self, fname: str, header: str = ""):
        _save(self, fname, header)

    @classmethod
    def load(cls, fname: str) -> "HilbertModel":
        return cls.from_dict(_read_json(fname))


class KernelModel:
    """Dual (kernel-expansion) model (reference ``kernel_model_t`` ``:338-715``)."""

    object_type = "model:kernel"

    def __init__(self, kernel, X: torch.Tensor, A: torch.Tensor, data_location: str = "", partial: int = -1,
                 fileformat: int = 0, rcoding=None, pretransform=None, direction: str = "rows"):
        self.kernel = kernel
        self.X = X if direction == "rows" else X.t()
        self.A = A if A.dim() == 2 else A[:, None]
        self.data_location, self.partial, self.fileformat = data_location, int(partial), int(fileformat)
        self.rcoding = list(rcoding) if rcoding is not None else None
        self.pretransform = pretransform

    @property
    def regression(self):
        return self.rcoding is None

    def get_input_size(self):
        return self.kernel.get_dim()

    def get_output_size(self):
        return self.A.shape[1]

    def decision_function(self, XT: torch.Tensor) -> torch.Tensor:
        if self.pretransform is not None:
            XT = self.pretransform.apply(XT, dim=ROWWISE)
        KT = self.kernel.gram(XT.to(self.X.device), Y=self.X)  # n_test x n_train
        return KT.to(self.A.dtype) @ self.A.to(KT.device)

    def predict(self, XT: torch.Tensor):
        DV = self.decision_function(XT)
        if self.regression:
            return DV, DV
        return _decode_max(DV, self.rcoding), DV

    def to_dict(self) -> dict:
        d = {"skylark_object_type": self.object_type, "skylark_version": __version__,
             "data_location": self.data_location, "partial": self.partial, "fileformat": self.fileformat}
        if self.pretransform is not None:
            d["pre_transform"] = self.pretransform.to_dict()
        d.update({"num_outputs": int(self.A.shape[1]), "input_size": int(self.kernel.get_dim()),
                  "regression": self.regression})
        if not self.regression:
            d["rcoding"] = _rcoding_to_dict(self.rcoding)
        d["kernel"] = self.kernel.to_dict()
        d["alpha"] = matrix_to_text(self.A)
        return d

    to_ptree = to_dict

    @classmethod
    def from_dict(cls, pt: dict, X: torch.Tensor | None = None) -> "KernelModel":
        k = kernel_from_dict(pt["kernel"])
        no = int(pt["num_outputs"])
        pre = deserialize_sketch(pt["pre_transform"]) if "pre_transform" in pt else None
        if X is None:
            from ..io import read_libsvm
            X, _ = read_libsvm(pt["data_location"], min_d=int(pt["input_size"]) if pre is None else 0,
                               max_n=int(pt.get("partial", -1)))
            X = X.to_dense() if X.layout != torch.strided else X
            if pre is not None:
                X = pre.apply(X, dim=ROWWISE)
        A = matrix_from_text(pt["alpha"], X.shape[0], no)
        rc = None if _b(pt["regression"]) else _rcoding_from_dict(pt["rcoding"], no)
        return cls(k, X, A, pt.get("data_location", ""), int(pt.get("partial", -1)), int(pt.get("fileformat", 0)),
                   rc, pre)

    def save(self, fname: str, header: str = ""):
        _save(self, fname, header)

    @classmethod
    def load(cls, fname: str, X: torch.Tensor | None = None) -> "KernelModel":
        return cls.from_dict(_read_json(fname), X)


class FeatureExpansionModel:
    """Weights over explicit feature transforms (reference ``feature_expansion_model_t`` ``:720-1130``)."""

    object_type = "model:feature_expansion"

    def __init__(self, transforms, W: torch.Tensor, scale_maps: bool = False, rcoding=None):
        self.transforms = list(transforms) if isinstance(transforms, (list, tuple)) else [transforms]
        self.W = W if W.dim() == 2 else W[:, None]
        self.scale_maps = bool(scale_maps)
        self.rcoding = list(rcoding) if rcoding is not None else None
        self.feature_size = sum(S.get_S() for S in self.transforms)

    @property
    def regression(self):
        return self.rcoding is None

    def get_input_size(self):
        return self.transforms[0].get_N()

    def get_output_size(self):
        return self.W.shape[1]

    def decision_function(self, XT: torch.Tensor) -> torch.Tensor:
        W = self.W.to(XT.device)
        YP = torch.zeros(XT.shape[0], W.shape[1], dtype=W.dtype, device=XT.device)
        st = 0
        for S in self.transforms:
            sj = S.get_S()
            Z = S.apply(XT, dim=ROWWISE).to(W.dtype)
            if self.scale_maps:
                Z = Z * math.sqrt(sj / self.feature_size)
            YP += Z @ W[st:st + sj]
            st += sj
        return YP

    def predict(self, XT: torch.Tensor):
        DV = self.decision_function(XT)
        if self.regression:
            return DV, DV
        return _decode_max(DV, self.rcoding), DV

    def to_dict(self) -> dict:
        d = {"skylark_object_type": self.object_type, "skylark_version": __version__,
             "num_outputs": int(self.W.shape[1]), "input_size": int(self.get_input_size()),
             "regression": self.regression}
        if not self.regression:
            d["rcoding"] = _rcoding_to_dict(self.rcoding)
        d["feature_mapping"] = {"number_transforms": len(self.transforms), "scale_maps": self.scale_maps,
                                "transforms": {str(i): S.to_dict() for i, S in enumerate(self.transforms)}}
        d["weights"] = matrix_to_text(self.W)
        return d

    to_ptree = to_dict

    @classmethod
    def from_dict(cls, pt: dict) -> "FeatureExpansionModel":
        fm = pt["feature_mapping"]
        nt = int(fm["number_transforms"])
        ts = [deserialize_sketch(fm["transforms"][str(i)]) for i in range(nt)]
        no = int(pt["num_outputs"])
        W = matrix_from_text(pt["weights"], sum(S.get_S() for S in ts), no)
        rc = None if _b(pt["regression"]) else _rcoding_from_dict(pt["rcoding"], no)
        return cls(ts, W, _b(fm["scale_maps"]), rc)

    def save(self, fname: str, header: str = ""):
        _save(self, fname, header)

    @classmethod
    def load(cls, fname: str) -> "FeatureExpansionModel":
        return cls.from_dict(_read_json(fname))


_MODELS = {c.object_type: c for c in (HilbertModel, KernelModel, FeatureExpansionModel)}


def model_from_dict(pt: dict):
    """Dispatch on ``skylark_object_type`` (reference ``model_container_t``)."""
    t = pt["skylark_object_type"]
    if t not in _MODELS:
        raise ValueError(f"unknown model type {t}")
    return _MODELS[t].from_dict(pt)


def load_model(fname: str):
    return model_from_dict(_read_json(fname))


hilbert_model_t = HilbertModel
kernel_model_t = KernelModel
feature_expansion_model_t = FeatureExpansionModel
