"""python-skylark ``skylark.ml.modeling`` (``python-skylark/skylark/ml/modeling.py``):
load a model file written by ``skylark_ml`` (our ``cli/ml.py`` writes the
same JSON) and predict with its random-feature maps."""
from __future__ import annotations

import torch

from .model import HilbertModel


class LinearizedKernelModel:
    """Linearised kernel model from a ``skylark_ml`` model file."""

    def __init__(self, fname: str):
        self._m = HilbertModel.load(fname)

    def get_input_dimension(self) -> int:
        return self._m.get_input_size()

    def predict(self, X) -> torch.Tensor:
        """Regression outputs (n x k) for a regression model; for a classifier
        the arg-max output column (0-based), as python-skylark returns."""
        D = self._m.decision_function(torch.as_tensor(X))
        return D if self._m.is_regression() else D.argmax(dim=1)
