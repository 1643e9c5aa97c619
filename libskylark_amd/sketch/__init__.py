"""Sketching transforms (reference ``sketch/``, ``python-skylark/skylark/sketch.py``)."""
from . import params  # noqa: F401
from .base import (COLUMNWISE, ROWWISE, SketchTransform, deserialize_sketch, from_json, from_ptree,
                   parse_dim, sketch_class, supported_sketch_transforms)
from .dense import CT, JLT, SJLT, SparseJLT
from .fjlt import FJLT, NURST, RFUT, UST, URST, FastJLT, NonUniformSampler, UniformSampler
from .frft import PPT, FastGaussianRFT, FastMaternRFT, Fastfood
from .hash import CWT, MMT, WZT, CountSketch
from .rft import (ExpSemigroupQRLT, ExpSemigroupRLT, GaussianQRFT, GaussianRFT, LaplacianQRFT,
                  LaplacianRFT, MaternRFT)

columnwise, rowwise = COLUMNWISE, ROWWISE
TensorSketch = PPT
RRT = GaussianRFT
MaternFastfood = FastMaternRFT

__all__ = [
    "COLUMNWISE", "ROWWISE", "SketchTransform", "deserialize_sketch", "from_json", "from_ptree",
    "JLT", "CT", "SJLT", "SparseJLT", "NURST", "NonUniformSampler", "UniformSampler", "FJLT", "FastJLT", "RFUT", "UST", "URST", "CWT", "CountSketch", "MMT", "WZT",
    "PPT", "TensorSketch", "RRT", "MaternFastfood", "GaussianRFT", "LaplacianRFT", "MaternRFT", "GaussianQRFT",
    "LaplacianQRFT", "FastGaussianRFT", "Fastfood", "FastMaternRFT", "ExpSemigroupRLT",
    "ExpSemigroupQRLT", "supported_sketch_transforms", "sketch_class", "parse_dim",
]
