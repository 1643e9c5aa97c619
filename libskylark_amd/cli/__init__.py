"""Command-line tools (reference ``nla/skylark_*.cpp``, ``ml/skylark_*.cpp``).

Run as ``python -m libskylark_amd.cli.<tool>`` (or ``torchrun ... -m`` for one
process per GPU): ``svd``, ``linear``, ``ml``, ``krr``, ``community``,
``graph_se``, ``convert2hdf5``.
"""
TOOLS = ("svd", "linear", "ml", "krr", "community", "graph_se", "convert2hdf5")
