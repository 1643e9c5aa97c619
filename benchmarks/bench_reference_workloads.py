"""Re-run the only workloads the reference publishes timings for (BASELINE.md
table 1; notebooks/libskylark_softlayer.ipynb, 6 MPI ranks on 3 cloud VMs)
through OUR command-line tools with the reference's exact flags, on one GPU.

Data: the reference ships only the USPS *test* split
(python-skylark/skylark/datasets/usps.hdf5, 2007 x 256, read with the
built-in HDF5 reader).  Timings use synthetic data of the published shapes
(usps.train 7291 x 256 with 10 classes, cpu.train 8192 x 12 regression, the
6-vertex two-triangle graph); the BlockADMM accuracy check trains on the
first 1500 real USPS test examples and validates on the other 507 (the
reference trained on all of usps.train: 94.72 % validation accuracy).

Each line: {"workload", "phase", "ours_s", "reference_s", "speedup"}.
usage: python benchmarks/bench_reference_workloads.py [--out file.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
USPS = "/root/reference/python-skylark/skylark/datasets/usps.hdf5"


def _write_libsvm(path, X, y):
    with open(path, "w") as f:
        for i in range(X.shape[0]):
            nz = np.nonzero(X[i])[0]
            f.write(f"{y[i]:g} " + " ".join(f"{j + 1}:{X[i, j]:.6g}" for j in nz) + "\n")


def make_data(tmp):
    rng = np.random.default_rng(0)
    n, d = 7291, 256
    centers = rng.uniform(-1, 1, size=(10, d))
    y = rng.integers(1, 11, size=n)
    X = np.clip(0.6 * centers[y - 1] + 0.4 * rng.normal(size=(n, d)), -1, 1)
    _write_libsvm(f"{tmp}/usps.train", X, y)
    n, d = 8192, 12
    X = rng.normal(size=(n, d))
    y = X @ rng.normal(size=d) + 0.1 * rng.normal(size=n)
    _write_libsvm(f"{tmp}/cpu.train", X, y)
    with open(f"{tmp}/two_triangles", "w") as f:
        f.write("1 2\n2 3\n1 3\n4 5\n5 6\n4 6\n3 4\n")
    if os.path.exists(USPS):
        import libskylark_amd as sk
        Xr, Yr = sk.io.read_hdf5(USPS)
        _write_libsvm(f"{tmp}/usps_real_a", Xr[:1500].numpy(), Yr[:1500].numpy())
        _write_libsvm(f"{tmp}/usps_real_b", Xr[1500:].numpy(), Yr[1500:].numpy())


def run_cli(tool, args, cwd):
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "-m", f"libskylark_amd.cli.{tool}"] + args, cwd=cwd,
                       capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{tool} failed:\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}")
    return r.stdout, wall


def phase(out, name):
    m = re.search(re.escape(name) + r".*?took ([0-9.e+-]+) sec", out, re.S)
    return float(m.group(1)) if m else None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        make_data(tmp)

        def emit(workload, ph, ours, ref, **extra):
            row = {"workload": workload, "phase": ph, "ours_s": ours, "reference_s": ref,
                   "speedup": round(ref / ours, 1) if ours else None, **extra}
            rows.append(row)
            print(json.dumps(row), flush=True)

        out, _ = run_cli("svd", ["-k", "10", "--prefix", f"{tmp}/usps", f"{tmp}/usps.train"], tmp)
        emit("skylark_svd -k 10 usps.train (7291x256)", "Computing approximate SVD",
             phase(out, "Computing approximate SVD"), 2.29)
        out, _ = run_cli("linear", [f"{tmp}/cpu.train", f"{tmp}/cpu.sol"], tmp)
        emit("skylark_linear cpu.train (8192x12)", "Solving the least squares",
             phase(out, "Solving the least squares"), 0.317)
        out, wall = run_cli("krr", ["-a", "1", "-k", "0", "-g", "10", "-f", "1000", "--model", f"{tmp}/krr_model",
                                    f"{tmp}/usps.train"], tmp)
        emit("skylark_krr -a 1 -k 0 -g 10 -f 1000 usps.train", "total training",
             phase(out, "Training"), 43.2)
        out, wall = run_cli("ml", ["-g", "10", "-k", "1", "-l", "2", "-i", "30", "-f", "1000",
                                   "--trainfile", f"{tmp}/usps.train", "--modelfile", f"{tmp}/ml_model"], tmp)
        it = re.findall(r"iteration (\d+) .*?time ([0-9.]+) seconds", out)
        emit("skylark_ml -g 10 -k 1 -l 2 -i 30 -f 1000 usps.train", "30 ADMM iterations",
             float(it[-1][1]) if it else None, 17.94)
        if os.path.exists(f"{tmp}/usps_real_a"):
            out, _ = run_cli("ml", ["-g", "10", "-k", "1", "-l", "2", "-i", "30", "-f", "1000",
                                    "--trainfile", f"{tmp}/usps_real_a", "--valfile", f"{tmp}/usps_real_b",
                                    "--modelfile", f"{tmp}/ml_model2"], tmp)
            acc = re.findall(r"accuracy ([0-9.]+)", out)
            emit("skylark_ml real USPS (train 1500 / validate 507 of usps.test)", "validation accuracy %",
                 None, None, accuracy=float(acc[-1]) if acc else None, reference_accuracy=94.72)
        out, _ = run_cli("graph_se", ["-k", "2", f"{tmp}/two_triangles", "--prefix", f"{tmp}/se"], tmp)
        emit("skylark_graph_se -k 2 two_triangles", "Computing embeddings", phase(out, "Computing embeddings"),
             3.42e-3)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
