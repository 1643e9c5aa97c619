"""Every example script runs end to end (small sizes, CPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("hp_dense.py", ["--m", "500", "--n", "60", "--s", "20"]),
         ("elemental.py", ["--m", "600", "--n", "10", "--t", "60"]),
         ("least_squares.py", ["--m", "2000", "--n", "20"]),
         ("condest.py", ["--m", "400", "--n", "30"]),
         ("asynch.py", ["--n", "500"]),
         ("random_features.py", ["--rows", "300", "--dim", "8", "--numfeatures", "64"]),
         ("regression.py", ["--m", "800", "--n", "10"])]


@pytest.mark.parametrize("script,args", CASES)
def test_example_runs(script, args):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), "--device", "cpu"] + args,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "took" in r.stdout
