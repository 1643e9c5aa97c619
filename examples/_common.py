"""Shared helpers for the example scripts (device choice, timing, imports)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def device(arg: str | None = None) -> torch.device:
    if arg:
        return torch.device(arg)
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


class Timer:
    def __init__(self, label: str):
        self.label = label

    def __enter__(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.t = time.perf_counter()
        print(f"{self.label}... ", end="", flush=True)
        return self

    def __exit__(self, *a):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        print(f"took {time.perf_counter() - self.t:.2e} sec", flush=True)
