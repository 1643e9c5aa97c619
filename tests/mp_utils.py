"""Multi-process (gloo, CPU) harness: run fn(rank, world, *args) in world ranks."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Arr:
    """A tensor result carried as a plain numpy array: torch's queue pickling
    shares CPU tensors through file descriptors served by the CHILD, which
    may already have exited when the parent unpickles (FileNotFoundError)."""

    def __init__(self, t):
        self.a = t.detach().cpu().numpy()


def _pack(x):
    import torch
    if isinstance(x, torch.Tensor):
        return _Arr(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_pack(v) for v in x)
    if isinstance(x, dict):
        return {k: _pack(v) for k, v in x.items()}
    return x


def _unpack(x):
    import torch
    if isinstance(x, _Arr):
        return torch.from_numpy(x.a)
    if isinstance(x, (list, tuple)):
        return type(x)(_unpack(v) for v in x)
    if isinstance(x, dict):
        return {k: _unpack(v) for k, v in x.items()}
    return x


def _worker(rank, world, port, fn, args, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        q.put((rank, "ok", _pack(res)))
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
    finally:
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def run_distributed(fn, world=2, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, status, res = q.get(timeout=timeout)
        if status != "ok":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {rank} failed:\n{res}")
        results[rank] = _unpack(res)
    for p in procs:
        p.join(timeout=30)
    return [results[r] for r in range(world)]
