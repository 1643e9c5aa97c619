"""Out-of-core sketching: apply a transform to a HOST-resident dense matrix by
streaming panels through the GPU (matrices beyond aggregate HBM).

Reference analogue: the reference bounds memory by realising the sketch
panel by panel (``sketch::params::blocksize``, ``sketch/sketch_params.hpp``)
and by chunked readers (``utility/io/libsvm_io.hpp:157-322``); it has no
device, so nothing like this pipeline.  MI355X design:

* panels of A are staged in two pinned host buffers and copied to two device
  buffers on a dedicated copy stream (``non_blocking`` H2D over PCIe), so the
  copy of panel i+1 overlaps the sketch kernels of panel i on the compute
  stream; events order reuse of both buffer pairs.  A host array that is
  already pinned is copied straight from its own pages;
* ROWWISE (A S^T): row panels are independent for every transform (linear
  sketches and nonlinear feature maps alike): ``out[r0:r1] = S(panel)``;
* COLUMNWISE (S A): for linear transforms (dense and hash families) row
  panels are partial products over the sketched dimension,
  ``out += S[:, r0:r1] A[r0:r1]`` (``apply_local_shard``, the same hook the
  distributed layer uses); other transforms (FJLT's global mixing, nonlinear
  feature maps) stream independent COLUMN panels instead.

The output stays on the device (``out_device`` to move it).
"""
from __future__ import annotations

import torch

from .base import COLUMNWISE, ROWWISE, parse_dim

PANEL_BYTES = 1 << 30   # 1 GiB host panels (two pinned + two device buffers)


def _linear_shards(sk) -> bool:
    return bool(getattr(sk, "linear_shards", False))


def apply_streamed(sk, A: torch.Tensor, dim=COLUMNWISE, *, device=None, panel_bytes: int = PANEL_BYTES,
                   out_device=None) -> torch.Tensor:
    """Sketch host matrix ``A`` (dense, CPU) on ``device`` panel by panel."""
    dim = parse_dim(dim)
    if A.is_cuda or A.layout != torch.strided or A.dim() != 2:
        raise ValueError("apply_streamed expects a dense 2-D host tensor")
    if A.shape[dim] != sk.getindim():
        raise ValueError(f"sketched dimension {A.shape[dim]} != transform input size {sk.getindim()}")
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    by_rows = dim == ROWWISE or _linear_shards(sk)
    m, n = A.shape
    esz = A.element_size()
    if by_rows:
        step = max(1, min(m, panel_bytes // max(1, n * esz)))
        spans = [(r0, min(m, r0 + step)) for r0 in range(0, m, step)]
        pshape = (step, n)
    else:
        step = max(1, min(n, panel_bytes // max(1, m * esz)))
        spans = [(c0, min(n, c0 + step)) for c0 in range(0, n, step)]
        pshape = (m, step)

    def panel_of(src, a, b):
        return src[a:b] if by_rows else src[:, a:b]

    out = None

    def consume(P, a, b):
        nonlocal out
        if dim == ROWWISE:
            R = sk.apply(P, dim=ROWWISE)
            if out is None:
                out = torch.empty(m, R.shape[1], dtype=R.dtype, device=R.device)
            out[a:b] = R
        elif by_rows:
            R = sk.apply_local_shard(P, COLUMNWISE, a)
            out = R if out is None else out.add_(R)
        else:
            R = sk.apply(P, dim=COLUMNWISE)
            if out is None:
                out = torch.empty(R.shape[0], n, dtype=R.dtype, device=R.device)
            out[:, a:b] = R

    if dev.type != "cuda":
        for a, b in spans:
            consume(panel_of(A, a, b), a, b)
    else:
        main = torch.cuda.current_stream(dev)
        copy = torch.cuda.Stream(device=dev)
        pinned_src = A.is_pinned()
        nbuf = min(2, len(spans))
        hbuf = [] if pinned_src else [torch.empty(pshape, dtype=A.dtype).pin_memory() for _ in range(nbuf)]
        dbuf = [torch.empty(pshape, dtype=A.dtype, device=dev) for _ in range(nbuf)]
        h2d = [torch.cuda.Event() for _ in range(nbuf)]
        used = [torch.cuda.Event() for _ in range(nbuf)]
        for i, (a, b) in enumerate(spans):
            j = i % nbuf
            w = b - a
            if pinned_src:
                src = panel_of(A, a, b)
            else:
                if i >= nbuf:
                    h2d[j].synchronize()            # pinned buffer j: previous copy done
                src = hbuf[j][:w] if by_rows else hbuf[j][:, :w]
                src.copy_(panel_of(A, a, b))        # host memcpy overlaps the device work
            dst = dbuf[j][:w] if by_rows else dbuf[j][:, :w]
            with torch.cuda.stream(copy):
                if i >= nbuf:
                    copy.wait_event(used[j])        # device buffer j consumed
                dst.copy_(src, non_blocking=True)
                h2d[j].record(copy)
            main.wait_event(h2d[j])
            consume(dst, a, b)
            used[j].record(main)
        for t in dbuf:
            t.record_stream(copy)
        # the pinned staging buffers are released to torch's host allocator,
        # which keeps them until the non_blocking copies recorded on them finish
    if out_device is not None:
        out = out.to(out_device)
    return out
