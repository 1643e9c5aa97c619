"""CountSketch-family application (hash_transform_t), native on gfx950.

GPU tensors go through the bucketed HIP kernels of ``hash_kernels.hip``; CPU
tensors (plumbing path) use torch ``index_add_``.  See the kernel file for the
design.  Determinism: dense inputs and rowwise CSR with short rows are always
bit-reproducible (no atomics); columnwise CSR accumulates with LDS float
atomics unless ``sketch.params.set_deterministic(True)``, which switches it to
int64 fixed-point accumulation (and rowwise CSR to one lane per row).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_hash_dense_colwise", [vp, i32, i64, i64, vp, vp, vp, i64, vp, i32, i64, i64, i32, vp])
_lib.register("sl_hash_dense_rowwise", [vp, i32, i64, i64, i64, vp, vp, vp, i64, vp, i32, i64, i64, i32, vp])
_lib.register("sl_hash_csr_colwise2", [vp, vp, i32, vp, i32, vp, vp, vp, i64, i64, vp, i64, i64, i32, i32, vp,
                                       C.c_double, vp])
_lib.register("sl_hash_csr_rowwise", [vp, vp, i32, vp, i32, i64, vp, vp, vp, i64, i64, i32, vp])
_lib.register("sl_cwt_csr_rowwise_sparse", [vp, vp, i32, vp, i32, i64, i32, vp, vp, i64, i32, vp, vp, vp, vp])
_lib.register("sl_cwt_csr_colwise_mark", [vp, vp, i32, i64, vp, i64, vp, i64, vp])
_lib.register("sl_dense_occ_compact", [vp, i32, i64, vp, i64, i64, i32, vp, vp, vp, i32, vp])

# dense staging limit of the columnwise CSR -> CSR path (S x ncols cells)
SPARSE_OUT_DENSE_CELLS = 1 << 28


class HashData:
    """Device-resident hash data + bucket permutation (built once per device)."""

    def __init__(self, idx: torch.Tensor, val: torch.Tensor, S: int):
        self.S = S
        self._host_idx = idx.to(torch.int64).cpu()
        self._host_val = val.to(torch.float64).cpu()
        self._cache = {}
        self.wmax = float(self._host_val.abs().max()) if self._host_val.numel() else 0.0

    def on(self, device):
        key = str(device)
        d = self._cache.get(key)
        if d is None:
            idx = self._host_idx.to(device)
            val = self._host_val.to(device)
            perm = torch.argsort(idx, stable=True)
            counts = torch.bincount(idx, minlength=self.S)
            bptr = torch.zeros(self.S + 1, dtype=torch.int64, device=device)
            bptr[1:] = torch.cumsum(counts, 0)
            d = (idx, val, perm, bptr)
            self._cache[key] = d
            self._cache[key + "/pval"] = _PVal(val[perm])
        return d

    def pval(self, device, perm=None) -> "_PVal":
        """Bucket-ordered weights ``val[perm]`` (f64 and f32), built once."""
        if perm is not None:
            return _PVal(self.on(device)[1][perm])
        self.on(device)
        return self._cache[str(device) + "/pval"]


class _PVal:
    def __init__(self, v64: torch.Tensor):
        self.f64 = v64.contiguous()
        self.f32 = v64.to(torch.float32).contiguous()

    def of(self, dt):
        return self.f64 if dt == torch.float64 else self.f32


def _group_for(avg: float) -> int:
    if avg >= 48:
        return 64
    if avg >= 12:
        return 16
    if avg >= 3:
        return 4
    return 1


def _out_dtype(dt):
    return torch.float64 if dt == torch.float64 else torch.float32


def apply_dense(hd: HashData, A: torch.Tensor, dim: int, in_offset: int = 0, out=None):
    """Columnwise (dim 0) or rowwise (dim 1) CountSketch of dense A.

    ``A`` may be a shard holding rows (dim 0) / columns (dim 1)
    ``[in_offset, in_offset + k)`` of the N-dimensional input; the result is
    the partial sketch of that shard (sum over shards = full sketch).
    """
    S = hd.S
    odt = _out_dtype(A.dtype)
    idx, val, perm, bptr = hd.on(A.device)
    if dim == 0:
        k, m = A.shape
        res = torch.zeros(S, m, dtype=odt, device=A.device) if out is None else out
        if not A.is_cuda:
            sl = slice(in_offset, in_offset + k)
            res.index_add_(0, idx[sl], A.to(odt) * val[sl].to(odt)[:, None])
            return res
        if A.stride(1) != 1:
            A = A.contiguous()
        pv = hd.pval(A.device)
        if in_offset != 0 or k != idx.numel():
            # restrict the bucket permutation to this shard's rows
            perm, bptr = _restrict(idx, in_offset, k, S)
            pv = hd.pval(A.device, perm)
        _lib.call("sl_hash_dense_colwise", _lib.ptr(A), _lib.dtype_code(A.dtype), A.stride(0), m,
                  _lib.ptr(perm), _lib.ptr(bptr), _lib.ptr(pv.f64), S, _lib.ptr(res), _lib.dtype_code(odt),
                  res.stride(0), in_offset, 1, vp(_lib.stream_of(A)))
        return res
    m, k = A.shape
    res = torch.zeros(m, S, dtype=odt, device=A.device) if out is None else out
    if not A.is_cuda:
        sl = slice(in_offset, in_offset + k)
        res.index_add_(1, idx[sl], A.to(odt) * val[sl].to(odt)[None, :])
        return res
    if A.stride(1) != 1:
        A = A.contiguous()
    esz = 8 if A.dtype == torch.float64 else 4
    if k * esz > 150 * 1024:
        sl = slice(in_offset, in_offset + k)
        res.index_add_(1, idx[sl], A.to(odt) * val[sl].to(odt)[None, :])
        return res
    if in_offset != 0 or k != idx.numel():
        perm, bptr = _restrict(idx, in_offset, k, S)
    _lib.call("sl_hash_dense_rowwise", _lib.ptr(A), _lib.dtype_code(A.dtype), A.stride(0), m, k,
              _lib.ptr(perm), _lib.ptr(bptr), _lib.ptr(val), S, _lib.ptr(res), _lib.dtype_code(odt),
              res.stride(0), in_offset, 1, vp(_lib.stream_of(A)))
    return res


def _restrict(idx, off, k, S):
    sub = idx[off:off + k]
    perm = torch.argsort(sub, stable=True) + off
    counts = torch.bincount(sub, minlength=S)
    bptr = torch.zeros(S + 1, dtype=torch.int64, device=idx.device)
    bptr[1:] = torch.cumsum(counts, 0)
    return perm, bptr


def _csr_parts(A: torch.Tensor):
    rp = A.crow_indices()
    ci = A.col_indices()
    vals = A.values()
    if rp.dtype != torch.int64:
        rp = rp.to(torch.int64)
    if vals.dtype not in (torch.float32, torch.float64):
        vals = vals.to(torch.float32)
    return rp.contiguous(), ci.contiguous(), vals.contiguous()


def apply_csr_dense_out(hd: HashData, A: torch.Tensor, dim: int, in_offset: int = 0):
    """CountSketch of a CSR matrix into a dense result."""
    S = hd.S
    vdt = A.values().dtype
    odt = torch.float64 if vdt == torch.float64 else torch.float32
    idx, val, perm, bptr = hd.on(A.device)
    nrows, ncols = A.shape
    if not A.is_cuda:
        coo = A.to_sparse_coo().coalesce()
        r, c = coo.indices()
        v = coo.values().to(odt)
        if dim == 0:
            res = torch.zeros(S, ncols, dtype=odt)
            res.index_put_((idx[r + in_offset], c), v * val[r + in_offset].to(odt), accumulate=True)
        else:
            res = torch.zeros(nrows, S, dtype=odt)
            res.index_put_((r, idx[c + in_offset]), v * val[c + in_offset].to(odt), accumulate=True)
        return res
    rp, ci, vals = _csr_parts(A)
    idx32 = 1 if ci.dtype == torch.int32 else 0
    if ci.dtype not in (torch.int32, torch.int64):
        ci = ci.to(torch.int64)
        idx32 = 0
    avg = vals.numel() / max(1, nrows)
    st = vp(_lib.stream_of(A))
    if dim == 0:
        res = torch.empty(S, ncols, dtype=odt, device=A.device)   # every cell is stored by its workgroup
        _csr_colwise(hd, A.device, rp, ci, idx32, vals, S, ncols, res, in_offset, avg, st)
    else:
        res = torch.zeros(nrows, S, dtype=odt, device=A.device)
        # one lane per row (atomic-free, deterministic) unless rows are long
        g = 1 if (_det() or avg < 12) else _group_for(avg)
        _lib.call("sl_hash_csr_rowwise", _lib.ptr(rp), _lib.ptr(ci), idx32, _lib.ptr(vals),
                  _lib.dtype_code(vals.dtype), nrows, _lib.ptr(idx), _lib.ptr(val), _lib.ptr(res),
                  res.stride(0), in_offset, g, st)
    return res


def _det() -> bool:
    from ..sketch import params
    return params.get_deterministic()


def _csr_colwise(hd, device, rp, ci, idx32, vals, S, ncols, res, in_offset, avg, st):
    """res (S x ncols, fully overwritten) = columnwise CountSketch of CSR rows
    [in_offset, in_offset + nrows)."""
    idx, val, perm, bptr = hd.on(device)
    nrows = rp.numel() - 1
    pv = hd.pval(device)
    if in_offset != 0 or nrows != idx.numel():
        perm, bptr = _restrict(idx, in_offset, nrows, S)
        pv = hd.pval(device, perm)
    det = _det()
    vmax = vals.abs().max().to(torch.float64).reshape(1) if (det and vals.numel()) else \
        torch.zeros(1, dtype=torch.float64, device=device)
    _lib.call("sl_hash_csr_colwise2", _lib.ptr(rp), _lib.ptr(ci), idx32, _lib.ptr(vals),
              _lib.dtype_code(vals.dtype), _lib.ptr(perm), _lib.ptr(bptr), _lib.ptr(pv.of(vals.dtype)), S, ncols,
              _lib.ptr(res), res.stride(0), in_offset, _group_for(avg), int(det), _lib.ptr(vmax), hd.wmax, st)


def apply_csr_sparse_out(hd: HashData, A: torch.Tensor, dim: int, in_offset: int = 0):
    """CountSketch CSR -> CSR (reference sketch/hash_transform_local_sparse.hpp:88-223):
    duplicate (row, col) pairs produced by the hashing are merged.  GPU inputs
    run the sort-free kernels of ``hash_sparse_out.hip``; shapes they do not
    cover (rowwise rows longer than 32 entries, a columnwise result beyond
    ``SPARSE_OUT_DENSE_CELLS``) take the generic coalesce."""
    if A.is_cuda:
        out = _csr_sparse_out_native(hd, A, dim, in_offset)
        if out is not None:
            return out
    return _csr_sparse_out_generic(hd, A, dim, in_offset)


def _finish_csr(cnt, nr, nc, fill, vdt, device):
    crow = torch.zeros(nr + 1, dtype=torch.int64, device=device)
    torch.cumsum(cnt, 0, out=crow[1:])
    nnz = int(crow[-1].item())
    ocol = torch.empty(nnz, dtype=torch.int64, device=device)
    oval = torch.empty(nnz, dtype=vdt, device=device)
    if nnz:
        fill(crow, ocol, oval)
    return torch.sparse_csr_tensor(crow, ocol, oval, size=(nr, nc))


def _csr_sparse_out_native(hd: HashData, A: torch.Tensor, dim: int, in_offset: int):
    S = hd.S
    idx, val, perm, bptr = hd.on(A.device)
    nrows, ncols = A.shape
    rp, ci, vals = _csr_parts(A)
    idx32 = 1 if ci.dtype == torch.int32 else 0
    if ci.dtype not in (torch.int32, torch.int64):
        ci, idx32 = ci.to(torch.int64), 0
    vdt = vals.dtype
    st = vp(_lib.stream_of(A))
    dev = A.device
    if dim == 1:
        maxlen = int((rp[1:] - rp[:-1]).max().item()) if nrows else 0
        if maxlen > 32:
            return None
        cnt = torch.empty(nrows, dtype=torch.int64, device=dev)
        args = (_lib.ptr(rp), _lib.ptr(ci), idx32, _lib.ptr(vals), _lib.dtype_code(vdt), nrows, maxlen,
                _lib.ptr(idx), _lib.ptr(val), in_offset)
        _lib.call("sl_cwt_csr_rowwise_sparse", *args, 0, _lib.ptr(cnt), None, None, st)
        return _finish_csr(cnt, nrows, S, lambda crow, oc, ov: _lib.call(
            "sl_cwt_csr_rowwise_sparse", *args, 1, _lib.ptr(crow), _lib.ptr(oc), _lib.ptr(ov), st), vdt, dev)
    if S * ncols > SPARSE_OUT_DENSE_CELLS:
        return None
    dense = torch.empty(S, ncols, dtype=vdt, device=dev)
    avg = vals.numel() / max(1, nrows)
    _csr_colwise(hd, dev, rp, ci, idx32, vals, S, ncols, dense, in_offset, avg, st)
    occ = torch.zeros(S, ncols, dtype=torch.uint8, device=dev)
    _lib.call("sl_cwt_csr_colwise_mark", _lib.ptr(rp), _lib.ptr(ci), idx32, nrows, _lib.ptr(idx), in_offset,
              _lib.ptr(occ), ncols, st)
    cnt = torch.empty(S, dtype=torch.int64, device=dev)
    dc = _lib.dtype_code(vdt)
    _lib.call("sl_dense_occ_compact", _lib.ptr(dense), dc, dense.stride(0), _lib.ptr(occ), S, ncols, 0,
              _lib.ptr(cnt), None, None, dc, st)
    return _finish_csr(cnt, S, ncols, lambda crow, oc, ov: _lib.call(
        "sl_dense_occ_compact", _lib.ptr(dense), dc, dense.stride(0), _lib.ptr(occ), S, ncols, 1,
        _lib.ptr(crow), _lib.ptr(oc), _lib.ptr(ov), dc, st), vdt, dev)


def _csr_sparse_out_generic(hd: HashData, A: torch.Tensor, dim: int, in_offset: int = 0):
    S = hd.S
    idx, val, _, _ = hd.on(A.device)
    coo = A.to_sparse_coo().coalesce()
    r, c = coo.indices()
    v = coo.values()
    vdt = v.dtype if v.dtype in (torch.float32, torch.float64) else torch.float32
    if dim == 0:
        nr, nc = S, A.shape[1]
        ii = torch.stack([idx[r + in_offset], c])
        vv = v.to(vdt) * val[r + in_offset].to(vdt)
    else:
        nr, nc = A.shape[0], S
        ii = torch.stack([r, idx[c + in_offset]])
        vv = v.to(vdt) * val[c + in_offset].to(vdt)
    out = torch.sparse_coo_tensor(ii, vv, size=(nr, nc)).coalesce()
    return out.to_sparse_csr()
