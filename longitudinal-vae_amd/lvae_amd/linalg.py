"""N x N Cholesky factor / solve over the C ABI (potrf.hip): the reference's own LAPACK calls

    LK1 = torch.cholesky(K1)                          (elbo_functions.py:26)
    iK1 = torch.cholesky_solve(torch.eye(N), LK1)     (elbo_functions.py:27-28)
    logdet11 = 2 * torch.sum(torch.log(torch.diag(LK1)))   (elbo_functions.py:29)

with the same names, argument order and error behaviour (a non-positive-definite input raises
torch.linalg.LinAlgError naming the first bad leading minor, as torch.cholesky does).  Batched over
leading dims.  float64 runs the fp64 blocked potrf / trsm; float32 the exact KL's own factorisation
(f16 3-product split, fp32-equivalent) and fp64-accumulated solves.  No autograd: the exact KL's
gradients come from lvae_amd.KL_closed's analytic backward.
"""
import torch

from . import _lib

__all__ = ["cholesky", "cholesky_ex", "cholesky_solve", "solve_triangular", "cholesky_logdet"]


def _batch(A):
    if A.dim() < 2 or A.shape[-1] != A.shape[-2]:
        raise ValueError("lvae_amd.linalg: expected [..., n, n]")
    n = A.shape[-1]
    return A.reshape(-1, n, n), n


def _check_dtype(t):
    if t.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"lvae_amd.linalg: float32 / float64 only, got {t.dtype}")


def cholesky_ex(A, upper=False):
    """(L, logdet, info) of A [..., n, n] (lower triangle read): L lower with a zero strict upper part,
    logdet = log|A| (fp64, [...]), info LAPACK-style ([...], int32; 0 = ok).  Never raises on info."""
    _check_dtype(A)
    Ab, n = _batch(A.contiguous())
    L = Ab.shape[0]
    lib = _lib.lib()
    out = torch.empty_like(Ab)
    logdet = torch.empty(L, dtype=torch.float64, device=A.device)
    info = torch.empty(L, dtype=torch.int32, device=A.device)
    st = _lib.stream_ptr(A.device)
    nn = n * n
    if A.dtype == torch.float64:
        rc = lib.lvae_potrf_f64(n, L, _lib.ptr(Ab), n, nn, _lib.ptr(out), n, nn, _lib.ptr(logdet), _lib.ptr(info), st)
    else:
        ws = torch.empty(int(lib.lvae_potrf_f32_workspace_size(n, L)), dtype=torch.uint8, device=A.device)
        rc = lib.lvae_potrf_f32(n, L, _lib.ptr(Ab), n, nn, _lib.ptr(out), n, nn, _lib.ptr(logdet), _lib.ptr(info),
                                _lib.ptr(ws), st)
    _lib.check(rc, "potrf")
    out = out.reshape(A.shape)
    if upper:
        out = out.transpose(-1, -2)
    return out, logdet.reshape(A.shape[:-2]), info.reshape(A.shape[:-2])


def _raise_info(info, what):
    bad = info.reshape(-1).nonzero()
    if bad.numel():
        b = int(bad[0, 0])
        raise torch.linalg.LinAlgError(
            f"{what}: batch element {b}: the leading minor of order {int(info.reshape(-1)[b])} is not "
            "positive-definite")


def cholesky(A, upper=False):
    """torch.cholesky(A) on the GPU (elbo_functions.py:26)."""
    L, _, info = cholesky_ex(A, upper)
    _raise_info(info, "lvae_amd.linalg.cholesky")
    return L


def cholesky_logdet(A):
    """(L, log|A|): the factor and elbo_functions.py:29's 2 sum log diag(L) in one call."""
    L, logdet, info = cholesky_ex(A)
    _raise_info(info, "lvae_amd.linalg.cholesky_logdet")
    return L, logdet


def _solve(Lf, B, sweeps):
    _check_dtype(Lf)
    if B.dtype != Lf.dtype:
        raise TypeError("lvae_amd.linalg: B and the factor must share a dtype")
    Lb, n = _batch(Lf.contiguous())
    if B.shape[-2] != n:
        raise ValueError("lvae_amd.linalg: B rows must match the factor")
    nrhs = B.shape[-1]
    batch = B.shape[:-2]
    if batch != Lf.shape[:-2]:
        raise ValueError("lvae_amd.linalg: B's batch shape must match the factor's")
    X = B.contiguous().clone().reshape(-1, n, nrhs)
    L = Lb.shape[0]
    lib = _lib.lib()
    ws = torch.empty(int(lib.lvae_trsm_workspace_size(n, L)), dtype=torch.uint8, device=B.device)
    st = _lib.stream_ptr(B.device)
    f64 = Lf.dtype == torch.float64
    if sweeps == "potrs":
        fn = lib.lvae_potrs_f64 if f64 else lib.lvae_potrs_f32
        rc = fn(n, nrhs, L, _lib.ptr(Lb), n, n * n, _lib.ptr(X), nrhs, n * nrhs, _lib.ptr(ws), st)
    else:
        fn = lib.lvae_trsm_f64 if f64 else lib.lvae_trsm_f32
        rc = fn(int(sweeps), n, nrhs, L, _lib.ptr(Lb), n, n * n, _lib.ptr(X), nrhs, n * nrhs, _lib.ptr(ws), st)
    _lib.check(rc, "potrs" if sweeps == "potrs" else "trsm")
    return X.reshape(B.shape)


def cholesky_solve(B, L, upper=False):
    """torch.cholesky_solve(B, L): A^-1 B with A = L L^T (elbo_functions.py:27-28)."""
    if upper:
        L = L.transpose(-1, -2)
    return _solve(L, B, "potrs")


def solve_triangular(L, B, transpose=False):
    """op(L)^-1 B for lower-triangular L (op = L, or L^T with transpose=True)."""
    return _solve(L, B, 1 if transpose else 0)
