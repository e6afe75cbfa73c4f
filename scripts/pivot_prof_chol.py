"""Dev: pivot 1's Cholesky split (a -DLVAE_PV_STAMP_CHOL build, LVAE_LIB), mean over dims: load + pending update,
per 32-column panel q the panel chain and the trailing update, then the rest (32 x 32 inverses, doubling, out), in us."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
from lvae_amd import _lib  # noqa: E402

lib = ctypes.CDLL(os.environ.get("LVAE_LIB", _lib.LIB_PATH))
lib.lvae_dev_pivot_prof.argtypes = [ctypes.c_void_p]
lib.lvae_spd_inv_chol_scratch_size.restype = ctypes.c_size_t
lib.lvae_spd_inv_chol_scratch_size.argtypes = [ctypes.c_int, ctypes.c_int]
lib.lvae_spd_inv_chol_f32.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6


def run(L, np_=4096, reps=3):
    nt = np_ // 256
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(L, np_, 256, device="cuda", generator=g)
    A0 = X @ X.transpose(1, 2) / 256 + 0.05 * torch.eye(np_, device="cuda")
    scratch = torch.empty(lib.lvae_spd_inv_chol_scratch_size(np_, L), dtype=torch.uint8, device="cuda")
    Ainv = torch.empty_like(A0)
    logdet = torch.empty(L, dtype=torch.float64, device="cuda")
    info = torch.empty(L, dtype=torch.int32, device="cuda")
    prof = torch.zeros(nt * L * 8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for r in range(reps + 1):
        A = A0.clone()
        lib.lvae_dev_pivot_prof(prof.data_ptr() if r == reps else None)
        rc = lib.lvae_spd_inv_chol_f32(np_, L, A.data_ptr(), scratch.data_ptr(), Ainv.data_ptr(), logdet.data_ptr(),
                                       info.data_ptr(), st)
        assert rc == 0
        torch.cuda.synchronize()
    lib.lvae_dev_pivot_prof(None)
    t = prof.view(nt, L, 8).double().cpu() / 100.0
    st = torch.cat([t[1], t[2], t[3]], dim=1)[:, :19]  # [L, 19]: stamps 0 .. 18 of pivot 1
    d = (st[:, 1:] - st[:, :-1]).mean(dim=0).tolist()
    parts = [f"load+pend {d[0]:.1f}"] + [f"q{q}: panel {d[1 + 2 * q]:.1f} upd {d[2 + 2 * q]:.1f}" for q in range(8)]
    parts.append(f"rest {d[17]:.1f}")
    print(f"L={L} pivot 1: " + ", ".join(parts) + f"; total {sum(d):.1f} us")

if __name__ == "__main__":
    for L in (2, 16):
        run(L)
