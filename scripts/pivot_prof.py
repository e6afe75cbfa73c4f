"""Dev: phase timestamps of the potrf pivots (chol_inv.hip, lvae_dev_pivot_prof) on the C-ABI inverse of
L random SPD matrices (np = 4096): per pivot the phases (load / pending update, Cholesky panels, 32 x 32
inverses, recursive doubling, planes out) and the gap since the previous pivot ended, in us."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
from lvae_amd import _lib  # noqa: E402

lib = ctypes.CDLL(_lib.LIB_PATH)
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
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = lib.lvae_spd_inv_chol_f32(np_, L, A.data_ptr(), scratch.data_ptr(), Ainv.data_ptr(), logdet.data_ptr(),
                                       info.data_ptr(), st)
        e1.record()
        assert rc == 0
        torch.cuda.synchronize()
    lib.lvae_dev_pivot_prof(None)
    assert int(info.abs().sum()) == 0
    t = prof.view(nt, L, 8).double().cpu() / 100.0  # us (100 MHz)
    print(f"L={L} np={np_}: inverse {e0.elapsed_time(e1):.2f} ms (last rep, stamps on)")
    print("  kb   load+pend  chol   trinv  rdbl   out    total  (mean over dims)   start-spread  gap-after-prev")
    prev_end = None
    for kb in range(nt):
        s = t[kb]
        ph = [(s[:, q + 1] - s[:, q]).mean().item() for q in range(5)]
        start, end = s[:, 0].min().item(), s[:, 5].max().item()
        spread = (s[:, 0].max() - s[:, 0].min()).item()
        gap = start - prev_end if prev_end is not None else 0.0
        print(f"  {kb:2d}  " + "  ".join(f"{p:6.1f}" for p in ph) + f"  {sum(ph):6.1f}   {spread:8.1f}   {gap:8.1f}")
        prev_end = end


if __name__ == "__main__":
    for L in [int(x) for x in os.environ.get("LS", "16,2").split(",")]:
        run(L)
