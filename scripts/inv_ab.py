"""Dev: wall time of the C-ABI SPD inverse (lvae_spd_inv_chol_f32: potrf + trtri + lauum) on L random SPD
matrices, np = 4096, under the schedule switches in the environment (LVAE_CI_PIPE, LVAE_CI_PIPE_LAUUM,
LVAE_CI_PAIR, LVAE_PIVOT_SPLIT) -- one process per setting (they are read once); prints median / min of
REPS timed calls (HIP events) and the residual |I - A X|_max of the last one."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
from lvae_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    L = int(os.environ.get("L", "2"))
    np_ = int(os.environ.get("NP", "4096"))
    reps = int(os.environ.get("REPS", "30"))
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(L, np_, 256, device="cuda", generator=g)
    A0 = X @ X.transpose(1, 2) / 256 + 0.05 * torch.eye(np_, device="cuda")
    scratch = torch.empty(lib.lvae_spd_inv_chol_scratch_size(np_, L), dtype=torch.uint8, device="cuda")
    Ainv = torch.empty_like(A0)
    logdet = torch.empty(L, dtype=torch.float64, device="cuda")
    info = torch.empty(L, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    A = A0.clone()
    ts = []
    for r in range(reps + 3):
        A.copy_(A0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = lib.lvae_spd_inv_chol_f32(np_, L, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
                                       ctypes.c_void_p(Ainv.data_ptr()), ctypes.c_void_p(logdet.data_ptr()),
                                       ctypes.c_void_p(info.data_ptr()), ctypes.c_void_p(st))
        e1.record()
        assert rc == 0
        torch.cuda.synchronize()
        if r >= 3:
            ts.append(e0.elapsed_time(e1))
    assert int(info.abs().sum()) == 0
    res = (torch.eye(np_, device="cuda") - A0[0].double() @ Ainv[0].double()).abs().max().item()
    ts.sort()
    env = {k: v for k, v in os.environ.items() if k.startswith("LVAE_")}
    print(f"L={L} np={np_} {env}: median {ts[len(ts) // 2]:.3f} ms, min {ts[0]:.3f} ms, |I-AX|max {res:.2e}")


if __name__ == "__main__":
    main()
