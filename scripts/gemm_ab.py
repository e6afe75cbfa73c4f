"""A/B of the S-GEMM cores (lvae_dev_syrk: variant 0 = 8-wave 2-stage x3_dma core, 1 = 4-wave 4-stage
x3_gemm4 core, 2 = variant 0 with the 4-row-block tile order, 3 = half tiles with two workgroups per CU,
4 = the product syrk_tiles_kernel: one split scale per dim) on random pre-split planes: time per launch
and agreement of the lower tiles."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
from lvae_amd import _lib  # noqa: E402

lib = ctypes.CDLL(_lib.LIB_PATH)
lib.lvae_dev_syrk.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p]


def run(np_, L, reps=5):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(L, np_, np_, device="cuda", generator=g) * 2.0 ** 12
    hi = x.half()
    lo = (x - hi.float()).half()
    planes = torch.cat([hi.reshape(-1), lo.reshape(-1)]).contiguous()
    rsc = torch.ones(L, np_, device="cuda")
    out = {}
    for v in VARIANTS:
        S = torch.zeros(L, np_, np_, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            assert lib.lvae_dev_syrk(v, np_, L, rsc.data_ptr(), planes.data_ptr(), S.data_ptr(), st) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            lib.lvae_dev_syrk(v, np_, L, rsc.data_ptr(), planes.data_ptr(), S.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flops = L * np_ * np_ * (np_ + 1)
        out[v] = (ms, S)
        print(f"np={np_} L={L} variant {v}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TF (fp32-equiv), "
              f"{flops / ms / 1e9 / 833.3:.3f} of x3 peak", flush=True)
    tril = torch.tril(torch.ones(np_, np_, device="cuda", dtype=torch.bool))
    a, b = out[VARIANTS[0]][1][:, tril], out[VARIANTS[-1]][1][:, tril]
    print(f"  max rel diff {float((a - b).abs().max() / b.abs().max()):.2e}", flush=True)


VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,2").split(",")]

if __name__ == "__main__":
    run(4096, 16)
    run(4096, 2)
    run(16384, 4, reps=2)
