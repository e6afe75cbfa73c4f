"""A/B of the S-GEMM cores (lvae_dev_syrk: variant 0 = 8-wave 2-stage x3_dma core, 1 = 4-wave 4-stage
x3_gemm4 core, 2 = variant 0 with the 4-row-block tile order, 3 = half tiles with two workgroups per CU,
4 = the product syrk_tiles_kernel: one split scale per dim, 5 / 6 = the chunk-major core x3_c16.hpp with a
4- / 5-stage ring, fed the same planes in the chunk-major layout) on random pre-split planes: time per
launch and agreement of the lower tiles."""
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


def chunk_major(p, L, np_):
    """[L, np, np] planes -> the c16 layout of x3_c16.hpp: [L][R][c][r][16], halves swapped on rows with bit 3."""
    x = p.view(L, np_ // 256, 256, np_ // 16, 16).permute(0, 1, 3, 2, 4).contiguous()
    sw = ((torch.arange(256, device=p.device) >> 3) & 1).bool()
    y = x.view(L, np_ // 256, np_ // 16, 256, 2, 8)
    y[:, :, :, sw] = y[:, :, :, sw].flip(-2)
    return y.reshape(-1)


def run(np_, L, reps=5):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(L, np_, np_, device="cuda", generator=g) * 2.0 ** 12
    hi = x.half()
    lo = (x - hi.float()).half()
    planes = torch.cat([hi.reshape(-1), lo.reshape(-1)]).contiguous()
    planes_c16 = torch.cat([chunk_major(hi, L, np_), chunk_major(lo, L, np_)]).contiguous() \
        if any(v >= 5 for v in VARIANTS) else None
    rsc = torch.ones(L, np_, device="cuda")
    out = {}
    for v in VARIANTS:
        S = torch.zeros(L, np_, np_, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        pl = planes_c16 if v >= 5 else planes
        for _ in range(2):
            assert lib.lvae_dev_syrk(v, np_, L, rsc.data_ptr(), pl.data_ptr(), S.data_ptr(), st) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            lib.lvae_dev_syrk(v, np_, L, rsc.data_ptr(), pl.data_ptr(), S.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flops = L * np_ * np_ * (np_ + 1)
        out[v] = (ms, S)
        print(f"np={np_} L={L} variant {v}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TF (fp32-equiv), "
              f"{flops / ms / 1e9 / 833.3:.3f} of x3 peak", flush=True)
    tril = torch.tril(torch.ones(np_, np_, device="cuda", dtype=torch.bool))
    b = out[VARIANTS[0]][1][:, tril]
    for v in VARIANTS[1:]:
        a = out[v][1][:, tril]
        print(f"  variant {v} vs {VARIANTS[0]}: max rel diff {float((a - b).abs().max() / b.abs().max()):.2e}", flush=True)


VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,2").split(",")]

if __name__ == "__main__":
    run(4096, 16)
    run(4096, 2)
    run(16384, 4, reps=2)
