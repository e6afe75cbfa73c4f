"""Per-workgroup probes of the sweep's interior update (sw_update_kernel<kSwU2>, pass k = 4) from the
-DLVAE_PV_TIMING build (diagnostic; wall clock 100 MHz): prologue / K loop / epilogue shares."""
import ctypes, os, sys
import numpy as np
import torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblvae_pvt.so"))
lib.lvae_spd_sweep_scratch_size.restype = ctypes.c_size_t
n, L = 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 16
torch.manual_seed(0)
X = torch.randn(L, n, n, device="cuda") / n ** 0.5
A0 = (X @ X.transpose(1, 2)).contiguous()
A0.diagonal(dim1=1, dim2=2).add_(1.0)
del X
scr = torch.zeros(lib.lvae_spd_sweep_scratch_size(n, L) // 4 + 64, device="cuda")
Kinv = torch.empty_like(A0)
ld = torch.zeros(L, dtype=torch.float64, device="cuda")
info = torch.zeros(L, dtype=torch.int32, device="cuda")
out = np.zeros(4096 * 6, dtype=np.uint64)
for rep in range(3):
    A = A0.clone()
    rc = lib.lvae_u2_timing(n, L, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(scr.data_ptr()),
                            ctypes.c_void_p(Kinv.data_ptr()), ctypes.c_void_p(ld.data_ptr()),
                            ctypes.c_void_p(info.data_ptr()), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
nt = n // 256
nwg = (nt - 2) * (nt - 1) // 2 * L
t = out.reshape(4096, 6)[:nwg].astype(np.int64)
t0 = t[:, 0].min()
start, staged, loop_end, end, wait, smid = (t[:, i] for i in range(6))
span = (end.max() - t0) / 100
print(f"U2 k=4: {nwg} workgroups, span {span:.1f} us")
d = lambda x: x / 100
print(f"per workgroup (us): total {d(end - start).mean():.2f} (min {d(end - start).min():.2f} max {d(end - start).max():.2f})")
print(f"  prologue (first chunk staged) {d(staged - start).mean():.2f}")
print(f"  K loop (7 more chunks)        {d(loop_end - staged).mean():.2f}  of which waits {d(wait).mean():.2f}")
print(f"  epilogue (C stores drained)   {d(end - loop_end).mean():.2f}")
# occupancy over time: how many workgroups are live, in 5-us bins
bins = np.arange(0, span + 5, 5)
live = [int(((start - t0) / 100 <= b).sum() - ((end - t0) / 100 <= b).sum()) for b in bins]
print("live workgroups per 5 us:", live)
order = np.argsort(start)
print("first starts (us):", list(np.round((start[order[:8]] - t0) / 100, 2)),
      "last starts:", list(np.round((start[order[-8:]] - t0) / 100, 2)))
print("gap between a CU's consecutive workgroups (us):", end="")
gaps = []
for s in np.unique(smid):
    idx = np.where(smid == s)[0]
    o = idx[np.argsort(start[idx])]
    gaps += list((start[o[1:]] - end[o[:-1]]) / 100)
if gaps:
    print(f" mean {np.mean(gaps):.2f} p90 {np.percentile(gaps, 90):.2f}; distinct smid {len(np.unique(smid))}")
