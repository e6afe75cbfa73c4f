"""Phase timestamps of sw_pivot_kernel (block 0) from the -DLVAE_PV_TIMING build (diagnostic)."""
import ctypes, os, sys
import torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblvae_pvt.so"))
lib.lvae_pv_timing.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p]
lib.lvae_spd_sweep_scratch_size.restype = ctypes.c_size_t
n, L = 256, int(sys.argv[1]) if len(sys.argv) > 1 else 16
g = torch.Generator().manual_seed(0)
X = torch.randn(L, n, n, generator=g, dtype=torch.float64) / n ** 0.5
A = (X @ X.transpose(1, 2) + torch.eye(n, dtype=torch.float64)).float().cuda().contiguous()
scr = torch.zeros(lib.lvae_spd_sweep_scratch_size(n, L) // 4, device="cuda")
ld = torch.zeros(L, dtype=torch.float64, device="cuda")
info = torch.zeros(L, dtype=torch.int32, device="cuda")
out = (ctypes.c_ulonglong * 64)()
for rep in range(3):
    A2 = A.clone()
    rc = lib.lvae_pv_timing(A2.data_ptr(), n, L, scr.data_ptr(), ld.data_ptr(), info.data_ptr(), out)
t = [out[i] for i in range(32)]
names = {0: "start", 1: "load"}
for q in range(8):
    names[2 + 2 * q] = f"panel{q}"
    names[3 + 2 * q] = f"trail{q}"
names.update({20: "diag inv", 24: "trtri64", 21: "trtri", 22: "lauum", 23: "out"})
prev = t[0]
for i in sorted((i for i in range(1, 32) if t[i]), key=lambda i: t[i]):
    print(f"{names.get(i, i):>18s} {(t[i] - prev) / 100:8.2f} us   (cum {(t[i] - t[0]) / 100:8.2f})")
    prev = t[i]
inv = torch.linalg.inv(A.double())
print("max rel err of -P^-1:", float(((-A2.double() - inv).abs().amax() / inv.abs().amax())))
print("rc", rc, "info", info.tolist()[:4], "logdet err", float((ld[0] / 3 - torch.logdet(A[0].double())).abs()))
