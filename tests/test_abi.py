"""CPU-side checks of the C ABI: the library loads without a GPU and exports every symbol
include/lvae_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "lvae_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lvae_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("lvae_gram_f64", "lvae_kl_closed_fwd_f32", "lvae_kl_closed_bwd_f32", "lvae_spd_inv_chol_f32",
                 "lvae_hensman_fwd_f64", "lvae_hensman_bwd_f64", "lvae_natgrad_update_f64"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from lvae_amd import _lib
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared_symbols()) <= set(_lib.SIGNATURES), "ctypes binding lacks a declared symbol"
    assert lib.lvae_version().startswith(b"lvae_hip")


def test_spec_struct_layout():
    """ctypes mirror of lvae_kernel_spec matches the C layout (2 + 16*2 + 16*4*3 int32)."""
    from lvae_amd import _lib
    assert ctypes.sizeof(_lib.KernelSpec) == 4 * (2 + 16 * 2 + 16 * 4 * 3)
    assert ctypes.sizeof(_lib.HensmanDims) == 72  # 5 int32 + pad, 2 double, int32 + pad, double, ptr, double


def test_host_queries_need_no_gpu():
    from lvae_amd import _lib
    lib = _lib.load()
    assert lib.lvae_kl_closed_padded_n(4096) == 4096
    assert lib.lvae_kl_closed_padded_n(200) == 256
    assert lib.lvae_kl_closed_workspace_size(4096, 16) > 3 * 16 * 4096 * 4096 * 4
    d = _lib.HensmanDims(16, 120, 5, 16, 6, 256.0, 1e-6, 1, 1.0)
    ws = lib.lvae_hensman_workspace_size(ctypes.byref(d))
    off = lib.lvae_hensman_iH_offset(ctypes.byref(d))
    assert ws > 0 and off % 256 == 0 and off + 16 * 120 * 120 * 8 <= ws


def test_compute_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lvae_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.lib()


def test_spec_compilation_sample_config():
    import lvae_amd as la
    cfg = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 0, 'cat_covariate': 3},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[], covariate_missing_val=[])
    k0, k1 = la.generate_kernel_batched(4, **cfg, id_covariate=2)
    s0, p0 = la.kernel_spec_and_params(k0)
    s1, p1 = la.kernel_spec_and_params(k1)
    assert (s0.n_comp, s0.n_params, tuple(p0.shape)) == (3, 6, (4, 6))
    assert (s1.n_comp, s1.n_params, tuple(p1.shape)) == (2, 3, (4, 3))
    # component kinds/dims follow GP_model.generate_kernel_batched order
    assert [s0.kind[r][0] for r in range(3)] == [_kind("rbf"), _kind("cat"), _kind("cat")]
    assert [s0.dim[r][0] for r in range(3)] == [0, 3, 4]
    kf = la.generate_kernel(**cfg, latent_dim=2)
    sf, pf = la.kernel_spec_and_params(kf)
    assert (sf.n_comp, sf.n_params) == (5, 9)
    # init values: lengthscale 2.5, scale ln 2 (GP_model.py:60, 92)
    import math
    assert abs(float(pf[0, 0]) - math.log(2)) < 1e-6 and abs(float(pf[0, 2]) - 2.5) < 1e-6


def _kind(k):
    from lvae_amd import _lib
    return _lib.KIND_CODE[k]
