"""ctypes binding of the C-ABI HIP library ``liblvae_hip.so`` (declared in include/lvae_hip.h).

This is the one backend of the package: there is no CPU or PyTorch fallback for the GP-prior
hot path.  If the shared object is missing, or no GPU is visible, every op raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblvae_hip.so")

MAX_COMP = 16
MAX_FAC = 4
ERR_LAUNCH = -1000

CAT, BIN, RBF, PER, LIN = 0, 1, 2, 3, 4
KIND_CODE = {"cat": CAT, "bin": BIN, "rbf": RBF, "per": PER, "lin": LIN}
N_FACTOR_PARAMS = {"cat": 0, "bin": 0, "rbf": 1, "per": 2, "lin": 0}


class KernelSpec(ctypes.Structure):
    _fields_ = [
        ("n_comp", ctypes.c_int32),
        ("n_params", ctypes.c_int32),
        ("n_fac", ctypes.c_int32 * MAX_COMP),
        ("scale_idx", ctypes.c_int32 * MAX_COMP),
        ("kind", (ctypes.c_int32 * MAX_FAC) * MAX_COMP),
        ("dim", (ctypes.c_int32 * MAX_FAC) * MAX_COMP),
        ("param_idx", (ctypes.c_int32 * MAX_FAC) * MAX_COMP),
    ]


class XView(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("stride_b", ctypes.c_int64), ("stride_l", ctypes.c_int64),
                ("ld", ctypes.c_int64)]


class HensmanDims(ctypes.Structure):
    _fields_ = [("L", ctypes.c_int32), ("M", ctypes.c_int32), ("P_b", ctypes.c_int32), ("T", ctypes.c_int32),
                ("Q", ctypes.c_int32), ("P_tot", ctypes.c_double), ("eps", ctypes.c_double),
                ("natural_gradient", ctypes.c_int32), ("ng_prior_share", ctypes.c_double),
                ("seg_len", ctypes.c_void_p), ("n_total", ctypes.c_double)]


def make_spec(components):
    """components: list of lists of (kind, dim) factors, in parameter order (see oracle header).
    Returns (KernelSpec, n_params)."""
    if len(components) > MAX_COMP:
        raise ValueError(f"at most {MAX_COMP} additive components")
    s = KernelSpec()
    s.n_comp = len(components)
    p = 0
    for r, comp in enumerate(components):
        if not 1 <= len(comp) <= MAX_FAC:
            raise ValueError(f"component {r}: 1..{MAX_FAC} factors")
        s.n_fac[r] = len(comp)
        s.scale_idx[r] = p
        p += 1
        for f, (kind, dim) in enumerate(comp):
            s.kind[r][f] = KIND_CODE[kind]
            s.dim[r][f] = int(dim)
            if N_FACTOR_PARAMS[kind]:
                s.param_idx[r][f] = p
                p += N_FACTOR_PARAMS[kind]
            else:
                s.param_idx[r][f] = -1
    s.n_params = p
    return s


_VP, _I32, _I64, _D, _SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_size_t
_SPEC = ctypes.POINTER(KernelSpec)
_DIMS = ctypes.POINTER(HensmanDims)

# name -> (restype, argtypes); every symbol include/lvae_hip.h declares
SIGNATURES = {
    "lvae_gram_f64": (_I32, [_SPEC, XView, XView, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _I64, _I64, _I64, _VP]),
    "lvae_gram_f32": (_I32, [_SPEC, XView, XView, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _I64, _I64, _I64, _VP]),
    "lvae_gram_bwd_workspace_size": (_SZ, [_I32, _I32, _I32, _I32]),
    "lvae_gram_bwd_f64": (_I32, [_SPEC, XView, XView, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _I64, _I64, _VP,
                                 _VP, _VP, _VP]),
    "lvae_kl_closed_padded_n": (_I32, [_I32]),
    "lvae_kl_closed_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_kl_closed_factor_f32": (_I32, [_SPEC, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP]),
    "lvae_kl_closed_reduce_f32": (_I32, [_SPEC, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _I32, _VP, _VP, _I32,
                                         _VP]),
    "lvae_kl_closed_fwd_f32": (_I32, [_SPEC, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _I32, _VP, _VP, _VP,
                                      _I32, _VP]),
    "lvae_kl_closed_bwd_f32": (_I32, [_SPEC, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _I32, _VP, _VP, _VP, _VP,
                                      _VP, _VP, _VP]),
    "lvae_kl_closed_bwd_latent_f32": (_I32, [_I32, _I32, _VP, _I32, _VP, _VP, _VP, _VP, _VP]),
    "lvae_kl_closed_bwd_hyper_f32": (_I32, [_SPEC, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "lvae_kl_closed_refine_state": (_I32, [_I32, _I32, _VP, _VP, _VP, _VP]),
    "lvae_kl_closed_hyper_state": (_I32, [_I32, _I32, _VP, _VP, _VP]),
    "lvae_vae_loss_fwd_f32": (_I32, [_VP, _VP, _VP, _VP, _I32, _I32, _VP, _VP, _VP, _VP]),
    "lvae_vae_loss_bwd_partials": (_SZ, [_I32]),
    "lvae_bias_relu_fwd_f32": (_I32, [_VP, _VP, _I32, _I32, _I32, _VP]),
    "lvae_act_bwd_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_act_bwd_f32": (_I32, [_VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP]),
    "lvae_vae_loss_bwd_f32": (_I32, [_VP, _VP, _VP, _VP, _VP, _VP, _I64, _VP, _I64, _I32, _I32, _VP, _VP, _VP]),
    "lvae_reparam_fwd_f32": (_I32, [_VP, _VP, _VP, _I64, _VP, _VP]),
    "lvae_reparam_bwd_f32": (_I32, [_VP, _VP, _VP, _I64, _VP, _VP]),
    "lvae_step_terms_fwd": (_I32, [_VP, _VP, _I32, _VP, ctypes.c_float, _D, _D, _I32, _VP, _VP, _VP, _VP, _VP]),
    "lvae_step_terms_bwd": (_I32, [_VP, _VP, _VP, _VP, ctypes.c_float, _D, _D, _I32, _VP, _VP, _VP, _VP]),
    "lvae_param_pack_fwd_f64": (_I32, [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP]),
    "lvae_param_pack_bwd_f64": (_I32, [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _I64, _I64, _VP, _VP]),
    "lvae_spd_inv_small_f64": (_I32, [_I32, _I32, _VP, _I64, _VP, _I64, _VP, _VP, _VP]),
    "lvae_gemm_small_f64": (_I32, [_I32, _I32, _I32, _I32, _I32, _D, _VP, _I32, _I64, _I64, _VP, _I32, _I64,
                                   _I64, _D, _VP, _I32, _I64, _I64, _I32, _I32, _VP]),
    "lvae_hensman_workspace_size": (_SZ, [_DIMS]),
    "lvae_hensman_fwd_f64": (_I32, [_SPEC, _SPEC, _DIMS, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                    _VP, _VP, _VP, _VP]),
    "lvae_hensman_fwd_part_f64": (_I32, [_I32, _SPEC, _SPEC, _DIMS, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                         _VP, _VP, _VP, _VP, _VP]),
    "lvae_hensman_bwd_f64": (_I32, [_SPEC, _SPEC, _DIMS, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                    _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "lvae_natgrad_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_natgrad_update_f64": (_I32, [_I32, _I32, _VP, _VP, _VP, _VP, _D, _VP, _VP, _VP, _VP]),
    "lvae_hensman_iH_offset": (_SZ, [_DIMS]),
    "lvae_relu_maxpool2_fwd_f32": (_I32, [_VP, _I64, _I32, _I32, _VP, _VP, _VP]),
    "lvae_relu_maxpool2_bwd_f32": (_I32, [_VP, _VP, _VP, _I64, _I32, _I32, _VP, _VP]),
    "lvae_relu_maxpool2_bias_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_conv1_relu_maxpool2_fwd_f32": (_I32, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP]),
    "lvae_relu_maxpool2_bias_fwd_f32": (_I32, [_VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP]),
    "lvae_relu_maxpool2_bias_bwd_f32": (_I32, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP]),
    "lvae_conv3x3_pool_wgrad_workspace_size": (_SZ, [_I32, _I32, _I32]),
    "lvae_deconv2_sigmoid_workspace_size": (_SZ, [_I32, _I32, _I32, _I32]),
    "lvae_deconv2_sigmoid_fwd_f32": (_I32, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP]),
    "lvae_deconv2_sigmoid_bwd_f32": (_I32, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP]),
    "lvae_conv3x3_pool_wgrad_f32": (_I32, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP]),
    "lvae_conv3x3_relu_maxpool2_fwd_f32": (_I32, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP]),
    "lvae_deconv4s2_relu_fwd_f32": (_I32, [_VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP]),
    "lvae_deconv4s2_relu_bwd_workspace_size": (_SZ, [_I32, _I32, _I32]),
    "lvae_deconv4s2_relu_bwd_f32": (_I32, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP,
                                            _VP]),
    "lvae_conv3x3_pool_dgrad_lds": (_SZ, [_I32, _I32, _I32]),
    "lvae_conv3x3_pool_dgrad_f32": (_I32, [_VP, _VP, _VP, _VP, _I32, _I32, _I32, _I32, _I32, _VP, _VP]),
    "lvae_spd_inv_chol_scratch_size": (_SZ, [_I32, _I32]),
    "lvae_spd_inv_chol_f32": (_I32, [_I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "lvae_potrf_f64": (_I32, [_I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP, _VP]),
    "lvae_potrf_f32_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_potrf_f32": (_I32, [_I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP, _VP, _VP]),
    "lvae_trsm_workspace_size": (_SZ, [_I32, _I32]),
    "lvae_trsm_f64": (_I32, [_I32, _I32, _I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP]),
    "lvae_trsm_f32": (_I32, [_I32, _I32, _I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP]),
    "lvae_potrs_f64": (_I32, [_I32, _I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP]),
    "lvae_potrs_f32": (_I32, [_I32, _I32, _I32, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP]),
    "lvae_predict_workspace_size": (_SZ, [_I32, _I32, _I32, _I32, _I32]),
    "lvae_predict_f64": (_I32, [_SPEC, _SPEC, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _I32, _VP, _VP,
                                _VP, _VP, _D, _VP, _VP, _VP, _VP]),
    "lvae_prof_enable": (_I32, [_I32]),
    "lvae_prof_collect": (_I32, [_VP, _VP, _I32]),
    "lvae_version": (ctypes.c_char_p, []),
}

_lib = None


def load(path=LIB_PATH):
    """Load the shared object and bind every declared symbol (no GPU needed to load)."""
    global _lib
    if _lib is not None:
        return _lib
    if path == LIB_PATH:  # (a diagnostic build in place of the in-tree one: scripts/gpu_hbstamp.sh)
        path = os.environ.get("LVAE_LIB", path)
    if not os.path.exists(path):
        raise RuntimeError(f"lvae_amd: HIP library {path} not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    missing = [name for name in SIGNATURES if not hasattr(lib, name)]
    if missing:
        raise RuntimeError(f"lvae_amd: {path} lacks declared symbols {missing} (stale build?)")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    """The library, for compute calls: requires a visible GPU."""
    if not torch.cuda.is_available():
        raise RuntimeError("lvae_amd: no GPU visible; the GP-prior hot path runs only through HIP")
    return load()


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("lvae_amd: tensor must live on the GPU")
    return ctypes.c_void_p(t.data_ptr())


def check(rc, what):
    if rc != 0:
        if rc == ERR_LAUNCH:
            raise RuntimeError(f"lvae_amd: {what}: HIP launch failed")
        raise ValueError(f"lvae_amd: {what}: bad argument #{-rc}")


def xview(t, stride_b, stride_l):
    """XView over a [.., n, Q] fp64 tensor whose last dim is contiguous."""
    assert t.dtype == torch.float64 and t.stride(-1) == 1
    return XView(ctypes.c_void_p(t.data_ptr()), int(stride_b), int(stride_l), int(t.stride(-2)))


PHASES = ["gram", "potrf", "potri", "kl_reduce", "syrk", "gram_bwd", "bwd_elem", "hensman_fwd", "hensman_bwd",
          "natgrad", "sweep_update", "hb_slab"]


def prof_enable(on=True):
    lib().lvae_prof_enable(1 if on else 0)


def prof_collect():
    """{phase: (total_ms, count)} since the last collect (synchronises on the recorded events)."""
    n = len(PHASES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int32 * n)()
    check(lib().lvae_prof_collect(ms, cnt, n), "prof_collect")
    return {PHASES[i]: (ms[i], cnt[i]) for i in range(n)}
