"""ctypes binding of libdclip.so (the C ABI declared in include/dclip.h).

The library is built in-tree (`python -c "import __graft_entry__; __graft_entry__.build()"`
or `make -C denseclip_vit_multimodal_amd/csrc`).  There is deliberately NO fallback:
if the library is missing or a call fails, a RuntimeError is raised.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCLIP_LIB", os.path.join(_HERE, "libdclip.so"))

F32, F16, BF16 = 0, 1, 2
EPI_STORE, EPI_GELU, EPI_RESIDUAL, EPI_GELU_BWD, EPI_SPLITK, EPI_STORE_SCALED = 0, 1, 2, 3, 4, 5
OPT_ATTN_FWD_WAVES, OPT_ATTN_DQ_WAVES, OPT_ATTN_DKDV_WAVES, OPT_GEMM_TILE, OPT_GEMM_TN_TILE = 0, 1, 2, 3, 4
OPT_ATTN_DKDV_QS, OPT_ATTN_FWD_KERNEL, OPT_ATTN_BWD_KERNEL, OPT_ATTN_BWD_BLOCK, OPT_GEMM_TN_COLSUM = 5, 6, 7, 8, 9
OPT_GEMM_EPI, OPT_GEMM_TAIL, OPT_ATTN_FP8_QK, OPT_ATTN_DQ_ISSUE, OPT_ATTN_DQ_ROWS = 10, 11, 12, 13, 14
OPT_ATTN_DQ_DEFER, OPT_GEMM_SCHED, OPT_GEMM_KLOOP = 15, 16, 17
OPT_ATTN_DQ_REDUCE = 18
OPT_ATTN_PREP_ORDER = 19
OPT_ATTN_DQ_DEFER = 15

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> argtypes (restype int)
_SIGS = {
    "dclip_layernorm_fwd": [_c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                            _i64, _i64, _f32, _c_void_p],
    "dclip_layernorm_bwd": [_c_void_p, _i32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32,
                            _c_void_p, _c_void_p, _i64, _i64, _c_void_p],
    "dclip_layernorm_bwd_res": [_c_void_p, _i32, _c_void_p, _i64, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                _c_void_p],
    "dclip_layernorm_bwd_ws_floats": [_i64, _i64],
    "dclip_layernorm_bwd_add": [_c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                _c_void_p],
    "dclip_layernorm_bwd_scaled_add": [_c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                       _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                       _c_void_p, _c_void_p, _i64, _i64, _f32, _c_void_p, _i32, _c_void_p, _c_void_p],
    "dclip_gemm": [_i32, _i32, _c_void_p, _i64, _c_void_p, _i64, _i64, _i64, _i64, _i32, _f32, _c_void_p, _c_void_p,
                   _c_void_p,
                   _i32, _i64, _c_void_p, _i32, _i64, _c_void_p, _i64, _c_void_p],
    "dclip_gemm_tn": [_i32, _i32, _c_void_p, _i64, _c_void_p, _i64, _i64, _i64, _i64, _i64, _i32, _f32, _c_void_p,
                      _c_void_p,
                      _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p],
    "dclip_attn_fwd": [_i32, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _f32, _c_void_p],
    "dclip_attn_bwd": [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32,
                       _i32, _f32, _c_void_p],
    "dclip_im2col": [_c_void_p, _i32, _c_void_p, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_tokens_fwd": [_c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p],
    "dclip_tokens_bwd": [_c_void_p, _c_void_p, _i32, _f32, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32,
                         _c_void_p],
    "dclip_pos_interp_fwd": [_c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_pos_interp_bwd": [_c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_transpose": [_c_void_p, _i32, _i64, _i64, _i64, _c_void_p, _i32, _i64, _i64, _i32, _i64, _i64, _i64,
                        _i32, _c_void_p, _c_void_p],
    "dclip_weight_refresh": [_c_void_p, _i32, _i64, _i32, _c_void_p],
    "dclip_row_mean_workspace": [_i32, _i64, _i32],
    "dclip_row_mean": [_c_void_p, _i32, _i64, _i64, _i64, _i32, _i64, _i32, _c_void_p, _c_void_p, _c_void_p],
    "dclip_score_map": [_c_void_p, _i32, _i64, _i64, _i64, _c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _f32,
                        _c_void_p],
    "dclip_score_concat": [_c_void_p, _i32, _i64, _i64, _i64, _i32, _c_void_p, _i32, _i32, _i32, _c_void_p, _i32, _i32,
                           _i32, _c_void_p],
    "dclip_bilinear_fwd": [_c_void_p, _i32, _c_void_p, _i32, _i64, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_bilinear_bwd": [_c_void_p, _i32, _c_void_p, _c_void_p, _i64, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_cast": [_c_void_p, _i32, _c_void_p, _i32, _i64, _f32, _c_void_p, _c_void_p],
    "dclip_grad_scale": [_c_void_p, _i64, _f32, _c_void_p, _c_void_p],
    "dclip_cityscapes_augment": [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p, _i32, _i32,
                                 _c_void_p, _c_void_p, _f32, _f32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                 _c_void_p],
    "dclip_color_jitter": [_c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p],
    "dclip_normalize_u8": [_c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p],
    "dclip_bn_eval": [_i32, _c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _f32, _c_void_p, _c_void_p,
                      _c_void_p, _c_void_p, _i32, _c_void_p],
    "dclip_row_scale_add": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i64, _i32, _c_void_p],
    "dclip_add_readout_amax": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _i64, _i32, _i32, _f32, _c_void_p,
                               _c_void_p],
    "dclip_add_readout_cast": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _i32, _i64, _i32, _i32, _f32,
                               _c_void_p],
    "dclip_add_readout_cast_scaled": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i32, _i32,
                                      _f32, _c_void_p, _i32, _c_void_p, _c_void_p],
    "dclip_layernorm_bwd_scaled": [_c_void_p, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                   _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64, _f32,
                                   _c_void_p, _i32, _c_void_p, _c_void_p],
    "dclip_bn_workspace": [_i64, _i32],
    "dclip_bn_fwd": [_i32, _c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _f32, _f32, _c_void_p, _c_void_p,
                     _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p],
    "dclip_bn_bwd": [_i32, _c_void_p, _c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                     _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p],
    "dclip_conv3x3": [_i32, _i32, _c_void_p, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _c_void_p, _i32, _c_void_p,
                      _i32, _i64, _i32, _i32, _i32, _c_void_p],
    "dclip_upsample_ce": [_i32, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p,
                          _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "dclip_upsample_silog": [_i32, _i32, _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _i32, _i32, _f32, _f32,
                             _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "dclip_upsample_ws_floats": [_i32, _i32, _i32, _i32],
    "dclip_conv3x3_wgrad": [_i32, _c_void_p, _i64, _i32, _c_void_p, _i64, _i64, _i64, _i32, _i32, _i32, _i32,
                            _c_void_p, _c_void_p, _i32, _i32, _c_void_p, _c_void_p],
    "dclip_set_option": [_i32, _i32],
    "dclip_cityscapes_prepare": [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p, _i32, _i32,
                                 _c_void_p, _c_void_p, _f32, _f32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                 _c_void_p],
    "dclip_attn_bwd_workspace": [_i32, _i32, _i32],
    "dclip_attn_bwd_fp8_workspace": [_i32, _i32, _i32],
    "dclip_attn_bwd_fp8": [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32,
                           _i32, _f32, _c_void_p],
    "dclip_attn_fwd_fp8": [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p],
    "dclip_attn_fwd_fp8_workspace": [_i32, _i32, _i32],
    "dclip_gemm_tn_plan": [_i64, _i64, _i64, _c_void_p, _c_void_p],
}
EXPORTED = sorted(list(_SIGS) + ["dclip_last_error", "dclip_abi_version"])

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def load(path=None):
    """Load libdclip.so (no GPU needed).  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeError(
                f"libdclip.so not found at {p}: build it with `make -C denseclip_vit_multimodal_amd/csrc` "
                "(the HIP path has no CPU fallback)")
        lib = ctypes.CDLL(p)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        lib.dclip_last_error.restype = ctypes.c_char_p
        lib.dclip_last_error.argtypes = []
        lib.dclip_abi_version.restype = ctypes.c_int
        lib.dclip_abi_version.argtypes = []
        lib.dclip_attn_bwd_workspace.restype = ctypes.c_int64  # a size, not a status
        lib.dclip_attn_bwd_fp8_workspace.restype = ctypes.c_int64
        lib.dclip_bn_workspace.restype = ctypes.c_int64
        lib.dclip_attn_fwd_fp8_workspace.restype = ctypes.c_int64
        lib.dclip_row_mean_workspace.restype = ctypes.c_int64
        lib.dclip_layernorm_bwd_ws_floats.restype = ctypes.c_int64
        lib.dclip_upsample_ws_floats.restype = ctypes.c_int64
        # kernel-variant knobs for A/B runs: DCLIP_OPTIONS="id=value,..." (DCLIP_OPT_* ids of dclip.h)
        for kv in filter(None, os.environ.get("DCLIP_OPTIONS", "").split(",")):
            k, v = kv.split("=")
            if lib.dclip_set_option(int(k), int(v)) != 0:
                raise NativeError(f"DCLIP_OPTIONS: {lib.dclip_last_error().decode()}")
        if path is None:
            _lib = lib
        return lib


def lib():
    return load()


def call(name, *args):
    """Invoke a C-ABI entry point; raise NativeError with dclip_last_error() on failure."""
    L = load()
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.dclip_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed ({rc}): {msg}")
    return rc
