"""ctypes binding of ``libdfd_hip.so`` (the C ABI declared in ``include/dfd_hip.h``).

The library is built in-tree (``csrc/Makefile`` / ``__graft_entry__.build()``) and loaded
AFTER torch, so it shares torch's HIP runtime (same ``libamdhip64.so.7`` soname) and
therefore its streams and device allocations.  There is no fallback: if the library or a
HIP device is missing, the product path raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded first: provides the HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DFD_HIP_LIB: an alternate in-tree build of the same library (A/B measurements, tools/ab_lib.sh)
LIB_PATH = os.environ.get("DFD_HIP_LIB") or os.path.join(_HERE, "libdfd_hip.so")

_lock = threading.Lock()
_lib = None

c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_f = ctypes.c_float
c_d = ctypes.c_double
c_p = ctypes.c_void_p
c_fpp = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    "dfd_last_error": (ctypes.c_char_p, []),
    "dfd_version": (c_i, []),
    "dfd_b0_tensor_count": (c_i, []),
    "dfd_b0_tensor_info": (c_i, [c_i, ctypes.c_char_p, c_i, ctypes.POINTER(c_i), ctypes.POINTER(c_i),
                                 ctypes.POINTER(c_i64)]),
    "dfd_b0_plan_create": (c_i, [c_i, c_i, c_i, c_i, ctypes.POINTER(c_p)]),
    "dfd_b0_plan_destroy": (None, [c_p]),
    "dfd_b0_workspace_bytes": (c_i64, [c_p]),
    "dfd_b0_bind": (c_i, [c_p, ctypes.POINTER(c_i64), c_i]),
    "dfd_b0_forward": (c_i, [c_p, c_p, c_p, ctypes.POINTER(c_i64), c_p, c_p, c_p, c_p, c_i, c_f]),
    "dfd_b0_backward": (c_i, [c_p, c_p, c_p, ctypes.POINTER(c_i64), c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i]),
    "dfd_b0_forward_ex": (c_i, [c_p, c_p, c_p, c_i, ctypes.POINTER(c_i64), ctypes.POINTER(c_f), c_p, c_p, c_p, c_p,
                                c_i, c_f]),
    "dfd_b0_backward_ex": (c_i, [c_p, c_p, c_p, c_i, ctypes.POINTER(c_i64), ctypes.POINTER(c_f), c_p, c_p, c_p, c_p,
                                 c_i, c_i, c_i, c_i]),
    "dfd_b0_plan_set_tuning": (c_i, [c_p, ctypes.c_char_p, c_i64]),
    "dfd_b0_segment_count": (c_i, []),
    "dfd_b0_saved_tensor": (c_i, [c_p, c_i, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    "dfd_b0_grad_tensor": (c_i, [c_p, c_i, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    "dfd_b0_fused_info": (c_i, [c_p, ctypes.POINTER(c_i), ctypes.POINTER(c_i64)]),
    "dfd_b0_plan_status": (c_i, [c_p, ctypes.POINTER(c_i)]),
    "dfd_b0_plan_clear_status": (c_i, [c_p]),
    "dfd_test_occupy": (c_i, [c_p, c_i, c_i64]),
    "dfd_test_group_sync": (c_i, [c_p, c_i, c_i, c_d, c_p, c_p]),
    "dfd_b0_probe_arm": (c_i, [c_p, c_i, c_i, c_i, c_i]),
    "dfd_b0_probe_read": (c_i, [c_p, ctypes.POINTER(c_f), c_i, ctypes.POINTER(c_i)]),
    "dfd_b0_probe_disarm": (c_i, [c_p]),
    "dfd_b0_segment_tensors": (c_i, [c_i, ctypes.POINTER(c_i), ctypes.POINTER(c_i)]),
    "dfd_head_work_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i]),
    "dfd_head_forward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_fpp, c_p, c_p, c_u64, c_f, c_p, c_p]),
    "dfd_head_backward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_fpp, c_p, c_p, c_u64, c_f, c_p, c_p, c_p,
                                c_p, c_fpp]),
    "dfd_ce_forward": (c_i, [c_p, c_p, c_p, c_p, c_i, c_i, c_i64, c_p, c_p]),
    "dfd_ce_backward": (c_i, [c_p, c_p, c_p, c_p, c_i, c_i, c_i64, c_p, c_p, c_p]),
    "dfd_grad_norm": (c_i, [c_p, c_p, c_i64, c_f, c_p, c_p]),
    "dfd_collate_frames": (c_i, [c_p, c_p, c_p, c_i64, c_i64, c_i, c_p]),
    "dfd_adam_step": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i64, c_d, c_d, c_d, c_d, c_d, c_i, c_d, c_i, c_p]),
    "dfd_grad_norm_scaled": (c_i, [c_p, c_p, c_i64, c_f, c_p, c_p, c_p]),
    "dfd_adam_step_scaled": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i64, c_d, c_d, c_d, c_d, c_d, c_d, c_i, c_p, c_p]),
    "dfd_loss_scale_update": (c_i, [c_p, c_p, c_d, c_d, c_i]),
    "dfd_set_tuning": (c_i64, [ctypes.c_char_p, c_i64]),
    "dfd_rn_im2col": (c_i, [c_p, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p]),
    "dfd_rn_stem_im2col": (c_i, [c_p, c_i, c_p, c_i, ctypes.POINTER(c_i64), ctypes.POINTER(c_f), c_i, c_i, c_i, c_p]),
    "dfd_rn_gemm": (c_i, [c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_i, c_i64, c_i, c_i]),
    "dfd_rn_stem_conv": (c_i, [c_p, c_i, c_p, c_i, ctypes.POINTER(c_i64), c_p, c_i, c_i, c_i, c_p, c_p, c_p]),
    "dfd_rn_conv": (c_i, [c_p, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_i, c_i, c_p]),
    "dfd_rn_maxpool": (c_i, [c_p, c_i, c_p, c_i, c_i, c_i, c_i, c_p]),
    "dfd_rn_avgpool": (c_i, [c_p, c_i, c_p, c_i, c_i, c_i, c_p]),
    "dfd_rn_conv_stat_rows": (c_i64, [c_i, c_i, c_i]),
    "dfd_rn_train_conv_fwd": (c_i, [c_p, c_p, ctypes.POINTER(c_i64), c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i,
                                    c_p, c_p, c_p]),
    "dfd_rn_bn_train_finalize": (c_i, [c_p, c_p, c_i, c_i64, c_i, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p]),
    "dfd_rn_bn_act": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i64, c_i, c_p]),
    "dfd_rn_pool_train_fwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_p]),
    "dfd_rn_pool_train_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p]),
    "dfd_rn_relu_bwd": (c_i, [c_p, c_p, c_p, c_i64, c_p]),
    "dfd_rn_gap_bwd": (c_i, [c_p, c_p, c_p, c_i, c_i, c_i, c_p]),
    "dfd_rn_bn_train_bwd": (c_i, [c_p, c_p, c_p, c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "dfd_rn_bn_train_bwd_relu": (c_i, [c_p, c_p, c_p, c_p, c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "dfd_rn_conv_dgrad": (c_i, [c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p]),
    "dfd_rn_conv_dgrad_res": (c_i, [c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "dfd_rn_conv_wgrad_slab_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_rn_conv_wgrad": (c_i, [c_p, c_p, ctypes.POINTER(c_i64), c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_p,
                                c_i64, c_p]),
    "dfd_rn16_pack_weights": (c_i, [c_p, c_p, c_i, c_i, c_i, c_p, c_p]),
    "dfd_rn16_pack_all": (c_i, [c_p, c_p, c_i, c_i64, c_p]),
    "dfd_rn16_conv_fwd": (c_i, [c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_p, c_p, ctypes.POINTER(c_i)]),
    "dfd_rn16_bn_finalize": (c_i, [c_p, c_p, c_i, c_i64, c_i, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p]),
    "dfd_rn16_bn_act": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i64, c_i, c_p]),
    "dfd_rn16_relu_bwd": (c_i, [c_p, c_p, c_p, c_i64, c_p]),
    "dfd_rn16_gap_bwd": (c_i, [c_p, c_p, c_p, c_i, c_i, c_i, c_p]),
    "dfd_rn16_bn_train_bwd": (c_i, [c_p, c_p, c_p, c_p, c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "dfd_rn16_conv_dgrad": (c_i, [c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_p, c_p]),
    "dfd_rn16_conv_wgrad_slab_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_rn16_conv_wgrad": (c_i, [c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_p, c_i64, c_p]),
    "dfd_rn16_cast": (c_i, [c_p, c_p, c_i, c_i64, c_p]),
    "dfd_pw_conv": (c_i, [c_p, c_i, c_p, c_p, c_p, c_p, c_i64, c_i, c_i, c_i, c_p, c_p, c_p, c_i, c_p,
                          ctypes.POINTER(c_i)]),
    "dfd_attention": (c_i, [c_p, c_i, c_i, c_i, c_i, c_f, c_p, c_i64, c_i, c_i, c_p, c_i64, c_p, c_p, c_i64, c_p,
                            c_i64]),
    "dfd_vgemm": (c_i, [c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i, c_i, c_i, c_p, c_i64]),
    "dfd_vgemm_tn_slab_floats": (c_i64, [c_i64, c_i, c_i]),
    "dfd_blaslt_calls": (c_i64, []),
    "dfd_sgemm": (c_i, [c_p, c_i, c_i, c_p, c_i, c_p, c_i, c_p, c_i, c_i, c_i, c_i, c_f, c_p]),
    "dfd_pw_conv_wgrad": (c_i, [c_p, c_i, c_p, c_p, c_i64, c_i, c_i, c_i, c_p, c_p, c_p, c_i, c_p, c_i64, c_p,
                                c_i]),
    "dfd_rnn_work_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i]),
    "dfd_rnn_scratch_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i]),
    "dfd_rnn_forward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_fpp, c_p, c_p, c_u64, c_f]),
    "dfd_rnn_backward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_fpp, c_p, c_p, c_p, c_fpp, c_u64, c_f]),
    "dfd_vit_param_count": (c_i, [c_i]),
    "dfd_vit_work_bytes": (c_i64, [c_i, c_i, c_i, c_i, c_i]),
    "dfd_vit_scratch_bytes": (c_i64, [c_i, c_i, c_i, c_i, c_i]),
    "dfd_vit_forward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, ctypes.POINTER(c_i64), c_fpp, c_p, c_p]),
    "dfd_vit_forward_ex": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, ctypes.POINTER(c_i64), c_fpp, c_p, c_p,
                                 c_i]),
    "dfd_vit_backward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_fpp, c_p, c_p, c_p, c_fpp]),
    "dfd_gcn_head_work_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_gcn_head_scratch_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_gcn_head_forward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_fpp, c_p, c_i, c_u64, c_f, c_p]),
    "dfd_gcn_head_backward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_fpp, c_p, c_p, c_i, c_u64, c_f, c_p,
                                    c_fpp, c_p]),
    "dfd_cnnlstm_work_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_cnnlstm_scratch_floats": (c_i64, [c_i, c_i, c_i, c_i, c_i, c_i, c_i]),
    "dfd_cnnlstm_forward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, ctypes.POINTER(c_i64), c_fpp, c_fpp,
                                  c_p, c_i, c_f, c_u64, c_f, c_p]),
    "dfd_cnnlstm_backward": (c_i, [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, ctypes.POINTER(c_i64), c_fpp, c_p,
                                   c_p, c_i, c_u64, c_f, c_p, c_fpp]),
}

EXPORTED = tuple(_SIGS.keys())


class DFDError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes library with typed signatures."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise DFDError(f"{p} not found: build it with `make -C deepfake-video-detection_amd/csrc` "
                           f"or __graft_entry__.build()")
        lib = ctypes.CDLL(p)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != 0:
        raise DFDError(load().dfd_last_error().decode(errors="replace"))


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_hip(t: torch.Tensor, what: str = "input") -> None:
    if not t.is_cuda:
        raise DFDError(f"{what} must be on a HIP device (got {t.device}); the MI355X path has no CPU fallback")
