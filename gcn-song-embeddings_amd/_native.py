"""ctypes binding of libpinsage_hip.so (the C-ABI in include/pinsage_hip.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``).
There is no CPU fallback: compute entry points need the HIP library AND a GPU,
and raise ``RuntimeError`` otherwise.  torch is imported first so the library
binds to the HIP runtime torch already loaded (same soname).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# PINSAGE_LIB: another build of the same C-ABI (A/B runs of compile-time variants)
LIB_PATH = os.environ.get("PINSAGE_LIB") or os.path.join(HERE, "libpinsage_hip.so")

_lib = None

vp = ctypes.c_void_p
i64 = ctypes.c_int64
i32 = ctypes.c_int32
f32 = ctypes.c_float
u64 = ctypes.c_uint64
u32 = ctypes.c_uint32


class EngineConfig(ctypes.Structure):
    _fields_ = [("n_items", i64), ("d_in", i64), ("hid", i64), ("out", i64), ("n_layers", i64),
                ("T", i64), ("max_pos", i64)]


class EngineOffsets(ctypes.Structure):
    _fields_ = [("ids", i64), ("pos_rank", i64), ("z", i64), ("dz", i64), ("scalars", i64),
                ("n_layers", i64), ("count_S", i64 * 8), ("count_N", i64 * 8),
                ("members_S", i64 * 8), ("members_N", i64 * 8), ("cap_S", i64 * 8),
                ("cap_N", i64 * 8), ("y", i64 * 8), ("param_offsets", i64 * 8),
                ("hinge", i64)]


# name -> (restype, argtypes)
_SIGS = {
    "pinsage_version": (ctypes.c_int, []),
    "pinsage_last_error": (ctypes.c_char_p, []),
    "pinsage_device_count": (ctypes.c_int, []),
    "pinsage_mt_state_bytes": (ctypes.c_int, []),
    "pinsage_mt_from_torch": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_mt_to_torch": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_mt_seed": (ctypes.c_int, [vp, u64]),
    "pinsage_mt_skip": (ctypes.c_int, [vp, i64]),
    "pinsage_mt_draws": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_mt_randperm_prefix": (ctypes.c_int, [vp, i64, i64, vp]),
    "pinsage_sample_batch_easy": (ctypes.c_int, [vp, vp, i64, i64, i64, vp, vp, vp]),
    "pinsage_batch_sampler_create": (ctypes.c_int, [vp, i64, i64, i64, vp]),
    "pinsage_batch_sampler_destroy": (None, [vp]),
    "pinsage_batch_sampler_next": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, vp, ctypes.c_int]),
    "pinsage_batch_sampler_peek": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_walk_mt_workspace": (i64, [i64, i64]),
    "pinsage_walk_mt": (ctypes.c_int, [vp, vp, i64, vp, i64, i64, f32, vp, vp, i64, vp, vp]),
    "pinsage_walk_philox": (ctypes.c_int, [vp, vp, i64, vp, i64, i64, f32, u64, u32, i64, vp, vp]),
    "pinsage_visit_topk_scratch": (i64, [i64, i64, i64]),
    "pinsage_visit_topk": (ctypes.c_int, [vp, vp, i64, i64, i64, i64, vp, vp, vp, vp, vp, i64, vp]),
    "pinsage_ppr_topk_workspace": (i64, [i64, i64, ctypes.c_int]),
    "pinsage_engine_set_gemm_choice": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_int]),
    "pinsage_engine_set_layer_table": (ctypes.c_int, [vp, i64, vp, vp, i64]),
    "pinsage_ppr_topk": (ctypes.c_int, [vp, vp, i64, vp, i64, i64, f32, i64, vp, u64, u32, i64, vp, i64,
                                        vp, vp, vp, vp, i64, vp]),
    "pinsage_ppr_topk_segments": (ctypes.c_int, [vp, vp, i64, vp, i64, vp, vp, vp, i64, f32, i64, u32, vp,
                                                 i64, vp, vp, vp, vp, i64, vp]),
    "pinsage_visit_dense": (ctypes.c_int, [vp, vp, i64, i64, i64, vp, vp]),
    "pinsage_fly_workspace_bytes": (i64, [i64, i64, i64, i64, i64]),
    "pinsage_fly_init_workspace": (ctypes.c_int, [vp, i64, i64, i64, i64, i64, vp]),
    "pinsage_fly_sample": (ctypes.c_int, [vp, vp, i64, vp, i64, i64, i64, i64, i64, f32, vp, vp, i64, vp, vp, vp,
                                          i64, vp, vp, vp, i64, vp, i64, i64, vp, i64, vp, vp]),
    "pinsage_engine_set_fly": (ctypes.c_int, [vp, i64, vp, vp, i64, i64]),
    "pinsage_fly_publish_err": (ctypes.c_int, [vp, vp, i64, i64, vp, i64, vp]),
    "pinsage_fly_gate_adam": (ctypes.c_int, [vp, vp, vp]),
    "pinsage_frontier_workspace": (i64, [i64]),
    "pinsage_frontier_step": (ctypes.c_int, [vp, i64, vp, i64, i64, i64, vp, vp, vp, vp]),
    "pinsage_frontier_local_idx": (ctypes.c_int, [vp, i64, vp, i64, i64, i64, vp, vp, vp]),
    "pinsage_linear": (ctypes.c_int, [vp, i64, vp, i64, i64, vp, vp, i64, ctypes.c_int, vp, i64, vp]),
    "pinsage_wgrad_scratch_bytes": (i64, [i64, i64]),
    "pinsage_wgrad_probe": (ctypes.c_int, [i64, i64, vp, i64, vp, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_int,
                                           vp]),
    "pinsage_wgrad_planes": (ctypes.c_int, [i64, i64, vp, i64, vp, i64, i64, vp, i64, i64, vp, vp, i64, vp,
                                            ctypes.c_int, vp, vp]),
    "pinsage_wgrad": (ctypes.c_int, [i64, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp,
                                     ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_float, vp]),
    "pinsage_gemm_ex": (ctypes.c_int, [i64, i64, i64, ctypes.c_int, ctypes.c_int, vp, i64, vp, vp, i64,
                                       vp, vp, i64, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, vp]),
    "pinsage_weighted_agg": (ctypes.c_int, [vp, i64, vp, vp, i64, i64, vp, vp]),
    "pinsage_conv_agg_project": (ctypes.c_int, [vp, i64, i64, vp, vp, i64, i64, vp, vp, i64, i64, vp, vp,
                                                i64, vp, vp, vp, vp, vp]),
    "pinsage_gather_rows": (ctypes.c_int, [vp, i64, i64, i64, vp, i64, vp, i64, vp]),
    "pinsage_concat_linear_l2norm": (ctypes.c_int, [vp, i64, vp, i64, i64, vp, i64, i64, vp, vp, i64, vp, vp,
                                                    vp]),
    "pinsage_norm_lrelu_backward": (ctypes.c_int, [vp, vp, vp, i64, i64, vp, vp]),
    "pinsage_gemm_set_prec": (ctypes.c_int, [ctypes.c_int]),
    "pinsage_gemm_get_prec": (ctypes.c_int, []),
    "pinsage_split_planes": (ctypes.c_int, [vp, i64, i64, i64, vp, vp]),
    "pinsage_linear_split_b": (ctypes.c_int, [vp, i64, vp, i64, i64, vp, vp, i64, vp, i64, ctypes.c_int,
                                              vp, i64, ctypes.c_int, vp]),
    "pinsage_triplet_loss_scratch_bytes": (i64, [i64, i64]),
    "pinsage_triplet_loss": (ctypes.c_int, [vp, i64, i64, ctypes.c_float, vp, vp, vp, vp]),
    "pinsage_split_ilv": (ctypes.c_int, [vp, i64, i64, i64, vp, i64, vp]),
    "pinsage_linear_ilv": (ctypes.c_int, [vp, i64, vp, i64, vp, i64, i64, vp, vp, i64, vp, i64, ctypes.c_int, vp,
                                          i64, vp]),
    "pinsage_step_stage": (ctypes.c_int, [vp, i64, i64, vp, i64, i64, vp, i64, vp, vp]),
    "pinsage_step_publish": (ctypes.c_int, [vp, i64, vp, i64, vp, vp]),
    "pinsage_stream_hold": (ctypes.c_int, [i64, vp]),
    "pinsage_engine_site_stream_k": (ctypes.c_int, [vp, ctypes.c_char_p]),
    "pinsage_stepper_create": (ctypes.c_int, [vp, i64, i64, i64, i64, i64, i64, i64, vp]),
    "pinsage_stepper_destroy": (None, [vp]),
    "pinsage_stepper_wait_ns": (i64, [vp]),
    "pinsage_stepper_stats": (ctypes.c_int, [vp, vp, ctypes.c_int]),
    "pinsage_stepper_set_graphs": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp]),
    "pinsage_stepper_sync_state": (ctypes.c_int, [vp, ctypes.c_int, i64]),
    "pinsage_stepper_step": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, vp]),
    "pinsage_segment_wmean": (ctypes.c_int, [vp, i64, i64, i64, vp, vp, vp, i64, ctypes.c_int, vp, i64,
                                             vp]),
    "pinsage_knn_scratch_bytes": (i64, [i64, i64]),
    "pinsage_knn_cosine": (ctypes.c_int, [vp, i64, i64, i64, vp, i64, i64, f32, vp, i64, vp, vp, vp]),
    "pinsage_engine_create": (ctypes.c_int, [ctypes.POINTER(EngineConfig), ctypes.POINTER(vp)]),
    "pinsage_engine_destroy": (None, [vp]),
    "pinsage_engine_live_count": (i64, []),
    "pinsage_engine_workspace_bytes": (i64, [vp]),
    "pinsage_engine_init_workspace": (i32, [vp, vp, vp]),
    "pinsage_engine_num_params": (i64, [vp]),
    "pinsage_engine_offsets": (ctypes.c_int, [vp, ctypes.POINTER(EngineOffsets)]),
    "pinsage_engine_set_tensors": (ctypes.c_int, [vp, vp, i64, vp, vp, i64, vp, vp, vp, vp]),
    "pinsage_engine_set_feature_planes": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_engine_set_frontier_fork": (ctypes.c_int, [vp, ctypes.c_int]),
    "pinsage_engine_set_feature_ilv": (ctypes.c_int, [vp, vp, i64]),
    "pinsage_engine_forward": (ctypes.c_int, [vp, vp, vp, i64, vp]),
    "pinsage_engine_forward_inference": (ctypes.c_int, [vp, vp, vp, i64, vp]),
    "pinsage_engine_frontier": (ctypes.c_int, [vp, vp, vp, i64, vp]),
    "pinsage_engine_forward_layers": (ctypes.c_int, [vp, vp, vp]),
    "pinsage_engine_set_fork": (ctypes.c_int, [vp, vp, vp, i64, vp]),
    "pinsage_engine_gather_output": (ctypes.c_int, [vp, vp, i64, vp, vp]),
    "pinsage_engine_loss": (ctypes.c_int, [vp, vp, i64, f32, ctypes.c_int, vp]),
    "pinsage_engine_set_output_grad": (ctypes.c_int, [vp, vp, vp, i64, vp]),
    "pinsage_engine_backward": (ctypes.c_int, [vp, vp, vp]),
    "pinsage_engine_reset_backward": (ctypes.c_int, [vp, vp, vp]),
    "pinsage_engine_backward_stage": (ctypes.c_int, [vp, vp, ctypes.c_int, vp]),
    "pinsage_engine_adam": (ctypes.c_int, [vp, vp, ctypes.c_double, ctypes.c_double, f32, vp]),
    "pinsage_engine_backward_adam": (ctypes.c_int, [vp, vp, vp, ctypes.c_double, ctypes.c_double, f32, vp]),
    "pinsage_engine_read_counts": (ctypes.c_int, [vp, vp, vp, vp, vp]),
    "pinsage_engine_set_hints": (ctypes.c_int, [vp, vp, vp]),
    "pinsage_engine_timing": (ctypes.c_int, [vp, ctypes.c_int]),
    "pinsage_engine_timing_collect": (ctypes.c_int, [vp]),
    "pinsage_engine_timing_get": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_char_p, i64,
                                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)]),
}

EXPORTED = tuple(_SIGS)


def lib():
    """Load the native library (raises ImportError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `make -C csrc` "
                              "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().pinsage_last_error().decode(errors="replace")
        if rc == -5:
            raise IndexError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def require_gpu():
    """The product path is HIP-only: fail loudly when no GPU is usable."""
    lib()
    if not torch.cuda.is_available():
        raise RuntimeError("pinsage_amd needs an AMD GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")


def device():
    require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Device/host pointer of a tensor (None -> NULL).  The C-ABI reads plain
    arrays: a strided 1-D view (e.g. a column of a [3, B] batch reshaped) would
    be read as if contiguous, so it is refused."""
    if t is None:
        return None
    if t.dim() == 1 and t.numel() > 1 and t.stride(0) != 1:
        raise ValueError("C-ABI pointer of a strided 1-D tensor (call .contiguous())")
    return ctypes.c_void_p(t.data_ptr())


# ----------------------------------------------------------------------------- MT19937
class MT:
    """Host MT19937 state with torch CPU-generator semantics (native)."""

    def __init__(self):
        self.buf = np.zeros(lib().pinsage_mt_state_bytes(), np.uint8)

    @property
    def p(self):
        return self.buf.ctypes.data_as(ctypes.c_void_p)

    @classmethod
    def from_torch(cls):
        g = cls()
        st = torch.get_rng_state().numpy()
        check(lib().pinsage_mt_from_torch(g.p, st.ctypes.data_as(vp), st.nbytes), "mt_from_torch")
        return g

    @classmethod
    def from_state(cls, st):
        """From a torch.get_rng_state() byte array (numpy uint8)."""
        g = cls()
        check(lib().pinsage_mt_from_torch(g.p, st.ctypes.data_as(vp), st.nbytes), "mt_from_torch")
        return g

    def to_state(self, st):
        """A copy of the torch state bytes st with this generator written in."""
        st = st.copy()
        check(lib().pinsage_mt_to_torch(self.p, st.ctypes.data_as(vp), st.nbytes), "mt_to_torch")
        return st

    def to_torch(self):
        torch.set_rng_state(torch.from_numpy(self.to_state(torch.get_rng_state().numpy())))

    def seed(self, s):
        lib().pinsage_mt_seed(self.p, s)
        return self

    def draws(self, n):
        out = np.empty(n, np.uint32)
        lib().pinsage_mt_draws(self.p, out.ctypes.data_as(vp), n)
        return out

    def skip(self, n):
        lib().pinsage_mt_skip(self.p, n)

    def randperm_prefix(self, n, k):
        k = min(k, n)
        out = np.empty(k, np.int64)
        check(lib().pinsage_mt_randperm_prefix(self.p, n, k, out.ctypes.data_as(vp)), "randperm")
        return out


class torch_rng:
    """Context manager: run native MT draws on torch's global CPU generator."""

    def __enter__(self):
        self.mt = MT.from_torch()
        return self.mt

    def __exit__(self, *exc):
        if exc[0] is None:
            self.mt.to_torch()
        return False
