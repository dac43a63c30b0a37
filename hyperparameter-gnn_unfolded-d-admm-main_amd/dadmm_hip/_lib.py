"""ctypes binding of ``libdadmm.so`` (the C ABI declared in ``include/dadmm.h``).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``). There is no
fallback: if the library is missing or cannot be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DADMM_LIB_VARIANT: an alternative build of the same library (timing experiments,
# scripts/time_variants.sh); it is still the HIP library, there is no other path
LIB_PATH = os.environ.get("DADMM_LIB_VARIANT") or os.path.join(_HERE, "libdadmm.so")

ABI_VERSION = 18
DADMM_OK, DADMM_EINVAL, DADMM_EUNSUPPORTED, DADMM_EHIP = 0, -1, -2, -3
VARIANT_UNFOLDED, VARIANT_GNN = 0, 1
STATUS_Y_NONFINITE, STATUS_U_NONFINITE, STATUS_GRAD_NAN, STATUS_YNEXT_NAN = 1, 2, 4, 8
STATUS_BARRIER_TIMEOUT = 0x100
STATUS_RECOMPUTE = 16      # ungated fused kernel: asymmetric shared adjacency; split: a wait timed out
GATE_ON, FLAGS_ZEROED = 1, 2

# every symbol include/dadmm.h declares
EXPORTED_SYMBOLS = (
    "dadmm_abi_version",
    "dadmm_last_error",
    "dadmm_operator_bytes",
    "dadmm_prepare_operator",
    "dadmm_forward",
    "dadmm_forward_record",
    "dadmm_split_scratch_bytes",
    "dadmm_split_flag_bytes",
    "dadmm_forward_split",
    "dadmm_stepwise_scratch_bytes",
    "dadmm_forward_stepwise",
    "dadmm_backward_scratch_bytes",
    "dadmm_backward",
    "dadmm_adjoint_scratch_bytes",
    "dadmm_adjoint",
    "dadmm_hyper_gcn",
    "dadmm_hyper_gcn_ex",
    "dadmm_hyper_linear",
    "dadmm_hyper_linear_ex",
    "dadmm_hyper_rownorm",
    "dadmm_hyper_head",
    "dadmm_hyper_linear_ln_scratch_bytes",
    "dadmm_hyper_linear_ln",
    "dadmm_hyper_gcn_train",
    "dadmm_hyper_gcn_train_bwd",
    "dadmm_hyper_linear_ln_train",
    "dadmm_hyper_rownorm_bwd_part_bytes",
    "dadmm_hyper_rownorm_bwd",
    "dadmm_hyper_head_act",
    "dadmm_hyper_wgrad_scratch_bytes",
    "dadmm_hyper_wgrad",
    "dadmm_hyper_colsum",
    "dadmm_hyper_transpose",
    "dadmm_hyper_train_work_bytes",
    "dadmm_hyper_train_forward",
    "dadmm_hyper_train_forward_ex",
    "dadmm_hyper_train_atb_mix",
    "dadmm_hyper_train_backward",
    "dadmm_hyper_train_dsave_floats",
    "dadmm_hyper_train_backward_deferred",
    "dadmm_hyper_train_wgrad",
    "dadmm_hyper_train_wgrad_scratch_bytes",
    "dadmm_hyper_linear_gcn_bwd",
    "dadmm_hyper_head_train",
    "dadmm_hyper_bn_running_scratch_bytes",
    "dadmm_hyper_bn_running_update",
    "dadmm_gnn_flag_bytes",
    "dadmm_gnn_begin",
    "dadmm_gnn_gram",
    "dadmm_gnn_gram_acc",
    "dadmm_gnn_step",
    "dadmm_gnn_finish",
    "dadmm_gnn_step_backward",
    "dadmm_gnn_step_backward_ex",
    "dadmm_normal_offset_step",
    "dadmm_prologue",
    "dadmm_tiled_scratch_bytes",
    "dadmm_forward_tiled",
    "dadmm_forward_tiled_record",
    "dadmm_graph_generate",
    "dadmm_loss_scratch_bytes",
    "dadmm_loss",
    "dadmm_loss_grad",
)


class DadmmError(RuntimeError):
    """A C-ABI call returned a non-zero code."""

    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed ({code}): {msg}")
        self.code = code


class Dims(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("P", ctypes.c_int32), ("m", ctypes.c_int32),
        ("n", ctypes.c_int32), ("K", ctypes.c_int32), ("variant", ctypes.c_int32),
        ("hyp_rows", ctypes.c_int32), ("graph_shared", ctypes.c_int32),
    ]


_lib = None



_fp = ctypes.POINTER(ctypes.c_float)
_f5 = ctypes.c_float * 5
_f3 = ctypes.c_float * 3


class HyperNet(ctypes.Structure):
    """dadmm_hyper_net (include/dadmm.h): the training hypernetwork's dimensions and parameters."""
    _fields_ = [("P", ctypes.c_int32), ("n", ctypes.c_int32), ("ld", ctypes.c_int32),
                ("width", ctypes.c_int32 * 5), ("dec_width", ctypes.c_int32 * 3), ("H", ctypes.c_int32),
                ("conv_w", ctypes.c_void_p * 5), ("conv_b", ctypes.c_void_p * 5),
                ("bn_w", ctypes.c_void_p * 5), ("bn_b", ctypes.c_void_p * 5), ("bn_eps", _f5),
                ("norm_w", ctypes.c_void_p), ("norm_b", ctypes.c_void_p), ("norm_eps", ctypes.c_float),
                ("dec_w", ctypes.c_void_p * 3), ("dec_b", ctypes.c_void_p * 3),
                ("ln_w", ctypes.c_void_p * 3), ("ln_b", ctypes.c_void_p * 3),
                ("ln_eps", _f3), ("dec_slope", _f3), ("dec_drop", _f3),
                ("fc_w", ctypes.c_void_p), ("fc_b", ctypes.c_void_p),
                ("drop_enc", ctypes.c_float), ("maxv", ctypes.c_float * 4),
                # ABI 17: eval-mode BatchNorm (running statistics) in the training kernels
                ("bn_rm", ctypes.c_void_p * 5), ("bn_rv", ctypes.c_void_p * 5), ("bn_eval", ctypes.c_int32)]


class HyperSaved(ctypes.Structure):
    """dadmm_hyper_saved: one iteration's saved activations."""
    _fields_ = [("y", ctypes.c_void_p * 5), ("m", ctypes.c_void_p * 5), ("mean", ctypes.c_void_p * 5),
                ("var", ctypes.c_void_p * 5), ("e", ctypes.c_void_p), ("dec_y", ctypes.c_void_p * 3),
                ("dec_xd", ctypes.c_void_p * 3), ("z", ctypes.c_void_p), ("hyp", ctypes.c_void_p)]


class HeadBwd(ctypes.Structure):
    """dadmm_head_bwd: the head-backward epilogue of dadmm_gnn_step_backward_ex."""
    _fields_ = [("z", ctypes.c_void_p), ("ghyp_add", ctypes.c_void_p), ("maxv", ctypes.c_float * 4),
                ("dz", ctypes.c_void_p)]


class HyperGrads(ctypes.Structure):
    """dadmm_hyper_grads: gradient accumulators and transposed weights of one backward pass."""
    _fields_ = [("conv_w", ctypes.c_void_p * 5), ("bn_wbc", ctypes.c_void_p * 5), ("norm_wb", ctypes.c_void_p),
                ("dec_w", ctypes.c_void_p * 3), ("dec_b", ctypes.c_void_p * 3), ("ln_wb", ctypes.c_void_p * 3),
                ("fc_w", ctypes.c_void_p), ("fc_b", ctypes.c_void_p),
                ("conv_wt", ctypes.c_void_p * 5), ("dec_wt", ctypes.c_void_p * 3), ("fc_wt", ctypes.c_void_p)]

def load() -> ctypes.CDLL:
    """Load libdadmm.so once; raises if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP library first (python -c "
            "'import __graft_entry__ as g; g.build()' or make -C csrc)")
    # torch (if imported) has already loaded its libamdhip64.so.7; the dynamic linker resolves
    # this library's DT_NEEDED entry to that same runtime by soname.
    L = ctypes.CDLL(LIB_PATH)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    L.dadmm_abi_version.restype = ctypes.c_int
    L.dadmm_abi_version.argtypes = []
    L.dadmm_last_error.restype = ctypes.c_char_p
    L.dadmm_last_error.argtypes = []
    L.dadmm_operator_bytes.restype = ctypes.c_size_t
    L.dadmm_operator_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_prepare_operator.restype = ctypes.c_int
    L.dadmm_prepare_operator.argtypes = [ctypes.POINTER(Dims), vp, vp, vp]
    L.dadmm_forward.restype = ctypes.c_int
    L.dadmm_forward.argtypes = [ctypes.POINTER(Dims)] + [vp] * 13
    L.dadmm_split_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_split_scratch_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_split_flag_bytes.restype = ctypes.c_size_t
    L.dadmm_split_flag_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_forward_split.restype = ctypes.c_int
    L.dadmm_forward_split.argtypes = [ctypes.POINTER(Dims)] + [vp] * 15
    L.dadmm_stepwise_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_stepwise_scratch_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_forward_stepwise.restype = ctypes.c_int
    L.dadmm_forward_record.restype = ctypes.c_int
    L.dadmm_forward_record.argtypes = [ctypes.POINTER(Dims)] + [vp] * 15
    L.dadmm_forward_stepwise.argtypes = [ctypes.POINTER(Dims)] + [vp] * 14 + [i32, vp, vp]
    L.dadmm_backward_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_backward_scratch_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_backward.restype = ctypes.c_int
    L.dadmm_backward.argtypes = [ctypes.POINTER(Dims)] + [vp] * 14
    L.dadmm_adjoint_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_adjoint_scratch_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.dadmm_adjoint.restype = ctypes.c_int
    L.dadmm_adjoint.argtypes = [ctypes.POINTER(Dims)] + [vp] * 14
    D = ctypes.POINTER(Dims)
    u64, i64, f32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_float
    L.dadmm_normal_offset_step.restype = u64
    L.dadmm_normal_offset_step.argtypes = [i64]
    L.dadmm_prologue.restype = ctypes.c_int
    L.dadmm_prologue.argtypes = [u64, u64, i64, i32, i32, f32, f32, vp, vp, vp, vp, i64, vp]
    L.dadmm_tiled_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_tiled_scratch_bytes.argtypes = [D]
    L.dadmm_forward_tiled.restype = ctypes.c_int
    L.dadmm_forward_tiled.argtypes = [D] + [vp] * 14
    L.dadmm_forward_tiled_record.restype = ctypes.c_int
    L.dadmm_forward_tiled_record.argtypes = [D] + [vp] * 16
    L.dadmm_graph_generate.restype = ctypes.c_int
    L.dadmm_graph_generate.argtypes = [i32, i32, f32, u64, i32] + [vp] * 7
    L.dadmm_loss_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_loss_scratch_bytes.argtypes = [i32, i64, i32]
    L.dadmm_loss.restype = ctypes.c_int
    L.dadmm_loss.argtypes = [i32] * 5 + [vp] * 7
    L.dadmm_loss_grad.restype = ctypes.c_int
    L.dadmm_loss_grad.argtypes = [i32] * 5 + [vp] * 6
    L.dadmm_gnn_flag_bytes.restype = ctypes.c_size_t
    L.dadmm_gnn_flag_bytes.argtypes = [i32]
    for name, args in (("dadmm_gnn_begin", [D] + [vp] * 7),
                       ("dadmm_gnn_gram", [D, vp, i32] + [vp] * 5),
                       ("dadmm_gnn_gram_acc", [D] + [vp] * 5),
                       ("dadmm_gnn_step", [D, i32] + [vp] * 14),
                       ("dadmm_gnn_finish", [D] + [vp] * 4),
                       ("dadmm_gnn_step_backward", [D, i32] + [vp] * 18),
                       ("dadmm_gnn_step_backward_ex", [D, i32] + [vp] * 17 + [ctypes.POINTER(HeadBwd), vp])):
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    for name, args in (("dadmm_hyper_gcn", [i32] * 4 + [vp, i32, i32, vp, i32] + [vp] * 3 + [i32]
                        + [vp] * 4 + [f32, f32, vp, i32, vp]),
                       ("dadmm_hyper_gcn_ex", [i32] * 4 + [vp, i32, vp, i32, vp, i32, vp, vp, i32]
                        + [vp] * 4 + [f32, f32, i32, vp, i32, vp]),
                       ("dadmm_hyper_linear", [i32] * 3 + [vp, i32, i32, vp, i32, vp, vp, vp, i32, vp]),
                       ("dadmm_hyper_linear_ex", [i32] * 3 + [vp, i32, i32, vp, i32, vp, vp, vp, i32, vp, i32,
                                                             vp]),
                       ("dadmm_hyper_rownorm", [i32, i32, vp, vp, vp, f32, i32, f32, vp, vp]),
                       ("dadmm_hyper_head", [i32, i32, i32, vp, i32, vp, vp] + [f32] * 4 + [vp, vp]),
                       ("dadmm_hyper_linear_ln", [i32, i32, i32, vp, i32, vp, vp, vp, vp, f32, i32,
                                                  f32, vp, vp, vp])):
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    L.dadmm_hyper_linear_ln_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_linear_ln_scratch_bytes.argtypes = [i32, i32, i32]
    # training mode (model.train()): forward with dropout / batch statistics, and the backward
    for name, args in (("dadmm_hyper_gcn_train", [i32] * 4 + [vp, i32, i32, vp, i32] + [vp] * 3 + [i32]
                        + [vp, vp, f32, f32, f32, u64, i32, vp, i32, vp, vp, vp, vp, vp, vp]),
                       ("dadmm_hyper_gcn_train_bwd", [i32] * 3 + [vp] * 5 + [f32, vp, i32, f32, f32, u64,
                                                                          i32, vp, vp, i32, vp]),
                       ("dadmm_hyper_linear_ln_train", [i32, i32, i32, vp, i32, vp, vp, vp, vp, f32, i32,
                                                        f32, f32, u64, i32, vp, vp, vp, vp]),
                       ("dadmm_hyper_rownorm_bwd", [i32, i32, vp, vp, vp, vp, f32, i32, f32, f32, u64,
                                                    i32, vp, vp, vp]),
                       ("dadmm_hyper_head_act", [i32, i32, i32, vp, vp] + [f32] * 4 + [vp, vp])):
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    L.dadmm_hyper_rownorm_bwd_part_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_rownorm_bwd_part_bytes.argtypes = [i32, i32]
    # one call per iteration (csrc/dadmm_hyper_net.cpp)
    L.dadmm_hyper_train_work_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_train_work_bytes.argtypes = [ctypes.POINTER(HyperNet), i32]
    L.dadmm_hyper_train_forward.restype = ctypes.c_int
    L.dadmm_hyper_train_forward.argtypes = [ctypes.POINTER(HyperNet), i32, vp, vp, vp, i32, u64,
                                            ctypes.POINTER(HyperSaved), vp, vp]
    L.dadmm_hyper_train_forward_ex.restype = ctypes.c_int
    L.dadmm_hyper_train_forward_ex.argtypes = [ctypes.POINTER(HyperNet), i32, vp, vp, vp, vp, i32, u64,
                                               ctypes.POINTER(HyperSaved), vp, vp]
    L.dadmm_hyper_train_atb_mix.restype = ctypes.c_int
    L.dadmm_hyper_train_atb_mix.argtypes = [ctypes.POINTER(HyperNet), i32, vp, vp, i32, vp, vp]
    L.dadmm_hyper_train_backward.restype = ctypes.c_int
    L.dadmm_hyper_train_backward.argtypes = [ctypes.POINTER(HyperNet), i32, vp, vp, vp, i32, u64,
                                             ctypes.POINTER(HyperSaved), vp, ctypes.POINTER(HyperGrads),
                                             vp, vp, vp]
    L.dadmm_hyper_train_dsave_floats.restype = ctypes.c_size_t
    L.dadmm_hyper_train_dsave_floats.argtypes = [ctypes.POINTER(HyperNet), i32]
    L.dadmm_hyper_train_backward_deferred.restype = ctypes.c_int
    L.dadmm_hyper_train_backward_deferred.argtypes = [ctypes.POINTER(HyperNet), i32, vp, vp, vp, i32, u64,
                                                      ctypes.POINTER(HyperSaved), vp, ctypes.POINTER(HyperGrads),
                                                      vp, vp, vp, i32, vp]
    L.dadmm_hyper_head_train.restype = ctypes.c_int
    L.dadmm_hyper_head_train.argtypes = [i32, i32, i32, vp, i32, vp, vp, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, vp, vp, vp]
    L.dadmm_hyper_linear_gcn_bwd.restype = ctypes.c_int
    L.dadmm_hyper_linear_gcn_bwd.argtypes = [i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, ctypes.c_float, vp,
                                             i32, ctypes.c_float, ctypes.c_float, ctypes.c_uint64, i32, vp, vp,
                                             i32, vp]
    L.dadmm_hyper_bn_running_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_bn_running_scratch_bytes.argtypes = [i32, vp, i32, i32]
    L.dadmm_hyper_bn_running_update.restype = ctypes.c_int
    L.dadmm_hyper_bn_running_update.argtypes = [i32, vp, vp, vp, vp, vp, vp, ctypes.c_int64, i32, i32, i32,
                                                vp, ctypes.c_double, vp, vp]
    L.dadmm_hyper_train_wgrad.restype = ctypes.c_int
    L.dadmm_hyper_train_wgrad.argtypes = [ctypes.POINTER(HyperNet), i32, i32, vp, ctypes.c_int64, vp,
                                          ctypes.POINTER(HyperSaved), ctypes.c_int64, vp, ctypes.c_int64,
                                          ctypes.POINTER(HyperGrads), vp, vp]
    L.dadmm_hyper_train_wgrad_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_train_wgrad_scratch_bytes.argtypes = [ctypes.POINTER(HyperNet), i32, i32]
    # training-mode parameter gradients (csrc/dadmm_hyper_grad.hip)
    L.dadmm_hyper_wgrad_scratch_bytes.restype = ctypes.c_size_t
    L.dadmm_hyper_wgrad_scratch_bytes.argtypes = [i32, i32, i32]
    for name, args in (("dadmm_hyper_wgrad", [i32, i32, i32, vp, i32, vp, i32, i32, vp, i32, vp, vp, i32,
                                              vp, vp]),
                       ("dadmm_hyper_colsum", [vp, i32, i32, i32, vp, i32, vp]),
                       ("dadmm_hyper_transpose", [i32, i32, vp, vp, vp])):
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    v = L.dadmm_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {v}, expected {ABI_VERSION}")
    _lib = L
    return L


def check(func: str, rc: int) -> None:
    if rc != DADMM_OK:
        raise DadmmError(func, rc, load().dadmm_last_error().decode(errors="replace"))
