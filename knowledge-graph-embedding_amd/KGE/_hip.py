"""ctypes binding of ``libkge_hip.so`` (C-ABI declared in ``include/kge_hip.h``).

The library is built in-tree by ``__graft_entry__.build()`` into
``KGE/_lib/libkge_hip.so``. ``lib()`` raises ``RuntimeError`` when it cannot be
loaded: the fused path never falls back silently.
"""

import ctypes
import os
import threading

import torch

ABI_VERSION = 8

KGE_OK, KGE_EINVAL, KGE_ERANGE, KGE_EHIP, KGE_ENOMEM_WORKSPACE, KGE_EUNSUPPORTED, KGE_EWORKSPACE = range(7)

MODEL_TRANSE, MODEL_TRANSH, MODEL_TRANSR, MODEL_TRANSD, MODEL_ROTATE, MODEL_DISTMULT, MODEL_RESCAL = range(7)
SIDE_H, SIDE_T, SIDE_HT = range(3)
IDX_I32, IDX_I64 = range(2)
SAMPLER_UNIFORM, SAMPLER_TYPED, SAMPLER_GIVEN = range(3)
OPT_NONE, OPT_SGD, OPT_GRAD, OPT_ADAM = range(4)
FLAG_NO_TABLE_CONSTRAINT = 1
FLAG_GRAD_ROWS_TOUCHED = 8
FLAG_GRAD_RENORM = 16
FLAG_PHASE_SCORE = 32
FLAG_PHASE_UPDATE = 64
FLAG_OWNER = 128
FLAG_OWNER_MERGE = 256
FLAG_DEBUG_NO_REL_SEG = 512   # test hook: relation rows in the update kernel (compact launches)
RANK_TRANS, RANK_ROT, RANK_MUL, RANK_DOT = range(4)
RANK_FLAG_LANE_PASS = 1
RPROJ_NONE, RPROJ_HYPER, RPROJ_RANK1 = range(3)

LIB_PATH = os.environ.get("KGE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                      "libkge_hip.so")   # KGE_LIB: a tuning variant (tools/variants.py)


class kge_table(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("rows", ctypes.c_int64), ("cols", ctypes.c_int64),
                ("ld", ctypes.c_int64)]


class kge_sampler_desc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("idx_dtype", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("offset", ctypes.c_uint64), ("n_entities", ctypes.c_int64), ("pool", ctypes.c_void_p),
                ("ent_type", ctypes.c_void_p), ("type_offsets", ctypes.c_void_p),
                ("type_members", ctypes.c_void_p), ("pos_in_type", ctypes.c_void_p),
                ("n_types", ctypes.c_int32), ("_pad", ctypes.c_int32)]


class kge_sample_desc(ctypes.Structure):
    _fields_ = [("sampler", kge_sampler_desc), ("X", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("side", ctypes.c_int32), ("negative_ratio", ctypes.c_int32), ("out", ctypes.c_void_p),
                ("status", ctypes.c_void_p)]


class kge_step_desc(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32), ("model", ctypes.c_int32),
        ("ent", kge_table), ("rel", kge_table), ("ent_aux", kge_table), ("rel_aux", kge_table),
        ("dim", ctypes.c_int32), ("dim_rel", ctypes.c_int32),
        ("pos", ctypes.c_void_p), ("idx_dtype", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("negative_ratio", ctypes.c_int32), ("corrupt_side", ctypes.c_int32),
        ("sampler", kge_sampler_desc), ("neg_ids", ctypes.c_void_p),
        ("score_kind", ctypes.c_int32), ("score_p", ctypes.c_float),
        ("loss_kind", ctypes.c_int32), ("margin", ctypes.c_float), ("temperature", ctypes.c_float),
        ("batch_scale", ctypes.c_float),
        ("constraint", ctypes.c_int32), ("constraint_weight", ctypes.c_float),
        ("rotate_limit", ctypes.c_float),
        ("optimizer", ctypes.c_int32), ("lr", ctypes.c_float), ("clip_norm", ctypes.c_float),
        ("loss_out", ctypes.c_void_p), ("loss_accum", ctypes.c_void_p),
        ("pos_score_out", ctypes.c_void_p), ("neg_score_out", ctypes.c_void_p),
        ("norm2_out", ctypes.c_void_p), ("status", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_uint64),
        ("prof_events", ctypes.c_void_p),
        ("flags", ctypes.c_int32), ("_pad", ctypes.c_int32),
        ("grad_out", ctypes.c_void_p * 4),
        ("shard_rows", ctypes.c_int64), ("global_entities", ctypes.c_int64),
        ("shard_count", ctypes.c_int32), ("_pad3", ctypes.c_int32),
        ("remote_rows_from", ctypes.c_int64), ("abort_flag", ctypes.c_void_p),
        ("owner_world", ctypes.c_int32), ("owner_rank", ctypes.c_int32),
        ("owner_batch", ctypes.c_int64), ("owner_rows_from", ctypes.c_int64),
        ("owner_records", ctypes.c_void_p), ("owner_stats", ctypes.c_void_p), ("owner_stats_out", ctypes.c_void_p),
        ("owner_key_capacity", ctypes.c_int64), ("owner_err", ctypes.c_void_p),
        ("owner_flags_in", ctypes.c_void_p), ("owner_flags_out", ctypes.c_void_p), ("owner_sticky", ctypes.c_void_p),
    ]


class kge_apply_desc(ctypes.Structure):
    _fields_ = [("optimizer", ctypes.c_int32), ("_pad", ctypes.c_int32), ("var", kge_table),
                ("grad", ctypes.c_void_p), ("norm2", ctypes.c_void_p), ("lr", ctypes.c_float),
                ("clip_norm", ctypes.c_float), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("beta_1", ctypes.c_float), ("beta_2", ctypes.c_float), ("epsilon", ctypes.c_float),
                ("_pad2", ctypes.c_int32), ("iteration", ctypes.c_int64), ("abort_flag", ctypes.c_void_p)]


class kge_rank_desc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("mode", ctypes.c_int32), ("proj", ctypes.c_int32),
                ("corrupt_side", ctypes.c_int32), ("cand", kge_table), ("cand_aux", kge_table),
                ("dim", ctypes.c_int32), ("clip", ctypes.c_int32), ("q0", ctypes.c_void_p), ("q1", ctypes.c_void_p),
                ("qw", ctypes.c_void_p), ("ldq", ctypes.c_int64), ("true_ids", ctypes.c_void_p),
                ("idx_dtype", ctypes.c_int32), ("score_kind", ctypes.c_int32), ("score_p", ctypes.c_float),
                ("flags", ctypes.c_int32), ("n", ctypes.c_int64), ("filt_beg", ctypes.c_void_p),
                ("filt_end", ctypes.c_void_p), ("filt_ent", ctypes.c_void_p), ("rank_out", ctypes.c_void_p),
                ("pos_score_out", ctypes.c_void_p), ("status", ctypes.c_void_p), ("filt_bits", ctypes.c_void_p),
                ("filt_bits_words", ctypes.c_int64)]


class kge_apply_rows_desc(ctypes.Structure):
    _fields_ = [("var", kge_table), ("rows", ctypes.c_void_p), ("n", ctypes.c_int64), ("grad", ctypes.c_void_p),
                ("grad_ld", ctypes.c_int64), ("norm2", ctypes.c_void_p), ("lr", ctypes.c_float),
                ("clip_norm", ctypes.c_float)]


class kge_exchange_desc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("idx_dtype", ctypes.c_int32), ("pos", ctypes.c_void_p),
                ("neg", ctypes.c_void_p), ("batch", ctypes.c_int64), ("n_neg", ctypes.c_int64),
                ("n_entities", ctypes.c_int64), ("world", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("loopback", ctypes.c_int32), ("_pad", ctypes.c_int32), ("local_rows", ctypes.c_int64),
                ("cap", ctypes.c_int64), ("htab", ctypes.c_void_p), ("hslots", ctypes.c_int64),
                ("pos_out", ctypes.c_void_p), ("neg_out", ctypes.c_void_p), ("req_ids", ctypes.c_void_p),
                ("req_cnt", ctypes.c_void_p), ("err_flag", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("zero_next", ctypes.c_void_p), ("zero_next_bytes", ctypes.c_int64)]


XROWS_GATHER, XROWS_SGD, XROWS_ACCUM, XROWS_POS = range(4)


class kge_exchange_rows_desc(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("idx_dtype", ctypes.c_int32), ("shard", kge_table),
                ("ids", ctypes.c_void_p), ("cnt", ctypes.c_void_p), ("world", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("source", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("cap", ctypes.c_int64), ("rows", ctypes.c_void_p), ("rows_ld", ctypes.c_int64),
                ("acc", ctypes.c_void_p), ("norm2", ctypes.c_void_p), ("lr", ctypes.c_float),
                ("clip_norm", ctypes.c_float), ("abort_flag", ctypes.c_void_p), ("status", ctypes.c_void_p)]


class kge_stream_desc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("idx_dtype", ctypes.c_int32), ("triples", ctypes.c_void_p),
                ("n_rows", ctypes.c_int64), ("start", ctypes.c_int64), ("batch", ctypes.c_int64),
                ("seed", ctypes.c_uint64), ("shuffle", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("out", ctypes.c_void_p)]


EXPORTS = ("kge_abi_version", "kge_last_error", "kge_step_workspace_bytes", "kge_step_plan_signature", "kge_step",
           "kge_sample",
           "kge_apply", "kge_apply_many", "kge_constrain_rows", "kge_rank", "kge_apply_rows", "kge_stream_batch",
           "kge_stream_permutation", "kge_stream_batch_perm", "kge_exchange_plan",
           "kge_exchange_rows", "kge_owner_record_floats", "kge_histogram", "kge_copy16")

_lock = threading.Lock()
_lib = None


def load(path=LIB_PATH):
    """Load the library and declare prototypes (no GPU call is made)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                "libkge_hip.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                % path)
        L = ctypes.CDLL(path)
        L.kge_abi_version.restype = ctypes.c_int32
        L.kge_last_error.restype = ctypes.c_char_p
        L.kge_step_workspace_bytes.restype = ctypes.c_uint64
        L.kge_step_workspace_bytes.argtypes = [ctypes.POINTER(kge_step_desc)]
        L.kge_step_plan_signature.restype = ctypes.c_uint32
        L.kge_step_plan_signature.argtypes = [ctypes.POINTER(kge_step_desc)]
        L.kge_owner_record_floats.restype = ctypes.c_int64
        L.kge_owner_record_floats.argtypes = [ctypes.POINTER(kge_step_desc)]
        L.kge_step.restype = ctypes.c_int
        L.kge_step.argtypes = [ctypes.POINTER(kge_step_desc), ctypes.c_void_p]
        L.kge_sample.restype = ctypes.c_int
        L.kge_sample.argtypes = [ctypes.POINTER(kge_sample_desc), ctypes.c_void_p]
        L.kge_apply.restype = ctypes.c_int
        L.kge_apply.argtypes = [ctypes.POINTER(kge_apply_desc), ctypes.c_void_p]
        L.kge_apply_many.restype = ctypes.c_int
        L.kge_apply_many.argtypes = [ctypes.POINTER(kge_apply_desc), ctypes.c_int32, ctypes.c_void_p]
        L.kge_apply_rows.restype = ctypes.c_int
        L.kge_apply_rows.argtypes = [ctypes.POINTER(kge_apply_rows_desc), ctypes.c_void_p]
        L.kge_rank.restype = ctypes.c_int
        L.kge_rank.argtypes = [ctypes.POINTER(kge_rank_desc), ctypes.c_void_p]
        L.kge_stream_batch.restype = ctypes.c_int
        L.kge_stream_batch.argtypes = [ctypes.POINTER(kge_stream_desc), ctypes.c_void_p]
        L.kge_stream_permutation.restype = ctypes.c_int
        L.kge_stream_permutation.argtypes = [ctypes.POINTER(kge_stream_desc), ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_void_p]
        L.kge_stream_batch_perm.restype = ctypes.c_int
        L.kge_stream_batch_perm.argtypes = [ctypes.POINTER(kge_stream_desc), ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int64, ctypes.c_void_p]
        L.kge_histogram.restype = ctypes.c_int
        L.kge_histogram.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.kge_copy16.restype = ctypes.c_int
        L.kge_copy16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.kge_exchange_plan.restype = ctypes.c_int
        L.kge_exchange_plan.argtypes = [ctypes.POINTER(kge_exchange_desc), ctypes.c_void_p]
        L.kge_exchange_rows.restype = ctypes.c_int
        L.kge_exchange_rows.argtypes = [ctypes.POINTER(kge_exchange_rows_desc), ctypes.c_void_p]
        L.kge_constrain_rows.restype = ctypes.c_int
        L.kge_constrain_rows.argtypes = [kge_table, ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]
        if L.kge_abi_version() != ABI_VERSION:
            raise RuntimeError("libkge_hip.so ABI %d != binding %d" % (L.kge_abi_version(), ABI_VERSION))
        _lib = L
        return L


def lib():
    return load()


def check(status, what):
    """Turn a kge_status into the reference's exception types."""
    if status == KGE_OK:
        return
    msg = "%s: %s" % (what, lib().kge_last_error().decode(errors="replace"))
    if status in (KGE_EINVAL, KGE_ERANGE):
        raise ValueError(msg)
    if status == KGE_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def check_device_status(status_tensor, what="kge"):
    """Raise if a kernel recorded a device-side error in the status word."""
    code = int(status_tensor.item())
    if code == KGE_OK:
        return
    status_tensor.zero_()
    raise_status_code(code, what)


def raise_status_code(code, what="kge"):
    """The exception of a device status word's value (KGE_OK: none)."""
    if code == KGE_OK:
        return
    if code == KGE_ERANGE:
        raise ValueError("%s: entity / relation id out of range (device check)" % what)
    if code == KGE_EINVAL:
        raise ValueError("%s: a typed-sampling pool is empty after removing the entity itself "
                         "(np.random.choice on an empty pool, utils.py:11-16)" % what)
    if code == KGE_EWORKSPACE:
        raise RuntimeError("%s: the step was refused: its workspace was last used by a different plan and was "
                           "not re-zeroed (kge_hip.h workspace rules); tables and outputs are unchanged" % what)
    raise RuntimeError("%s: device status %d" % (what, code))


def table(t):
    """kge_table view of a 2-D fp32 tensor (row stride from the tensor)."""
    if t.dtype != torch.float32 or not t.is_cuda:
        raise ValueError("embedding tables must be float32 CUDA tensors")
    t2 = t.view(t.shape[0], -1) if t.dim() != 2 else t   # never copies
    if t2.stride(1) != 1:
        raise ValueError("embedding tables must be row-major (unit column stride)")
    return kge_table(t2.data_ptr(), t2.shape[0], t2.shape[1], t2.stride(0))


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
