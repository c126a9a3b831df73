"""ctypes binding of libfedcodec.so (include/fedcodec.h).

The library is the ONLY compute path: if it is missing or fails to load, every call raises
``FedCodecUnavailable`` — there is deliberately no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfedcodec.so")

# --- constants mirrored from include/fedcodec.h --------------------------------------
FC_OK = 0
FC_STATUS_OK, FC_STATUS_RETRY_EXACT, FC_STATUS_OVERFLOW, FC_STATUS_TIMEOUT = 0, 1, 2, 3
FC_CODEC_TOP, FC_CODEC_RAND, FC_CODEC_DROPOUT_BIASED, FC_CODEC_DROPOUT_UNBIASED = 1, 2, 3, 4
FC_CODEC_QSGD = 5
FC_KEY_MAGNITUDE, FC_KEY_PHILOX = 0, 1
FC_FMT_IDXVAL, FC_FMT_BITMAP, FC_FMT_QSGD, FC_FMT_DENSE = 0, 1, 2, 3
FC_PART_SAMPLE, FC_PART_FINISH = 1, 2
FC_CHUNK = 8192
HDR_BYTES = 96


class FedCodecError(RuntimeError):
    """A C-ABI call returned an error code (message from fc_last_error())."""


class FedCodecUnavailable(RuntimeError):
    """libfedcodec.so is not built / not loadable: the HIP path is mandatory."""


class PacketHdr(ctypes.Structure):
    _fields_ = [("thresh", ctypes.c_uint64), ("lower", ctypes.c_uint64),
                ("n", ctypes.c_uint32), ("k", ctypes.c_uint32),
                ("n_entries", ctypes.c_uint32), ("index_bits", ctypes.c_uint32),
                ("codec", ctypes.c_uint32), ("status", ctypes.c_uint32),
                ("n_definite", ctypes.c_uint32), ("n_cand", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("offset", ctypes.c_uint64),
                ("p", ctypes.c_double), ("chunk", ctypes.c_uint32),
                ("format", ctypes.c_uint32), ("key_mode", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 3)]


class PacketView(ctypes.Structure):
    _fields_ = [("idx", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("bitmap", ctypes.c_void_p), ("cnt", ctypes.c_void_p),
                ("hdr", ctypes.c_void_p), ("qoff", ctypes.c_void_p),
                ("weight", ctypes.c_float), ("reserved", ctypes.c_uint32)]


class EncodeJob(ctypes.Structure):
    _fields_ = [("g", ctypes.c_void_p), ("idx", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("cnt", ctypes.c_void_p), ("hdr", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("offset", ctypes.c_uint64),
                ("qoff", ctypes.c_void_p)]


assert ctypes.sizeof(PacketHdr) == HDR_BYTES
assert ctypes.sizeof(EncodeJob) == 64
assert ctypes.sizeof(PacketView) == 56

_u64, _i32, _sz, _vp, _dbl = (ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                              ctypes.c_double)

#: every entry point declared in include/fedcodec.h: name -> (restype, argtypes)
SIGNATURES = {
    "fc_abi_version": (_i32, []),
    "fc_last_error": (ctypes.c_char_p, []),
    "fc_num_chunks": (_u64, [_u64]),
    "fc_workspace_bytes": (_sz, [_u64]),
    "fc_packet_capacity": (_u64, [_u64]),
    "fc_workspace_init": (_i32, [_vp, _sz, _vp]),
    "fc_topk_encode": (_i32, [_vp, _u64, _u64, _i32, _u64, _u64, _vp, _vp, _u64, _vp, _vp,
                              _vp, _vp, _sz, _vp]),
    "fc_topk_encode_dense": (_i32, [_vp, _u64, _u64, _vp, _vp, _u64, _vp, _vp, _vp, _vp, _sz,
                                    _vp, _vp]),
    "fc_topk_encode_decode": (_i32, [_vp, _u64, _u64, _vp, _vp, _u64, _vp, _vp, _vp, _vp, _sz,
                                     _vp, _vp]),
    "fc_workspace_bytes_batch": (_sz, [_u64, _i32]),
    "fc_topk_encode_batch": (_i32, [_vp, _i32, _u64, _u64, _i32, _u64, _vp, _sz, _vp]),
    "fc_topk_encode_batch_part": (_i32, [_vp, _i32, _u64, _u64, _i32, _u64, _vp, _sz, _i32, _vp]),
    "fc_topk_encode_exact": (_i32, [_vp, _u64, _u64, _i32, _u64, _u64, _vp, _vp, _u64, _vp,
                                    _vp, _vp, _vp, _sz, _vp]),
    "fc_mask_encode": (_i32, [_vp, _u64, _i32, _vp, _dbl, _u64, _u64, _i32, _vp, _vp, _vp,
                              _u64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "fc_decode_dense": (_i32, [ctypes.POINTER(PacketView), _i32, _u64, _vp, _i32, _vp]),
    "fc_decode_accumulate": (_i32, [_vp, _i32, _i32, _u64, _vp, _vp]),
    "fc_decode_accumulate_continue": (_i32, [_vp, _i32, _i32, _u64, _vp, _vp]),
    "fc_weighted_sum_dense": (_i32, [_vp, _vp, _i32, _u64, _vp, _vp]),
    "fc_weighted_sum_dense_continue": (_i32, [_vp, _vp, _i32, _u64, _vp, _vp]),
    "fc_div_scalar": (_i32, [_vp, _u64, ctypes.c_float, _vp]),
    "fc_flat_stage": (_i32, [_vp, _vp, _i32, _u64, _vp, _vp, _i32, _vp]),
    "fc_qsgd_code_words": (_u64, [_u64, _i32]),
    "fc_qsgd_workspace_bytes": (_sz, []),
    "fc_qsgd_encode": (_i32, [_vp, _u64, _i32, _u64, _u64, _vp, _u64, _vp, _vp, _sz, _vp]),
    "fc_qsgd_decode": (_i32, [ctypes.POINTER(PacketView), _u64, _vp, _vp]),
    "fc_qsgd_decode_accumulate": (_i32, [_vp, _i32, _u64, _vp, _i32, _vp]),
    "fc_topk_dense_f64": (_i32, [_vp, _u64, _u64, _i32, _u64, _u64, _vp, _vp, _sz, _vp]),
    "fc_topk_dense_f64_sampled": (_i32, [_vp, _u64, _u64, _vp, _vp, _sz, _vp, _vp]),
    "fc_mask_dense_f64": (_i32, [_vp, _u64, _i32, _vp, _dbl, _u64, _u64, _vp, _vp]),
    "fc_mask_dense_f32": (_i32, [_vp, _u64, _i32, _vp, _dbl, _u64, _u64, _vp, _vp]),
    "fc_weighted_sum_dense_f64": (_i32, [_vp, _i32, _vp, _i32, _u64, _vp, _i32, _vp]),
    "fc_div_scalar_f64": (_i32, [_vp, _u64, _dbl, _vp]),
    "fc_mt_plan_bytes": (_sz, [_u64, _i32]),
    "fc_mt_workspace_bytes": (_sz, [_i32]),
    "fc_mt_plan": (_i32, [_u64, _i32, _vp, _sz, _vp]),
    "fc_mt_begin": (_i32, [_vp, _sz, _u64, _i32, _vp, ctypes.c_uint32, _vp, _sz, _vp]),
    "fc_mt_binomial": (_i32, [_vp, _sz, _u64, _i32, _i32, _dbl, _vp, _vp, _sz, _vp]),
    "fc_mt_jump_poly": (_i32, [_u64, _vp]),
    "fc_mt_charpoly": (_i32, [_vp]),
    "fc_fused_order_begin": (_i32, [_vp]),
    "fc_fused_order_end": (_i32, [_vp]),
    "fc_timing_begin": (_i32, [ctypes.c_uint32]),
    "fc_timing_end": (_i32, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
}

FC_TIME_COMPACT, FC_TIME_DECODE, FC_TIME_ENGINE, FC_TIME_SAMPLE = 1, 2, 4, 8
TIME_CLASSES = ("compact", "decode", "engine", "sample")


class KernelTimer:
    """HIP-event timing of selected kernel classes on the stream they are launched on."""

    def __init__(self, mask: int = 0xF):
        self.mask = mask
        self.ms = {}
        self.launches = {}

    def __enter__(self):
        check(load().fc_timing_begin(self.mask), "fc_timing_begin")
        return self

    def __exit__(self, *exc):
        ms = (ctypes.c_double * 4)()
        n = (ctypes.c_uint64 * 4)()
        check(load().fc_timing_end(ms, n), "fc_timing_end")
        self.ms = {c: ms[i] for i, c in enumerate(TIME_CLASSES)}
        self.launches = {c: int(n[i]) for i, c in enumerate(TIME_CLASSES)}
        return False

    def avg_us(self, cls: str) -> float:
        n = self.launches.get(cls, 0)
        return 1e3 * self.ms[cls] / n if n else float("nan")

_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """Load and declare libfedcodec.so (torch is imported first: one HIP runtime)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (binds libamdhip64.so.7 from torch before our .so)
        if not os.path.exists(path):
            raise FedCodecUnavailable(
                f"{path} not built — run `python -m openmsftl_amd.build` (hipcc, gfx950)")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:
            raise FedCodecUnavailable(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                if path == LIB_PATH:            # the product library must export every entry
                    raise
                continue                        # an older A/B build (tools/ab.py --lib)
            fn.restype = res
            fn.argtypes = args
        # the product library is ABI 4; an A/B build (tools/ab.py --lib) may predate the bump
        # (3 differs only in the documented fc_topk_encode_dense packet contract)
        if lib.fc_abi_version() not in ((4,) if path == LIB_PATH else (3, 4)):
            raise FedCodecUnavailable("libfedcodec.so ABI mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != FC_OK:
        msg = load().fc_last_error()
        raise FedCodecError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
