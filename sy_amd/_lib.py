"""ctypes binding of libsydelta.so (include/sydelta.h).

The product path has no CPU fallback: if the in-tree library is missing or fails
to load, importing this module raises immediately.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsydelta.so")

SYDELTA_OK = 0
SYDELTA_E_NODEV = -1
SYDELTA_E_OOM = -2
SYDELTA_E_INVAL = -3
SYDELTA_E_KERNEL = -4
SYDELTA_E_IO = -5

OP_COPY = 0
OP_DATA = 1


class BlockChecksumC(ctypes.Structure):
    _fields_ = [("index", ctypes.c_uint64), ("offset", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("weak", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("strong", ctypes.c_uint64)]


class OpC(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("a", ctypes.c_uint64),
                ("b", ctypes.c_uint64)]


class MatchStatsC(ctypes.Structure):
    _fields_ = [("positions", ctypes.c_uint64), ("weak_hits", ctypes.c_uint64), ("verified_hits", ctypes.c_uint64),
                ("copy_ops", ctypes.c_uint64), ("data_ops", ctypes.c_uint64), ("literal_bytes", ctypes.c_uint64)]


class BlockCompareStatsC(ctypes.Structure):
    _fields_ = [("blocks", ctypes.c_uint64), ("changed_blocks", ctypes.c_uint64), ("literal_bytes", ctypes.c_uint64),
                ("bytes_written", ctypes.c_uint64)]


class ChangeRatioC(ctypes.Structure):
    _fields_ = [("change_ratio", ctypes.c_double), ("blocks_sampled", ctypes.c_uint64),
                ("blocks_changed", ctypes.c_uint64), ("use_delta", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("threshold", ctypes.c_double)]


class DeltaStatsC(ctypes.Structure):
    _fields_ = [("operations_count", ctypes.c_uint64), ("literal_bytes", ctypes.c_uint64),
                ("bytes_written", ctypes.c_uint64)]


# Every symbol declared in include/sydelta.h: (name, restype, argtypes)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_i = ctypes.c_int
_pp = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = [
    ("sydelta_abi_version", _i, []),
    ("sydelta_last_error", ctypes.c_char_p, []),
    ("sydelta_device_count", _i, [ctypes.POINTER(_i)]),
    ("sydelta_set_devices", _i, [ctypes.POINTER(_i), _i]),
    ("sydelta_set_thread_device", _i, [_i]),
    ("sydelta_thread_device", _i, [ctypes.POINTER(_i)]),
    ("sydelta_trim", None, []),
    ("sydelta_calculate_block_size", _u64, [_u64]),
    ("sydelta_signature_device", _i, [_i, _vp, _u64, _u64, _vp, _vp, _vp]),
    ("sydelta_index_create", _i, [_i, _vp, _vp, _u64, _u64, _u64, _i, _vp, _pp]),
    ("sydelta_index_free", None, [_vp]),
    ("sydelta_match_device", _i, [_vp, _vp, _u64, _vp, _pp]),
    ("sydelta_delta_num_ops", _u64, [_vp]),
    ("sydelta_delta_ops", ctypes.POINTER(OpC), [_vp]),
    ("sydelta_delta_source_size", _u64, [_vp]),
    ("sydelta_delta_block_size", _u64, [_vp]),
    ("sydelta_delta_literal", ctypes.POINTER(ctypes.c_uint8), [_vp, _u64]),
    ("sydelta_delta_stats", _i, [_vp, ctypes.POINTER(MatchStatsC)]),
    ("sydelta_delta_compression_ratio", ctypes.c_double, [_vp]),
    ("sydelta_delta_free", None, [_vp]),
    ("sydelta_compute_checksums_buf", _i, [_i, _vp, _u64, _u64, ctypes.POINTER(BlockChecksumC), _u64,
                                           ctypes.POINTER(_u64)]),
    ("sydelta_generate_delta_buf", _i, [_i, _vp, _u64, ctypes.POINTER(BlockChecksumC), _u64, _u64, _pp]),
    ("sydelta_compute_checksums", _i, [ctypes.c_char_p, _u64, ctypes.POINTER(ctypes.POINTER(BlockChecksumC)),
                                       ctypes.POINTER(_u64)]),
    ("sydelta_checksums_free", None, [_vp]),
    ("sydelta_generate_delta_streaming", _i, [ctypes.c_char_p, ctypes.POINTER(BlockChecksumC), _u64, _u64, _pp]),
    ("sydelta_generate_delta", _i, [ctypes.c_char_p, ctypes.POINTER(BlockChecksumC), _u64, _u64, _pp]),
    ("sydelta_apply_delta", _i, [ctypes.c_char_p, _vp, ctypes.c_char_p, ctypes.POINTER(DeltaStatsC)]),
    ("sydelta_apply_delta_device", _i, [_i, _vp, _u64, _vp, _vp, _u64, _vp, _u64, _vp, ctypes.POINTER(DeltaStatsC)]),
    ("sydelta_adler32_hash", _u32, [_vp, _u64]),
    ("sydelta_signature_batch_device", _i, [_i, _vp, _vp, _vp, _u64, _u64, _vp, _vp, _vp]),
    ("sydelta_index_create_batch", _i, [_i, _vp, _vp, _vp, _vp, _u64, _u64, _i, _vp, _pp]),
    ("sydelta_match_batch_device", _i, [_vp, _vp, _vp, _vp, _u64, _vp, _pp]),
    ("sydelta_delta_pairs_device", _i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u64, _vp, _pp]),
    ("sydelta_delta_batch_count", _u64, [_vp]),
    ("sydelta_delta_batch_get", _vp, [_vp, _u64]),
    ("sydelta_delta_batch_stats", _i, [_vp, ctypes.POINTER(MatchStatsC)]),
    ("sydelta_delta_batch_free", None, [_vp]),
    ("sydelta_chunk_classify", _i, [_vp, _vp, _u64, _u64, _u64, _u64, _u64, _vp, _pp]),
    ("sydelta_chunk_walk", _i, [_vp, _u64, ctypes.POINTER(_u64), _pp]),
    ("sydelta_chunk_free", None, [_vp]),
    ("sydelta_delta_new", _vp, [_u64, _u64]),
    ("sydelta_delta_append", _i, [_vp, _vp]),
    ("sydelta_delta_from_ops", _vp, [_vp, _u64, _u64, _u64]),
    ("sydelta_delta_multi_device", _i, [ctypes.POINTER(_i), _i, ctypes.POINTER(_vp), ctypes.POINTER(_u64),
                                        ctypes.POINTER(_vp), ctypes.POINTER(_u64), ctypes.POINTER(_u64), _u64, _u64,
                                        _pp]),
    ("sydelta_checksums_to_json", _u64, [_vp, _u64, _vp, _u64]),
    ("sydelta_checksums_from_json", _i, [_vp, _u64, ctypes.POINTER(ctypes.POINTER(BlockChecksumC)),
                                         ctypes.POINTER(_u64)]),
    ("sydelta_delta_to_json", _i, [_vp, _vp, _u64, _vp, _u64, ctypes.POINTER(_u64)]),
    ("sydelta_delta_to_json_device", _i, [_vp, _vp, _u64, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    ("sydelta_delta_from_json", _i, [_vp, _u64, _pp]),
    ("sydelta_checksums_to_json_device", _i, [_vp, _vp, _u64, _u64, _u64, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    ("sydelta_checksums_from_json_device", _i, [_vp, _u64, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    ("sydelta_delta_from_json_device", _i, [_vp, _u64, _vp, _u64, ctypes.POINTER(_u64), _pp, _vp]),
    ("sydelta_zstd_bound", _u64, [_u64]),
    ("sydelta_zstd_compress_device", _i, [_i, _vp, _u64, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    ("sydelta_block_compare_device", _i, [_i, _vp, _u64, _vp, _u64, _u64, _vp, _vp, ctypes.POINTER(BlockCompareStatsC)]),
    ("sydelta_estimate_change_ratio_device", _i, [_i, _vp, _u64, _vp, _u64, _u64, ctypes.c_int64, ctypes.c_double,
                                                  _vp, ctypes.POINTER(ChangeRatioC)]),
    ("sydelta_estimate_change_ratio", _i, [ctypes.c_char_p, ctypes.c_char_p, _u64, ctypes.c_int64, ctypes.c_double,
                                           ctypes.POINTER(ChangeRatioC)]),
    ("sydelta_xxh3_device", _i, [_i, _vp, _u64, _vp, _vp]),
    ("sydelta_xxh3_batch_device", _i, [_i, _vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    ("sydelta_set_profiling", None, [_i]),
    ("sydelta_profile_json", ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t, _i]),
    ("sydelta_walk_counters", _i, [ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    ("sydelta_expand_counters", _i, [ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    ("sydelta_synth_fill", _i, [_vp, _u64, _u64, _vp]),
    ("sydelta_synth_mutate", _i, [_vp, _vp, _u64, _u64, _u32, _vp]),
    ("sydelta_synth_fill_range", _i, [_vp, _u64, _u64, _u64, _vp]),
    ("sydelta_synth_mutate_blocks", _i, [_vp, _vp, _u64, _u64, _u64, _u64, _u32, _vp]),
]


def _load() -> ctypes.CDLL:
    # One HIP runtime per process: torch (the harness's device-memory plumbing) ships
    # its own libamdhip64 with the same soname as /opt/rocm's.  Loading torch first makes
    # libsydelta bind to that copy; loaded the other way round, the two runtimes both
    # initialise and the second finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsydelta.so not found at {LIB_PATH}; build it with `python -m sy_amd.build` "
            "(there is no CPU fallback for the delta hot path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class SyDeltaError(OSError):
    """Raised for a negative status; mirrors the reference's io::Error."""

    def __init__(self, code: int, msg: str):
        super().__init__(code, msg)
        self.code = code


def check(rc: int) -> None:
    if rc != SYDELTA_OK:
        msg = lib.sydelta_last_error()
        raise SyDeltaError(rc, msg.decode() if msg else f"sydelta error {rc}")
