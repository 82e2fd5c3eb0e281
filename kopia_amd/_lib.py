"""Loader for the native library ``kopia_amd/libkcdc.so`` (C ABI: include/kcdc.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``).  There is
no Python or CPU fallback: if the library is missing this module raises, and
GPU entry points return KCDC_E* errors that the wrappers raise as exceptions.
"""
from __future__ import annotations

import ctypes as C
import os
from functools import lru_cache

HERE = os.path.dirname(os.path.abspath(__file__))
# KCDC_LIB: an alternative build of the same library, for A/B timing experiments only
# (tools/crypt_bench.py, tools/hash_bench.py).  It is honoured only together with
# KCDC_ALLOW_VARIANT_LIB=1, so a stray environment variable can never swap the product library.
_ALT = os.environ.get("KCDC_LIB")
if _ALT and os.environ.get("KCDC_ALLOW_VARIANT_LIB") != "1":
    raise RuntimeError("KCDC_LIB names a variant build; set KCDC_ALLOW_VARIANT_LIB=1 to load it (experiments only)")
LIB_PATH = _ALT or os.path.join(HERE, "libkcdc.so")

KCDC_OK = 0
KCDC_ENOENT = -2
KCDC_EIO = -5
KCDC_ENOMEM = -12
KCDC_ENODEV = -19
KCDC_EINVAL = -22
KCDC_EOVERFLOW = -75
KCDC_EFBIG = -27
KCDC_EBADMSG = -74

KIND_FIXED, KIND_BUZHASH, KIND_RABINKARP = 0, 1, 2
COUNT_FAILED = (1 << 64) - 1  # KCDC_COUNT_FAILED: the batch launch failed on the device
TEST_SPIN_CAP, TEST_NO_STEAL, TEST_FORCE_ERROR, TEST_HASH_LANES, TEST_NO_SERVER, TEST_NO_HELP = 1, 2, 3, 4, 5, 6
TEST_ID_RING = 7
TEST_LANE_CAP = 8
STAT_GIVEUPS, STAT_DONE, STAT_STEALS, STAT_HELPS, STAT_TICKET_AUDIT = 1, 2, 3, 4, 5
STAT_TICKETS, STAT_ENTRIES, STAT_WAVES = 10, 11, 12


class KcdcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"kcdc error {code}: {msg}")
        self.code = code


class AlgoInfo(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pooled", C.c_int32), ("avg", C.c_uint64), ("min_size", C.c_uint64),
                ("max_size", C.c_uint64), ("mask", C.c_uint64)]


_P = C.c_void_p
_SIGS = {
    "kcdc_last_error": (C.c_char_p, []),
    "kcdc_version": (C.c_char_p, []),
    "kcdc_device_count": (C.c_int, []),
    "kcdc_supported_algorithms": (C.c_int, [C.POINTER(C.c_char_p), C.c_int]),
    "kcdc_default_algorithm": (C.c_char_p, []),
    "kcdc_lookup": (C.c_int, [C.c_char_p, C.POINTER(AlgoInfo)]),
    "kcdc_max_segment_size": (C.c_int64, [C.c_char_p]),
    "kcdc_cut_capacity": (C.c_uint64, [C.c_char_p, C.c_uint64]),
    "kcdc_custom_algorithm": (C.c_char_p, [C.c_int32, C.c_uint64]),
    "kcdc_tables": (C.c_int, [_P, _P, _P, _P]),
    "kcdc_splitter_new": (_P, [C.c_char_p, C.c_int]),
    "kcdc_splitter_next": (C.c_int64, [_P, _P, C.c_size_t]),
    "kcdc_splitter_max_segment_size": (C.c_int64, [_P]),
    "kcdc_splitter_reset": (None, [_P]),
    "kcdc_splitter_close": (None, [_P]),
    "kcdc_split_batch_device": (C.c_int, [C.c_char_p, _P, _P, C.c_uint32, _P, C.c_uint64, _P, _P, _P]),
    "kcdc_split_batch_host": (C.c_int, [C.c_char_p, _P, _P, C.c_uint32, _P, C.c_uint64, _P, _P, C.c_int]),
    "kcdc_long_workspace_bytes": (C.c_size_t, [C.c_char_p, C.c_uint64]),
    "kcdc_split_long_device": (C.c_int, [C.c_char_p, _P, C.c_uint64, _P, C.c_uint64, _P, _P, C.c_size_t, _P]),
    "kcdc_fill_prng": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, _P]),
    "kcdc_split_files_device": (C.c_int, [C.c_char_p, _P, _P, C.c_uint32, _P, C.c_uint64, _P, _P, _P]),
    "kcdc_gorand_read": (C.c_int, [C.c_int64, _P, C.c_uint64]),
    "kcdc_group_new": (_P, [C.c_char_p, C.c_int, C.c_uint32, C.c_uint32]),
    "kcdc_group_splitter": (_P, [_P]),
    "kcdc_group_free": (None, [_P]),
    "kcdc_split_batch_host_devices": (C.c_int, [C.c_char_p, _P, C.c_int, _P, _P, C.c_uint32, _P, C.c_uint64, _P, _P]),
    "kcdc_lpt_assign": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P]),
    "kcdc_bw_batcher_new": (_P, [C.c_char_p, C.c_int, C.c_uint64, C.c_uint32]),
    "kcdc_bw_batcher_free": (None, [_P]),
    "kcdc_bw_batcher_new_devices": (_P, [C.c_char_p, _P, C.c_int, C.c_uint64, C.c_uint32]),
    "kcdc_bw_batcher_devices": (C.c_int, [_P]),
    "kcdc_bw_open": (_P, [_P]),
    "kcdc_bw_open_hint": (_P, [_P, C.c_uint64]),
    "kcdc_bw_device": (C.c_int, [_P]),
    "kcdc_bw_write": (C.c_int, [_P, _P, C.c_size_t]),
    "kcdc_bw_cuts": (C.c_int64, [_P, _P, C.c_uint64]),
    "kcdc_bw_cuts_ids": (C.c_int64, [_P, _P, _P, C.c_uint32, C.c_uint64]),
    "kcdc_bw_batcher_hash": (C.c_int, [_P, C.c_char_p, _P, C.c_uint32]),
    "kcdc_bw_finish": (C.c_int, [_P]),
    "kcdc_bw_free": (None, [_P]),
    "kcdc_bw_rounds": (C.c_int64, [_P]),
    "kcdc_bw_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int]),
    "kcdc_test_set": (C.c_int, [C.c_int32, C.c_int64]),
    "kcdc_test_occupy": (C.c_int, [C.c_uint32, C.c_uint32, _P]),
    "kcdc_test_queue_stat": (C.c_int64, [C.c_int32]),
    "kcdc_test_ws_copy": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64]),
    "kcdc_test_server_requests": (C.c_int64, []),
    "kcdc_hash_algorithms": (C.c_int, [C.POINTER(C.c_char_p), C.c_int]),
    "kcdc_hash_size": (C.c_int, [C.c_char_p]),
    "kcdc_hash_chunks_device": (C.c_int, [C.c_char_p, _P, _P, _P, _P, C.c_uint32, C.c_char_p, C.c_uint32, _P,
                                          C.c_uint32, _P]),
    "kcdc_encryption_algorithms": (C.c_int, [C.POINTER(C.c_char_p), C.c_int]),
    "kcdc_encryption_overhead": (C.c_int, [C.c_char_p]),
    "kcdc_crypt_workspace_size": (C.c_uint64, [C.c_uint32]),
    "kcdc_encrypt_chunks_device": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint32, _P, _P, _P, C.c_uint32, _P,
                                             C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint64, _P]),
    "kcdc_decrypt_chunks_device": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint32, _P, _P, _P, C.c_uint32, _P,
                                             C.c_uint32, C.c_uint32, _P, _P, _P, _P, C.c_uint64, _P]),
    "kcdc_compression_algorithms": (C.c_int, [C.POINTER(C.c_char_p), C.c_int]),
    "kcdc_compression_header_id": (C.c_int64, [C.c_char_p]),
    "kcdc_compress_bound": (C.c_uint64, [C.c_uint64]),
    "kcdc_compress_workspace_size": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "kcdc_compress_chunks_device": (C.c_int, [C.c_char_p, _P, _P, _P, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint64,
                                              _P]),
}


@lru_cache(maxsize=1)
def lib() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build()) first; "
                          "there is no CPU fallback")
    # One HIP runtime per process: torch's wheel bundles libamdhip64 (SONAME
    # libamdhip64.so.7, but its libraries NEED "libamdhip64.so" via RPATH).  If
    # libkcdc.so loaded /opt/rocm's copy first, torch would map a second runtime
    # and fail to initialise; loading torch first lets libkcdc bind to torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def last_error() -> str:
    msg = lib().kcdc_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> int:
    if rc < 0:
        raise KcdcError(rc, last_error())
    return rc


def exported_symbols() -> list[str]:
    return list(_SIGS)
