"""ctypes binding of libsgx.so (the C ABI declared in include/sgx.h).

There is no fallback: if the in-tree HIP library is missing or cannot be loaded, every
entry point raises.  Negative return codes are mapped to the exception types the JVM side
would throw (ShuffleTransport.scala:49-51,71 / the reference's IllegalArgument- and
IllegalStateExceptions, NvkvShuffleMapOutputWriter.scala:108, DpuShuffleExecutorComponents
.scala:28-30).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsgx.so")

SGX_OK = 0
SGX_ERR_INVALID, SGX_ERR_STATE, SGX_ERR_HIP, SGX_ERR_COMM = -1, -2, -3, -4
SGX_ERR_IO, SGX_ERR_NOMEM, SGX_ERR_NOT_FOUND, SGX_ERR_UNSUPPORTED, SGX_ERR_TIMEOUT = -5, -6, -7, -8, -9
PART_HASH, PART_RANGE_I64, PART_RANGE_BYTES10 = 0, 1, 2
MEM_HOST, MEM_DEVICE, MEM_DEVICE_RETAINED = 0, 1, 2
AGG_GROUP, AGG_SUM = 0, 1
SER_FIXED, SER_KRYO = 0, 1
STAGES = ("hist", "scan", "scatter", "allgather", "alltoall", "regroup", "sort", "group", "serialize",
          "deserialize", "combine", "compress", "decompress")
HIST_ATOMIC, HIST_BALLOT = 0, 1
RANK_ORDERED, RANK_MATCH = 0, 1
FLAG_NO_WRITE_COMBINING, FLAG_NO_WIDE_STAGED, FLAG_SORT_ALL_DIGITS, FLAG_DEBUG_SYNC = 1, 2, 4, 8
FLAG_LZ4_LANE_DECODE = 16
FLAG_NO_SPLIT_SCATTER = 32
FLAG_NO_BUCKET_SORT = 64
FLAG_ASSUME_LDS_DISORDER = 128
FLAG_NO_PADDED_MAP = 256
FLAG_PAD_ANY_SIZE = 512
FLAG_NO_SEG_WINDOW = 1024
FLAG_NO_DEFERRED_APPEND = 2048
FLAG_NO_P2P_EXCHANGE = 4096
FLAG_NO_OVERLAP_WRITES = 8192
FLAG_TEST_P2P_UNAVAILABLE = 16384
LAYOUT_CONTIGUOUS, LAYOUT_PADDED, LAYOUT_SERIALIZED_PADDED = 0, 1, 2
PLACE_EVEN, PLACE_BYTES = 0, 1
WRITER_SORT, WRITER_UNSAFE = 0, 1
ABI_VERSION = 7


class ShuffleError(RuntimeError):
    """Base of every error raised through the C ABI (OperationStatus.FAILURE)."""

    code = -100


class IllegalArgumentException(ShuffleError, ValueError):
    code = SGX_ERR_INVALID


class IllegalStateException(ShuffleError):
    code = SGX_ERR_STATE


class DeviceError(ShuffleError):
    code = SGX_ERR_HIP


class TransportError(ShuffleError):
    code = SGX_ERR_COMM


class ShuffleIOException(ShuffleError, IOError):
    code = SGX_ERR_IO


class DeviceOutOfMemory(ShuffleError, MemoryError):
    code = SGX_ERR_NOMEM


class BlockNotFoundException(ShuffleError, KeyError):
    code = SGX_ERR_NOT_FOUND


class UnsupportedOperationException(ShuffleError):
    code = SGX_ERR_UNSUPPORTED


class DeviceTimeout(ShuffleError):
    code = SGX_ERR_TIMEOUT


_BY_CODE = {c.code: c for c in (IllegalArgumentException, IllegalStateException, DeviceError,
                                TransportError, ShuffleIOException, DeviceOutOfMemory,
                                BlockNotFoundException, UnsupportedOperationException, DeviceTimeout)}

_lib = None
_lock = threading.Lock()

_i32, _i64, _u64, _vp, _cp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_char_p
_P64, _P32 = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes).  Must cover every function declared in include/sgx.h.
SIGNATURES = {
    "sgx_create": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "sgx_destroy": (None, [_vp]),
    "sgx_release_thread": (ctypes.c_int, [_vp]),
    "sgx_set_map_side_combine": (ctypes.c_int, [_vp, _i32, _i32]),
    "sgx_set_map_writer": (ctypes.c_int, [_vp, _i32, _i32]),
    "sgx_map_begin": (ctypes.c_int, [_vp, _i32, _i64]),
    "sgx_map_append": (ctypes.c_int, [_vp, _i32, _i64, _vp, _i64, _i32, _i32]),
    "sgx_map_commit": (ctypes.c_int, [_vp, _i32, _i64, _vp]),
    "sgx_comm_init_host": (ctypes.c_int, [_vp, _i32, _i32, _vp]),
    "sgx_pool_get": (ctypes.c_int, [_vp, _i64, _i32, ctypes.POINTER(_vp), _P64]),
    "sgx_pool_put": (ctypes.c_int, [_vp, _vp]),
    "sgx_pool_preallocate": (ctypes.c_int, [_vp, _i64, _i32, _i32]),
    "sgx_pool_stats": (ctypes.c_int, [_vp, _P64, _P64]),
    "sgx_last_error": (_cp, []),
    "sgx_abi_version": (_i32, []),
    "sgx_lds_order_ok": (_i32, [_vp]),
    "sgx_register_shuffle": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _i64, _i32, _i32]),
    "sgx_unregister_shuffle": (ctypes.c_int, [_vp, _i32]),
    "sgx_set_serializer": (ctypes.c_int, [_vp, _i32, _i32]),
    "sgx_lz4_frame_partitions": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "sgx_lz4_unframe": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _P64]),
    "sgx_lz4_unframe_streams": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _P64]),
    "sgx_set_compression": (ctypes.c_int, [_vp, _i32, _i32, _i32]),
    "sgx_write_map": (ctypes.c_int, [_vp, _i32, _i64, _vp, _i64, _i32, _i32, _vp]),
    "sgx_map_lengths": (ctypes.c_int, [_vp, _i32, _i64, _vp]),
    "sgx_map_data": (ctypes.c_int, [_vp, _i32, _i64, ctypes.POINTER(_vp), _P64]),
    "sgx_map_layout": (ctypes.c_int, [_vp, _i32, _i64, _P32]),
    "sgx_write_index": (ctypes.c_int, [_vp, _i32, _i64, _cp, _cp, _vp]),
    "sgx_check_index_and_data": (ctypes.c_int, [_cp, _cp, _i32, _vp]),
    "sgx_index_block_range": (ctypes.c_int, [_cp, _i32, _i32, _P64, _P64]),
    "sgx_get_unique_id": (ctypes.c_int, [_vp]),
    "sgx_comm_init": (ctypes.c_int, [_vp, _i32, _i32, _vp]),
    "sgx_comm_size": (ctypes.c_int, [_vp, _P32, _P32]),
    "sgx_exchange": (ctypes.c_int, [_vp, _i32]),
    "sgx_exchange_maps": (ctypes.c_int, [_vp, _i32, _vp, _i64]),
    "sgx_exchange_fail": (ctypes.c_int, [_vp, _i32, _i32]),
    "sgx_import_blocks": (ctypes.c_int, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _i32, _vp, _P64]),
    "sgx_release_import": (ctypes.c_int, [_vp, _i32, _i64]),
    "sgx_shuffle_reducers": (ctypes.c_int, [_vp, _i32, _vp, _vp]),
    "sgx_plan_exchange_maps": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sgx_fetch_blocks": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i64, _vp, _i64, _i32, _vp]),
    "sgx_read_sorted": (ctypes.c_int, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _i64, _i32, _vp]),
    "sgx_read_records": (ctypes.c_int, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _i64, _i32, _vp]),
    "sgx_range_bounds": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "sgx_bootstrap_serve": (ctypes.c_int, [_i32, _i32, _vp, _i32]),
    "sgx_bootstrap_join": (ctypes.c_int, [ctypes.c_char_p, _i32, _i32, _i32, _vp, _vp]),
    "sgx_read_grouped": (ctypes.c_int, [_vp, _i32, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _i64, _i64, _i32,
                                        _vp, _vp]),
    "sgx_last_read_records": (ctypes.c_int, [_vp, _vp]),
    "sgx_progress": (ctypes.c_int, [_vp]),
    "sgx_sync": (ctypes.c_int, [_vp]),
    "sgx_stats_reset": (ctypes.c_int, [_vp]),
    "sgx_stats_get": (ctypes.c_int, [_vp, _vp, _vp]),
    "sgx_exchange_bytes": (ctypes.c_int, [_vp, _vp]),
    "sgx_set_overlap_writes": (ctypes.c_int, [_vp, ctypes.c_int32]),
    "sgx_plan_exchange": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _P64]),
    "sgx_copy_items": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i32]),
    "sgx_reducer_owner": (_i32, [_i32, _i32, _i32]),
    "sgx_plan_exchange_ranges": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _P64]),
    "sgx_balanced_ranges": (ctypes.c_int, [_vp, _i32, _i32, _vp]),
    "sgx_even_ranges": (ctypes.c_int, [_i32, _i32, _vp]),
    "sgx_set_reducer_placement": (ctypes.c_int, [_vp, _i32, _i32]),
    "sgx_round_reducers": (ctypes.c_int, [_vp, _i32, _i64, _vp, _vp]),
    "sgx_gen_uniform16": (ctypes.c_int, [_vp, _vp, _i64, _u64, _i64]),
    "sgx_gen_zipf16": (ctypes.c_int, [_vp, _vp, _i64, _u64, _i64, _vp, _i64]),
    "sgx_gen_terasort100": (ctypes.c_int, [_vp, _vp, _i64, _u64, _i64]),
    "sgx_device_alloc": (ctypes.c_int, [_vp, _i64, ctypes.POINTER(_vp)]),
    "sgx_device_free": (ctypes.c_int, [_vp, _vp]),
    "sgx_memcpy": (ctypes.c_int, [_vp, _vp, _vp, _i64]),
}


# tools/ab_run.py only: bind what an older engine build exports (its missing calls are unused)
ALLOW_MISSING = False


def lib() -> ctypes.CDLL:
    """Load the in-tree libsgx.so (raises if it was not built: no CPU fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is missing: build the HIP extension first "
                    "(python -c 'import __graft_entry__ as g; g.build()'); "
                    "sparkucx_amd has no CPU fallback")
            L = ctypes.CDLL(LIB_PATH)
            L.sgx_abi_version.restype = _i32
            if L.sgx_abi_version() != ABI_VERSION:
                raise ImportError(f"{LIB_PATH} has ABI {L.sgx_abi_version()}, the bindings expect {ABI_VERSION}: rebuild")
            for name, (res, args) in SIGNATURES.items():
                if ALLOW_MISSING and not hasattr(L, name):
                    continue  # an older build under A/B measurement (tools/ab_run.py)
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


# sgx_host_comm (include/sgx.h): the caller's collectives of the host exchange backend
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _i64, _vp)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _P64, _P64, _vp, _P64, _P64)


class HostCommStruct(ctypes.Structure):
    _fields_ = [("user", _vp), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


def last_error() -> str:
    msg = lib().sgx_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, what: str = "") -> int:
    """Raise the mapped exception for a negative return code."""
    if rc >= 0:
        return rc
    cls = _BY_CODE.get(rc, ShuffleError)
    raise cls(f"{what}: {last_error()} (code {rc})" if what else f"{last_error()} (code {rc})")
