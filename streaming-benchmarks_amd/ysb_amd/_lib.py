"""ctypes binding of libysb_hip.so (include/ysb_hip.h).

The library is built in-tree (streaming-benchmarks_amd/lib/libysb_hip.so) by
`make -C streaming-benchmarks_amd` / __graft_entry__.build().  There is no CPU
fallback: if the library is missing, importing a compute entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# YSB_LIB_VARIANT=stamps selects the diagnostic build (tools/stamps.py only)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libysb_hip%s.so" % (
    "_" + os.environ["YSB_LIB_VARIANT"] if os.environ.get("YSB_LIB_VARIANT") else ""))

YSB_OK = 0
YSB_PENDING = 1
ERRORS = {-1: "YSB_ERR_ARG", -2: "YSB_ERR_HIP", -3: "YSB_ERR_STATE", -4: "YSB_ERR_CAPACITY",
          -5: "YSB_ERR_FORMAT", -6: "YSB_ERR_RCCL", -7: "YSB_ERR_NOMEM", -8: "YSB_ERR_DATA"}

YSB_F_TIMING = 0x1
YSB_F_REQUIRE_IP = 0x2
YSB_F_NO_LDS_COUNT = 0x4
YSB_F_SPARSE_FAST_JOIN = 0x8
YSB_F_FORMAT_TBL = 0x10
YSB_F_RECORD_COUNT = 0x20
YSB_F_NO_RECORD_COUNT = 0x40
YSB_F_COMPACT_FIRST = 0x80
YSB_F_FLAT_FIRST = 0x100
YSB_F_LAYOUT_AUTO = 0x200   # the default since ABI 2 (accepted, ignored)
YSB_F_STRICT = 0x400
YSB_F_LAYOUT_FIXED = 0x800
YSB_F_H2D_SDMA = 0x1000
YSB_SUM_TRUTH_BLOCKS = 0
YSB_SUM_PENDING_BLOCKS = 1
YSB_SUM_OWNED = 2
INT64_MIN = -(1 << 63)
UNIQUE_ID_BYTES = 128


class YsbConfig(C.Structure):
    _fields_ = [("time_divisor_ms", C.c_int64), ("n_campaigns", C.c_uint32), ("window_ring", C.c_uint32),
                ("max_ads", C.c_uint64), ("max_batch_events", C.c_uint64), ("max_batch_bytes", C.c_uint64),
                ("ring_base_bucket", C.c_int64), ("overflow_capacity", C.c_uint64), ("flags", C.c_uint32),
                ("reserved", C.c_uint32)]


class YsbStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("events", "views", "joined", "join_misses", "parse_errors",
                                          "time_errors", "out_of_ring", "overflow_dropped", "batches", "deferred",
                                          "foreign_shard")]


class YsbCount(C.Structure):
    _fields_ = [("campaign", C.c_uint32), ("reserved", C.c_uint32), ("window_ms", C.c_int64),
                ("count", C.c_uint64)]


class YsbExchangeInfo(C.Structure):
    _fields_ = [("exchanges", C.c_uint64), ("bytes", C.c_uint64), ("ms", C.c_double), ("last_buckets", C.c_uint32),
                ("last_width", C.c_uint32), ("full_ring_bytes", C.c_uint64), ("critical_ms", C.c_double),
                ("rs_ms", C.c_double), ("exposed_ms", C.c_double)]


class YsbRebase(C.Structure):
    _fields_ = [("first_line", C.c_uint64), ("lead_shift", C.c_int64)]


class YsbLaunchDesc(C.Structure):
    _fields_ = [("layout", C.c_uint32), ("record_mode", C.c_uint32), ("hbm_table", C.c_uint32), ("tbl", C.c_uint32)]


ALLREDUCE_MAX_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64)
REDUCE_SCATTER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32)


class YsbCollectives(C.Structure):
    _fields_ = [("allreduce_max_u64", ALLREDUCE_MAX_FN), ("reduce_scatter_sum", REDUCE_SCATTER_FN),
                ("user", C.c_void_p)]


class YsbSegment(C.Structure):
    _fields_ = [("d_bytes", C.c_void_p), ("nbytes", C.c_uint64), ("d_line_off", C.c_void_p),
                ("n_events", C.c_uint64)]


class YsbGenParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_campaigns", C.c_uint32), ("ads_per_campaign", C.c_uint32),
                ("t0_ms", C.c_int64), ("events_per_sec", C.c_uint64), ("with_skew", C.c_uint32),
                ("n_users", C.c_uint32), ("ad_subset", C.POINTER(C.c_uint32)), ("n_ad_subset", C.c_uint32),
                ("event_stream", C.c_uint32),
                ("format", C.c_uint32), ("variant", C.c_uint32)]


_P = C.c_void_p
_I = C.c_int
_U32 = C.c_uint32
_U64 = C.c_uint64
_I64 = C.c_int64
_PU8 = C.c_void_p
_PU32 = C.c_void_p

# name -> (restype, argtypes); every function include/ysb_hip.h declares.
SIGNATURES = {
    "ysb_abi_version": (_I, []),
    "ysb_device_count": (_I, []),
    "ysb_device_sync": (_I, [_I]),
    "ysb_device_numa_node": (_I, [_I]),
    "ysb_config_default": (None, [C.POINTER(YsbConfig)]),
    "ysb_open": (_I, [C.POINTER(_P), _I, C.POINTER(YsbConfig)]),
    "ysb_close": (_I, [_P]),
    "ysb_last_error": (C.c_char_p, [_P]),
    "ysb_load_ad_map": (_I, [_P, C.POINTER(C.c_char_p), C.POINTER(_U32), C.POINTER(_U32), _U64]),
    "ysb_load_ad_map_packed": (_I, [_P, C.c_void_p, _U32, C.c_void_p, _U64]),
    "ysb_load_ad_map_shard": (_I, [_P, C.POINTER(C.c_char_p), C.POINTER(_U32), C.POINTER(_U32), _U64, _U32, _U32]),
    "ysb_load_ad_map_packed_shard": (_I, [_P, C.c_void_p, _U32, C.c_void_p, _U64, _U32, _U32]),
    "ysb_slot_buffers": (_I, [_P, _I, C.POINTER(_P), C.POINTER(_P)]),
    "ysb_submit": (_I, [_P, _I, _PU8, _U64, _PU32, _U64]),
    "ysb_wait": (_I, [_P, _I]),
    "ysb_slot_capacity": (_I, [_P, C.POINTER(_U64), C.POINTER(_U64)]),
    "ysb_submit_raw": (_I, [_P, _I, _PU8, _U64]),
    "ysb_host_register": (_I, [_P, _P, _U64]),
    "ysb_host_unregister": (_I, [_P, _P]),
    "ysb_rebase_table": (_I, [_P, C.c_void_p, _U64, _I64]),
    "ysb_submit_raw_mapped": (_I, [_P, _I, _PU8, _U64, C.POINTER(YsbRebase)]),
    "ysb_submit_mapped": (_I, [_P, _I, _PU8, _U64, _PU32, _U64, C.POINTER(YsbRebase)]),
    "ysb_split_lines_device": (_I, [_P, _PU8, _U64, _PU32, _U64, C.POINTER(_U64)]),
    "ysb_copy_time": (_I, [_P, C.POINTER(C.c_double), C.POINTER(_U64), C.POINTER(_U64)]),
    "ysb_submit_device": (_I, [_P, _PU8, _U64, _PU32, _U64]),
    "ysb_submit_device_segments": (_I, [_P, C.c_void_p, _U32]),
    "ysb_sync": (_I, [_P]),
    "ysb_drain": (_I, [_P, _I64, _I64, _I, C.POINTER(YsbCount), _U64, C.POINTER(_U64)]),
    "ysb_stats_get": (_I, [_P, C.POINTER(YsbStats)]),
    "ysb_flush_begin": (_I, [_P, _I64, _I64]),
    "ysb_flush_end": (_I, [_P, _I, C.POINTER(YsbCount), _U64, C.POINTER(_U64), C.POINTER(_I)]),
    "ysb_reset": (_I, [_P]),
    "ysb_ring_range": (_I, [_P, C.POINTER(_I64), C.POINTER(_U32)]),
    "ysb_ring_advance": (_I, [_P, _I64]),
    "ysb_kernel_time": (_I, [_P, C.POINTER(C.c_double), C.POINTER(_U64)]),
    "ysb_path_time": (_I, [_P, C.POINTER(C.c_double), C.POINTER(_U64), C.POINTER(_U64)]),
    "ysb_stream": (_P, [_P]),
    "ysb_launch_info": (_I, [_P, C.POINTER(YsbLaunchDesc)]),
    "ysb_layout_of_line": (_I, [C.c_char_p, _U64, _I, C.c_void_p, C.POINTER(_U32), C.POINTER(_U32)]),
    "ysb_device_alloc": (_I, [_P, _U64, C.POINTER(_P)]),
    "ysb_device_free": (_I, [_P, _P]),
    "ysb_memcpy_h2d": (_I, [_P, _P, _P, _U64]),
    "ysb_memcpy_d2h": (_I, [_P, _P, _P, _U64]),
    "ysb_group_unique_id": (_I, [C.c_char_p]),
    "ysb_group_init": (_I, [_P, _I, _I, C.c_char_p]),
    "ysb_group_reduce_scatter": (_I, [_P]),
    "ysb_group_exchange_pipelined": (_I, [_P]),
    "ysb_group_init_host": (_I, [_P, _I, _I, C.POINTER(YsbCollectives)]),
    "ysb_group_exchange_info": (_I, [_P, C.POINTER(YsbExchangeInfo), _I]),
    "ysb_exchange_info_size": (_U64, []),
    "ysb_exchange_plan": (_I, [C.c_void_p, _U32, _U32, C.c_void_p, C.POINTER(_U32), C.POINTER(_U32)]),
    "ysb_group_checksum": (_I, [_P, _I, _U32, C.c_void_p]),
    "ysb_group_owned": (_I, [_P, C.POINTER(_U32), C.POINTER(_U32)]),
    "ysb_group_info": (_I, [_P, C.POINTER(_I), C.POINTER(_I)]),
    "ysb_ad_shard": (_U32, [C.c_char_p, _U32, _U32]),
    "ysb_group_block": (_I, [_U32, _I, _I, C.POINTER(_U32), C.POINTER(_U32)]),
    "ysb_route_lines": (_I, [_PU8, _U64, _PU32, _U64, _U32, _PU32, C.c_void_p]),
    "ysb_gen_default": (None, [C.POINTER(YsbGenParams)]),
    "ysb_gen_ids": (_I, [C.POINTER(YsbGenParams), _P, _P]),
    "ysb_gen_events_host": (_I, [C.POINTER(YsbGenParams), _U64, _U64, _PU8, _U64, _PU32, C.POINTER(_U64)]),
    "ysb_gen_events_host_mt": (_I, [C.POINTER(YsbGenParams), _U64, _U64, _PU8, _U64, _PU32, C.POINTER(_U64), _U32]),
    "ysb_gen_events_device": (_I, [_P, C.POINTER(YsbGenParams), _U64, _U64, _PU8, _U64, _PU32, C.POINTER(_U64)]),
    "ysb_gen_max_line_bytes": (_U64, [C.POINTER(YsbGenParams)]),
    "ysb_truth_accumulate": (_I, [_P, C.POINTER(YsbGenParams), _U64, _U64]),
    "ysb_truth_compare": (_I, [_P, C.POINTER(_U64), C.POINTER(_U64), C.POINTER(_U64)]),
    "ysb_truth_read": (_I, [_P, C.c_void_p, _U64, C.POINTER(_I64)]),
    "ysb_gen_dump": (_I, [C.POINTER(YsbGenParams), _U64, C.c_char_p]),
    "ysb_json_to_tbl": (_I, [_PU8, _U64, _PU32, _U64, _PU8, _U64, _PU32, C.POINTER(_U64)]),
    "ysb_gen_dump_shards": (_I, [C.POINTER(YsbGenParams), _U64, C.c_char_p, _U32]),
}

ABI_VERSION = 5   # include/ysb_hip.h YSB_ABI_VERSION this binding is written against

_lib = None


class YsbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "?"), code, msg))
        self.code = code


def lib():
    """The loaded library.  Raises if the in-tree build is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libysb_hip.so not built at %s: run `make -C streaming-benchmarks_amd` "
                              "(or __graft_entry__.build())" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        # the structs this binding lays out must be the library's (ysb_exchange_info grew in
        # ABI 4: an older caller's struct would be written past its end)
        if L.ysb_abi_version() != ABI_VERSION:
            raise ImportError("%s has ABI %d, this binding is written for ABI %d: rebuild the library"
                              % (LIB_PATH, L.ysb_abi_version(), ABI_VERSION))
        if L.ysb_exchange_info_size() != C.sizeof(YsbExchangeInfo):
            raise ImportError("ysb_exchange_info is %d bytes in the library, %d in this binding"
                              % (L.ysb_exchange_info_size(), C.sizeof(YsbExchangeInfo)))
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != YSB_OK:
        msg = lib().ysb_last_error(ctx)
        raise YsbError(rc, msg.decode() if msg else "")
    return rc
