"""ctypes binding of oracle/liboracle.so (oracle/ysb_oracle.c).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() (as the checker)
and bench.py's cpu_baseline leg (as the timed CPU port).  Parity status: unpinned
against the reference (see ysb_oracle.c header); pinned against oracle/dostats.py
and the committed fixtures in tests/golden/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("events", "views", "joined", "join_misses", "parse_errors", "time_errors")]


class OracleRow(C.Structure):
    _fields_ = [("campaign", C.c_uint32), ("pad", C.c_uint32), ("bucket", C.c_int64), ("count", C.c_uint64)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.oracle_admap_new.restype = C.c_void_p
        L.oracle_admap_put.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32]
        L.oracle_admap_free.argtypes = [C.c_void_p]
        L.oracle_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int64,
                                 C.c_int, C.c_int, C.POINTER(C.POINTER(OracleRow)), C.POINTER(C.c_uint64),
                                 C.POINTER(OracleStats)]
        L.oracle_run_fmt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int64,
                                     C.c_int, C.c_int, C.c_int, C.POINTER(C.POINTER(OracleRow)),
                                     C.POINTER(C.c_uint64), C.POINTER(OracleStats)]
        L.oracle_free_rows.argtypes = [C.POINTER(OracleRow)]
        _LIB = L
    return _LIB


class AdMap:
    def __init__(self, ad_ids, campaign_idx):
        L = lib()
        self._h = L.oracle_admap_new()
        for a, c in zip(ad_ids, campaign_idx):
            b = a.encode() if isinstance(a, str) else bytes(a)
            L.oracle_admap_put(self._h, b, len(b), int(c))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_admap_free(self._h)
            self._h = None


def run(admap: AdMap, data, offsets, divisor=10000, require_ip=False, threads=1, fmt="json"):
    """Returns (rows dict {(campaign, bucket): count}, stats dict).  fmt: "json" or "tbl"."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    rows = C.POINTER(OracleRow)()
    nrows = C.c_uint64()
    st = OracleStats()
    rc = L.oracle_run_fmt(admap._h, buf.ctypes.data, buf.size, off.ctypes.data, off.size, int(divisor),
                          int(require_ip), int(fmt == "tbl"), int(threads), C.byref(rows), C.byref(nrows),
                          C.byref(st))
    if rc:
        raise RuntimeError("oracle_run failed")
    out = {(rows[i].campaign, rows[i].bucket): rows[i].count for i in range(nrows.value)}
    L.oracle_free_rows(rows)
    return out, {n: getattr(st, n) for n, _ in OracleStats._fields_}
