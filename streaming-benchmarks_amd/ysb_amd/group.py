"""Multi-GPU partitioning: the host side of the keyBy(0) replacement
(flink-benchmarks/.../AdvertisingTopologyNative.java:118-119).

Each rank (one process per GPU) counts the events of its ad_id shard into its own
[C_pad][W] (campaign, window) table; ysb_group_reduce_scatter (RCCL over xGMI, inside
libysb_hip.so) then sums the tables so that rank r owns campaigns owned_block(C, r, N).
These helpers are host functions of the same library (no GPU needed): the router for
batches that are not pre-sharded, the ownership split, and the batch splitter.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib


def owned_block(n_campaigns: int, rank: int, nranks: int):
    """[lo, hi) campaign indices rank `rank` owns after the reduce-scatter."""
    lo, hi = C.c_uint32(), C.c_uint32()
    check(lib().ysb_group_block(n_campaigns, rank, nranks, C.byref(lo), C.byref(hi)))
    return lo.value, hi.value


def route_lines(raw, offs, nranks: int):
    """(shard per line as uint32, lines per shard as uint64) of a host batch."""
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint32)
    n = offs.size
    shard = np.zeros(max(n, 1), dtype=np.uint32)
    counts = np.zeros(nranks, dtype=np.uint64)
    check(lib().ysb_route_lines(C.c_void_p(raw.ctypes.data), raw.size, C.c_void_p(offs.ctypes.data), n,
                                nranks, C.c_void_p(shard.ctypes.data), C.c_void_p(counts.ctypes.data)))
    return shard[:n], counts


def split_batch(raw, offs, shard, r: int):
    """The lines of shard r as a new packed batch (bytes, u32 offsets)."""
    raw = np.asarray(raw, dtype=np.uint8)
    offs = np.asarray(offs, dtype=np.uint64)
    ends = np.append(offs[1:], raw.size) if offs.size else offs
    sel = np.nonzero(np.asarray(shard) == r)[0]
    lens = (ends[sel] - offs[sel]).astype(np.uint64)
    new_off = np.zeros(sel.size, dtype=np.uint64)
    if sel.size:
        new_off[1:] = np.cumsum(lens)[:-1]
    idx = np.concatenate([np.arange(offs[i], ends[i], dtype=np.uint64) for i in sel]) if sel.size else \
        np.zeros(0, dtype=np.uint64)
    return raw[idx.astype(np.int64)], new_off.astype(np.uint32)


def table_rows(table, ring_lo, c_off=0):
    """{(campaign, bucket): count} of the non-zero cells of a campaign-major ring table
    [rows][W] (cell (c, b mod W) holds bucket b of [ring_lo, ring_lo + W)); row i is
    campaign c_off + i.  The layout of the device ring, the owned block and the truth table."""
    t = np.asarray(table)
    W = t.shape[-1]
    t = t.reshape(-1, W)
    cs, ss = np.nonzero(t)
    buckets = ring_lo + ((ss.astype(np.int64) - ring_lo) % W)
    return {(int(c) + c_off, int(b)): int(t[c, s]) for c, s, b in zip(cs, ss, buckets)}


def exchange_plan(slot_max, nranks: int):
    """(slots, width) every rank derives from the all-reduced per-bucket maxima of its
    pending counts (ysb_exchange_plan, the library's own host function): the ring slots
    holding a count on some rank, ascending, and the cell width in bytes (1, 4 or 8) whose
    sum over nranks cannot wrap."""
    m = np.ascontiguousarray(slot_max, dtype=np.uint64)
    W = m.size
    slots = np.zeros(max(W, 1), dtype=np.uint32)
    n, w = C.c_uint32(), C.c_uint32()
    check(lib().ysb_exchange_plan(C.c_void_p(m.ctypes.data), W, nranks, C.c_void_p(slots.ctypes.data),
                                  C.byref(n), C.byref(w)))
    return slots[:n.value].copy(), w.value


def ring_agreement(bases):
    """The common ring base the ranks agree on (ysb_group_init / the first exchange): the
    smallest base any rank holds (None: no rank has one yet)."""
    known = [b for b in bases if b is not None]
    return min(known) if known else None


def exchange_mismatches(expected, per_rank):
    """Post-exchange check: per_rank = [(owned_lo, owned_hi, {(campaign, bucket): count}), ...]
    as every owner drained after the reduce-scatter.  Returns (cells whose summed count
    differs from `expected`, ring rows an owner reported outside its campaign block, cells
    compared).  Side-list rows (buckets outside the ring) are additive deltas any rank may
    report, so a caller with out-of-ring events counts them apart."""
    merged = {}
    outside = 0
    for lo, hi, rows in per_rank:
        for (c, b), v in rows.items():
            if not lo <= c < hi:
                outside += 1
            merged[(c, b)] = merged.get((c, b), 0) + v
    keys = set(expected) | set(merged)
    mism = sum(1 for k in keys if expected.get(k, 0) != merged.get(k, 0))
    return mism, outside, len(keys)
