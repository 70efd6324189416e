"""Seeded generator of the data/ generator's event format (data/src/setup/core.clj:61-98,
163-181), file-dump mode included.  Host generation runs in the C library (no GPU
needed); device generation writes straight into HBM (YsbContext.gen_events_device).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import YsbGenParams, check, lib

AD_TYPES = ("banner", "modal", "sponsored-search", "mail", "mobile")   # core.clj:68
MORE_AD_TYPES = AD_TYPES + ("native-video", "interstitial", "rewarded")  # GEN_MORE_AD_TYPES
GEN_RANDOM_IP, GEN_MORE_AD_TYPES, GEN_COMPACT, GEN_REORDER, GEN_MIXED, GEN_MIXED_BLOCKS = 1, 2, 4, 8, 16, 32
EVENT_TYPES = ("view", "click", "purchase")                            # core.clj:69


class GenParams:
    """Generator parameters; defaults: seed 42, 100 campaigns x 10 ads (core.clj:15,52),
    t0 1.7e12 ms, 100,000 events per second of event time."""

    def __init__(self, seed=42, n_campaigns=100, ads_per_campaign=10, t0_ms=1_700_000_000_000,
                 events_per_sec=100_000, with_skew=False, n_users=0, ad_subset=None, event_stream=0,
                 fmt="json", variant=0):
        self.c = YsbGenParams()
        lib().ysb_gen_default(C.byref(self.c))
        self.c.seed = seed
        self.c.n_campaigns = n_campaigns
        self.c.ads_per_campaign = ads_per_campaign
        self.c.t0_ms = t0_ms
        self.c.events_per_sec = events_per_sec
        # True / 1: +-50 ms skew and 1e-5 late events (core.clj:166-174); 2: the skew only
        self.c.with_skew = with_skew if isinstance(with_skew, int) and not isinstance(with_skew, bool) else int(bool(with_skew))
        if self.c.with_skew > 2:
            raise ValueError("with_skew must be 0 (off), 1 (skew + late events) or 2 (skew only)")
        self.c.n_users = n_users
        self.c.event_stream = event_stream
        if fmt not in ("json", "tbl"):
            raise ValueError("fmt must be 'json' or 'tbl'")
        self.c.format = 1 if fmt == "tbl" else 0   # YSB_GEN_TBL: the fork's .tbl rows
        # variant: GEN_RANDOM_IP | GEN_MORE_AD_TYPES | GEN_COMPACT | GEN_REORDER (off-vocabulary layouts)
        self.c.variant = variant
        self._subset = None
        if ad_subset is not None:
            self._subset = np.ascontiguousarray(ad_subset, dtype=np.uint32)
            self.c.ad_subset = self._subset.ctypes.data_as(C.POINTER(C.c_uint32))
            self.c.n_ad_subset = self._subset.size

    @property
    def n_ads(self):
        return self.c.n_campaigns * self.c.ads_per_campaign

    def ids(self):
        """(campaign_ids, ad_ids) as lists of 36-char str; ad a -> campaign a // ads_per_campaign."""
        cb = C.create_string_buffer(36 * self.c.n_campaigns)
        ab = C.create_string_buffer(36 * self.n_ads)
        check(lib().ysb_gen_ids(C.byref(self.c), cb, ab))
        craw, araw = cb.raw.decode(), ab.raw.decode()
        return ([craw[36 * i:36 * i + 36] for i in range(self.c.n_campaigns)],
                [araw[36 * i:36 * i + 36] for i in range(self.n_ads)])

    def ids_packed(self):
        """(campaign ids, ad ids) as uint8 arrays of 36-byte UUIDs back to back (large maps)."""
        cb = np.zeros(36 * self.c.n_campaigns, dtype=np.uint8)
        ab = np.zeros(36 * self.n_ads, dtype=np.uint8)
        check(lib().ysb_gen_ids(C.byref(self.c), C.c_void_p(cb.ctypes.data), C.c_void_p(ab.ctypes.data)))
        return cb, ab

    def ad_campaign_index_array(self):
        return (np.arange(self.n_ads, dtype=np.uint64) // self.c.ads_per_campaign).astype(np.uint32)

    def ad_campaign_index(self):
        return [a // self.c.ads_per_campaign for a in range(self.n_ads)]

    def max_line_bytes(self):
        return int(lib().ysb_gen_max_line_bytes(C.byref(self.c)))

    def events_host_tbl(self, first, n):
        """Events [first, first+n) as .tbl rows (bytes, u32 offsets)."""
        return json_to_tbl(*self.events_host(first, n))

    def events_host(self, first, n):
        """(bytes as uint8 array, uint32 line offsets) of events [first, first+n)."""
        cap = n * self.max_line_bytes()
        out = np.empty(max(cap, 1), dtype=np.uint8)
        off = np.empty(max(n, 1), dtype=np.uint32)
        nb = C.c_uint64()
        check(lib().ysb_gen_events_host(C.byref(self.c), first, n, C.c_void_p(out.ctypes.data), cap,
                                        C.c_void_p(off.ctypes.data), C.byref(nb)))
        return out[:nb.value], off[:n]

    def write_host(self, first, n, out, off, threads=1):
        """Events [first, first+n) written straight into out (a uint8 array or view, e.g. a
        pinned slot) with their offsets in off (uint32); threads > 1: ysb_gen_events_host_mt.
        Returns the bytes written."""
        nb = C.c_uint64()
        check(lib().ysb_gen_events_host_mt(C.byref(self.c), first, n, C.c_void_p(out.ctypes.data), out.size,
                                           C.c_void_p(off.ctypes.data), C.byref(nb), max(1, int(threads))))
        return nb.value

    def dump(self, n_events, directory):
        check(lib().ysb_gen_dump(C.byref(self.c), n_events, str(directory).encode()))

    def dump_shards(self, n_events, directory, nranks):
        """Pre-sharded replay files kafka-json.<r>.txt (ad_id-hash routing) + id/map files."""
        check(lib().ysb_gen_dump_shards(C.byref(self.c), n_events, str(directory).encode(), nranks))


def json_to_tbl(raw, offs):
    """Generator-format JSON lines -> the fork's .tbl rows (bytes as uint8 array, u32 offsets)."""
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint32)
    out = np.empty(max(raw.size, 1), dtype=np.uint8)
    oo = np.empty(max(offs.size, 1), dtype=np.uint32)
    nb = C.c_uint64()
    check(lib().ysb_json_to_tbl(C.c_void_p(raw.ctypes.data), raw.size, C.c_void_p(offs.ctypes.data), offs.size,
                                C.c_void_p(out.ctypes.data), out.size, C.c_void_p(oo.ctypes.data), C.byref(nb)))
    return out[:nb.value], oo[:offs.size]


def ad_shard(ad_id, nranks: int) -> int:
    b = ad_id.encode() if isinstance(ad_id, str) else bytes(ad_id)
    return int(lib().ysb_ad_shard(b, len(b), nranks))


def shard_ads(ad_ids, nranks):
    """Ad indices per rank under the ad_id-hash partitioning (include/ysb_hip.h ysb_ad_shard)."""
    out = [[] for _ in range(nranks)]
    for i, a in enumerate(ad_ids):
        out[ad_shard(a, nranks)].append(i)
    return out


def shard_packed(keys, nranks: int, key_len: int = 36):
    """ysb_ad_shard of n keys of key_len bytes packed back to back (a uint8 array), vectorised:
    the library's key_hash (zero-padded little-endian words) and key_shard restated in numpy
    for 10M-ad maps, where one ctypes call per key would take minutes.  Equal to ad_shard
    key by key (tests/test_generator.py)."""
    k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, key_len)
    n = k.shape[0]
    if nranks <= 1:
        return np.zeros(n, dtype=np.uint32)
    nw = (key_len + 3) // 4
    pad = np.zeros((n, 4 * nw), dtype=np.uint8)
    pad[:, :key_len] = k
    w = pad.view("<u4")
    with np.errstate(over="ignore"):
        h = np.full(n, (0x811C9DC5 ^ ((key_len * 0x9E3779B1) & 0xFFFFFFFF)) & 0xFFFFFFFF, dtype=np.uint32)
        for j in range(nw):
            h = (h ^ w[:, j]) * np.uint32(0x01000193)
            h ^= h >> np.uint32(15)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
        z = h.astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (((z >> np.uint64(32)) * np.uint64(nranks)) >> np.uint64(32)).astype(np.uint32)


KEY_ORDER_NAMES = ("user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time", "ip_address")


def layout_of_line(line: bytes, require_ip: bool = False):
    """The layout sampling's decision for one line (ysb_layout_of_line): (layout, key order
    as names or None, compact).  0 the generator's, 1 compact generator order, 2 the
    flat-object tier first, 3 a learned key order."""
    order = np.zeros(8, dtype=np.uint32)
    n, cp = C.c_uint32(), C.c_uint32()
    lay = lib().ysb_layout_of_line(bytes(line), len(line), int(require_ip), C.c_void_p(order.ctypes.data),
                                   C.byref(n), C.byref(cp))
    if lay < 0:
        raise ValueError("bad arguments")
    names = [KEY_ORDER_NAMES[i] for i in order[:n.value]] if lay == 3 else None
    return lay, names, bool(cp.value)
