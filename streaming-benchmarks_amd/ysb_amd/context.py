"""YsbContext: one device context of the GPU advertising operator.

Mirrors the lifecycle of the reference operators it replaces
(flink-benchmarks/.../AdvertisingTopologyNative.java:438-533):
  RedisJoinBolt(Map) / open()         -> YsbContext(...) + load_ad_map(...)
  flatMap(...) per record             -> submit(...) / submit_device(...) per batch
  CampaignProcessorCommon.flushWindows -> drain(...)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import INT64_MIN, YsbConfig, YsbCount, YsbExchangeInfo, YsbLaunchDesc, YsbSegment, YsbStats, check, lib


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else C.c_void_p(0)


def device_count():
    """The HIP devices this process sees (ysb_device_count: hipGetDeviceCount, no framework's
    device query -- a torch build that cannot see the GPU does not change it)."""
    return int(lib().ysb_device_count())


def device_sync(device):
    """hipDeviceSynchronize on `device` through the library's own HIP runtime (ysb_device_sync):
    the bench's device-wide wait without initialising a framework's HIP runtime, which may be
    another one than the library's (ABI 5)."""
    check(lib().ysb_device_sync(int(device)), None)


def rank_device(local_rank, n_visible):
    """The device a rank uses (one context per GPU): its LOCAL_RANK, unless the launcher left
    each process fewer visible devices (e.g. one per rank through HIP_VISIBLE_DEVICES): then
    the (LOCAL_RANK mod n_visible)-th.  With none visible the local rank is kept, so the
    context's open fails loudly instead of silently sharing device 0."""
    if n_visible <= 0:
        return local_rank
    return local_rank if local_rank < n_visible else local_rank % n_visible


class YsbContext:
    def __init__(self, device=0, n_campaigns=100, time_divisor_ms=10000, window_ring=1024,
                 max_batch_events=1 << 20, max_batch_bytes=256 << 20, ring_base_bucket=None,
                 overflow_capacity=1 << 20, timing=False, require_ip=False, lds_count=True,
                 sparse_fast_join=False, input_format="json", record_count=None, compact_first=False,
                 flat_first=False, layout_auto=True, strict=False, h2d_sdma=False):
        L = lib()
        cfg = YsbConfig()
        L.ysb_config_default(C.byref(cfg))
        cfg.time_divisor_ms = time_divisor_ms
        cfg.n_campaigns = n_campaigns
        cfg.window_ring = window_ring
        cfg.max_batch_events = max_batch_events
        cfg.max_batch_bytes = max_batch_bytes
        cfg.ring_base_bucket = INT64_MIN if ring_base_bucket is None else ring_base_bucket
        cfg.overflow_capacity = overflow_capacity
        cfg.flags = ((_lib.YSB_F_TIMING if timing else 0) | (_lib.YSB_F_REQUIRE_IP if require_ip else 0)
                     | (0 if lds_count else _lib.YSB_F_NO_LDS_COUNT)
                     | (_lib.YSB_F_SPARSE_FAST_JOIN if sparse_fast_join else 0)
                 | (_lib.YSB_F_FORMAT_TBL if input_format == "tbl" else 0)
                 | (_lib.YSB_F_COMPACT_FIRST if compact_first else 0)
                 | (_lib.YSB_F_FLAT_FIRST if flat_first else 0)
                 | (0 if layout_auto else _lib.YSB_F_LAYOUT_FIXED)
                 | (_lib.YSB_F_STRICT if strict else 0)
                 | (_lib.YSB_F_H2D_SDMA if h2d_sdma else 0)
                 | (0 if record_count is None else
                    _lib.YSB_F_RECORD_COUNT if record_count else _lib.YSB_F_NO_RECORD_COUNT))
        if input_format not in ("json", "tbl"):
            raise ValueError("input_format must be 'json' or 'tbl'")
        h = C.c_void_p()
        check(L.ysb_open(C.byref(h), device, C.byref(cfg)), None)
        self._h = h
        self.cfg = cfg
        self.device = device

    # -- lifecycle ---------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            lib().ysb_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        return check(rc, self._h)

    # -- join table --------------------------------------------------------------------
    def load_ad_map(self, ad_ids, campaign_idx, shard=None):
        """ad_ids: sequence of str/bytes; campaign_idx: matching campaign indices.

        shard = (rank, nranks): load only the ads of this rank's ad_id-hash shard
        (ysb_load_ad_map_shard) -- the join table sharded 1/N per GPU
        for input that is pre-sharded by the same hash (bench.py's ranks,
        ysb_gen_dump_shards).  The library keeps the shard: a view of another shard's ad
        counts as stats()["foreign_shard"] (an error with strict=True), not as a join miss."""
        keys = [a.encode() if isinstance(a, str) else bytes(a) for a in ad_ids]
        rank, nranks = shard if shard is not None else (0, 1)
        if not 0 <= rank < nranks:
            raise ValueError("shard rank out of range")
        n = len(keys)
        arr = (C.c_char_p * max(n, 1))(*keys)
        lens = (C.c_uint32 * max(n, 1))(*[len(k) for k in keys])
        camp = (C.c_uint32 * max(n, 1))(*[int(c) for c in campaign_idx])
        self._c(lib().ysb_load_ad_map_shard(self._h, arr, lens, camp, n, rank, nranks))

    def load_ad_map_packed(self, keys, campaign_idx, key_len=36, shard=None):
        """keys: uint8 array of n * key_len bytes; campaign_idx: n uint32; shard as load_ad_map."""
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        cidx = np.ascontiguousarray(campaign_idx, dtype=np.uint32)
        if k.size != cidx.size * key_len:
            raise ValueError("keys must hold n * key_len bytes")
        rank, nranks = shard if shard is not None else (0, 1)
        self._c(lib().ysb_load_ad_map_packed_shard(self._h, _ptr(k), key_len, _ptr(cidx), cidx.size, rank, nranks))

    # -- batches -----------------------------------------------------------------------
    def slot_buffers(self, slot):
        b, o = C.c_void_p(), C.c_void_p()
        self._c(lib().ysb_slot_buffers(self._h, slot, C.byref(b), C.byref(o)))
        return b.value, o.value

    def submit(self, data, offsets, slot=0):
        """Host batch (bytes / uint8 array + uint32 line offsets), double-buffered slot."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        self._c(lib().ysb_submit(self._h, slot, _ptr(buf), buf.size, _ptr(off), off.size))

    def wait(self, slot):
        self._c(lib().ysb_wait(self._h, slot))

    def slot_capacity(self):
        """(max_bytes, max_events) of each pinned slot (ysb_slot_capacity)."""
        b, e = C.c_uint64(), C.c_uint64()
        self._c(lib().ysb_slot_capacity(self._h, C.byref(b), C.byref(e)))
        return b.value, e.value

    def submit_raw(self, data, slot=0):
        """Raw batch (ysb_submit_raw): whole lines as bytes, the line starts found on the GPU
        (readLine's terminators); the scan launches at the next call on the context."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        self._c(lib().ysb_submit_raw(self._h, slot, _ptr(buf), buf.size))

    def host_register(self, arr, nbytes=None):
        """ysb_host_register: pins and maps a host numpy array for zero-copy raw batches (the
        array must stay alive and unmoved until host_unregister or close).  nbytes: the length
        to register from arr's start when it is not arr.nbytes (a file mapping's whole pages)."""
        self._c(lib().ysb_host_register(self._h, C.c_void_p(arr.ctypes.data),
                                        arr.nbytes if nbytes is None else int(nbytes)))

    def host_unregister(self, arr):
        self._c(lib().ysb_host_unregister(self._h, C.c_void_p(arr.ctypes.data)))

    def rebase_table(self, time_at, lead_base):
        """ysb_rebase_table: per line (time digits' offset) | (bucket index << 16), uint32."""
        t = np.ascontiguousarray(time_at, dtype=np.uint32)
        self._c(lib().ysb_rebase_table(self._h, _ptr(t), t.size, int(lead_base)))

    def submit_raw_mapped(self, arr, offset, nbytes, slot=0, rebase=None):
        """ysb_submit_raw_mapped: the raw batch arr[offset:offset + nbytes] of a registered
        array, read in place by the device; rebase = (first_line, lead_shift) or None."""
        rb = _lib.YsbRebase(*rebase) if rebase is not None else None
        self._c(lib().ysb_submit_raw_mapped(self._h, slot, C.c_void_p(arr.ctypes.data + offset), nbytes,
                                            C.byref(rb) if rb is not None else None))

    def submit_mapped(self, arr, offset, nbytes, d_off, n, slot=0, rebase=None):
        """ysb_submit_mapped: arr[offset:offset + nbytes] of a registered array with its n line
        offsets already in device memory (d_off); rebase = (first_line, lead_shift) or None."""
        rb = _lib.YsbRebase(*rebase) if rebase is not None else None
        self._c(lib().ysb_submit_mapped(self._h, slot, C.c_void_p(arr.ctypes.data + offset), nbytes,
                                        C.c_void_p(d_off), n, C.byref(rb) if rb is not None else None))

    def split_lines_device(self, d_bytes, nbytes, d_off, cap):
        """ysb_split_lines_device: the line starts of a device batch into d_off; returns n."""
        n = C.c_uint64()
        self._c(lib().ysb_split_lines_device(self._h, C.c_void_p(d_bytes), nbytes, C.c_void_p(d_off), cap,
                                             C.byref(n)))
        return n.value

    def copy_time(self):
        """(total ms, copies, bytes) of the slot H2D copies since the last call (timing=True)."""
        t, k, b = C.c_double(), C.c_uint64(), C.c_uint64()
        self._c(lib().ysb_copy_time(self._h, C.byref(t), C.byref(k), C.byref(b)))
        return t.value, k.value, b.value

    def submit_device(self, d_bytes, nbytes, d_off, n):
        self._c(lib().ysb_submit_device(self._h, C.c_void_p(d_bytes), nbytes, C.c_void_p(d_off), n))

    def submit_device_segments(self, segs):
        """Several device batches [(d_bytes, nbytes, d_off, n), ...] in one kernel launch."""
        arr = (YsbSegment * max(len(segs), 1))()
        for i, (d_b, nb, d_o, n) in enumerate(segs):
            arr[i] = YsbSegment(d_b, nb, d_o, n)
        self._c(lib().ysb_submit_device_segments(self._h, arr, len(segs)))

    def sync(self):
        self._c(lib().ysb_sync(self._h))

    # -- results -----------------------------------------------------------------------
    def drain(self, bucket_lo=INT64_MIN, bucket_hi=(1 << 63) - 1, clear=False):
        """Returns {(campaign, window_ms): count} for buckets in [bucket_lo, bucket_hi)."""
        n = C.c_uint64()
        self._c(lib().ysb_drain(self._h, bucket_lo, bucket_hi, 0, None, 0, C.byref(n)))
        rows = (YsbCount * max(n.value, 1))()
        self._c(lib().ysb_drain(self._h, bucket_lo, bucket_hi, int(clear), rows, n.value, C.byref(n)))
        return {(rows[i].campaign, rows[i].window_ms): rows[i].count for i in range(n.value)}

    def flush_begin(self, bucket_lo=INT64_MIN, bucket_hi=(1 << 63) - 1):
        """ysb_flush_begin: the ring's deltas of [bucket_lo, bucket_hi) compacted behind every
        submitted batch, without waiting."""
        self._c(lib().ysb_flush_begin(self._h, bucket_lo, bucket_hi))

    def flush_end(self, wait=True):
        """The oldest begun flush as ({(campaign, window_ms): count}, more), or None while it is
        pending (wait=False)."""
        n, more = C.c_uint64(), C.c_int()
        rc = lib().ysb_flush_end(self._h, int(wait), None, 0, C.byref(n), C.byref(more))
        if rc == _lib.YSB_PENDING:
            return None
        self._c(rc)
        rows = (YsbCount * max(n.value, 1))()
        self._c(lib().ysb_flush_end(self._h, 1, rows, n.value, C.byref(n), C.byref(more)))
        return {(rows[i].campaign, rows[i].window_ms): rows[i].count for i in range(n.value)}, bool(more.value)

    def drain_buckets(self, **kw):
        """Same as drain() keyed by (campaign, bucket) instead of window_ms."""
        d = self.cfg.time_divisor_ms
        return {(c, w // d): v for (c, w), v in self.drain(**kw).items()}

    def stats(self):
        s = YsbStats()
        self._c(lib().ysb_stats_get(self._h, C.byref(s)))
        return {n: getattr(s, n) for n, _ in YsbStats._fields_}

    def reset(self):
        self._c(lib().ysb_reset(self._h))

    def ring_range(self):
        lo, w = C.c_int64(), C.c_uint32()
        self._c(lib().ysb_ring_range(self._h, C.byref(lo), C.byref(w)))
        return lo.value, w.value

    def ring_advance(self, new_lo):
        """Moves the ring to [new_lo, new_lo + W); leaving buckets go to the exact host list."""
        self._c(lib().ysb_ring_advance(self._h, int(new_lo)))

    def kernel_time(self):
        """(total ms, launches) of the scan kernel since the last call (needs timing=True)."""
        t, k = C.c_double(), C.c_uint64()
        self._c(lib().ysb_kernel_time(self._h, C.byref(t), C.byref(k)))
        return t.value, k.value

    def path_time(self):
        """(total ms, launches, record-mode launches so far): the whole device sequence of
        the launches the last kernel_time() call collected (scan + general path + record
        mode's partition and count kernels)."""
        t, k, r = C.c_double(), C.c_uint64(), C.c_uint64()
        self._c(lib().ysb_path_time(self._h, C.byref(t), C.byref(k), C.byref(r)))
        return t.value, k.value, r.value

    def launch_info(self):
        """The scan instantiation of the last launch: layout (0 generator, 1 compact, 2 flat,
        3 learned order, 4 per-tile dispatch), record_mode, hbm_table, tbl."""
        d = YsbLaunchDesc()
        self._c(lib().ysb_launch_info(self._h, C.byref(d)))
        return {n: getattr(d, n) for n, _ in YsbLaunchDesc._fields_}

    def stream(self):
        s = lib().ysb_stream(self._h)
        if not s:   # a pending raw batch could not launch (sticky until reset)
            raise _lib.YsbError(-3, (lib().ysb_last_error(self._h) or b"").decode())
        return s

    # -- device memory -----------------------------------------------------------------
    def device_alloc(self, nbytes):
        p = C.c_void_p()
        self._c(lib().ysb_device_alloc(self._h, nbytes, C.byref(p)))
        return p.value

    def device_free(self, p):
        self._c(lib().ysb_device_free(self._h, C.c_void_p(p)))

    def h2d(self, d_dst, arr):
        arr = np.ascontiguousarray(arr)
        self._c(lib().ysb_memcpy_h2d(self._h, C.c_void_p(int(d_dst)), _ptr(arr), arr.nbytes))

    def d2h(self, arr, d_src):
        self._c(lib().ysb_memcpy_d2h(self._h, _ptr(arr), C.c_void_p(int(d_src)), arr.nbytes))
        return arr

    # -- multi-GPU ------------------------------------------------------------------------
    @staticmethod
    def group_unique_id() -> bytes:
        buf = C.create_string_buffer(_lib.UNIQUE_ID_BYTES)
        check(lib().ysb_group_unique_id(buf), None)
        return buf.raw

    def group_init(self, rank, nranks, uid: bytes):
        self._c(lib().ysb_group_init(self._h, rank, nranks, C.create_string_buffer(uid, _lib.UNIQUE_ID_BYTES)))

    def group_init_host(self, rank, nranks, dist):
        """ysb_group_init_host over torch.distributed (e.g. gloo) as the transport: the
        library's exchange with the process group's collectives on host memory (N ranks on
        one GPU, where RCCL refuses two ranks per device)."""
        import torch

        def amax(_user, buf, n):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                t = torch.from_numpy((a ^ np.uint64(1 << 63)).view(np.int64).copy())
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                a[:] = t.numpy().view(np.uint64) ^ np.uint64(1 << 63)
                return 0
            except Exception:   # noqa: BLE001 (a failing callback fails the call)
                return 1

        def rsum(_user, send, recv, count, width):
            try:
                cell = {1: np.uint8, 4: np.int32, 8: np.int64}[width]
                nb = count * width
                s_ = np.frombuffer((C.c_char * (nb * nranks)).from_address(send), dtype=cell).copy()
                out = torch.zeros(count, dtype={1: torch.uint8, 4: torch.int32, 8: torch.int64}[width])
                dist.reduce_scatter_tensor(out, torch.from_numpy(s_))
                C.memmove(recv, out.numpy().ctypes.data, nb)
                return 0
            except Exception:   # noqa: BLE001
                return 1
        self._coll = _lib.YsbCollectives(_lib.ALLREDUCE_MAX_FN(amax), _lib.REDUCE_SCATTER_FN(rsum), None)
        self._c(lib().ysb_group_init_host(self._h, rank, nranks, C.byref(self._coll)))

    def group_reduce_scatter(self):
        """The complete exchange: every pending count reaches its owner."""
        self._c(lib().ysb_group_reduce_scatter(self._h))

    def group_exchange_pipelined(self):
        """The streaming exchange (ysb_group_exchange_pipelined): no host wait, packs with the
        previous call's plan; what it leaves pending travels with a later exchange."""
        self._c(lib().ysb_group_exchange_pipelined(self._h))

    def exchange_info(self, reset=False):
        """Exchange accounting (ysb_group_exchange_info): exchanges, bytes, ms, last_buckets,
        last_width, full_ring_bytes, critical_ms, rs_ms, exposed_ms."""
        x = YsbExchangeInfo()
        self._c(lib().ysb_group_exchange_info(self._h, C.byref(x), int(reset)))
        return {n: getattr(x, n) for n, _ in YsbExchangeInfo._fields_}

    def checksum(self, what, nranks=1):
        """Linear table checksums (ysb_group_checksum): what = 'truth' / 'pending' (one per
        owner block of nranks) or 'owned' (this rank's owned table)."""
        code = {"truth": _lib.YSB_SUM_TRUTH_BLOCKS, "pending": _lib.YSB_SUM_PENDING_BLOCKS,
                "owned": _lib.YSB_SUM_OWNED}[what]
        out = np.zeros(max(nranks, 1), dtype=np.uint64)
        self._c(lib().ysb_group_checksum(self._h, code, nranks, _ptr(out)))
        return [int(v) for v in (out[:1] if what == "owned" else out[:nranks])]

    def group_info(self):
        """(rank, nranks) as RCCL's communicator reports them (ncclCommUserRank / ncclCommCount)."""
        r, n = C.c_int(), C.c_int()
        self._c(lib().ysb_group_info(self._h, C.byref(r), C.byref(n)))
        return r.value, n.value

    def group_owned(self):
        lo, hi = C.c_uint32(), C.c_uint32()
        self._c(lib().ysb_group_owned(self._h, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    # -- generator on this device ------------------------------------------------------------
    def gen_events_device(self, params, first, n, d_out, cap, d_off):
        nb = C.c_uint64()
        self._c(lib().ysb_gen_events_device(self._h, C.byref(params.c), first, n, C.c_void_p(d_out), cap,
                                            C.c_void_p(d_off), C.byref(nb)))
        return nb.value

    def truth_accumulate(self, params, first, n):
        self._c(lib().ysb_truth_accumulate(self._h, C.byref(params.c), first, n))

    def truth_read(self):
        """(truth table [n_campaigns][W] uint64, ring base bucket): the generator truth."""
        out = np.zeros((self.cfg.n_campaigns, self.cfg.window_ring), dtype=np.uint64)
        lo = C.c_int64()
        self._c(lib().ysb_truth_read(self._h, _ptr(out), out.size, C.byref(lo)))
        return out, lo.value

    def truth_compare(self):
        m, t, r = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._c(lib().ysb_truth_compare(self._h, C.byref(m), C.byref(t), C.byref(r)))
        return m.value, t.value, r.value
