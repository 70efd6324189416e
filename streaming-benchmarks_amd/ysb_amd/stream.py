"""Streaming mode of the GPU advertising operator (BASELINE configs[4]).

The reference runs the chain record by record inside Flink tasks and flushes window
deltas to Redis from a 1 s timer thread (CampaignProcessorCommon.java:35-55, 91-98).
Here the operator:

  * appends event lines into one of two library-owned pinned slots (zero-copy) and
    submits a slot when it is full or a batch interval (100 ms, the job's
    setBufferTimeout(100), AdvertisingTopologyNative.java:79) has passed; the H2D copy
    and the fused kernel run asynchronously while the other slot fills;
  * tracks an event-time watermark = largest event_time seen - max out-of-orderness
    (the generator's skew is +-50 ms, core.clj:166-174);
  * flushes every flush interval (1 s, as the reference) and whenever the watermark
    passes the end of a window: ysb_drain(clear) -> sink rows (HINCRBY deltas, so late
    events are still counted exactly, as the reference's writeWindow does);
  * records, per window, the close latency = wall time of the flush that first follows
    the window's end under the watermark - window end (bucket_ms + 10 000), the
    quantity get-stats reports as time_updated - window time (core.clj:149), shifted
    to the window end;
  * follows the watermark with the device ring (ysb_ring_advance), keeping a lateness
    horizon (60 s of late events, core.clj:170) on the device.

ShardedStreamingOperator drives N such slot pairs (one context per GPU) with one global
watermark (configs[4]: "feeding double-buffered pinned batches to 8 GPUs").

The context is duck-typed (slot_buffers / submit_raw / wait / sync / drain_rows /
ring_advance / ring_range) so the host logic is testable on CPU with a stand-in.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from ._lib import check, lib

_ET_KEY = b'"event_time": "'


def last_event_time(buf: np.ndarray, start: int, end: int):
    """event_time (ms) of the line buf[start:end], or None: the watermark source, the
    job's timestamp extractor applied to one line per batch."""
    line = buf[start:end].tobytes()
    k = line.rfind(_ET_KEY)
    if k < 0:
        return None
    k += len(_ET_KEY)
    e = line.find(b'"', k)
    try:
        return int(line[k:e])
    except ValueError:
        return None


class SlotContext:
    """Adapter of YsbContext for the operator: zero-copy slot views and row drains."""

    def __init__(self, ctx):
        self.ctx = ctx
        cfg = ctx.cfg
        self.cap_bytes = int(cfg.max_batch_bytes)
        self.cap_events = int(cfg.max_batch_events)
        self.divisor = int(cfg.time_divisor_ms)
        self.W = int(cfg.window_ring)
        self._views = []
        for s in (0, 1):
            b, o = ctx.slot_buffers(s)
            bv = np.ctypeslib.as_array(C.cast(b, C.POINTER(C.c_uint8)), shape=(self.cap_bytes,))
            ov = np.ctypeslib.as_array(C.cast(o, C.POINTER(C.c_uint32)), shape=(self.cap_events,))
            self._views.append((b, o, bv, ov))

    def slot_views(self, slot):
        return self._views[slot]

    def submit_slot(self, slot, nbytes, n):
        b, o, _, _ = self._views[slot]
        check(lib().ysb_submit(self.ctx._h, slot, C.c_void_p(b), nbytes, C.c_void_p(o), n), self.ctx._h)

    def wait(self, slot):
        self.ctx.wait(slot)

    def drain_rows(self):
        """All deltas since the last drain as [(campaign, bucket, count)]."""
        d = self.divisor
        return [(c, w // d, n) for (c, w), n in sorted(self.ctx.drain(clear=True).items())]

    def sync(self):
        self.ctx.sync()

    def ring_range(self):
        try:
            return self.ctx.ring_range()
        except Exception:
            return None

    def ring_advance(self, lo):
        self.ctx.ring_advance(lo)


class WindowBook:
    """Window bookkeeping of a flush: the windows seen, when the watermark closed each
    (close latency), late deltas, and the running totals of everything written."""

    def __init__(self, divisor):
        self.d = divisor
        self.seen_buckets = set()
        self.closed = {}          # bucket -> close latency (ms), None for late-only windows
        self.late_rows = 0        # deltas written for already-closed windows
        self.totals = {}          # (campaign, bucket) -> count, everything written
        self.rows_written = 0
        self.flushed_wm = None    # watermark at the previous flush
        self.first_wm = None      # watermark after the first batch

    def account(self, rows, now, watermark):
        d = self.d
        for c, b, n in rows:
            if b not in self.seen_buckets:
                self.seen_buckets.add(b)
                # first seen after the previous flush's watermark had passed its end:
                # a window of late events only, not a window that closes (no latency)
                ref = self.flushed_wm if self.flushed_wm is not None else self.first_wm
                if ref is not None and (b + 1) * d <= ref:
                    self.closed[b] = None
            if b in self.closed:
                self.late_rows += 1
            self.totals[(c, b)] = self.totals.get((c, b), 0) + n
        self.rows_written += len(rows)
        if watermark is not None:
            self.flushed_wm = watermark
            for b in sorted(self.seen_buckets):
                if b not in self.closed and (b + 1) * d <= watermark:
                    self.closed[b] = now - (b + 1) * d

    def open_windows(self):
        return len([b for b in self.seen_buckets if b not in self.closed])

    def latency_summary(self):
        v = np.array(sorted(x for x in self.closed.values() if x is not None), dtype=np.float64)
        late_only = sum(1 for x in self.closed.values() if x is None)
        if v.size == 0:
            return {"windows": 0, "late_only_windows": late_only}
        return {"windows": int(v.size), "p50_ms": float(np.percentile(v, 50)),
                "p99_ms": float(np.percentile(v, 99)), "max_ms": float(v.max()),
                "late_only_windows": late_only}


class StreamingOperator:
    def __init__(self, sctx, sink=None, batch_interval_ms=100, flush_interval_ms=1000,
                 max_out_of_orderness_ms=100, lateness_horizon_ms=60_000, clock_ms=None,
                 auto_flush=True):
        self.s = sctx
        self.sink = sink
        self.batch_interval_ms = batch_interval_ms
        self.flush_interval_ms = flush_interval_ms
        self.ooo = max_out_of_orderness_ms
        self.horizon_buckets = -(-lateness_horizon_ms // sctx.divisor) + 1
        self.clock = clock_ms or (lambda: time.time() * 1000.0)
        self.auto_flush = auto_flush   # False: a ShardedStreamingOperator flushes the shards
        self.slot = 0
        self.fill_bytes = 0
        self.fill_events = 0
        self.batch_open_ms = None
        self.max_time = None
        self.watermark = None
        self.last_flush_ms = self.clock()
        self.book = WindowBook(sctx.divisor)
        self.events = 0
        self.batches = 0
        self.flushes = 0
        self.open_at_end = 0
        # back-pressure: submits forced by a full slot (before the batch interval), and the
        # time spent waiting for the other slot's H2D before it could be refilled
        self.full_submits = 0
        self.wait_ms = 0.0
        self.wait_max_ms = 0.0

    # the book's fields, as attributes of the operator (reports, tests)
    seen_buckets = property(lambda self: self.book.seen_buckets)
    closed = property(lambda self: self.book.closed)
    late_rows = property(lambda self: self.book.late_rows)
    totals = property(lambda self: self.book.totals)
    rows_written = property(lambda self: self.book.rows_written)

    # -- filling -----------------------------------------------------------------------
    def free_space(self):
        return self.s.cap_bytes - self.fill_bytes, self.s.cap_events - self.fill_events

    def append(self, raw: np.ndarray, offs: np.ndarray):
        """Copies lines into the open slot (submitting full slots as needed)."""
        n, i = offs.size, 0
        while i < n:
            fb, fe = self.free_space()
            # lines [i, j) that fit
            ends = np.append(offs[i + 1:], raw.size).astype(np.int64)
            lens = ends - offs[i:].astype(np.int64)
            cum = np.cumsum(lens)
            j = i + int(min(fe, np.searchsorted(cum, fb, side="right")))
            if j == i:
                if self.fill_events == 0:
                    raise ValueError("line larger than a slot")
                self.submit()
                continue
            self._copy_in(raw, offs, i, j)
            i = j
            if self.fill_events == self.s.cap_events or self.fill_bytes == self.s.cap_bytes:
                self.submit()

    def _copy_in(self, raw, offs, i, j):
        _, _, bv, ov = self.s.slot_views(self.slot)
        if self.fill_events == 0:
            self.batch_open_ms = self.clock()
        a = int(offs[i])
        e = int(offs[j]) if j < offs.size else raw.size
        nb = e - a
        bv[self.fill_bytes:self.fill_bytes + nb] = raw[a:e]
        ov[self.fill_events:self.fill_events + (j - i)] = offs[i:j] - a + self.fill_bytes
        self.fill_bytes += nb
        self.fill_events += j - i

    def fill_with(self, producer):
        """producer(bytes_view, offs_view, cap_bytes, cap_events) -> (nbytes, n): writes lines
        straight into the open slot's pinned memory (zero-copy).  One call per slot."""
        _, _, bv, ov = self.s.slot_views(self.slot)
        if self.fill_events == 0:
            self.batch_open_ms = self.clock()
        fb, fe = self.free_space()
        nb, n = producer(bv[self.fill_bytes:], ov[self.fill_events:], fb, fe)
        if n:
            ov[self.fill_events:self.fill_events + n] += self.fill_bytes
        self.fill_bytes += nb
        self.fill_events += n

    def due(self):
        return self.fill_events > 0 and self.clock() - self.batch_open_ms >= self.batch_interval_ms

    def full(self, line_bytes):
        """The open slot cannot take another line of line_bytes (or another event)."""
        fb, fe = self.free_space()
        return fe == 0 or fb < line_bytes

    def submit_full(self):
        """Submits a slot that filled up before its batch interval (counted as back-pressure)."""
        if self.fill_events:
            self.full_submits += 1
            self.submit()

    # -- submission / watermark --------------------------------------------------------
    def submit(self):
        if self.fill_events == 0:
            return
        _, _, bv, ov = self.s.slot_views(self.slot)
        t = last_event_time(bv, int(ov[self.fill_events - 1]), self.fill_bytes)
        self.s.submit_slot(self.slot, self.fill_bytes, self.fill_events)
        self.events += self.fill_events
        self.batches += 1
        self.slot ^= 1
        t0 = time.perf_counter()
        self.s.wait(self.slot)          # the other slot's H2D is done: it may be refilled
        w = (time.perf_counter() - t0) * 1e3
        self.wait_ms += w
        self.wait_max_ms = max(self.wait_max_ms, w)
        self.fill_bytes = self.fill_events = 0
        if t is not None:
            self.max_time = t if self.max_time is None else max(self.max_time, t)
            wm = self.max_time - self.ooo
            closes = self.watermark is not None and wm // self.s.divisor > self.watermark // self.s.divisor
            if self.watermark is None:
                self.book.first_wm = wm
            self.watermark = wm if self.watermark is None else max(self.watermark, wm)
            if closes and self.auto_flush:
                self.flush()           # a window ended under the watermark: close it now
        if self.auto_flush and self.clock() - self.last_flush_ms >= self.flush_interval_ms:
            self.flush()

    def follow_ring(self, watermark):
        """Moves the device ring behind the watermark, keeping the lateness horizon."""
        rr = self.s.ring_range()
        if rr is not None and watermark is not None:
            target = watermark // self.s.divisor - self.horizon_buckets
            if target > rr[0]:
                self.s.ring_advance(target)

    def flush(self):
        now = self.clock()
        rows = self.s.drain_rows()
        self.flushes += 1
        self.last_flush_ms = now
        self.book.account(rows, now, self.watermark)
        if rows and self.sink is not None:
            self.sink([(c, b * self.s.divisor, n) for c, b, n in rows])
        self.follow_ring(self.watermark)
        return len(rows)

    def close(self):
        """End of input: submit the open slot and flush everything.  Windows the watermark
        has not closed by then are not part of the latency figures (open_at_end)."""
        self.submit()
        self.s.sync()
        self.flush()
        self.open_at_end = self.book.open_windows()

    # -- report ------------------------------------------------------------------------
    def latency_summary(self):
        return self.book.latency_summary()


class ShardedStreamingOperator:
    """configs[4] across GPUs: one double-buffered slot pair and context per GPU (shard),
    events routed by ad_id hash (ysb_route_lines, the keyBy(0) of
    AdvertisingTopologyNative.java:118 applied at the source) or produced per shard, and
    ONE event-time watermark: the minimum over the shards' watermarks (Flink's watermark
    at a keyed operator is the minimum over its input channels), reduced across processes
    by `watermark_reduce` when the shards live in several ranks.  A window closes when the
    global watermark passes its end; every shard then drains its deltas of it, and the
    deltas go to the sink additively (HINCRBY, as parallel CampaignProcessor instances
    write theirs: CampaignProcessorCommon.java:69-89) -- the streaming path needs no count
    exchange.

    Driven by tick(): submit every shard's open slot, reduce the watermark, flush on a
    window close or every `flush_every` ticks (a tick count, so that ranks running in
    lockstep take the same decisions and enter the same collectives)."""

    def __init__(self, sctxs, sink=None, flush_every=10, max_out_of_orderness_ms=100,
                 lateness_horizon_ms=60_000, clock_ms=None, watermark_reduce=None):
        self.clock = clock_ms or (lambda: time.time() * 1000.0)
        self.shards = [StreamingOperator(sc, sink=None, max_out_of_orderness_ms=max_out_of_orderness_ms,
                                         lateness_horizon_ms=lateness_horizon_ms, clock_ms=self.clock,
                                         auto_flush=False) for sc in sctxs]
        self.n = len(self.shards)
        self.d = sctxs[0].divisor
        self.sink = sink
        self.flush_every = flush_every
        self.reduce = watermark_reduce
        self.book = WindowBook(self.d)
        self.watermark = None
        self.ticks = 0
        self.last_flush_tick = 0
        self.flushes = 0
        self.open_at_end = 0

    totals = property(lambda self: self.book.totals)
    events = property(lambda self: sum(s.events for s in self.shards))
    batches = property(lambda self: sum(s.batches for s in self.shards))
    full_submits = property(lambda self: sum(s.full_submits for s in self.shards))
    wait_ms = property(lambda self: sum(s.wait_ms for s in self.shards))
    wait_max_ms = property(lambda self: max(s.wait_max_ms for s in self.shards))

    # -- input ---------------------------------------------------------------------------
    def append(self, raw, offs):
        """Routes a host batch by ad_id hash over the local shards."""
        from .group import route_lines, split_batch
        if self.n == 1:
            self.shards[0].append(raw, offs)
            return
        shard, _ = route_lines(raw, offs, self.n)
        for r in range(self.n):
            br, bo = split_batch(raw, offs, shard, r)
            if bo.size:
                self.shards[r].append(br, bo)

    def append_shard(self, r, raw, offs):
        self.shards[r].append(raw, offs)

    def fill_with(self, r, producer):
        self.shards[r].fill_with(producer)

    # -- watermark / flush ----------------------------------------------------------------
    def local_watermark(self):
        wms = [s.watermark for s in self.shards if s.watermark is not None]
        return min(wms) if len(wms) == self.n else None

    def tick(self):
        for s in self.shards:
            s.submit()
        self.ticks += 1
        wm = self.local_watermark()
        if self.reduce is not None:
            wm = self.reduce(wm)            # min over ranks (None while any rank has none)
        closes = False
        if wm is not None:
            if self.watermark is None:
                self.book.first_wm = wm
            closes = self.watermark is not None and wm // self.d > self.watermark // self.d
            self.watermark = wm if self.watermark is None else max(self.watermark, wm)
        if closes or self.ticks - self.last_flush_tick >= self.flush_every:
            self.flush()

    def flush(self):
        now = self.clock()
        rows = []
        for s in self.shards:
            rows.extend(s.s.drain_rows())
        self.flushes += 1
        self.last_flush_tick = self.ticks
        self.book.account(rows, now, self.watermark)
        if rows and self.sink is not None:
            self.sink([(c, b * self.d, n) for c, b, n in rows])
        for s in self.shards:
            s.follow_ring(self.watermark)
        return len(rows)

    def close(self):
        for s in self.shards:
            s.submit()
            s.s.sync()
        self.flush()
        self.open_at_end = self.book.open_windows()

    def latency_summary(self):
        return self.book.latency_summary()
