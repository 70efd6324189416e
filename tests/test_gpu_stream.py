"""GPU: device-side drain compaction, ring advance, the streaming operator end to end
(pinned double-buffered slots -> H2D -> fused kernel -> watermark close), and
config 3's large tables (1M campaigns / 10M ads), all checked exactly against the
CPU oracle or the generator truth."""
import numpy as np
import pytest

from oracle import oracle
from ysb_amd import YsbError, GenParams, YsbContext
from ysb_amd.stream import SlotContext, StreamingOperator

pytestmark = pytest.mark.gpu


def oracle_rows(g, raw, offs):
    _, aids = g.ids()
    return oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs)


def test_drain_compaction_and_ring_advance_exact():
    g = GenParams(seed=21, n_campaigns=30, ads_per_campaign=10, events_per_sec=2000, with_skew=True)
    raw, offs = g.events_host(0, 120_000)            # 60 s of event time: 7 buckets
    rows, _ = oracle_rows(g, raw, offs)
    _, aids = g.ids()
    with YsbContext(n_campaigns=30, window_ring=16, max_batch_bytes=64 << 20, max_batch_events=1 << 18) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        half = offs.size // 2
        ctx.submit(raw[:offs[half]], offs[:half])
        lo, W = ctx.ring_range()
        # not clearing: the whole table twice, identical
        a = ctx.drain_buckets()
        assert a == ctx.drain_buckets()
        # move the ring forward over the first buckets: their counts go to the host list
        ctx.ring_advance(lo + 3)
        assert ctx.ring_range() == (lo + 3, W)
        ctx.submit(raw[offs[half]:], offs[half:] - offs[half], slot=1)
        got = ctx.drain_buckets()
        assert got == rows
        # range drains with clear: disjoint, and together everything
        b0 = min(b for _, b in rows)
        first = ctx.drain_buckets(bucket_lo=b0, bucket_hi=b0 + 2, clear=True)
        rest = ctx.drain_buckets(clear=True)
        assert set(first) | set(rest) == set(rows) and not (set(first) & set(rest))
        assert ctx.drain_buckets() == {}
        # backwards too
        ctx.ring_advance(lo - 20)
        assert ctx.ring_range() == (lo - 20, W)


def test_streaming_operator_end_to_end_exact():
    g = GenParams(seed=5, n_campaigns=100, ads_per_campaign=10, events_per_sec=20_000, with_skew=True,
                  n_users=100, t0_ms=1_700_000_000_000)
    n = 600_000                                          # 30 s of event time
    _, aids = g.ids()
    clock = {"t": 1_700_000_000_000.0}
    with YsbContext(n_campaigns=100, window_ring=16, max_batch_bytes=2 << 20, max_batch_events=4096) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        sctx = SlotContext(ctx)
        written = []
        op = StreamingOperator(sctx, sink=written.extend, clock_ms=lambda: clock["t"],
                               lateness_horizon_ms=20_000)
        first = 0

        def produce(bv, ov, cap_b, cap_e):
            m = min(cap_e, n - first, cap_b // g.max_line_bytes())
            raw, offs = g.events_host(first, m)
            bv[:raw.size] = raw
            ov[:m] = offs
            return raw.size, m

        while first < n:
            op.fill_with(produce)
            first = op.events + op.fill_events
            clock["t"] = 1_700_000_000_000 + first * 1000 / 20_000 + 3   # real time follows event time
            op.submit()
        op.close()
        raw, offs = g.events_host(0, n)
        rows, st = oracle_rows(g, raw, offs)
        assert op.totals == rows
        s = ctx.stats()
        assert s["events"] == n and s["parse_errors"] == 0 and s["joined"] == st["joined"]
        lat = op.latency_summary()
        assert lat["windows"] >= 2 and lat["p99_ms"] < 1000
        lo, _ = ctx.ring_range()
        assert lo > min(b for _, b in rows)              # the ring followed the watermark
        tot = {}
        for c, w, k in written:
            tot[(c, w // 10000)] = tot.get((c, w // 10000), 0) + k
        assert tot == rows


@pytest.mark.timeout(400)
def test_config3_large_tables_truth():
    """1M campaigns x 10 ads: the join table and the count table live in HBM (no LDS
    counters); full-table truth comparison on 4M generated events."""
    g = GenParams(seed=42, n_campaigns=1_000_000, ads_per_campaign=10, events_per_sec=100_000)
    _, ab = g.ids_packed()
    with YsbContext(n_campaigns=1_000_000, window_ring=16, max_batch_bytes=1 << 20,
                    max_batch_events=1 << 12) as ctx:
        ctx.load_ad_map_packed(ab, g.ad_campaign_index_array())
        n = 4_000_000
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        ctx.submit_device(d_b, nb, d_o, n)
        ctx.truth_accumulate(g, 0, n)
        mism, truth, ring = ctx.truth_compare()
        st = ctx.stats()
        assert mism == 0 and truth == ring and st["join_misses"] == 0 and st["parse_errors"] == 0
        assert st["joined"] == st["views"] and st["views"] > n // 4
        assert ctx.path_time()[2] == 1                   # counted in record mode (ysb_count.hip)
        rows = ctx.drain_buckets()
        assert sum(rows.values()) == truth
        # the first 20k events also through the CPU oracle, with the map entries they use
        off = ctx.d2h(np.empty(n, dtype=np.uint32), d_o)
        m = 20_000
        raw = ctx.d2h(np.empty(int(off[m]), dtype=np.uint8), d_b)
        keys = ab.view("S36")
        order = np.argsort(keys, kind="stable")
        sk = keys[order]
        used = np.unique(np.array([raw[off[i] + 113:off[i] + 149].tobytes() for i in range(m)], dtype="S36"))
        pos = np.searchsorted(sk, used)
        assert (sk[pos] == used).all()
        camp = (order[pos] // 10).astype(np.uint32)
        exp, _ = oracle.run(oracle.AdMap([u.decode() for u in used], camp), raw, off[:m])
        ctx.reset()                                      # keeps the 10M-entry table
        ctx.submit_device(d_b, int(off[m]), d_o, m)
        assert ctx.drain_buckets() == exp


def test_out_of_ring_cells_exact_through_side_map():
    # 60 s per 1000 events at 100 ev/s: 80k events span 80 buckets, the ring holds 16
    g = GenParams(seed=9, n_campaigns=40, ads_per_campaign=5, events_per_sec=100, with_skew=True)
    raw, offs = g.events_host(0, 80_000)
    rows, st = oracle_rows(g, raw, offs)
    _, aids = g.ids()
    with YsbContext(n_campaigns=40, window_ring=16, max_batch_bytes=64 << 20, max_batch_events=1 << 18) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(raw, offs)
        s = ctx.stats()
        assert s["out_of_ring"] > 0 and s["overflow_dropped"] == 0
        assert ctx.drain_buckets() == rows
        # twice through (the map was emptied by the drain pull; counts accumulate again)
        ctx.submit(raw, offs, slot=1)
        ctx.submit(raw, offs, slot=0)
        assert ctx.drain_buckets() == {k: 3 * v for k, v in rows.items()}


def test_side_capacity_exhaustion_is_reported():
    """Counts the device could not place (map AND fallback list full within one launch)
    fail ysb_sync / ysb_drain with YSB_ERR_CAPACITY until ysb_reset: never silent."""
    g = GenParams(seed=9, n_campaigns=40, ads_per_campaign=5, events_per_sec=100)
    raw, offs = g.events_host(0, 80_000)
    _, aids = g.ids()
    with YsbContext(n_campaigns=40, window_ring=16, overflow_capacity=16, max_batch_bytes=64 << 20,
                    max_batch_events=1 << 18) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(raw, offs)
        with pytest.raises(YsbError) as e:
            ctx.sync()
        assert e.value.code == -4 and "lost" in str(e.value)
        with pytest.raises(YsbError) as e:
            ctx.drain()
        assert e.value.code == -4
        assert ctx.stats()["overflow_dropped"] > 0       # the stats stay readable
        ctx.reset()
        ctx.sync()                                       # cleared by the reset


def test_side_map_spills_to_host_between_launches():
    """A small out-of-ring map never fills across batches: ysb_sync empties it into the
    exact host list once a quarter full, so many small batches stay exact."""
    g = GenParams(seed=9, n_campaigns=40, ads_per_campaign=5, events_per_sec=100, with_skew=True)
    raw, offs = g.events_host(0, 80_000)
    rows, _ = oracle_rows(g, raw, offs)
    _, aids = g.ids()
    with YsbContext(n_campaigns=40, window_ring=16, overflow_capacity=512, max_batch_bytes=64 << 20,
                    max_batch_events=1 << 18) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        step = 2000
        for i in range(0, offs.size, step):
            j = min(i + step, offs.size)
            end = int(offs[j]) if j < offs.size else raw.size
            ctx.submit(raw[offs[i]:end], offs[i:j] - offs[i], slot=(i // step) & 1)
            ctx.sync()
        assert ctx.stats()["overflow_dropped"] == 0
        assert ctx.drain_buckets() == rows


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4])
def test_sharded_streaming_n_contexts_exact(n):
    """configs[4] rehearsal on one GPU: n contexts (one per would-be GPU), each with its
    own pinned double-buffered slots fed by its ad_id shard's event stream (skew and late
    events), one global watermark; the deltas equal the CPU oracle's counts over every
    event the producers made (oracle/ysb_oracle.c: an independent restatement, not the
    HIP batch path)."""
    from ysb_amd import shard_ads
    from ysb_amd.stream import ShardedStreamingOperator
    base = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
    _, aids = base.ids()
    subsets = shard_ads(aids, n)
    gens = [GenParams(seed=42, event_stream=1 + r, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000,
                      ad_subset=subsets[r], with_skew=True, n_users=100, t0_ms=1_700_000_000_000)
            for r in range(n)]
    per_tick, ticks = 2000, 600                      # 20 ms of event time per tick, 12 s
    ctxs = [YsbContext(n_campaigns=100, window_ring=16, max_batch_bytes=per_tick * 300,
                       max_batch_events=per_tick * 2) for _ in range(n)]
    for c in ctxs:
        c.load_ad_map(aids, base.ad_campaign_index())
    clk = [1_700_000_000_000.0]
    op = ShardedStreamingOperator([SlotContext(c) for c in ctxs], clock_ms=lambda: clk[0], flush_every=50)
    produced = [0] * n

    def producer(r):
        def fill(bv, ov, cap_b, cap_e):
            raw, offs = gens[r].events_host(produced[r], per_tick)
            bv[:raw.size] = raw
            ov[:per_tick] = offs
            produced[r] += per_tick
            return raw.size, per_tick
        return fill
    for t in range(ticks):
        clk[0] = 1_700_000_000_000 + (t + 1) * 20 + 5
        for r in range(n):
            op.fill_with(r, producer(r))
        op.tick()
    op.close()
    from oracle import oracle
    am = oracle.AdMap(aids, base.ad_campaign_index())
    ref = {}
    for r in range(n):
        raw, offs = gens[r].events_host(0, produced[r])
        rows, _ = oracle.run(am, raw, offs)
        for k, v in rows.items():
            ref[k] = ref.get(k, 0) + v
    for c in ctxs:
        c.close()
    assert op.totals == ref
    assert op.events == n * per_tick * ticks
    lat = op.latency_summary()
    assert lat["windows"] >= 1 and lat["p99_ms"] < 1000


def test_async_flushes_sum_to_the_drain_without_stopping_the_stream():
    """ysb_flush_begin / ysb_flush_end (ABI 4): a flush begun after each of 8 device batches
    submitted back to back, taken without waiting where it is done and in order otherwise, plus
    one final drain, equal the C oracle's counts exactly -- each delta in exactly one flush or
    the drain; at most 4 flushes outstanding; a pending flush reports YSB_PENDING, not an error."""
    import numpy as np
    from oracle import oracle
    from ysb_amd import YsbError
    g = GenParams(seed=61, events_per_sec=20_000)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    n, parts = 400_000, 8
    raw, offs = g.events_host(0, n)
    rows, ost = oracle.run(oracle.AdMap(aids, camp), raw, offs, threads=8)
    ends = [int(x) for x in offs] + [int(raw.size)]
    got, flushes = {}, []
    with YsbContext(device=0, n_campaigns=100, window_ring=64) as ctx:
        ctx.load_ad_map(aids, camp)
        bufs = []
        for p in range(parts):
            a, b = p * n // parts, (p + 1) * n // parts
            piece = raw[ends[a]:ends[b]]
            d_b, d_o = ctx.device_alloc(piece.size + 64), ctx.device_alloc(4 * (b - a) + 64)
            ctx.h2d(d_b, piece)
            ctx.h2d(d_o, (np.asarray(ends[a:b], dtype=np.int64) - ends[a]).astype(np.uint32))
            bufs.append((d_b, int(piece.size), d_o, b - a))
        ctx.sync()

        def take(wait):
            r = ctx.flush_end(wait=wait)
            if r is None:
                return False
            assert not r[1]
            flushes.append(len(r[0]))
            for k, v in r[0].items():
                got[k] = got.get(k, 0) + v
            return True
        pending = 0
        for d_b, nb, d_o, m in bufs:
            ctx.submit_device(d_b, nb, d_o, m)
            ctx.flush_begin()
            pending += 1
            if pending == 4:
                with pytest.raises(YsbError):
                    ctx.flush_begin()
                assert take(True)
                pending -= 1
            while pending and take(False):
                pending -= 1
        while pending:
            assert take(True)
            pending -= 1
        for k, v in ctx.drain(clear=True).items():
            got[k] = got.get(k, 0) + v
        st = ctx.stats()
        for d_b, _, d_o, _ in bufs:
            ctx.device_free(d_b)
            ctx.device_free(d_o)
    assert len(flushes) == parts and sum(flushes) > 0
    assert {(c, w // 10000): v for (c, w), v in got.items()} == rows
    for k, v in ost.items():
        assert st[k] == v, (k, st[k], v)


def test_async_flush_over_its_row_cap_leaves_the_rest_for_the_next():
    """A flush holds at most 2^20 rows (ysb_flush_begin): 200k campaigns x ~7 windows of views
    (~1.3M nonzero cells; record mode, its u8 delta ring folded in first) need two flushes --
    the first returns 2^20 rows with more = 1 and keeps the rest on the device, the second
    returns them with more = 0; together they equal the generator truth exactly, and nothing
    is left for a drain."""
    from ysb_amd.group import table_rows
    C, W, n = 200_000, 16, 12_000_000
    g = GenParams(seed=67, n_campaigns=C, ads_per_campaign=10, events_per_sec=n // 65)
    _, ab = g.ids_packed()
    with YsbContext(device=0, n_campaigns=C, window_ring=W, ring_base_bucket=g.c.t0_ms // 10000 - 8,
                    max_batch_bytes=1 << 20, max_batch_events=1 << 12) as ctx:
        ctx.load_ad_map_packed(ab, g.ad_campaign_index_array())
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        ctx.submit_device(d_b, nb, d_o, n)
        ctx.truth_accumulate(g, 0, n)
        truth, lo = ctx.truth_read()
        want = {(c, b * 10000): v for (c, b), v in table_rows(truth, lo).items()}
        assert len(want) > (1 << 20), len(want)
        ctx.flush_begin()
        first, more = ctx.flush_end(wait=True)
        assert more and len(first) == 1 << 20
        ctx.flush_begin()
        second, more2 = ctx.flush_end(wait=True)
        assert not more2 and len(first) + len(second) == len(want)
        assert not (set(first) & set(second))
        got = dict(first)
        got.update(second)
        assert got == want
        assert ctx.drain(clear=True) == {}
        ctx.device_free(d_b)
        ctx.device_free(d_o)
