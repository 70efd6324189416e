"""Streaming operator host logic (ysb_amd/stream.py) on CPU: slot filling, batch
submission, the event-time watermark, window close + latency, late deltas, ring
following.  The device is replaced by a stand-in that counts each submitted slot
with the CPU oracle (test infrastructure); the GPU version of the same stream is in
tests/test_gpu_stream.py."""
import numpy as np
import pytest

import golden_data as gd
from oracle import oracle
from ysb_amd import GenParams
from ysb_amd.stream import StreamingOperator, last_event_time


class OracleSlots:
    """Duck-typed SlotContext: two host slots; submit counts the slot with the oracle."""

    def __init__(self, admap, cap_bytes, cap_events, divisor=10000, W=16):
        self.am = admap
        self.cap_bytes, self.cap_events, self.divisor, self.W = cap_bytes, cap_events, divisor, W
        self.views = [(0, 0, np.zeros(cap_bytes, np.uint8), np.zeros(cap_events, np.uint32)) for _ in range(2)]
        self.pending = {}
        self.ring = None
        self.advances = []
        self.submits = []

    def slot_views(self, slot):
        return self.views[slot]

    def submit_slot(self, slot, nbytes, n):
        _, _, bv, ov = self.views[slot]
        rows, _ = oracle.run(self.am, bv[:nbytes].tobytes(), ov[:n].copy())
        for k, v in rows.items():
            self.pending[k] = self.pending.get(k, 0) + v
        self.submits.append((slot, nbytes, n))
        if self.ring is None and rows:
            self.ring = min(b for _, b in rows) - self.W // 8

    def wait(self, slot):
        pass

    def sync(self):
        pass

    def drain_rows(self):
        out = sorted((c, b, n) for (c, b), n in self.pending.items())
        self.pending = {}
        return out

    def ring_range(self):
        return None if self.ring is None else (self.ring, self.W)

    def ring_advance(self, lo):
        self.advances.append(lo)
        self.ring = lo


class Clock:
    def __init__(self, t=0.0):
        self.t = t

    def __call__(self):
        return self.t


def admap_gen(g):
    _, aids = g.ids()
    return oracle.AdMap(aids, g.ad_campaign_index())


def test_last_event_time():
    line = b'{"user_id": "a", "event_time": "1700000012345", "ip_address": "1.2.3.4"}\n'
    buf = np.frombuffer(b"xx" + line, dtype=np.uint8)
    assert last_event_time(buf, 2, buf.size) == 1700000012345
    assert last_event_time(np.frombuffer(b'{"a": "b"}', dtype=np.uint8), 0, 10) is None


def test_fixture_through_small_slots_is_exact():
    ads, camp = gd.ad_arrays()
    raw, offs = gd.events("gen_s7")
    slots = OracleSlots(oracle.AdMap(ads, camp), cap_bytes=4096, cap_events=12)
    written = []
    op = StreamingOperator(slots, sink=written.extend, clock_ms=Clock())
    op.append(np.frombuffer(raw, dtype=np.uint8), np.asarray(offs, dtype=np.uint32))
    op.close()
    exp, _ = gd.expected("gen_s7")
    assert op.totals == exp
    assert op.events == len(offs)
    assert all(n <= 12 for _, _, n in slots.submits) and all(b <= 4096 for _, b, _ in slots.submits)
    # sink rows are (campaign, window_ms, delta); their sum is the expected table
    tot = {}
    for c, w, n in written:
        tot[(c, w // 10000)] = tot.get((c, w // 10000), 0) + n
    assert tot == exp


def test_watermark_closes_windows_with_latency_and_late_deltas():
    g = GenParams(seed=11, n_campaigns=10, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  t0_ms=1_700_000_000_000)
    raw, offs = g.events_host(0, 60_000)      # 60 s of event time at 1000 ev/s
    clk = Clock(1_700_000_000_000.0)
    slots = OracleSlots(admap_gen(g), cap_bytes=1 << 20, cap_events=1000)
    op = StreamingOperator(slots, clock_ms=clk, batch_interval_ms=100, lateness_horizon_ms=20_000)
    # real-time replay: 100 ms of events per batch, the clock 5 ms past the batch's end
    per = 100
    for i in range(0, offs.size, per):
        j = min(offs.size, i + per)
        clk.t = 1_700_000_000_000 + (j * 1000) / 1000 + 5
        e = offs[j] if j < offs.size else raw.size
        op.append(raw[offs[i]:e], (offs[i:j] - offs[i]).astype(np.uint32))
        op.submit()
    # a late event for the first window, after it closed
    k = next(i for i in range(offs.size) if b'"event_type": "view"' in raw[offs[i]:offs[i + 1]].tobytes())
    late = raw[offs[k]:offs[k + 1]].tobytes()
    op.append(np.frombuffer(late, dtype=np.uint8), np.zeros(1, np.uint32))
    op.close()
    ref, _ = oracle.run(admap_gen(g), np.concatenate([raw, np.frombuffer(late, np.uint8)]),
                        np.append(offs, raw.size).astype(np.uint32))
    assert op.totals == ref
    lat = op.latency_summary()
    assert lat["windows"] >= 5
    # windows close on the first submit past their end (+ out-of-orderness), not on the 1 s timer
    assert 0 <= lat["p50_ms"] <= 100 + 5 + op.ooo
    assert op.late_rows >= 1
    # the ring followed the watermark, keeping the horizon behind it
    assert slots.advances and slots.advances == sorted(slots.advances)
    assert slots.advances[-1] <= op.watermark // 10000 - op.horizon_buckets


def test_flush_timer_without_window_close():
    ads, camp = gd.ad_arrays()
    raw, offs = gd.events("gen_s7")
    clk = Clock(0.0)
    slots = OracleSlots(oracle.AdMap(ads, camp), cap_bytes=1 << 20, cap_events=1 << 12)
    written = []
    op = StreamingOperator(slots, sink=written.extend, clock_ms=clk, flush_interval_ms=1000,
                           max_out_of_orderness_ms=10**9)    # watermark never closes a window
    a = np.frombuffer(raw, dtype=np.uint8)
    o = np.asarray(offs, dtype=np.uint32)
    op.append(a[:o[10]], o[:10])
    op.submit()
    assert op.flushes == 0 and not written
    clk.t = 1500.0
    op.append(a[o[10]:o[20]], o[10:20] - o[10])
    op.submit()
    assert op.flushes == 1 and written


def test_line_larger_than_slot_is_an_error():
    ads, camp = gd.ad_arrays()
    raw, offs = gd.events("gen_s7")
    op = StreamingOperator(OracleSlots(oracle.AdMap(ads, camp), cap_bytes=64, cap_events=4), clock_ms=Clock())
    with pytest.raises(ValueError):
        op.append(np.frombuffer(raw, dtype=np.uint8), np.asarray(offs, dtype=np.uint32))


def test_sharded_streaming_operators_share_one_redis():
    """configs[4] across GPUs: one operator per rank on its ad_id shard of the stream
    (ysb_route_lines); their HINCRBY deltas meet in one Redis, exactly as the reference's
    parallel CampaignProcessor instances' do -- no exchange needed on the streaming path."""
    from fake_redis import FakeRedis
    from ysb_amd import route_lines, split_batch
    from ysb_amd.redis_sink import RedisWindowWriter, RespClient, check_correct
    g = GenParams(seed=23, n_campaigns=10, ads_per_campaign=10, events_per_sec=2000, with_skew=True,
                  t0_ms=1_700_000_000_000)
    raw, offs = g.events_host(0, 60_000)
    camps, aids = g.ids()
    shard, _ = route_lines(raw, offs, 3)
    srv = FakeRedis()
    try:
        for r in range(3):
            br, bo = split_batch(raw, offs, shard, r)
            cli = RespClient("127.0.0.1", srv.port)
            writer = RedisWindowWriter(cli, camps, clock_ms=lambda: 0)
            op = StreamingOperator(OracleSlots(admap_gen(g), cap_bytes=1 << 18, cap_events=700),
                                   sink=writer.write, clock_ms=Clock(1_700_000_000_000.0))
            op.append(br, bo)
            op.close()
            cli.close()
        ref, _ = oracle.run(admap_gen(g), raw, offs)
        expected = {}
        for (c, b), n in ref.items():
            expected.setdefault(camps[c], {})[b] = n
        cli = RespClient("127.0.0.1", srv.port)
        res = check_correct(cli, expected)
        cli.close()
        assert res and all(s == "CORRECT" for _, _, s, _ in res)
    finally:
        srv.close()


def test_sharded_operator_global_watermark_exact():
    """configs[4] host logic across 3 shards in one process: lines routed by ad_id hash,
    one watermark = the minimum over the shards, windows closed on it, deltas additive."""
    from ysb_amd.stream import ShardedStreamingOperator
    g = GenParams(seed=31, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  t0_ms=1_700_000_000_000)
    raw, offs = g.events_host(0, 45_000)               # 45 s of event time
    clk = Clock(1_700_000_000_000.0)
    shards = [OracleSlots(admap_gen(g), cap_bytes=1 << 18, cap_events=400) for _ in range(3)]
    written = []
    op = ShardedStreamingOperator(shards, sink=written.extend, clock_ms=clk, flush_every=10,
                                  lateness_horizon_ms=20_000)
    per = 100                                           # 100 ms of events per tick
    for i in range(0, offs.size, per):
        j = min(offs.size, i + per)
        clk.t = 1_700_000_000_000 + j + 5
        e = offs[j] if j < offs.size else raw.size
        op.append(raw[offs[i]:e], (offs[i:j] - offs[i]).astype(np.uint32))
        op.tick()
    op.close()
    ref, _ = oracle.run(admap_gen(g), raw, offs)
    assert op.totals == ref
    tot = {}
    for c, w, n in written:
        tot[(c, w // 10000)] = tot.get((c, w // 10000), 0) + n
    assert tot == ref
    assert all(s.events > 0 for s in op.shards) and op.events == offs.size
    lat = op.latency_summary()
    assert lat["windows"] >= 3 and 0 <= lat["p50_ms"] <= 100 + 5 + 100
    # every shard's ring follows the one global watermark
    assert all(s.advances and s.advances[-1] <= op.watermark // 10000 - op.shards[0].horizon_buckets
               for s in shards)


def test_sharded_operator_waits_for_every_shard():
    """The global watermark is the minimum: a shard without data holds every window open."""
    from ysb_amd.stream import ShardedStreamingOperator
    g = GenParams(seed=31, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000, t0_ms=1_700_000_000_000)
    raw, offs = g.events_host(0, 30_000)
    shards = [OracleSlots(admap_gen(g), cap_bytes=1 << 20, cap_events=4000) for _ in range(2)]
    op = ShardedStreamingOperator(shards, clock_ms=Clock(0.0), flush_every=1000)
    op.append_shard(0, raw, offs)
    op.tick()
    assert op.watermark is None and op.latency_summary()["windows"] == 0
    op.append_shard(1, raw[:offs[1]], offs[:1])       # shard 1's first event: t0
    op.tick()
    assert op.watermark == 1_700_000_000_000 - 100
