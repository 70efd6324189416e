"""GPU: record mode of the window count (ysb_count.hip) -- joined views appended as ring
cell records, partitioned by campaign block and summed in LDS, each touched ring cell
added once -- against the atomic mode and the CPU oracle, including out-of-ring views
(side map), a hot campaign that overflows the record sub-buffers (atomic fallback) and
multi-segment launches."""
import numpy as np
import pytest

from oracle import oracle
from ysb_amd import GenParams, YsbContext

pytestmark = pytest.mark.gpu


def counts(aids, camp, n_campaigns, raw, offs, record, ring=16, segments=1):
    with YsbContext(n_campaigns=n_campaigns, window_ring=ring, record_count=record,
                    max_batch_bytes=raw.size + 64, max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        if segments == 1:
            ctx.submit(raw, offs)
        else:
            d_b = ctx.device_alloc(raw.size + 64 * segments)
            d_o = ctx.device_alloc(4 * offs.size + 64)
            cuts = [int(x) for x in np.linspace(0, offs.size, segments + 1)]
            segs, pos = [], 0
            for a, b in zip(cuts[:-1], cuts[1:]):
                lo = int(offs[a])
                hi = int(offs[b]) if b < offs.size else raw.size
                db = d_b + pos
                ctx.h2d(db, raw[lo:hi])
                ctx.h2d(d_o + 4 * a, (offs[a:b] - lo).astype(np.uint32))
                segs.append((db, hi - lo, d_o + 4 * a, b - a))
                pos += (hi - lo + 15) // 16 * 16
            ctx.submit_device_segments(segs)
        rows = ctx.drain_buckets()
        st = ctx.stats()
        nrec = ctx.path_time()[2]
    return rows, st, nrec


@pytest.fixture(scope="module")
def big_map():
    g = GenParams(seed=11, n_campaigns=200_000, ads_per_campaign=2, events_per_sec=1000, with_skew=True)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 300_000)
    return g, aids, raw, offs


@pytest.mark.timeout(300)
def test_record_mode_equals_atomics_and_oracle(big_map):
    g, aids, raw, offs = big_map
    camp = g.ad_campaign_index()
    exp, est = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    rows_r, st_r, nrec_r = counts(aids, camp, 200_000, raw, offs, record=True)
    rows_a, st_a, nrec_a = counts(aids, camp, 200_000, raw, offs, record=False)
    assert nrec_r == 1 and nrec_a == 0
    assert st_r["out_of_ring"] > 0                      # 30 buckets of event time, a 16-bucket ring
    assert rows_r == exp and rows_a == exp
    for k, v in est.items():
        assert st_r[k] == v and st_a[k] == v, k


@pytest.mark.timeout(300)
def test_record_mode_hot_campaign_overflows_to_atomics(big_map):
    g, aids, raw, offs = big_map
    camp = [7] * len(aids)                               # every view into one campaign: one level-1 bin
    exp, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    rows, _, nrec = counts(aids, camp, 200_000, raw, offs, record=True)
    assert nrec == 1 and rows == exp


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ring", [16, 128])
def test_record_mode_multi_segment_launch(big_map, ring):
    g, aids, raw, offs = big_map
    camp = g.ad_campaign_index()
    exp, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    rows, _, nrec = counts(aids, camp, 200_000, raw, offs, record=True, ring=ring, segments=5)
    assert nrec == 1 and rows == exp


@pytest.mark.timeout(300)
def test_record_mode_flat_tier_lines(big_map):
    """Lines in another key order (the scan's flat tier) counted in record mode: the flat
    tier hands the same key words / time / view flag on, so counts equal the oracle's."""
    g, aids, raw, offs = big_map
    camp = g.ad_campaign_index()
    data = raw.tobytes()
    data = data.replace(b'{"user_id": ', b'{"XXXX_id": ').replace(b', "page_id": ', b', "user_id": ')
    data = data.replace(b'{"XXXX_id": ', b'{"page_id": ')
    raw2 = np.frombuffer(data, dtype=np.uint8)
    exp, est = oracle.run(oracle.AdMap(aids, camp), raw2, offs)
    rows, st, nrec = counts(aids, camp, 200_000, raw2, offs, record=True)
    assert nrec == 1 and rows == exp and st["deferred"] == 0
    for k, v in est.items():
        assert st[k] == v, k


@pytest.fixture(scope="module")
def huge_map():
    g = GenParams(seed=13, n_campaigns=600_000, ads_per_campaign=2, events_per_sec=1000)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 200_000)
    return g, aids, raw, offs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("record", [True, False])
def test_bucket_table_sparse_and_misses(huge_map, record):
    """The HBM-resident (bucket-layout) cuckoo table: 1.2M ads, a tenth of them missing
    from the map (join misses, dropped) and every other remaining key left out of the
    table (as a failed placement would: their views take the general path) -- counts and
    counters equal the oracle's, in record and in atomic mode."""
    g, aids, raw, offs = huge_map
    camp = g.ad_campaign_index()
    keep = [i for i in range(len(aids)) if i % 10 != 3]
    a2, c2 = [aids[i] for i in keep], [camp[i] for i in keep]
    exp, est = oracle.run(oracle.AdMap(a2, c2), raw, offs)
    with YsbContext(n_campaigns=600_000, window_ring=16, record_count=record, sparse_fast_join=True,
                    max_batch_bytes=raw.size + 64, max_batch_events=offs.size + 1, timing=True) as ctx:
        ctx.load_ad_map(a2, c2)
        ctx.submit(raw, offs)
        rows = ctx.drain_buckets()
        st = ctx.stats()
        ctx.kernel_time()
        nrec = ctx.path_time()[2]
    assert nrec == (1 if record else 0)
    assert st["deferred"] > 0 and st["join_misses"] > 0
    assert rows == exp
    for k, v in est.items():
        assert st[k] == v, k


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fold_events", [None, "50000"])
def test_record_delta_ring_folds(big_map, monkeypatch, fold_events):
    """Record mode counts into a saturating u8 delta ring folded into the u64 ring before
    anything reads it.  Eight launches back to back with a stats read and a drain-with-clear
    in between -- with no bound (folds only at the drains) and with the test hook's bound of
    50k events (a fold before every launch) -- equal the oracle."""
    if fold_events:
        monkeypatch.setenv("YSB_DELTA_FOLD_EVENTS", fold_events)
    g, aids, raw, offs = big_map
    camp = g.ad_campaign_index()
    n = offs.size
    cuts = [int(x) for x in np.linspace(0, n, 9)]
    with YsbContext(n_campaigns=200_000, window_ring=16, record_count=True, timing=True,
                    max_batch_bytes=raw.size + 64, max_batch_events=n + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        d_b = ctx.device_alloc(raw.size + 64 * 9)
        d_o = ctx.device_alloc(4 * n + 64)
        chunks, pos = [], 0
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo = int(offs[a])
            hi = int(offs[b]) if b < n else raw.size
            ctx.h2d(d_b + pos, raw[lo:hi])
            ctx.h2d(d_o + 4 * a, (offs[a:b] - lo).astype(np.uint32))
            chunks.append((d_b + pos, hi - lo, d_o + 4 * a, b - a))
            pos += (hi - lo + 15) // 16 * 16
        got = {}

        def add(rows):
            for k, v in rows.items():
                got[k] = got.get(k, 0) + v
        for ch in chunks[:3]:
            ctx.submit_device(*ch)
        assert ctx.stats()["events"] == cuts[3]
        for ch in chunks[3:5]:
            ctx.submit_device(*ch)
        add(ctx.drain_buckets(clear=True))
        for ch in chunks[5:]:
            ctx.submit_device(*ch)
        add(ctx.drain_buckets(clear=True))
        assert ctx.path_time()[2] == 8
    exp, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    assert got == exp


@pytest.mark.timeout(300)
def test_record_delta_saturates_into_u64_ring(big_map):
    """Hot cells: every view in 50 campaigns (~125 views per cell per launch), six launches
    back to back without a read in between -- the u8 delta cells pass 255 within two or three
    launches and hand their sums to the u64 ring (ysb_count.hip add16).  Exact vs six times
    the oracle."""
    g, aids, raw, offs = big_map
    camp = [i % 50 for i in range(len(aids))]
    exp, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    with YsbContext(n_campaigns=200_000, window_ring=16, record_count=True,
                    max_batch_bytes=raw.size + 64, max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
        ctx.h2d(d_b, raw)
        ctx.h2d(d_o, offs)
        for _ in range(6):
            ctx.submit_device(d_b, raw.size, d_o, offs.size)
        rows = ctx.drain_buckets()
        assert ctx.path_time()[2] == 6
    assert max(exp.values()) > 255 // 6 * 2
    assert rows == {k: 6 * v for k, v in exp.items()}
