"""GPU parity of ysb_submit_device_segments (several batches, one scan launch): the same
counts and counters as the golden fixtures, the C oracle and batch-by-batch submits --
including deferred lines in later segments (the general path maps each deferred line
back to its segment) and empty / ragged segments."""
import numpy as np
import pytest

import golden_data as gd
from oracle import oracle
from ysb_amd import GenParams, YsbError
from test_gpu_parity import check_against, make_ctx, split_batches

pytestmark = pytest.mark.gpu

RAGGED = [1, 0, 63, 64, 65, 127, 300, 2, 0, 129]   # tile-unaligned, empty, tiny segments


def upload_segments(ctx, raw, offs, sizes):
    segs, bufs = [], []
    for b, o in split_batches(raw, offs, sizes):
        d_b = ctx.device_alloc(len(b) + 64)
        d_o = ctx.device_alloc(4 * len(o) + 64)
        if len(b):
            ctx.h2d(d_b, np.frombuffer(b, dtype=np.uint8))
        if len(o):
            ctx.h2d(d_o, np.asarray(o, dtype=np.uint32))
        segs.append((d_b, len(b), d_o, len(o)))
        bufs += [d_b, d_o]
    return segs, bufs


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
@pytest.mark.parametrize("sparse", [False, True])
def test_fixture_segments(stem, require_ip, sparse):
    raw, offs = gd.events(stem)
    with make_ctx(require_ip=require_ip, sparse_fast_join=sparse) as ctx:
        segs, bufs = upload_segments(ctx, raw, offs, RAGGED)
        assert len(segs) <= 16
        ctx.submit_device_segments(segs)
        check_against(ctx, *gd.expected(stem, require_ip))
        for d in bufs:
            ctx.device_free(d)


@pytest.mark.parametrize("seed", [1, 2])
def test_orgjson_fuzz_segments_match_oracle(seed):
    """The org.json fuzz corpus (mostly general-path lines) in 7 segments."""
    import orgjson_fuzz as fz
    ads, camp = gd.ad_arrays()
    lines = fz.lines(seed, 3000, ads)
    raw = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).tolist()
    rows, ost = oracle.run(oracle.AdMap(ads, camp), raw, offs)
    with make_ctx(ads=(ads, camp)) as ctx:
        segs, _ = upload_segments(ctx, raw, offs, [500, 1, 700, 0, 333, 1000])
        ctx.submit_device_segments(segs)
        st = ctx.stats()
        assert st["deferred"] > 0
        for k, v in ost.items():
            assert st[k] == v, (k, st[k], v)
        assert ctx.drain_buckets() == rows


def test_generated_segments_equal_per_batch_and_oracle():
    """1.5M generated events in 6 unequal device batches (skewed, late events, 50 ads
    missing from the map, a ring of 16 buckets): one launch == six launches == oracle."""
    g = GenParams(seed=4321, events_per_sec=1000, with_skew=True)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    sizes = [400_000, 1, 250_000, 64 * 1001, 300_000, 485_935]
    results = []
    for mode in ("segments", "per_batch"):
        with make_ctx(n_campaigns=100, ads=(aids[:950], camp[:950]), window_ring=16,
                      overflow_capacity=1 << 22) as ctx:
            segs, first = [], 0
            for n in sizes:
                cap = n * g.max_line_bytes() + 64
                d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
                nb = ctx.gen_events_device(g, first, n, d_b, cap, d_o)
                segs.append((d_b, nb, d_o, n))
                first += n
            if mode == "segments":
                ctx.submit_device_segments(segs)
            else:
                for s in segs:
                    ctx.submit_device(*s)
            st = ctx.stats()
            results.append((ctx.drain_buckets(), st))
            if mode == "segments":
                data = [ctx.d2h(np.empty(nb, dtype=np.uint8), d_b) for (d_b, nb, _, _) in segs]
                offs = [ctx.d2h(np.empty(n, dtype=np.uint32), d_o) for (_, _, d_o, n) in segs]
    (rows_s, st_s), (rows_b, st_b) = results
    assert rows_s == rows_b and st_s == st_b
    assert st_s["events"] == sum(sizes) and st_s["join_misses"] > 0 and st_s["out_of_ring"] > 0
    # oracle on the concatenated batches
    base = np.cumsum([0] + [len(d) for d in data[:-1]])
    all_off = np.concatenate([o.astype(np.uint64) + b for o, b in zip(offs, base)])
    rows, ost = oracle.run(oracle.AdMap(aids[:950], camp[:950]), np.concatenate(data), all_off, threads=8)
    for k, v in ost.items():
        assert st_s[k] == v, (k, st_s[k], v)
    assert rows_s == rows


def test_segments_truth_at_scale():
    """30M events as two 15M-event (3.8 GB) segments in one launch: byte offsets past
    2^31 in both, counts == generator truth."""
    g = GenParams(seed=77, events_per_sec=100_000)
    n, seg = 30_000_000, 15_000_000
    with make_ctx(n_campaigns=100, ads=(g.ids()[1], g.ad_campaign_index())) as ctx:
        cap = seg * g.max_line_bytes()
        segs = []
        for first in range(0, n, seg):
            d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * seg)
            nb = ctx.gen_events_device(g, first, seg, d_b, cap, d_o)
            segs.append((d_b, nb, d_o, seg))
        ctx.submit_device_segments(segs)
        ctx.sync()
        for first in range(0, n, seg):
            ctx.truth_accumulate(g, first, seg)
        mism, truth, ring = ctx.truth_compare()
        st = ctx.stats()
    assert st["events"] == n and st["parse_errors"] == 0 and st["deferred"] == 0
    assert mism == 0 and truth == ring == st["joined"]


def test_segment_arguments_rejected():
    with make_ctx() as ctx:
        d = ctx.device_alloc(1024)
        with pytest.raises(YsbError):
            ctx.submit_device_segments([(d, 16, d, 1)] * 17)
        with pytest.raises(YsbError):
            ctx.submit_device_segments([(d, 16, d, 1), (d + 3, 16, d, 1)])
        ctx.submit_device_segments([])          # nothing to do
        ctx.submit_device_segments([(d, 0, d, 0)])
        ctx.sync()
        assert ctx.stats()["events"] == 0


@pytest.mark.parametrize("pct,chunk", [(20, 16), (50, 5)])
def test_dynamic_share_equals_static(monkeypatch, pct, chunk):
    """The optional dynamic tile claims (YSB_DYN_PCT / YSB_DYN_CHUNK, read at ysb_open;
    off by default) count exactly what the static schedule counts: 3.2M skewed events in
    two segments large enough for the dynamic share, half the keys deferred."""
    g = GenParams(seed=2024, events_per_sec=5000, with_skew=True)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    sizes = [1_700_000, 1_500_000]
    out = []
    for env in (None, (pct, chunk)):
        if env:
            monkeypatch.setenv("YSB_DYN_PCT", str(env[0]))
            monkeypatch.setenv("YSB_DYN_CHUNK", str(env[1]))
        with make_ctx(n_campaigns=100, ads=(aids[:980], camp[:980]), sparse_fast_join=True,
                      window_ring=64, overflow_capacity=1 << 22) as ctx:
            segs, first = [], 0
            for n in sizes:
                cap = n * g.max_line_bytes() + 64
                d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
                nb = ctx.gen_events_device(g, first, n, d_b, cap, d_o)
                segs.append((d_b, nb, d_o, n))
                first += n
            ctx.submit_device_segments(segs)
            ctx.submit_device_segments(segs)   # twice: the claim counters are reset between launches
            out.append((ctx.drain_buckets(), ctx.stats()))
        monkeypatch.delenv("YSB_DYN_PCT", raising=False)
        monkeypatch.delenv("YSB_DYN_CHUNK", raising=False)
    (rows_s, st_s), (rows_d, st_d) = out
    assert st_s["events"] == 2 * sum(sizes) and st_s["deferred"] > 0 and st_s["join_misses"] > 0
    assert st_d == st_s
    assert rows_d == rows_s
