"""One-GPU rehearsal of bench.py's N-rank setup (the driver runs N = 2/4/8 on a full node;
RCCL refuses two ranks on one device, so the collective itself is not run here).

Each rank's context is built exactly as bench.py builds it (its own generator stream
over its shard of the shared ad ids, window_ring 1024, the ring base every rank derives
from the shared t0), all on cuda:0.  What ysb_group_reduce_scatter needs before summing
tables cell by cell is checked directly: every rank's ring starts at the same bucket
(ysb_capi.cpp agree_ring would otherwise move a later-starting ring), every rank counts
exactly its generator truth, and the sum over ranks equals the campaign-major
reduce-scatter result (owner blocks, ysb_group_owned's padding rule).  A one-rank RCCL
group runs bench.py's own post-exchange check (exchange_check) for real."""
import os
import sys
from collections import Counter

import pytest

from ysb_amd import GenParams, YsbContext, owned_block, shard_ads

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu


def rank_params(world, rank, rate=100_000):
    # bench.py main(): base ids, then per-rank stream 1 + rank over shard_ads(...)[rank]
    base = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=rate)
    cids, aids = base.ids()
    camp = base.ad_campaign_index()
    if world == 1:
        return base, aids, camp
    subset = shard_ads(aids, world)[rank]
    g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=100, ads_per_campaign=10,
                  events_per_sec=rate, ad_subset=subset)
    return g, aids, camp


@pytest.mark.parametrize("world", [2, 8])
def test_bench_ranks_share_ring_base_and_sum_to_truth(world):
    n = 2_000_000
    rings, tables, total_joined = [], [], 0
    for rank in range(world):
        g, aids, camp = rank_params(world, rank)
        with YsbContext(device=0, n_campaigns=100, window_ring=1024, ring_base_bucket=g.c.t0_ms // 10000 - 128,
                        max_batch_bytes=16 << 20, max_batch_events=1 << 16) as ctx:
            # bench.py: each rank loads only its ad_id-hash shard of the join table
            ctx.load_ad_map(aids, camp, shard=(rank, world))
            cap = n * g.max_line_bytes()
            d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
            nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
            ctx.sync()
            ctx.truth_accumulate(g, 0, n)
            mism, truth, ring = ctx.truth_compare()
            st = ctx.stats()
            assert st["events"] == n and st["parse_errors"] == 0 and st["join_misses"] == 0
            assert mism == 0 and truth == ring == st["joined"], (rank, mism, truth, ring)
            rings.append(ctx.ring_range())
            tables.append(ctx.drain_buckets())
            total_joined += st["joined"]
    # the reduce-scatter precondition: one ring base on every rank
    assert len(set(rings)) == 1, rings
    merged = Counter()
    for t in tables:
        merged.update(t)
    assert sum(merged.values()) == total_joined
    # owner blocks tile the campaigns; each owner's block of the merged table is what its
    # d_owned holds after the exchange
    blocks = [owned_block(100, r, world) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == 100
    assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
    owned = sum(v for (c, _), v in merged.items() for lo, hi in blocks if lo <= c < hi)
    assert owned == total_joined


def test_one_rank_group_runs_bench_config3_ranks():
    """bench.config3_ranks -- the configs[2]-table leg every N > 1 run times -- on a real
    one-rank RCCL group: its pipelined range exchange per step, the exchange fields of its
    line (rs / exposed / hidden per step), and its checksum check, exact."""
    import bench
    os.environ.pop("WORLD_SIZE", None)
    d = bench.Dist(1)
    d.resolve_device()
    args = bench.parse_args(["--c3-events", "8000000", "--extra-steps", "3", "--warmup", "1"])
    r = bench.config3_ranks(args, d)
    ex, chk = r["exchange"], r["check"]
    assert chk["checksum_blocks_mismatched"] == 0 and chk["truth_mismatched_cells"] == 0
    assert chk["truth_views"] == chk["counted_views"] > 0 and chk["join_misses"] == 0
    assert chk["foreign_shard"] == 0 and chk["parse_errors"] == 0
    for k in ("rs_ms_per_step", "exposed_ms_per_step", "hidden_ms_per_step"):
        assert ex[k] >= 0, (k, ex)
    assert abs(ex["hidden_ms_per_step"] - max(ex["rs_ms_per_step"] - ex["exposed_ms_per_step"], 0.0)) <= 2e-4
    assert r["record_mode"] and r["n_gpus"] == 1


def test_one_rank_group_runs_bench_exchange_check():
    """A real (one-rank) RCCL group: ysb_group_init agrees on the ring, the reduce-scatter
    moves the table into the owned block, and bench.exchange_check -- the code the N-rank
    run executes -- finds the owners' rows equal to the truth."""
    import bench
    g, aids, camp = rank_params(1, 0)
    n = 3_000_000
    with YsbContext(device=0, n_campaigns=100, window_ring=1024, max_batch_bytes=16 << 20,
                    max_batch_events=1 << 16) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        assert ctx.group_info() == (0, 1)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        segs = [(0, n, d_b, nb, d_o)]

        def submit_all():
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
        submit_all()
        ctx.group_reduce_scatter()                       # first exchange: agrees on the ring
        os.environ.pop("WORLD_SIZE", None)
        d = bench.Dist(1)
        chk = bench.exchange_check(d, ctx, g, segs, submit_all)
        ex = chk["exchange"]
        assert chk["truth_mismatched_cells"] == 0 and chk["truth_views"] == chk["counted_views"] > 0
        assert ex["post_exchange_mismatched_cells"] == 0 and ex["owner_rows_outside_block"] == 0
        assert ex["owned_views"] == ex["truth_views_summed"] == chk["truth_views"]
        assert ex["rccl_ranks"] == [1] and ex["owned_blocks"] == [[0, 100]]
        # after ysb_group_init, ring_advance is collective (one rank: trivially agreed)
        lo, w = ctx.ring_range()
        ctx.ring_advance(lo + 1)
        assert ctx.ring_range() == (lo + 1, w)


def test_sharded_join_table_classifies_foreign_shard_views():
    """A rank's sharded table (ysb_load_ad_map_shard) joins exactly its own shard's ads.
    Another rank's events are views of a foreign shard: counted as foreign_shard, not as
    join misses (mis-routed input), and with strict=True ysb_sync fails with YSB_ERR_DATA.
    An ad of the rank's own shard that the map lacks stays a join miss, as RedisJoinBolt
    drops an unknown ad (AdvertisingTopologyNative.java:465-467)."""
    from ysb_amd import YsbError, ad_shard
    world = 4
    n = 200_000
    g0, aids, camp = rank_params(world, 0)
    g1, _, _ = rank_params(world, 1)
    for strict in (False, True):
        with YsbContext(device=0, n_campaigns=100, window_ring=1024, ring_base_bucket=g0.c.t0_ms // 10000 - 128,
                        max_batch_bytes=16 << 20, max_batch_events=1 << 16, strict=strict) as ctx:
            ctx.load_ad_map(aids, camp, shard=(0, world))
            cap = n * g0.max_line_bytes()
            d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
            nb = ctx.gen_events_device(g1, 0, n, d_b, cap, d_o)   # rank 1's events
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
            if strict:
                with pytest.raises(YsbError) as e:
                    ctx.sync()
                assert e.value.code == -8 and "another rank" in str(e.value)
            else:
                ctx.sync()
            st = ctx.stats()
            assert st["joined"] == 0 and st["join_misses"] == 0
            assert st["foreign_shard"] == st["views"] > 0
            ctx.reset()
            nb = ctx.gen_events_device(g0, 0, n, d_b, cap, d_o)   # its own
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
            ctx.sync()
            st = ctx.stats()
            assert st["join_misses"] == 0 and st["foreign_shard"] == 0 and st["joined"] == st["views"] > 0
    # a map without some of shard 0's own ads: their views are real join misses
    mine = [i for i, a in enumerate(aids) if ad_shard(a, world) == 0]
    drop = set(mine[:5])
    keep = [i for i in range(len(aids)) if i not in drop]
    with YsbContext(device=0, n_campaigns=100, window_ring=1024, ring_base_bucket=g0.c.t0_ms // 10000 - 128,
                    max_batch_bytes=16 << 20, max_batch_events=1 << 16, strict=True) as ctx:
        ctx.load_ad_map([aids[i] for i in keep], [camp[i] for i in keep], shard=(0, world))
        raw, offs = g0.events_host(0, 60_000)
        ctx.submit(raw, offs)
        ctx.sync()   # real misses are not an error in strict mode (the reference drops them)
        st = ctx.stats()
    from oracle import oracle
    rows, ost = oracle.run(oracle.AdMap([aids[i] for i in keep], [camp[i] for i in keep]), raw, offs)
    assert st["foreign_shard"] == 0 and st["join_misses"] == ost["join_misses"] > 0
    assert st["joined"] == ost["joined"]


def _config3_rank(n_campaigns=200_000):
    g = GenParams(seed=42, n_campaigns=n_campaigns, ads_per_campaign=10, events_per_sec=100_000)
    _, ab = g.ids_packed()
    return g, ab


def test_one_rank_group_range_exchange_config3_sized():
    """The range-limited exchange on a real (one-rank) RCCL group at configs[2]-like size
    (200k campaigns x 10 ads, W = 128, record mode with the u8 delta ring): only the buckets
    holding counts travel, as 1-byte cells while nranks x max <= 255; the owned table then
    equals the generator truth (rows and linear checksums), nothing stays pending, and the
    exchange's accounting reports what moved."""
    from ysb_amd import table_rows
    g, ab = _config3_rank()
    n = 4_000_000
    with YsbContext(device=0, n_campaigns=200_000, window_ring=128, max_batch_bytes=1 << 20,
                    max_batch_events=1 << 12, record_count=True) as ctx:
        ctx.load_ad_map_packed(ab, g.ad_campaign_index_array())
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        for k in range(3):   # three steps: count, exchange (the ring agreed at the first)
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
            ctx.group_reduce_scatter()
            x = ctx.exchange_info()
            assert x["exchanges"] == k + 1
            assert x["last_width"] == 1, x            # ~0.2 views per cell per step
            assert 0 < x["last_buckets"] <= 128
        # rows of whole aligned 4-slot groups: each run of buckets widened by < 4 slots per end
        assert x["bytes"] % (3 * 200_000) == 0 and x["ms"] > 0
        # complete exchanges: the compute stream waits for every reduce-scatter at its unpack
        assert 0 < x["rs_ms"] <= x["ms"] and 0 <= x["exposed_ms"] <= x["ms"], x
        row = x["bytes"] // (3 * 200_000)
        assert row % 4 == 0 and x["last_buckets"] <= row <= x["last_buckets"] + 6
        assert x["full_ring_bytes"] == 200_000 * 128 * 8
        _, _, nrec = ctx.path_time()
        assert nrec == 3                               # every launch in record mode
        for _ in range(3):
            ctx.truth_accumulate(g, 0, n)
        truth, lo = ctx.truth_read()
        expected = table_rows(truth, lo)
        got = ctx.drain_buckets()
        assert got == expected
        assert ctx.checksum("owned")[0] == ctx.checksum("truth")[0]
        assert ctx.checksum("pending") == [0]
        st = ctx.stats()
        assert st["overflow_dropped"] == 0 and st["out_of_ring"] == 0


def test_one_rank_group_ring_advance_to_lower_base_moves_to_side_list():
    """After ysb_group_init, ring_advance is a collective; moving the ring to a LOWER base
    runs the branch agree_ring takes on a later-starting rank (move_ring): the buckets the
    new range no longer holds go to the exact side list, and the drain (owned table +
    pending ring + side list) still equals the oracle."""
    from oracle import oracle
    g, aids, camp = rank_params(1, 0, rate=1000)
    raw, offs = g.events_host(0, 300_000)   # 300 s of event time: ~30 buckets
    rows, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    with YsbContext(device=0, n_campaigns=100, window_ring=32, max_batch_bytes=256 << 20,
                    max_batch_events=1 << 20) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        ctx.submit(raw, offs)
        ctx.group_reduce_scatter()
        lo, w = ctx.ring_range()
        ctx.ring_advance(lo - 10)                 # buckets [lo + 22, lo + 32) leave the ring
        assert ctx.ring_range() == (lo - 10, w)
        got = ctx.drain_buckets()
        assert got == rows
        ctx.submit(raw, offs)                     # counts after the move: ring + side again
        ctx.group_reduce_scatter()
        got = ctx.drain_buckets()
        assert got == {k: 2 * v for k, v in rows.items()}


def _escape_ad(line, mode):
    """The same event with its ad_id written with \\u escapes (every 5th value byte) and,
    for mode 1, the key name too ("ad\\u005fid"); mode 2 single-quotes the value."""
    i = line.index(b'"ad_id": "')
    v0 = i + 10
    val = line[v0:v0 + 36]
    if mode == 2:
        return line[:i] + b"\"ad_id\": '" + val + b"'" + line[v0 + 37:]
    ev = b"".join(b"\\u%04x" % c if k % 5 == 0 else bytes([c]) for k, c in enumerate(val))
    key = b'"ad\\u005fid": "' if mode == 1 else b'"ad_id": "'
    return line[:i] + key + ev + line[v0 + 36:]


@pytest.mark.parametrize("world", [2, 3])
def test_routed_escaped_ad_ids_join_on_their_shard(world):
    """ysb_route_lines hashes the DECODED ad_id (and finds an escaped key name), as the
    device's shard test does: lines whose ad_id is written with \\u escapes, an escaped key or
    single quotes are routed to the rank that holds their ad in its sharded join table, so no
    view is foreign_shard and the joined views and counts equal the C oracle's on the whole
    stream."""
    import numpy as np
    from oracle import oracle
    from ysb_amd import route_lines
    g = GenParams(seed=77, events_per_sec=1000)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    raw, off = g.events_host(0, 30_000)
    lines = [bytes(raw[a:b]) for a, b in zip(off, list(off[1:]) + [raw.size])]
    lines = [_escape_ad(ln, k % 3) if k % 4 else ln for k, ln in enumerate(lines)]
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    rows, ost = oracle.run(oracle.AdMap(aids, camp), data, offs.tolist())
    shard, _ = route_lines(np.frombuffer(data, dtype=np.uint8), offs, world)
    shard = np.asarray(shard)
    got, joined = Counter(), 0
    for r in range(world):
        mine = [lines[i] for i in np.nonzero(shard == r)[0]]
        with YsbContext(n_campaigns=100, strict=False) as ctx:
            ctx.load_ad_map(aids, camp, shard=(r, world))
            if mine:
                ctx.submit(b"".join(mine), np.cumsum([0] + [len(x) for x in mine[:-1]]).astype(np.uint32))
            st = ctx.stats()
            assert st["foreign_shard"] == 0, (r, st)
            joined += st["joined"]
            got.update(ctx.drain_buckets())
    assert joined == ost["joined"]
    assert dict(got) == rows


def _buggy_word_add(o, v):
    """Round 4's carry test in xunpack8: True when it let a byte pair add as a
    word although the byte sum passes 255."""
    t = (o & 0x7F) + (v & 0x7F)
    return (((o & v) | ((o | v) & ~t)) & 0x80) == 0 and o + v > 255


def test_owned_u8_accumulator_carries_across_exchanges_without_reads():
    """Four complete exchanges of the same batch with NO read of the owned table in between
    (no drain or checksum folds the u8 accumulator): ~83 views per cell and exchange, so the
    owned bytes pass 127 and then 255 with the incoming byte below 128 -- the case round 4's
    per-byte carry test missed (256 counts lost, one leaked into the next cell).  The drain
    after the fourth equals 4 x the C oracle's counts; the test first checks that its own
    cells do hit that case."""
    from oracle import oracle
    g, aids, camp = rank_params(1, 0, rate=2500)
    raw, offs = g.events_host(0, 300_000)
    rows, _ = oracle.run(oracle.AdMap(aids, camp), raw, offs)
    hits = 0
    for v in rows.values():
        o = 0
        for _ in range(4):
            if o + v > 255:
                hits += _buggy_word_add(o, v)
                o = 0
            else:
                o += v
    assert hits > 0 and max(rows.values()) <= 255
    with YsbContext(device=0, n_campaigns=100, window_ring=64, max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        for k in range(4):
            ctx.submit(raw, offs, slot=k & 1)
            ctx.group_reduce_scatter()
            assert ctx.exchange_info()["last_width"] == 1
        assert ctx.drain_buckets() == {key: 4 * v for key, v in rows.items()}


def test_device_count_does_not_depend_on_torch(monkeypatch):
    """bench.py maps LOCAL_RANK -> device with the library's hipGetDeviceCount, so a torch
    build that cannot see the GPU (seen on this pool: "No HIP GPUs are available" while HIP
    worked) cannot put every rank on device 0."""
    import torch
    import bench
    from ysb_amd import device_count
    n = device_count()
    assert n >= 1
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    for local in (0, n - 1, n, 3 * n + 1):
        monkeypatch.setenv("LOCAL_RANK", str(local))
        d = bench.Dist(1)
        assert d.resolve_device() == (local if local < n else local % n)
        assert d.n_visible == n
