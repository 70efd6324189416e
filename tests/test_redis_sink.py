"""CPU: the Redis writer produces the reference's output schema
(CampaignProcessorCommon.java:69-89, AdvertisingSpark.scala:184-208), and the
generator's own readers (check-correct core.clj:215-237, get-stats :130-149) read
the golden counts back as CORRECT.  Runs against tests/fake_redis.py."""
import uuid
from collections import defaultdict

import pytest

import golden_data as gd
from fake_redis import FakeRedis
from ysb_amd.redis_sink import RespClient, RedisWindowWriter, check_correct, get_stats, new_setup, write_ad_map


@pytest.fixture
def redis():
    srv = FakeRedis()
    cli = RespClient("127.0.0.1", srv.port)
    yield srv, cli
    cli.close()
    srv.close()


def golden_rows():
    rows, _ = gd.expected("gen_s7")
    return [(c, b * 10000, n) for (c, b), n in sorted(rows.items())]


def dostats_shape():
    camps = gd.campaigns()
    rows, _ = gd.expected("gen_s7")
    out = defaultdict(dict)
    for (c, b), n in rows.items():
        out[camps[c]][b] = n
    return out


def reference_write_window(cli, campaign, window_ts, count, now):
    """The per-window sequence of CampaignProcessorCommon.writeWindow, one command at a time."""
    w = cli.execute("HMGET", campaign, window_ts)[0]
    if w is None:
        w = str(uuid.uuid4())
        cli.execute("HSET", campaign, window_ts, w)
        lst = cli.execute("HMGET", campaign, "windows")[0]
        if lst is None:
            lst = str(uuid.uuid4())
            cli.execute("HSET", campaign, "windows", lst)
        cli.execute("LPUSH", lst, window_ts)
    cli.execute("HINCRBY", w, "seen_count", count)
    cli.execute("HSET", w, "time_updated", now)
    cli.execute("LPUSH", "time_updated", now)


def canonical(kv):
    """The store with UUID-valued names replaced by labels of the (campaign, window)
    or campaign they belong to, so two stores can be compared."""
    names = {}
    for k, v in kv.items():
        if isinstance(v, dict) and "windows" in v:
            names[v["windows"]] = "list:" + k
            for f, x in v.items():
                if f != "windows":
                    names[x] = "win:%s:%s" % (k, f)
    out = {}
    for k, v in kv.items():
        kk = names.get(k, k)
        if isinstance(v, dict):
            out[kk] = {f: names.get(x, x) for f, x in v.items()}
        elif isinstance(v, list):
            out[kk] = sorted(v) if kk.startswith("list:") else list(v)
        else:
            out[kk] = v
    return out


def test_writer_schema_and_check_correct(redis):
    srv, cli = redis
    camps = gd.campaigns()
    new_setup(cli, camps)
    rows = golden_rows()
    # deltas over two flushes: HINCRBY accumulates, windows are created once
    half = [(c, w, n // 2) for c, w, n in rows]
    rest = [(c, w, n - n // 2) for c, w, n in rows]
    wr = RedisWindowWriter(cli, camps, clock_ms=lambda: 1_700_000_099_000)
    wr.write(half)
    wr.write(rest)
    res = check_correct(cli, dostats_shape())
    assert res and all(s == "CORRECT" for _, _, s, _ in res)
    kv = srv.kv
    per_campaign = defaultdict(set)
    for c, w, _ in rows:
        per_campaign[camps[c]].add(str(w))
    for camp, wins in per_campaign.items():
        h = kv[camp]
        assert set(h) == wins | {"windows"}
        assert sorted(kv[h["windows"]]) == sorted(wins)          # one LPUSH per window
        for w in wins:
            assert set(kv[h[w]]) == {"seen_count", "time_updated"}
    assert len(kv["time_updated"]) == sum(1 for r in half if r[2]) + len(rest)
    assert kv["campaigns"] == set(camps)


def test_writer_equals_sequential_reference_algorithm(redis):
    srv, cli = redis
    camps = gd.campaigns()
    rows = golden_rows()
    ref = FakeRedis()
    rcli = RespClient("127.0.0.1", ref.port)
    try:
        for batch in (rows[::2], rows[1::2], rows[::3]):
            RedisWindowWriter(cli, camps, clock_ms=lambda: 7).write(batch)   # fresh cache: reads Redis
            for c, w, n in batch:
                reference_write_window(rcli, camps[c], str(w), n, "7")
        assert canonical(srv.kv) == canonical(ref.kv)
    finally:
        rcli.close()
        ref.close()


def test_two_round_trips_per_flush(redis):
    srv, cli = redis
    camps = gd.campaigns()
    wr = RedisWindowWriter(cli, camps)
    wr.write(golden_rows())
    assert wr.round_trips == 2
    wr.write(golden_rows())    # every window cached: writes only
    assert wr.round_trips == 3


def test_get_stats_and_mismatch_reports(redis):
    srv, cli = redis
    camps = gd.campaigns()
    new_setup(cli, camps)
    write_ad_map(cli, gd.ad_map())
    assert cli.execute("GET", next(iter(gd.ad_map()))) in camps
    rows = golden_rows()
    RedisWindowWriter(cli, camps, clock_ms=lambda: 1_700_000_123_456).write(rows[1:])
    st = get_stats(cli)
    assert sorted(s for s, _ in st) == sorted(n for _, _, n in rows[1:])
    assert all(u == 1_700_000_123_456 - w for (_, u), (_, w, _) in zip(sorted(st, key=lambda x: x[1], reverse=True),
                                                                       sorted(rows[1:], key=lambda r: r[1])))
    exp = dostats_shape()
    c0, w0, n0 = rows[0]
    res = {(c, b): s for c, b, s, _ in check_correct(cli, exp)}
    assert res[(camps[c0], w0 // 10000)] == "MISSING"
    RedisWindowWriter(cli, camps).write([(c0, w0, n0 + 1)])
    res = {(c, b): s for c, b, s, _ in check_correct(cli, exp)}
    assert res[(camps[c0], w0 // 10000)] == "DIFFER"
    assert sum(s == "CORRECT" for s in res.values()) == len(rows) - 1
