"""CPU: the seeded generator (host side of the C library) reproduces the data/
generator's format (core.clj:90-97) and the committed fixture byte for byte."""
import json
import os
import re

import pytest

import golden_data as gd
from ysb_amd import AD_TYPES, EVENT_TYPES, AdCampaignMap, GenParams, shard_ads

UUID4 = re.compile(r"^[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}$")
LINE = re.compile(r'^\{"user_id": "([^"]+)", "page_id": "([^"]+)", "ad_id": "([^"]+)", "ad_type": "([^"]+)", '
                  r'"event_type": "([^"]+)", "event_time": "(-?[0-9]+)", "ip_address": "1\.2\.3\.4"\}\n$')


def gen_from_fixture():
    p = gd.gen_params()
    return GenParams(seed=p["seed"], n_campaigns=p["n_campaigns"], ads_per_campaign=p["ads_per_campaign"],
                     t0_ms=p["t0_ms"], events_per_sec=p["events_per_sec"], with_skew=p["with_skew"]), p


def test_host_generator_matches_fixture_bytes():
    g, p = gen_from_fixture()
    data, off = g.events_host(0, p["n_events"])
    raw, offs = gd.events("gen_s7")
    assert bytes(data) == raw
    assert list(off) == offs


def test_ids_match_fixture():
    g, _ = gen_from_fixture()
    cids, aids = g.ids()
    assert cids == gd.campaigns()
    m = gd.ad_map()
    assert set(aids) == set(m)
    for i, a in enumerate(aids):   # (partition 10 ads): ad i -> campaign i // 10 (core.clj:52)
        assert m[a] == cids[i // 10]
        assert UUID4.match(a)


def test_line_format_and_distribution():
    g = GenParams(seed=3, events_per_sec=100)
    data, off = g.events_host(0, 6000)
    raw = bytes(data)
    cids, aids = g.ids()
    aset = set(aids)
    types, ets, times = {}, {}, []
    for i in range(len(off)):
        ln = raw[off[i]:(off[i + 1] if i + 1 < len(off) else len(raw))].decode()
        m = LINE.match(ln)
        assert m, ln
        assert UUID4.match(m.group(1)) and UUID4.match(m.group(2)) and m.group(3) in aset
        types[m.group(4)] = types.get(m.group(4), 0) + 1
        ets[m.group(5)] = ets.get(m.group(5), 0) + 1
        times.append(int(m.group(6)))
        json.loads(ln)
    assert set(types) == set(AD_TYPES) and set(ets) == set(EVENT_TYPES)
    assert all(abs(v - 2000) < 200 for v in ets.values())
    # catch-up mode: 10 ms per event (core.clj:95)
    assert times == [1_700_000_000_000 + 10 * i for i in range(6000)]
    assert abs(len(raw) / len(off) - 254.07) < 1.0   # mean line 254.07 B


def test_skew_semantics():
    g = GenParams(seed=5, events_per_sec=1000, with_skew=True)
    data, off = g.events_host(0, 200000)
    raw = bytes(data)
    late = 0
    for i in range(0, len(off)):
        s = off[i]
        j = raw.index(b'"event_time": "', s) + 15
        t = int(raw[j:raw.index(b'"', j)])
        d = t - (1_700_000_000_000 + i)
        assert -60000 - 49 <= d <= 50   # +-50 ms skew, late by < 60 s (core.clj:166-174)
        late += d < -49
    assert 0 <= late <= 10


def test_skew_only_mode_is_never_late():
    """with_skew=2: the same +-50 ms skew draws, no late events (the streaming leg's
    out-of-order workload); with_skew=1 on the same seed differs only on its late events."""
    n = 200_000
    a = GenParams(seed=5, events_per_sec=1000, with_skew=2)
    b = GenParams(seed=5, events_per_sec=1000, with_skew=True)
    ra, oa = a.events_host(0, n)
    rb, ob = b.events_host(0, n)
    ta, tb = [], []
    for raw, off, out in ((bytes(ra), oa, ta), (bytes(rb), ob, tb)):
        for i in range(n):
            j = raw.index(b'"event_time": "', off[i]) + 15
            out.append(int(raw[j:raw.index(b'"', j)]) - (1_700_000_000_000 + i))
    assert all(-49 <= d <= 50 for d in ta)
    diff = [i for i in range(n) if ta[i] != tb[i]]
    assert 0 < len(diff) <= 10 and all(tb[i] < ta[i] for i in diff)


def test_first_offset_and_subsets():
    g = GenParams(seed=9)
    d1, o1 = g.events_host(0, 100)
    d2, o2 = g.events_host(50, 50)
    assert bytes(d1[o1[50]:]) == bytes(d2)
    cids, aids = g.ids()
    parts = shard_ads(aids, 4)
    assert sorted(sum(parts, [])) == list(range(1000))
    assert all(len(p) > 150 for p in parts)
    gs = GenParams(seed=9, ad_subset=parts[2])
    d, o = gs.events_host(0, 500)
    raw = bytes(d)
    allowed = {aids[i] for i in parts[2]}
    for i in range(len(o)):
        j = raw.index(b'"ad_id": "', o[i]) + 10
        assert raw[j:j + 36].decode() in allowed


def test_dump_mode(tmp_path):
    g = GenParams(seed=21, n_campaigns=5, ads_per_campaign=10)
    g.dump(1000, tmp_path)
    names = sorted(os.listdir(tmp_path))
    assert names == ["ad-ids.txt", "ad-to-campaign-ids.txt", "ad-to-campaign.csv", "campaign-ids.txt",
                     "kafka-json.txt"]
    cids, aids = g.ids()
    assert (tmp_path / "campaign-ids.txt").read_text().split() == cids
    assert (tmp_path / "ad-ids.txt").read_text().split() == aids
    jm = AdCampaignMap.from_json_lines((tmp_path / "ad-to-campaign-ids.txt").read_bytes(), cids)
    cm = AdCampaignMap.from_csv((tmp_path / "ad-to-campaign.csv").read_bytes(), cids)
    assert jm.ad_to_campaign == cm.ad_to_campaign
    assert jm.arrays() == (aids, [i // 10 for i in range(50)])
    data, off = g.events_host(0, 1000)
    assert (tmp_path / "kafka-json.txt").read_bytes() == bytes(data)


def test_json_map_line_format(tmp_path):
    g = GenParams(seed=1, n_campaigns=2, ads_per_campaign=10)
    g.dump(0, tmp_path)
    first = (tmp_path / "ad-to-campaign-ids.txt").read_text().splitlines()[0]
    assert re.match(r'^\{ "[0-9a-f-]{36}": "[0-9a-f-]{36}"\}$', first)   # core.clj:58


@pytest.mark.parametrize("rate", [1, 100, 100_000, 7_000_001])
def test_event_time_rate(rate):
    g = GenParams(seed=2, events_per_sec=rate)
    data, off = g.events_host(123456, 3)
    raw = bytes(data)
    for k in range(3):
        j = raw.index(b'"event_time": "', off[k]) + 15
        assert int(raw[j:raw.index(b'"', j)]) == 1_700_000_000_000 + ((123456 + k) * 1000) // rate


def test_cli_shards_and_tbl(tmp_path):
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "streaming-benchmarks_amd",
                       "bin", "ysb_gen")
    subprocess.run([exe, "-d", str(tmp_path), "-n", "500", "--shards", "2", "--tbl", "--seed", "5"], check=True)
    parts = [(tmp_path / ("kafka-json.%d.txt" % r)).read_bytes().splitlines() for r in range(2)]
    assert not (tmp_path / "kafka-json.txt").exists()
    rows = (tmp_path / "events.tbl").read_bytes().splitlines()
    assert len(rows) == 500 == sum(len(p) for p in parts)
    import json as _json
    tbl_set = set(rows)
    for ln in parts[0] + parts[1]:
        ev = _json.loads(ln)
        assert "|".join(ev[k] for k in ("user_id", "page_id", "ad_id", "ad_type", "event_type",
                                        "event_time")).encode() in tbl_set


@pytest.mark.parametrize("kw", [dict(), dict(with_skew=True, events_per_sec=1000), dict(n_users=50, seed=9),
                                dict(event_stream=3, ad_subset=list(range(0, 1000, 7)))])
def test_tbl_format_is_json_to_tbl(kw):
    """format YSB_GEN_TBL writes exactly what ysb_json_to_tbl makes of the JSON lines."""
    rows, roff = GenParams(fmt="tbl", **kw).events_host(1000, 20_000)
    conv, coff = GenParams(**kw).events_host_tbl(1000, 20_000)
    assert rows.tobytes() == conv.tobytes() and list(roff) == list(coff)


@pytest.mark.parametrize("variant", [8, 8 | 4, 8 | 1, 8 | 4 | 1 | 2])
def test_variant_lines_decode_to_the_same_events(variant):
    """Every layout variant (reordered keys, compact, random ip) writes the same event a
    JSON parser reads from the generator's own line (json.loads dicts equal, the ip aside
    when it is random)."""
    import json
    from ysb_amd import GEN_RANDOM_IP, GEN_MORE_AD_TYPES
    base = variant & (GEN_RANDOM_IP | GEN_MORE_AD_TYPES)
    g0 = GenParams(seed=11, n_campaigns=10, ads_per_campaign=10, events_per_sec=1000, with_skew=True, variant=base)
    g1 = GenParams(seed=11, n_campaigns=10, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                   variant=variant)
    a, _ = g0.events_host(0, 3000)
    b, ob = g1.events_host(0, 3000)
    la, lb = bytes(a).split(b"\n")[:-1], bytes(b).split(b"\n")[:-1]
    assert len(la) == len(lb) == 3000 and ob[0] == 0
    for x, y in zip(la, lb):
        assert json.loads(x) == json.loads(y)
    if variant & 8:
        assert not lb[0].startswith(b'{"user_id"')


def test_shard_packed_equals_ad_shard():
    """The vectorised shard of packed 36-byte ids (bench.py's 10M-ad shards) equals the
    library's ysb_ad_shard key by key, also for keys of other lengths."""
    import numpy as np
    from ysb_amd import ad_shard, shard_packed
    g = GenParams(seed=3, n_campaigns=500, ads_per_campaign=4)
    _, ab = g.ids_packed()
    _, aids = g.ids()
    for n in (1, 2, 3, 8):
        assert shard_packed(ab, n).tolist() == [ad_shard(a, n) for a in aids]
    odd = np.frombuffer(b"".join(b"ad-%05d-x" % i for i in range(300)), dtype=np.uint8)   # 10-byte keys
    assert shard_packed(odd, 5, key_len=10).tolist() == [ad_shard(b"ad-%05d-x" % i, 5) for i in range(300)]


def test_layout_sampling_decisions():
    """The layout every submit reads off its batch's first line (ysb_layout_of_line, host
    code): the generator's own lines -> 0, compact -> 1, another key order -> 3 with that
    order, and everything the learned-order check cannot express -> 2."""
    from ysb_amd import GEN_COMPACT, GEN_RANDOM_IP, GEN_REORDER, layout_of_line
    first = lambda v: bytes(GenParams(seed=1, variant=v).events_host(0, 1)[0])   # noqa: E731
    assert layout_of_line(first(0)) == (0, None, False)
    assert layout_of_line(first(GEN_RANDOM_IP)) == (0, None, False)
    assert layout_of_line(first(GEN_COMPACT)) == (1, None, True)
    lay, order, cp = layout_of_line(first(GEN_REORDER))
    assert lay == 3 and not cp
    assert order == ["ad_type", "event_time", "ad_id", "ip_address", "user_id", "event_type", "page_id"]
    lay, order, cp = layout_of_line(first(GEN_REORDER | GEN_COMPACT))
    assert lay == 3 and cp and len(order) == 7
    g = first(0)
    no_ip = g.replace(b', "ip_address": "1.2.3.4"', b'')
    assert layout_of_line(no_ip)[0] == 3 and layout_of_line(no_ip)[1][-1] == "event_time"
    assert layout_of_line(no_ip, require_ip=True)[0] == 2          # ip_address required, absent
    for bad in (g.replace(b'{"', b'{ "', 1),                         # space after '{'
                g.replace(b'", "page_id"', b'","page_id"'),          # mixed spacing
                g.replace(b'"ad_type"', b'"ad_kind"'),               # another key
                g[:-2] + b', "ad_type": "x"}\n',                     # a repeated key
                g.replace(b'"user_id": "', b'"user_id": "z'),        # a 37-byte id
                g.replace(b'"view"', b'"v\\u0069ew"').replace(b'"click"', b'"cl\\u0069ck"')
                 .replace(b'"purchase"', b'"purch\\u0061se"'),       # an escape
                g.replace(b'"1.2.3.4"', b'1234'),                    # a non-string value
                b"", b"not json"):
        assert layout_of_line(bad)[0] == 2, bad


def test_threaded_host_generator_is_byte_identical():
    """ysb_gen_events_host_mt (the loaded streaming leg's producer) writes the same bytes and
    offsets as the single-threaded generator, for every variant and with skew."""
    import numpy as np
    from ysb_amd import GEN_COMPACT, GEN_REORDER, GenParams
    for variant in (0, GEN_COMPACT, GEN_REORDER):
        g = GenParams(seed=13, events_per_sec=20_000_000, with_skew=True, n_users=100, variant=variant)
        raw, offs = g.events_host(1000, 50_000)
        out = np.zeros(50_000 * g.max_line_bytes(), dtype=np.uint8)
        off = np.zeros(50_000, dtype=np.uint32)
        for threads in (1, 3, 16):
            nb = g.write_host(1000, 50_000, out, off, threads)
            assert nb == raw.size and np.array_equal(out[:nb], raw) and np.array_equal(off, offs), (variant, threads)


def test_mixed_variant_interleaves_four_producers_per_event():
    """GEN_MIXED: line i is exactly line i of one of the four producers' generators (the
    generator's layout, compact, reordered keys, random ip with 8 ad_types), each about a
    quarter of the lines -- the same events, so the same truth."""
    import numpy as np
    from ysb_amd import GEN_COMPACT, GEN_MIXED, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER, GenParams

    def lines(v):
        raw, off = GenParams(seed=17, events_per_sec=1000, with_skew=True, variant=v).events_host(0, 4000)
        b = raw.tobytes()
        return [b[a:e] for a, e in zip(off, list(off[1:]) + [len(b)])]
    mixed = lines(GEN_MIXED)
    pools = [lines(v) for v in (0, GEN_COMPACT, GEN_REORDER, GEN_RANDOM_IP | GEN_MORE_AD_TYPES)]
    hits = np.zeros(4, dtype=int)
    for i, ln in enumerate(mixed):
        m = [k for k in range(4) if pools[k][i] == ln]
        assert len(m) == 1, (i, ln)
        hits[m[0]] += 1
    assert hits.min() > 800, hits


def test_mixed_blocks_variant_runs_of_one_producer():
    """GEN_MIXED_BLOCKS: the four producers of GEN_MIXED in runs of 256 events -- every line
    is exactly that line of one producer's generator, one producer per run, each producer
    running some of the runs (the same events, so the same truth)."""
    from ysb_amd import GEN_COMPACT, GEN_MIXED_BLOCKS, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER, GenParams

    def lines(v):
        raw, off = GenParams(seed=17, events_per_sec=1000, with_skew=True, variant=v).events_host(0, 8192)
        b = raw.tobytes()
        return [b[a:e] for a, e in zip(off, list(off[1:]) + [len(b)])]
    mixed = lines(GEN_MIXED_BLOCKS)
    pools = [lines(v) for v in (0, GEN_COMPACT, GEN_REORDER, GEN_RANDOM_IP | GEN_MORE_AD_TYPES)]
    runs = []
    for r in range(len(mixed) // 256):
        owners = set()
        for i in range(256 * r, 256 * (r + 1)):
            m = [k for k in range(4) if pools[k][i] == mixed[i]]
            assert m, (i, mixed[i])
            owners.add(m[0] if len(m) == 1 else -1)
        owners.discard(-1)   # a line two producers write alike (none expected)
        assert len(owners) == 1, (r, owners)
        runs.append(owners.pop())
    assert len(set(runs)) == 4, runs
