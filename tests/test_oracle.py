"""CPU: the oracle restatements against the committed golden fixtures and against
known answers derived by hand from the reference's arithmetic."""
import numpy as np
import pytest

import golden_data as gd
from oracle import dostats, oracle


@pytest.fixture(scope="module")
def admap():
    ads, camp = gd.ad_arrays()
    return oracle.AdMap(ads, camp)


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
@pytest.mark.parametrize("threads", [1, 3])
def test_c_oracle_matches_golden(admap, stem, require_ip, threads):
    raw, offs = gd.events(stem)
    rows, st = oracle.run(admap, raw, offs, require_ip=require_ip, threads=threads)
    exp_rows, exp_st = gd.expected(stem, require_ip)
    assert st == exp_st
    assert rows == exp_rows


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
def test_python_oracle_matches_golden(stem, require_ip):
    raw, _ = gd.events(stem)
    lines, _ = dostats.split_lines(raw)
    idx = gd.campaign_index()
    r = dostats.run(lines, gd.ad_map(), 10000, require_ip)
    exp_rows, exp_st = gd.expected(stem, require_ip)
    assert r.stats() == exp_st
    assert {(idx[c], b): v for (c, b), v in r.counts.items()} == exp_rows


def test_ad_map_formats_agree():
    with open(gd.path("gen_s7.ad_to_campaign.txt"), "rb") as f:
        j = dostats.load_ad_map_json_lines(f.read())
    with open(gd.path("gen_s7.ad_to_campaign.csv"), "rb") as f:
        c = dostats.load_ad_map_csv(f.read())
    assert j == c and len(j) == 100


def test_later_duplicate_wins():
    # HashMap.put (AdvertisingTopologyNative.java:53) / merge (core.clj:106): the later entry wins
    assert dostats.load_ad_map_csv(b"a,x\na,y\n") == {"a": "y"}
    assert dostats.load_ad_map_json_lines(b'{ "a": "x"}\n{ "a": "y"}\n') == {"a": "y"}
    m = oracle.AdMap(["a", "a"], [1, 2])
    line = b'{"user_id": "u", "page_id": "p", "ad_id": "a", "ad_type": "t", "event_type": "view", "event_time": "20000"}\n'
    rows, _ = oracle.run(m, line, [0])
    assert rows == {(2, 2): 1}


# Known answers derived from CampaignProcessorCommon.java:28,58 (Long.parseLong(t) / 10000L,
# truncating toward zero) and :103 (window timestamp = bucket * 10000).
@pytest.mark.parametrize("t,bucket", [
    ("1700000000000", 170000000), ("1700000009999", 170000000), ("1700000010000", 170000001),
    ("0", 0), ("9999", 0), ("-5", 0), ("-9999", 0), ("-10000", -1), ("-15000", -1),
    ("+20000", 2), ("0009999", 0), ("9223372036854775807", 922337203685477),
    ("-9223372036854775808", -922337203685477),
])
def test_bucket_known_answers(t, bucket):
    m = oracle.AdMap(["ad"], [0])
    line = ('{"user_id": "u", "page_id": "p", "ad_id": "ad", "ad_type": "t", "event_type": "view", '
            '"event_time": "%s"}' % t).encode()
    rows, st = oracle.run(m, line, [0])
    assert st["joined"] == 1 and st["time_errors"] == 0
    assert rows == {(0, bucket): 1}
    assert dostats.java_div(dostats.parse_long(t), 10000) == bucket


@pytest.mark.parametrize("t", ["", "-", "+", "1.5", "17e3", " 1", "1 ", "9223372036854775808",
                               "-9223372036854775809", "0x10", "١٢"])
def test_time_errors(t):
    m = oracle.AdMap(["ad"], [0])
    line = ('{"user_id": "u", "page_id": "p", "ad_id": "ad", "ad_type": "t", "event_type": "view", '
            '"event_time": "%s"}' % t).encode()
    rows, st = oracle.run(m, line, [0])
    assert st["time_errors"] == 1 and rows == {}


def test_oracles_agree_on_generated_stream():
    from ysb_amd import GenParams
    g = GenParams(seed=11, events_per_sec=37, with_skew=True)
    cids, aids = g.ids()
    data, off = g.events_host(0, 30000)
    am = oracle.AdMap(aids[:900], g.ad_campaign_index()[:900])   # 100 ads unmapped -> misses
    rows, st = oracle.run(am, data, off, threads=4)
    raw = bytes(data)
    lines = [raw[off[i]:(off[i + 1] if i + 1 < len(off) else len(raw))] for i in range(len(off))]
    r = dostats.run(lines, dict(zip(aids[:900], g.ad_campaign_index()[:900])))
    assert st == r.stats() and st["join_misses"] > 0
    assert rows == r.counts
    assert sum(rows.values()) == st["joined"]


def test_threads_do_not_change_results(admap):
    raw, offs = gd.events("gen_s7")
    a = oracle.run(admap, raw, offs, threads=1)
    b = oracle.run(admap, raw, offs, threads=7)
    assert a == b


def test_offsets_as_numpy(admap):
    raw, offs = gd.events("gen_s7")
    a = oracle.run(admap, np.frombuffer(raw, dtype=np.uint8), np.asarray(offs, dtype=np.uint32))
    assert a == oracle.run(admap, raw, offs)


def test_split_lines_follows_readline():
    # BufferedReader.readLine (AdvertisingTopologyNative.java:153-159): \n, \r\n, lone \r
    lines, offs = dostats.split_lines(b"a\nb\r\nc\rd\r\re")
    assert lines == [b"a\n", b"b\r\n", b"c\r", b"d\r", b"\r", b"e"] and offs == [0, 2, 5, 7, 9, 10]
    assert dostats.split_lines(b"a\n\nb") == ([b"a\n", b"\n", b"b"], [0, 2, 3])
    assert dostats.split_lines(b"") == ([], [])
