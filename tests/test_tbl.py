"""CPU: the fork's pipe-delimited .tbl format (MockWindowedFlatMap,
AdvertisingTopologyNative.java:197-226): both oracles against the committed
fixtures, and the library's JSON -> .tbl converter against the fixture bytes."""
import numpy as np
import pytest

import golden_data as gd
from oracle import dostats, oracle
from ysb_amd import GenParams, json_to_tbl


@pytest.fixture(scope="module")
def admap():
    ads, camp = gd.ad_arrays()
    return oracle.AdMap(ads, camp)


@pytest.mark.parametrize("stem", gd.TBL_FIXTURES)
@pytest.mark.parametrize("threads", [1, 4])
def test_c_oracle_tbl_matches_golden(admap, stem, threads):
    raw, offs = gd.tbl_events(stem)
    rows, st = oracle.run(admap, raw, offs, threads=threads, fmt="tbl")
    exp_rows, exp_st = gd.expected(stem)
    assert rows == exp_rows
    assert st == exp_st


@pytest.mark.parametrize("stem", gd.TBL_FIXTURES)
def test_python_oracle_tbl_matches_golden(stem):
    raw, _ = gd.tbl_events(stem)
    lines, _ = dostats.split_lines(raw)
    idx = gd.campaign_index()
    m = gd.ad_map()
    r = dostats.run(lines, {a: idx[c] for a, c in m.items()}, fmt="tbl")
    exp_rows, exp_st = gd.expected(stem)
    assert r.counts == exp_rows and r.stats() == exp_st


def test_tbl_and_json_agree_on_generator_events(admap):
    raw, offs = gd.events("gen_s7")
    traw, toffs = gd.tbl_events("gen_s7_tbl")
    assert oracle.run(admap, raw, offs) == oracle.run(admap, traw, toffs, fmt="tbl")


def test_converter_matches_fixture_bytes():
    raw, offs = gd.events("gen_s7")
    out, oo = json_to_tbl(np.frombuffer(raw, dtype=np.uint8), np.asarray(offs, dtype=np.uint32))
    traw, toffs = gd.tbl_events("gen_s7_tbl")
    assert out.tobytes() == traw
    assert list(oo) == list(toffs)


def test_converter_rejects_other_layouts():
    from ysb_amd import YsbError
    bad = b'{"user_id": "u", "page_id": "p", "ad_id": "a\\u0041", "ad_type": "t", "event_type": "view", ' \
          b'"event_time": "1", "ip_address": "1"}\n'
    with pytest.raises(YsbError):
        json_to_tbl(np.frombuffer(bad, dtype=np.uint8), np.zeros(1, dtype=np.uint32))


def test_generator_tbl_rows():
    g = GenParams(seed=3, n_campaigns=4, ads_per_campaign=2)
    raw, offs = g.events_host_tbl(0, 50)
    lines = raw.tobytes().split(b"\n")[:-1]
    assert len(lines) == 50 and all(ln.count(b"|") == 5 for ln in lines)
