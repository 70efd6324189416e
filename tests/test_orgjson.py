"""CPU: the org.json 20180813 restatement (oracle/orgjson.py) -- known answers for its
grammar and typing rules, and differential agreement with the C restatement
(oracle/ysb_oracle.c) line by line over a seeded corpus (tests/orgjson_fuzz.py)."""
import pytest

import golden_data as gd
import orgjson_fuzz as fz
from oracle import dostats, oracle, orgjson


# JSONObject.stringToValue's result type for unquoted text (see orgjson.py's header).
@pytest.mark.parametrize("tok,kind", [
    (b"true", "bool"), (b"TRUE", "bool"), (b"False", "bool"), (b"fal\xc5\xbfe", "bool"), (b"nUlL", "null"),
    (b"truex", "str"), (b"view", "str"), (b"a b", "str"),
    (b"0", "long"), (b"-1", "long"), (b"9223372036854775807", "long"), (b"-9223372036854775808", "long"),
    (b"9223372036854775808", "str"), (b"01", "str"), (b"-01", "str"), (b"+1", "str"), (b"1_000", "str"),
    (b"-0", "double"), (b"1.5", "double"), (b"1.", "double"), (b"-.5", "double"), (b"1e5", "double"),
    (b"1E-5", "double"), (b"1.5f", "double"), (b"1.5D", "double"), (b"0e99999", "double"),
    (b"1e308", "double"), (b"1.7976931348623157e308", "double"), (b"1.7976931348623159e308", "str"),
    (b"1e309", "str"), (b"1e", "str"), (b"1e+", "str"), (b"1.2.3", "str"), (b"1d", "str"), (b"1.5ff", "str"),
    (b"0x1p3", "str"), (b"0x1.8p1", "double"), (b"0xEp1", "double"), (b"0x1.fffffffffffff7p1023", "double"),
    (b"0x1.fffffffffffff8p1023", "str"), (b"0x.8p1", "double"), (b"0x1.8", "str"), (b"-NaN", "str"),
    (b"-Infinity", "str"), (b"NaN", "str"),
])
def test_token_kind(tok, kind):
    assert orgjson.token_kind(tok) == kind


# Whole-line known answers: does new JSONObject(line) + getString x6 succeed?
@pytest.mark.parametrize("line,ok", [
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', True),
    (b"{user_id:u,page_id:p,ad_id:a,ad_type:t,event_type:view,event_time:'1'}", True),
    (b"{user_id:u,page_id:p,ad_id:a,ad_type:t,event_type:view,event_time:1}", False),        # Integer
    (b"{'user_id':'u';'page_id':'p';'ad_id':'a';'ad_type':'t';'event_type':'view';'event_time':'1';}", True),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"} trailing', True),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1",,}', False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1","x":1,x:2}', False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1","w":{"a":1,"a":1}}',
     False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1","w":[{"a":1},{"a":1}]}',
     True),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1\r"}', False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1\\\'"}', True),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"\x00}', False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}\x00', True),
    (b'\x01\x1f{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', True),
    (b'{"user_id"="u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', False),
    (b'{"user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view"}', False),
    (b"", False), (b"[]", False), (b"{}", False), (b"{", False), (b"{\"a\": [", False),
    # a producer's extra fields (the GPU flat tier takes exactly one plain-string extra pair)
    (b'{"src": "w", "user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', True),
    (b'{"user_id":"u","page_id":"p","ad_idx":"7","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', True),
    (b'{"a1":"x","a2":"y","user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}',
     True),
    (b'{"a1":"x","a1":"y","user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}',
     False),                                                                                   # putOnce: duplicate
    (b'{"":"x","user_id":"u","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}', True),
    (b'{"user_id":"u","user_id":"v","page_id":"p","ad_id":"a","ad_type":"t","event_type":"view","event_time":"1"}',
     False),
])
def test_line_known_answers(line, ok):
    def parses(ln):
        try:
            dostats.parse_event(ln)
            return True
        except dostats.ParseError:
            return False

    assert parses(line) == ok
    ads, camp = ["a"], [0]
    _, st = oracle.run(oracle.AdMap(ads, camp), line + b"\n", [0])
    assert (st["parse_errors"] == 0) == ok


def test_escape_decoding():
    obj = orgjson.parse_object(b'{"k": "a\\u0062\\u+063\\u-001\\ud83d\\ude00\\ud83d\\t"}')
    assert obj[b"k"] == ("str", b"abc\xef\xbf\xbf\xf0\x9f\x98\x80\xed\xa0\xbd\t")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_c_oracle_agrees_with_python_line_by_line(seed):
    ads, camp = gd.ad_arrays()
    m, idx = gd.ad_map(), gd.campaign_index()
    am = oracle.AdMap(ads, camp)
    for require_ip in (False, True):
        for line in fz.lines(seed, 1200, ads):
            r = dostats.run([line], m, 10000, require_ip)
            rows, st = oracle.run(am, line, [0], require_ip=require_ip)
            assert st == r.stats(), line
            assert rows == {(idx[c], b): v for (c, b), v in r.counts.items()}, line


def test_fuzz_corpus_is_balanced():
    ads, _ = gd.ad_arrays()
    r = dostats.run(fz.lines(1, 2000, ads), gd.ad_map())
    assert r.joined > 300 and r.parse_errors > 600 and r.join_misses > 30 and r.time_errors > 5


def test_strict_and_orgjson_agree_on_generator_lines():
    """dostats reads the generator's file with a strict parser (clj-json); the Flink chain
    with org.json.  On the generator's own format they must agree exactly."""
    raw, _ = gd.events("gen_s7")
    lines, _ = dostats.split_lines(raw)
    a = dostats.run(lines, gd.ad_map())
    b = dostats.run(lines, gd.ad_map(), strict=True)
    assert a.stats() == b.stats() and a.counts == b.counts
    assert a.parse_errors == 0
