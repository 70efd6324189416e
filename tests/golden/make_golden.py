"""Generates the committed golden fixtures in tests/golden/.

    python tests/golden/make_golden.py

Fixtures (all data, no reference source):
  gen_s7.jsonl                 1500 events in the data/ generator's line format
                               (core.clj:90-97), produced by the pure-Python restatement
                               of the seeded generator below (independent of the C/HIP
                               generator, which tests must reproduce byte for byte)
  gen_s7.ad_to_campaign.txt    `{ "AD": "CAMPAIGN"}` lines (core.clj:58)
  gen_s7.ad_to_campaign.csv    `ad,campaign` lines (AdvertisingTopologyNative.java:52)
  gen_s7.campaign_ids.txt      campaign UUIDs (core.clj:24-31)
  edge.jsonl / edge_long.jsonl hand-written edge cases (boundaries, reordering,
                               escapes, errors, misses, an over-size line)
  edge_orgjson.jsonl           hand-written cases for org.json 20180813's own grammar
                               (unquoted and single-quoted text, ';' separators, trailing
                               commas, text after '}', duplicate keys at any level,
                               stringToValue typing, NUL / control bytes)
  gen_s7.tbl                   the same 1500 events as the fork's pipe-delimited rows
                               (MockWindowedFlatMap, AdvertisingTopologyNative.java:197-226)
  edge_tbl.tbl                 hand-written .tbl edge cases (String.split trailing-empty
                               rule, too few items, \r\n, empty fields, misses, errors)
  *.expected.csv               campaign_uuid,window_ms,count from oracle/dostats.py
  *.expected.json              the chain's counters (events, views, joined, ...)

Expected outputs come from oracle/dostats.py, whose JSON reading is oracle/orgjson.py
(the org.json 20180813 restatement), a Python implementation independent of both
oracle/ysb_oracle.c and the GPU tokenizer.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import dostats  # noqa: E402

M64 = (1 << 64) - 1


def mix64(z):
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def stream_key(seed, s):
    return mix64((seed * 0x9E3779B97F4A7C15 + s) & M64)


def draw(key, i):
    return mix64((key + (i + 1) * 0x9E3779B97F4A7C15) & M64)


S_CAMPAIGN, S_AD, S_USER, S_PAGE, S_CHOICE, S_SKEW = 1, 2, 3, 4, 5, 6
AD_TYPES = ("banner", "modal", "sponsored-search", "mail", "mobile")
EVENT_TYPES = ("view", "click", "purchase")


def uuid(key, k):
    hi = (draw(key, 2 * k) & ~0xF000 & M64) | 0x4000
    lo = (draw(key, 2 * k + 1) & 0x3FFFFFFFFFFFFFFF) | 0x8000000000000000
    h = "%016x%016x" % (hi, lo)
    return "%s-%s-%s-%s-%s" % (h[0:8], h[8:12], h[12:16], h[16:20], h[20:32])


class PyGen:
    """Pure-Python restatement of the seeded generator (streaming-benchmarks_amd/csrc/ysb_common.h)."""

    def __init__(self, seed, n_campaigns, ads_per_campaign, t0_ms, events_per_sec, with_skew):
        self.seed, self.nc, self.apc = seed, n_campaigns, ads_per_campaign
        self.t0, self.rate, self.skew = t0_ms, events_per_sec, with_skew

    def campaigns(self):
        k = stream_key(self.seed, S_CAMPAIGN)
        return [uuid(k, c) for c in range(self.nc)]

    def ads(self):
        k = stream_key(self.seed, S_AD)
        return [uuid(k, a) for a in range(self.nc * self.apc)]

    def event(self, i):
        c = draw(stream_key(self.seed, S_CHOICE), i)
        ad = ((c >> 32) * (self.nc * self.apc)) >> 32
        at = (c & 0xFFFF) % 5
        et = ((c >> 16) & 0xFFFF) % 3
        t = self.t0 + (i * 1000) // self.rate
        if self.skew:
            r = draw(stream_key(self.seed, S_SKEW), i)
            t += 50 - r % 100
            if ((r >> 17) % 100000) == 0:
                t -= (r >> 40) % 60000
        return ad, at, et, t

    def line(self, i):
        ad, at, et, t = self.event(i)
        return ('{"user_id": "' + uuid(stream_key(self.seed, S_USER), i)
                + '", "page_id": "' + uuid(stream_key(self.seed, S_PAGE), i)
                + '", "ad_id": "' + uuid(stream_key(self.seed, S_AD), ad)
                + '", "ad_type": "' + AD_TYPES[at]
                + '", "event_type": "' + EVENT_TYPES[et]
                + '", "event_time": "' + str(t)
                + '", "ip_address": "1.2.3.4"}\n')


GEN = dict(seed=7, n_campaigns=10, ads_per_campaign=10, t0_ms=1_700_000_000_000, events_per_sec=20,
           with_skew=True)
N_GEN = 1500


def edge_lines(ads, campaigns):
    a0, a1, a2 = ads[0], ads[11], ads[57]
    U = "0f8c1e7a-1111-4222-8333-944455556666"
    P = "1a2b3c4d-aaaa-4bbb-8ccc-ddddeeeeffff"

    def ev(ad=a0, et="view", t="1700000000000", at="banner", extra="", user=U, page=P):
        return ('{"user_id": "%s", "page_id": "%s", "ad_id": "%s", "ad_type": "%s", "event_type": "%s", '
                '"event_time": "%s", "ip_address": "1.2.3.4"%s}' % (user, page, ad, at, et, t, extra))

    esc_ad = a1.replace("-", "\\u002d")
    L = [
        ev(t="1700000000000"),                       # exactly on a bucket boundary
        ev(t="1700000009999"),                       # last ms of that bucket
        ev(t="1700000010000"),                       # first ms of the next
        ev(ad=a1, t="1700000012345", at="sponsored-search"),
        ev(ad=a2, et="click"),
        ev(ad=a2, et="purchase"),
        '{"event_time": "1700000020000", "ad_id": "%s", "event_type": "view", "user_id": "u", '
        '"page_id": "p", "ad_type": "mail"}' % a0,                                   # reordered, no ip
        '{ "user_id" :"u","page_id":"p" ,\t"ad_id":\t"%s","ad_type" : "modal", "event_type":"view",'
        '"event_time":"1700000020001"  }' % a1,                                     # whitespace variants
        ev(extra=', "x": 1.5e3, "y": true, "z": null, "w": {"a": [1, "b\\"c", {}], "k": -0.25}'),
        ev(extra=', "ip2": false, "arr": [], "obj": {}'),
        '{"user_id": "u", "page_id": "p", "ad_id": "%s", "event_type": "view", "event_time": "1700000000001"}'
        % a0,                                                                           # ad_type missing
        ev(et="5").replace('"event_type": "5"', '"event_type": 5'),                    # non-string
        ev(extra=', "ad_id": "%s"' % a1),                                             # duplicate key
        ev(et="vi\\u0065w", t="1700000030000"),                                      # escaped value
        ev(ad=esc_ad, t="1700000030001"),                                             # escaped ad id
        ev(t="1700000030002").replace('"ad_id"', '"ad\\u005fid"'),                    # escaped key
        ev(user="a\\/b\\\\c", page='x\\", \\"ad_id\\": \\"fake', t="1700000030003"),  # quotes inside a value
        ev(et="View"), ev(et="view "), ev(et="viewx"), ev(et=""),
        ev(ad="not-an-ad"), ev(ad=a0.upper()), ev(ad=a0 + " "),                     # misses
        ev(t="-5"), ev(t="-15000"), ev(t="+1700000040000"), ev(t="0001700000040001"),
        ev(t="9223372036854775807"), ev(t="-9223372036854775808"),
        ev(t="17e3"), ev(t=""), ev(t="9223372036854775808"), ev(t=" 1700000000000"), ev(t="1.5"),
        ev(ad="missing-ad", t="bogus"),                                               # miss: time never parsed
        ev(et="click", t="bogus"),                                                    # not a view: same
        ev()[:-1],                                                                    # missing closing brace
        ev()[:-1] + ",}",                                                             # trailing comma
        ev().replace('"', "'"),                                                       # single quotes
        "",                                                                           # empty line
        "[]",
        ev() + " x",                                                                  # trailing garbage
        '{"user_id": "u',                                                             # unterminated string
        ev(extra=', "n": NaN'),
        ev(extra=', "e": "\\x"'),                                                     # invalid escape
        ev(t="1700000050000") + "\r",                                                 # CRLF line ending
        ev(user="tab\there", t="1700000050001"),                                      # raw control char
        ev(user="héllo €", t="1700000050002"),                              # non-ASCII UTF-8
        ev(extra=', "x": 1, "x": 2', t="1700000050003"),                              # dup unrecognised key
        ev(t="1700000050004").replace('"ip_address": "1.2.3.4"', '"ip_address": 5'),  # non-string ip
        ev(t="1700000050005").replace('"ip_address": "1.2.3.4"', '"ip_address": "1.2.3.4", "ip_address": "x"'),
        '{}',
        '   {"user_id": "u", "page_id": "p", "ad_id": "%s", "ad_type": "a", "event_type": "view", '
        '"event_time": "1700000060000"}   ' % a2,
    ]
    return [ln.encode("utf-8") + b"\n" for ln in L]


def long_lines(ads):
    a0 = ads[3]
    big = "z" * 70000
    out = []
    for k in range(40):
        out.append(('{"user_id": "u%d", "page_id": "p", "ad_id": "%s", "ad_type": "mail", "event_type": "view", '
                    '"event_time": "%d"}\n' % (k, a0, 1_700_000_000_000 + 997 * k)).encode())
    out.insert(17, ('{"user_id": "%s", "page_id": "p", "ad_id": "%s", "ad_type": "mail", "event_type": "view", '
                    '"event_time": "1700000100000"}\n' % (big, a0)).encode())
    return out


def to_tbl(json_line: bytes) -> bytes:
    ev = json.loads(json_line)
    return ("|".join(ev[k] for k in ("user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time"))
            + "\n").encode()


def tbl_edge_lines(ads):
    a0, a1 = ads[0], ads[7]
    L = [
        "u|p|%s|banner|view|1700000000000" % a0,               # no terminator (last line style)
        "u|p|%s|banner|view|1700000009999\r" % a0,             # \r\n terminator
        "u|p|%s|banner|view|1700000010000|extra|fields" % a0,  # more than 6 items
        "u|p|%s|banner|view|" % a0,                            # trailing empty dropped: 5 items
        "u|p|%s|banner|view||" % a0,                           # still 5 after the drop
        "u|p|%s|banner|view||x" % a0,                          # items[5] = "" -> parseLong throws
        "u|p|%s|banner|view" % a0,                             # 5 items
        "|p|%s||view|1700000020000" % a1,                      # empty items kept
        "u|p|%s|banner|View|1700000020000" % a1,               # case-sensitive filter
        "u|p|%s|banner|click|1700000020000" % a1,
        "u|p|nope|banner|view|1700000020000",                  # join miss
        "u|p|%s|banner|view|+1700000030000" % a1,              # Long.parseLong accepts '+'
        "u|p|%s|banner|view|-5" % a1,                          # bucket 0 (truncation)
        "u|p|%s|banner|view|-10001" % a1,                      # bucket -1
        "u|p|%s|banner|view|17e3" % a1,                        # time error
        "u|p|%s|banner|view|9223372036854775807" % a1,         # Long.MAX_VALUE
        "u|p|%s|banner|view|9223372036854775808" % a1,         # overflow -> time error
        "",                                                    # empty line
        "||||||",                                              # all empty
        "u|p|%s |banner|view|1700000040000" % a1,              # key with a space: miss
        "u|p|%s|banner|view|1700000040000|" % a1,              # trailing '|' after items[5]
    ]
    return [ln.encode() + b"\n" for ln in L]


def orgjson_lines(ads):
    a0, a1, a2 = ads[0], ads[11], ads[57]
    U = "0f8c1e7a-1111-4222-8333-944455556666"

    def ev(t, ad=a0, et="view", at="banner", ip="1.2.3.4", extra=""):
        return ('{"user_id": "%s", "page_id": "p", "ad_id": "%s", "ad_type": %s, "event_type": %s, '
                '"event_time": %s, "ip_address": %s%s}' % (U, ad, at if at[:1] in "'\"" or at == "" else '"%s"' % at,
                                                          et if et[:1] in "'\"" else '"%s"' % et,
                                                          t if t[:1] in "'\"" else '"%s"' % t,
                                                          ip if ip[:1] in "'\"" else '"%s"' % ip, extra))

    def raw(at="banner", et="view", t="1700000100000", ip="1.2.3.4", ad=None, extra=""):
        """unquoted values spliced in as given"""
        return ('{"user_id": "u", "page_id": "p", "ad_id": "%s", "ad_type": %s, "event_type": %s, '
                '"event_time": %s, "ip_address": %s%s}' % (ad or a1, at, et, t, ip, extra))

    deep = "".join('{"k%d": ' % k for k in range(40)) + '"x"' + "}" * 40
    L = [
        # unquoted text (nextValue's unquoted branch; stringToValue leaves a String)
        "{user_id: u, page_id: p, ad_id: %s, ad_type: banner, event_type: view, event_time: 01700000100000}" % a0,
        "{user_id: u, page_id: p, ad_id: %s, ad_type: banner, event_type: view, event_time: 1700000100000}" % a0,
        raw(et="view  ", t="'1700000100001'"),                    # trailing spaces trimmed
        raw(et="vi ew", t="'1700000100002'"),                      # inner space kept
        raw(et="VIEW", t="'1700000100003'"),
        raw(et="true", t="'1700000100004'"),                       # Boolean: not a string
        raw(et="nULl", t="'1700000100005'"),                       # JSONObject.NULL
        raw(at="1.5", t="'1700000100006'"),                        # Double
        raw(at="1e400", t="'1700000100007'"),                      # infinite: stays a String
        raw(at="0x1p1", t="'1700000100008'"),                      # not decimal notation, not a Long
        raw(at="0x1.8p1", t="'1700000100009'"),                    # hex Double
        raw(at="-0", t="'1700000100010'"),                         # Double -0.0
        raw(at="007", t="'1700000100011'"),                        # Long.toString != text: String
        raw(at="9223372036854775808", t="'1700000100012'"),        # beyond Long: String
        raw(at="-9223372036854775808", t="'1700000100013'"),       # Long.MIN_VALUE
        raw(at="1.5f", t="'1700000100014'"),                       # Double (suffix)
        raw(at="1e", t="'1700000100015'"),                         # bad exponent: String
        raw(at="fal\u017fe", t="'1700000100016'"),   # long s folds to S
        raw(at="1.7976931348623157e308", t="'1700000100017'"),     # Double.MAX_VALUE
        raw(at="1.7976931348623159e308", t="'1700000100018'"),     # rounds to Infinity
        raw(t="1700000100019"),                                    # Long event_time: not a string
        raw(t="1.700000100019e12"),                                # Double event_time
        raw(t="+1700000100020"),                                   # '+' first: String, parseLong ok
        raw(ip="1.2.3.4", t="'1700000100021'"),                    # unquoted ip: a String
        raw(ip="1.5", t="'1700000100022'"),                        # Double ip (require_ip only)
        raw(ip="[1, 2]", t="'1700000100023'"),
        raw(ad="'%s'" % a2, t="'1700000100024'").replace('"ad_id": "\'', '"ad_id": \'').replace("'\", \"ad_type", "', \"ad_type"),
        # single quotes, escapes
        ev("'1700000110000'", et="'view'", at="'mail'"),
        ev("1700000110001", et="vi\\u0065w"),
        ev("1700000110002", et="vi\\u+065w"),                    # Integer.parseInt accepts a sign
        ev("1700000110003", et="vi\\u-065w"),                    # (char)-0x65 = U+FF9B
        ev("1700000110004", extra=', "q": "it\\\'s"'),          # \' is an org.json escape
        ev("1700000110005", extra=", 'q': \"a'b\", 'r': 'a\"b'"),  # the other quote is plain text
        ev("1700000110006", extra=', "q": "\\x"'),               # illegal escape
        ev("1700000110007", extra=', "q": "\\u12g4"'),
        ev("1700000110008", extra=', "q": "a\x01b\x7fc"'),       # raw C0 / DEL inside strings: kept
        # separators and structure
        ev("1700000120000").replace(", ", "; "),                    # ';' between pairs
        ev("1700000120001")[:-1] + ";}",                            # trailing ';'
        ev("1700000120002")[:-1] + ",,}",                           # empty pair: Missing value
        ev("1700000120003") + "}}}",                                # text after the object is never read
        ev("1700000120004") + ' {"more": ',
        ev("1700000120005").replace('"ad_type":', '"ad_type" ='),  # '=' is not a key separator
        ev("1700000120006").replace('"ad_type": "banner"', '"ad_type": "banner" "x"'),
        "x" + ev("1700000120007"),                                  # text before '{'
        "\x01\x1f" + ev("1700000120008").replace(", ", ",\x02\x0b"),   # all C0 chars are whitespace
        ev("1700000120009", extra=', "a": [,1,,]'),                 # empty array slots are nulls
        ev("1700000120010", extra=', "a": [1;2]'),                  # ';' does not separate array items
        ev("1700000120011", extra=', "a": [1, [2, {"b": [3]}],]'),
        ev("1700000120012", extra=', "a": #'),                      # '#' ends unquoted text: Missing value
        ev("1700000120013", extra=", \"a\": b/c"),                 # '/' ends unquoted text
        ev("1700000120014", extra=', "": 1, "n": null'),
        ev("1700000120015", extra=', "d": ' + deep),                # 41 levels of nesting
        # keys
        '{user_id: "u", page_id: "p", ad_id: "%s", ad_type: "t", event_type: "view", event_time: "1700000130000"}' % a2,
        "{'user_id': 'u', 'page_id': 'p', 'ad_\\u0069d': '%s', 'ad_type': 't', 'event_type': 'view', "
        "'event_time': '1700000130001'}" % a2,
        ev("1700000130002", extra=', {"k": 1}: 2, [3]: 4, 5: 6'),  # container / number keys
        # duplicate keys: org.json throws for any repeated key, at any level
        ev("1700000140000", extra=', "x": 1, "x": 2'),
        ev("1700000140001", extra=', "x": 1, x: 2'),
        ev("1700000140002", extra=', "1": 1, 1: 2'),                # Integer 1 -> "1"
        ev("1700000140003", extra=', "true": 1, TRUE: 2'),          # Boolean.TRUE -> "true"
        ev("1700000140004", extra=', "null": 1, Null: 2'),
        ev("1700000140005", extra=', "w": {"a": 1, "a": 2}'),       # nested
        ev("1700000140006", extra=', "w": [{"a": 1}, {"a": 2}]'),   # different objects: fine
        ev("1700000140007", extra=', "w": {"ad_id": "x", "event_type": 1}'),   # other object's keys
        ev("1700000140008", extra=', "q\\u0031": 1, "q1": 2'),
        ev("1700000140009", extra=', "01": 1, 01: 2'),              # "01" stays a String
        # NUL is the end of input; a raw CR / LF inside a string throws
        ev("1700000150000") + "\x00garbage",
        ev("1700000150001").replace('"p"', '"p\x00"'),
        ev("1700000150002").replace('"p"', '"p\rq"'),
        ev("1700000150003").replace('"banner"', "banner\x00"),
        "{" + "\x00",
        "{'user_id': 'u",
        "{\"a\": [",
        "{\"a\": b",
    ]
    return [ln.encode("utf-8", errors="surrogatepass") + b"\n" for ln in L]


def write_expected(stem, lines, ad_map, campaign_of, require_ip=False, fmt="json"):
    lines, _ = dostats.split_lines(b"".join(lines))   # the records readLine yields from the file
    r = dostats.run(lines, ad_map, 10000, require_ip, fmt)
    suffix = ".ip" if require_ip else ""
    with open(os.path.join(HERE, stem + suffix + ".expected.csv"), "w") as f:
        f.write("campaign_id,window_ms,count\n")
        for (camp, b), v in sorted(r.counts.items(), key=lambda kv: (campaign_of[kv[0][0]], kv[0][1])):
            f.write("%s,%d,%d\n" % (camp, b * 10000, v))
    with open(os.path.join(HERE, stem + suffix + ".expected.json"), "w") as f:
        json.dump(r.stats(), f, indent=1, sort_keys=True)
        f.write("\n")
    return r


def main():
    g = PyGen(**GEN)
    camps, ads = g.campaigns(), g.ads()
    ad_map = {a: camps[i // GEN["ads_per_campaign"]] for i, a in enumerate(ads)}
    campaign_of = {c: i for i, c in enumerate(camps)}
    with open(os.path.join(HERE, "gen_s7.campaign_ids.txt"), "w") as f:
        f.write("".join(c + "\n" for c in camps))
    with open(os.path.join(HERE, "gen_s7.ad_to_campaign.txt"), "w") as f:
        f.write("".join('{ "%s": "%s"}\n' % (a, ad_map[a]) for a in ads))
    with open(os.path.join(HERE, "gen_s7.ad_to_campaign.csv"), "w") as f:
        f.write("".join("%s,%s\n" % (a, ad_map[a]) for a in ads))
    gen = [g.line(i).encode() for i in range(N_GEN)]
    with open(os.path.join(HERE, "gen_s7.jsonl"), "wb") as f:
        f.write(b"".join(gen))
    write_expected("gen_s7", gen, ad_map, campaign_of)
    edge = edge_lines(ads, camps)
    with open(os.path.join(HERE, "edge.jsonl"), "wb") as f:
        f.write(b"".join(edge))
    write_expected("edge", edge, ad_map, campaign_of)
    write_expected("edge", edge, ad_map, campaign_of, require_ip=True)
    oj = orgjson_lines(ads)
    with open(os.path.join(HERE, "edge_orgjson.jsonl"), "wb") as f:
        f.write(b"".join(oj))
    write_expected("edge_orgjson", oj, ad_map, campaign_of)
    write_expected("edge_orgjson", oj, ad_map, campaign_of, require_ip=True)
    lng = long_lines(ads)
    with open(os.path.join(HERE, "edge_long.jsonl"), "wb") as f:
        f.write(b"".join(lng))
    write_expected("edge_long", lng, ad_map, campaign_of)
    tbl = [to_tbl(ln) for ln in gen]
    with open(os.path.join(HERE, "gen_s7.tbl"), "wb") as f:
        f.write(b"".join(tbl))
    write_expected("gen_s7_tbl", tbl, ad_map, campaign_of, fmt="tbl")
    et = tbl_edge_lines(ads)
    with open(os.path.join(HERE, "edge_tbl.tbl"), "wb") as f:
        f.write(b"".join(et))
    write_expected("edge_tbl", et, ad_map, campaign_of, fmt="tbl")
    with open(os.path.join(HERE, "gen_s7.params.json"), "w") as f:
        json.dump(dict(GEN, n_events=N_GEN), f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
