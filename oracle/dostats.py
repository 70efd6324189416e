"""Second CPU restatement of the YSB hot path, in Python.

TEST INFRASTRUCTURE ONLY (imported by tests/ and tests/golden/make_golden.py); the
product never imports it.  Parity status: UNPINNED against the reference itself --
the reference is Java/Clojure, cannot run here, and ships no golden vectors
(data/test/setup/core_test.clj:8-10 always fails).  It exists to pin
oracle/ysb_oracle.c through an independent implementation.

It follows:
  dostats                 data/src/setup/core.clj:101-128   (campaign -> bucket -> count)
  DeserializeBolt         flink-benchmarks/.../AdvertisingTopologyNative.java:263-272
                          new JSONObject(line) + getString x6: oracle/orgjson.py (org.json
                          20180813).  parse_event_strict is the Jackson-style strict view
                          dostats itself reads the file with (clj-json 0.5.3, core.clj:103);
                          on the generator's lines the two agree (tests/test_orgjson.py).
  EventFilterBolt         :434              event_type.equals("view")
  RedisJoinBolt           :461-474          map miss -> drop (dostats instead counts
                                            under a nil campaign, core.clj:112; the
                                            Flink chain is the drop-in target)
  CampaignProcessorCommon streaming-benchmark-common/.../CampaignProcessorCommon.java:57-60
                          bucket = Long.parseLong(event_time) / 10000 (truncating)
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field

from oracle import orgjson

REQUIRED_FLINK = ("user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time")
RECOGNISED = REQUIRED_FLINK + ("ip_address",)
_LONG = re.compile(r"[+-]?[0-9]+\Z")
_TERM = re.compile(rb"\r\n|\r|\n")


class ParseError(Exception):
    pass


def _reject_constant(name):  # NaN / Infinity are not JSON
    raise ParseError(name)


def parse_event(line: bytes, require_ip: bool = False) -> dict:
    """new JSONObject(line) + getString of the required fields (org.json 20180813,
    oracle/orgjson.py); raises ParseError where DeserializeBolt would throw."""
    try:
        obj = orgjson.parse_object(line)
    except (orgjson.JSONException, RecursionError) as e:
        raise ParseError(str(e)) from None
    out = {}
    for k in (RECOGNISED if require_ip else REQUIRED_FLINK):
        v = orgjson.string_value(obj.get(k.encode()))
        if v is None:
            raise ParseError("JSONObject[%s] not a string." % k)
        out[k] = v.decode("utf-8", errors="surrogateescape")
    return out


def parse_event_strict(line: bytes, require_ip: bool = False) -> dict:
    """The strict (RFC 8259, Jackson-style) reading of a line: dostats' own view of the
    generator's file; raises ParseError on malformed JSON, a duplicate recognised key or
    a missing / non-string field."""
    text = line.decode("utf-8", errors="surrogateescape")
    if not text.lstrip(" \t\n\r").startswith("{"):
        raise ParseError("not an object")
    try:
        pairs = json.loads(text, strict=False, object_pairs_hook=lambda p: p,
                           parse_constant=_reject_constant)
    except (ValueError, RecursionError) as e:
        raise ParseError(str(e)) from None
    out = {}
    for k, v in pairs:
        if k in RECOGNISED:
            if k in out:
                raise ParseError("Duplicate key " + k)
            out[k] = v
    required = RECOGNISED if require_ip else REQUIRED_FLINK
    for k in required:
        if not isinstance(out.get(k), str):
            raise ParseError("JSONObject[%s] not a string." % k)
    return out


def parse_tbl(line: bytes) -> dict:
    """MockWindowedFlatMap (AdvertisingTopologyNative.java:197-226): readLine, then
    line.split("\\|") with Java's limit-0 semantics (trailing empty items dropped);
    items[5] missing -> ParseError (ArrayIndexOutOfBounds)."""
    text = line.decode("utf-8", errors="surrogateescape")
    if text.endswith("\n"):
        text = text[:-1]
    if text.endswith("\r"):
        text = text[:-1]
    items = text.split("|")
    while items and items[-1] == "":
        items.pop()
    if len(items) < 6:
        raise ParseError("ArrayIndexOutOfBounds")
    return dict(zip(("user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time"), items[:6]))


def parse_long(s: str) -> int:
    """java.lang.Long.parseLong for ASCII input."""
    if not _LONG.match(s):
        raise ValueError(s)
    v = int(s)
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError(s)
    return v


def java_div(t: int, d: int) -> int:
    q = abs(t) // d
    return -q if t < 0 else q


@dataclass
class Result:
    counts: dict = field(default_factory=dict)   # (campaign, bucket) -> count
    events: int = 0
    views: int = 0
    joined: int = 0
    join_misses: int = 0
    parse_errors: int = 0
    time_errors: int = 0

    def stats(self) -> dict:
        return {k: getattr(self, k) for k in
                ("events", "views", "joined", "join_misses", "parse_errors", "time_errors")}


def run(lines, ad_to_campaign: dict, divisor: int = 10000, require_ip: bool = False, fmt: str = "json",
        strict: bool = False) -> Result:
    """lines: iterable of bytes (one event each); ad_to_campaign: str -> campaign key;
    fmt "json" (DeserializeBolt, org.json) or "tbl" (MockWindowedFlatMap's .tbl rows);
    strict=True reads JSON with parse_event_strict instead."""
    r = Result()
    parse = parse_event_strict if strict else parse_event
    for line in lines:
        r.events += 1
        try:
            ev = parse_tbl(line) if fmt == "tbl" else parse(line, require_ip)
        except ParseError:
            r.parse_errors += 1
            continue
        if ev["event_type"] != "view":
            continue
        r.views += 1
        campaign = ad_to_campaign.get(ev["ad_id"])
        if campaign is None:
            r.join_misses += 1
            continue
        r.joined += 1
        try:
            t = parse_long(ev["event_time"])
        except ValueError:
            r.time_errors += 1
            continue
        key = (campaign, java_div(t, divisor))
        r.counts[key] = r.counts.get(key, 0) + 1
    return r


def load_ad_map_json_lines(data: bytes) -> dict:
    """ad-to-campaign-ids.txt: `{ "AD": "CAMPAIGN"}` per line, merged left to right
    (core.clj:58 writes it, core.clj:104-106 reads it with reduce merge)."""
    m = {}
    for ln in data.splitlines():
        if ln.strip():
            m.update(json.loads(ln.decode("utf-8")))
    return m


def load_ad_map_csv(data: bytes) -> dict:
    """ad,campaign per line, kv[0] -> kv[1], later wins (AdvertisingTopologyNative.java:47-56)."""
    m = {}
    for ln in data.decode("utf-8").splitlines():
        kv = ln.split(",")
        m[kv[0]] = kv[1]
    return m


def split_lines(data: bytes):
    """Lines as the reference's BufferedReader.readLine cuts them (AdvertisingTopologyNative.
    java:153-159): "\\n", "\\r\\n" and a lone "\\r" end a line; each line keeps its
    terminator bytes.  Returns (lines, offsets): line i spans [off[i], off[i+1])."""
    offs, lines, p = [], [], 0
    n = len(data)
    for m in _TERM.finditer(data):
        offs.append(p)
        lines.append(data[p:m.end()])
        p = m.end()
    if p < n:
        offs.append(p)
        lines.append(data[p:])
    return lines, offs
