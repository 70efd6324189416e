"""Seeded generator of event lines that exercise org.json 20180813's grammar (quoting
styles, separators, escapes, unquoted-text typing, duplicate keys, nesting, truncation,
NUL / control bytes).  Used by tests/test_orgjson.py (C oracle vs Python restatement)
and tests/test_gpu_parity.py (GPU vs C oracle)."""
from __future__ import annotations

import random

FIELDS = ("user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time", "ip_address")

_TOKENS = ["true", "False", "NULL", "nuLl", "1", "-1", "01", "-0", "0", "1.5", "1e5", "1e400", "1.", "-.5",
           "0x1p3", "0x1.8p1", "0xEp1", "1.5f", "1d", "1e", "NaN", "-Infinity", "9223372036854775807",
           "9223372036854775808", "-9223372036854775808", "+5", "abc", "a b", "it's", "view", "VIEW",
           "fal\u017fe", "1.7976931348623159e308", "\u00e9t\u00e9"]
_ESCAPES = ["\\n", "\\t", "\\\\", "\\/", '\\"', "\\'", "\\u0041", "\\u+041", "\\u-041", "\\u00e9", "\\ud83d\\ude00",
            "\\ud83d", "\\ude00", "\\x", "\\u12", "\\u12g4", "\\0", "\\"]


def _str(rng, text, quote=None):
    """text as a quoted string (escapes sprinkled in) or unquoted."""
    q = quote or rng.choice(['"', '"', '"', "'", ""])
    if q == "" and not rng.wild and (not text or any(c in ',:]}/\\"[{;=#' for c in text)):
        q = '"'
    if q == "":
        return text
    if rng.random() < rng.wild * 0.3:
        k = rng.randrange(len(text) + 1)
        text = text[:k] + rng.choice(_ESCAPES) + text[k:]
    other = "'" if q == '"' else '"'
    if rng.random() < 0.05:
        text = text + other
    return q + text.replace(q, "\\" + q) + q


def _value(rng, depth, ctx):
    r = rng.random()
    if r < 0.55:
        return _str(rng, rng.choice(ctx["misc"]))
    if r < 0.75:
        return rng.choice(_TOKENS)
    if depth < 3 and r < 0.88:
        return _object(rng, depth + 1, ctx, top=False)
    if depth < 3:
        items = [_value(rng, depth + 1, ctx) if rng.random() < 0.85 else "" for _ in range(rng.randrange(4))]
        return "[" + rng.choice([", ", ","]).join(items) + rng.choice(["", ",", " "]) + "]"
    return _str(rng, "x")


def _object(rng, depth, ctx, top):
    keys = list(FIELDS[:6] if rng.random() < 0.7 else FIELDS) if top else []
    rng.shuffle(keys) if rng.random() < 0.3 else None
    for _ in range(rng.randrange(3) if rng.wild or not top else 0):
        keys.insert(rng.randrange(len(keys) + 1), rng.choice(["x", "y", "1", "true", "", "ad_id", "w"]))
    if top and rng.random() < 0.08:
        keys.append(rng.choice(FIELDS))
    pairs = []
    for k in keys:
        ks = _str(rng, k) if rng.random() > rng.wild * 0.1 else rng.choice(["1", "TRUE", "null", "{}", "[1]"])
        if top and k in ctx["fields"]:
            v = _str(rng, rng.choice(ctx["fields"][k])) if rng.random() > rng.wild * 0.3 else rng.choice(_TOKENS)
        else:
            v = _value(rng, depth, ctx)
        sep = rng.choice([": ", ":", " : ", ":", "\t:\x01", ": "])
        pairs.append(ks + sep + v)
    body = rng.choice([", ", ",", ", ", "; ", " ,\x1f"]).join(pairs)
    tail = rng.choice(["", "", "", ",", ";", " ", ",,"] if rng.wild else ["", ",", ";", " "])
    lead = rng.choice(["", "", "", " ", "\x02", "x"] if rng.wild else ["", " ", "\x02"])
    after = rng.choice(["", "", "", "", " x", "}", "\x00junk", "{"])
    return lead + "{" + body + tail + "}" + after


class _Rng(random.Random):
    wild = 0.0


def lines(seed, n, ads, times=None):
    """n event lines (bytes, '\\n'-terminated); ads: ad ids that join."""
    rng = _Rng(seed)
    times = times or [str(1_700_000_000_000 + 997 * k) for k in range(50)] + ["+1700000000000", "0001", "-5", "1e3"]
    ctx = {
        "fields": {
            "user_id": ["u", "0f8c1e7a-1111-4222-8333-944455556666", ""],
            "page_id": ["p", "page"],
            "ad_id": list(ads[:20]) + ["nope", ads[0].upper(), ads[1] + " "],
            "ad_type": ["banner", "mail"],
            "event_type": ["view"] * 6 + ["click", "View", "view "],
            "event_time": times,
            "ip_address": ["1.2.3.4"],
        },
        "misc": ["a", "b c", "view", "", "\u00e9", "q\"r"],
    }
    out = []
    for _ in range(n):
        rng.wild = 1.0 if rng.random() < 0.4 else 0.0              # 60 % of lines mostly well-formed
        s = _object(rng, 1, ctx, top=True)
        r = rng.random()
        if r < 0.04:
            s = s[: rng.randrange(len(s) + 1)]                       # truncated
        elif r < 0.06:
            k = rng.randrange(len(s) + 1)
            s = s[:k] + rng.choice(["\x00", "\r", "\x7f", "\u00ff"]) + s[k:]
        out.append(s.replace("\n", "\\n").encode("utf-8", errors="surrogatepass") + b"\n")
    return out
