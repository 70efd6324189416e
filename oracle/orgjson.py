"""CPU restatement of org.json 20180813 as DeserializeBolt uses it: `new JSONObject(line)`
then `getString` of the event fields.

TEST INFRASTRUCTURE ONLY (imported by tests/, oracle/dostats.py and
tests/golden/make_golden.py); the product never imports it.

The library is a third-party dependency absent from /root/reference:
  org.json:json:20180813   (pom.xml:20,24,76-79; flink-benchmarks/pom.xml:25-27)
Call sites it serves: AdvertisingTopologyNative.java:263-272 (DeserializeBolt),
storm-benchmarks/.../AdvertisingTopology.java:55-62, AdvertisingSpark.scala:125-133.
Parity status: UNPINNED -- no JDK here and the reference holds no vectors at the JSON
boundary; this file restates the library's published algorithm (JSONTokener.next /
nextClean / nextString / nextValue, JSONObject(JSONTokener), JSONArray(JSONTokener),
JSONObject.stringToValue, JSONObject.getString), and oracle/ysb_oracle.c restates the
same rules independently in C.

Model: the input is the line's bytes; every structural character is ASCII and every
non-ASCII byte is >= ' ' and not a delimiter, exactly as Java's non-ASCII chars are, so
working on UTF-8 bytes gives the same token boundaries as Java's UTF-16 chars.
Decoded strings are compared as UTF-8, with code units from \\u escapes combined into
one code point when a high surrogate is immediately followed by a low one (Java string
equality over valid UTF-8 input).  The rules:

  * A NUL byte acts as end of input (JSONTokener.next returns 0 and sets eof for it).
  * nextClean skips every char <= ' ' (all C0 controls, not only JSON whitespace).
  * Strings open with '"' or '\\''; escapes b t n f r u " ' \\\\ /; anything else after
    a backslash throws; a raw CR or LF or the end of input inside a string throws.
    \\uXXXX is Integer.parseInt(next(4), 16): an optional sign then hex digits, cast
    to char (\\u-001 is U+FFFF).
  * Unquoted text runs while c >= ' ' and c is not one of  , : ] } / \\\\ " [ { ; = #
    (spaces included), then String.trim(); empty -> "Missing value".  stringToValue
    turns it into Boolean / NULL (equalsIgnoreCase true/false/null), Integer/Long
    (Long.valueOf round-trips exactly), Double (decimal notation: '.', 'e', 'E' or "-0",
    Double.valueOf accepts it and it is finite) or else a String.
  * Objects: '{', then pairs `key : value` separated by ',' or ';'; a separator may be
    followed directly by '}' (trailing comma); the key is nextValue().toString(); any
    repeated key throws "Duplicate key"; text after the closing '}' is never read.
  * Arrays: '[' ... ']', ',' separated, an empty slot is a null, "[1,]" closes.
  * getString: the value must exist and be a String (quoted or unquoted text that
    stringToValue leaves a String).

Documented limits: keys that are Doubles or nested containers are
compared by their source text (Java compares Double.toString / JSONObject.toString,
which are JDK- and HashMap-order dependent); nesting deeper than MAX_DEPTH throws here
(Java's limit is the thread stack); a \\uXXXX escape whose four chars are non-ASCII
Unicode digits is rejected (Character.digit would accept them).  Whenever Java reads
past the end of input and then steps back, every continuation of the parse throws, so
that case throws immediately here.
"""
from __future__ import annotations

MAX_DEPTH = 64

_DELIM = frozenset(b',:]}/\\"[{;=#')
_QUOTES = (0x22, 0x27)
_SIMPLE_ESC = {0x62: 8, 0x74: 9, 0x6E: 10, 0x66: 12, 0x72: 13, 0x22: 0x22, 0x27: 0x27, 0x5C: 0x5C, 0x2F: 0x2F}
_HEXV = {c: int(chr(c), 16) for c in b"0123456789abcdefABCDEF"}

# 2**1024 - 2**970: the midpoint between Double.MAX_VALUE and 2**1024.  A decimal at or
# above it rounds (half-even; MAX_VALUE's significand is odd) to Infinity.
_DBL_HALF = (1 << 1024) - (1 << 970)


class JSONException(Exception):
    pass


class _Tok:
    """JSONTokener over one line."""
    __slots__ = ("s", "n", "p", "eof")

    def __init__(self, s: bytes):
        z = s.find(b"\0")
        self.s = s if z < 0 else s[:z]
        self.n = len(self.s)
        self.p = 0
        self.eof = False

    def next(self) -> int:
        if self.p >= self.n:
            self.eof = True
            return -1
        self.eof = False
        c = self.s[self.p]
        self.p += 1
        return c

    def back(self):
        if self.eof:
            raise JSONException("end of input")
        self.p -= 1

    def next_clean(self) -> int:
        while True:
            c = self.next()
            if c < 0 or c > 0x20:
                return c

    def next_string(self, quote: int) -> bytes:
        out = bytearray()
        pend = -1   # a high surrogate from \\u waiting for its low half

        def flush():
            nonlocal pend
            if pend >= 0:
                _put_cp(out, pend)
                pend = -1

        while True:
            c = self.next()
            if c < 0 or c == 0x0A or c == 0x0D:
                raise JSONException("Unterminated string")
            if c == 0x5C:
                c = self.next()
                if c == 0x75:   # 'u'
                    u = _parse_hex4(self)
                    if pend >= 0 and 0xDC00 <= u < 0xE000:
                        _put_cp(out, 0x10000 + ((pend - 0xD800) << 10) + (u - 0xDC00))
                        pend = -1
                        continue
                    flush()
                    if 0xD800 <= u < 0xDC00:
                        pend = u
                    else:
                        _put_cp(out, u)
                    continue
                v = _SIMPLE_ESC.get(c)
                if v is None:
                    raise JSONException("Illegal escape.")
                flush()
                out.append(v)
                continue
            if c == quote:
                flush()
                return bytes(out)
            flush()
            out.append(c)

    def next_value(self, depth: int):
        """-> (kind, payload, start, end): kind 'str' (decoded bytes), 'tok' (trimmed
        unquoted text), 'obj' (dict of key -> (kind, payload)) or 'arr'."""
        c = self.next_clean()
        if c in _QUOTES:
            a = self.p - 1
            v = self.next_string(c)
            return "str", v, a, self.p
        if c == 0x7B:   # '{'
            self.back()
            a = self.p
            v = self.object(depth + 1)
            return "obj", v, a, self.p
        if c == 0x5B:   # '['
            self.back()
            a = self.p
            self.array(depth + 1)
            return "arr", None, a, self.p
        a = self.p - 1 if c >= 0 else self.p
        while c >= 0x20 and c not in _DELIM:
            c = self.next()
        self.back()
        tok = self.s[a:self.p].rstrip(b" ")
        if not tok:
            raise JSONException("Missing value")
        return "tok", tok, a, self.p

    def object(self, depth: int) -> dict:
        if depth > MAX_DEPTH:
            raise JSONException("nesting")
        if self.next_clean() != 0x7B:
            raise JSONException("A JSONObject text must begin with '{'")
        fields = {}
        while True:
            c = self.next_clean()
            if c < 0:
                raise JSONException("A JSONObject text must end with '}'")
            if c == 0x7D:
                return fields
            self.back()
            kind, val, a, b = self.next_value(depth)
            key = _key_text(kind, val, self.s[a:b])
            if self.next_clean() != 0x3A:
                raise JSONException("Expected a ':' after a key")
            if key in fields:
                raise JSONException("Duplicate key")
            vkind, vval, _, _ = self.next_value(depth)
            fields[key] = (vkind, vval)
            c = self.next_clean()
            if c == 0x2C or c == 0x3B:
                if self.next_clean() == 0x7D:
                    return fields
                self.back()
            elif c == 0x7D:
                return fields
            else:
                raise JSONException("Expected a ',' or '}'")

    def array(self, depth: int):
        if depth > MAX_DEPTH:
            raise JSONException("nesting")
        if self.next_clean() != 0x5B:
            raise JSONException("A JSONArray text must start with '['")
        if self.next_clean() == 0x5D:
            return
        self.back()
        while True:
            if self.next_clean() == 0x2C:
                self.back()                 # an empty slot: JSONObject.NULL
            else:
                self.back()
                self.next_value(depth)
            c = self.next_clean()
            if c == 0x2C:
                if self.next_clean() == 0x5D:
                    return
                self.back()
            elif c == 0x5D:
                return
            else:
                raise JSONException("Expected a ',' or ']'")


def _put_cp(out: bytearray, cp: int):
    """One code point (or lone surrogate unit) as UTF-8 (3-byte form for surrogates)."""
    if cp < 0x80:
        out.append(cp)
    elif cp < 0x800:
        out += bytes((0xC0 | cp >> 6, 0x80 | cp & 0x3F))
    elif cp < 0x10000:
        out += bytes((0xE0 | cp >> 12, 0x80 | cp >> 6 & 0x3F, 0x80 | cp & 0x3F))
    else:
        out += bytes((0xF0 | cp >> 18, 0x80 | cp >> 12 & 0x3F, 0x80 | cp >> 6 & 0x3F, 0x80 | cp & 0x3F))


def _parse_hex4(t: _Tok) -> int:
    """(char) Integer.parseInt(next(4), 16)."""
    four = []
    for _ in range(4):
        c = t.next()
        if c < 0:
            raise JSONException("Substring bounds error")
        four.append(c)
    neg = False
    digits = four
    if four[0] in (0x2B, 0x2D):
        neg = four[0] == 0x2D
        digits = four[1:]
    v = 0
    for c in digits:
        h = _HEXV.get(c)
        if h is None:
            raise JSONException("Illegal escape.")
        v = v * 16 + h
    return (-v if neg else v) & 0xFFFF


# ---- JSONObject.stringToValue ---------------------------------------------------------

def _ieq(tok: bytes, word: bytes) -> bool:
    """String.equalsIgnoreCase(word) for the words true / false / null: ASCII case
    folding, plus U+017F (long s, UTF-8 C5 BF) whose upper case is 'S'."""
    t = tok.replace(b"\xc5\xbf", b"s")
    return t.lower() == word


def _java_long_roundtrip(t: bytes) -> bool:
    """Long.valueOf(t) succeeds and Long.toString equals t: canonical decimal in range."""
    neg = t[:1] == b"-"
    d = t[1:] if neg else t
    if not d or not all(0x30 <= c <= 0x39 for c in d):
        return False
    if len(d) > 1 and d[0] == 0x30:
        return False
    if neg and d == b"0":
        return False
    v = int(d)
    return v <= (1 << 63) if neg else v < (1 << 63)


def _java_double_finite(t: bytes) -> bool:
    """Double.valueOf(t) parses (FloatingDecimal.readJavaFormatString) and is finite."""
    i, n = 0, len(t)
    if i < n and t[i] in (0x2B, 0x2D):
        i += 1
    if i + 1 < n and t[i] == 0x30 and t[i + 1] in (0x78, 0x58):
        return _java_hex_finite(t[i + 2:])
    digits = bytearray()
    int_digits = 0
    seen_dot = False
    while i < n:
        c = t[i]
        if 0x30 <= c <= 0x39:
            digits.append(c)
            if not seen_dot:
                int_digits += 1
        elif c == 0x2E and not seen_dot:
            seen_dot = True
        else:
            break
        i += 1
    if not digits:
        return False
    exp = 0
    if i < n and t[i] in (0x65, 0x45):
        i += 1
        sign = 1
        if i < n and t[i] in (0x2B, 0x2D):
            sign = -1 if t[i] == 0x2D else 1
            i += 1
        a = i
        while i < n and 0x30 <= t[i] <= 0x39:
            i += 1
        if i == a:
            return False
        exp = sign * int(t[a:i])
    if i < n and not (i == n - 1 and t[i] in b"fFdD"):
        return False
    # value = 0.d1 d2 ... x 10**mag with d1 the first non-zero digit
    f = next((k for k, c in enumerate(digits) if c != 0x30), None)
    if f is None:
        return True                                  # zero
    mag = int_digits - f + exp
    if mag < 309:
        return True
    if mag > 309:
        return False
    sig = digits[f:].rstrip(b"0")
    h = str(_DBL_HALF).encode()                      # 309 digits
    return sig.ljust(len(h), b"0") < h.ljust(len(sig), b"0")


def _java_hex_finite(t: bytes) -> bool:
    """The hexadecimal branch after "0x": (hex+ '.'? | hex* '.' hex+) [pP] [+-]? digit+ [fFdD]?"""
    i, n = 0, len(t)
    mant = bytearray()
    frac = 0
    seen_dot = False
    while i < n:
        c = t[i]
        if c in _HEXV:
            mant.append(c)
            if seen_dot:
                frac += 1
        elif c == 0x2E and not seen_dot:
            seen_dot = True
        else:
            break
        i += 1
    if not mant or i >= n or t[i] not in (0x70, 0x50):
        return False
    i += 1
    neg = False
    if i < n and t[i] in (0x2B, 0x2D):
        neg = t[i] == 0x2D
        i += 1
    a = i
    while i < n and 0x30 <= t[i] <= 0x39:
        i += 1
    if i == a:
        return False
    if i < n and not (i == n - 1 and t[i] in b"fFdD"):
        return False
    e = int(t[a:i])
    if e > 0x7FFFFFFF:                               # Integer.parseInt overflow: inf / zero
        return neg
    m = int(bytes(mant), 16)
    if m == 0:
        return True
    top = m.bit_length() - 1 + (-e if neg else e) - 4 * frac
    if top != 1023:
        return top < 1023
    L = m.bit_length()
    if L <= 53:
        return True
    # rounds up to 2**1024 only when the top 53 bits are all ones (odd) and the next is set
    return (m >> (L - 54)) != (1 << 54) - 1


def token_kind(tok: bytes) -> str:
    """stringToValue's result type: 'bool', 'null', 'long', 'double' or 'str'."""
    if _ieq(tok, b"true") or _ieq(tok, b"false"):
        return "bool"
    if _ieq(tok, b"null"):
        return "null"
    c0 = tok[0]
    if 0x30 <= c0 <= 0x39 or c0 == 0x2D:
        if b"." in tok or b"e" in tok or b"E" in tok or tok == b"-0":
            if _java_double_finite(tok):
                return "double"
        elif _java_long_roundtrip(tok):
            return "long"
    return "str"


def _key_text(kind: str, val, raw: bytes) -> bytes:
    """key = nextValue().toString() (see the header for the Double / container limit)."""
    if kind == "str":
        return val
    if kind == "tok":
        k = token_kind(val)
        if k == "bool":
            return b"true" if _ieq(val, b"true") else b"false"
        if k == "null":
            return b"null"
        return val
    return raw


def string_value(field) -> bytes | None:
    """getString: the String's bytes, or None where it throws "not a string"."""
    if field is None:
        return None
    kind, val = field
    if kind == "str":
        return val
    if kind == "tok" and token_kind(val) == "str":
        return val
    return None


def parse_object(line: bytes) -> dict:
    """new JSONObject(line): canonical key bytes -> (kind, payload); raises JSONException."""
    return _Tok(line).object(1)
