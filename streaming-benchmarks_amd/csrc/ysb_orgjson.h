// ysb_orgjson.h -- the general-path event parser on the GPU: org.json 20180813's
// `new JSONObject(line)` + `getString` as DeserializeBolt calls them
// (flink-benchmarks/.../AdvertisingTopologyNative.java:263-272; org.json is the
// third-party dependency pom.xml:24 pins).  Included by ysb_scan.hip after the byte
// sources, Span and the key matchers; used by the deferred-line kernel and the ring
// auto-base probe only (the canonical fast path never calls it).
//
// The grammar (same rules as oracle/orgjson.py and oracle/ysb_oracle.c; DESIGN.md
// section 3 lists them and the documented limits):
//   * a NUL byte ends the input; nextClean skips every byte <= ' ';
//   * strings open with '"' or '\''; escapes b t n f r u " ' \ /; a raw CR / LF or the
//     end inside a string throws; \uXXXX is (char) Integer.parseInt(next(4), 16), a
//     leading sign allowed;
//   * unquoted text runs while c >= ' ' and c is none of , : ] } / \ " [ { ; = #, is
//     trimmed, and "" throws; stringToValue types it (Boolean / NULL / Long / Double /
//     String);
//   * objects: pairs separated by ',' or ';', a separator may precede '}', any repeated
//     key throws (keys: decoded strings, "true"/"false"/"null" for those literals, the
//     source text otherwise), nothing after the top-level '}' is read;
//   * arrays: ',' separated, empty slots allowed, "[1,]" closes;
//   * nesting deeper than OJ_MAX_DEPTH throws; reading past the end and stepping back
//     throws at once (every continuation of org.json's parse throws there).
#pragma once

namespace ysb {

constexpr int OJ_MAX_DEPTH = 64;
constexpr int OJ_TOP_KEYS = 16;   // top-level keys checked through hashes (later ones: re-walk)

__device__ __forceinline__ bool oj_delim(u32 c) {
    return c == ',' || c == ':' || c == ']' || c == '}' || c == '/' || c == '\\' || c == '"' || c == '[' ||
           c == '{' || c == ';' || c == '=' || c == '#';
}

// \uXXXX at p (p = the backslash): the UTF-16 unit (char) Integer.parseInt(XXXX, 16).
// The caller has validated the four characters.
template <class S>
__device__ __forceinline__ u32 oj_unit(const S& src, int p) {
    const u32 d0 = src.b(p + 2);
    if (d0 == '+' || d0 == '-') {
        const u32 v = (hex_val(src.b(p + 3)) << 8) | (hex_val(src.b(p + 4)) << 4) | hex_val(src.b(p + 5));
        return d0 == '-' ? (0x10000u - v) & 0xFFFFu : v;
    }
    return (hex_val(d0) << 12) | (hex_val(src.b(p + 3)) << 8) | (hex_val(src.b(p + 4)) << 4) | hex_val(src.b(p + 5));
}

template <class S>
__device__ __forceinline__ bool oj_plain_u(const S& src, int p, int e) {   // "\uXXXX", four hex digits
    return p + 5 < e && src.b(p) == '\\' && src.b(p + 1) == 'u' && is_hex(src.b(p + 2)) && is_hex(src.b(p + 3)) &&
           is_hex(src.b(p + 4)) && is_hex(src.b(p + 5));
}

__device__ __forceinline__ int oj_utf8(u32 cp, u8 (&o)[4]) {   // lone surrogates: 3-byte form
    if (cp < 0x80) { o[0] = (u8)cp; return 1; }
    if (cp < 0x800) { o[0] = (u8)(0xC0 | (cp >> 6)); o[1] = (u8)(0x80 | (cp & 0x3F)); return 2; }
    if (cp < 0x10000) {
        o[0] = (u8)(0xE0 | (cp >> 12)); o[1] = (u8)(0x80 | ((cp >> 6) & 0x3F)); o[2] = (u8)(0x80 | (cp & 0x3F));
        return 3;
    }
    o[0] = (u8)(0xF0 | (cp >> 18)); o[1] = (u8)(0x80 | ((cp >> 12) & 0x3F));
    o[2] = (u8)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (u8)(0x80 | (cp & 0x3F));
    return 4;
}

// One decoded item of the (validated) string content [p, e): writes its UTF-8 bytes to
// o, returns their count and advances p.  A high-surrogate \u escape directly followed
// by a low one is one code point (Java string equality).
template <class S>
__device__ __forceinline__ int oj_decode_one(const S& src, int& p, int e, u8 (&o)[4]) {
    const u32 c = src.b(p);
    if (c != '\\') { o[0] = (u8)c; ++p; return 1; }
    const u32 x = src.b(p + 1);
    if (x != 'u') {
        o[0] = (u8)(x == 'b' ? 8u : x == 't' ? 9u : x == 'n' ? 10u : x == 'f' ? 12u : x == 'r' ? 13u : x);
        p += 2;
        return 1;
    }
    u32 cp = oj_unit(src, p);
    p += 6;
    if (cp >= 0xD800 && cp < 0xDC00 && oj_plain_u(src, p, e)) {
        const u32 lo = oj_unit(src, p);
        if (lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            p += 6;
        }
    }
    return oj_utf8(cp, o);
}

// Decodes the (validated) escaped string [s, e) as UTF-8 into buf (at most cap bytes
// written); returns the full decoded length.
template <class S>
__device__ __noinline__ int decode_str(const S& src, int s, int e, u8* buf, int cap) {
    int n = 0, p = s;
    while (p < e) {
        u8 o[4];
        const int k = oj_decode_one(src, p, e, o);
        for (int j = 0; j < k; ++j, ++n)
            if (n < cap) buf[n] = o[j];
    }
    return n;
}

template <class S>
__device__ __noinline__ u32 match_key_esc(const S& src, int s, int e) {
    u8 buf[20];
    const int n = decode_str(src, s, e, buf, 16);
    if (n > 12) return 0u;
    for (int k = n; k < 20; ++k) buf[k] = 0;
    return match_key_raw(BufSrc{buf}, 0, n);
}

// ---- JSONObject.stringToValue --------------------------------------------------------
enum : int { OJ_STR = 0, OJ_TRUE, OJ_FALSE, OJ_NULL, OJ_LONG, OJ_DOUBLE };

// String.equalsIgnoreCase(w), w one of true / false / null: ASCII folding plus U+017F
// (long s, C5 BF) whose upper case is 'S'.
template <class S>
__device__ __forceinline__ bool oj_ieq(const S& src, int a, int b, const char* w) {
    int i = a;
    for (; *w; ++w) {
        if (i >= b) return false;
        u32 c = src.b(i);
        if (*w == 's' && c == 0xC5u && i + 1 < b && src.b(i + 1) == 0xBFu) { i += 2; continue; }
        if (c - 'A' < 26u) c += 32;
        if (c != (u32)(u8)*w) return false;
        ++i;
    }
    return i == b;
}

__constant__ const char OJ_DBL_HALF[310] =   // 2^1024 - 2^970: decimals at or above round to Infinity
    "179769313486231580793728971405303415079934132710037826936173778980444968292764750946649017977587207096330"
    "286416692887910946555547851940402630657488671505820681908902000708383676273854845817711531764475730270069"
    "855571366959622842914819860834936475292719074168444365510704342711559699508093042880177904174497792";

__device__ __forceinline__ bool oj_sfx(u32 c) { return c == 'f' || c == 'F' || c == 'd' || c == 'D'; }

// Double.valueOf's hexadecimal branch on [a, b) (after "0x"): accepted and finite?
template <class S>
__device__ __noinline__ bool oj_hex_finite(const S& src, int a, int b) {
    int i = a, nd = 0, frac = 0, first = -1, lead = 0;
    bool dot = false;
    for (; i < b; ++i) {
        const u32 c = src.b(i);
        if (is_hex(c)) {
            if (first < 0 && hex_val(c) != 0) { first = nd; lead = (int)hex_val(c); }
            ++nd;
            if (dot) ++frac;
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    const int mend = i;
    if (nd == 0 || i >= b || (src.b(i) | 0x20u) != 'p') return false;
    ++i;
    bool neg = false;
    if (i < b && (src.b(i) == '+' || src.b(i) == '-')) { neg = src.b(i) == '-'; ++i; }
    const int ea = i;
    i64 ex = 0;
    bool big = false;
    for (; i < b && src.b(i) - '0' < 10u; ++i) {
        ex = ex * 10 + (i64)(src.b(i) - '0');
        if (ex > 0x7FFFFFFF) { big = true; ex = 0x7FFFFFFF; }
    }
    if (i == ea) return false;
    if (i < b && !(i == b - 1 && oj_sfx(src.b(i)))) return false;
    if (big) return neg;                       // Integer.parseInt overflow: zero / Infinity
    if (first < 0) return true;                // zero
    int lb = 0;
    while ((1 << (lb + 1)) <= lead) ++lb;
    const i64 L = 4 * (i64)(nd - first - 1) + lb + 1;
    const i64 top = L - 1 + (neg ? -ex : ex) - 4 * (i64)frac;
    if (top != 1023) return top < 1023;
    if (L <= 53) return true;
    // rounds up to 2^1024 iff the leading 54 significant bits are all ones
    int bits = 0, idx = 0;
    for (int k = a; k < mend && bits < 54; ++k) {
        const u32 c = src.b(k);
        if (c == '.') continue;
        if (idx++ < first) continue;
        const u32 v = hex_val(c);
        const int nb = bits == 0 ? lb + 1 : 4;
        for (int t = nb - 1; t >= 0 && bits < 54; --t, ++bits)
            if (!((v >> t) & 1u)) return true;
    }
    return bits < 54;
}

// Double.valueOf(text) accepted (FloatingDecimal.readJavaFormatString) and finite.
template <class S>
__device__ __noinline__ bool oj_double_finite(const S& src, int a, int b) {
    int i = a;
    if (i < b && (src.b(i) == '+' || src.b(i) == '-')) ++i;
    if (i + 1 < b && src.b(i) == '0' && (src.b(i + 1) | 0x20u) == 'x') return oj_hex_finite(src, i + 2, b);
    int nd = 0, ints = 0, first = -1;
    bool dot = false;
    const int d0 = i;
    for (; i < b; ++i) {
        const u32 c = src.b(i);
        if (c - '0' < 10u) {
            if (first < 0 && c != '0') first = nd;
            ++nd;
            if (!dot) ++ints;
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    const int dend = i;
    if (nd == 0) return false;
    i64 ex = 0;
    if (i < b && (src.b(i) | 0x20u) == 'e') {
        ++i;
        bool neg = false;
        if (i < b && (src.b(i) == '+' || src.b(i) == '-')) { neg = src.b(i) == '-'; ++i; }
        const int ea = i;
        for (; i < b && src.b(i) - '0' < 10u; ++i)
            if (ex < 100000000) ex = ex * 10 + (i64)(src.b(i) - '0');
        if (i == ea) return false;
        if (neg) ex = -ex;
    }
    if (i < b && !(i == b - 1 && oj_sfx(src.b(i)))) return false;
    if (first < 0) return true;                                   // zero
    const i64 mag = (i64)ints - first + ex;                       // value = 0.d... x 10^mag
    if (mag != 309) return mag < 309;
    int h = 0, idx = 0;
    for (int k = d0; k < dend; ++k) {
        const u32 c = src.b(k);
        if (c == '.') continue;
        if (idx++ < first) continue;
        const u32 hc = h < 309 ? (u32)(u8)OJ_DBL_HALF[h] : (u32)'0';
        ++h;
        if (c != hc) return c < hc;
    }
    for (; h < 309; ++h)
        if (OJ_DBL_HALF[h] != '0') return true;
    return false;                                                 // the midpoint: Infinity
}

// Long.valueOf(text) succeeds and Long.toString equals the text.
template <class S>
__device__ __forceinline__ bool oj_long_roundtrip(const S& src, int a, int b) {
    const bool neg = src.b(a) == '-';
    const int i = a + (neg ? 1 : 0);
    const int nd = b - i;
    if (nd <= 0 || nd > 19) return false;
    if (nd > 1 && src.b(i) == '0') return false;
    if (neg && nd == 1 && src.b(i) == '0') return false;
    for (int k = i; k < b; ++k)
        if (src.b(k) - '0' >= 10u) return false;
    if (nd < 19) return true;
    const char* lim = neg ? "9223372036854775808" : "9223372036854775807";
    for (int k = 0; k < 19; ++k) {
        const u32 c = src.b(i + k), l = (u32)(u8)lim[k];
        if (c != l) return c < l;
    }
    return true;
}

template <class S>
__device__ __noinline__ int oj_token_kind(const S& src, int a, int b) {
    if (oj_ieq(src, a, b, "true")) return OJ_TRUE;
    if (oj_ieq(src, a, b, "false")) return OJ_FALSE;
    if (oj_ieq(src, a, b, "null")) return OJ_NULL;
    const u32 c0 = src.b(a);
    if (c0 - '0' < 10u || c0 == '-') {
        bool decimal = (b - a == 2 && c0 == '-' && src.b(a + 1) == '0');
        for (int k = a; k < b && !decimal; ++k) {
            const u32 c = src.b(k);
            decimal = c == '.' || c == 'e' || c == 'E';
        }
        if (decimal) {
            if (oj_double_finite(src, a, b)) return OJ_DOUBLE;
        } else if (oj_long_roundtrip(src, a, b)) {
            return OJ_LONG;
        }
    }
    return OJ_STR;
}

// ---- keys ----------------------------------------------------------------------------
// A key as toString() sees it: a decoded string [s, e) (esc = escapes inside), raw
// source text [s, e), or one of the literals "true" / "false" / "null".
enum : int { OJK_STR = 0, OJK_RAW, OJK_TRUE, OJK_FALSE, OJK_NULL };
struct OjKey { int kind, s, e; };

template <class S>
struct OjKeyIter {
    const S& src;
    OjKey k;
    int p, nb, ib;
    u8 o[4];
    const char* lit;
    __device__ OjKeyIter(const S& s_, const OjKey& k_) : src(s_), k(k_), p(k_.s), nb(0), ib(0) {
        lit = k.kind == OJK_TRUE ? "true" : k.kind == OJK_FALSE ? "false" : k.kind == OJK_NULL ? "null" : nullptr;
    }
    __device__ int next() {
        if (lit) return *lit ? (int)(u8)*lit++ : -1;
        if (ib < nb) return o[ib++];
        if (p >= k.e) return -1;
        if (k.kind == OJK_RAW) return (int)src.b(p++);
        nb = oj_decode_one(src, p, k.e, o);
        ib = 1;
        return o[0];
    }
};

template <class S>
__device__ __noinline__ bool oj_key_equal(const S& src, const OjKey& a, const OjKey& b) {
    OjKeyIter<S> x(src, a), y(src, b);
    for (;;) {
        const int c = x.next(), d = y.next();
        if (c != d) return false;
        if (c < 0) return true;
    }
}

// FNV-1a of a key's toString() bytes (the duplicate-key prefilter of the top-level object).
template <class S>
__device__ __noinline__ u32 oj_key_hash(const S& src, const OjKey& k) {
    OjKeyIter<S> it(src, k);
    u32 h = 2166136261u;
    for (int c = it.next(); c >= 0; c = it.next()) h = (h ^ (u32)c) * 16777619u;
    return h;
}

// ---- skipping over already-validated text ----------------------------------------------
template <class S>
__device__ __forceinline__ int oj_skip_clean(const S& src, int p, int e) {
    while (p < e && src.b(p) <= 0x20u) ++p;
    return p;
}
// (The bounds below never bind on validated text; they keep a wave from spinning if
// they ever did.)
template <class S>
__device__ __forceinline__ int oj_skip_string(const S& src, int p, int e) {   // p at the opening quote
    const u32 q = src.b(p++);
    while (p < e) {
        const u32 c = src.b(p);
        if (c == '\\') { p += 2; continue; }
        ++p;
        if (c == q) return p;
    }
    return e;
}
template <class S>
__device__ __forceinline__ int oj_token_end(const S& src, int p, int e) {
    while (p < e && src.b(p) >= 0x20u && !oj_delim(src.b(p))) ++p;
    return p;
}
template <class S>
__device__ __noinline__ int oj_skip_value(const S& src, int p, int e) {   // p at the value's first byte
    int depth = 0;
    do {
        p = oj_skip_clean(src, p, e);
        if (p >= e) return e;
        const u32 c = src.b(p);
        if (c == '"' || c == '\'') p = oj_skip_string(src, p, e);
        else if (c == '{' || c == '[') { ++depth; ++p; }
        else if (c == '}' || c == ']') { --depth; ++p; }
        else if (c == ',' || c == ':' || c == ';') ++p;
        else p = max(oj_token_end(src, p, e), p + 1);
    } while (depth > 0);
    return p;
}
// The key of a validated pair starting at p; *after = the position after it.
template <class S>
__device__ __forceinline__ OjKey oj_key_at(const S& src, int p, int e, int* after) {
    const u32 c = src.b(p);
    if (c == '"' || c == '\'') {
        const int q = oj_skip_string(src, p, e);
        *after = q;
        return OjKey{OJK_STR, p + 1, q - 1};
    }
    if (c == '{' || c == '[') {
        const int q = oj_skip_value(src, p, e);
        *after = q;
        return OjKey{OJK_RAW, p, q};
    }
    const int q = oj_token_end(src, p, e);
    *after = q;
    int t = q;
    while (t > p && src.b(t - 1) == ' ') --t;
    const int kind = oj_token_kind(src, p, t);
    return OjKey{kind == OJ_TRUE ? OJK_TRUE : kind == OJ_FALSE ? OJK_FALSE : kind == OJ_NULL ? OJK_NULL : OJK_RAW, p, t};
}

// Is key k (starting at kpos) a repeat of an earlier key of the object whose '{' is at
// open?  Re-walks that object's earlier pairs (already validated).
template <class S>
__device__ __noinline__ bool oj_dup_key(const S& src, int open, int kpos, int e, const OjKey& k) {
    int p = open + 1;
    for (;;) {
        p = oj_skip_clean(src, p, e);
        if (p >= kpos) return false;
        int q;
        const OjKey k2 = oj_key_at(src, p, e, &q);
        if (oj_key_equal(src, k, k2)) return true;
        const int before = p;
        p = oj_skip_clean(src, q, e) + 1;                 // ':'
        p = oj_skip_value(src, p, e);
        p = oj_skip_clean(src, p, e) + 1;                 // ',' or ';'
        if (p <= before) return false;
    }
}

// ---- the parser ------------------------------------------------------------------------
template <class S>
struct OjTok {
    const S& src;
    int p, e;
    bool eof;
    int wi = -1;   // index of the cached source word (sequential reads: one load per 4 bytes)
    u32 w = 0;
    __device__ int next() {
        if (p >= e) { eof = true; return -1; }
        eof = false;
        if ((p >> 2) != wi) {
            wi = p >> 2;
            w = src.load4(p & ~3);
        }
        const int c = (int)((w >> ((p & 3) << 3)) & 0xFFu);
        ++p;
        return c;
    }
    __device__ bool back() {
        if (eof) return false;
        --p;
        return true;
    }
    __device__ int clean() {
        for (;;) {
            const int c = next();
            if (c < 0 || c > 0x20) return c;
        }
    }
};

// Advances t.p over bytes nextString only steps over -- neither the quote q, a backslash
// nor a byte below ' ' (NUL, CR, LF and the other control bytes the per-byte loop below
// decides) -- four at a time.
template <class S>
__device__ __forceinline__ void oj_skip_plain(OjTok<S>& t, int q) {
    const u32 qq = (u32)q * 0x01010101u;
    while (t.p + 4 <= t.e) {
        const u32 x = t.src.load4(t.p);
        const u32 z = zero_bytes(x ^ qq) | zero_bytes(x ^ 0x5C5C5C5Cu) | zero_bytes(x & 0xE0E0E0E0u);
        if (z != 0u) {
            t.p += (int)(__builtin_ctz(z) >> 3);
            return;
        }
        t.p += 4;
    }
}

// nextString after the opening quote q: validates up to the closing quote.
template <class S>
__device__ __forceinline__ bool oj_string(OjTok<S>& t, int q, int& esc) {
    for (;;) {
        oj_skip_plain(t, q);
        int c = t.next();
        if (c < 0 || c == '\n' || c == '\r') return false;                // Unterminated string
        if (c == q) return true;
        if (c != '\\') continue;
        esc = 1;
        c = t.next();
        if (c == 'u') {
            const int d0 = t.next(), d1 = t.next(), d2 = t.next(), d3 = t.next();
            if (d3 < 0 || d2 < 0 || d1 < 0 || d0 < 0) return false;        // Substring bounds error
            if (!(d0 == '+' || d0 == '-' || is_hex((u32)d0)) || !is_hex((u32)d1) || !is_hex((u32)d2) ||
                !is_hex((u32)d3))
                return false;                                              // NumberFormatException
            continue;
        }
        if (!(c == 'b' || c == 't' || c == 'n' || c == 'f' || c == 'r' || c == '"' || c == '\'' || c == '\\' ||
              c == '/'))
            return false;                                                  // Illegal escape.
    }
}

// One value (nextValue): a string (content [a, b), esc), unquoted text ([a, b) trimmed),
// or the opening bracket of an object / array at a (consumed).
enum : int { OJV_STR = 0, OJV_TOK, OJV_OBJ, OJV_ARR };
struct OjVal { int kind, a, b, esc; };

template <class S>
__device__ __forceinline__ bool oj_value(OjTok<S>& t, OjVal& v) {
    int c = t.clean();
    if (c == '"' || c == '\'') {
        v.kind = OJV_STR;
        v.a = t.p;
        v.esc = 0;
        if (!oj_string(t, c, v.esc)) return false;
        v.b = t.p - 1;
        return true;
    }
    if (c == '{' || c == '[') {
        v.kind = c == '{' ? OJV_OBJ : OJV_ARR;
        v.a = t.p - 1;
        return true;
    }
    v.kind = OJV_TOK;
    v.a = c < 0 ? t.p : t.p - 1;
    while (c >= 0x20 && !oj_delim((u32)c)) c = t.next();
    if (!t.back()) return false;
    int b = t.p;
    while (b > v.a && t.src.b(b - 1) == ' ') --b;                         // String.trim()
    v.b = b;
    return b > v.a;                                                        // "" -> Missing value
}

// What a container is to its parent, and the parser's states.
enum : u8 { OJR_TOP = 0, OJR_KEY, OJR_VALUE, OJR_ELEM };
enum : int { OJS_KEY = 0, OJS_COLON, OJS_VALUE, OJS_OSEP, OJS_AFIRST, OJS_AELEM, OJS_ASEP };

// new JSONObject(line [s, e)) then getString of the fields in `require`: false where
// DeserializeBolt would throw.  ad / et / tm receive the String values of the
// top-level ad_id / event_type / event_time.
template <class S>
__device__ __noinline__ bool parse_line(const S& src, int s, int e, u32 require, Span& ad, Span& et, Span& tm) {
    int end = e;                                                           // NUL: end of input
    for (int q = s & ~3; q < e; q += 4) {                                  // word at a time
        const u32 w = src.load4(q);
        const u32 z = (w - 0x01010101u) & ~w & 0x80808080u;                // a zero byte (exact for the lowest)
        if (z == 0u) continue;
        int k = 0;
        for (; k < 4; ++k) {
            const int pos = q + k;
            if (pos >= s && pos < e && ((w >> (8 * k)) & 0xFFu) == 0u) break;
        }
        if (k < 4) { end = q + k; break; }
    }
    OjTok<S> t{src, s, end, false, -1, 0u};
    if (t.clean() != '{') return false;                                    // must begin with '{'
    int open[OJ_MAX_DEPTH + 1];                                            // each open container's bracket
    u8 role[OJ_MAX_DEPTH + 1];
    int depth = 1;
    open[1] = t.p - 1;
    role[1] = OJR_TOP;
    int state = OJS_KEY, kpos = 0;
    OjKey key{OJK_RAW, 0, 0};
    u32 kid = 0, seen = 0;
    u32 khash[OJ_TOP_KEYS];   // the top-level object's key hashes so far
    int ntop = 0;
    for (;;) {
        OjVal v;
        u8 nested = 0;          // != 0: v opened a container in this role
        bool closed = false;    // the innermost container closed
        int c;
        switch (state) {
        case OJS_KEY:                                                      // a key, or '}'
            c = t.clean();
            if (c < 0) return false;                                       // must end with '}'
            if (c == '}') { closed = true; break; }
            t.back();
            kpos = t.p;
            if (!oj_value(t, v)) return false;
            if (v.kind == OJV_OBJ || v.kind == OJV_ARR) { nested = OJR_KEY; break; }
            kid = 0;
            if (v.kind == OJV_STR) {
                key = OjKey{OJK_STR, v.a, v.b};
                if (depth == 1) kid = v.esc ? match_key_esc(src, v.a, v.b) : match_key_raw(src, v.a, v.b - v.a);
            } else {
                const int k = oj_token_kind(src, v.a, v.b);
                key = OjKey{k == OJ_TRUE ? OJK_TRUE : k == OJ_FALSE ? OJK_FALSE : k == OJ_NULL ? OJK_NULL : OJK_RAW,
                            v.a, v.b};
                if (depth == 1 && key.kind == OJK_RAW) kid = match_key_raw(src, v.a, v.b - v.a);
            }
            state = OJS_COLON;
            continue;
        case OJS_COLON:
            if (t.clean() != ':') return false;                            // Expected a ':' after a key
            if (depth == 1 && ntop < OJ_TOP_KEYS) {
                // top level: compare hashes with the earlier keys', re-walk only on a hit
                const u32 h = oj_key_hash(src, key);
                bool hit = false;
#pragma unroll
                for (int k = 0; k < OJ_TOP_KEYS; ++k) hit |= k < ntop && khash[k] == h;
                if (hit && oj_dup_key(src, open[depth], kpos, end, key)) return false;   // Duplicate key
#pragma unroll
                for (int k = 0; k < OJ_TOP_KEYS; ++k)
                    if (k == ntop) khash[k] = h;
                ++ntop;
            } else if (oj_dup_key(src, open[depth], kpos, end, key)) {
                return false;                                                   // Duplicate key
            }
            state = OJS_VALUE;
            continue;
        case OJS_VALUE:
            if (!oj_value(t, v)) return false;
            if (v.kind == OJV_OBJ || v.kind == OJV_ARR) { kid = 0; nested = OJR_VALUE; break; }
            if (kid && (v.kind == OJV_STR || oj_token_kind(src, v.a, v.b) == OJ_STR)) {   // getString
                const Span sp{v.a, v.b, v.kind == OJV_STR ? v.esc : 0};
                if (kid == K_AD) ad = sp;
                else if (kid == K_ETYPE) et = sp;
                else if (kid == K_ETIME) tm = sp;
                seen |= kid;
            }
            kid = 0;
            state = OJS_OSEP;
            continue;
        case OJS_OSEP:                                                     // ',' / ';' / '}'
            c = t.clean();
            if (c == ',' || c == ';') {
                if (t.clean() == '}') { closed = true; break; }
                if (!t.back()) return false;
                state = OJS_KEY;
                continue;
            }
            if (c == '}') { closed = true; break; }
            return false;                                                  // Expected a ',' or '}'
        case OJS_AFIRST:
            c = t.clean();
            if (c == ']') { closed = true; break; }
            if (!t.back()) return false;
            state = OJS_AELEM;
            continue;
        case OJS_AELEM:
            c = t.clean();
            if (!t.back()) return false;
            if (c == ',') { state = OJS_ASEP; continue; }                  // an empty slot: NULL
            if (!oj_value(t, v)) return false;
            if (v.kind == OJV_OBJ || v.kind == OJV_ARR) { nested = OJR_ELEM; break; }
            state = OJS_ASEP;
            continue;
        default:                                                           // OJS_ASEP
            c = t.clean();
            if (c == ',') {
                if (t.clean() == ']') { closed = true; break; }
                if (!t.back()) return false;
                state = OJS_AELEM;
                continue;
            }
            if (c == ']') { closed = true; break; }
            return false;                                                  // Expected a ',' or ']'
        }
        if (nested) {
            if (++depth > OJ_MAX_DEPTH) return false;
            open[depth] = v.a;
            role[depth] = nested;
            state = v.kind == OJV_OBJ ? OJS_KEY : OJS_AFIRST;
            continue;
        }
        if (closed) {
            const u8 r = role[depth];
            const int op = open[depth];
            if (--depth == 0) return (seen & require) == require;          // nothing after '}' is read
            if (r == OJR_KEY) {                                            // toString() of a container
                key = OjKey{OJK_RAW, op, t.p};
                kpos = op;
                kid = 0;
                state = OJS_COLON;
            } else {
                state = r == OJR_VALUE ? OJS_OSEP : OJS_ASEP;
            }
        }
    }
}

}  // namespace ysb
