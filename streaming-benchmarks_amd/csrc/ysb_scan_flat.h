// ysb_scan_flat.h -- flat objects in any key order (the flat tier) and a learned
// key order (layout 3) for Kernel 1 and the deferred-line kernel: other producers' JSON
// lines that org.json reads as DeserializeBolt does (AdvertisingTopologyNative.java:257-276).
// Part of the scan kernel's translation unit: included by ysb_scan.hip only, after the
// definitions it uses (the LDS sources, spans, load_span, the org.json machine).
#pragma once

namespace ysb {

// ---- the flat tier's key table (round 5) ---------------------------------------------------
// DeserializeBolt's seven keys named by one LDS read instead of a compare chain (A/B: +2-3 %
// on the flat tier and the mixed interleave, profiles/AB_LOG.md round 5).  With the key's
// first eight bytes in kw[0], kw[1] (text, closing quote, separator), x = kw[0] ^ (kw[1] >> 8)
// and slot = bits 20..23 of x ^ (x >> 1): a perfect hash of the seven keys' texts (found by
// search; shifts and xors only, no quarter-rate multiply; ad_id's kw[1] holds the separator's
// first bytes, `": "` or `":"`, and both land in its slot).  Entry = {kw[0], kw[1] & m1,
// kw[2] & m2, meta}, meta = id | kl << 8 | s1 << 16 | s2 << 24, m1 = ~0 >> s1,
// m2 = 0xFFFFFF >> s2: the key's text and closing quote compared exactly as the compare chain
// did; an empty slot (meta 0) names nothing.
constexpr int KEYTAB_BYTES = 256;
struct KeyDef {
    u32 w0, w1, w2, id, kl;   // w1 / w2: the bytes the key owns (text and closing quote)
    u32 h1;                   // kw[1] as the hash sees it (with the separator's bytes)
};
constexpr KeyDef KEYDEFS[8] = {
    {w4('a', 'd', '_', 'i'), w4('d', '"', 0, 0), 0u, K_AD, 5u, w4('d', '"', ':', ' ')},
    {w4('a', 'd', '_', 'i'), w4('d', '"', 0, 0), 0u, K_AD, 5u, w4('d', '"', ':', '"')},
    {w4('u', 's', 'e', 'r'), w4('_', 'i', 'd', '"'), 0u, K_USER, 7u, w4('_', 'i', 'd', '"')},
    {w4('p', 'a', 'g', 'e'), w4('_', 'i', 'd', '"'), 0u, K_PAGE, 7u, w4('_', 'i', 'd', '"')},
    {w4('a', 'd', '_', 't'), w4('y', 'p', 'e', '"'), 0u, K_ADTYPE, 7u, w4('y', 'p', 'e', '"')},
    {w4('e', 'v', 'e', 'n'), w4('t', '_', 't', 'y'), w4('p', 'e', '"', 0), K_ETYPE, 10u, w4('t', '_', 't', 'y')},
    {w4('e', 'v', 'e', 'n'), w4('t', '_', 't', 'i'), w4('m', 'e', '"', 0), K_ETIME, 10u, w4('t', '_', 't', 'i')},
    {w4('i', 'p', '_', 'a'), w4('d', 'd', 'r', 'e'), w4('s', 's', '"', 0), K_IP, 10u, w4('d', 'd', 'r', 'e')},
};
__host__ __device__ constexpr u32 keytab_slot(u32 kw0, u32 kw1) {
    const u32 x = kw0 ^ (kw1 >> 8);
    return ((x ^ (x >> 1)) >> 20) & 15u;
}
struct KeyTab { u32 w[64]; };
constexpr KeyTab make_keytab() {
    KeyTab t{};
    for (const KeyDef& d : KEYDEFS) {
        const u32 s = keytab_slot(d.w0, d.h1);
        const u32 s1 = d.kl == 5u ? 16u : 0u, s2 = d.kl == 10u ? 0u : 24u;
        t.w[4 * s] = d.w0;
        t.w[4 * s + 1] = d.w1;
        t.w[4 * s + 2] = d.w2;
        t.w[4 * s + 3] = d.id | d.kl << 8 | s1 << 16 | s2 << 24;
    }
    return t;
}
constexpr bool keytab_perfect() {   // two different keys never share a slot
    for (int i = 0; i < 8; ++i)
        for (int j = i + 1; j < 8; ++j)
            if (KEYDEFS[i].id != KEYDEFS[j].id &&
                keytab_slot(KEYDEFS[i].w0, KEYDEFS[i].h1) == keytab_slot(KEYDEFS[j].w0, KEYDEFS[j].h1))
                return false;
    return true;
}
static_assert(keytab_perfect(), "keytab_slot must separate the seven keys");
constexpr KeyTab KEYTAB = make_keytab();

// ---- the general path's flat tier --------------------------------------------------------
// A flat object of plain double-quoted string pairs whose keys are all DeserializeBolt's
// -- in any order, with any whitespace nextClean skips, ',' or ';' between pairs and a
// separator allowed before '}' -- is decided here with word-at-a-time string scans over
// the staged line instead of org.json's character machine.  On exactly this subset the
// steps are JSONObject(JSONTokener)'s: nextClean '{'; per pair nextClean -> '"' ->
// nextString, nextClean ':', nextClean '"' -> nextString, putOnce; nextClean ',' | ';'
// (then '}' closes) | '}' (org.json 20180813 JSONObject.java constructor).  Anything
// else -- another key, a repeated key, a value that is not a plain string, a quote other
// than '"', an escape, a control byte or NUL, a missing field -- returns false having
// counted nothing, and parse_line decides the line.
// true: the line is a flat object of the subset above with every field of `require` (and
// the three the topology reads); ad / et / tm = the values' spans
// The flat-first / learned-order instantiations' parser of the same subset plus ONE other
// key with a plain string value (a producer's extra field: org.json puts it, DeserializeBolt
// never reads it; a second one goes to parse_line, which sees a repeat as putOnce does): a
// key of DeserializeBolt's seven is named by its first four bytes and its remaining bytes
// and closing quote compared in place (a key with an escape fails the compare and the
// plain-string scan alike, as it fails match_key_raw); the separators
// `": "` / `":"` after a key and `", "` / `","` / `}` after a value are compared in place,
// any other spacing takes the ft_clean scans; the id values are checked as 36-byte UUIDs
// in one step.  Positions read past e are never accepted (each fast compare checks the
// bytes it uses are < e).
template <class S>
__device__ __forceinline__ bool flat_parse_fast(const S& src, int s, int e, u32 require, Span& ad, Span& et,
                                                Span& tm) {
    u32 c = 0;
    int p = ft_clean<S, true>(src, s, e, c);
    if (p < 0 || c != '{') return false;
    p = ft_clean<S, true>(src, p + 1, e, c);             // the first key, or '}'
    if (p < 0) return false;
    u32 seen = 0;
    if (c != '}') {
        if (c != '"') return false;
        int kq = p;                                       // the next key's opening quote
        for (;;) {
            const u32 k0 = src.load4(kq + 1);
            u32 id = 0;
            int kl = 0;
            if (k0 == w4('a', 'd', '_', 'i')) {
                kl = 5;
                id = src.b(kq + 5) == 'd' ? K_AD : 0u;
            } else if (k0 == w4('u', 's', 'e', 'r')) {
                kl = 7;
                id = src.load4(kq + 4) == w4('r', '_', 'i', 'd') ? K_USER : 0u;
            } else if (k0 == w4('p', 'a', 'g', 'e')) {
                kl = 7;
                id = src.load4(kq + 4) == w4('e', '_', 'i', 'd') ? K_PAGE : 0u;
            } else if (k0 == w4('a', 'd', '_', 't')) {
                kl = 7;
                id = src.load4(kq + 4) == w4('t', 'y', 'p', 'e') ? K_ADTYPE : 0u;
            } else if (k0 == w4('e', 'v', 'e', 'n')) {
                kl = 10;
                const u32 k1 = src.load4(kq + 5), k2 = src.load4(kq + 7);
                id = (k1 == w4('t', '_', 't', 'y') && k2 == w4('t', 'y', 'p', 'e'))   ? K_ETYPE
                     : (k1 == w4('t', '_', 't', 'i') && k2 == w4('t', 'i', 'm', 'e')) ? K_ETIME
                                                                                        : 0u;
            } else if (k0 == w4('i', 'p', '_', 'a')) {
                kl = 10;
                id = (src.load4(kq + 5) == w4('d', 'd', 'r', 'e') && src.load4(kq + 7) == w4('r', 'e', 's', 's')) ? K_IP
                                                                                                                 : 0u;
            }
            int ke = kq + 1 + kl;                         // the key's closing quote
            if (id == 0u || ke >= e || src.b(ke) != '"') {
                // another key (a producer's extra field): skipped when it is a plain string
                // with a plain string value, at most one per line -- org.json puts it and
                // DeserializeBolt never reads it; a second one could repeat it (putOnce
                // throws), so that line, and any other value form, goes to parse_line
                ke = ft_string_end(src, kq + 1, e);
                if (ke < 0 || (seen & K_OTHER) != 0u) return false;
                id = K_OTHER;
            } else if ((seen & id) != 0u) {
                return false;                             // a repeated key: putOnce throws
            }
            seen |= id;
            // ':' and the value's opening quote
            int vq;
            const u32 w = src.load4(ke + 1);
            if ((w & 0xFFFFFFu) == (w4(':', ' ', '"', 0) & 0xFFFFFFu) && ke + 3 < e) {
                vq = ke + 3;
            } else if ((w & 0xFFFFu) == (w4(':', '"', 0, 0) & 0xFFFFu) && ke + 2 < e) {
                vq = ke + 2;
            } else {
                p = ft_clean<S, true>(src, ke + 1, e, c);
                if (p < 0 || c != ':') return false;
                p = ft_clean<S, true>(src, p + 1, e, c);
                if (p < 0 || c != '"') return false;
                vq = p;
            }
            int ve = -1;
            if (id & (K_AD | K_USER | K_PAGE)) {          // 36 plain bytes and the closing quote
                u32 f = 0;
#pragma unroll
                for (int k = 0; k < 9; ++k) f |= ft_flags(src.load4(vq + 1 + 4 * k));
                if (f == 0u && vq + 37 < e && src.b(vq + 37) == '"') ve = vq + 37;
            }
            if (ve < 0) ve = ft_string_end(src, vq + 1, e);
            if (ve < 0) return false;
            const Span sp{vq + 1, ve, 0};
            if (id == K_AD) ad = sp;
            else if (id == K_ETYPE) et = sp;
            else if (id == K_ETIME) tm = sp;
            // ', "' / ',"' and the next key, or '}'
            const u32 x = src.load4(ve + 1);
            if ((x & 0xFFFFFFu) == (w4(',', ' ', '"', 0) & 0xFFFFFFu) && ve + 3 < e) {
                kq = ve + 3;
                continue;
            }
            if ((x & 0xFFFFu) == (w4(',', '"', 0, 0) & 0xFFFFu) && ve + 2 < e) {
                kq = ve + 2;
                continue;
            }
            if ((x & 0xFFu) == '}' && ve + 1 < e) break;
            p = ft_clean<S, true>(src, ve + 1, e, c);
            if (p < 0) return false;
            if (c == '}') break;
            if (c != ',' && c != ';') return false;
            p = ft_clean<S, true>(src, p + 1, e, c);     // the next key, or '}' after a separator
            if (p < 0) return false;
            if (c == '}') break;
            if (c != '"') return false;
            kq = p;
        }
    }
    const u32 need = require | K_AD | K_ETYPE | K_ETIME;
    return (seen & need) == need;
}

// 36 value bytes (w[0..8]) are plain string bytes: no quote, backslash or byte < 0x20.
// Fast test: every byte in [0x2D, 0x7F) and not a backslash (UUID text always is); else
// the exact flags.
__device__ __forceinline__ bool plain36(const u32 (&w)[10]) {
    u32 lo = 0xFFFFFFFFu, hi = 0, bs = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        lo &= w[k] + 0x53535353u;   // bit 7 set per byte iff byte >= 0x2D (bytes < 0x80: no carries)
        hi |= w[k];
        bs |= zero_bytes(w[k] ^ 0x5C5C5C5Cu);
    }
    if (((lo & 0x80808080u) == 0x80808080u) & ((hi & 0x80808080u) == 0u) & (bs == 0u)) return true;
    u32 f = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) f |= ft_flags(w[k]);
    return f == 0u;
}

// plain36's fast test as a u32 (0 = every byte of w[0..8] in [0x2D, 0x7F) and not a
// backslash); nonzero says only that the fast test failed (the exact flags decide).
// With every byte < 0x80 (the `hi` term), (w ^ 0x5C5C5C5C) + 0x7F7F7F7F sets
// bit 7 of a byte iff it is not '\\' and w + 0x53535353 iff it is >= 0x2D, with no carry
// between bytes -- two adds (one v_xad_u32) and two ands per word instead of a zero-byte test.
__device__ __forceinline__ u32 plain36_bad(const u32 (&w)[10]) {
    u32 acc = 0xFFFFFFFFu, hi = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        acc &= (w[j] + 0x53535353u) & ((w[j] ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu);
        hi |= w[j];
    }
    return ((acc & 0x80808080u) ^ 0x80808080u) | (hi & 0x80808080u);
}

// The length of a short value named from its vocabulary -- the generator's closed sets
// (core.clj:68-69,96,181): an ad_type of the five, an event_type of the three, a 13-digit
// event_time, ip "1.2.3.4" -- from the words at its first byte (A: >= 5 realigned words), or 0
// when it is none of them (the caller then scans for its closing quote).  Every byte up to the
// closing quote is compared (or shown to be a digit), so a value named is a plain string.
// KI: learn_key's index (3 ad_type, 4 event_type, 5 event_time, 6 ip_address).
template <int KI>
__device__ __forceinline__ int vocab_len(const u32* A) {
    if constexpr (KI == 3) {
        if (A[0] == w4('b', 'a', 'n', 'n') && (A[1] & 0xFFFFFFu) == (w4('e', 'r', '"', 0) & 0xFFFFFFu)) return 6;
        if (A[0] == w4('m', 'a', 'i', 'l') && (A[1] & 0xFFu) == '"') return 4;
        if (A[0] == w4('m', 'o', 'd', 'a') && (A[1] & 0xFFFFu) == w4('l', '"', 0, 0)) return 5;
        if (A[0] == w4('m', 'o', 'b', 'i') && (A[1] & 0xFFFFFFu) == (w4('l', 'e', '"', 0) & 0xFFFFFFu)) return 6;
        if (A[0] == w4('s', 'p', 'o', 'n') && A[1] == w4('s', 'o', 'r', 'e') && A[2] == w4('d', '-', 's', 'e') &&
            A[3] == w4('a', 'r', 'c', 'h') && (A[4] & 0xFFu) == '"')
            return 16;
        return 0;
    } else if constexpr (KI == 4) {
        if (A[0] == w4('v', 'i', 'e', 'w') && (A[1] & 0xFFu) == '"') return 4;
        if (A[0] == w4('c', 'l', 'i', 'c') && (A[1] & 0xFFFFu) == w4('k', '"', 0, 0)) return 5;
        if (A[0] == w4('p', 'u', 'r', 'c') && A[1] == w4('h', 'a', 's', 'e') && (A[2] & 0xFFu) == '"') return 8;
        return 0;
    } else if constexpr (KI == 5) {
        u32 bad = 0;
        swar_digits4(A[0], bad);
        swar_digits4(A[1], bad);
        swar_digits4(A[2], bad);
        bad |= ((A[3] & 0xFFu) - '0') > 9u;
        return (bad == 0u && ((A[3] >> 8) & 0xFFu) == '"') ? 13 : 0;
    } else {
        return (A[0] == w4('1', '.', '2', '.') && A[1] == w4('3', '.', '4', '"')) ? 7 : 0;
    }
}

// Round 4: the flat-first / learned-order instantiations' flat tier on the staged LDS line
// (flat_parse_fast's subset and decisions), with the common forms taken branch-free:
//   * the key named from the four realigned words at its text (load_span: five aligned
//     reads) by compares and selects -- no if-chain, so lanes whose lines carry different
//     keys at the same pair (several producers interleaved) do not serialise on it;
//   * the key's closing quote and `": "` / `":"` read from the same words;
//   * an id value (ad / user / page) as one 10-word span: 36 plain bytes by plain36's
//     cheap test, its closing quote and the separator after it (`", "` / `","` / `"}`);
//   * any other value by ft_string_end and one word for its separator.
// Every other form (other whitespace, ';', a key that is not DeserializeBolt's, an id that
// is not 36 plain bytes) takes the same per-byte steps as flat_parse_fast: a divergent slow
// branch that the common lines never enter.
__device__ __forceinline__ bool flat_parse_lds(const LdsSrc& src, int s, int e, u32 require, Span& ad, Span& et,
                                               Span& tm, u32 (&adw)[9]) {
    u32 c = 0;
    int kq;                                           // the next key's opening quote
    if ((src.load4(s) & 0xFFFFu) == w4('{', '"', 0, 0) && s + 1 < e) {
        kq = s + 1;
    } else {
        int p = ft_clean<LdsSrc, true>(src, s, e, c);
        if (p < 0 || c != '{') return false;
        p = ft_clean<LdsSrc, true>(src, p + 1, e, c);
        if (p < 0) return false;
        if (c == '}') return (require | K_AD | K_ETYPE | K_ETIME) == 0u;   // {} (never: the chain's keys are required)
        if (c != '"') return false;
        kq = p;
    }
    u32 seen = 0;
    bool closed = false;
#pragma unroll 1
    for (int k = 0; k < 9 && !closed; ++k) {          // at most 7 keys + one extra field: 8 pairs
        u32 kw[4];
        load_span(src, kq + 1, kw);
        const bool isAD = kw[0] == w4('a', 'd', '_', 'i') && (kw[1] & 0xFFFFu) == w4('d', '"', 0, 0);
        const bool is7 = (kw[1] == w4('_', 'i', 'd', '"') && (kw[0] == w4('u', 's', 'e', 'r') || kw[0] == w4('p', 'a', 'g', 'e'))) ||
                         (kw[0] == w4('a', 'd', '_', 't') && kw[1] == w4('y', 'p', 'e', '"'));
        const bool ev = kw[0] == w4('e', 'v', 'e', 'n');
        const u32 k2 = kw[2] & 0xFFFFFFu;
        const bool isET = ev && kw[1] == w4('t', '_', 't', 'y') && k2 == (w4('p', 'e', '"', 0) & 0xFFFFFFu);
        const bool isTM = ev && kw[1] == w4('t', '_', 't', 'i') && k2 == (w4('m', 'e', '"', 0) & 0xFFFFFFu);
        const bool isIP = kw[0] == w4('i', 'p', '_', 'a') && kw[1] == w4('d', 'd', 'r', 'e') && k2 == (w4('s', 's', '"', 0) & 0xFFFFFFu);
        u32 id = isAD ? K_AD : isET ? K_ETYPE : isTM ? K_ETIME : isIP ? K_IP : 0u;
        if (is7) id = kw[0] == w4('u', 's', 'e', 'r') ? K_USER : kw[0] == w4('p', 'a', 'g', 'e') ? K_PAGE : K_ADTYPE;
        // the key's closing quote at kq + 1 + kl; the 4 bytes after it
        const u32 x = isAD ? __builtin_amdgcn_alignbyte(kw[2], kw[1], 2) : is7 ? kw[2] : __builtin_amdgcn_alignbyte(kw[3], kw[2], 3);
        const int ke = kq + 1 + (isAD ? 5 : is7 ? 7 : 10);
        int vq;                                       // the value's opening quote
        if (id != 0u && (x & 0xFFFFFFu) == (w4(':', ' ', '"', 0) & 0xFFFFFFu) && ke + 3 < e) {
            vq = ke + 3;
        } else if (id != 0u && (x & 0xFFFFu) == (w4(':', '"', 0, 0) & 0xFFFFu) && ke + 2 < e) {
            vq = ke + 2;
        } else {                                      // slow: another key, other whitespace
            int kend = ke;
            if (id == 0u) {   // a producer's extra field: at most one, a plain string key
                kend = ft_string_end(src, kq + 1, e);
                if (kend < 0 || (seen & K_OTHER) != 0u) return false;
                id = K_OTHER;
            }
            int p = ft_clean<LdsSrc, true>(src, kend + 1, e, c);
            if (p < 0 || c != ':') return false;
            p = ft_clean<LdsSrc, true>(src, p + 1, e, c);
            if (p < 0 || c != '"') return false;
            vq = p;
        }
        if ((seen & id) != 0u) return false;          // a repeated key: putOnce throws
        seen |= id;
        int ve = -1;
        u32 y = 0;                                    // the closing quote and the 3 bytes after it
        u32 w[10];                                    // the value's words, for every key
        load_span(src, vq + 1, w);
        if (id & (K_AD | K_USER | K_PAGE)) {
            if (plain36(w) && vq + 37 < e && (w[9] & 0xFFu) == '"') {
                ve = vq + 37;
                y = w[9];
                if (id == K_AD) {
#pragma unroll
                    for (int j = 0; j < 9; ++j) adw[j] = w[j];
                }
            }
        } else {                                      // round 4: a short value named from its vocabulary
            const int la = id == K_ADTYPE ? vocab_len<3>(w) : id == K_ETYPE ? vocab_len<4>(w)
                         : id == K_ETIME ? vocab_len<5>(w) : id == K_IP ? vocab_len<6>(w) : 0;
            if (la && vq + 1 + la < e) {
                ve = vq + 1 + la;
                y = src.load4(ve);
            }
        }
        if (ve < 0) {
            ve = ft_string_end(src, vq + 1, e);
            if (ve < 0) return false;
            y = src.load4(ve);
        }
        const Span sp{vq + 1, ve, 0};
        if (id == K_AD) ad = sp;
        else if (id == K_ETYPE) et = sp;
        else if (id == K_ETIME) tm = sp;
        // ', "' / ',"' and the next key, or '}'
        if (y == w4('"', ',', ' ', '"') && ve + 3 < e) { kq = ve + 3; continue; }
        if ((y & 0xFFFFFFu) == (w4('"', ',', '"', 0) & 0xFFFFFFu) && ve + 2 < e) { kq = ve + 2; continue; }
        if ((y & 0xFFFFu) == w4('"', '}', 0, 0) && ve + 1 < e) { closed = true; continue; }
        int p = ft_clean<LdsSrc, true>(src, ve + 1, e, c);
        if (p < 0) return false;
        if (c == '}') { closed = true; continue; }
        if (c != ',' && c != ';') return false;
        p = ft_clean<LdsSrc, true>(src, p + 1, e, c);  // the next key, or '}' after a separator
        if (p < 0) return false;
        if (c == '}') { closed = true; continue; }
        if (c != '"') return false;
        kq = p;
    }
    // (a ninth pair is a repeat: putOnce would throw -- not closed, not taken)
    const u32 need = require | K_AD | K_ETYPE | K_ETIME;
    return closed && (seen & need) == need;
}

// vocab_len's sets for a key id known only at run time (K_ADTYPE / K_ETYPE / K_ETIME / K_IP,
// else 0), each candidate's bytes compared as u32 differences (no bool logic, see below).
__device__ __forceinline__ int bl2_vocab(u32 id, const u32 (&A)[10]) {
    int la = 0;
    if (id == K_ADTYPE) {
        const u32 dBN = (A[0] ^ w4('b', 'a', 'n', 'n')) | ((A[1] ^ w4('e', 'r', '"', 0)) & 0xFFFFFFu);
        const u32 dML = (A[0] ^ w4('m', 'a', 'i', 'l')) | ((A[1] ^ '"') & 0xFFu);
        const u32 dMD = (A[0] ^ w4('m', 'o', 'd', 'a')) | ((A[1] ^ w4('l', '"', 0, 0)) & 0xFFFFu);
        const u32 dMB = (A[0] ^ w4('m', 'o', 'b', 'i')) | ((A[1] ^ w4('l', 'e', '"', 0)) & 0xFFFFFFu);
        const u32 dSP = (A[0] ^ w4('s', 'p', 'o', 'n')) | (A[1] ^ w4('s', 'o', 'r', 'e')) | (A[2] ^ w4('d', '-', 's', 'e')) |
                        (A[3] ^ w4('a', 'r', 'c', 'h')) | ((A[4] ^ '"') & 0xFFu);
        la = dBN == 0u ? 6 : dML == 0u ? 4 : dMD == 0u ? 5 : dMB == 0u ? 6 : dSP == 0u ? 16 : 0;
    } else if (id == K_ETYPE) {
        const u32 dV = (A[0] ^ w4('v', 'i', 'e', 'w')) | ((A[1] ^ '"') & 0xFFu);
        const u32 dC = (A[0] ^ w4('c', 'l', 'i', 'c')) | ((A[1] ^ w4('k', '"', 0, 0)) & 0xFFFFu);
        const u32 dP = (A[0] ^ w4('p', 'u', 'r', 'c')) | (A[1] ^ w4('h', 'a', 's', 'e')) | ((A[2] ^ '"') & 0xFFu);
        la = dV == 0u ? 4 : dC == 0u ? 5 : dP == 0u ? 8 : 0;
    } else if (id == K_ETIME) {
        u32 bad = 0;
        swar_digits4(A[0], bad);
        swar_digits4(A[1], bad);
        swar_digits4(A[2], bad);
        bad |= (((A[3] & 0xFFu) - '0') > 9u ? 1u : 0u) | (((A[3] >> 8) & 0xFFu) ^ '"');
        la = bad == 0u ? 13 : 0;
    } else if (id == K_IP) {
        la = ((A[0] ^ w4('1', '.', '2', '.')) | (A[1] ^ w4('3', '.', '4', '"'))) == 0u ? 7 : 0;
    }
    return la;
}

// Round 4 (YSB_FLAT_BL): flat_parse_lds's common forms with no slow branch per pair -- for
// batches whose lines carry different key orders (several producers interleaved), where
// every per-pair branch of a per-lane walk diverges.  Per pair, for every lane at once: the
// key named (round 5: by the key table kt in LDS, KEYTAB above), `": "` / `":"`, the value -- an id as 36 plain bytes by
// plain36's cheap test, any other value named from its vocabulary or, when it is none of
// them, by the string scan -- and `", "` / `","` / `"}` after it; the loop runs while any
// lane is open (a uniform exit).  Any other form (another key, a repeat, other spacing, a
// value that is not 36 / vocabulary / plain, a missing field) only marks the lane out, and
// the caller hands the line to flat_parse_lds, which decides it: a subset of its lines, the
// same spans.
// A bool is a lane mask in scalar registers: every && / || / ! of two bools is a scalar
// instruction, and every bool carried across the loop's blocks is merged by three more --
// issue slots the wave spends beside its VALU work.  Here a pair's checks OR into one u32
// (`bad`: 0 = the pair is in the common forms), the lane state is a u32 (1 open, 2 closed,
// 0 out: the caller's flat_parse_lds decides the line) and each decision is one compare.
__device__ __forceinline__ bool flat_parse_bl2(const LdsSrc& src, int s, int e, u32 require, Span& ad, Span& et,
                                               Span& tm, u32 (&adw)[9], const u32* kt) {
    // (u32)(a - b) >> 31: 1 when a < b (positions < 2^31)
    u32 st = (((src.load4(s) & 0xFFFFu) ^ w4('{', '"', 0, 0)) | ((u32)(e - 2 - s) >> 31)) == 0u ? 1u : 0u;
    int kq = s + 1;
    u32 seen = 0;
    int ads = s, ets = s, ete = s, tms = s, tme = s;
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
        if (__ballot(st == 1u) == 0ull) break;
        const u32 open = st == 1u ? 1u : 0u;
        kq = open ? kq : s + 1;                       // an idle lane reads inside its line
        u32 kw[4];
        load_span(src, kq + 1, kw);
        // the key named by its slot in the key table (one LDS read; see KEYTAB above)
        const u32 slot = keytab_slot(kw[0], kw[1]);
        const uint4 en = *reinterpret_cast<const uint4*>(kt + 4 * slot);
        const u32 m1 = 0xFFFFFFFFu >> ((en.w >> 16) & 31u), m2 = 0xFFFFFFu >> (en.w >> 24);
        const u32 dk = (kw[0] ^ en.x) | ((kw[1] & m1) ^ en.y) | ((kw[2] & m2) ^ en.z);
        const u32 id = dk == 0u ? (en.w & 0xFFu) : 0u;
        const u32 k7 = id & (K_USER | K_PAGE | K_ADTYPE);
        const u32 x = id == K_AD ? __builtin_amdgcn_alignbyte(kw[2], kw[1], 2) : k7 ? kw[2] : __builtin_amdgcn_alignbyte(kw[3], kw[2], 3);
        const int ke = kq + 1 + (id == K_AD ? 5 : k7 ? 7 : 10);
        const u32 s3 = (x ^ w4(':', ' ', '"', 0)) & 0xFFFFFFu;
        const u32 s2 = (x ^ w4(':', '"', 0, 0)) & 0xFFFFu;
        const int vq = ke + (s3 == 0u ? 3 : 2);
        u32 bad = min(s3, s2) | (id == 0u ? 1u : 0u) | (seen & id) | ((u32)(e - 1 - vq) >> 31);
        u32 w[10];
        load_span(src, vq + 1, w);
        int ve;
        u32 y;
        if (id & (K_AD | K_USER | K_PAGE)) {
            bad |= plain36_bad(w) | ((w[9] ^ '"') & 0xFFu);
            ve = vq + 37;
            y = w[9];
        } else {
            int la = bl2_vocab(id, w);
            if (__builtin_expect((bad | (u32)la) == 0u, 0)) {   // a value outside the vocabularies
                const int q = ft_string_end(src, vq + 1, e);
                la = q > vq ? q - vq - 1 : 0;
            }
            bad |= la == 0 ? 1u : 0u;
            ve = vq + 1 + la;
            y = src.load4(ve);
        }
        const u32 n3 = y ^ w4('"', ',', ' ', '"');
        const u32 n2 = (y ^ w4('"', ',', '"', 0)) & 0xFFFFFFu;
        const u32 cl = (y ^ w4('"', '}', 0, 0)) & 0xFFFFu;
        const int nk = n3 == 0u ? ve + 3 : n2 == 0u ? ve + 2 : ve + 1;   // the next key's quote / the '}'
        bad |= (n3 == 0u || n2 == 0u || cl == 0u) ? ((u32)(e - 1 - nk) >> 31) : 1u;
        const u32 idg = (open != 0u && bad == 0u) ? id : 0u;
        ads = idg == K_AD ? vq + 1 : ads;
        ets = idg == K_ETYPE ? vq + 1 : ets;
        ete = idg == K_ETYPE ? ve : ete;
        tms = idg == K_ETIME ? vq + 1 : tms;
        tme = idg == K_ETIME ? ve : tme;
        seen |= idg;
        st = open == 0u ? st : bad != 0u ? 0u : cl == 0u ? 2u : 1u;
        kq = nk;
    }
    const u32 need = require | K_AD | K_ETYPE | K_ETIME;
    if (((st ^ 2u) | ((seen & need) ^ need)) != 0u) return false;
    ad = Span{ads, ads + 36, 0};
    et = Span{ets, ete, 0};
    tm = Span{tms, tme, 0};
    load_span(src, ads, adw);
    return true;
}

// YSB_DIAG_FLAT_IDX (a timing diagnostic, round 6; never used for results): the first half of
// the wave-cooperative structural index the round-5 review asked for, on the lane's own line --
// every 16-B chunk of [s, e) read from LDS (one ds_read_b128) and classified (quote bytes
// exactly, backslash and control bytes), the quote positions extracted in order by bit scans,
// as the owner lane's walk would consume them -- with nothing named or parsed after it.  Its
// cost is a lower bound of the index design's; the caller counts nothing.  A checksum keeps
// the work alive.
__device__ __forceinline__ u32 flat_index_only(const LdsSrc& src, int s, int e) {
    u32 acc = 0, nq = 0, bad = 0;
    int q = s & ~15;
#pragma unroll 1
    for (; q < e; q += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(src.d + (q >> 2));
        const u32 w[4] = {v.x, v.y, v.z, v.w};
        u32 qm = 0, bm = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 x = w[k] ^ 0x22222222u;
            const u32 z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);   // quote bytes, exact
            const u32 b = zero_bytes(w[k] ^ 0x5C5C5C5Cu) | zero_bytes(w[k] & 0xE0E0E0E0u);
            qm |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
            bm |= (((b >> 7) & 1u) | ((b >> 14) & 2u) | ((b >> 21) & 4u) | ((b >> 28) & 8u)) << (4 * k);
        }
        const u32 lo = q < s ? 0xFFFFu << (s - q) : 0xFFFFu;
        const u32 hi = q + 16 > e - 1 ? (1u << (e - 1 - q)) - 1u : 0xFFFFu;   // (the line's '\n' is no byte of it)
        qm &= lo & hi;
        bad |= bm & lo & hi;
        while (qm) {   // the owner's walk takes the quotes in order
            acc = acc * 31u + (u32)(q + __builtin_ctz(qm));
            ++nq;
            qm &= qm - 1u;
        }
    }
    return acc ^ (nq << 24) ^ bad;
}

// FAST (the flat-first instantiation only): the whitespace skips' first step outside their
// loops, and the id values (ad / user / page) checked as 36-byte UUIDs in one step before
// the string scan -- the same decisions, fewer divergent loop trips.
template <class S, bool FAST = false>
__device__ __forceinline__ bool flat_parse(const S& src, int s, int e, u32 require, Span& ad, Span& et, Span& tm) {
    u32 c = 0;
    int p = ft_clean<S, FAST>(src, s, e, c);
    if (p < 0 || c != '{') return false;
    u32 seen = 0;
    for (;;) {
        p = ft_clean<S, FAST>(src, p + 1, e, c);             // a key, or '}'
        if (p < 0) return false;
        if (c == '}') break;                                  // {} or a separator before '}'
        if (c != '"') return false;
        const int ke = ft_string_end(src, p + 1, e);
        if (ke < 0) return false;
        const u32 id = match_key_raw(src, p + 1, ke - p - 1);
        if (id == 0u || (seen & id) != 0u) return false;      // another key, or a repeat
        seen |= id;
        p = ft_clean<S, FAST>(src, ke + 1, e, c);
        if (p < 0 || c != ':') return false;
        p = ft_clean<S, FAST>(src, p + 1, e, c);
        if (p < 0 || c != '"') return false;
        int ve = -1;
        if constexpr (FAST) {
            if (id & (K_AD | K_USER | K_PAGE)) {   // 36 plain bytes and the closing quote
                u32 f = 0;
#pragma unroll
                for (int k = 0; k < 9; ++k) f |= ft_flags(src.load4(p + 1 + 4 * k));
                if (f == 0u && p + 37 < e && src.b(p + 37) == '"') ve = p + 37;
            }
        }
        if (ve < 0) ve = ft_string_end(src, p + 1, e);
        if (ve < 0) return false;
        const Span sp{p + 1, ve, 0};
        if (id == K_AD) ad = sp;
        else if (id == K_ETYPE) et = sp;
        else if (id == K_ETIME) tm = sp;
        p = ft_clean<S, FAST>(src, ve + 1, e, c);
        if (p < 0) return false;
        if (c == '}') break;
        if (c != ',' && c != ';') return false;
    }
    const u32 need = require | K_AD | K_ETYPE | K_ETIME;
    return (seen & need) == need;
}

// The scan kernel's fourth tier: a flat line whose ad_id is 36 plain bytes, in the form
// the canonical tiers hand on (key words, event_time offset and first 20 bytes, view).
// Other ad_id lengths go to the deferred-line kernel (its table lookup takes any key).
template <class S, bool FAST = false>
__device__ __forceinline__ bool flat_tier(const S& src, int ls, int le, u32 require, CanonA& a, CanonB& b,
                                          const u32* kt = nullptr) {
    Span ad{0, 0, 0}, et{0, 0, 0}, tm{0, 0, 0};
    bool okp;
    if constexpr (FAST && std::is_same<S, LdsSrc>::value) {
        u32 adw[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) adw[k] = 0u;
        okp = flat_parse_bl2(src, ls, le, require, ad, et, tm, adw, kt);
        if (__builtin_expect(!okp, 0)) okp = flat_parse_lds(src, ls, le, require, ad, et, tm, adw);
        if (!okp || ad.e - ad.s != 36) return false;
        const bool fast_ad = adw[0] | adw[1] | adw[8];   // the id fast path kept the ad_id's words
#pragma unroll
        for (int k = 0; k < 9; ++k) a.kw[k] = fast_ad ? adw[k] : src.load4(ad.s + 4 * k);
    } else {
        if constexpr (FAST) okp = flat_parse_fast(src, ls, le, require, ad, et, tm);
        else okp = flat_parse<S, FAST>(src, ls, le, require, ad, et, tm);
        if (!okp || ad.e - ad.s != 36) return false;
#pragma unroll
        for (int k = 0; k < 9; ++k) a.kw[k] = src.load4(ad.s + 4 * k);
    }
    a.t0 = tm.s - ls;
    b.tlen = tm.e - tm.s;
#pragma unroll
    for (int k = 0; k < 5; ++k) b.td[k] = 4 * k < b.tlen ? src.load4(tm.s + 4 * k) : 0u;
    b.view = et.e - et.s == 4 && src.load4(et.s) == VIEW_W;
    return true;
}

// ---- layout 3: a learned key order --------------------------------------------------------
// Another producer's serializer writes every line with the same key order and the same
// spacing (", " / ": " or compact "," / ":").  The host reads that order off the batch's
// first line (ysb_capi.cpp learn_layout) and the scan then checks each line against it
// the way the vocabulary path checks the generator's: per pair, the key text with its
// separator and the value's opening quote compared in place as words (one aligned read
// span, one shift), a 36-byte id value and the separator after it in one span, any other
// value's closing quote found 16 bytes per step -- no key naming, no whitespace skips, the
// key order a uniform (scalar) branch.  Every byte up to the closing '}' is compared or
// shown to be a plain string byte, so an accepted line parses as org.json parses it
// (JSONObject(JSONTokener) on this subset: nextClean, nextString, putOnce, ',' / '}');
// any other line goes on to the flat tier, then the general parser.

// key index -> its text (ScanParams.learn_order)
__host__ __device__ constexpr const char* learn_key(int i) {
    return i == 0 ? "user_id" : i == 1 ? "page_id" : i == 2 ? "ad_id" : i == 3 ? "ad_type" : i == 4 ? "event_type"
         : i == 5 ? "event_time" : "ip_address";
}
constexpr int cstr_len(const char* s) { return *s ? 1 + cstr_len(s + 1) : 0; }
// the key text, its closing quote, the separator and the value's opening quote
template <int KI, bool CP>
struct KeyLit {
    static constexpr int KL = cstr_len(learn_key(KI));
    static constexpr int LEN = KL + (CP ? 3 : 4);
    static constexpr WordTpl<4> tpl() {
        char buf[20] = {};
        const char* k = learn_key(KI);
        int n = 0;
        for (; k[n]; ++n) buf[n] = k[n];
        buf[n++] = '"';
        buf[n++] = ':';
        if (!CP) buf[n++] = ' ';
        buf[n++] = '"';
        return make_words<4>(buf, 0, n);
    }
};

// One pair of a learned order: the key literal at p, its value, the separator after it
// (", " + the next key's quote, or the closing quote + '}' when `last`), its checks ORed into a
// u32 (0 = the pair is in the learned form; no bool lane-mask logic, see flat_parse_bl2).  p
// moves to the next key's text, or (last) to the '}'.  KI 0..2: 36-byte id values.
template <int KI, bool CP>
__device__ __forceinline__ u32 learned_pair_u(const LdsSrc& src, int& p, int e, bool last, u32 (&kw)[9], int& vs,
                                              int& ve) {
    using K = KeyLit<KI, CP>;
    constexpr WordTpl<4> T = K::tpl();
    constexpr u32 SEP = CP ? w4('"', ',', '"', 0) : w4('"', ',', ' ', '"');
    constexpr u32 SEPM = CP ? 0x00FFFFFFu : 0xFFFFFFFFu;
    constexpr int SEPL = CP ? 3 : 4;
    u32 kwd[4];
    load_span(src, p, kwd);
    u32 bad = words_diff(kwd, T);
    const int v = p + K::LEN;
    vs = v;
    if constexpr (KI <= 2) {
        u32 w[10];
        load_span(src, v, w);
        u32 pb = plain36_bad(w);
        if (__builtin_expect(pb != 0u, 0)) {   // not UUID-like: the exact plain-string flags
            pb = 0;
#pragma unroll
            for (int j = 0; j < 9; ++j) pb |= ft_flags(w[j]);
        }
        bad |= pb | (last ? (w[9] ^ w4('"', '}', 0, 0)) & 0xFFFFu : (w[9] ^ SEP) & SEPM);
        ve = v + 36;
        if constexpr (KI == 2) {
#pragma unroll
            for (int k = 0; k < 9; ++k) kw[k] = w[k];
        }
    } else {
        u32 A[5];
        load_span(src, v, A);
        u32 A10[10];
#pragma unroll
        for (int j = 0; j < 10; ++j) A10[j] = j < 5 ? A[j] : 0u;
        const u32 id = KI == 3 ? K_ADTYPE : KI == 4 ? K_ETYPE : KI == 5 ? K_ETIME : K_IP;
        const int la = bl2_vocab(id, A10);
        ve = v + la;
        if (__builtin_expect(la == 0, 0)) ve = ft_string_end(src, v, e);
        bad |= (u32)(ve - v) >> 31;              // ve < v: no closing quote
        const u32 x = src.load4(ve >= v ? ve : v);
        bad |= last ? (x ^ w4('"', '}', 0, 0)) & 0xFFFFu : (x ^ SEP) & SEPM;
    }
    p = last ? ve + 1 : ve + SEPL;
    return bad;
}

template <bool CP>
__device__ __forceinline__ bool learned_parse(const LdsSrc& src, int s, int e, const ScanParams& P, CanonA& a,
                                              CanonB& b) {
    u32 bad = (src.load4(s) & 0xFFFFu) ^ w4('{', '"', 0, 0);
    int p = s + 2;
    int ets = s, ete = s, tms = s, tme = s;
    u32 kw[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) kw[k] = 0u;
    const int n = (int)P.learn_n;
#pragma unroll 1
    for (int k = 0; k < n; ++k) {
        const bool last = k + 1 == n;
        int vs = 0, ve = 0;
        u32 pb;
        switch ((P.learn_code >> (3 * k)) & 7u) {   // uniform: a scalar branch
        case 0: pb = learned_pair_u<0, CP>(src, p, e, last, kw, vs, ve); break;
        case 1: pb = learned_pair_u<1, CP>(src, p, e, last, kw, vs, ve); break;
        case 2: pb = learned_pair_u<2, CP>(src, p, e, last, kw, vs, ve); break;
        case 3: pb = learned_pair_u<3, CP>(src, p, e, last, kw, vs, ve); break;
        case 4: pb = learned_pair_u<4, CP>(src, p, e, last, kw, vs, ve); ets = vs; ete = ve; break;
        case 5: pb = learned_pair_u<5, CP>(src, p, e, last, kw, vs, ve); tms = vs; tme = ve; break;
        default: pb = learned_pair_u<6, CP>(src, p, e, last, kw, vs, ve); break;
        }
        bad |= pb;
        p = bad == 0u ? p : s + 2;   // a failed lane keeps reading inside its line (result ignored)
    }
    bad |= (u32)(e - 1 - p) >> 31;   // the '}' (every compared byte lies before it)
#pragma unroll
    for (int k = 0; k < 9; ++k) a.kw[k] = kw[k];
    a.t0 = tms - s;
    b.tlen = tme - tms;
    load_span(src, tms, b.td);
    b.view = ete - ets == 4 && src.load4(ets) == VIEW_W;
    return bad == 0u;
}

// The deferred-line kernel's use: true = decided here (ok = counted); false = nothing
// counted, parse it in full.
__device__ __forceinline__ bool flat_line(const LdsSrc3& src, int s, int e, const ScanParams& P, Tally& t,
                                          u32& campaign, i64& bucket, bool& ok) {
    Span ad{0, 0, 0}, et{0, 0, 0}, tm{0, 0, 0};
    if (!flat_parse(src, s, e, P.require_mask, ad, et, tm)) return false;
    t.ev++;
    ok = finish_line(src, ad, et, tm, P, t, campaign, bucket);
    return true;
}

// Long.parseLong of a canonical line's event_time, then the bucket.  13 unsigned digits
// (epoch milliseconds 2001..2286) take a SWAR path; any other form the general one.
// FASTDIV (the .tbl instantiations, VALU-bound): with the reference's 10 s windows the
// bucket of a 13-digit time comes from its digit groups in 32-bit arithmetic,
// t / 10^4 = g0 * 10^5 + g1 * 10 + (g2 * 10 + d12) / 10^4 (exact: t >= 0, the first two
// terms of t are multiples of 10^4, and the result is below 10^9), instead of building the
// 64-bit t and a 64-bit magic-number division.
template <bool FASTDIV = false>
__device__ __forceinline__ bool canonical_bucket(const LdsSrc& src, const CanonB& b, int tms, const ScanParams& P,
                                                 i64& bucket) {
    i64 tv;
    bool ok = false;
    if (b.tlen == 13) {
        u32 bad = 0;
        const u32 g0 = swar_digits4(b.td[0], bad), g1 = swar_digits4(b.td[1], bad), g2 = swar_digits4(b.td[2], bad);
        const u32 d12 = (b.td[3] & 0xFFu) - '0';
        bad |= d12 > 9u;
        if constexpr (FASTDIV) {
            if (P.div.d == 10000 && bad == 0u) {
                bucket = (i64)(g0 * 100000u + g1 * 10u + (g2 * 10u + d12) / 10000u);
                return true;
            }
        }
        tv = (i64)(((u64)(g0 * 10000u + g1) * 10000u + g2) * 10u + d12);
        ok = bad == 0u;
    }
    if (ok) {
    } else if (b.tlen <= 20) {   // signs, other lengths, errors: the general digit loop decides
        ok = parse_digits_regs(b.td, b.tlen, tv);
    } else {
        ok = parse_digits(src, tms, tms + b.tlen, tv);
    }
    if (ok) bucket = div_trunc(tv, P.div);
    return ok;
}

// Out-of-ring cell (c, b) += v in the device hash map; false if the key cannot express
// the bucket or 64 probes find no slot (the caller then appends to the fallback list).
__device__ __forceinline__ bool side_add(const ScanParams& P, u32 c, i64 b, u32 v) {
    const i64 half = (i64)1 << (63 - P.side_cbits);
    if (b < -half || b >= half) return false;
    const unsigned long long key = ((unsigned long long)(b + half) << P.side_cbits) | c;
    const u32 h = (u32)(mix64(key) >> 32);
    for (u32 i = 0; i < 64u && i <= P.side_mask; ++i) {
        SideSlot* sl = &P.side[(h + i) & P.side_mask];
        const unsigned long long k = atomicCAS(&sl->key, SIDE_EMPTY, key);
        if (k == SIDE_EMPTY || k == key) {
            if (k == SIDE_EMPTY) atomicAdd(P.side_used, 1u);
            atomicAdd(&sl->count, (unsigned long long)v);
            return true;
        }
    }
    return false;
}

// Adds v views to (campaign, bucket): the ring cell if the bucket is live, else the
// exact side map (or its fallback list).
__device__ __forceinline__ void global_add(const ScanParams& P, i64 ring_lo, bool ring_set,
                                           u32 c, i64 b, u32 v, Tally& t) {
    if (ring_set) {
        const i64 rel = b - ring_lo;
        if (rel >= 0 && rel < (i64)P.ring_w) {
            atomicAdd(&P.counts[(u64)c * P.ring_w + (u64)(b & (i64)(P.ring_w - 1))], (unsigned long long)v);
            return;
        }
    }
    t.oor += v;
    if (side_add(P, c, b, v)) return;
    const u32 idx = atomicAdd(P.ovf_count, 1u);
    if (idx < P.ovf_cap) {
        OvfEntry en;
        en.campaign = c; en.count = v; en.bucket = b;
        P.ovf[idx] = en;
    } else {
        atomicAdd(&P.stats[ST_OVF_DROPPED], (unsigned long long)v);
    }
}

}  // namespace ysb
