// ysb_scan_canon.h -- the JSON fast paths of Kernel 1: the generator's layout
// and compact JSON as canonical tiers and vocabulary stages (DeserializeBolt,
// AdvertisingTopologyNative.java:257-276, on the generator's lines, core.clj:90-97).
// Part of the scan kernel's translation unit: included by ysb_scan.hip only, after the
// definitions it uses (the LDS sources, spans, load_span, the org.json machine).
#pragma once

namespace ysb {

// ---------------------------------------------------------------------------
// Fast path: the generator's layout (core.clj:90-96) -- the seven keys in order,
// ": " and ", " separators, string values without quotes or backslashes, the
// three UUID values 36 bytes long.  Every structural byte up to the closing '}' is
// compared, every value byte is shown free of '"', '\\' and NUL / CR / LF, and the
// variable tail's quotes are located exactly, which makes it exactly org.json's parse
// of such a line; any other line returns false and takes the general parser
// (ysb_orgjson.h).  Two dependent LDS batches per line.
// ---------------------------------------------------------------------------

// Per byte, bit 7 set if the byte may be '"', '\\' or a control byte below 0x0E (NUL
// ends org.json's input; a raw CR / LF inside a string throws): SWAR has-zero of
// w ^ '"' and w ^ '\\', has-less-than 0x0E of w.  Superset: a byte just above a true
// hit can be flagged falsely, never missed, and every candidate the parser relies on
// is verified by a compare (a control byte fails the compare and defers the line).
__device__ __forceinline__ u32 cand_z(u32 w) {
    const u32 tq = w ^ 0x22222222u, tb = w ^ 0x5C5C5C5Cu;
    return (((tq - 0x01010101u) & ~tq) | ((tb - 0x01010101u) & ~tb) | ((w - 0x0E0E0E0Eu) & ~w)) & 0x80808080u;
}
// The same flags packed to bits 0..3 (bit i = byte i), via the full-rate 24-bit
// multiply (bits 7/15/23 -> 28/29/30) plus bit 31.
__device__ __forceinline__ u32 cand_nib(u32 w) {
    const u32 z = cand_z(w);
    return (__umul24(z, 0x00204081u) | (z & 0x80000000u)) >> 28;
}

// The line's first 164 bytes: structural bytes (compared) and the three UUID values
// (scanned for candidates), as 41 little-endian words.
constexpr int PREFIX_WORDS = 41;
struct PrefixTpl {
    u32 e[PREFIX_WORDS];   // expected structural bytes
    u32 m[PREFIX_WORDS];   // 0xFF per structural byte
    u32 v[PREFIX_WORDS];   // 0x80 per value byte
};
// The prefix up to the ad_type value: parts[0] UUID parts[1] UUID parts[2] UUID parts[3].
constexpr PrefixTpl make_prefix_tpl(const char* p0, const char* p1, const char* p2, const char* p3) {
    PrefixTpl t{};
    const char* parts[4] = {p0, p1, p2, p3};
    int pos = 0;
    for (int k = 0; k < 4; ++k) {
        for (const char* q = parts[k]; *q; ++q, ++pos) {
            t.e[pos >> 2] |= (u32)(u8)*q << (8 * (pos & 3));
            t.m[pos >> 2] |= 0xFFu << (8 * (pos & 3));
        }
        if (k < 3)
            for (int j = 0; j < 36; ++j, ++pos) t.v[pos >> 2] |= 0x80u << (8 * (pos & 3));
    }
    return t;
}
constexpr PrefixTpl make_prefix_tpl() { return make_prefix_tpl(YSB_P0, YSB_P1, YSB_P2, YSB_P3); }

// Up to 20 expected bytes (a separator run) as 5 words + byte masks.
struct SepTpl {
    u32 e[5];
    u32 m[5];
};
constexpr SepTpl make_sep(const char* str) {
    SepTpl t{};
    int pos = 0;
    for (const char* q = str; *q; ++q, ++pos) {
        t.e[pos >> 2] |= (u32)(u8)*q << (8 * (pos & 3));
        t.m[pos >> 2] |= 0xFFu << (8 * (pos & 3));
    }
    return t;
}
__device__ __forceinline__ u32 sep_diff(const u32 (&w)[5], const SepTpl& t) {
    u32 d = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k)
        if (t.m[k]) d |= (w[k] ^ t.e[k]) & t.m[k];
    return d;
}

struct CanonA {   // after the first LDS batch
    u32 kw[9];     // the 36 ad_id bytes (.tbl: bytes 74..109)
    int e3, e4, e5, e6;   // closing quotes of ad_type, event_type, event_time, ip_address
                          // (.tbl: e3, e4 = the 4th and 5th '|'; e5, e6 = '|' bitmap of bytes 96..159)
    int t0;        // line offset of the event_time value
};

// ---------------------------------------------------------------------------
// Canonical tiers (lines the vocabulary path below does not take): the generator's seven
// keys in its order with any string values -- other ip addresses, ad_types, event_types
// or event_time lengths -- in two layouts, the generator's (": " and ", ", CP = false)
// and compact JSON (":" and ",", CP = true).  Stage 1 reads the line's first 160-164
// bytes and 28 more raw dwords: the prefix is compared with a template (structural bytes
// exact, the three 36-byte UUID values shown free of '"', '\\' and control bytes), and
// the tail's value ends are the next quote candidates of a SWAR bitmap; stage 2 compares
// the three tail separators, the closing "}" and fetches event_type / event_time.  Every
// byte up to '}' is compared or classified, so an accepted line parses exactly as
// org.json parses it; anything else goes on to the general parser.
// ---------------------------------------------------------------------------
template <bool CP>
struct CanonGeo {
    static constexpr int PREFIX = CP ? 157 : 164;     // bytes before the ad_type value
    static constexpr int PW = (PREFIX + 3) / 4;        // prefix words compared
    static constexpr int TB = (PREFIX / 4) * 4;        // the tail bitmap starts at this (aligned) byte
    static constexpr int TW = 28;                      // raw tail dwords scanned
    static constexpr int MAXLEN = TB + 4 * TW - 3;     // longest line the tier takes
    static constexpr int MINLEN = CP ? 207 : 220;
    static constexpr int AD = CP ? 108 : 113;          // the ad_id value
    static constexpr int SEP = CP ? 16 : 18;           // "<value>", "<key>": "<value>"
};
constexpr PrefixTpl make_compact_tpl() {
    return make_prefix_tpl("{\"user_id\":\"", "\",\"page_id\":\"", "\",\"ad_id\":\"", "\",\"ad_type\":\"");
}

template <bool CP>
__device__ __forceinline__ bool canon_stage1(const LdsSrc& src, int s, int e, CanonA& c) {
    using G = CanonGeo<CP>;
    constexpr PrefixTpl T = CP ? make_compact_tpl() : make_prefix_tpl();
    const int L = e - s;
    if (L < G::MINLEN || L > G::MAXLEN) return false;
    const int a = s >> 2;
    const u32 sb = (u32)(s & 3);
    u32 P[G::PW + 1];
#pragma unroll
    for (int k = 0; k <= G::PW; ++k) P[k] = src.d[a + k];
    u32 R[G::TW];   // raw dwords from line offset TB - sb
#pragma unroll
    for (int k = 0; k < G::TW; ++k) R[k] = src.d[a + G::TB / 4 + k];
    // prefix: XOR-accumulated compares and candidate flags; d == 0 <=> all hold
    u32 d = 0, W[G::PW];
#pragma unroll
    for (int j = 0; j < G::PW; ++j) {
        W[j] = __builtin_amdgcn_alignbyte(P[j + 1], P[j], sb);   // line bytes 4j..4j+3
        if (T.m[j] == 0xFFFFFFFFu) d |= W[j] ^ T.e[j];
        else if (T.m[j] != 0u) d |= (W[j] ^ T.e[j]) & T.m[j];
        if (T.v[j] != 0u) d |= cand_z(W[j]) & T.v[j];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k)
        c.kw[k] = __builtin_amdgcn_alignbyte(W[G::AD / 4 + k + 1], W[G::AD / 4 + k], (u32)(G::AD & 3));
    // tail: candidate bitmap, bit i = line byte TB - sb + i
    u32 B[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < G::TW; ++k) B[k >> 3] |= cand_nib(R[k]) << (4 * (k & 7));
    const int tb0 = G::TB - (int)sb;
    // first candidate at or after line offset p (p >= tb0), via a 64-bit window
    auto nextq = [&](int p) -> int {
        const int q = p - tb0;
        const int k = q >> 5;
        const u32 lo = k == 0 ? B[0] : k == 1 ? B[1] : k == 2 ? B[2] : k == 3 ? B[3] : 0u;
        const u32 hi = k == 0 ? B[1] : k == 1 ? B[2] : k == 2 ? B[3] : 0u;
        const u64 w = (((u64)hi << 32) | lo) >> (q & 31);
        return w ? p + (int)__builtin_ctzll(w) : (1 << 20);
    };
    c.e3 = nextq(G::PREFIX);          // end of ad_type
    c.e4 = nextq(c.e3 + G::SEP);      // end of event_type
    c.e5 = nextq(c.e4 + G::SEP);      // end of event_time
    c.e6 = nextq(c.e5 + G::SEP);      // end of ip_address
    c.t0 = c.e4 + G::SEP;
    return d == 0u && c.e6 + 2 <= L;
}

// ---- word-at-a-time byte scans (the vocabulary path's ip value, the flat tier) -------------

// The next byte > ' ' at or after p (its position; c = the byte), or -1 if the end of
// the line or a NUL comes first.  Four bytes per step; of the two flag sets the lowest
// flagged byte is exact (a false flag only sits above a true one: zero_bytes' borrow
// above a zero byte, the +0x5F carry above a byte >= 0xA1, itself flagged by its top bit).
template <class S, bool FAST = false>
__device__ __forceinline__ int ft_clean(const S& src, int p, int e, u32& c) {
    if constexpr (FAST) {
        // the first four bytes outside the loop: nearly every call ends there, and the
        // loop becomes a region the wave skips when no lane needs it
        if (p < e) {
            const u32 x = src.load4(p);
            const u32 z = (((x + 0x5F5F5F5Fu) | x) & 0x80808080u) | zero_bytes(x);
            if (z != 0u) {
                const int k = __builtin_ctz(z) >> 3;
                c = (x >> (8 * k)) & 0xFFu;
                return (p + k < e && c != 0u) ? p + k : -1;
            }
            p += 4;
        }
    }
    for (; p < e; p += 4) {
        const u32 x = src.load4(p);
        const u32 z = (((x + 0x5F5F5F5Fu) | x) & 0x80808080u) | zero_bytes(x);
        if (z != 0u) {
            const int k = __builtin_ctz(z) >> 3;
            c = (x >> (8 * k)) & 0xFFu;
            return (p + k < e && c != 0u) ? p + k : -1;
        }
    }
    return -1;
}

// The closing '"' of a string whose content starts at p, or -1 if a backslash, a control
// byte or the end of the line comes first (lowest flagged byte exact, as above).  16
// bytes per step: four independent LDS words (may read up to 15 bytes past e; a flag
// there is rejected by the at < e test).
__device__ __forceinline__ u32 ft_flags(u32 w) {
    return zero_bytes(w ^ 0x22222222u) | zero_bytes(w ^ 0x5C5C5C5Cu) | zero_bytes(w & 0xE0E0E0E0u);
}
template <class S>
__device__ __forceinline__ int ft_string_end(const S& src, int p, int e) {
    int q = p & ~3;
    u32 first = 0xFFFFFFFFu << ((p & 3) << 3);
    for (;;) {
        u32 w[4], z[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = src.d[(q >> 2) + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = ft_flags(w[k]);
        z[0] &= first;
        u32 zz = 0, ww = 0;
        int base = 0;
#pragma unroll
        for (int k = 3; k >= 0; --k)
            if (z[k] != 0u) { zz = z[k]; ww = w[k]; base = 4 * k; }
        if (zz != 0u) {
            const int bi = __builtin_ctz(zz) >> 3;
            const int at = q + base + bi;
            return (at < e && ((ww >> (8 * bi)) & 0xFFu) == '"') ? at : -1;
        }
        q += 16;
        first = 0xFFFFFFFFu;
        if (q >= e) return -1;
    }
}

struct CanonB {   // after the second LDS batch
    bool view;
    u32 td[5];     // event_time bytes (first 20)
    int tlen;
};


// Stage 2: the variable tail -- the three separators, the closing "}", the event_type
// value and the event_time digits -- in one batch of LDS reads.
template <bool CP>
__device__ __forceinline__ bool canon_stage2(const LdsSrc& src, int s, int e, const CanonA& a, CanonB& c) {
    using G = CanonGeo<CP>;
    constexpr SepTpl S4 = make_sep(CP ? "\",\"event_type\":\"" : "\", \"event_type\": \"");
    constexpr SepTpl S5 = make_sep(CP ? "\",\"event_time\":\"" : "\", \"event_time\": \"");
    constexpr SepTpl S6 = make_sep(CP ? "\",\"ip_address\":\"" : "\", \"ip_address\": \"");
    u32 t4[5], t5[5], t6[5], t7[1], ev[1];
    load_span(src, s + a.e3, t4);
    load_span(src, s + a.e4, t5);
    load_span(src, s + a.e5, t6);
    load_span(src, s + a.e6, t7);
    load_span(src, s + a.e3 + G::SEP, ev);
    load_span(src, s + a.t0, c.td);
    u32 d = sep_diff(t4, S4) | sep_diff(t5, S5) | sep_diff(t6, S6);
    d |= (t7[0] & 0xFFFFu) ^ w4('"', '}', 0, 0);
    // org.json's JSONObject(String) stops at the closing '}': whatever follows it (normally
    // the '\n') is never read.
    if (d != 0u) return false;
    c.view = (a.e4 - (a.e3 + G::SEP) == 4) && ev[0] == VIEW_W;
    c.tlen = a.e5 - a.t0;
    return true;
}

// Four ASCII digits (byte 0 most significant) -> 0..9999; bad != 0 if any byte is not a digit.
__device__ __forceinline__ u32 swar_digits4(u32 w, u32& bad) {
    const u32 dgt = w - 0x30303030u;                                        // per byte, borrow-free when valid
    bad |= (w & 0xF0F0F0F0u) ^ 0x30303030u;                                 // high nibbles must be 3
    bad |= (dgt + 0x76767676u) & 0x80808080u;                               // low nibbles must be <= 9
    const u32 pr = (dgt & 0x00FF00FFu) * 10u + ((dgt >> 8) & 0x00FF00FFu); // two 2-digit halves
    return (pr & 0xFFFFu) * 100u + (pr >> 16);
}

// ---------------------------------------------------------------------------
// Vocabulary fast path: the generator's lines are the template
// above with values from closed sets -- ad_type one of banner / modal / sponsored-search /
// mail / mobile, event_type one of view / click / purchase (core.clj:68-69,164-165), a
// 13-digit event_time and ip_address "1.2.3.4" (:96,:181).  Stage 1 reads the 164-byte
// prefix plus 36 bytes (the ad_type value and where event_type starts), names the ad_type
// by an exact compare and the event_type by its first byte; every later position then
// follows, and stage 2 compares the rest of the line up to the closing '}' exactly
// (separators, keys, the event_type value, the ip value) and checks the 13 time bytes are
// digits.  So every byte up to '}' is either compared or shown to be a UUID byte free of
// '"', '\\' and control bytes or a digit: the line parses exactly as org.json parses
// it.  No candidate scan of the tail.  A line it rejects tries the canonical tiers
// (canon_stage1/2: other values, then compact JSON) before the general parser.
// ---------------------------------------------------------------------------
constexpr int VOC_WORDS = 50;            // line bytes 0..199

// Expected bytes [from, to) of str as N words + byte masks (compile time).
template <int N>
struct WordTpl {
    u32 e[N];
    u32 m[N];
};
template <int N>
constexpr WordTpl<N> make_words(const char* str, int from, int to) {
    WordTpl<N> t{};
    for (int pos = from; pos < to; ++pos) {
        t.e[pos >> 2] |= (u32)(u8)str[pos] << (8 * (pos & 3));
        t.m[pos >> 2] |= 0xFFu << (8 * (pos & 3));
    }
    return t;
}
template <int N>
__device__ __forceinline__ u32 words_diff(const u32 (&w)[N], const WordTpl<N>& t) {
    u32 d = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (t.m[k] == 0xFFFFFFFFu) d |= w[k] ^ t.e[k];
        else if (t.m[k] != 0u) d |= (w[k] ^ t.e[k]) & t.m[k];
    }
    return d;
}
// bytes POS..POS+3 / byte POS of the line from its aligned words W (compile-time POS)
template <int POS, int N>
__device__ __forceinline__ u32 word_at(const u32 (&W)[N]) {
    if constexpr ((POS & 3) == 0) return W[POS >> 2];
    else return __builtin_amdgcn_alignbyte(W[(POS >> 2) + 1], W[POS >> 2], (u32)(POS & 3));
}
template <int POS, int N>
__device__ __forceinline__ u32 byte_at(const u32 (&W)[N]) {
    return (W[POS >> 2] >> (8 * (POS & 3))) & 0xFFu;
}

// The vocabulary path for the generator's layout (CP = false: ": " and ", ") and the same
// keys as compact JSON (CP = true: ":" and ",", the third tier's lines).
template <bool CP>
__device__ __forceinline__ bool vocab_stage1(const LdsSrc& src, int s, int e, CanonA& c) {
    using G = CanonGeo<CP>;
    constexpr PrefixTpl T = CP ? make_compact_tpl() : make_prefix_tpl();
    constexpr int PF = G::PREFIX, SEP = G::SEP, AD = G::AD;
    constexpr int MINLEN = PF + 4 + 4 + 3 * SEP + 13 + 7 + 2;   // shortest ad_type and event_type
    static_assert(PF + 16 + SEP < 4 * VOC_WORDS, "the event_type's first byte is among the words read");
    const int L = e - s;
    if (L < MINLEN) return false;
    const int a = s >> 2;
    const u32 sb = (u32)(s & 3);
    u32 P[VOC_WORDS + 1];
#pragma unroll
    for (int k = 0; k <= VOC_WORDS; ++k) P[k] = src.d[a + k];
    u32 d = 0, W[VOC_WORDS];
#pragma unroll
    for (int j = 0; j < VOC_WORDS; ++j) W[j] = __builtin_amdgcn_alignbyte(P[j + 1], P[j], sb);   // bytes 4j..4j+3
#pragma unroll
    for (int j = 0; j < G::PW; ++j) {
        if (T.m[j] == 0xFFFFFFFFu) d |= W[j] ^ T.e[j];
        else if (T.m[j] != 0u) d |= (W[j] ^ T.e[j]) & T.m[j];
        if (T.v[j] != 0u) d |= cand_z(W[j]) & T.v[j];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k)   // the ad_id bytes
        c.kw[k] = __builtin_amdgcn_alignbyte(W[(AD >> 2) + 1 + k], W[(AD >> 2) + k], (u32)(AD & 3));
    // ad_type at byte PF, exactly one of the five
    const u32 a0 = word_at<PF>(W), a1 = word_at<PF + 4>(W);
    int La = 0;
    if (a0 == w4('b', 'a', 'n', 'n') && (a1 & 0xFFFFu) == w4('e', 'r', 0, 0)) La = 6;
    else if (a0 == w4('m', 'a', 'i', 'l')) La = 4;
    else if (a0 == w4('m', 'o', 'd', 'a') && (a1 & 0xFFu) == 'l') La = 5;
    else if (a0 == w4('m', 'o', 'b', 'i') && (a1 & 0xFFFFu) == w4('l', 'e', 0, 0)) La = 6;
    else if (a0 == w4('s', 'p', 'o', 'n') && a1 == w4('s', 'o', 'r', 'e') && word_at<PF + 8>(W) == w4('d', '-', 's', 'e') &&
             word_at<PF + 12>(W) == w4('a', 'r', 'c', 'h'))
        La = 16;
    // event_type's first byte at PF + La + SEP
    u32 et0 = La == 4   ? byte_at<PF + 4 + SEP>(W)
              : La == 5 ? byte_at<PF + 5 + SEP>(W)
              : La == 6 ? byte_at<PF + 6 + SEP>(W)
                        : byte_at<PF + 16 + SEP>(W);
    if (__builtin_expect(La == 0 && d == 0u, 0)) {
        // another ad_type (a branch the generator's lines never take): any plain string
        // value -- no quote, backslash or control byte before its closing quote; stage 2
        // checks everything after that quote as for the five
        const int q = ft_string_end(src, s + PF, e);
        if (q > s + PF && q - s - PF <= 64) {
            La = q - s - PF;
            et0 = src.b(q + SEP);
        }
    }
    const int Le = et0 == 'v' ? 4 : et0 == 'c' ? 5 : et0 == 'p' ? 8 : 0;
    c.e3 = PF + La;            // closing quote of ad_type
    c.e4 = c.e3 + SEP + Le;    // of event_type
    c.e5 = c.e4 + SEP + 13;    // of event_time
    c.e6 = c.e5 + SEP + 7;     // of ip_address
    c.t0 = c.e4 + SEP;
    return d == 0u && La != 0 && Le != 0 && c.e6 + 2 <= L;
}

template <bool CP>
__device__ __forceinline__ bool vocab_stage2(const LdsSrc& src, int s, int e, const CanonA& a, CanonB& c) {
    using G = CanonGeo<CP>;
    constexpr int SEP = G::SEP;
    constexpr WordTpl<5> S4 = make_words<5>(CP ? "\",\"event_type\":\"" : "\", \"event_type\": \"", 0, SEP);
    constexpr WordTpl<5> S5 = make_words<5>(CP ? "\",\"event_time\":\"" : "\", \"event_time\": \"", 0, SEP);
    constexpr const char* TAIL = CP ? "\",\"ip_address\":\"1.2.3.4\"}" : "\", \"ip_address\": \"1.2.3.4\"}";
    constexpr WordTpl<7> S6 = make_words<7>(TAIL, 0, SEP);              // the key
    constexpr WordTpl<7> IP = make_words<7>(TAIL, SEP, SEP + 9);        // 1.2.3.4"}
    u32 t4[5], ev[2], t5[5], t6[7];
    load_span(src, s + a.e3, t4);
    load_span(src, s + a.e3 + SEP, ev);
    load_span(src, s + a.e4, t5);
    load_span(src, s + a.e4 + SEP, c.td);
    load_span(src, s + a.e5, t6);
    const u32 d = words_diff(t4, S4) | words_diff(t5, S5);
    const u32 dkey = words_diff(t6, S6), dip = words_diff(t6, IP);
    // the event_type value: exactly the one its first byte named
    const int Le = a.e4 - a.e3 - SEP;
    const bool etok = Le == 4   ? ev[0] == w4('v', 'i', 'e', 'w')
                      : Le == 5 ? (ev[0] == w4('c', 'l', 'i', 'c') && (ev[1] & 0xFFu) == 'k')
                                : (ev[0] == w4('p', 'u', 'r', 'c') && ev[1] == w4('h', 'a', 's', 'e'));
    // the event_time value: 13 ASCII digits
    u32 bad = 0;
    swar_digits4(c.td[0], bad);
    swar_digits4(c.td[1], bad);
    swar_digits4(c.td[2], bad);
    bad |= ((c.td[3] & 0xFFu) - '0') > 9u;
    c.view = Le == 4;
    c.tlen = 13;
    // org.json's JSONObject(String) stops at the closing '}': what follows is never read.
    const bool pre = d == 0u && dkey == 0u && etok && bad == 0u;
    if (__builtin_expect(pre && dip != 0u, 0)) {
        // another ip address (a branch the generator's lines never take): any plain string
        // value -- no quote, backslash or control byte before its closing quote -- then '}'
        const int q = ft_string_end(src, s + a.e5 + SEP, e);
        return q >= 0 && q + 1 < e && src.b(q + 1) == '}';
    }
    return pre && dip == 0u;
}

}  // namespace ysb
