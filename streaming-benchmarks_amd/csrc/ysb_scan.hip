// ysb_scan.hip -- Kernel 1: the fused YSB advertising hot path on gfx950.
//
// One pass over a batch of JSON event lines does what the reference's Flink chain
// does per record (flink-benchmarks/.../AdvertisingTopologyNative.java:122-138,
// storm-benchmarks/.../AdvertisingTopology.java:53-176):
//
//   DeserializeBolt   new JSONObject(line).getString(...)          (:263-272)
//   EventFilterBolt   event_type.equals("view")                     (:434)
//   project           (ad_id, event_time)                           (Storm :103-107)
//   RedisJoinBolt     campaign = ad_campaign.get(ad_id), drop miss  (:461-474)
//   CampaignProcessorCommon.execute
//                     bucket = Long.parseLong(event_time) / 10000;
//                     windows[bucket][campaign].seenCount++         (CampaignProcessorCommon.java:57-67)
//
// Structure (DESIGN.md "Kernel 1"): one-wave workgroups (64 lines per tile), 8 per
// CU, each walking a contiguous run of tiles.  Phase A streams a tile's bytes
// HBM -> registers -> LDS with 16-byte nontemporal buffer loads issued one tile ahead.
// Phase B gives each lane one line: the canonical fast path checks the generator's
// layout against a compile-time template in two batches of LDS reads and extracts the
// 36-byte ad_id, event_type and event_time; the join probes the 2-choice cuckoo table
// (raw UUID words); joined views are counted into per-workgroup LDS (campaign, window)
// counters flushed to the HBM ring with 64-bit atomics when the workgroup's window
// moves.  Any other line goes to a deferred list that defer_kernel parses with the
// general org.json parser (ysb_orgjson.h).  scan_kernel<*, true> does the same for the
// fork's pipe-delimited rows (tbl_stage1/2, deferred rows through process_tbl_line).
#include <type_traits>

#include "ysb_kernels.h"

namespace ysb {

// Key ids (bit masks) of the fields DeserializeBolt reads.
enum : u32 {
    K_USER = 1u << 0, K_PAGE = 1u << 1, K_AD = 1u << 2, K_ADTYPE = 1u << 3,
    K_ETYPE = 1u << 4, K_ETIME = 1u << 5, K_IP = 1u << 6,
    K_OTHER = 1u << 7   // flat_parse_fast: a key DeserializeBolt does not read
};

__host__ __device__ constexpr u32 w4(char a, char b, char c, char d) {
    return (u32)(u8)a | ((u32)(u8)b << 8) | ((u32)(u8)c << 16) | ((u32)(u8)d << 24);
}
constexpr u32 VIEW_W = w4('v', 'i', 'e', 'w');

// ---------------------------------------------------------------------------
// Byte sources.  Positions are ints relative to the source base.
// ---------------------------------------------------------------------------
struct LdsSrc {
    const u32* d;   // tile bytes as dwords
    __device__ __forceinline__ u32 b(int p) const { return (d[p >> 2] >> ((p & 3) << 3)) & 0xFFu; }
    __device__ __forceinline__ u32 load4(int p) const {
        const u32 lo = d[p >> 2], hi = d[(p >> 2) + 1];
        return __builtin_amdgcn_alignbyte(hi, lo, (u32)(p & 3));
    }
};

// The same through an explicitly LDS-qualified pointer, for code that is not inlined into
// the kernel (the general parser): ds_read instead of flat loads.
typedef __attribute__((address_space(3))) const u32 lds_u32;
struct LdsSrc3 {
    lds_u32* d;
    __device__ __forceinline__ u32 b(int p) const { return (d[p >> 2] >> ((p & 3) << 3)) & 0xFFu; }
    __device__ __forceinline__ u32 load4(int p) const {
        const u32 lo = d[p >> 2], hi = d[(p >> 2) + 1];
        return __builtin_amdgcn_alignbyte(hi, lo, (u32)(p & 3));
    }
};

struct GlbSrc {  // slow path for tiles that do not fit the LDS tile
    const u8* base;
    u64 n;
    __device__ __forceinline__ u32 b(int p) const { return (u64)p < n ? base[p] : 0u; }
    __device__ __forceinline__ u32 load4(int p) const {
        return b(p) | (b(p + 1) << 8) | (b(p + 2) << 16) | (b(p + 3) << 24);
    }
};

struct BufSrc {  // decoded (un-escaped) strings
    const u8* buf;
    __device__ __forceinline__ u32 b(int p) const { return buf[p]; }
    __device__ __forceinline__ u32 load4(int p) const {
        return (u32)buf[p] | ((u32)buf[p + 1] << 8) | ((u32)buf[p + 2] << 16) | ((u32)buf[p + 3] << 24);
    }
};

struct Span { int s, e; int esc; };

__device__ __forceinline__ bool is_hex(u32 c) {
    return (c - '0') < 10u || ((c | 0x20u) - 'a') < 6u;
}
__device__ __forceinline__ u32 hex_val(u32 c) { return (c - '0') < 10u ? c - '0' : (c | 0x20u) - 'a' + 10; }


// Key id of the key string [s, s+len) (0 = a key DeserializeBolt does not read).
template <class S>
__device__ __forceinline__ u32 match_key_raw(const S& src, int s, int len) {
    if (len == 5) {
        return (src.load4(s) == w4('a', 'd', '_', 'i') && src.b(s + 4) == 'd') ? K_AD : 0u;
    }
    if (len == 7) {
        const u32 a = src.load4(s), b = src.load4(s + 3);
        if (a == w4('u', 's', 'e', 'r') && b == w4('r', '_', 'i', 'd')) return K_USER;
        if (a == w4('p', 'a', 'g', 'e') && b == w4('e', '_', 'i', 'd')) return K_PAGE;
        if (a == w4('a', 'd', '_', 't') && b == w4('t', 'y', 'p', 'e')) return K_ADTYPE;
        return 0u;
    }
    if (len == 10) {
        const u32 a = src.load4(s), b = src.load4(s + 4), c = src.load4(s + 6);
        if (a == w4('e', 'v', 'e', 'n')) {
            if (b == w4('t', '_', 't', 'y') && c == w4('t', 'y', 'p', 'e')) return K_ETYPE;
            if (b == w4('t', '_', 't', 'i') && c == w4('t', 'i', 'm', 'e')) return K_ETIME;
            return 0u;
        }
        if (a == w4('i', 'p', '_', 'a') && b == w4('d', 'd', 'r', 'e') && c == w4('r', 'e', 's', 's')) return K_IP;
    }
    return 0u;
}

// bytes of x that are zero (exact for the lowest one: a false flag only sits above a true one)
__device__ __forceinline__ u32 zero_bytes(u32 x) { return (x - 0x01010101u) & ~x & 0x80808080u; }

}  // namespace ysb

#include "ysb_orgjson.h"

namespace ysb {

template <class S>
__device__ __forceinline__ bool span_is_view(const S& src, const Span& et) {
    if (!et.esc) return et.e - et.s == 4 && src.load4(et.s) == VIEW_W;
    u8 buf[12];
    const int n = decode_str(src, et.s, et.e, buf, 8);
    return n == 4 && buf[0] == 'v' && buf[1] == 'i' && buf[2] == 'e' && buf[3] == 'w';
}

// ad_id value -> zero-padded key words (false if longer than any table key can be).
template <class S>
__device__ __forceinline__ bool span_key(const S& src, const Span& ad, u32 (&kw)[KEY_WORDS], u32& klen) {
    if (!ad.esc) {
        const int len = ad.e - ad.s;
        if (len > (int)MAX_KEY_BYTES) return false;
        klen = (u32)len;
#pragma unroll
        for (int k = 0; k < (int)KEY_WORDS; ++k) {
            const int r = len - 4 * k;
            u32 w = r > 0 ? src.load4(ad.s + 4 * k) : 0u;
            if (r > 0 && r < 4) w &= (1u << (8 * r)) - 1u;
            kw[k] = w;
        }
        return true;
    }
    u8 buf[MAX_KEY_BYTES + 4];
    const int n = decode_str(src, ad.s, ad.e, buf, MAX_KEY_BYTES);
    if (n > (int)MAX_KEY_BYTES) return false;
    klen = (u32)n;
#pragma unroll
    for (int k = 0; k < (int)KEY_WORDS; ++k) {
        u32 w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * k + j < n) w |= (u32)buf[4 * k + j] << (8 * j);
        kw[k] = w;
    }
    return true;
}

__device__ __forceinline__ u32 key_hash_dev(const u32 (&w)[KEY_WORDS], u32 len) {
    u32 h = 0x811C9DC5u ^ (len * 0x9E3779B1u);
    const u32 nw = (len + 3) >> 2;
#pragma unroll
    for (u32 k = 0; k < KEY_WORDS; ++k) {
        if (k < nw) {
            h = (h ^ w[k]) * 0x01000193u;
            h ^= h >> 15;
        }
    }
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

// RedisJoinBolt's ad_campaign.get(ad_id) (AdvertisingTopologyNative.java:464) as a
// linear probe of the HBM/L2-resident table; -1 on a miss.
__device__ __forceinline__ int probe(const u32* __restrict__ table, u32 mask, const u32 (&kw)[KEY_WORDS], u32 klen) {
    u32 h = key_hash_dev(kw, klen);
    for (u32 i = 0; i <= mask; ++i) {
        const uint4* slot = reinterpret_cast<const uint4*>(table + (u64)((h + i) & mask) * SLOT_WORDS);
        const uint4 s0 = slot[0];
        if (s0.y == EMPTY_SLOT) return -1;
        if (s0.x == klen) {
            const uint4 s1 = slot[1], s2 = slot[2], s3 = slot[3];
            const u32 diff = (s0.z ^ kw[0]) | (s0.w ^ kw[1]) | (s1.x ^ kw[2]) | (s1.y ^ kw[3]) |
                             (s1.z ^ kw[4]) | (s1.w ^ kw[5]) | (s2.x ^ kw[6]) | (s2.y ^ kw[7]) |
                             (s2.z ^ kw[8]) | (s2.w ^ kw[9]) | (s3.x ^ kw[10]) | (s3.y ^ kw[11]) |
                             (s3.z ^ kw[12]) | (s3.w ^ kw[13]);
            if (diff == 0) return (int)s0.y;
        }
    }
    return -1;
}

// Long.parseLong(event_time) (CampaignProcessorCommon.java:58): [+-]?[0-9]+ within int64.
template <class S>
__device__ __forceinline__ bool parse_digits(const S& src, int p, int e, i64& out) {
    if (p >= e) return false;
    bool neg = false;
    const u32 c0 = src.b(p);
    if (c0 == '-') { neg = true; ++p; }
    else if (c0 == '+') { ++p; }
    if (p >= e) return false;
    u64 acc = 0;
    const u32 last_max = neg ? 8u : 7u;
    for (; p < e; ++p) {
        const u32 d = src.b(p) - '0';
        if (d > 9u) return false;
        if (acc >= 922337203685477580ULL) {
            if (acc > 922337203685477580ULL || d > last_max) return false;
        }
        acc = acc * 10u + d;
    }
    out = neg ? (i64)(0 - acc) : (i64)acc;
    return true;
}

template <class S>
__device__ __forceinline__ bool span_long(const S& src, const Span& tm, i64& out) {
    if (!tm.esc) return parse_digits(src, tm.s, tm.e, out);
    u8 buf[68];
    const int n = decode_str(src, tm.s, tm.e, buf, 64);
    if (n > 64) return false;
    return parse_digits(BufSrc{buf}, 0, n, out);
}

// N realigned words of the source starting at byte p (N+1 aligned LDS reads, issued
// back to back, then one v_alignbyte each).
template <int N>
__device__ __forceinline__ void load_span(const LdsSrc& src, int p, u32 (&w)[N]) {
    u32 a[N + 1];
    const int base = p >> 2;
#pragma unroll
    for (int k = 0; k <= N; ++k) a[k] = src.d[base + k];
    const u32 sh = (u32)(p & 3);
#pragma unroll
    for (int k = 0; k < N; ++k) w[k] = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sh);
}

// Long.parseLong over <= 20 bytes held in registers.
__device__ __forceinline__ bool parse_digits_regs(const u32 (&w)[5], int len, i64& out) {
    if (len <= 0 || len > 20) return false;
    const u32 c0 = w[0] & 0xFFu;
    const bool neg = c0 == '-';
    const int k0 = (c0 == '-' || c0 == '+') ? 1 : 0;
    if (k0 >= len) return false;
    u64 acc = 0;
    bool ok = true;
    const u32 last_max = neg ? 8u : 7u;
#pragma unroll
    for (int k = 0; k < 20; ++k) {
        if (k >= k0 && k < len) {
            const u32 d = ((w[k >> 2] >> ((k & 3) * 8)) & 0xFFu) - '0';
            ok &= d <= 9u;
            if (acc >= 922337203685477580ULL) ok &= !(acc > 922337203685477580ULL || d > last_max);
            acc = acc * 10u + d;
        }
    }
    out = neg ? (i64)(0 - acc) : (i64)acc;
    return ok;
}

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
// Vocabulary fast path (YSB_VOCAB, the default): the generator's lines are the template
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
#ifndef YSB_VOCAB
#define YSB_VOCAB 1
#endif
#ifndef YSB_FLAT_TIER
#define YSB_FLAT_TIER 1   // flat objects in any key order: in the scan (fourth tier) and the deferred-line kernel
#endif
#ifndef YSB_CANON_TIERS
#define YSB_CANON_TIERS 1
#endif
#ifndef YSB_FLAT_FAST_TIER4
#define YSB_FLAT_FAST_TIER4 0   // A/B only: flat_parse_fast as the default kernel's fourth tier
#endif
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

// ---------------------------------------------------------------------------
// .tbl fast path (YSB_F_FORMAT_TBL): the generator's rows, user|page|ad|ad_type|
// event_type|event_time\n with 36-byte UUIDs -- the first three '|' at bytes 36, 73 and
// 110, the next two found in a '|' bitmap of the line's first 160 bytes, no other '|'
// before the terminator.  Then line.split("\\|") (MockWindowedFlatMap,
// AdvertisingTopologyNative.java:197-226) has items[2] = bytes 74..109, items[4] between
// the 4th and 5th '|', items[5] = the rest up to the "\n" / "\r\n" readLine strips.  Any
// other row is deferred to process_tbl_line.  Same two-batch shape as the JSON path.
// ---------------------------------------------------------------------------
constexpr int TBL_WORDS = 40;                          // bytes 0..159 of the line
#ifndef YSB_TBL_READ64
#define YSB_TBL_READ64 0     // round 3 A/B: 1 (ds_read2_b64) -2 %, 2 (ds_read_b64) -1 %
#endif
#ifndef YSB_TBL_ZCMP
#define YSB_TBL_ZCMP 1
#endif
constexpr int TBL_MIN_LEN = 116, TBL_MAX_LEN = 4 * TBL_WORDS;

// Per byte, bit 7 set if the byte may be '|' (SWAR has-zero of w ^ '|'); the lowest flag
// of a word is always a true '|', a flag above a true one may be false.
__device__ __forceinline__ u32 bar_nib(u32 w) {
    const u32 t = w ^ 0x7C7C7C7Cu;
    const u32 z = ((t - 0x01010101u) & ~t) & 0x80808080u;
    return (__umul24(z, 0x00204081u) | (z & 0x80000000u)) >> 28;
}

__device__ __forceinline__ bool tbl_stage1(const LdsSrc& src, int s, int e, CanonA& c) {
    const int L = e - s;
    if (L < TBL_MIN_LEN || L > TBL_MAX_LEN) return false;
    const u32 sb = (u32)(s & 3);
    u32 P[TBL_WORDS + 1];
#if YSB_TBL_READ64
    // 8-byte reads (ds_read_b64: half the instructions of dword reads, banks (a/4) mod 64)
    // from the row start rounded down to 8 bytes, then one dword select per word
    const int a8 = s >> 3;
    const u32 odd = 0u - (u32)((s >> 2) & 1);   // all ones: the row starts in the pair's upper dword
    u32 R[TBL_WORDS + 2];
#pragma unroll
    for (int k = 0; k < TBL_WORDS / 2 + 1; ++k) {
        const uint2 v = reinterpret_cast<const uint2*>(src.d)[a8 + k];
#if YSB_TBL_READ64 == 2
        asm volatile("" ::: "memory");   // keep ds_read_b64 (paired into ds_read2_b64: 8 cycles, banks mod 32)
#endif
        R[2 * k] = v.x;
        R[2 * k + 1] = v.y;
    }
#pragma unroll
    for (int k = 0; k <= TBL_WORDS; ++k) P[k] = (R[k] & ~odd) | (R[k + 1] & odd);   // v_bfi, not an indexed select
#else
    const int a = s >> 2;
#pragma unroll
    for (int k = 0; k <= TBL_WORDS; ++k) P[k] = src.d[a + k];
#endif
    u32 W[TBL_WORDS];
    u32 B[5] = {0u, 0u, 0u, 0u, 0u};   // bit i = line byte i may be '|'
#if YSB_TBL_ZCMP
    // bytes 0..95: the '|' flags of each word compared with the only pattern a generator
    // row has there -- '|' at 36 and 73 (word 9 byte 0, word 18 byte 1), no other byte
    // flagged (a false flag above a true '|' only rejects the line); no bitmap is packed
    u32 dz = 0;
#pragma unroll
    for (int j = 0; j < TBL_WORDS; ++j) {
        W[j] = __builtin_amdgcn_alignbyte(P[j + 1], P[j], sb);   // line bytes 4j..4j+3
        if (j < 24) {
            const u32 t = W[j] ^ 0x7C7C7C7Cu;
            const u32 z = ((t - 0x01010101u) & ~t) & 0x80808080u;
            dz |= j == 9 ? z ^ 0x80u : j == 18 ? z ^ 0x8000u : z;
        } else {
            B[j >> 3] |= bar_nib(W[j]) << (4 * (j & 7));
        }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) c.kw[k] = __builtin_amdgcn_alignbyte(W[19 + k], W[18 + k], 2u);   // bytes 74..109
    // the first three '|' exactly at 36, 73, 110 (each the lowest flag of its word: true)
    const bool fixed = dz == 0u && (B[3] & 0x7FFFu) == (1u << 14);
#else
#pragma unroll
    for (int j = 0; j < TBL_WORDS; ++j) {
        W[j] = __builtin_amdgcn_alignbyte(P[j + 1], P[j], sb);   // line bytes 4j..4j+3
        B[j >> 3] |= bar_nib(W[j]) << (4 * (j & 7));
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) c.kw[k] = __builtin_amdgcn_alignbyte(W[19 + k], W[18 + k], 2u);   // bytes 74..109
    // the first three '|' exactly at 36, 73, 110 (each the lowest flag of its word: true)
    const bool fixed = B[0] == 0u && B[1] == (1u << 4) && B[2] == (1u << 9) && (B[3] & 0x7FFFu) == (1u << 14);
#endif
    const u64 hi = ((u64)B[4] << 32) | (B[3] & ~0x7FFFu);   // bytes 96..159, above 110
    const int p3 = hi ? 96 + (int)__builtin_ctzll(hi) : (1 << 20);
    const u64 hi2 = hi & (hi - 1);
    const int p4 = hi2 ? 96 + (int)__builtin_ctzll(hi2) : (1 << 20);
    c.e3 = p3;
    c.e4 = p4;
    c.e5 = (int)B[3];
    c.e6 = (int)B[4];
    c.t0 = p4 + 1;
    return fixed && p4 + 2 <= L;
}

// Phase A of a .tbl tile: the 16 '|' flags of a 16-byte chunk (bit i = byte i may be '|',
// the SWAR flags of bar_nib: a flag above a true '|' in its dword may be false).
__device__ __forceinline__ u32 bar_chunk(const uint4& v) {
    return bar_nib(v.x) | (bar_nib(v.y) << 4) | (bar_nib(v.z) << 8) | (bar_nib(v.w) << 12);
}

// tbl_stage1 from the tile's '|' bitmap (Geom::BITMAP): the row's flags for bytes 0..159
// are 5 dwords of the bitmap shifted by the row's start (6 LDS reads instead of the row's
// 41), the ad_id's 36 bytes 10 more.  The flags are those of tile dwords, not row dwords,
// so a false flag may sit on any byte right above a true '|': the fixed-position checks
// only reject on an extra flag, and p3 / p4 are verified to be '|' in tbl_stage2, as there.
__device__ __forceinline__ bool tbl_stage1_bm(const LdsSrc& src, const u32* bm, int s, int e, CanonA& c) {
    const int L = e - s;
    if (L < TBL_MIN_LEN || L > TBL_MAX_LEN) return false;
    const int wb = s >> 5;
    const u32 sh = (u32)(s & 31);
    u32 M[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) M[k] = bm[wb + k];
    u32 B[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) B[k] = __builtin_amdgcn_alignbit(M[k + 1], M[k], sh);   // row bytes 32k..32k+31
    const int ka = (s + 74) >> 2;
    const u32 kb = (u32)((s + 74) & 3);
    u32 Q[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) Q[k] = src.d[ka + k];
#pragma unroll
    for (int k = 0; k < 9; ++k) c.kw[k] = __builtin_amdgcn_alignbyte(Q[k + 1], Q[k], kb);   // bytes 74..109
    // the first three '|' exactly at 36, 73, 110, nothing else flagged below 110
    const bool fixed = B[0] == 0u && B[1] == (1u << 4) && B[2] == (1u << 9) && (B[3] & 0x7FFFu) == (1u << 14);
    const u64 hi = ((u64)B[4] << 32) | (B[3] & ~0x7FFFu);   // bytes 96..159, above 110
    const int p3 = hi ? 96 + (int)__builtin_ctzll(hi) : (1 << 20);
    const u64 hi2 = hi & (hi - 1);
    const int p4 = hi2 ? 96 + (int)__builtin_ctzll(hi2) : (1 << 20);
    c.e3 = p3;
    c.e4 = p4;
    c.e5 = (int)B[3];
    c.e6 = (int)B[4];
    c.t0 = p4 + 1;
    return fixed && p4 + 2 <= L;
}

// Stage 2: the two '|' verified, the terminator stripped, no '|' after the fifth, the
// event_type and event_time fetched -- one batch of LDS reads.
__device__ __forceinline__ bool tbl_stage2(const LdsSrc& src, int s, int e, const CanonA& a, CanonB& c) {
    u32 t3[2], t4[1], tl[1];
    load_span(src, s + a.e3, t3);
    load_span(src, s + a.e4, t4);
    load_span(src, s + a.e4 + 1, c.td);
    load_span(src, e - 4, tl);                            // the line's last 4 bytes
    int end = e - s;                                      // readLine: "\n", then a '\r' before it
    const bool nl = (tl[0] >> 24) == '\n';
    end -= nl ? 1 : 0;
    end -= (((tl[0] >> (nl ? 16 : 24)) & 0xFFu) == '\r') ? 1 : 0;
    bool ok = (t3[0] & 0xFFu) == '|' && (t4[0] & 0xFFu) == '|' && end > a.e4 + 1;
    // no '|' in (p4, end): bits of the 64-bit bitmap of bytes 96..159
    const u64 bm = ((u64)(u32)a.e6 << 32) | (u32)a.e5;
    const int lo = a.e4 + 1 - 96, hi = end - 96;          // [lo, hi) must be clear
    const u64 m = (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull)) & ~((1ull << lo) - 1ull);
    ok &= (bm & m) == 0ull;
    c.view = a.e4 - a.e3 - 1 == 4 && __builtin_amdgcn_alignbyte(t3[1], t3[0], 1u) == VIEW_W;
    c.tlen = end - (a.e4 + 1);
    return ok;
}

// One line end to end: returns 0 not counted, 1 counted (campaign/bucket set).
// Per-thread tallies go to st[].
struct Tally { u32 ev, view, join, miss, perr, terr, oor, frn; };

// A view whose ad_id missed the table: dropped (RedisJoinBolt, :465-467) and counted as a
// join miss -- or, when this context holds one shard of the table (P.shard_n > 1) and the
// key belongs to another, as a foreign-shard view (mis-routed input).
__device__ __forceinline__ void count_miss(const ScanParams& P, const u32 (&kw)[KEY_WORDS], u32 klen, bool keyed,
                                           Tally& t) {
    if (keyed && P.shard_n > 1u && key_shard(key_hash_dev(kw, klen), P.shard_n) != P.shard_rank) t.frn++;
    else t.miss++;
}

// A parsed event's filter, join and bucket (the bolts after DeserializeBolt).
template <class S>
__device__ __forceinline__ bool finish_line(const S& src, const Span& ad, const Span& et, const Span& tm,
                                            const ScanParams& P, Tally& t, u32& campaign, i64& bucket) {
    if (!span_is_view(src, et)) return false;                // EventFilterBolt
    t.view++;
    u32 kw[KEY_WORDS];
    u32 klen = 0;
    int c = -1;
    const bool keyed = span_key(src, ad, kw, klen);
    if (keyed) c = probe(P.table, P.table_mask, kw, klen);   // RedisJoinBolt
    if (c < 0) { count_miss(P, kw, klen, keyed, t); return false; }
    t.join++;
    i64 tv;
    if (!span_long(src, tm, tv)) { t.terr++; return false; }   // CampaignProcessorCommon :58
    campaign = (u32)c;
    bucket = div_trunc(tv, P.div);
    return true;
}

// The general path (lines that are not in the generator's layout).
template <class S>
__device__ __forceinline__ bool process_line(const S& src, int s, int e, const ScanParams& P,
                                             Tally& t, u32& campaign, i64& bucket) {
    Span ad{0, 0, 0}, et{0, 0, 0}, tm{0, 0, 0};
    t.ev++;
    if (!parse_line(src, s, e, P.require_mask, ad, et, tm)) { t.perr++; return false; }
    return finish_line(src, ad, et, tm, P, t, campaign, bucket);
}

// ---- the general path's flat tier --------------------------------------------------------
#ifndef YSB_FLAT_LDS
#define YSB_FLAT_LDS 1   // round 4: flat_parse_lds for the flat-first / learned-order instantiations
#endif
#ifndef YSB_FLAT_VOCAB
#define YSB_FLAT_VOCAB 1   // round 4: flat_parse_lds names short values from the generator's vocabularies
#endif
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

#ifndef YSB_PLAIN_XAD
#define YSB_PLAIN_XAD 1   // round 4: plain36_bad's backslash test as an xor and an add per word (A/B +2 % flat tier)
#endif
// plain36's fast test as a u32 (0 = every byte of w[0..8] in [0x2D, 0x7F) and not a
// backslash); nonzero says only that the fast test failed (the exact flags decide).
// YSB_PLAIN_XAD: with every byte < 0x80 (the `hi` term), (w ^ 0x5C5C5C5C) + 0x7F7F7F7F sets
// bit 7 of a byte iff it is not '\\' and w + 0x53535353 iff it is >= 0x2D, with no carry
// between bytes -- two adds (one v_xad_u32) and two ands per word instead of a zero-byte test.
__device__ __forceinline__ u32 plain36_bad(const u32 (&w)[10]) {
#if YSB_PLAIN_XAD
    u32 acc = 0xFFFFFFFFu, hi = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        acc &= (w[j] + 0x53535353u) & ((w[j] ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu);
        hi |= w[j];
    }
    return ((acc & 0x80808080u) ^ 0x80808080u) | (hi & 0x80808080u);
#else
    u32 lo = 0xFFFFFFFFu, hi = 0, bs = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        lo &= w[j] + 0x53535353u;
        hi |= w[j];
        bs |= zero_bytes(w[j] ^ 0x5C5C5C5Cu);
    }
    return ((lo & 0x80808080u) ^ 0x80808080u) | (hi & 0x80808080u) | bs;
#endif
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
#if YSB_FLAT_VOCAB
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
#else
        if (id & (K_AD | K_USER | K_PAGE)) {
            u32 w[10];
            load_span(src, vq + 1, w);
            if (plain36(w) && vq + 37 < e && (w[9] & 0xFFu) == '"') {
                ve = vq + 37;
                y = w[9];
                if (id == K_AD) {
#pragma unroll
                    for (int j = 0; j < 9; ++j) adw[j] = w[j];
                }
            }
        }
#endif
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

#ifndef YSB_FLAT_BL
#define YSB_FLAT_BL 1   // round 4: flat_parse_bl2 before flat_parse_lds in the flat-first / learned-order tier
#endif
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
// key named (as in flat_parse_lds), `": "` / `":"`, the value -- an id as 36 plain bytes by
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
                                               Span& tm, u32 (&adw)[9]) {
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
        const u32 d7 = kw[1] ^ w4('_', 'i', 'd', '"');
        const u32 dEV = kw[0] ^ w4('e', 'v', 'e', 'n');
        const u32 k2 = kw[2] & 0xFFFFFFu;
        const u32 dAD = (kw[0] ^ w4('a', 'd', '_', 'i')) | ((kw[1] ^ w4('d', '"', 0, 0)) & 0xFFFFu);
        const u32 dUS = (kw[0] ^ w4('u', 's', 'e', 'r')) | d7;
        const u32 dPG = (kw[0] ^ w4('p', 'a', 'g', 'e')) | d7;
        const u32 dAT = (kw[0] ^ w4('a', 'd', '_', 't')) | (kw[1] ^ w4('y', 'p', 'e', '"'));
        const u32 dET = dEV | (kw[1] ^ w4('t', '_', 't', 'y')) | (k2 ^ (w4('p', 'e', '"', 0) & 0xFFFFFFu));
        const u32 dTM = dEV | (kw[1] ^ w4('t', '_', 't', 'i')) | (k2 ^ (w4('m', 'e', '"', 0) & 0xFFFFFFu));
        const u32 dIP = (kw[0] ^ w4('i', 'p', '_', 'a')) | (kw[1] ^ w4('d', 'd', 'r', 'e')) | (k2 ^ (w4('s', 's', '"', 0) & 0xFFFFFFu));
        const u32 id = dAD == 0u ? K_AD : dUS == 0u ? K_USER : dPG == 0u ? K_PAGE : dAT == 0u ? K_ADTYPE
                     : dET == 0u ? K_ETYPE : dTM == 0u ? K_ETIME : dIP == 0u ? K_IP : 0u;
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
__device__ __forceinline__ bool flat_tier(const S& src, int ls, int le, u32 require, CanonA& a, CanonB& b) {
    Span ad{0, 0, 0}, et{0, 0, 0}, tm{0, 0, 0};
    bool okp;
#if YSB_FLAT_LDS
    if constexpr (FAST && std::is_same<S, LdsSrc>::value) {
        u32 adw[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) adw[k] = 0u;
#if YSB_FLAT_BL
        okp = flat_parse_bl2(src, ls, le, require, ad, et, tm, adw);
        if (__builtin_expect(!okp, 0)) okp = flat_parse_lds(src, ls, le, require, ad, et, tm, adw);
#else
        okp = flat_parse_lds(src, ls, le, require, ad, et, tm, adw);
#endif
        if (!okp || ad.e - ad.s != 36) return false;
        const bool fast_ad = adw[0] | adw[1] | adw[8];   // the id fast path kept the ad_id's words
#pragma unroll
        for (int k = 0; k < 9; ++k) a.kw[k] = fast_ad ? adw[k] : src.load4(ad.s + 4 * k);
    } else
#endif
    {
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

#ifndef YSB_LEARN_VOCAB
#define YSB_LEARN_VOCAB 1   // round 4: learned-order short values named from the generator's vocabularies first
#endif

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

// the closing quote of the learned order's value at v named by vocab_len, or -1
template <int KI>
__device__ __forceinline__ int vocab_value_end(const LdsSrc& src, int v) {
    u32 A[5];
    load_span(src, v, A);
    const int la = vocab_len<KI>(A);
    return la ? v + la : -1;
}

// One pair of a learned order: the key literal at p, its value, the separator after it
// (", " + the next key's quote, or the closing quote + '}' when `last`).  p moves to the
// next key's text, or (last) to the '}'.  KI 0..2: 36-byte id values.
template <int KI, bool CP>
__device__ __forceinline__ bool learned_pair(const LdsSrc& src, int& p, int e, bool last, u32 (&kw)[9], int& vs,
                                             int& ve) {
    using K = KeyLit<KI, CP>;
    constexpr WordTpl<4> T = K::tpl();
    constexpr u32 SEP = CP ? w4('"', ',', '"', 0) : w4('"', ',', ' ', '"');
    constexpr u32 SEPM = CP ? 0x00FFFFFFu : 0xFFFFFFFFu;
    constexpr int SEPL = CP ? 3 : 4;
    u32 kwd[4];
    load_span(src, p, kwd);
    bool ok = words_diff(kwd, T) == 0u;
    const int v = p + K::LEN;
    vs = v;
    if constexpr (KI <= 2) {
        u32 w[10];
        load_span(src, v, w);
        ok &= plain36(w);
        ok &= last ? (w[9] & 0xFFFFu) == w4('"', '}', 0, 0) : (w[9] & SEPM) == SEP;
        ve = v + 36;
        if constexpr (KI == 2) {
#pragma unroll
            for (int k = 0; k < 9; ++k) kw[k] = w[k];
        }
    } else {
#if YSB_LEARN_VOCAB
        ve = vocab_value_end<KI>(src, v);         // round 4: the value named, not scanned
        if (__builtin_expect(ve < 0, 0)) ve = ft_string_end(src, v, e);
#else
        ve = ft_string_end(src, v, e);
#endif
        ok &= ve >= v;
        const u32 x = src.load4(ok ? ve : v);
        ok &= last ? (x & 0xFFFFu) == w4('"', '}', 0, 0) : (x & SEPM) == SEP;
    }
    p = last ? ve + 1 : ve + SEPL;
    return ok;
}

#ifndef YSB_LEARN_U32
#define YSB_LEARN_U32 1   // round 4: learned_pair's checks as one u32 (no scalar lane-mask logic, see flat_parse_bl2)
#endif
// learned_pair with its checks ORed into a u32 (0 = the pair is in the learned form).
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
#if YSB_LEARN_U32
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
#else
    bool ok = (src.load4(s) & 0xFFFFu) == w4('{', '"', 0, 0);
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
        bool pk;
        switch ((P.learn_code >> (3 * k)) & 7u) {   // uniform: a scalar branch
        case 0: pk = learned_pair<0, CP>(src, p, e, last, kw, vs, ve); break;
        case 1: pk = learned_pair<1, CP>(src, p, e, last, kw, vs, ve); break;
        case 2: pk = learned_pair<2, CP>(src, p, e, last, kw, vs, ve); break;
        case 3: pk = learned_pair<3, CP>(src, p, e, last, kw, vs, ve); break;
        case 4: pk = learned_pair<4, CP>(src, p, e, last, kw, vs, ve); ets = vs; ete = ve; break;
        case 5: pk = learned_pair<5, CP>(src, p, e, last, kw, vs, ve); tms = vs; tme = ve; break;
        default: pk = learned_pair<6, CP>(src, p, e, last, kw, vs, ve); break;
        }
        ok &= pk;
        if (!ok) p = s + 2;   // a failed lane keeps reading inside its line (result ignored)
    }
    ok &= p < e;              // the '}' (every compared byte lies before it)
#pragma unroll
    for (int k = 0; k < 9; ++k) a.kw[k] = kw[k];
    a.t0 = tms - s;
    b.tlen = tme - tms;
    load_span(src, tms, b.td);
    b.view = ete - ets == 4 && src.load4(ets) == VIEW_W;
    return ok;
#endif
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

// ---------------------------------------------------------------------------
// LDS layout (dynamic, 16-byte aligned carve, no static __shared__)
// ---------------------------------------------------------------------------
constexpr int LDS_BYTES = Geom<false>::LDS;   // the JSON geometry (Geom<true> for .tbl rows)

struct TileInfo {
    u64 first;
    u32 count;
    u32 s0;        // byte offset of the tile's first line
    u32 delta;     // s0 - 16-byte aligned base
    u32 len;       // bytes in LDS (from the aligned base)
    u32 e;         // end offset of the tile's last line
    bool oversize; // does not fit TILE_CAP (or offsets are not monotone)
};

// Tile bounds come from the LDS copy tb[] (loaded once per workgroup), so no HBM
// round trip sits between two tiles.
#ifndef YSB_TILE_TRUNCATE
#define YSB_TILE_TRUNCATE 1
#endif
template <int CAP>
__device__ __forceinline__ TileInfo tile_info(const ScanParams& P, u64 t, u64 t_begin, const u32* tb) {
    TileInfo ti;
    ti.first = t * TILE_LINES;
    const u64 rem = P.n - ti.first;
    ti.count = rem < (u64)TILE_LINES ? (u32)rem : (u32)TILE_LINES;
    // wave-uniform by construction; readfirstlane lets the compiler keep them (and the
    // buffer descriptors built from them) in SGPRs (no waterfall loops)
    // (readfirstlane returns int: keep it unsigned before widening, offsets reach 4 GiB)
    const u32 s0 = (u32)__builtin_amdgcn_readfirstlane(tb[t - t_begin]);
    const u64 e = (u32)__builtin_amdgcn_readfirstlane(tb[t - t_begin + 1]);
    ti.s0 = s0;
    ti.e = (u32)e;
    ti.delta = s0 & 15u;   // P.bytes is 16-byte aligned
    const bool sane = (u64)s0 <= e && e <= P.nbytes;
    const u64 len = sane ? e - s0 + ti.delta : ~0ULL;
#if YSB_TILE_TRUNCATE
    // a tile of long lines is staged up to its capacity: the lines that end inside it are
    // parsed, the rest deferred (the whole tile before)
    ti.oversize = !sane;
    if (sane && len > (u64)CAP) ti.e = s0 - ti.delta + (u32)CAP;
    ti.len = ti.oversize ? 0u : (u32)(len < (u64)CAP ? len : (u64)CAP);
#else
    ti.oversize = !sane || len > (u64)CAP;
    ti.len = ti.oversize ? 0u : (u32)len;
#endif
    return ti;
}

// Cache policy of the once-read batch stream: nontemporal (aux 2), so it does not
// displace the join table from L2 (MI355X_MICROARCH.md, row nt-weights).
#ifndef YSB_AUX_NT
#define YSB_AUX_NT 2
#endif
constexpr int AUX_NT = YSB_AUX_NT;

#ifndef YSB_SETPRIO
#define YSB_SETPRIO 1
#endif

// The campaign of key k in a 128-B bucket (EMPTY_SLOT: not there); full = all three
// entries taken (only then may the key sit in its second bucket)
__device__ __forceinline__ u32 bucket_find(const uint4 (&q)[CB_Q], const u32* k, bool& full) {
    u32 w[CB_WORDS];
#pragma unroll
    for (int j = 0; j < (int)CB_Q; ++j) {
        w[4 * j] = q[j].x;
        w[4 * j + 1] = q[j].y;
        w[4 * j + 2] = q[j].z;
        w[4 * j + 3] = q[j].w;
    }
    u32 found = EMPTY_SLOT;
    full = true;
#pragma unroll
    for (int e = 0; e < (int)CB_ENTRIES; ++e) {
        u32 d = 0;
#pragma unroll
        for (int j = 0; j < (int)CKEY_WORDS; ++j) d |= w[e * CB_STRIDE + j] ^ k[j];
        const u32 c = w[e * CB_STRIDE + CKEY_WORDS];
        if (c == EMPTY_SLOT) full = false;
        else if (d == 0u) found = c;
    }
    return found;
}
#ifndef YSB_PREFETCH_DEPTH
#define YSB_PREFETCH_DEPTH 1
#endif
#ifndef YSB_LINE_INTERLEAVE
#define YSB_LINE_INTERLEAVE 1
#endif
// The tile line a lane parses.  Interleaved: lanes 0..31 take the even lines, 32..63 the
// odd ones, so the start banks of the lines a 32-lane half reads (dword mod 32, lines
// ~63.5 dwords apart) step by one bank instead of crowding into half of them.
__device__ __forceinline__ u32 lane_line(int tid) {
#if YSB_LINE_INTERLEAVE
    return ((u32)(tid & 31) << 1) | ((u32)tid >> 5);
#else
    return (u32)tid;
#endif
}

// The next tile's bytes and line offsets, HBM -> registers.  Bounds-checked buffer
// loads through per-tile descriptors (base = the tile, num_records = its length, so
// chunks past the tile read zeros and never fault); per-lane offsets are
// loop-invariant, so issuing costs no VALU.  Always the same number of loads per lane,
// so later waits can count them (vmcnt) instead of draining everything.
template <int CPT>
__device__ __forceinline__ void issue_tile_loads(const ScanParams& P, const TileInfo& ti, uint4 (&pre)[CPT],
                                                 u32& my_off, u32& my_end) {
    const int tid = threadIdx.x;
    const u8* tbase = P.bytes + (ti.s0 - ti.delta);
    // A 16-byte access that straddles num_records reads as all zeros, so the range is the
    // tile rounded up to 16 bytes: with a 16-byte aligned base, a chunk holding any batch
    // byte never leaves the batch's last page.
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(tbase), 0, (int)((ti.len + 15u) & ~15u), 0x00020000);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * (j * SCAN_TPB + tid), 0, AUX_NT);
        pre[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    const u64 left = P.n - min(ti.first, P.n);
    const u32 nrec = (u32)min<u64>((u64)ti.count + 1u, left) * 4u;   // my_end of the tile's last line included
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u32*>(P.off + min(ti.first, P.n)), 0, (int)nrec, 0x00020000);
    const u32 li = lane_line(tid);
    my_off = __builtin_amdgcn_raw_buffer_load_b32(ro, 4 * li, 0, 0);
    my_end = __builtin_amdgcn_raw_buffer_load_b32(ro, 4 * li + 4, 0, 0);   // 0 past the batch end
}

__device__ __forceinline__ u32 wave_sum(u32 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void flush_tally(const ScanParams& P, const Tally& tl, int lane) {
    const u32 sums[8] = {wave_sum(tl.ev), wave_sum(tl.view), wave_sum(tl.join), wave_sum(tl.miss),
                         wave_sum(tl.perr), wave_sum(tl.terr), wave_sum(tl.oor), wave_sum(tl.frn)};
    if (lane == 0) {
        const u32 slots[8] = {ST_EVENTS, ST_VIEWS, ST_JOINED, ST_MISSES, ST_PARSE_ERR, ST_TIME_ERR, ST_OUT_OF_RING,
                              ST_FOREIGN};
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (sums[k]) atomicAdd(&P.stats[slots[k]], (unsigned long long)sums[k]);
    }
}

// Appends the flagged lines of the wave to the deferred list (one atomic per wave).
__device__ __forceinline__ void defer_append(const ScanParams& P, bool dfr, u64 line, int lane) {
    const unsigned long long m = __ballot(dfr);
    if (!m) return;
    u32 base = 0;
    if (lane == 0) {
        base = atomicAdd(P.defer_count, (u32)__popcll(m));
        atomicAdd(&P.stats[ST_DEFERRED], (unsigned long long)__popcll(m));
    }
    base = __shfl(base, 0, 64);
    if (dfr) {
        const u32 r = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
        if (base + r < P.defer_cap) P.defer[base + r] = (u32)line;
    }
}

// LDS window counters: flush every non-zero cell of the window at lbase to the ring.
__device__ __forceinline__ void flush_window(const ScanParams& P, u32* lcnt, u32 ncells, u32 WL, i64 lbase,
                                             i64 ring_lo, bool ring_set, Tally& tl) {
    for (u32 i = threadIdx.x; i < ncells; i += SCAN_TPB) {
        const u32 v = lcnt[i];
        if (v) {
            lcnt[i] = 0;
#ifndef YSB_DIAG_NO_FLUSH
            global_add(P, ring_lo, ring_set, i >> P.lds_wl_log2, lbase + (i64)(i & (WL - 1)), v, tl);
#endif
        }
    }
}

#ifdef YSB_STAMPS
// Diagnostic build only: wave-level s_memtime phase accounting (cdna_hip_programming.md
// section 7, "In-kernel stamps").  The values go to P.dbg, never into results.
#define STAMP_DECL unsigned long long st_acc[N_STAMPS] = {0}, st_last = stamp_now();
#define STAMP(i) do { const unsigned long long n_ = stamp_now(); st_acc[i] += n_ - st_last; st_last = n_; } while (0)
__device__ __forceinline__ unsigned long long stamp_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
#define STAMP_DECL
#define STAMP(i) do { } while (0)
#endif

// Record mode: ring cell index -> (campaign, bucket) for the atomic fallback (a record the
// workgroup's full HBM sub-buffer cannot take).
__device__ __forceinline__ void rec_fallback(const ScanParams& P, u32 cell, i64 ring_lo, bool ring_set, Tally& tl) {
    const u32 wl2 = 31u - (u32)__builtin_clz(P.ring_w);
    const u32 c = cell >> wl2;
    const i64 slot = (i64)(cell & (P.ring_w - 1));
    const i64 b = ring_lo + ((slot - ring_lo) & (i64)(P.ring_w - 1));
    global_add(P, ring_lo, ring_set, c, b, 1u, tl);
    *P.pend_dirty = 1u;   // the u64 ring holds pending counts now (the exchange reads it)
}

// Record mode: writes n (<= 32) staged records of bin b, ring positions [fl, fl + n), to
// the workgroup's HBM sub-buffer of the bin -- one store by lanes 0..n-1, a whole 128-B
// line when n = 32 -- or, once that sub-buffer is full, to the ring atomics (slower,
// exact).  Lane b of gcur = records in bin b's sub-buffer; one wave.
__device__ __forceinline__ void rec_write(const ScanParams& P, const u32* ring, u32 b, u32 fl, u32 n, u32& gcur,
                                          int lane, i64 ring_lo, bool ring_set, Tally& tl) {
    const u32 g = (u32)__builtin_amdgcn_readlane((int)gcur, (int)b);
    const bool fits = g + n <= P.rec_cap;
    if ((u32)lane < n) {
        const u32 v = ring[b * REC_RING + ((fl + (u32)lane) & (REC_RING - 1))];
        if (fits) P.rec[((u64)blockIdx.x * P.rec_bins + b) * P.rec_cap + g + (u32)lane] = v;
        else rec_fallback(P, v, ring_lo, ring_set, tl);
    }
    if (fits && lane == (int)b) gcur = g + n;
}

// SERIAL: HBM-resident cuckoo table, second slot probed only after a first-slot miss (a
// separate instantiation so the cache-resident configuration's code is untouched).
// TBL: the fork's .tbl rows (tbl_stage1/2) instead of JSON lines (vocab_stage1/2).
// REC: record mode (ysb_count.hip): in-ring joined views become ring-cell records.
// LAY: the JSON layout tried first (the same grammar and counts; only the order of the
// tiers differs).  0: the generator's (the default); 1, compact JSON first
// (YSB_F_COMPACT_FIRST): the compact layout's vocabulary path is the first stage and the
// generator layout a later tier; 2, any key order (YSB_F_FLAT_FIRST): the flat tier is the
// only stage (every line a canonical tier takes, it takes too), with its FAST steps.
template <bool SERIAL, bool TBL, bool REC, int LAY = 0>
__global__ __launch_bounds__(SCAN_TPB) __attribute__((amdgpu_waves_per_eu((Geom<TBL>::WG_PER_CU * SCAN_TPB + 255) / 256))) void scan_kernel(const ScanParams P0) {
    using G = Geom<TBL, REC>;
    constexpr int CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) u8 smem[];
    u32* tile32 = reinterpret_cast<u32*>(smem + G::OFF_TILE);
    u32* lcnt = reinterpret_cast<u32*>(smem + G::OFF_LCNT);
    i64* misc64 = reinterpret_cast<i64*>(smem + G::OFF_MISC);   // [0] lbase, [1] lset, [2..5] scratch
    u32* tb = reinterpret_cast<u32*>(smem + G::OFF_TB);
    u32* bm32w = reinterpret_cast<u32*>(smem + G::OFF_BM);   // .tbl '|' bitmap (G::BITMAP)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
#ifdef YSB_WGTIME
    const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    // P: the launch parameters with the batch fields (bytes, off, n, nbytes, line_base)
    // of the segment being scanned
    ScanParams P = P0;

    const i64 ring_lo = P.ring[0];
    const bool ring_set = P.ring[1] != 0;
    const u32 WL = P.lds_wl;
    const u32 ncells = WL ? P.n_campaigns * WL : 0u;
    for (u32 i = tid; i < ncells; i += SCAN_TPB) lcnt[i] = 0;
    // record mode (no LDS window counters): the counter area holds a 64-record staging ring
    // per level-1 bin (lcnt), the misc area the rings' cursors rcur[b] = records staged;
    // lane b of gcur = records of bin b in this workgroup's HBM sub-buffer
    u32* rcur = reinterpret_cast<u32*>(misc64);
    u32 gcur = 0;
    if (REC && tid < REC_BINS_MAX) rcur[tid] = 0;
    // rebase requests of the LDS window (double-buffered by tile parity): the largest
    // bucket that fell ahead of the window, INT64_MIN = none
    if (!REC && tid < 2) misc64[tid] = INT64_MIN;

    Tally tl{0, 0, 0, 0, 0, 0, 0, 0};
    // Prefetch depth: tile t + PF_DEPTH is issued once tile t sits in LDS.  Depth 2 keeps
    // two tiles in flight per wave (two register buffers, the loop unrolled by two).
    constexpr int PF_DEPTH = YSB_PREFETCH_DEPTH;
    // Depth 2 (two register buffers) measured -2 % on v11 and spills to scratch inside the
    // per-segment run loop: only depth 1 is built.
    static_assert(PF_DEPTH == 1, "YSB_PREFETCH_DEPTH must be 1");
    // this workgroup's run of tiles [t_begin, t_end) in the current segment
    u64 t_begin = 0, t_end = 0, n_run = 0;
    TileInfo none{0, 0u, 0u, 0u, 0u, 0u, true};
    uint4 preA[CPT];
    u32 offA = 0, endA = 0;
    TileInfo infA = none;
    u32 tseq = 0;   // tiles stepped so far (window-request parity across segments)
    // The LDS window's base, identical in every thread (each applies the same requests).
    i64 lbase = 0;
    bool lset = false;

    const LdsSrc lsrc{tile32};
    const uint4* ct4 = reinterpret_cast<const uint4*>(P.ctable);
#if YSB_SETPRIO
    // static priority for every other workgroup: the two waves of a SIMD stop trading
    // VALU issue by age (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);
#endif
    STAMP_DECL
    // One tile: its bytes arrive in pre (issued PF_DEPTH tiles ago), the tile PF_DEPTH
    // ahead is issued into the same registers once they are in LDS.
    auto tile_step = [&](u64 t, TileInfo& inf, uint4 (&pre)[CPT], u32& pre_off, u32& pre_end) {
        const TileInfo cur = inf;
        const u32 my_off = pre_off;
        const u32 li = lane_line(tid);
        const u32 my_end = (cur.first + li + 1 < P.n) ? pre_end : (u32)P.nbytes;
#ifdef YSB_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // diagnostic: separate the prefetch wait
        STAMP(6);
#endif
        // ---- Phase A: registers -> LDS -----------------------------------------------
        // Chunks past the tile hold zeros (bounds-checked loads), so they are written
        // unconditionally; only the last round is cut at TILE_CHUNKS (a whole wave).
        if (!cur.oversize) {
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
                const u32 k = (u32)(j * SCAN_TPB + tid);
                if (j * SCAN_TPB + SCAN_TPB <= G::CHUNKS || k < (u32)G::CHUNKS) {
                    reinterpret_cast<uint4*>(tile32)[k] = pre[j];
                }
                if constexpr (G::BITMAP && YSB_TBL_BITMAP != 3) {
                    // chunk k's 16 flags -> bitmap halfword k: the odd lane's flags join the
                    // even lane's (DPP swap within pairs), one dword store per pair
                    const u32 f = bar_chunk(pre[j]);
                    const u32 fo = (u32)__builtin_amdgcn_mov_dpp((int)f, 0xB1, 0xF, 0xF, false);   // quad_perm(1,0,3,2)
                    if (!(tid & 1) && (j * SCAN_TPB + SCAN_TPB <= G::CHUNKS || k < (u32)G::CHUNKS))
                        bm32w[k >> 1] = f | (fo << 16);
                }
            }
        }
        // The previous tile asked to move the LDS window: flush it (its counts are all
        // in, the end barrier saw to that) and re-centre, before this tile counts.
        const int par = (int)(tseq++ & 1);
        if (WL) {
            const i64 req = misc64[par ^ 1];
            if (req != INT64_MIN) {
                if (lset) flush_window(P, lcnt, ncells, WL, lbase, ring_lo, ring_set, tl);
                lbase = req - (i64)(WL / 2) + 1;
                lset = true;
            }
        }
        STAMP(0);
        __syncthreads();
        if (!REC && tid == 0) misc64[par ^ 1] = INT64_MIN;   // every thread has read it (REC: the ring cursors live there)
        STAMP(1);
#ifdef YSB_DIAG_A_ONLY
        inf = t + PF_DEPTH < t_end ? tile_info<G::CAP>(P, t + PF_DEPTH, t_begin, tb) : none;
        issue_tile_loads(P, inf, pre, pre_off, pre_end);
        __syncthreads();
        return;
#endif
        // ---- Phase B1: canonical parse from LDS; any other line is deferred -------
        bool ok1 = false, elig = false;
        int ls = 0, le = 0;
        CanonA ca;
#pragma unroll
        for (int k = 0; k < 9; ++k) ca.kw[k] = 0u;
        ca.t0 = 0;
        CanonB cb;
        cb.view = false;
        if (li < cur.count && !cur.oversize && my_off >= cur.s0 && my_end >= my_off && my_end <= cur.e) {
            elig = true;
            ls = (int)(my_off - cur.s0 + cur.delta);
            le = (int)(my_end - cur.s0 + cur.delta);
            if constexpr (G::BITMAP && YSB_TBL_BITMAP == 1) ok1 = tbl_stage1_bm(lsrc, bm32w, ls, le, ca);
            else if constexpr (TBL) ok1 = tbl_stage1(lsrc, ls, le, ca);
            else if constexpr (LAY == 2) ok1 = flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, ca, cb);
            else if constexpr (LAY == 3) {
                ok1 = P.learn_cp ? learned_parse<true>(lsrc, ls, le, P, ca, cb) : learned_parse<false>(lsrc, ls, le, P, ca, cb);
                // a line off the learned order: the flat tier (any order or spacing)
                if (__builtin_expect(!ok1, 0)) ok1 = flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, ca, cb);
            }
            else if constexpr (LAY == 4) {}   // below, once the wave's mode is known
            else if constexpr (YSB_VOCAB != 0) ok1 = vocab_stage1<LAY == 1>(lsrc, ls, le, ca);
            else ok1 = canon_stage1<false>(lsrc, ls, le, ca);
        }
        // LAY 4 (round 4, several producers in one batch): per-tile dispatch.  Each lane names
        // its line's class from its first 12 bytes (the generator's `{"user_id": ` / compact
        // `{"user_id":"` / anything else); one ballot per class makes the tile's mode, uniform
        // in the wave: all one canonical class -> that vocabulary path, all "else" with a
        // sampled learned order -> the learned-order parse, a tile of mixed classes -> the
        // flat tier.  Lanes a producer's path rejects take the flat tier after it (`fl`).
        // Tiles of one producer (producers writing in runs of lines) run at its speed.
        int mode = 0;
        bool fl = false;
        if constexpr (LAY == 4) {
            u32 cls = 0;
            if (elig) {
                const u32 h2 = lsrc.load4(ls + 8);
                const bool up = lsrc.load4(ls) == w4('{', '"', 'u', 's') && lsrc.load4(ls + 4) == w4('e', 'r', '_', 'i') &&
                                (h2 & 0xFFFFFFu) == (w4('d', '"', ':', 0) & 0xFFFFFFu);
                cls = up && (h2 >> 24) == ' ' ? 1u : up && (h2 >> 24) == '"' ? 2u : 3u;
            }
            const u64 b1 = __ballot(cls == 1u), b2 = __ballot(cls == 2u), b3 = __ballot(cls == 3u);
            mode = (b2 | b3) == 0ull ? 1 : (b1 | b3) == 0ull ? 2 : ((b1 | b2) == 0ull && P.learn_n) ? 3 : 4;
            if (elig) {
                if (mode == 1) ok1 = vocab_stage1<false>(lsrc, ls, le, ca);
                else if (mode == 2) ok1 = vocab_stage1<true>(lsrc, ls, le, ca);
                else if (mode == 3) {
                    ok1 = P.learn_cp ? learned_parse<true>(lsrc, ls, le, P, ca, cb) : learned_parse<false>(lsrc, ls, le, P, ca, cb);
                    fl = !ok1;
                } else {
                    fl = true;
                }
            }
        }
        bool pend = false, dfr = false, tok = false;
        i64 bucket = 0;
        bool ok2 = false;
        if (li < cur.count) {
            if constexpr (TBL) ok2 = ok1 && tbl_stage2(lsrc, ls, le, ca, cb);
            else if constexpr (LAY == 2 || LAY == 3) ok2 = ok1;
            else if constexpr (LAY == 4) {
                if (mode == 1) ok2 = ok1 && vocab_stage2<false>(lsrc, ls, le, ca, cb);
                else if (mode == 2) ok2 = ok1 && vocab_stage2<true>(lsrc, ls, le, ca, cb);
                else ok2 = ok1;
                if (mode <= 2) fl = elig && !ok2;
            }
            else if constexpr (YSB_VOCAB != 0) ok2 = ok1 && vocab_stage2<LAY == 1>(lsrc, ls, le, ca, cb);
            else ok2 = ok1 && canon_stage2<false>(lsrc, ls, le, ca, cb);
        }
#if YSB_CANON_TIERS
        if constexpr (!TBL && YSB_VOCAB != 0 && LAY < 2) {
            // second and third tiers for the lanes the vocabulary path rejected (a branch
            // no lane takes on the generator's own lines): any values in the generator's
            // layout, then the same keys as compact JSON
            if (__builtin_expect(elig && !ok2, 0)) {
                CanonA c2;
                CanonB b2;
                b2.view = false;
                // both canonical layouts open with {"user_id": then ' ' or '"' (byte 11)
                const u32 h2 = lsrc.load4(ls + 8);
                const bool up = lsrc.load4(ls) == w4('{', '"', 'u', 's') && lsrc.load4(ls + 4) == w4('e', 'r', '_', 'i') &&
                                (h2 & 0xFFFFFFu) == (w4('d', '"', ':', 0) & 0xFFFFFFu);
                bool t = false;
                if constexpr (LAY == 1) {   // the generator layout: its vocabulary path, then its canonical tier
                    if (up && (h2 >> 24) == ' ') {
                        t = vocab_stage1<false>(lsrc, ls, le, c2) && vocab_stage2<false>(lsrc, ls, le, c2, b2);
                        if (!t) t = canon_stage1<false>(lsrc, ls, le, c2) && canon_stage2<false>(lsrc, ls, le, c2, b2);
                    } else if (up && (h2 >> 24) == '"') {
                        t = canon_stage1<true>(lsrc, ls, le, c2) && canon_stage2<true>(lsrc, ls, le, c2, b2);
                    }
                } else {
                if (up && (h2 >> 24) == ' ')
                    t = canon_stage1<false>(lsrc, ls, le, c2) && canon_stage2<false>(lsrc, ls, le, c2, b2);
                else if (up && (h2 >> 24) == '"') {   // compact JSON: its vocabulary path, then its canonical tier
                    t = vocab_stage1<true>(lsrc, ls, le, c2) && vocab_stage2<true>(lsrc, ls, le, c2, b2);
                    if (!t) t = canon_stage1<true>(lsrc, ls, le, c2) && canon_stage2<true>(lsrc, ls, le, c2, b2);
                }
                }
#if YSB_FLAT_TIER
                if (!t) t = flat_tier<LdsSrc, YSB_FLAT_FAST_TIER4 != 0>(lsrc, ls, le, P.require_mask, c2, b2);   // any key order / spacing
#endif
                if (t) {
                    ca = c2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
#else
        (void)elig;
#endif
        if constexpr (LAY == 4) {
            if (elig && fl) {   // the flat tier: a mixed tile's lines, and the lanes its path rejected
                CanonA c2;
                CanonB b2;
                b2.view = false;
                if (flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, c2, b2)) {
                    ca = c2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        dfr = li < cur.count && !ok2;   // bad offsets, other layouts, escapes, over-size tiles
        pend = ok2 && cb.view;                                             // EventFilterBolt
        // RedisJoinBolt's lookup (36-byte keys), views only (a third of the lanes:
        // scattered loads cost address-unit time per lane), issued before the time parse
        // and the next tile's prefetch so their latency hides under both and waiting for
        // them never waits for the prefetch.
        // Cache-resident table (config 2): both cuckoo slots at once.  HBM-resident table
        // (config 3, SERIAL): the key's first 128-B bucket; the second only when the key
        // is not in a full first bucket (ysb_common.h CB_*), ~0.1 % of the keys.
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0, a2 = a0, b0 = a0, b1 = a0, b2 = a0;
        uint4 q[CB_Q];
#pragma unroll
        for (int j = 0; j < (int)CB_Q; ++j) q[j] = a0;
        u32 ib_s = 0;
#ifdef YSB_DIAG_NO_PROBE
        if (pend) {   // diagnostic build: the first slot / entry "holds" the key, campaign from its bytes
            a0 = make_uint4(ca.kw[0], ca.kw[1], ca.kw[2], ca.kw[3]);
            a1 = make_uint4(ca.kw[4], ca.kw[5], ca.kw[6], ca.kw[7]);
            a2 = make_uint4(ca.kw[8], ca.kw[0] % P.n_campaigns, 0, 0);
            q[0] = a0;
            q[1] = a1;
            q[2] = a2;
        }
        if (false) {
#else
        if (pend) {
#endif
            u32 ia, ib;
            cuckoo_slots36(ca.kw, P.cseed, P.ctable_mask, &ia, &ib);
            if constexpr (SERIAL) {
#pragma unroll
                for (int j = 0; j < (int)CB_Q; ++j) q[j] = ct4[CB_Q * (u64)ia + j];
                ib_s = ib;
            } else {
                a0 = ct4[CSLOT_Q * (u64)ia]; a1 = ct4[CSLOT_Q * (u64)ia + 1]; a2 = ct4[CSLOT_Q * (u64)ia + 2];
                b0 = ct4[CSLOT_Q * (u64)ib]; b1 = ct4[CSLOT_Q * (u64)ib + 1]; b2 = ct4[CSLOT_Q * (u64)ib + 2];
            }
        }
        if (ok2) {
            tl.ev++;
            if (pend) {
                tl.view++;
                tok = canonical_bucket<TBL>(lsrc, cb, ls + ca.t0, P, bucket);   // Long.parseLong
            }
        }
        defer_append(P, dfr, P.line_base + cur.first + li, lane);
        STAMP(2);
        // ---- prefetch the next tile (lands while this one is parsed) -----------
        // Issued on every iteration (the last one loads nothing: out-of-range buffer
        // loads return zeros) so every path has the same count of loads in flight and
        // the waits below stay counted.
        inf = t + PF_DEPTH < t_end ? tile_info<G::CAP>(P, t + PF_DEPTH, t_begin, tb) : none;
        issue_tile_loads(P, inf, pre, pre_off, pre_end);
        // ---- Phase B2: join result ------------------------------------------------
        bool valid = false, dfr2 = false;
        u32 campaign = 0;
        if (pend) {
            const u32* k = ca.kw;
            u32 ci;
            if constexpr (SERIAL) {
                bool full;
                ci = bucket_find(q, k, full);
#ifndef YSB_DIAG_NO_PROBE2
                if (ci == EMPTY_SLOT && full) {   // the second bucket
#pragma unroll
                    for (int j = 0; j < (int)CB_Q; ++j) q[j] = ct4[CB_Q * (u64)ib_s + j];
                    ci = bucket_find(q, k, full);
                }
#endif
            } else {
                const u32 da = (a0.x ^ k[0]) | (a0.y ^ k[1]) | (a0.z ^ k[2]) | (a0.w ^ k[3]) | (a1.x ^ k[4]) |
                               (a1.y ^ k[5]) | (a1.z ^ k[6]) | (a1.w ^ k[7]) | (a2.x ^ k[8]);
                const u32 db = (b0.x ^ k[0]) | (b0.y ^ k[1]) | (b0.z ^ k[2]) | (b0.w ^ k[3]) | (b1.x ^ k[4]) |
                               (b1.y ^ k[5]) | (b1.z ^ k[6]) | (b1.w ^ k[7]) | (b2.x ^ k[8]);
                ci = (da == 0u && a2.y != EMPTY_SLOT) ? a2.y : (db == 0u ? b2.y : EMPTY_SLOT);
            }
            if (ci == EMPTY_SLOT) {
                if (P.ctable_partial) {   // the key may be one the cuckoo build left out
                    dfr2 = true;
                    tl.ev--;
                    tl.view--;
                } else {
                    tl.miss++;                                              // drop (:465-467)
                }
            } else {
                tl.join++;
                campaign = ci;
                valid = tok;
                if (!tok) tl.terr++;
            }
        }
        if (P.ctable_partial) defer_append(P, dfr2, P.line_base + cur.first + li, lane);
        STAMP(3);
        // ---- count: LDS window counters; events outside go straight to the ring -----
        bool rec_has = false;
        u32 rec_bin = 0, rec_val = 0;
        if (WL) {
            if (valid) {
                const i64 rel = bucket - lbase;
                if (lset && rel >= 0 && rel < (i64)WL) {
                    atomicAdd(&lcnt[(campaign << P.lds_wl_log2) + (u32)rel], 1u);
                } else {
                    global_add(P, ring_lo, ring_set, campaign, bucket, 1u, tl);
                    if (!lset || rel >= (i64)WL) atomicMax(reinterpret_cast<long long*>(&misc64[par]), (long long)bucket);
                }
            }
        } else if (valid) {
#ifndef YSB_DIAG_NO_COUNT
            if constexpr (REC) {
                const i64 rel = bucket - ring_lo;
                if (ring_set && rel >= 0 && rel < (i64)P.ring_w) {   // in the ring: a record
                    rec_has = true;
                    rec_bin = campaign >> P.rec_shift;
                    rec_val = campaign * P.ring_w + (u32)(bucket & (i64)(P.ring_w - 1));
                } else {
                    global_add(P, ring_lo, ring_set, campaign, bucket, 1u, tl);
                }
            } else {
                global_add(P, ring_lo, ring_set, campaign, bucket, 1u, tl);
            }
#endif
        }
#ifdef YSB_DIAG_NO_REC
        rec_has = false;   // diagnostic build: views found and parsed, never counted
#endif
        if constexpr (REC) {
            // stage this tile's records, a 32-lane half at a time (a half adds <= 32 to a
            // bin whose ring holds < 32 unwritten ones: the 64-record ring never overflows);
            // the lane whose record takes position 32k + 31 completed line k of its bin
            // and has it written out (no cursor reads: one LDS round trip per half)
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const bool mine = rec_has && (tid >> 5) == half;
                u32 pos = 0;
                if (mine) {
                    pos = atomicAdd(&rcur[rec_bin], 1u);
                    lcnt[rec_bin * REC_RING + (pos & (REC_RING - 1))] = rec_val;
                }
                unsigned long long done = __ballot(mine && (pos & 31u) == 31u);
                while (done) {
                    const int src = (int)__builtin_ctzll(done);
                    done &= done - 1;
                    const u32 b = (u32)__builtin_amdgcn_readlane((int)rec_bin, src);
                    const u32 p = (u32)__builtin_amdgcn_readlane((int)pos, src);
                    rec_write(P, lcnt, b, p - 31u, 32u, gcur, lane, ring_lo, ring_set, tl);
                }
            }
        }
        STAMP(4);
        __syncthreads();
        STAMP(5);
    };
    // One run of tiles [t_begin, t_end) of the current segment (P's batch fields).
    auto run_tiles = [&]() {
        n_run += t_end - t_begin;
        // tile bounds of this run: off[t * TILE_LINES] for t in [t_begin, t_end], nbytes past the
        // end (the previous run's last step ended at a barrier: tb is free)
        for (u32 i = tid; i <= (u32)(t_end - t_begin); i += SCAN_TPB) {
            const u64 f = (t_begin + i) * TILE_LINES;
            tb[i] = f < P.n ? P.off[f] : (u32)P.nbytes;
        }
        __syncthreads();
        infA = tile_info<G::CAP>(P, t_begin, t_begin, tb);
        issue_tile_loads(P, infA, preA, offA, endA);
        for (u64 t = t_begin; t < t_end; ++t) tile_step(t, infA, preA, offA, endA);
    };
    auto use_segment = [&](const ScanSeg& sg) {
        P.bytes = sg.bytes;
        P.off = sg.off;
        P.n = sg.n;
        P.nbytes = sg.nbytes;
        P.line_base = sg.line_base;
        none.first = sg.n;
    };
    // Static share: the first n_static tiles of each segment, split evenly over the grid
    // (workgroup b: q tiles, one more for b < r).
    const u64 wg = blockIdx.x;
    for (u32 sgi = 0; sgi < P0.n_segs; ++sgi) {
        const ScanSeg& sg = P0.seg[sgi];
        t_begin = wg * sg.tiles_per_block + (wg < sg.static_rem ? wg : (u64)sg.static_rem);
        t_end = t_begin + sg.tiles_per_block + (wg < sg.static_rem ? 1u : 0u);
        if (t_begin >= t_end) continue;
        use_segment(sg);
        run_tiles();
    }
    // Dynamic share: the tiles past n_static, claimed in chunks of dyn_chunk from one
    // counter per segment by whichever workgroups finish their static share first (the
    // slower CUs' lag is absorbed instead of becoming the launch's tail).  The next
    // claim is issued before the current chunk runs, so its latency hides under it.
    if (P0.dyn_chunk) {
        u32 sgi = 0;
        u32 claim = 0;
        auto claim_next = [&](u32 si) -> u32 {
            u32 c = 0;
            if (lane == 0) c = atomicAdd(&P0.dyn_ctr[si], 1u);
            return c;
        };
        while (sgi < P0.n_segs && P0.seg[sgi].n_static >= P0.seg[sgi].n_tiles) ++sgi;
        if (sgi < P0.n_segs) claim = claim_next(sgi);
        while (sgi < P0.n_segs) {
            const ScanSeg& sg = P0.seg[sgi];
            const u32 c = (u32)__builtin_amdgcn_readfirstlane(__shfl(claim, 0, 64));
            t_begin = sg.n_static + (u64)c * P0.dyn_chunk;
            if (t_begin >= sg.n_tiles) {   // this segment's pool is empty: the next one
                ++sgi;
                while (sgi < P0.n_segs && P0.seg[sgi].n_static >= P0.seg[sgi].n_tiles) ++sgi;
                if (sgi < P0.n_segs) claim = claim_next(sgi);
                continue;
            }
            t_end = min<u64>(t_begin + P0.dyn_chunk, sg.n_tiles);
            claim = claim_next(sgi);
            use_segment(sg);
            run_tiles();
        }
    }
    if constexpr (REC) {   // the staged tails (partial lines), then the records per sub-buffer
        // the tails: the records after each bin's last complete line
        for (u32 b = 0; b < P.rec_bins; ++b) {
            const u32 staged = rcur[b], n = staged & 31u;
            if (n) rec_write(P, lcnt, b, staged - n, n, gcur, lane, ring_lo, ring_set, tl);
        }
        if (tid < (int)P.rec_bins) P.rec_n[(u64)blockIdx.x * P.rec_bins + tid] = gcur;
    }
    if (n_run == 0) return;   // no segment has tiles for this workgroup (nothing touched)
#ifdef YSB_STAMPS
    if (lane == 0) {
        unsigned long long* o = P.dbg + ((u64)blockIdx.x * (SCAN_TPB / 64) + (threadIdx.x >> 6)) * N_STAMPS;
        for (int i = 0; i < 7; ++i) o[i] += st_acc[i];
        o[7] += n_run;
    }
#endif
    // ---- final flush + stats ---------------------------------------------------------
    if (WL && lset) flush_window(P, lcnt, ncells, WL, lbase, ring_lo, ring_set, tl);
    flush_tally(P, tl, lane);
#ifdef YSB_WGTIME
    // diagnostic build (tools/wgtime.py): the workgroup's start / end, 100 MHz clock
    if (lane == 0) {
        unsigned long long* o = P.dbg + (u64)blockIdx.x * N_STAMPS;
        o[0] = wg_t0;
        o[1] = __builtin_amdgcn_s_memrealtime();
        o[2] = n_run;
    }
#endif
}

// ---------------------------------------------------------------------------
// The fork's live input format: pipe-delimited .tbl lines
// (MockWindowedFlatMap.flatMap, flink-benchmarks/.../AdvertisingTopologyNative.java:197-226):
//   items = line.split("\\|")   (java.lang.String.split: trailing empty items dropped)
//   (items[0..5]) = (user_id, page_id, ad_id, ad_type, event_type, event_time)
// fewer than 6 items after the trailing-empty drop -> ArrayIndexOutOfBounds (a parse
// error); then the same filter / join / bucket as the JSON chain (event_time = items[5],
// the Storm/Spark projection).  The line is the batch line minus its "\n" / "\r\n"
// terminator (BufferedReader.readLine, :153-159).
// ---------------------------------------------------------------------------
template <class S>
__device__ __forceinline__ bool process_tbl_line(const S& src, int s, int e, const ScanParams& P, Tally& t,
                                                 u32& campaign, i64& bucket) {
    t.ev++;
    if (e > s && src.b(e - 1) == '\n') --e;
    if (e > s && src.b(e - 1) == '\r') --e;
    // the first six '|' (p[5] = e when there are only five)
    int p[6];
    int k = 0;
    for (int q = s; q < e && k < 6; ++q)
        if (src.b(q) == '|') p[k++] = q;
    if (k < 5) { t.perr++; return false; }
    if (k == 5) p[5] = e;
    // items[5] exists iff something other than '|' follows the fifth '|'
    bool tail = p[5] > p[4] + 1;
    for (int q = p[5]; !tail && q < e; ++q) tail = src.b(q) != '|';
    if (!tail) { t.perr++; return false; }
    const Span et{p[3] + 1, p[4], 0};
    if (!(et.e - et.s == 4 && src.load4(et.s) == VIEW_W)) return false;   // EventFilterBolt
    t.view++;
    const Span ad{p[1] + 1, p[2], 0};
    u32 kw[KEY_WORDS];
    u32 klen = 0;
    int c = -1;
    const bool keyed = span_key(src, ad, kw, klen);
    if (keyed) c = probe(P.table, P.table_mask, kw, klen);   // RedisJoinBolt
    if (c < 0) { count_miss(P, kw, klen, keyed, t); return false; }
    t.join++;
    i64 tv;
    if (!parse_digits(src, p[4] + 1, p[5], tv)) { t.terr++; return false; }   // Long.parseLong
    campaign = (u32)c;
    bucket = div_trunc(tv, P.div);
    return true;
}

// Kernel 1b: the lines the fast path deferred (any layout other than the generator's,
// escapes, non-canonical ad ids, over-size tiles, bad offsets) through the general
// org.json parser (ysb_orgjson.h; .tbl rows: process_tbl_line).  Each lane stages its
// line into its own LDS region first (16-byte loads; regions 81 dwords apart, so the
// lanes' byte reads fall in distinct banks) and parses from there; longer lines are
// parsed straight from HBM.  With nothing deferred every workgroup returns at once.  Exact always; ~0 lines on generator data.
// The last workgroup to finish resets the list for the next batch.
#ifndef YSB_DEFER_TPB
#define YSB_DEFER_TPB 64          // one-wave workgroups, 20.7 KB of LDS each ...
#endif
#ifndef YSB_DEFER_WG_PER_CU
#define YSB_DEFER_WG_PER_CU 7     // ... seven per CU (the parse is latency-bound: more waves)
#endif
constexpr int DEFER_TPB = YSB_DEFER_TPB;
constexpr int DEFER_REGION_DW = 81;                       // per-lane LDS region (odd: bank spread)
constexpr int DEFER_STAGE_MAX = 4 * DEFER_REGION_DW - 16 - 16;   // line bytes staged (+ align, slack)
constexpr int DEFER_CHUNKS = (15 + DEFER_STAGE_MAX + 15) / 16;   // 16-B chunks a staged line can span
static_assert(4 * DEFER_CHUNKS + 1 <= DEFER_REGION_DW, "staged chunks + the slack word fit the region");

__global__ __launch_bounds__(DEFER_TPB) void defer_kernel(const ScanParams P0) {
    __shared__ u32 stage[DEFER_TPB * DEFER_REGION_DW];
    ScanParams P = P0;   // batch fields: the segment of the line being parsed
    const int tid = threadIdx.x, lane = tid & 63;
    if (blockIdx.x == 0 && tid == 0 && P.used_out) *P.used_out = *P.side_used;   // the scan's fill level, for the host
    const u32 total = *P.defer_count;
    if (total == 0u) return;   // nothing deferred (generator data): every workgroup leaves at once
    const u32 cnt = min(total, P.defer_cap);
    const i64 ring_lo = P.ring[0];
    const bool ring_set = P.ring[1] != 0;
    Tally tl{0, 0, 0, 0, 0, 0, 0, 0};
    u32* region = stage + tid * DEFER_REGION_DW;
    for (u32 i = blockIdx.x * DEFER_TPB + tid; i < cnt; i += gridDim.x * DEFER_TPB) {
        u64 li = P.defer[i];   // index among all segments' lines
        u32 sgi = 0;
        while (sgi + 1 < P0.n_segs && li >= P0.seg[sgi + 1].line_base) ++sgi;
        P.bytes = P0.seg[sgi].bytes;
        P.off = P0.seg[sgi].off;
        P.n = P0.seg[sgi].n;
        P.nbytes = P0.seg[sgi].nbytes;
        li -= P0.seg[sgi].line_base;
        const u64 ls = P.off[li];
        const u64 le = li + 1 < P.n ? (u64)P.off[li + 1] : P.nbytes;
        if (ls > le || le > P.nbytes || le - ls > 0x7FFFFFFFull) {
            tl.ev++;
            tl.perr++;
            continue;
        }
        u32 campaign;
        i64 bucket;
        bool ok;
        const u64 a16 = ls & ~15ull;
        const int sh = (int)(ls - a16), len = (int)(le - ls);
        if (len <= DEFER_STAGE_MAX) {
            const int nch = (sh + len + 15) >> 4;
            // every chunk's load issued before any is stored (one memory latency per line,
            // not one per chunk); P.bytes is 16-byte aligned
            uint4 v[DEFER_CHUNKS];
#pragma unroll
            for (int k = 0; k < DEFER_CHUNKS; ++k) {
                const u64 at = a16 + 16ull * (u64)k;
                v[k] = (k < nch && at + 16 <= P.nbytes) ? *reinterpret_cast<const uint4*>(P.bytes + at)
                                                        : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int k = 0; k < DEFER_CHUNKS; ++k) {
                if (k < nch) {
                    region[4 * k] = v[k].x;
                    region[4 * k + 1] = v[k].y;
                    region[4 * k + 2] = v[k].z;
                    region[4 * k + 3] = v[k].w;
                }
            }
            const u64 last = a16 + 16ull * (u64)(nch - 1);
            if (last + 16 > P.nbytes) {                        // the batch's last chunk: bytes, zeros past it
                for (int b = 0; b < 16; ++b) {
                    const u32 x = last + b < P.nbytes ? (u32)P.bytes[last + b] : 0u;
                    if ((b & 3) == 0) region[4 * (nch - 1) + (b >> 2)] = 0u;
                    region[4 * (nch - 1) + (b >> 2)] |= x << (8 * (b & 3));
                }
            }
            region[4 * nch] = 0u;                           // slack for word reads past the end
            const LdsSrc3 lsrc{(lds_u32*)region};
            if (P.tbl) ok = process_tbl_line(lsrc, sh, sh + len, P, tl, campaign, bucket);
#if YSB_FLAT_TIER
            else if (flat_line(lsrc, sh, sh + len, P, tl, campaign, bucket, ok)) {}
#endif
            else ok = process_line(lsrc, sh, sh + len, P, tl, campaign, bucket);
        } else {
            const GlbSrc gsrc{P.bytes + ls, le - ls};
            ok = P.tbl ? process_tbl_line(gsrc, 0, len, P, tl, campaign, bucket)
                       : process_line(gsrc, 0, len, P, tl, campaign, bucket);
        }
        if (ok) {
            global_add(P, ring_lo, ring_set, campaign, bucket, 1u, tl);
            *P.pend_dirty = 1u;   // the u64 ring holds pending counts now (the exchange reads it)
        }
    }
    flush_tally(P, tl, lane);
    __syncthreads();
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(P.defer_done, 1u) == gridDim.x - 1) {
            if (*P.defer_count > P.defer_cap) atomicAdd(&P.stats[ST_PARSE_ERR], (unsigned long long)(*P.defer_count - P.defer_cap));
            *P.defer_count = 0;
            *P.defer_done = 0;
        }
    }
}

// Ring auto-base: the first joined view with a valid time among the first 256 lines
// fixes the ring at min bucket - W/8 (room for out-of-order / late events).
__global__ __launch_bounds__(AUX_TPB) void ring_autobase_kernel(ScanParams P, i64* ring) {
    __shared__ i64 scratch[AUX_TPB / 64];
    if (ring[1] != 0) return;
    const int tid = threadIdx.x;
    i64 b = INT64_MAX;
    if ((u64)tid < P.n) {
        const u64 ls = P.off[tid];
        const u64 le = ((u64)tid + 1 < P.n) ? (u64)P.off[tid + 1] : P.nbytes;
        if (ls <= le && le <= P.nbytes && le - ls < 0x7FFFFFFFull) {
            Tally tl{0, 0, 0, 0, 0, 0, 0, 0};
            u32 c;
            i64 bk;
            const GlbSrc gsrc{P.bytes + ls, le - ls};
            if (process_line(gsrc, 0, (int)(le - ls), P, tl, c, bk)) b = bk;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const i64 x = __shfl_xor(b, o, 64);
        b = x < b ? x : b;
    }
    if ((tid & 63) == 0) scratch[tid >> 6] = b;
    __syncthreads();
    if (tid == 0) {
        i64 r = scratch[0];
        for (int w = 1; w < AUX_TPB / 64; ++w) r = scratch[w] < r ? scratch[w] : r;
        if (r != INT64_MAX) {
            ring[0] = r - (i64)(P.ring_w / 8);
            ring[1] = 1;
        }
    }
}


// One wave per 64-line tile, staged through LDS like the JSON scan; one line per lane.

// Ring auto-base for .tbl batches (the JSON one is ring_autobase_kernel).
__global__ __launch_bounds__(AUX_TPB) void tbl_ring_autobase_kernel(ScanParams P, i64* ring) {
    __shared__ i64 scratch[AUX_TPB / 64];
    if (ring[1] != 0) return;
    const int tid = threadIdx.x;
    i64 b = INT64_MAX;
    if ((u64)tid < P.n) {
        const u64 ls = P.off[tid];
        const u64 le = ((u64)tid + 1 < P.n) ? (u64)P.off[tid + 1] : P.nbytes;
        if (ls <= le && le <= P.nbytes && le - ls < 0x7FFFFFFFull) {
            Tally tl{0, 0, 0, 0, 0, 0, 0, 0};
            u32 c;
            i64 bk;
            const GlbSrc gsrc{P.bytes + ls, le - ls};
            if (process_tbl_line(gsrc, 0, (int)(le - ls), P, tl, c, bk)) b = bk;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const i64 x = __shfl_xor(b, o, 64);
        b = x < b ? x : b;
    }
    if ((tid & 63) == 0) scratch[tid >> 6] = b;
    __syncthreads();
    if (tid == 0) {
        i64 r = scratch[0];
        for (int w = 1; w < AUX_TPB / 64; ++w) r = scratch[w] < r ? scratch[w] : r;
        if (r != INT64_MAX) {
            ring[0] = r - (i64)(P.ring_w / 8);
            ring[1] = 1;
        }
    }
}

void launch_tbl_ring_autobase(const ScanParams& p, hipStream_t s) {
    if (p.n == 0) return;
    hipLaunchKernelGGL(tbl_ring_autobase_kernel, dim3(1), dim3(AUX_TPB), 0, s, p, const_cast<i64*>(p.ring));
}

void launch_scan(const ScanParams& p, hipStream_t s) {
    if (p.n == 0) return;
    const dim3 g(p.grid), b(SCAN_TPB);
    // record mode only with HBM-resident tables (large configurations: serial probes)
    if (p.tbl) {
        if (p.rec_on) hipLaunchKernelGGL((scan_kernel<true, true, true>), g, b, (Geom<true, true>::LDS), s, p);
        else if (p.probe_serial) hipLaunchKernelGGL((scan_kernel<true, true, false>), g, b, Geom<true>::LDS, s, p);
        else hipLaunchKernelGGL((scan_kernel<false, true, false>), g, b, Geom<true>::LDS, s, p);
    } else {
        // HBM-resident join table (configs[2]): record mode or serial probes, each with the
        // layout instantiations too (round 4), so other producers' layouts keep their fast tier
        if (p.rec_on) {
            if (p.layout == 1) hipLaunchKernelGGL((scan_kernel<true, false, true, 1>), g, b, (Geom<false, true>::LDS), s, p);
            else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<true, false, true, 2>), g, b, (Geom<false, true>::LDS), s, p);
            else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<true, false, true, 3>), g, b, (Geom<false, true>::LDS), s, p);
            else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<true, false, true, 4>), g, b, (Geom<false, true>::LDS), s, p);
            else hipLaunchKernelGGL((scan_kernel<true, false, true>), g, b, (Geom<false, true>::LDS), s, p);
        } else if (p.probe_serial) {
            if (p.layout == 1) hipLaunchKernelGGL((scan_kernel<true, false, false, 1>), g, b, Geom<false>::LDS, s, p);
            else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<true, false, false, 2>), g, b, Geom<false>::LDS, s, p);
            else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<true, false, false, 3>), g, b, Geom<false>::LDS, s, p);
            else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<true, false, false, 4>), g, b, Geom<false>::LDS, s, p);
            else hipLaunchKernelGGL((scan_kernel<true, false, false>), g, b, Geom<false>::LDS, s, p);
        } else if (p.layout == 1) hipLaunchKernelGGL((scan_kernel<false, false, false, 1>), g, b, Geom<false>::LDS, s, p);
        else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<false, false, false, 2>), g, b, Geom<false>::LDS, s, p);
        else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<false, false, false, 3>), g, b, Geom<false>::LDS, s, p);
        else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<false, false, false, 4>), g, b, Geom<false>::LDS, s, p);
        else hipLaunchKernelGGL((scan_kernel<false, false, false>), g, b, Geom<false>::LDS, s, p);
    }
}

void launch_defer(const ScanParams& p, int blocks, hipStream_t s) {
    if (p.n == 0) return;
    hipLaunchKernelGGL(defer_kernel, dim3(YSB_DEFER_WG_PER_CU * blocks), dim3(DEFER_TPB), 0, s, p);
}

void launch_ring_autobase(const ScanParams& p, hipStream_t s) {
    if (p.n == 0) return;
    hipLaunchKernelGGL(ring_autobase_kernel, dim3(1), dim3(AUX_TPB), 0, s, p, const_cast<i64*>(p.ring));
}

int scan_lds_bytes() { return LDS_BYTES; }

}  // namespace ysb
