// ysb_common.h -- definitions shared by host C++ and gfx950 device code.
//
//  * the synthetic event generator (a seeded, counter-based restatement of the
//    data/ Clojure generator's line format, data/src/setup/core.clj:90-96), so the
//    host dumper and the device generator emit byte-identical lines;
//  * the device ad -> campaign table layout and its hash;
//  * exact int64 division by the (runtime) window divisor, as Java's
//    Long.parseLong(t) / time_divisor (CampaignProcessorCommon.java:58).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define YSB_HD __host__ __device__ __forceinline__
#else
#define YSB_HD static inline
#endif

namespace ysb {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;

// ---------------------------------------------------------------------------
// Counter-based RNG (splitmix64 finaliser).  draw(stream, i) is a pure function
// of (seed, stream, i), so any event can be generated independently -- on any
// thread, any GPU, any host -- which is what makes the dump reproducible.
// ---------------------------------------------------------------------------
YSB_HD u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
YSB_HD u64 stream_key(u64 seed, u32 stream) {
    return mix64(seed * 0x9E3779B97F4A7C15ULL + stream);
}
YSB_HD u64 draw(u64 key, u64 i) { return mix64(key + (i + 1) * 0x9E3779B97F4A7C15ULL); }

enum : u32 {
    S_CAMPAIGN = 1, S_AD = 2, S_USER = 3, S_PAGE = 4, S_CHOICE = 5, S_SKEW = 6,
    S_USERPOOL = 7, S_PAGEPOOL = 8
};

// java.util.UUID.randomUUID() layout: version 4, IETF variant, lower-case hex,
// 8-4-4-4-12 (core.clj:20-22).
YSB_HD void uuid_words(u64 key, u64 k, u64* hi, u64* lo) {
    u64 h = draw(key, 2 * k), l = draw(key, 2 * k + 1);
    *hi = (h & ~0xF000ULL) | 0x4000ULL;
    *lo = (l & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
}
YSB_HD char hexdig(u32 v) { return (char)(v < 10 ? '0' + v : 'a' + (v - 10)); }
YSB_HD void uuid_format(u64 hi, u64 lo, char* out) {
    int o = 0;
    for (int i = 0; i < 16; ++i) {
        if (i == 8 || i == 12) out[o++] = '-';
        out[o++] = hexdig((u32)(hi >> (60 - 4 * i)) & 0xF);
    }
    for (int i = 0; i < 16; ++i) {
        if (i == 0 || i == 4) out[o++] = '-';
        out[o++] = hexdig((u32)(lo >> (60 - 4 * i)) & 0xF);
    }
}

// Generator constants (core.clj:68-69, 90-96).
#define YSB_P0 "{\"user_id\": \""
#define YSB_P1 "\", \"page_id\": \""
#define YSB_P2 "\", \"ad_id\": \""
#define YSB_P3 "\", \"ad_type\": \""
#define YSB_P4 "\", \"event_type\": \""
#define YSB_P5 "\", \"event_time\": \""
#define YSB_P6 "\", \"ip_address\": \"1.2.3.4\"}"
enum { LEN_P0 = 13, LEN_P1 = 15, LEN_P2 = 13, LEN_P3 = 15, LEN_P4 = 18, LEN_P5 = 18, LEN_P6 = 27 };
enum { LINE_FIXED = LEN_P0 + LEN_P1 + LEN_P2 + LEN_P3 + LEN_P4 + LEN_P5 + LEN_P6 + 3 * 36 + 1 };  // 228

YSB_HD const char* ad_type_str(u32 k) {
    return k == 0 ? "banner" : k == 1 ? "modal" : k == 2 ? "sponsored-search" : k == 3 ? "mail" : k == 4 ? "mobile"
         : k == 5 ? "native-video" : k == 6 ? "interstitial" : "rewarded";
}
YSB_HD u32 ad_type_len(u32 k) { return k == 0 ? 6 : k == 1 ? 5 : k == 2 ? 16 : k == 3 ? 4 : k == 4 ? 6 : k == 5 ? 12 : k == 6 ? 12 : 8; }
YSB_HD const char* event_type_str(u32 k) { return k == 0 ? "view" : k == 1 ? "click" : "purchase"; }
YSB_HD u32 event_type_len(u32 k) { return k == 0 ? 4 : k == 1 ? 5 : 8; }

// POD generator spec (host or device pointer in `subset`).
struct GenSpec {
    u64 seed;            // ids (campaigns, ads): shared by every rank
    u64 ev_seed;         // per-event draws: seed, or seed mixed with the event stream
    u32 n_campaigns, ads_per_campaign;
    i64 t0_ms;
    u64 events_per_sec;
    u32 with_skew, n_users;
    const u32* subset;   // ad indices to draw from (nullptr: all)
    u32 n_pick;          // number of ads drawn from
    u32 tbl;             // 1: the fork's .tbl rows instead of JSON lines
    u32 variant;         // GEN_V_* layout variants of the JSON lines (parity / tier tests)
};

// Off-vocabulary layouts of the same events (the generator's own stream is variant 0):
// other producers' lines that the vocabulary fast path does not take.
enum : u32 {
    GEN_V_RANDOM_IP = 1u,      // ip_address a random dotted quad instead of "1.2.3.4"
    GEN_V_MORE_AD_TYPES = 2u,  // ad_type one of 8 (adds native-video / interstitial / rewarded)
    GEN_V_COMPACT = 4u,        // no space after ':' and ',' (compact JSON)
    GEN_V_REORDER = 8u,        // the seven pairs in another (fixed) key order
    GEN_V_MIXED = 16u,         // four producers interleaved line by line: each event's layout is
                               // one of {generator, compact, reordered, random ip + 8 ad_types},
                               // drawn per event (the mutation tests' interleave, unmutated)
    GEN_V_MIXED_BLOCKS = 32u,  // the same four producers in runs of 256 events (a consumer's
                               // batches from several partitions): drawn per run
};
enum : u32 { S_IP = 9, S_MIX = 10 };

// The layout variant of event i (GEN_V_MIXED: drawn per event; GEN_V_MIXED_BLOCKS: per run of
// 256 events; else the spec's).
YSB_HD u32 event_variant(const GenSpec& s, u64 i) {
    if (!(s.variant & (GEN_V_MIXED | GEN_V_MIXED_BLOCKS))) return s.variant;
    const u64 unit = (s.variant & GEN_V_MIXED_BLOCKS) ? i >> 8 : i;
    const u32 k = (u32)(draw(stream_key(s.ev_seed, S_MIX), unit) >> 62);
    return k == 0 ? 0u : k == 1 ? (u32)GEN_V_COMPACT : k == 2 ? (u32)GEN_V_REORDER : (u32)(GEN_V_RANDOM_IP | GEN_V_MORE_AD_TYPES);
}

struct GenEvent {
    u32 ad, ad_type, event_type;
    i64 time_ms;
};

YSB_HD GenEvent gen_event(const GenSpec& s, u64 i) {
    GenEvent e;
    u64 c = draw(stream_key(s.ev_seed, S_CHOICE), i);
    u32 idx = (u32)(((c >> 32) * (u64)s.n_pick) >> 32);   // rand-nth ads (core.clj:92)
    e.ad = s.subset ? s.subset[idx] : idx;
    e.ad_type = (u32)(c & 0xFFFF) % ((event_variant(s, i) & GEN_V_MORE_AD_TYPES) ? 8u : 5u);   // rand-nth ad-types (:93)
    e.event_type = (u32)((c >> 16) & 0xFFFF) % 3u;         // rand-nth event-types (:94)
    i64 t = s.t0_ms + (i64)((i * 1000ULL) / s.events_per_sec);   // (+ start-time (* n 10)) (:95)
    if (s.with_skew) {                                      // make-kafka-event-at (:166-174)
        u64 r = draw(stream_key(s.ev_seed, S_SKEW), i);
        t += 50 - (i64)(r % 100);
        if (s.with_skew == 1 && ((r >> 17) % 100000ULL) == 0) t -= (i64)((r >> 40) % 60000ULL);   // 2: skew only
    }
    e.time_ms = t;
    return e;
}

YSB_HD u32 dec_len(i64 v) {
    u64 m = v < 0 ? (u64)0 - (u64)v : (u64)v;
    u32 n = 1;
    while (m >= 10) { m /= 10; ++n; }
    return n + (v < 0 ? 1u : 0u);
}
YSB_HD u32 dec_format(i64 v, char* out) {
    u32 n = dec_len(v);
    u64 m = v < 0 ? (u64)0 - (u64)v : (u64)v;
    u32 o = n;
    do { out[--o] = (char)('0' + (m % 10)); m /= 10; } while (m);
    if (v < 0) out[0] = '-';
    return n;
}

// The random dotted quad of event i (GEN_V_RANDOM_IP): bytes of one draw.
YSB_HD u32 gen_ip(const GenSpec& s, u64 i) { return (u32)draw(stream_key(s.ev_seed, S_IP), i); }
YSB_HD u32 ip_len(u32 ip) {
    u32 n = 3;   // the dots
    for (int k = 0; k < 4; ++k) n += dec_len((i64)((ip >> (8 * k)) & 0xFF));
    return n;
}

YSB_HD u32 gen_line_len(const GenSpec& s, u64 i, const GenEvent& e) {
    const u32 var = ad_type_len(e.ad_type) + event_type_len(e.event_type) + dec_len(e.time_ms);
    if (s.tbl) return 3u * 36u + 5u + 1u + var;
    u32 n = (u32)LINE_FIXED + var;
    const u32 v = event_variant(s, i);
    if (v & GEN_V_RANDOM_IP) n += ip_len(gen_ip(s, i)) - 7u;
    if (v & GEN_V_COMPACT) n -= 13u;   // 7 ": " and 6 ", " lose their space
    return n;
}

YSB_HD char* put_str(char* o, const char* s, u32 n) {
    for (u32 k = 0; k < n; ++k) o[k] = s[k];
    return o + n;
}

// A variant line (GEN_V_RANDOM_IP / GEN_V_COMPACT / GEN_V_REORDER): the same seven keys,
// in the generator's order or (GEN_V_REORDER) in the order ad_type, event_time, ad_id,
// ip_address, user_id, event_type, page_id; the separators with or without their space;
// the ip a random dotted quad.  Same pieces, so gen_line_len holds for every variant.
YSB_HD u32 gen_line_write_variant(const GenSpec& s, u64 i, const GenEvent& e, char* out, u32 variant) {
    const bool cp = (variant & GEN_V_COMPACT) != 0;
    const char* sep = cp ? "\",\"" : "\", \"";       // between a value and the next key
    const char* col = cp ? "\":\"" : "\": \"";       // between a key and its value
    const u32 ls = cp ? 3u : 4u;
    const u32 order_gen[7] = {0, 1, 2, 3, 4, 5, 6};
    const u32 order_re[7] = {3, 5, 2, 6, 0, 4, 1};
    const u32* order = (variant & GEN_V_REORDER) ? order_re : order_gen;
    char* o = out;
    u64 hi, lo;
    *o++ = '{';
    *o++ = '"';
    for (u32 k = 0; k < 7; ++k) {
        if (k) o = put_str(o, sep, ls);
        switch (order[k]) {
        case 0:
            o = put_str(o, "user_id", 7);
            o = put_str(o, col, ls);
            if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_USER), i, &hi, &lo);
            else uuid_words(stream_key(s.ev_seed, S_USER), draw(stream_key(s.ev_seed, S_USERPOOL), i) % s.n_users, &hi, &lo);
            uuid_format(hi, lo, o); o += 36;
            break;
        case 1:
            o = put_str(o, "page_id", 7);
            o = put_str(o, col, ls);
            if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_PAGE), i, &hi, &lo);
            else uuid_words(stream_key(s.ev_seed, S_PAGE), draw(stream_key(s.ev_seed, S_PAGEPOOL), i) % s.n_users, &hi, &lo);
            uuid_format(hi, lo, o); o += 36;
            break;
        case 2:
            o = put_str(o, "ad_id", 5);
            o = put_str(o, col, ls);
            uuid_words(stream_key(s.seed, S_AD), e.ad, &hi, &lo);
            uuid_format(hi, lo, o); o += 36;
            break;
        case 3:
            o = put_str(o, "ad_type", 7);
            o = put_str(o, col, ls);
            o = put_str(o, ad_type_str(e.ad_type), ad_type_len(e.ad_type));
            break;
        case 4:
            o = put_str(o, "event_type", 10);
            o = put_str(o, col, ls);
            o = put_str(o, event_type_str(e.event_type), event_type_len(e.event_type));
            break;
        case 5:
            o = put_str(o, "event_time", 10);
            o = put_str(o, col, ls);
            o += dec_format(e.time_ms, o);
            break;
        default:
            o = put_str(o, "ip_address", 10);
            o = put_str(o, col, ls);
            if (variant & GEN_V_RANDOM_IP) {
                const u32 ip = gen_ip(s, i);
                for (int q = 0; q < 4; ++q) {
                    if (q) *o++ = '.';
                    o += dec_format((i64)((ip >> (8 * q)) & 0xFF), o);
                }
            } else {
                o = put_str(o, "1.2.3.4", 7);
            }
            break;
        }
    }
    *o++ = '"';
    *o++ = '}';
    *o++ = '\n';
    return (u32)(o - out);
}

// One event line, exactly the str of core.clj:90-96 plus the "\n" of :97; with s.tbl
// the same event as the fork's .tbl row (MockWindowedFlatMap, AdvertisingTopologyNative.
// java:197-226): user_id|page_id|ad_id|ad_type|event_type|event_time\n, which is what
// ysb_json_to_tbl makes of the JSON line.
YSB_HD u32 gen_line_write(const GenSpec& s, u64 i, const GenEvent& e, char* out) {
    char* o = out;
    u64 hi, lo;
    if (s.tbl) {
        if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_USER), i, &hi, &lo);
        else uuid_words(stream_key(s.ev_seed, S_USER), draw(stream_key(s.ev_seed, S_USERPOOL), i) % s.n_users, &hi, &lo);
        uuid_format(hi, lo, o); o += 36;
        *o++ = '|';
        if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_PAGE), i, &hi, &lo);
        else uuid_words(stream_key(s.ev_seed, S_PAGE), draw(stream_key(s.ev_seed, S_PAGEPOOL), i) % s.n_users, &hi, &lo);
        uuid_format(hi, lo, o); o += 36;
        *o++ = '|';
        uuid_words(stream_key(s.seed, S_AD), e.ad, &hi, &lo);
        uuid_format(hi, lo, o); o += 36;
        *o++ = '|';
        o = put_str(o, ad_type_str(e.ad_type), ad_type_len(e.ad_type));
        *o++ = '|';
        o = put_str(o, event_type_str(e.event_type), event_type_len(e.event_type));
        *o++ = '|';
        o += dec_format(e.time_ms, o);
        *o++ = '\n';
        return (u32)(o - out);
    }
    const u32 v = event_variant(s, i);
    if (v & (GEN_V_RANDOM_IP | GEN_V_COMPACT | GEN_V_REORDER)) return gen_line_write_variant(s, i, e, out, v);
    o = put_str(o, YSB_P0, LEN_P0);
    if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_USER), i, &hi, &lo);
    else uuid_words(stream_key(s.ev_seed, S_USER), draw(stream_key(s.ev_seed, S_USERPOOL), i) % s.n_users, &hi, &lo);
    uuid_format(hi, lo, o); o += 36;
    o = put_str(o, YSB_P1, LEN_P1);
    if (s.n_users == 0) uuid_words(stream_key(s.ev_seed, S_PAGE), i, &hi, &lo);
    else uuid_words(stream_key(s.ev_seed, S_PAGE), draw(stream_key(s.ev_seed, S_PAGEPOOL), i) % s.n_users, &hi, &lo);
    uuid_format(hi, lo, o); o += 36;
    o = put_str(o, YSB_P2, LEN_P2);
    uuid_words(stream_key(s.seed, S_AD), e.ad, &hi, &lo);
    uuid_format(hi, lo, o); o += 36;
    o = put_str(o, YSB_P3, LEN_P3);
    o = put_str(o, ad_type_str(e.ad_type), ad_type_len(e.ad_type));
    o = put_str(o, YSB_P4, LEN_P4);
    o = put_str(o, event_type_str(e.event_type), event_type_len(e.event_type));
    o = put_str(o, YSB_P5, LEN_P5);
    o += dec_format(e.time_ms, o);
    o = put_str(o, YSB_P6, LEN_P6);
    *o++ = '\n';
    return (u32)(o - out);
}

// ---------------------------------------------------------------------------
// Device ad -> campaign table: open addressing, linear probing, 64-byte slots
// (one cache line per probe).  Slot words: [0] key length, [1] campaign index
// (EMPTY_SLOT = free), [2..15] key bytes, zero padded.  Keys are exact byte
// strings, i.e. HashMap<String,String>.get semantics on the ad_id string
// (AdvertisingTopologyNative.java:464).
// ---------------------------------------------------------------------------
enum : u32 { SLOT_WORDS = 16, KEY_WORDS = 14, MAX_KEY_BYTES = 56, EMPTY_SLOT = 0xFFFFFFFFu };

// Hash of a zero-padded key held as little-endian 32-bit words.
YSB_HD u32 key_hash(const u32* w, u32 len) {
    u32 h = 0x811C9DC5u ^ (len * 0x9E3779B1u);
    u32 nw = (len + 3) >> 2;
    for (u32 k = 0; k < nw; ++k) {
        h = (h ^ w[k]) * 0x01000193u;
        h ^= h >> 15;
    }
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

// ---------------------------------------------------------------------------
// 36-byte-key cuckoo table (the join's fast path).  Every map key of exactly 36
// bytes (the UUID strings core.clj:31-32 and java.util.UUID.toString() produce, but
// any 36 bytes) sits in one of its two slots, so a lookup is exactly two slot loads
// issued together and a raw 9-word compare -- no decoding, no key validation.
// Slot words: [key bytes 0..35 as 9 little-endian u32, campaign (EMPTY_SLOT = free),
// 0 x 6] = 64 bytes, of which a probe loads the first 48 (three 16-byte loads).  The
// 64-byte stride keeps every slot inside one 128-byte line (48-byte slots straddle two
// for a quarter of the probes): config 3's HBM-resident table +3 %, config 2 +0.3 %
// (gpurun_out/c16, c16h, c16i).
// The slot hash folds the words with per-seed additive salts (the carries make a
// colliding key family seed-dependent, so a failed build is cured by a new seed),
// then avalanches: x = XOR rotl(w_k + s_k, R_k), y = SUM (w_k ^ s'_k).
// ---------------------------------------------------------------------------
#ifndef YSB_CSLOT_WORDS
#define YSB_CSLOT_WORDS 16
#endif
enum : u32 { CSLOT_WORDS = YSB_CSLOT_WORDS, CKEY_WORDS = 9, CSLOT_CAMP = 9, CSLOT_Q = YSB_CSLOT_WORDS / 4 };
// HBM-resident tables (beyond the L2s: configs[2]'s 10M ads) use BUCKETS instead: 128 B =
// 3 entries of [9 key words, campaign] at a 10-word stride (+ 2 spare words).  A key goes
// to its first bucket while that has a free entry, to its second only when the first is
// full (cuckoo eviction keeps a full bucket full), so a lookup reads one 128-B line and
// reads the second bucket only when the key is not in a FULL first bucket -- at 2 buckets
// per key ~0.1 % of keys instead of the ~8 % a one-key slot table leaves in its second
// slot, each of which cost the whole wave a dependent HBM round trip.
enum : u32 { CB_WORDS = 32, CB_ENTRIES = 3, CB_STRIDE = 10, CB_Q = CB_WORDS / 4 };

struct CuckooSeed {
    u32 s[CKEY_WORDS];   // additive salts of the XOR fold
    u32 t[CKEY_WORDS];   // XOR salts of the sum fold
    u32 fa, fb;          // finaliser salts
};

YSB_HD u32 rotl32(u32 x, u32 r) { return (x << r) | (x >> (32u - r)); }   // 1 <= r <= 31
YSB_HD u32 fmix32(u32 h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

YSB_HD void cuckoo_slots36(const u32* w, const CuckooSeed& cs, u32 mask, u32* a, u32* b) {
    const u32 R[CKEY_WORDS] = {1, 6, 11, 16, 21, 26, 31, 4, 9};
    u32 x = 0, y = 0;
#pragma unroll
    for (u32 k = 0; k < CKEY_WORDS; ++k) {
        x ^= rotl32(w[k] + cs.s[k], R[k]);
        y += w[k] ^ cs.t[k];
    }
    const u32 ha = fmix32(x ^ cs.fa);
    const u32 hb = fmix32(y ^ cs.fb ^ rotl32(x, 16));
    *a = ha & mask;
    const u32 bb = hb & mask;
    *b = bb == *a ? ((bb + 1) & mask) : bb;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host build of the bucket-layout table (ysb_load_ad_map): key i (9 words) with campaign
// camp[i] into nb buckets (ct: nb * CB_WORDS words, cleared here).  A key goes to its
// first bucket while that has a free entry, else to its second; with both full it takes a
// random entry of the bucket it is headed for (which so stays full) and the evicted key
// tries only its other bucket.  So a key sits in its second bucket only while its first
// is full -- the probe's rule.  Returns the keys left out (keep_going: placement goes on
// without them, a partial table; else it stops at the first).
static inline u64 cuckoo_build_buckets(const u32* keys, const u32* camp, u64 n, const CuckooSeed& cs, u64 nb,
                                       u64 seed, bool keep_going, u32* ct) {
    for (u64 i = 0; i < nb * CB_WORDS; ++i) ct[i] = 0;
    for (u64 b = 0; b < nb; ++b)
        for (u32 e = 0; e < CB_ENTRIES; ++e) ct[b * CB_WORDS + e * CB_STRIDE + CKEY_WORDS] = EMPTY_SLOT;
    const u32 mask = (u32)(nb - 1);
    u64 rng = seed, homeless = 0;
    for (u64 i = 0; i < n; ++i) {
        u32 k[CKEY_WORDS];
        for (u32 j = 0; j < CKEY_WORDS; ++j) k[j] = keys[i * CKEY_WORDS + j];
        u32 c = camp[i];
        u32 a, b;
        cuckoo_slots36(k, cs, mask, &a, &b);
        u32 pos = a;
        bool placed = false;
        for (int kicks = 0; kicks <= 500 && !placed; ++kicks) {
            const u32 cands[2] = {pos, pos == a ? b : a};
            for (int ci = 0; ci < (kicks == 0 ? 2 : 1) && !placed; ++ci) {
                u32* bk = &ct[(u64)cands[ci] * CB_WORDS];
                for (u32 e = 0; e < CB_ENTRIES && !placed; ++e)
                    if (bk[e * CB_STRIDE + CKEY_WORDS] == EMPTY_SLOT) {
                        for (u32 j = 0; j < CKEY_WORDS; ++j) bk[e * CB_STRIDE + j] = k[j];
                        bk[e * CB_STRIDE + CKEY_WORDS] = c;
                        placed = true;
                    }
            }
            if (placed) break;
            rng = mix64(rng + 1);
            u32* en = &ct[(u64)pos * CB_WORDS + (u32)(rng % CB_ENTRIES) * CB_STRIDE];
            for (u32 j = 0; j < CKEY_WORDS; ++j) {
                const u32 t = en[j];
                en[j] = k[j];
                k[j] = t;
            }
            const u32 oc = en[CKEY_WORDS];
            en[CKEY_WORDS] = c;
            c = oc;
            cuckoo_slots36(k, cs, mask, &a, &b);
            pos = (pos == a) ? b : a;   // the evicted key's other bucket
        }
        if (!placed) {
            ++homeless;
            if (!keep_going) return homeless;
        }
    }
    return homeless;
}

// Host restatement of the scan's bucket probe (ysb_scan.hip bucket_find + the second
// bucket after a miss in a full first one): the campaign, or EMPTY_SLOT.
static inline u32 cuckoo_lookup_buckets(const u32* ct, u64 nb, const CuckooSeed& cs, const u32* k) {
    u32 a, b;
    cuckoo_slots36(k, cs, (u32)(nb - 1), &a, &b);
    for (int round = 0; round < 2; ++round) {
        const u32* bk = &ct[(u64)(round ? b : a) * CB_WORDS];
        bool full = true;
        for (u32 e = 0; e < CB_ENTRIES; ++e) {
            const u32 c = bk[e * CB_STRIDE + CKEY_WORDS];
            if (c == EMPTY_SLOT) { full = false; continue; }
            bool eq = true;
            for (u32 j = 0; j < CKEY_WORDS; ++j) eq &= bk[e * CB_STRIDE + j] == k[j];
            if (eq) return c;
        }
        if (!full) return EMPTY_SLOT;
    }
    return EMPTY_SLOT;
}

static inline CuckooSeed cuckoo_seed(u64 seed) {
    CuckooSeed cs;
    for (u32 k = 0; k < CKEY_WORDS; ++k) {
        const u64 r = mix64(seed + 2 * k + 1);
        cs.s[k] = (u32)r;
        cs.t[k] = (u32)(r >> 32);
    }
    const u64 f = mix64(seed ^ 0xF1F1F1F1F1F1F1F1ULL);
    cs.fa = (u32)f;
    cs.fb = (u32)(f >> 32);
    return cs;
}
#endif

// ---------------------------------------------------------------------------
// Exact Java long division t / d (truncating toward zero) for a runtime d >= 1,
// as a multiply-high: for n < 2^63, floor(n/d) = mulhi(n, M) >> s with
// l = ceil(log2 d), M = ceil(2^(63+l) / d) < 2^64, s = l - 1 (Granlund-Montgomery).
// INT64_MIN (|t| = 2^63) is precomputed.
// ---------------------------------------------------------------------------
struct DivMagic {
    u64 M;
    u32 s;
    u32 is_one;
    i64 d;
    i64 q_min;   // INT64_MIN / d
};

#if !defined(__HIP_DEVICE_COMPILE__)
static inline DivMagic div_magic(i64 d) {
    DivMagic m;
    m.d = d;
    m.q_min = INT64_MIN / d;
    m.is_one = d == 1;
    u32 l = 0;
    while (l < 63 && ((u64)1 << l) < (u64)d) ++l;
    if (d == 1) { m.M = 0; m.s = 0; return m; }
    // M = ceil(2^(63+l)/d) computed with 128-bit arithmetic
    unsigned __int128 num = (unsigned __int128)1 << (63 + l);
    unsigned __int128 q = num / (u64)d;
    if (num % (u64)d) q += 1;
    m.M = (u64)q;
    m.s = l - 1;
    return m;
}
#endif

YSB_HD u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}

YSB_HD i64 div_trunc(i64 t, const DivMagic& m) {
    if (m.is_one) return t;
    if (t == INT64_MIN) return m.q_min;
    u64 n = t < 0 ? (u64)(-t) : (u64)t;
    u64 q = mulhi64(n, m.M) >> m.s;
    return t < 0 ? -(i64)q : (i64)q;
}

// Stats slots in the device stats array.
enum : u32 {
    ST_EVENTS = 0, ST_VIEWS, ST_JOINED, ST_MISSES, ST_PARSE_ERR, ST_TIME_ERR,
    ST_OUT_OF_RING, ST_OVF_DROPPED, ST_DEFERRED, ST_FOREIGN, ST_COUNT_
};

// ysb_ad_shard: the rank of nranks whose join-table shard holds a key (zero-padded words,
// len <= MAX_KEY_BYTES); host and device (the deferred-line kernel's miss path) alike.
YSB_HD u32 key_shard(u32 h, u32 nranks) { return (u32)(((mix64(h) >> 32) * (u64)nranks) >> 32); }

// Weight of the (campaign, bucket) cell in the linear table checksums (ysb_group_checksum):
// odd, so a single wrong count always changes the sum; sums of tables add like the tables.
YSB_HD u64 cell_weight(u32 campaign, i64 bucket) {
    return mix64(((u64)campaign << 40) ^ ((u64)bucket * 0x9E3779B97F4A7C15ULL)) | 1ull;
}

// Out-of-ring (campaign, bucket) cells: an open-addressing device hash map with one
// 64-bit key per cell (bucket offset by 2^(63 - cbits) in the high bits, campaign in
// the low cbits = bit_width(n_campaigns) bits, so the all-ones key never occurs and marks
// an empty slot).  Insert = one 64-bit CAS, then a 64-bit atomic add.
struct SideSlot {
    unsigned long long key;
    unsigned long long count;
};
constexpr unsigned long long SIDE_EMPTY = ~0ull;

struct OvfEntry {
    u32 campaign;
    u32 count;
    i64 bucket;
};

}  // namespace ysb
