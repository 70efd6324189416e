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

// ---- diagnostic builds (make diag / variant; never used for results) ----------------------
// Each flag cuts one part of the scan so that a profile attributes time to it: the results
// of such a build are wrong by design (profiles/AB_LOG.md, "where the time goes").  The
// stamps builds (YSB_STAMPS: in-kernel phase stamps, YSB_WGTIME: per-workgroup start / end)
// are the other diagnostics (tools/stamps.py, tools/wgtime.py).
#ifndef YSB_DIAG_A_ONLY
#define YSB_DIAG_A_ONLY 0      // Phase A only: tiles staged into LDS, nothing parsed
#endif
#ifndef YSB_DIAG_NO_PROBE
#define YSB_DIAG_NO_PROBE 0    // no join-table loads: the key "found" in the first slot
#endif
#ifndef YSB_DIAG_NO_PROBE2
#define YSB_DIAG_NO_PROBE2 0   // no second-bucket probe (HBM-resident table)
#endif
#ifndef YSB_DIAG_NO_COUNT
#define YSB_DIAG_NO_COUNT 0    // joined views not counted (no records, no ring atomics)
#endif
#ifndef YSB_DIAG_NO_REC
#define YSB_DIAG_NO_REC 0      // record mode: views parsed, never staged
#endif
#ifndef YSB_DIAG_NO_FLUSH
#define YSB_DIAG_NO_FLUSH 0    // LDS window counters never flushed to the ring
#endif
#ifndef YSB_DIAG_FLAT_IDX
#define YSB_DIAG_FLAT_IDX 0    // layout 2: the structural index's classification only (round 6)
#endif

namespace ysb {

constexpr bool DIAG_A_ONLY = YSB_DIAG_A_ONLY, DIAG_NO_PROBE = YSB_DIAG_NO_PROBE,
               DIAG_NO_PROBE2 = YSB_DIAG_NO_PROBE2, DIAG_NO_COUNT = YSB_DIAG_NO_COUNT,
               DIAG_NO_REC = YSB_DIAG_NO_REC, DIAG_NO_FLUSH = YSB_DIAG_NO_FLUSH,
               DIAG_FLAT_IDX = YSB_DIAG_FLAT_IDX;

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

}  // namespace ysb

#include "ysb_scan_canon.h"
#include "ysb_scan_tbl.h"

namespace ysb {

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

}  // namespace ysb

#include "ysb_scan_flat.h"

namespace ysb {

// LDS layout (dynamic, 16-byte aligned carve, no static __shared__)
// ---------------------------------------------------------------------------
constexpr int LDS_BYTES = Geom<false>::LDS;
// layouts 2-4 (the flat tier) launch with the key table past the geometry's LDS; the JSON
// geometries keep their workgroups per CU with it
constexpr int FLAT_KT_LDS = KEYTAB_BYTES;
static_assert((Geom<false>::LDS + FLAT_KT_LDS + 1279) / 1280 * 1280 * Geom<false>::WG_PER_CU <= 163840 &&
                  (Geom<false, true>::LDS + FLAT_KT_LDS + 1279) / 1280 * 1280 * Geom<false, true>::WG_PER_CU <= 163840,
              "the flat tier's key table must not cost a workgroup per CU");   // the JSON geometry (Geom<true> for .tbl rows)

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
    // a tile of long lines is staged up to its capacity: the lines that end inside it are
    // parsed, the rest deferred (the whole tile before)
    ti.oversize = !sane;
    if (sane && len > (u64)CAP) ti.e = s0 - ti.delta + (u32)CAP;
    ti.len = ti.oversize ? 0u : (u32)(len < (u64)CAP ? len : (u64)CAP);
    return ti;
}

// Cache policy of the once-read batch stream: nontemporal (aux 2), so it does not
// displace the join table from L2 (MI355X_MICROARCH.md, row nt-weights).
constexpr int AUX_NT = 2;

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
// The tile line a lane parses.  Interleaved: lanes 0..31 take the even lines, 32..63 the
// odd ones, so the start banks of the lines a 32-lane half reads (dword mod 32, lines
// ~63.5 dwords apart) step by one bank instead of crowding into half of them.
__device__ __forceinline__ u32 lane_line(int tid) {
    return ((u32)(tid & 31) << 1) | ((u32)tid >> 5);
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
            if constexpr (!DIAG_NO_FLUSH)
                global_add(P, ring_lo, ring_set, i >> P.lds_wl_log2, lbase + (i64)(i & (WL - 1)), v, tl);
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
    // the flat tier's key table past the geometry's LDS (layouts 2-4 launch with KEYTAB_BYTES more)
    u32* keytab = reinterpret_cast<u32*>(smem + G::LDS);
    if constexpr (!TBL && LAY >= 2) {
        if (threadIdx.x < 64) keytab[threadIdx.x] = KEYTAB.w[threadIdx.x];
        __syncthreads();
    }

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
    // Prefetch depth: tile t + PF_DEPTH is issued once tile t sits in LDS (depth 2, two
    // register buffers, measured -2 % and spilled: profiles/AB_LOG.md).
    constexpr int PF_DEPTH = 1;
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
    // static priority for every other workgroup: the two waves of a SIMD stop trading
    // VALU issue by age (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);
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
        if constexpr (DIAG_A_ONLY) {
            inf = t + PF_DEPTH < t_end ? tile_info<G::CAP>(P, t + PF_DEPTH, t_begin, tb) : none;
            issue_tile_loads(P, inf, pre, pre_off, pre_end);
            __syncthreads();
            return;
        }
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
            if constexpr (TBL) ok1 = tbl_stage1(lsrc, ls, le, ca);
            else if constexpr (LAY == 2 && DIAG_FLAT_IDX) {
                const u32 x = flat_index_only(lsrc, ls, le);   // timing diagnostic: nothing counted
                if (x == 0x9E3779B9u) tl.miss += 1;
            }
            else if constexpr (LAY == 2) ok1 = flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, ca, cb, keytab);
            else if constexpr (LAY == 3) {
                ok1 = P.learn_cp ? learned_parse<true>(lsrc, ls, le, P, ca, cb) : learned_parse<false>(lsrc, ls, le, P, ca, cb);
                // a line off the learned order: the flat tier (any order or spacing)
                if (__builtin_expect(!ok1, 0)) ok1 = flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, ca, cb, keytab);
            }
            else if constexpr (LAY == 4) {}   // below, once the wave's mode is known
            else ok1 = vocab_stage1<LAY == 1>(lsrc, ls, le, ca);
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
            else ok2 = ok1 && vocab_stage2<LAY == 1>(lsrc, ls, le, ca, cb);
        }
        if constexpr (!TBL && LAY < 2) {
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
                if (!t) t = flat_tier<LdsSrc, false>(lsrc, ls, le, P.require_mask, c2, b2);   // any key order / spacing
                if (t) {
                    ca = c2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        if constexpr (LAY == 4) {
            if (elig && fl) {   // the flat tier: a mixed tile's lines, and the lanes its path rejected
                CanonA c2;
                CanonB b2;
                b2.view = false;
                if (flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, c2, b2, keytab)) {
                    ca = c2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        dfr = li < cur.count && !ok2 && !(DIAG_FLAT_IDX && LAY == 2);   // bad offsets, other layouts, escapes, over-size tiles
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
        if constexpr (DIAG_NO_PROBE) {
            if (pend) {   // diagnostic build: the first slot / entry "holds" the key, campaign from its bytes
                a0 = make_uint4(ca.kw[0], ca.kw[1], ca.kw[2], ca.kw[3]);
                a1 = make_uint4(ca.kw[4], ca.kw[5], ca.kw[6], ca.kw[7]);
                a2 = make_uint4(ca.kw[8], ca.kw[0] % P.n_campaigns, 0, 0);
                q[0] = a0;
                q[1] = a1;
                q[2] = a2;
            }
        }
        if (pend && !DIAG_NO_PROBE) {
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
                if (!DIAG_NO_PROBE2 && ci == EMPTY_SLOT && full) {   // the second bucket
#pragma unroll
                    for (int j = 0; j < (int)CB_Q; ++j) q[j] = ct4[CB_Q * (u64)ib_s + j];
                    ci = bucket_find(q, k, full);
                }
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
        } else if (valid && !DIAG_NO_COUNT) {
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
        }
        if constexpr (DIAG_NO_REC) rec_has = false;   // diagnostic build: views found and parsed, never counted
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
            else if (flat_line(lsrc, sh, sh + len, P, tl, campaign, bucket, ok)) {}
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
            else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<true, false, true, 2>), g, b, (Geom<false, true>::LDS + FLAT_KT_LDS), s, p);
            else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<true, false, true, 3>), g, b, (Geom<false, true>::LDS + FLAT_KT_LDS), s, p);
            else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<true, false, true, 4>), g, b, (Geom<false, true>::LDS + FLAT_KT_LDS), s, p);
            else hipLaunchKernelGGL((scan_kernel<true, false, true>), g, b, (Geom<false, true>::LDS), s, p);
        } else if (p.probe_serial) {
            if (p.layout == 1) hipLaunchKernelGGL((scan_kernel<true, false, false, 1>), g, b, Geom<false>::LDS, s, p);
            else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<true, false, false, 2>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
            else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<true, false, false, 3>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
            else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<true, false, false, 4>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
            else hipLaunchKernelGGL((scan_kernel<true, false, false>), g, b, Geom<false>::LDS, s, p);
        } else if (p.layout == 1) hipLaunchKernelGGL((scan_kernel<false, false, false, 1>), g, b, Geom<false>::LDS, s, p);
        else if (p.layout == 2) hipLaunchKernelGGL((scan_kernel<false, false, false, 2>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
        else if (p.layout == 3) hipLaunchKernelGGL((scan_kernel<false, false, false, 3>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
        else if (p.layout == 4) hipLaunchKernelGGL((scan_kernel<false, false, false, 4>), g, b, (Geom<false>::LDS + FLAT_KT_LDS), s, p);
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
