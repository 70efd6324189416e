// ysb_scan_tbl.h -- the .tbl fast path of Kernel 1 (MockWindowedFlatMap's
// pipe-delimited rows, AdvertisingTopologyNative.java:197-226).
// Part of the scan kernel's translation unit: included by ysb_scan.hip only, after the
// definitions it uses (the LDS sources, spans, load_span, the org.json machine).
#pragma once

namespace ysb {

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
    const int a = s >> 2;
#pragma unroll
    for (int k = 0; k <= TBL_WORDS; ++k) P[k] = src.d[a + k];
    u32 W[TBL_WORDS];
    u32 B[5] = {0u, 0u, 0u, 0u, 0u};   // bit i = line byte i may be '|'
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

}  // namespace ysb
