// ysb_host.cpp -- host-only parts of the C ABI (no HIP calls, usable without a GPU):
// the multi-GPU partitioning that replaces Flink's keyBy(0) shuffle
// (flink-benchmarks/.../AdvertisingTopologyNative.java:118) and the sharded file-dump
// mode of the generator.
//
//   ysb_group_block      campaign block a rank owns after ysb_group_reduce_scatter
//   ysb_route_lines      per-line ad_id shard of a host batch (host router)
//   ysb_gen_dump_shards  kafka-json.<r>.txt per shard (config 4's pre-sharded files)
//   ysb_json_to_tbl      the fork's events.tbl rows from generator JSON lines
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ysb_hip.h"
#include "ysb_common.h"

using namespace ysb;

namespace {

bool is_ws(u8 c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// End of the string whose content starts at p (index of its closing quote q), or -1.
long scan_string(const u8* s, long p, long e, u8 q = '"') {
    while (p < e) {
        if (s[p] == q) return p;
        if (s[p] == '\\') p += 2;
        else ++p;
    }
    return -1;
}

// Skips one non-string JSON value (number, literal, nested object/array); -1 if malformed.
long skip_value(const u8* s, long p, long e) {
    if (p >= e) return -1;
    if (s[p] == '{' || s[p] == '[') {
        int depth = 0;
        while (p < e) {
            const u8 c = s[p];
            if (c == '"') {
                const long q = scan_string(s, p + 1, e);
                if (q < 0) return -1;
                p = q + 1;
                continue;
            }
            if (c == '{' || c == '[') ++depth;
            else if ((c == '}' || c == ']') && --depth == 0) return p + 1;
            ++p;
        }
        return -1;
    }
    while (p < e && s[p] != ',' && s[p] != '}' && !is_ws(s[p])) ++p;
    return p;
}


// ---- org.json string decoding, as the device decodes a key (ysb_orgjson.h decode_str) ----------

bool hex_digit(u8 c, u32* v) {
    if (c >= '0' && c <= '9') { *v = c - '0'; return true; }
    if (c >= 'a' && c <= 'f') { *v = c - 'a' + 10; return true; }
    if (c >= 'A' && c <= 'F') { *v = c - 'A' + 10; return true; }
    return false;
}

// \uXXXX at p (the backslash): Integer.parseInt(XXXX, 16) as a UTF-16 unit -- a leading sign
// takes three digits (\u-001 is U+FFFF), as JSONTokener.next(4) + parseInt read it.
bool utf16_unit(const u8* s, long p, long e, bool sign_ok, u32* out) {
    if (p + 5 >= e || s[p] != '\\' || s[p + 1] != 'u') return false;
    const u8 d0 = s[p + 2];
    u32 v = 0, d;
    if (sign_ok && (d0 == '+' || d0 == '-')) {
        for (int k = 3; k < 6; ++k) {
            if (!hex_digit(s[p + k], &d)) return false;
            v = v << 4 | d;
        }
        *out = d0 == '-' ? (0x10000u - v) & 0xFFFFu : v;
        return true;
    }
    for (int k = 2; k < 6; ++k) {
        if (!hex_digit(s[p + k], &d)) return false;
        v = v << 4 | d;
    }
    *out = v;
    return true;
}

void put_utf8(u32 cp, std::string& o) {   // lone surrogates: the 3-byte form
    if (cp < 0x80) { o += (char)cp; return; }
    if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); return; }
    if (cp < 0x10000) {
        o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        return;
    }
    o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
    o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
}

// The string content s[a, b) with its escapes decoded to UTF-8, byte for byte what the
// device's decode_str produces (so the host route and the device's shard test hash the same
// key): \b \t \n \f \r, \x -> x, \uXXXX (a high surrogate directly followed by a low one is
// one code point).  An escape org.json would reject is kept raw: such a line fails to parse
// on the device, where its shard does not matter.
std::string decode_escapes(const u8* s, long a, long b) {
    std::string o;
    o.reserve((size_t)(b - a));
    for (long p = a; p < b;) {
        const u8 c = s[p];
        if (c != '\\' || p + 1 >= b) { o += (char)c; ++p; continue; }
        const u8 x = s[p + 1];
        if (x != 'u') {
            o += (char)(x == 'b' ? 8 : x == 't' ? 9 : x == 'n' ? 10 : x == 'f' ? 12 : x == 'r' ? 13 : x);
            p += 2;
            continue;
        }
        u32 cp;
        if (!utf16_unit(s, p, b, true, &cp)) { o += (char)c; ++p; continue; }
        p += 6;
        u32 lo;
        if (cp >= 0xD800 && cp < 0xDC00 && utf16_unit(s, p, b, false, &lo) && lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            p += 6;
        }
        put_utf8(cp, o);
    }
    return o;
}

}  // namespace

// The top-level "ad_id" string value of one line: its content span [*vs, *ve) and whether
// it holds escapes (*esc).  Keys are compared decoded, as org.json compares them, so an
// escaped key name ("ad_id") is found too; strings may be double- or single-quoted.
// Generator lines (data/src/setup/core.clj:90-96) have the value at byte 113; other
// layouts take a small key scan.  Returns false when the line has no string ad_id.
static bool find_ad_id(const u8* s, long n, long* vs, long* ve, bool* esc) {
    static const char canon[] = "\"ad_id\": \"";   // bytes 103..112 of a generator line
    *esc = false;
    if (n > 150 && std::memcmp(s + 103, canon, 10) == 0 && s[149] == '"' &&
        std::memchr(s + 113, '"', 36) == nullptr && std::memchr(s + 113, '\\', 36) == nullptr &&
        std::memcmp(s, "{\"user_id\": \"", 13) == 0) {
        // the fixed prefix is only trusted when the two UUIDs before it are plain
        if (!std::memchr(s + 13, '"', 36) && !std::memchr(s + 64, '"', 36) &&
            !std::memchr(s + 13, '\\', 36) && !std::memchr(s + 64, '\\', 36) &&
            std::memcmp(s + 49, "\", \"page_id\": \"", 15) == 0 && std::memcmp(s + 100, "\", ", 3) == 0) {
            *vs = 113;
            *ve = 149;
            return true;
        }
    }
    auto has_bs = [&](long a, long b) { return std::memchr(s + a, '\\', (size_t)(b - a)) != nullptr; };
    long p = 0;
    while (p < n && is_ws(s[p])) ++p;
    if (p >= n || s[p] != '{') return false;
    ++p;
    while (true) {
        while (p < n && is_ws(s[p])) ++p;
        if (p >= n || (s[p] != '"' && s[p] != '\'')) return false;
        const long ke = scan_string(s, p + 1, n, s[p]);
        if (ke < 0) return false;
        bool is_ad = ke - p - 1 == 5 && std::memcmp(s + p + 1, "ad_id", 5) == 0;
        if (!is_ad && has_bs(p + 1, ke)) is_ad = decode_escapes(s, p + 1, ke) == "ad_id";
        p = ke + 1;
        while (p < n && is_ws(s[p])) ++p;
        if (p >= n || s[p] != ':') return false;
        ++p;
        while (p < n && is_ws(s[p])) ++p;
        if (p >= n) return false;
        if (s[p] == '"' || s[p] == '\'') {
            const long q = scan_string(s, p + 1, n, s[p]);
            if (q < 0) return false;
            if (is_ad) {
                *vs = p + 1;
                *ve = q;
                *esc = has_bs(p + 1, q);
                return true;
            }
            p = q + 1;
        } else {
            p = skip_value(s, p, n);
            if (p < 0) return false;
        }
        while (p < n && is_ws(s[p])) ++p;
        if (p < n && (s[p] == ',' || s[p] == ';')) { ++p; continue; }
        return false;   // '}' without an ad_id, or malformed
    }
}

extern "C" {

int ysb_group_block(uint32_t n_campaigns, int rank, int nranks, uint32_t* lo, uint32_t* hi) {
    if (nranks < 1 || rank < 0 || rank >= nranks) return YSB_ERR_ARG;
    const u32 cp = (n_campaigns + (u32)nranks - 1) / (u32)nranks * (u32)nranks;
    const u32 per = cp / (u32)nranks;
    const u32 l = std::min<u32>(n_campaigns, (u32)rank * per);
    if (lo) *lo = l;
    if (hi) *hi = std::min<u32>(n_campaigns, l + per);
    return YSB_OK;
}

int ysb_route_lines(const uint8_t* bytes, uint64_t nbytes, const uint32_t* line_off, uint64_t n,
                    uint32_t nranks, uint32_t* out_shard, uint64_t* shard_counts) {
    if ((!bytes && nbytes) || (!line_off && n) || (!out_shard && n) || nranks == 0) return YSB_ERR_ARG;
    if (shard_counts) std::fill(shard_counts, shard_counts + nranks, 0ull);
    for (u64 i = 0; i < n; ++i) {
        const u64 s = line_off[i];
        const u64 e = i + 1 < n ? (u64)line_off[i + 1] : nbytes;
        u32 r = 0;
        long vs, ve;
        bool esc;
        if (s <= e && e <= nbytes && find_ad_id(bytes + s, (long)(e - s), &vs, &ve, &esc)) {
            if (!esc) {
                r = ysb_ad_shard(reinterpret_cast<const char*>(bytes + s + vs), (u32)(ve - vs), nranks);
            } else {   // the decoded key, as the device hashes it
                const std::string k = decode_escapes(bytes + s, vs, ve);
                r = ysb_ad_shard(k.data(), (u32)k.size(), nranks);
            }
        }
        out_shard[i] = r;
        if (shard_counts) shard_counts[r]++;
    }
    return YSB_OK;
}

int ysb_json_to_tbl(const uint8_t* bytes, uint64_t nbytes, const uint32_t* line_off, uint64_t n, uint8_t* out,
                    uint64_t cap, uint32_t* out_off, uint64_t* out_nbytes) {
    if ((!bytes && nbytes) || (!line_off && n) || (n && (!out || !out_off)) || !out_nbytes) return YSB_ERR_ARG;
    static const char* const keys[7] = {"user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time",
                                        "ip_address"};
    u64 o = 0;
    for (u64 i = 0; i < n; ++i) {
        const u64 s = line_off[i];
        const u64 e = i + 1 < n ? (u64)line_off[i + 1] : nbytes;
        if (s > e || e > nbytes) return YSB_ERR_FORMAT;
        // the quoted strings of the line: key, value, key, value, ...
        long q[14][2];
        int k = 0;
        for (u64 p = s; p < e; ++p) {
            if (bytes[p] == '\\') return YSB_ERR_FORMAT;
            if (bytes[p] != '"') continue;
            u64 t = p + 1;
            while (t < e && bytes[t] != '"' && bytes[t] != '\\') ++t;
            if (t >= e || bytes[t] != '"' || k == 14) return YSB_ERR_FORMAT;
            q[k][0] = (long)(p + 1);
            q[k][1] = (long)t;
            ++k;
            p = t;
        }
        if (k != 14) return YSB_ERR_FORMAT;
        for (int f = 0; f < 7; ++f) {
            const size_t kl = std::strlen(keys[f]);
            if ((size_t)(q[2 * f][1] - q[2 * f][0]) != kl || std::memcmp(bytes + q[2 * f][0], keys[f], kl) != 0)
                return YSB_ERR_FORMAT;
        }
        if (o > 0xFFFFFFFFull) return YSB_ERR_CAPACITY;
        out_off[i] = (u32)o;
        for (int f = 0; f < 6; ++f) {   // items[0..5] (the .tbl rows carry no ip_address)
            const u64 len = (u64)(q[2 * f + 1][1] - q[2 * f + 1][0]);
            if (o + len + 1 > cap) return YSB_ERR_CAPACITY;
            std::memcpy(out + o, bytes + q[2 * f + 1][0], len);
            o += len;
            out[o++] = f < 5 ? '|' : '\n';
        }
    }
    *out_nbytes = o;
    return YSB_OK;
}

int ysb_gen_dump_shards(const ysb_gen_params* p, uint64_t n_events, const char* dir, uint32_t nranks) {
    if (!p || !dir || nranks == 0) return YSB_ERR_ARG;
    int rc = ysb_gen_dump(p, 0, dir);   // id files and both ad-map formats (no events)
    if (rc) return rc;
    std::remove((std::string(dir) + "/kafka-json.txt").c_str());
    std::vector<FILE*> f(nranks, nullptr);
    for (u32 r = 0; r < nranks; ++r) {
        const std::string path = std::string(dir) + "/kafka-json." + std::to_string(r) + ".txt";
        f[r] = std::fopen(path.c_str(), "wb");
        if (!f[r]) {
            for (FILE* x : f) if (x) std::fclose(x);
            return YSB_ERR_ARG;
        }
    }
    const u64 chunk = 1 << 16;
    const u64 cap = chunk * ysb_gen_max_line_bytes(p);
    std::vector<u8> buf(cap);
    std::vector<u32> off(chunk), shard(chunk);
    for (u64 first = 0; first < n_events && rc == YSB_OK; first += chunk) {
        const u64 m = std::min<u64>(chunk, n_events - first);
        uint64_t nb = 0;
        rc = ysb_gen_events_host(p, first, m, buf.data(), cap, off.data(), &nb);
        if (rc) break;
        rc = ysb_route_lines(buf.data(), nb, off.data(), m, nranks, shard.data(), nullptr);
        for (u64 i = 0; i < m && rc == YSB_OK; ++i) {
            const u64 e = i + 1 < m ? (u64)off[i + 1] : nb;
            std::fwrite(buf.data() + off[i], 1, e - off[i], f[shard[i]]);
        }
    }
    for (FILE* x : f) std::fclose(x);
    return rc;
}

}  // extern "C"
