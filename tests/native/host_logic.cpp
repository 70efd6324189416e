// Host-side checks of the arithmetic shared with the device (ysb_common.h):
// exact Java long division by a runtime divisor, and the ad-table hash.
// Built and run by tests/test_capi.py with g++ (no GPU).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "ysb_common.h"

using namespace ysb;

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

int main() {
    const i64 divisors[] = {1, 2, 3, 7, 10, 1000, 9999, 10000, 10001, 60000, 86400000, 1LL << 40,
                            (1LL << 62) + 12345, INT64_MAX};
    std::mt19937_64 rng(1234);
    for (i64 d : divisors) {
        DivMagic m = div_magic(d);
        const i64 edge[] = {0, 1, -1, d - 1, d, d + 1, -d + 1, -d, -d - 1, INT64_MAX, INT64_MIN, INT64_MIN + 1,
                            1700000000000LL, -1700000000000LL, 1700000009999LL};
        for (i64 t : edge) CHECK(div_trunc(t, m) == t / d);
        for (int k = 0; k < 200000; ++k) {
            i64 t = (i64)rng();
            if (k & 1) t >>= (k % 60);
            CHECK(div_trunc(t, m) == t / d);
        }
    }
    // key hash: zero padding beyond len must not matter
    u32 a[KEY_WORDS] = {0}, b[KEY_WORDS];
    std::memcpy(a, "0f8c1e7a-1111-4222-8333-944455556666", 36);
    std::memcpy(b, a, sizeof a);
    CHECK(key_hash(a, 36) == key_hash(b, 36));
    CHECK(key_hash(a, 36) != key_hash(a, 35));
    // generator line length == bytes written
    GenSpec s{};
    s.seed = 5; s.n_campaigns = 100; s.ads_per_campaign = 10; s.t0_ms = -123456789; s.events_per_sec = 3;
    s.n_pick = 1000;
    char line[400];
    for (u32 tbl = 0; tbl < 2; ++tbl) {   // JSON lines and .tbl rows, every layout variant
        for (u32 v = 0; v < 8; ++v) {
            s.tbl = tbl;
            s.variant = v;
            for (u64 i = 0; i < 5000; ++i) {
                GenEvent e = gen_event(s, i);
                CHECK(gen_line_len(s, i, e) == gen_line_write(s, i, e, line));
            }
        }
    }
    // uuid_pack: canonical lower-case UUID strings pack injectively into 128 bits; every
    // other 36 bytes (upper-case hex, a non-hex byte, a misplaced dash) is rejected
    {
        std::mt19937_64 ur(4242);
        std::vector<std::vector<u32>> seen;
        for (int t = 0; t < 20000; ++t) {
            char str[37];
            uuid_format(ur(), ur(), str);
            u32 w[9], k[4];
            std::memcpy(w, str, 36);
            CHECK(uuid_pack(w, k));
            // unpack by hand: the nibbles in uuid_pack's bit order give the string back
            const u32 f0 = k[0] & 0xFFFF, f1 = k[0] >> 16, f6 = k[1] & 0xFFFF, f7 = k[1] >> 16, f8 = k[2] & 0xFFFF;
            const u32 g2 = (k[2] >> 16) & 0xFFF, g3 = (k[2] >> 28) | ((k[3] & 0xFF) << 4), g4 = (k[3] >> 8) & 0xFFF,
                      g5 = k[3] >> 20;
            auto hx = [](u32 v) { return (char)(v < 10 ? '0' + v : 'a' + v - 10); };
            char back[37];
            const u32 f[4] = {f0, f1, 0, 0};
            for (int i = 0; i < 8; ++i) back[i] = hx((f[i / 4] >> (4 * (i % 4))) & 0xF);
            back[8] = '-';
            for (int i = 0; i < 3; ++i) back[9 + i] = hx((g2 >> (4 * i)) & 0xF);
            back[12] = hx(g3 & 0xF); back[13] = '-'; back[14] = hx((g3 >> 4) & 0xF); back[15] = hx(g3 >> 8);
            back[16] = hx(g4 & 0xF); back[17] = hx((g4 >> 4) & 0xF); back[18] = '-'; back[19] = hx(g4 >> 8);
            for (int i = 0; i < 3; ++i) back[20 + i] = hx((g5 >> (4 * i)) & 0xF);
            back[23] = '-';
            const u32 ff[3] = {f6, f7, f8};
            for (int i = 0; i < 12; ++i) back[24 + i] = hx((ff[i / 4] >> (4 * (i % 4))) & 0xF);
            CHECK(std::memcmp(back, str, 36) == 0);
            // any single-byte change is rejected or packs differently
            for (int pos = 0; pos < 36; pos += 5) {
                char m[37];
                std::memcpy(m, str, 37);
                const char subs[] = {'A', 'g', '-', 'F', '0', ' ', 'a'};
                m[pos] = subs[(t + pos) % 7];
                if (m[pos] == str[pos]) continue;
                u32 w2[9], k2[4];
                std::memcpy(w2, m, 36);
                if (uuid_pack(w2, k2)) CHECK(std::memcmp(k, k2, 16) != 0);
            }
        }
        u32 w[9], k[4];
        std::memcpy(w, "0F8C1E7A-1111-4222-8333-944455556666", 36);
        CHECK(!uuid_pack(w, k));
        std::memcpy(w, "0f8c1e7a11111-4222-8333-944455556666", 36);
        CHECK(!uuid_pack(w, k));
        std::memcpy(w, "0f8c1e7a-1111-4222-8333-94445555666g", 36);
        CHECK(!uuid_pack(w, k));
        std::memcpy(w, "0f8c1e7a-1111-4222-8333-944455556666", 36);
        CHECK(uuid_pack(w, k));
    }
    // bucket-layout cuckoo table: every placed key is found by the probe's rule, a key in
    // its second bucket only while its first is full, and absent keys are not found
    for (u64 nb : {16384ull, 8192ull}) {   // load 41 % and 81 % of the entries
        const u64 n = 20000;
        std::vector<u32> keys(n * CB_KEYW), camp(n), ct(nb * CB_WORDS);
        std::mt19937_64 kr(nb);
        for (auto& w : keys) w = (u32)kr();
        for (u64 i = 0; i < n; ++i) camp[i] = (u32)(i % 1000);
        const CuckooSeed cs = cuckoo_seed(77 + nb);
        const u64 homeless = cuckoo_build_buckets(keys.data(), camp.data(), n, cs, nb, 99, true, ct.data());
        CHECK(homeless == 0);
        u64 second = 0;
        for (u64 i = 0; i < n; ++i) {
            const u32* k = &keys[i * CB_KEYW];
            CHECK(cuckoo_lookup_buckets(ct.data(), nb, cs, k) == camp[i]);
            u32 a, b;
            cuckoo_slots_k4(k, cs, (u32)(nb - 1), &a, &b);
            bool in_a = false, a_full = true;
            for (u32 e = 0; e < CB_ENTRIES; ++e) {
                const u32* en = &ct[(u64)a * CB_WORDS + e * CB_STRIDE];
                if (en[CB_KEYW] == EMPTY_SLOT) a_full = false;
                else if (std::memcmp(en, k, 4 * CB_KEYW) == 0) in_a = true;
            }
            if (!in_a) { CHECK(a_full); ++second; }
        }
        if (nb == 16384) CHECK(second < n / 20);
        for (int t = 0; t < 2000; ++t) {   // keys not in the table
            u32 k[CB_KEYW];
            for (auto& w : k) w = (u32)kr();
            CHECK(cuckoo_lookup_buckets(ct.data(), nb, cs, k) == EMPTY_SLOT);
        }
    }
    std::printf("%s\n", fails ? "FAILED" : "OK");
    return fails ? 1 : 0;
}
