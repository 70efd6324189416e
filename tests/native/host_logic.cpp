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
    // bucket-layout cuckoo table: every placed key is found by the probe's rule, a key in
    // its second bucket only while its first is full, and absent keys are not found
    for (u64 nb : {16384ull, 8192ull}) {   // load 41 % and 81 % of the entries
        const u64 n = 20000;
        std::vector<u32> keys(n * CKEY_WORDS), camp(n), ct(nb * CB_WORDS);
        std::mt19937_64 kr(nb);
        for (auto& w : keys) w = (u32)kr();
        for (u64 i = 0; i < n; ++i) camp[i] = (u32)(i % 1000);
        const CuckooSeed cs = cuckoo_seed(77 + nb);
        const u64 homeless = cuckoo_build_buckets(keys.data(), camp.data(), n, cs, nb, 99, true, ct.data());
        CHECK(homeless == 0);
        u64 second = 0;
        for (u64 i = 0; i < n; ++i) {
            const u32* k = &keys[i * CKEY_WORDS];
            CHECK(cuckoo_lookup_buckets(ct.data(), nb, cs, k) == camp[i]);
            u32 a, b;
            cuckoo_slots36(k, cs, (u32)(nb - 1), &a, &b);
            bool in_a = false, a_full = true;
            for (u32 e = 0; e < CB_ENTRIES; ++e) {
                const u32* en = &ct[(u64)a * CB_WORDS + e * CB_STRIDE];
                if (en[CKEY_WORDS] == EMPTY_SLOT) a_full = false;
                else if (std::memcmp(en, k, 36) == 0) in_a = true;
            }
            if (!in_a) { CHECK(a_full); ++second; }
        }
        if (nb == 16384) CHECK(second < n / 20);
        for (int t = 0; t < 2000; ++t) {   // keys not in the table
            u32 k[CKEY_WORDS];
            for (auto& w : k) w = (u32)kr();
            CHECK(cuckoo_lookup_buckets(ct.data(), nb, cs, k) == EMPTY_SLOT);
        }
    }
    std::printf("%s\n", fails ? "FAILED" : "OK");
    return fails ? 1 : 0;
}
