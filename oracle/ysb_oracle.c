/*
 * ysb_oracle.c -- CPU restatement of the YSB advertising hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / the timed CPU port; the product
 * (streaming-benchmarks_amd/) never links or calls it.
 *
 * Parity status: UNPINNED against the reference itself.  The reference is
 * Java/Clojure (no JDK, Leiningen or network here) and holds no golden vectors
 * (data/test/setup/core_test.clj:8-10 is a placeholder that always fails), so
 * this file is pinned by (a) an independent second restatement built on Python's
 * json module (oracle/dostats.py) over the committed fixtures in tests/golden/,
 * and (b) hand-derived known answers from the reference's arithmetic.
 *
 * What it restates, line by line:
 *   DeserializeBolt.flatMap   new JSONObject(line); getString x6
 *                             flink-benchmarks/.../AdvertisingTopologyNative.java:257-276
 *                             (org.json 20180813: duplicate keys throw; getString on a
 *                             non-string throws)
 *   EventFilterBolt.filter    event_type.equals("view")                  :430-436
 *   project(ad_id, event_time)  storm-benchmarks/.../AdvertisingTopology.java:103-107
 *   RedisJoinBolt.flatMap     ad_campaign.get(ad_id); null -> drop        :461-474
 *   CampaignProcessorCommon.execute
 *                             Long.parseLong(event_time) / 10000L; seenCount++
 *                             streaming-benchmark-common/.../CampaignProcessorCommon.java:57-67
 *   dostats                   campaign -> bucket -> count                 data/src/setup/core.clj:101-128
 *   MockWindowedFlatMap       .tbl rows: line.split("\\|")                   :197-226 (oracle_run_fmt)
 *
 * JSON contract (shared with the GPU path, see DESIGN.md "Parity contract"):
 * RFC 8259 objects; raw control characters inside strings are accepted
 * (json.loads(strict=False)); org.json leniencies (single quotes, unquoted
 * strings, trailing commas, '=' / ';' separators) are rejected.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t events, views, joined, join_misses, parse_errors, time_errors; } oracle_stats;
typedef struct { uint32_t campaign; uint32_t pad; int64_t bucket; uint64_t count; } oracle_row;

/* ---------------- ad_id -> campaign map (java.util.HashMap<String,String>) ---------------- */
typedef struct { char* key; uint32_t len; uint32_t campaign; } ad_entry;
typedef struct { ad_entry* e; uint64_t cap, n; } ad_map;

static uint64_t fnv1a(const unsigned char* s, uint32_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (uint32_t i = 0; i < n; ++i) { h ^= s[i]; h *= 1099511628211ULL; }
    return h;
}

void* oracle_admap_new(void) {
    ad_map* m = (ad_map*)calloc(1, sizeof *m);
    m->cap = 1024;
    m->e = (ad_entry*)calloc(m->cap, sizeof(ad_entry));
    return m;
}

static void admap_insert(ad_map* m, char* key, uint32_t len, uint32_t campaign) {
    uint64_t i = fnv1a((const unsigned char*)key, len) & (m->cap - 1);
    for (;; i = (i + 1) & (m->cap - 1)) {
        ad_entry* x = &m->e[i];
        if (!x->key) { x->key = key; x->len = len; x->campaign = campaign; m->n++; return; }
        if (x->len == len && memcmp(x->key, key, len) == 0) { x->campaign = campaign; free(key); return; } /* put: later wins */
    }
}

int oracle_admap_put(void* mp, const char* key, uint32_t len, uint32_t campaign) {
    ad_map* m = (ad_map*)mp;
    if (2 * (m->n + 1) > m->cap) {
        ad_entry* old = m->e;
        uint64_t oc = m->cap;
        m->cap *= 2;
        m->e = (ad_entry*)calloc(m->cap, sizeof(ad_entry));
        m->n = 0;
        for (uint64_t i = 0; i < oc; ++i)
            if (old[i].key) admap_insert(m, old[i].key, old[i].len, old[i].campaign);
        free(old);
    }
    char* k = (char*)malloc(len ? len : 1);
    memcpy(k, key, len);
    admap_insert(m, k, len, campaign);
    return 0;
}

static int admap_get(const ad_map* m, const unsigned char* key, uint32_t len, uint32_t* campaign) {
    uint64_t i = fnv1a(key, len) & (m->cap - 1);
    for (;; i = (i + 1) & (m->cap - 1)) {
        const ad_entry* x = &m->e[i];
        if (!x->key) return 0;
        if (x->len == len && memcmp(x->key, key, len) == 0) { *campaign = x->campaign; return 1; }
    }
}

void oracle_admap_free(void* mp) {
    ad_map* m = (ad_map*)mp;
    if (!m) return;
    for (uint64_t i = 0; i < m->cap; ++i) free(m->e[i].key);
    free(m->e);
    free(m);
}

/* ---------------- a strict JSON reader for one line ---------------- */
typedef struct {
    const unsigned char* s;
    size_t n, p;
} rd;

static int ws(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
static void skipws(rd* r) { while (r->p < r->n && ws(r->s[r->p])) r->p++; }
static int hexv(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

/* Reads a string at r->p (which is '"'); decodes into out (cap bytes kept),
 * returns decoded length or -1.  Decoding to UTF-8 mirrors Java's String equality
 * of the decoded value. */
static long read_string(rd* r, unsigned char* out, size_t cap) {
    size_t n = 0;
    r->p++;
#define PUT(ch) do { if (n < cap) out[n] = (unsigned char)(ch); n++; } while (0)
    while (r->p < r->n) {
        int c = r->s[r->p];
        if (c == '"') { r->p++; return (long)n; }
        if (c != '\\') { PUT(c); r->p++; continue; }
        if (r->p + 1 >= r->n) return -1;
        int x = r->s[r->p + 1];
        switch (x) {
            case '"': PUT('"'); r->p += 2; break;
            case '\\': PUT('\\'); r->p += 2; break;
            case '/': PUT('/'); r->p += 2; break;
            case 'b': PUT(8); r->p += 2; break;
            case 'f': PUT(12); r->p += 2; break;
            case 'n': PUT(10); r->p += 2; break;
            case 'r': PUT(13); r->p += 2; break;
            case 't': PUT(9); r->p += 2; break;
            case 'u': {
                if (r->p + 5 >= r->n) return -1;
                unsigned cp = 0;
                for (int k = 2; k < 6; ++k) {
                    int h = hexv(r->s[r->p + k]);
                    if (h < 0) return -1;
                    cp = cp * 16 + (unsigned)h;
                }
                r->p += 6;
                if (cp >= 0xD800 && cp < 0xDC00 && r->p + 5 < r->n && r->s[r->p] == '\\' && r->s[r->p + 1] == 'u') {
                    unsigned lo = 0;
                    int ok = 1;
                    for (int k = 2; k < 6; ++k) {
                        int h = hexv(r->s[r->p + k]);
                        if (h < 0) { ok = 0; break; }
                        lo = lo * 16 + (unsigned)h;
                    }
                    if (ok && lo >= 0xDC00 && lo < 0xE000) {
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        r->p += 6;
                    }
                }
                if (cp < 0x80) PUT(cp);
                else if (cp < 0x800) { PUT(0xC0 | (cp >> 6)); PUT(0x80 | (cp & 0x3F)); }
                else if (cp < 0x10000) { PUT(0xE0 | (cp >> 12)); PUT(0x80 | ((cp >> 6) & 0x3F)); PUT(0x80 | (cp & 0x3F)); }
                else { PUT(0xF0 | (cp >> 18)); PUT(0x80 | ((cp >> 12) & 0x3F)); PUT(0x80 | ((cp >> 6) & 0x3F)); PUT(0x80 | (cp & 0x3F)); }
                break;
            }
            default: return -1;
        }
    }
#undef PUT
    return -1;
}

static int read_value(rd* r, int depth);

static int read_number(rd* r) {
    size_t p = r->p;
    if (p < r->n && r->s[p] == '-') p++;
    if (p >= r->n) return 0;
    if (r->s[p] == '0') p++;
    else if (r->s[p] >= '1' && r->s[p] <= '9') { while (p < r->n && r->s[p] >= '0' && r->s[p] <= '9') p++; }
    else return 0;
    if (p < r->n && r->s[p] == '.') {
        size_t q = ++p;
        while (p < r->n && r->s[p] >= '0' && r->s[p] <= '9') p++;
        if (p == q) return 0;
    }
    if (p < r->n && (r->s[p] == 'e' || r->s[p] == 'E')) {
        p++;
        if (p < r->n && (r->s[p] == '+' || r->s[p] == '-')) p++;
        size_t q = p;
        while (p < r->n && r->s[p] >= '0' && r->s[p] <= '9') p++;
        if (p == q) return 0;
    }
    r->p = p;
    return 1;
}

static int read_lit(rd* r, const char* w) {
    size_t k = strlen(w);
    if (r->p + k > r->n || memcmp(r->s + r->p, w, k) != 0) return 0;
    r->p += k;
    return 1;
}

static int read_container(rd* r, int depth, int obj) {
    if (depth > 64) return 0;
    r->p++;
    skipws(r);
    int close = obj ? '}' : ']';
    if (r->p < r->n && r->s[r->p] == close) { r->p++; return 1; }
    for (;;) {
        skipws(r);
        if (obj) {
            if (r->p >= r->n || r->s[r->p] != '"') return 0;
            unsigned char tmp[1];
            if (read_string(r, tmp, 0) < 0) return 0;
            skipws(r);
            if (r->p >= r->n || r->s[r->p] != ':') return 0;
            r->p++;
            skipws(r);
        }
        if (!read_value(r, depth + 1)) return 0;
        skipws(r);
        if (r->p >= r->n) return 0;
        if (r->s[r->p] == ',') { r->p++; continue; }
        if (r->s[r->p] == close) { r->p++; return 1; }
        return 0;
    }
}

static int read_value(rd* r, int depth) {
    if (r->p >= r->n) return 0;
    int c = r->s[r->p];
    if (c == '"') { unsigned char tmp[1]; return read_string(r, tmp, 0) >= 0; }
    if (c == '{') return read_container(r, depth, 1);
    if (c == '[') return read_container(r, depth, 0);
    if (c == 't') return read_lit(r, "true");
    if (c == 'f') return read_lit(r, "false");
    if (c == 'n') return read_lit(r, "null");
    return read_number(r);
}

/* The fields DeserializeBolt reads (AdvertisingTopologyNative.java:267-272) and,
 * for the Storm/Spark deserializers, ip_address (AdvertisingTopology.java:62). */
static const char* const KEYS[7] = {"user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time", "ip_address"};

typedef struct {
    unsigned char ad[64]; long ad_len;
    unsigned char et[16]; long et_len;
    unsigned char tm[256]; long tm_len;
} fields;

/* 1 = parsed; 0 = org.json would have thrown */
static int parse_event(const unsigned char* s, size_t n, unsigned require, fields* f) {
    rd r = {s, n, 0};
    unsigned seen = 0;
    skipws(&r);
    if (r.p >= r.n || s[r.p] != '{') return 0;
    r.p++;
    skipws(&r);
    if (r.p < r.n && s[r.p] == '}') {
        r.p++;
    } else {
        for (;;) {
            skipws(&r);
            if (r.p >= r.n || s[r.p] != '"') return 0;
            unsigned char key[16];
            long kl = read_string(&r, key, sizeof key);
            if (kl < 0) return 0;
            int kid = -1;
            for (int k = 0; k < 7; ++k)
                if ((size_t)kl == strlen(KEYS[k]) && memcmp(key, KEYS[k], (size_t)kl) == 0) kid = k;
            skipws(&r);
            if (r.p >= r.n || s[r.p] != ':') return 0;
            r.p++;
            skipws(&r);
            if (r.p >= r.n) return 0;
            if (kid >= 0) {
                if (seen & (1u << kid)) return 0;   /* org.json: Duplicate key */
                seen |= 1u << kid;
            }
            if (s[r.p] == '"') {
                unsigned char scratch[1];
                long vl;
                if (kid == 2) { vl = read_string(&r, f->ad, sizeof f->ad); f->ad_len = vl; }
                else if (kid == 4) { vl = read_string(&r, f->et, sizeof f->et); f->et_len = vl; }
                else if (kid == 5) { vl = read_string(&r, f->tm, sizeof f->tm); f->tm_len = vl; }
                else vl = read_string(&r, scratch, 0);
                if (vl < 0) return 0;
            } else {
                if (kid >= 0 && (require & (1u << kid))) return 0;   /* getString: not a string */
                if (!read_value(&r, 1)) return 0;
            }
            skipws(&r);
            if (r.p >= r.n) return 0;
            if (s[r.p] == ',') { r.p++; continue; }
            if (s[r.p] == '}') { r.p++; break; }
            return 0;
        }
    }
    skipws(&r);
    if (r.p != r.n) return 0;
    return (seen & require) == require;
}

/* The fork's .tbl rows: MockWindowedFlatMap.flatMap (AdvertisingTopologyNative.java:
 * 197-226) -- items = line.split("\\|") (java.lang.String.split, limit 0: trailing empty
 * items dropped), items[0..5] = user_id, page_id, ad_id, ad_type, event_type, event_time;
 * fewer than 6 items throw (ArrayIndexOutOfBounds).  The line is the batch line minus
 * its "\n" / "\r\n" terminator (BufferedReader.readLine, :153-159).
 * 1 = parsed; 0 = the reference would have thrown. */
static void copy_field(const unsigned char* s, long a, long b, unsigned char* out, size_t cap, long* len) {
    *len = b - a;
    if ((size_t)(b - a) <= cap) memcpy(out, s + a, (size_t)(b - a));
}

static int parse_tbl(const unsigned char* s, size_t n, fields* f) {
    long e = (long)n;
    if (e > 0 && s[e - 1] == '\n') --e;
    if (e > 0 && s[e - 1] == '\r') --e;
    long bar[6];
    int k = 0;
    for (long i = 0; i < e && k < 6; ++i)
        if (s[i] == '|') bar[k++] = i;
    if (k < 5) return 0;
    if (k == 5) bar[5] = e;
    /* items[5] exists iff a non-'|' byte follows the fifth '|' */
    int tail = 0;
    for (long i = bar[4] + 1; i < e && !tail; ++i) tail = s[i] != '|';
    if (!tail) return 0;
    copy_field(s, bar[1] + 1, bar[2], f->ad, sizeof f->ad, &f->ad_len);
    copy_field(s, bar[3] + 1, bar[4], f->et, sizeof f->et, &f->et_len);
    copy_field(s, bar[4] + 1, bar[5], f->tm, sizeof f->tm, &f->tm_len);
    return 1;
}

/* Long.parseLong: [+-]?[0-9]+ in int64 range */
static int parse_long(const unsigned char* s, long n, int64_t* out) {
    if (n <= 0) return 0;
    long i = 0;
    int neg = 0;
    if (s[0] == '-') { neg = 1; i = 1; }
    else if (s[0] == '+') i = 1;
    if (i >= n) return 0;
    uint64_t acc = 0, lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
    for (; i < n; ++i) {
        if (s[i] < '0' || s[i] > '9') return 0;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (acc > (lim - d) / 10) return 0;
        acc = acc * 10 + d;
    }
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return 1;
}

/* ---------------- (campaign, bucket) -> count ---------------- */
typedef struct { uint32_t used, campaign; int64_t bucket; uint64_t count; } cell;
typedef struct { cell* c; uint64_t cap, n; } count_map;

static uint64_t cell_hash(uint32_t c, int64_t b) {
    uint64_t z = ((uint64_t)c << 40) ^ (uint64_t)b;
    z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdULL;
    return z ^ (z >> 33);
}

static void cm_add(count_map* m, uint32_t c, int64_t b, uint64_t v) {
    if (2 * (m->n + 1) > m->cap) {
        cell* old = m->c;
        uint64_t oc = m->cap;
        m->cap = m->cap ? m->cap * 2 : 1024;
        m->c = (cell*)calloc(m->cap, sizeof(cell));
        m->n = 0;
        for (uint64_t i = 0; i < oc; ++i)
            if (old[i].used) cm_add(m, old[i].campaign, old[i].bucket, old[i].count);
        free(old);
    }
    uint64_t i = cell_hash(c, b) & (m->cap - 1);
    for (;; i = (i + 1) & (m->cap - 1)) {
        cell* x = &m->c[i];
        if (!x->used) { x->used = 1; x->campaign = c; x->bucket = b; x->count = v; m->n++; return; }
        if (x->campaign == c && x->bucket == b) { x->count += v; return; }
    }
}

typedef struct {
    const ad_map* m;
    const unsigned char* bytes;
    uint64_t nbytes;
    const uint32_t* off;
    uint64_t lo, hi, n;
    int64_t divisor;
    unsigned require;
    int tbl;                 /* 1: .tbl rows instead of JSON */
    count_map out;
    oracle_stats st;
} job;

static void* run_job(void* arg) {
    job* j = (job*)arg;
    fields f;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        uint64_t s = j->off[i], e = i + 1 < j->n ? j->off[i + 1] : j->nbytes;
        j->st.events++;
        if (e < s || e > j->nbytes) { j->st.parse_errors++; continue; }
        f.ad_len = f.et_len = f.tm_len = 0;
        const int ok = j->tbl ? parse_tbl(j->bytes + s, (size_t)(e - s), &f)
                              : parse_event(j->bytes + s, (size_t)(e - s), j->require, &f);
        if (!ok) { j->st.parse_errors++; continue; }
        if (!(f.et_len == 4 && memcmp(f.et, "view", 4) == 0)) continue;           /* EventFilterBolt */
        j->st.views++;
        uint32_t campaign;
        if (f.ad_len > (long)sizeof f.ad || !admap_get(j->m, f.ad, (uint32_t)f.ad_len, &campaign)) {
            j->st.join_misses++;                                                    /* RedisJoinBolt: drop */
            continue;
        }
        j->st.joined++;
        int64_t t;
        if (f.tm_len > (long)sizeof f.tm || !parse_long(f.tm, f.tm_len, &t)) { j->st.time_errors++; continue; }
        int64_t bucket = t / j->divisor;   /* C99 truncates toward zero, as Java's long / does */
        cm_add(&j->out, campaign, bucket, 1);
    }
    return NULL;
}

static int row_cmp(const void* a, const void* b) {
    const oracle_row* x = (const oracle_row*)a;
    const oracle_row* y = (const oracle_row*)b;
    if (x->campaign != y->campaign) return x->campaign < y->campaign ? -1 : 1;
    if (x->bucket != y->bucket) return x->bucket < y->bucket ? -1 : 1;
    return 0;
}

/* Runs the chain over n lines ([off[i], off[i+1]) / last ends at nbytes) with
 * `threads` workers (contiguous line ranges).  Rows are sorted by
 * (campaign, bucket).  Returns 0 on success. */
int oracle_run_fmt(const void* admap, const uint8_t* bytes, uint64_t nbytes, const uint32_t* off, uint64_t n,
                   int64_t divisor, int require_ip, int tbl, int threads, oracle_row** rows_out, uint64_t* nrows,
                   oracle_stats* st);

int oracle_run(const void* admap, const uint8_t* bytes, uint64_t nbytes, const uint32_t* off, uint64_t n,
               int64_t divisor, int require_ip, int threads, oracle_row** rows_out, uint64_t* nrows,
               oracle_stats* st) {
    return oracle_run_fmt(admap, bytes, nbytes, off, n, divisor, require_ip, 0, threads, rows_out, nrows, st);
}

/* Same, tbl = 1 for the fork's .tbl rows. */
int oracle_run_fmt(const void* admap, const uint8_t* bytes, uint64_t nbytes, const uint32_t* off, uint64_t n,
                   int64_t divisor, int require_ip, int tbl, int threads, oracle_row** rows_out, uint64_t* nrows,
                   oracle_stats* st) {
    if (divisor < 1 || threads < 1) return -1;
    if ((uint64_t)threads > n && n) threads = (int)n;
    if (n == 0) threads = 1;
    job* jobs = (job*)calloc((size_t)threads, sizeof(job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        jobs[t].m = (const ad_map*)admap;
        jobs[t].bytes = bytes;
        jobs[t].nbytes = nbytes;
        jobs[t].off = off;
        jobs[t].n = n;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].divisor = divisor;
        jobs[t].require = require_ip ? 0x7Fu : 0x3Fu;
        jobs[t].tbl = tbl;
        if (threads > 1) pthread_create(&th[t], NULL, run_job, &jobs[t]);
        else run_job(&jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    count_map all = {0, 0, 0};
    memset(st, 0, sizeof *st);
    for (int t = 0; t < threads; ++t) {
        for (uint64_t i = 0; i < jobs[t].out.cap; ++i)
            if (jobs[t].out.c[i].used) cm_add(&all, jobs[t].out.c[i].campaign, jobs[t].out.c[i].bucket, jobs[t].out.c[i].count);
        free(jobs[t].out.c);
        st->events += jobs[t].st.events;
        st->views += jobs[t].st.views;
        st->joined += jobs[t].st.joined;
        st->join_misses += jobs[t].st.join_misses;
        st->parse_errors += jobs[t].st.parse_errors;
        st->time_errors += jobs[t].st.time_errors;
    }
    oracle_row* rows = (oracle_row*)malloc((all.n ? all.n : 1) * sizeof(oracle_row));
    uint64_t k = 0;
    for (uint64_t i = 0; i < all.cap; ++i)
        if (all.c[i].used) {
            rows[k].campaign = all.c[i].campaign;
            rows[k].pad = 0;
            rows[k].bucket = all.c[i].bucket;
            rows[k].count = all.c[i].count;
            ++k;
        }
    free(all.c);
    qsort(rows, k, sizeof(oracle_row), row_cmp);
    *rows_out = rows;
    *nrows = k;
    free(jobs);
    free(th);
    return 0;
}

void oracle_free_rows(oracle_row* r) { free(r); }
