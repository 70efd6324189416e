// ysb_gen_api.cpp -- the data/ generator (core.clj:61-98,163-204) behind the C ABI: ids,
// host and device event lines, the file-dump mode, and the generator-truth tables the
// tests and bench check counts against.
#include "ysb_ctx.h"

using namespace ysb;

extern "C" {

void ysb_gen_default(ysb_gen_params* p) {
    std::memset(p, 0, sizeof *p);
    p->seed = 42;
    p->n_campaigns = 100;
    p->ads_per_campaign = 10;
    p->t0_ms = 1700000000000LL;
    p->events_per_sec = 100000;
    p->with_skew = 0;
    p->n_users = 0;
}

static GenSpec spec_of(const ysb_gen_params* p, const u32* subset) {
    GenSpec s{};
    s.seed = p->seed;
    // stream 0 keeps the single-stream byte format of the committed fixtures
    s.ev_seed = p->event_stream ? mix64(p->seed ^ (0xD1B54A32D192ED03ULL * p->event_stream)) : p->seed;
    s.n_campaigns = p->n_campaigns;
    s.ads_per_campaign = p->ads_per_campaign;
    s.t0_ms = p->t0_ms;
    s.events_per_sec = p->events_per_sec;
    s.with_skew = p->with_skew;
    s.n_users = p->n_users;
    s.subset = subset;
    s.n_pick = subset ? p->n_ad_subset : p->n_campaigns * p->ads_per_campaign;
    s.tbl = p->format == YSB_GEN_TBL;
    s.variant = p->variant;
    return s;
}

static bool gen_ok(const ysb_gen_params* p) {
    // with_skew: 0 off, 1 the reference's skew and late events, 2 the skew only (any other value
    // would silently change the truth tables)
    return p && p->n_campaigns && p->ads_per_campaign && p->events_per_sec && p->format <= YSB_GEN_TBL &&
           p->with_skew <= 2 &&
           p->variant <= (YSB_GEN_RANDOM_IP | YSB_GEN_MORE_AD_TYPES | YSB_GEN_COMPACT | YSB_GEN_REORDER | YSB_GEN_MIXED |
                          YSB_GEN_MIXED_BLOCKS) &&
           (!p->ad_subset || p->n_ad_subset) && (u64)p->n_campaigns * p->ads_per_campaign < (1ull << 32);
}

int ysb_gen_ids(const ysb_gen_params* p, char* campaign_ids, char* ad_ids) {
    if (!gen_ok(p)) return fail(nullptr, YSB_ERR_ARG, "bad generator parameters");
    u64 hi, lo;
    if (campaign_ids)
        for (u32 c = 0; c < p->n_campaigns; ++c) {
            uuid_words(stream_key(p->seed, S_CAMPAIGN), c, &hi, &lo);
            uuid_format(hi, lo, campaign_ids + 36ull * c);
        }
    if (ad_ids)
        for (u64 a = 0; a < (u64)p->n_campaigns * p->ads_per_campaign; ++a) {
            uuid_words(stream_key(p->seed, S_AD), a, &hi, &lo);
            uuid_format(hi, lo, ad_ids + 36ull * a);
        }
    return YSB_OK;
}

uint64_t ysb_gen_max_line_bytes(const ysb_gen_params*) { return (u64)LINE_FIXED + 16 + 8 + 20 + 8; }

int ysb_gen_events_host(const ysb_gen_params* p, uint64_t first, uint64_t n, uint8_t* out, uint64_t cap,
                        uint32_t* line_off, uint64_t* nbytes) {
    if (!gen_ok(p) || (n && (!out || !line_off)) || !nbytes) return fail(nullptr, YSB_ERR_ARG, "bad generator arguments");
    const GenSpec s = spec_of(p, p->ad_subset);
    u64 o = 0;
    char line[320];
    for (u64 i = 0; i < n; ++i) {
        const GenEvent e = gen_event(s, first + i);
        const u32 len = gen_line_write(s, first + i, e, line);
        if (o + len > cap) return fail(nullptr, YSB_ERR_CAPACITY, "generator output exceeds %llu bytes", (unsigned long long)cap);
        if (o > 0xFFFFFFFFull) return fail(nullptr, YSB_ERR_CAPACITY, "batch exceeds 4 GiB (u32 offsets)");
        line_off[i] = (u32)o;
        std::memcpy(out + o, line, len);
        o += len;
    }
    *nbytes = o;
    return YSB_OK;
}

int ysb_gen_events_host_mt(const ysb_gen_params* p, uint64_t first, uint64_t n, uint8_t* out, uint64_t cap,
                           uint32_t* line_off, uint64_t* nbytes, uint32_t threads) {
    if (!gen_ok(p) || (n && (!out || !line_off)) || !nbytes) return fail(nullptr, YSB_ERR_ARG, "bad generator arguments");
    const u32 T = (u32)std::max<u64>(1, std::min<u64>({(u64)std::max(threads, 1u), (u64)64, n / 4096 + 1}));
    if (T == 1) return ysb_gen_events_host(p, first, n, out, cap, line_off, nbytes);
    const GenSpec s = spec_of(p, p->ad_subset);
    // lengths (line_off as scratch) and per-thread sums, the bases, then the lines in place
    std::vector<u64> sum(T + 1, 0);
    auto span = [&](u32 t, u64* a, u64* b) { *a = n * t / T; *b = n * (t + 1) / T; };
    std::vector<std::thread> th;
    for (u32 t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            u64 a, b, acc = 0;
            span(t, &a, &b);
            for (u64 i = a; i < b; ++i) {
                const u32 l = gen_line_len(s, first + i, gen_event(s, first + i));
                line_off[i] = l;
                acc += l;
            }
            sum[t + 1] = acc;
        });
    for (auto& x : th) x.join();
    th.clear();
    for (u32 t = 0; t < T; ++t) sum[t + 1] += sum[t];
    if (sum[T] > cap) return fail(nullptr, YSB_ERR_CAPACITY, "generator output exceeds %llu bytes", (unsigned long long)cap);
    if (sum[T] > 0xFFFFFFFFull + 1) return fail(nullptr, YSB_ERR_CAPACITY, "batch exceeds 4 GiB (u32 offsets)");
    for (u32 t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            u64 a, b, o = sum[t];
            span(t, &a, &b);
            char line[320];
            for (u64 i = a; i < b; ++i) {
                const u32 len = gen_line_write(s, first + i, gen_event(s, first + i), line);
                line_off[i] = (u32)o;
                std::memcpy(out + o, line, len);
                o += len;
            }
        });
    for (auto& x : th) x.join();
    *nbytes = sum[T];
    return YSB_OK;
}

static int upload_subset(ysb_ctx* c, const ysb_gen_params* p, const u32** dptr) {
    *dptr = nullptr;
    if (!p->ad_subset) return YSB_OK;
    if (c->d_subset_n < p->n_ad_subset) {
        hipFree(c->d_subset);
        c->d_subset = nullptr;
        HIPCHK(c, hipMalloc(&c->d_subset, (u64)p->n_ad_subset * 4));
        c->d_subset_n = p->n_ad_subset;
    }
    HIPCHK(c, hipMemcpy(c->d_subset, p->ad_subset, (u64)p->n_ad_subset * 4, hipMemcpyHostToDevice));
    *dptr = c->d_subset;
    return YSB_OK;
}

int ysb_gen_events_device(ysb_ctx* c, const ysb_gen_params* p, uint64_t first, uint64_t n, uint8_t* d_out,
                          uint64_t cap, uint32_t* d_off, uint64_t* nbytes) {
    if (!c) return YSB_ERR_ARG;
    if (!gen_ok(p) || !nbytes || (n && (!d_out || !d_off))) return fail(c, YSB_ERR_ARG, "bad generator arguments");
    if (n > 0x7FFFFFFFull) return fail(c, YSB_ERR_ARG, "at most 2^31-1 events per call");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    const u32* dsub = nullptr;
    int rc = upload_subset(c, p, &dsub);
    if (rc) return rc;
    const GenSpec s = spec_of(p, dsub);
    const u64 cap32 = std::min<u64>(cap, 0xFFFFFFFFull);   // u32 line offsets
    hipError_t e = gen_events_device(s, first, n, d_out, cap32, d_off, nbytes, c->s_comp);
    if (e == hipErrorInvalidValue && *nbytes > cap32)
        return fail(c, YSB_ERR_CAPACITY, "generator output %llu B exceeds cap %llu B (u32 offsets: <= 4 GiB per batch)",
                    (unsigned long long)*nbytes, (unsigned long long)cap);
    if (e != hipSuccess) return fail(c, YSB_ERR_HIP, "device generator: %s", hipGetErrorString(e));
    return YSB_OK;
}

int ysb_truth_accumulate(ysb_ctx* c, const ysb_gen_params* p, uint64_t first, uint64_t n) {
    if (!c) return YSB_ERR_ARG;
    if (!gen_ok(p)) return fail(c, YSB_ERR_ARG, "bad generator parameters");
    if (p->n_campaigns > c->cfg.n_campaigns) return fail(c, YSB_ERR_ARG, "generator has more campaigns than the context");
    int prc = launch_pending_raw(c);
    if (prc) return prc;
    HIPCHK(c, hipSetDevice(c->device));
    const u64 cells = (u64)c->c_pad * c->cfg.window_ring;
    if (!c->d_truth) {
        HIPCHK(c, hipMalloc(&c->d_truth, cells * 8));
        HIPCHK(c, hipMemset(c->d_truth, 0, cells * 8));
        HIPCHK(c, hipMalloc(&c->d_truth_out, 8));
        HIPCHK(c, hipMemset(c->d_truth_out, 0, 8));
        if (!c->d_cmp) HIPCHK(c, hipMalloc(&c->d_cmp, 32));
    }
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    int rc = read_ring(c);
    if (rc) return rc;
    if (!c->ring_known) return fail(c, YSB_ERR_STATE, "ring base not set (submit a batch first or set ring_base_bucket)");
    const u32* dsub = nullptr;
    if ((rc = upload_subset(c, p, &dsub))) return rc;
    launch_truth(spec_of(p, dsub), first, n, c->div, c->d_truth, c->cfg.window_ring, c->d_ring, c->d_truth_out, c->s_comp);
    HIPCHK(c, hipGetLastError());
    return YSB_OK;
}

int ysb_truth_compare(ysb_ctx* c, uint64_t* mismatched, uint64_t* truth_total, uint64_t* ring_total) {
    if (!c) return YSB_ERR_ARG;
    if (!c->d_truth) return fail(c, YSB_ERR_STATE, "no truth accumulated");
    HIPCHK(c, hipSetDevice(c->device));
    int frc = launch_pending_raw(c);
    if (!frc) frc = fold_delta(c);
    if (frc) return frc;
    HIPCHK(c, hipMemsetAsync(c->d_cmp, 0, 32, c->s_comp));
    launch_compare(c->d_truth, c->d_counts, (u64)c->c_pad * c->cfg.window_ring, c->d_cmp, c->s_comp);
    unsigned long long r[3], outside = 0;
    HIPCHK(c, hipMemcpyAsync(r, c->d_cmp, 24, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipMemcpyAsync(&outside, c->d_truth_out, 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (mismatched) *mismatched = r[0];
    if (truth_total) *truth_total = r[1] + outside;
    if (ring_total) *ring_total = r[2];
    return YSB_OK;
}

int ysb_truth_read(ysb_ctx* c, uint64_t* out, uint64_t cells, int64_t* ring_lo) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    if (!c->d_truth) return fail(c, YSB_ERR_STATE, "no truth accumulated");
    const u64 need = (u64)c->cfg.n_campaigns * c->cfg.window_ring;
    if (cells < need) return fail(c, YSB_ERR_CAPACITY, "truth table needs %llu cells", (unsigned long long)need);
    int rc = sync_streams(c);
    if (rc) return rc;
    if ((rc = read_ring(c))) return rc;
    HIPCHK(c, hipMemcpy(out, c->d_truth, need * 8, hipMemcpyDeviceToHost));
    if (ring_lo) *ring_lo = c->ring_lo;
    return YSB_OK;
}

int ysb_gen_dump(const ysb_gen_params* p, uint64_t n_events, const char* dir) {
    if (!gen_ok(p) || !dir) return fail(nullptr, YSB_ERR_ARG, "bad generator arguments");
    const u64 A = (u64)p->n_campaigns * p->ads_per_campaign;
    std::vector<char> cids(36ull * p->n_campaigns), aids(36ull * A);
    int rc = ysb_gen_ids(p, cids.data(), aids.data());
    if (rc) return rc;
    auto open = [&](const char* name) {
        std::string path = std::string(dir) + "/" + name;
        return std::fopen(path.c_str(), "wb");
    };
    FILE* f = open("campaign-ids.txt");
    if (!f) return fail(nullptr, YSB_ERR_ARG, "cannot write into %s", dir);
    for (u32 c = 0; c < p->n_campaigns; ++c) std::fprintf(f, "%.36s\n", &cids[36ull * c]);
    std::fclose(f);
    f = open("ad-ids.txt");
    if (!f) return fail(nullptr, YSB_ERR_ARG, "cannot write into %s", dir);
    for (u64 a = 0; a < A; ++a) std::fprintf(f, "%.36s\n", &aids[36ull * a]);
    std::fclose(f);
    f = open("ad-to-campaign-ids.txt");   // core.clj:58
    FILE* g = open("ad-to-campaign.csv");   // AdvertisingTopologyNative.java:52
    if (!f || !g) return fail(nullptr, YSB_ERR_ARG, "cannot write into %s", dir);
    for (u64 a = 0; a < A; ++a) {
        const u64 cc = a / p->ads_per_campaign;
        std::fprintf(f, "{ \"%.36s\": \"%.36s\"}\n", &aids[36 * a], &cids[36 * cc]);
        std::fprintf(g, "%.36s,%.36s\n", &aids[36 * a], &cids[36 * cc]);
    }
    std::fclose(f);
    std::fclose(g);
    f = open(p->format == YSB_GEN_TBL ? "events.tbl" : "kafka-json.txt");   // core.clj:76-97 / conf :6
    if (!f) return fail(nullptr, YSB_ERR_ARG, "cannot write into %s", dir);
    const GenSpec s = spec_of(p, p->ad_subset);
    std::vector<char> buf(1 << 22);
    size_t used = 0;
    for (u64 i = 0; i < n_events; ++i) {
        if (used + 320 > buf.size()) { std::fwrite(buf.data(), 1, used, f); used = 0; }
        used += gen_line_write(s, i, gen_event(s, i), buf.data() + used);
    }
    std::fwrite(buf.data(), 1, used, f);
    std::fclose(f);
    return YSB_OK;
}

}  // extern "C"
