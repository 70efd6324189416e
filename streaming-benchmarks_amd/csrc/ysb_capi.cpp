// ysb_capi.cpp -- the C ABI of include/ysb_hip.h: context lifecycle, the device ad ->
// campaign tables, sync / drain / ring / stats, measurement getters and device memory helpers.
// Batches are in ysb_submit.cpp, the multi-GPU group in ysb_group.cpp, the generator in
// ysb_gen_api.cpp (all over the context of ysb_ctx.h).
#include "ysb_ctx.h"

#include <unistd.h>

#include <cctype>

using namespace ysb;

thread_local std::string g_open_err;

int fail(ysb_ctx* c, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    else g_open_err = buf;
    return code;
}

extern "C" {

int ysb_abi_version(void) { return YSB_ABI_VERSION; }

int ysb_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

// Why this process's HIP runtime sees no device: the likely cause named (Weak 6 of the round-5
// review: torch 2.10 bundles its own libamdhip64 / libhsa-runtime64, and whichever runtime
// opens the GPU first in a process is the one that sees it).
static int no_device(hipError_t e) {
    const bool kfd = access("/dev/kfd", F_OK) == 0;
    const char* vis = getenv("HIP_VISIBLE_DEVICES");
    if (!vis) vis = getenv("ROCR_VISIBLE_DEVICES");
    if (kfd && !(vis && *vis == '\0'))
        return fail(nullptr, YSB_ERR_HIP,
                    "no HIP device available to this library's HIP runtime (hipGetDeviceCount: %s) although "
                    "/dev/kfd exists: another HIP/HSA runtime in this process (e.g. the libamdhip64 a framework "
                    "such as torch bundles) probably opened the GPU first -- load libysb_hip and call "
                    "ysb_device_count / ysb_open before any other GPU runtime initialises (INTEGRATION.md 1.4a)%s%s",
                    hipGetErrorString(e), vis ? "; *_VISIBLE_DEVICES=" : "", vis ? vis : "");
    return fail(nullptr, YSB_ERR_HIP, "no HIP device available (hipGetDeviceCount: %s%s)", hipGetErrorString(e),
                kfd ? "" : "; no /dev/kfd: no AMD GPU driver in this environment");
}

int ysb_device_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return -1;
    for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = std::fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node;
}

int ysb_device_sync(int device) {
    int ndev = 0;
    const hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return no_device(e);
    if (device < 0 || device >= ndev) return fail(nullptr, YSB_ERR_ARG, "device %d out of range (%d)", device, ndev);
    hipError_t r = hipSetDevice(device);
    if (r == hipSuccess) r = hipDeviceSynchronize();
    if (r != hipSuccess) return fail(nullptr, YSB_ERR_HIP, "hipDeviceSynchronize(%d): %s", device, hipGetErrorString(r));
    return YSB_OK;
}

void ysb_config_default(ysb_config* c) {
    std::memset(c, 0, sizeof *c);
    c->time_divisor_ms = 10000;
    c->n_campaigns = 100;
    c->window_ring = 1024;
    c->max_ads = 1000;
    c->max_batch_events = 1u << 20;
    c->max_batch_bytes = 256ull << 20;
    c->ring_base_bucket = INT64_MIN;
    c->overflow_capacity = 1u << 20;
    c->flags = 0;
}

const char* ysb_last_error(const ysb_ctx* c) { return c ? c->err.c_str() : g_open_err.c_str(); }

static void destroy(ysb_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->s_comp) hipStreamSynchronize(c->s_comp);
    if (c->s_copy) hipStreamSynchronize(c->s_copy);
    if (c->s_split) hipStreamSynchronize(c->s_split);
    if (c->s_x) hipStreamSynchronize(c->s_x);
    if (c->comm) ncclCommDestroy(c->comm);
    hipFree(c->d_table);
    hipFree(c->d_ctable);
    hipFree(c->d_counts);
    hipFree(c->d_owned);
    hipFree(c->d_owned8);
    hipFree(c->d_rs_tmp);
    hipFree(c->d_rows);
    hipFree(c->d_rows_n);
    hipFree(c->d_ring);
    hipHostFree(c->h_ring);
    hipFree(c->d_ovf);
    hipFree(c->d_ovf_count);
    hipFree(c->d_side);
    hipFree(c->d_stats);
    hipFree(c->d_truth);
    hipFree(c->d_truth_out);
    hipFree(c->d_cmp);
    hipFree(c->d_subset);
    hipFree(c->d_defer);
    hipFree(c->d_defer_ctr);
    hipFree(c->d_dbg);
    for (int s = 0; s < 2; ++s) {
        hipHostFree(c->h_bytes[s]);
        hipHostFree(c->h_off[s]);
        hipFree(c->d_bytes[s]);
        hipFree(c->d_off[s]);
        if (c->ev_h2d[s]) hipEventDestroy(c->ev_h2d[s]);
        if (c->ev_kdone[s]) hipEventDestroy(c->ev_kdone[s]);
    }
    for (auto& p : c->tev) for (hipEvent_t e : p) hipEventDestroy(e);
    hipFree(c->d_rec);
    hipFree(c->d_rec_n);
    hipFree(c->d_delta);
    hipFree(c->d_dirty);
    hipFree(c->d_xmax);
    hipHostFree(c->h_xmax);
    for (hipEvent_t e : c->xplan_ev)
        if (e) hipEventDestroy(e);
    hipFree(c->d_xslots);
    for (int k = 0; k < 2; ++k) {
        hipFree(c->d_xsend[k]);
        hipFree(c->d_xrecv[k]);
        if (c->ev_xpacked[k]) hipEventDestroy(c->ev_xpacked[k]);
        if (c->ev_xdone[k]) hipEventDestroy(c->ev_xdone[k]);
    }
    if (c->s_x) hipStreamDestroy(c->s_x);
    for (auto& p : c->xev) for (hipEvent_t e : p) hipEventDestroy(e);
    hipFree(c->d_part);
    hipFree(c->d_runs);
    if (c->ev_ring) hipEventDestroy(c->ev_ring);
    hipHostFree(c->h_sample);
    for (hipEvent_t e : c->ev_sample)
        if (e) hipEventDestroy(e);
    hipHostFree(c->h_used);
    if (c->ev_used) hipEventDestroy(c->ev_used);
    for (int s = 0; s < 2; ++s) {
        hipFree(c->d_roff[s]);
        if (c->ev_raw[s]) hipEventDestroy(c->ev_raw[s]);
    }
    hipFree(c->d_split_chunk);
    hipFree(c->d_rawn);
    hipHostFree(c->h_rawn);
    for (auto& p : c->cev) for (hipEvent_t e : p) hipEventDestroy(e);
    hipFree(c->d_rebase);
    for (auto& r : c->host_ranges) hipHostUnregister(reinterpret_cast<void*>(r.first));
    for (auto& f : c->fl) {
        hipHostFree(f.h_rows);
        hipHostFree(f.h_n);
        if (f.ev) hipEventDestroy(f.ev);
    }
    hipFree(c->d_fl_n);
    if (c->s_split) hipStreamDestroy(c->s_split);
    if (c->s_comp) hipStreamDestroy(c->s_comp);
    if (c->s_copy) hipStreamDestroy(c->s_copy);
    delete c;
}

static int alloc_counts(ysb_ctx* c) {
    const u64 cells = (u64)c->c_pad * c->cfg.window_ring;
    hipFree(c->d_counts);
    c->d_counts = nullptr;
    HIPCHK(c, hipMalloc(&c->d_counts, cells * 8));
    HIPCHK(c, hipMemset(c->d_counts, 0, cells * 8));
    return YSB_OK;
}

int ysb_open(ysb_ctx** out, int device, const ysb_config* cfg_in) {
    if (!out) return fail(nullptr, YSB_ERR_ARG, "out is NULL");
    *out = nullptr;
    ysb_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else ysb_config_default(&cfg);
    if (cfg.time_divisor_ms < 1) return fail(nullptr, YSB_ERR_ARG, "time_divisor_ms must be >= 1");
    if (cfg.n_campaigns == 0) return fail(nullptr, YSB_ERR_ARG, "n_campaigns must be > 0");
    if (!is_pow2(cfg.window_ring) || cfg.window_ring < 16)
        return fail(nullptr, YSB_ERR_ARG, "window_ring must be a power of two >= 16");
    if (cfg.max_batch_bytes == 0 || cfg.max_batch_bytes > (4ull << 30) - 64)
        return fail(nullptr, YSB_ERR_ARG, "max_batch_bytes must be in (0, 4 GiB)");
    if (cfg.overflow_capacity == 0 || cfg.overflow_capacity > 0xFFFFFFFFull)
        return fail(nullptr, YSB_ERR_ARG, "overflow_capacity must be in [1, 2^32)");
    int ndev = 0;
    const hipError_t de = hipGetDeviceCount(&ndev);
    if (de != hipSuccess || ndev == 0) return no_device(de);
    if (device < 0 || device >= ndev) return fail(nullptr, YSB_ERR_ARG, "device %d out of range (%d)", device, ndev);

    ysb_ctx* c = new ysb_ctx();
    c->device = device;
    c->cfg = cfg;
    c->c_pad = cfg.n_campaigns;
    c->div = div_magic(cfg.time_divisor_ms);
    int rc = YSB_OK;
    auto bad = [&](int code) { g_open_err = c->err; destroy(c); return code; };
    if (hipSetDevice(device) != hipSuccess) { fail(c, YSB_ERR_HIP, "hipSetDevice(%d) failed", device); return bad(YSB_ERR_HIP); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) c->cus = prop.multiProcessorCount;
    // scan schedule overrides (timing experiments): YSB_DYN_PCT=0 -> all static
    if (const char* e = getenv("YSB_DYN_PCT")) c->dyn_pct = (u32)strtoul(e, nullptr, 10);
    if (const char* e = getenv("YSB_DELTA_FOLD_EVENTS")) {
        const u64 v = strtoull(e, nullptr, 10);
        if (v > 0 && v < c->delta_limit) c->delta_limit = v;
    }
    if (const char* e = getenv("YSB_DYN_CHUNK")) c->dyn_chunk = (u32)strtoul(e, nullptr, 10);
    if (hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_copy, hipStreamNonBlocking) != hipSuccess) {
        fail(c, YSB_ERR_HIP, "stream creation failed");
        return bad(YSB_ERR_HIP);
    }
    for (int s = 0; s < 2; ++s) {
        if (hipEventCreateWithFlags(&c->ev_h2d[s], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_kdone[s], hipEventDisableTiming) != hipSuccess) {
            fail(c, YSB_ERR_HIP, "event creation failed");
            return bad(YSB_ERR_HIP);
        }
    }
    if (hipEventCreateWithFlags(&c->ev_ring, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_used, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&c->h_used, 16) != hipSuccess) {
        fail(c, YSB_ERR_HIP, "event creation failed");
        return bad(YSB_ERR_HIP);
    }
    if ((rc = alloc_counts(c)) != YSB_OK) return bad(rc);
    // out-of-ring map: load <= 1/2 at overflow_capacity distinct cells
    c->side_slots = 64;
    while (c->side_slots < 2 * cfg.overflow_capacity) c->side_slots <<= 1;
    c->side_cbits = 1;
    while (c->side_cbits < 32 && (1ull << c->side_cbits) <= cfg.n_campaigns) ++c->side_cbits;   // bit_width
    // stats and the map's slot count share one allocation: ysb_sync reads both in one copy
    if (hipMalloc(&c->d_side, c->side_slots * sizeof(SideSlot)) != hipSuccess ||
        hipMalloc(&c->d_stats, (ST_COUNT_ + 1) * 8) != hipSuccess ||
        hipMemset(c->d_stats, 0, (ST_COUNT_ + 1) * 8) != hipSuccess ||
        hipMalloc(&c->d_dirty, 16) != hipSuccess || hipMemset(c->d_dirty, 0, 16) != hipSuccess) {
        fail(c, YSB_ERR_NOMEM, "device allocation failed");
        return bad(YSB_ERR_NOMEM);
    }
    c->d_side_used = reinterpret_cast<u32*>(c->d_stats + ST_COUNT_);
    launch_side_clear(c->d_side, c->side_slots, c->s_comp);
    if (hipStreamSynchronize(c->s_comp) != hipSuccess) {
        fail(c, YSB_ERR_HIP, "side map initialisation failed");
        return bad(YSB_ERR_HIP);
    }
    if (hipMalloc(&c->d_ring, 16) != hipSuccess || hipHostMalloc(&c->h_ring, 16) != hipSuccess ||
        hipMalloc(&c->d_ovf, cfg.overflow_capacity * sizeof(OvfEntry)) != hipSuccess ||
        hipMalloc(&c->d_ovf_count, 16) != hipSuccess) {
        fail(c, YSB_ERR_NOMEM, "device allocation failed");
        return bad(YSB_ERR_NOMEM);
    }
    i64 ring[2] = {0, 0};
    if (cfg.ring_base_bucket != INT64_MIN) {
        ring[0] = cfg.ring_base_bucket;
        ring[1] = 1;
        c->ring_known = true;
        c->ring_lo = cfg.ring_base_bucket;
    }
    if (hipMemcpy(c->d_ring, ring, 16, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(c->d_ovf_count, 0, 16) != hipSuccess) {
        fail(c, YSB_ERR_HIP, "initialisation copy failed");
        return bad(YSB_ERR_HIP);
    }
    // LDS window counters: WL = largest power of two with n_campaigns * WL <= LCNT_CAP
    if (!(cfg.flags & YSB_F_NO_LDS_COUNT)) {
        u32 wl = 0;
        for (u32 w = 2; (u64)w * cfg.n_campaigns <= (u64)LCNT_CAP && w <= cfg.window_ring; w <<= 1) wl = w;
        c->lds_wl = wl;
        c->lds_wl_log2 = wl ? log2u(wl) : 0;
    }
    *out = c;
    return YSB_OK;
}

int ysb_close(ysb_ctx* c) {
    destroy(c);
    return YSB_OK;
}

// ---- ad table -------------------------------------------------------------------------

static int load_map(ysb_ctx* c, const char* const* ad_ids, const uint32_t* lens, const uint32_t* campaign_idx,
                    uint64_t n);

int ysb_load_ad_map_packed(ysb_ctx* c, const char* keys, uint32_t key_len, const uint32_t* campaign_idx,
                           uint64_t n) {
    return ysb_load_ad_map_packed_shard(c, keys, key_len, campaign_idx, n, 0, 1);
}

int ysb_load_ad_map_packed_shard(ysb_ctx* c, const char* keys, uint32_t key_len, const uint32_t* campaign_idx,
                                 uint64_t n, uint32_t rank, uint32_t nranks) {
    if (!c) return YSB_ERR_ARG;
    if (n && (!keys || !campaign_idx)) return fail(c, YSB_ERR_ARG, "NULL ad map arrays");
    std::vector<const char*> ptr(n);
    std::vector<u32> len(n, key_len);
    for (u64 i = 0; i < n; ++i) ptr[i] = keys + i * key_len;
    return ysb_load_ad_map_shard(c, ptr.data(), len.data(), campaign_idx, n, rank, nranks);
}

int ysb_load_ad_map(ysb_ctx* c, const char* const* ad_ids, const uint32_t* lens, const uint32_t* campaign_idx,
                    uint64_t n) {
    return ysb_load_ad_map_shard(c, ad_ids, lens, campaign_idx, n, 0, 1);
}

// The entries of this rank's shard only (the host-side hash the router and the generator's
// shard files use, ysb_ad_shard), then the tables; the context keeps its shard so that the
// deferred-line kernel can tell a foreign key's miss from a real one.
int ysb_load_ad_map_shard(ysb_ctx* c, const char* const* ad_ids, const uint32_t* lens, const uint32_t* campaign_idx,
                          uint64_t n, uint32_t rank, uint32_t nranks) {
    if (!c) return YSB_ERR_ARG;
    if (nranks == 0 || rank >= nranks) return fail(c, YSB_ERR_ARG, "bad shard %u / %u", rank, nranks);
    if (n && (!ad_ids || !campaign_idx)) return fail(c, YSB_ERR_ARG, "NULL ad map arrays");
    int rc = launch_pending_raw(c);   // a batch submitted before the new map joins against the old one
    if (rc) return rc;
    if (nranks == 1) {
        rc = load_map(c, ad_ids, lens, campaign_idx, n);
    } else {
        std::vector<const char*> p;
        std::vector<u32> l, cm;
        for (u64 i = 0; i < n; ++i) {
            const u32 len = lens ? lens[i] : 36u;
            if (ad_ids[i] && ysb_ad_shard(ad_ids[i], len, nranks) != rank) continue;
            p.push_back(ad_ids[i]);
            l.push_back(len);
            cm.push_back(campaign_idx[i]);
        }
        rc = load_map(c, p.data(), l.data(), cm.data(), p.size());
    }
    if (rc) return rc;
    c->shard_rank = rank;
    c->shard_n = nranks;
    return YSB_OK;
}

static int load_map(ysb_ctx* c, const char* const* ad_ids, const uint32_t* lens, const uint32_t* campaign_idx,
                    uint64_t n) {
    // the tables live on this context's GPU, whichever device the calling thread last set
    // (one process may drive several contexts, e.g. one per GPU of a node)
    HIPCHK(c, hipSetDevice(c->device));
    u64 slots = 64;
    while (slots < 2 * n) slots <<= 1;   // load factor <= 0.5
    if (slots > (1ull << 31)) return fail(c, YSB_ERR_CAPACITY, "ad map too large (%llu)", (unsigned long long)n);
    std::vector<u32> tab(slots * SLOT_WORDS, 0);
    for (u64 s = 0; s < slots; ++s) tab[s * SLOT_WORDS + 1] = EMPTY_SLOT;
    const u32 mask = (u32)(slots - 1);
    for (u64 i = 0; i < n; ++i) {
        const u32 len = lens ? lens[i] : 36u;
        if (len > MAX_KEY_BYTES) return fail(c, YSB_ERR_FORMAT, "ad id %llu longer than %u bytes", (unsigned long long)i, MAX_KEY_BYTES);
        if (campaign_idx[i] >= c->cfg.n_campaigns)
            return fail(c, YSB_ERR_FORMAT, "campaign index %u >= n_campaigns %u", campaign_idx[i], c->cfg.n_campaigns);
        if (!ad_ids[i] && len) return fail(c, YSB_ERR_ARG, "ad id %llu is NULL", (unsigned long long)i);
        u32 kw[KEY_WORDS] = {0};
        if (len) std::memcpy(kw, ad_ids[i], len);
        const u32 h = key_hash(kw, len);
        for (u64 pr = 0;; ++pr) {
            u32* sl = &tab[(u64)((h + pr) & mask) * SLOT_WORDS];
            if (sl[1] == EMPTY_SLOT) {
                sl[0] = len;
                sl[1] = campaign_idx[i];
                std::memcpy(sl + 2, kw, sizeof kw);
                break;
            }
            if (sl[0] == len && std::memcmp(sl + 2, kw, sizeof kw) == 0) {   // HashMap.put: later wins
                sl[1] = campaign_idx[i];
                break;
            }
        }
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (slots != c->table_slots) {
        hipFree(c->d_table);
        c->d_table = nullptr;
        HIPCHK(c, hipMalloc(&c->d_table, tab.size() * 4));
        c->table_slots = slots;
    }
    HIPCHK(c, hipMemcpy(c->d_table, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    // every 36-byte key also goes into the two-choice cuckoo table (load <= 1/4)
    typedef std::array<u32, CKEY_WORDS> Key36;
    // the distinct 36-byte keys with their final (later-wins) campaign: the general
    // table already holds exactly that set
    std::vector<std::pair<Key36, u32>> keys36;
    for (u64 sl = 0; sl < slots; ++sl) {
        const u32* e = &tab[sl * SLOT_WORDS];
        if (e[1] == EMPTY_SLOT || e[0] != 36) continue;
        Key36 k;
        std::memcpy(k.data(), e + 2, 36);
        keys36.push_back({k, e[1]});
    }
    bool partial = false;
    if (c->cfg.flags & YSB_F_SPARSE_FAST_JOIN) {
        for (size_t i = 0; 2 * i + 1 < keys36.size(); ++i) keys36[i] = keys36[2 * i + 1];
        keys36.resize(keys36.size() / 2);
        partial = true;
    }
    u64 cslots = 64;
    while (cslots < 4 * keys36.size()) cslots <<= 1;
    // tables far beyond the L2s (32 MiB) go to HBM per probe: bucket layout
    const bool buckets = cslots * CSLOT_WORDS * 4 > (64ull << 20);
    if (buckets) {
        // buckets >= YSB_BUCKETS_X4 / 4 per key (3 entries each)
        cslots = 64;
        while (cslots * 4 < (u64)YSB_BUCKETS_X4 * keys36.size()) cslots <<= 1;
    }
    const u32 unit = buckets ? CB_WORDS : CSLOT_WORDS;
    std::vector<u32> kw, cv;   // bucket layout: the keys as words, their campaigns
    if (buckets) {
        kw.resize(keys36.size() * CKEY_WORDS);
        cv.resize(keys36.size());
        for (size_t i = 0; i < keys36.size(); ++i) {
            std::memcpy(&kw[i * CKEY_WORDS], keys36[i].first.data(), 36);
            cv[i] = keys36[i].second;
        }
    }
    std::vector<u32> ct;
    CuckooSeed cs{};
    u64 seed = 0x5EEDC0FFEEULL;
    for (int attempt = 0;; ++attempt) {
        if (attempt == 16) { cslots <<= 1; attempt = 0; }
        if (cslots > (1ull << 26)) {
            // No placement found (a key family the hash cannot separate): keep the
            // table without the keys that did not fit; the scan defers its misses to
            // the general path, so the join stays exact.
            cslots = 1ull << 26;
            partial = true;
        }
        seed = mix64(seed + (u64)attempt + cslots);
        cs = cuckoo_seed(seed);
        ct.assign(cslots * unit, 0);
        const u32 cm = (u32)(cslots - 1);
        bool ok = true;
        if (buckets) {
            const u64 homeless = cuckoo_build_buckets(kw.data(), cv.data(), keys36.size(), cs, cslots, seed, partial,
                                                      ct.data());
            ok = homeless == 0;
            if (ok || partial) break;
            continue;
        }
        for (u64 s = 0; s < cslots; ++s) ct[s * CSLOT_WORDS + CSLOT_CAMP] = EMPTY_SLOT;
        for (const auto& kv : keys36) {
            Key36 k = kv.first;
            u32 camp = kv.second;
            u32 a, b;
            cuckoo_slots36(k.data(), cs, cm, &a, &b);
            u32 pos = a;
            int kicks = 0;
            while (true) {
                u32* sl = &ct[(u64)pos * CSLOT_WORDS];
                if (sl[CSLOT_CAMP] == EMPTY_SLOT) {
                    std::memcpy(sl, k.data(), 36);
                    sl[CSLOT_CAMP] = camp;
                    break;
                }
                // evict the occupant to its other slot
                Key36 ok_;
                std::memcpy(ok_.data(), sl, 36);
                const u32 oc = sl[CSLOT_CAMP];
                std::memcpy(sl, k.data(), 36);
                sl[CSLOT_CAMP] = camp;
                k = ok_;
                camp = oc;
                u32 oa, ob;
                cuckoo_slots36(k.data(), cs, cm, &oa, &ob);
                pos = (pos == oa) ? ob : oa;
                if (++kicks > 500) { ok = false; break; }
            }
            if (!ok && !partial) break;   // partial: the homeless key is simply left out
        }
        if (ok || partial) break;
    }
    if (cslots != c->ctable_slots) {
        hipFree(c->d_ctable);
        c->d_ctable = nullptr;
        HIPCHK(c, hipMalloc(&c->d_ctable, ct.size() * 4));
        c->ctable_slots = cslots;
    }
    HIPCHK(c, hipMemcpy(c->d_ctable, ct.data(), ct.size() * 4, hipMemcpyHostToDevice));
    c->cseed = cs;
    c->ctable_buckets = buckets;
    c->ctable_partial = partial;
    c->table_loaded = true;
    return YSB_OK;
}

void poll_ring(ysb_ctx* c) {
    if (c->ring_known || !c->ring_query_pending) return;
    if (hipEventQuery(c->ev_ring) == hipSuccess) {
        c->ring_query_pending = false;
        if (c->h_ring[1]) { c->ring_known = true; c->ring_lo = c->h_ring[0]; }
    }
}

// The delta ring into the u64 ring (queued on the compute stream), delta cleared.
int fold_delta(ysb_ctx* c) {
    if (!c->d_delta || c->delta_bound == 0) return YSB_OK;
    launch_fold(c->d_counts, c->d_delta, c->delta_cells, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->delta_bound = 0;
    c->pend_u64 = true;   // pending counts now sit in the u64 ring
    return YSB_OK;
}

int sync_streams(ysb_ctx* c) {
    int rc = launch_pending_raw(c);
    if (!rc) rc = finish_unpack(c);   // a pipelined exchange's owner block
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->s_copy));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (c->s_x) HIPCHK(c, hipStreamSynchronize(c->s_x));
    poll_ring(c);
    return YSB_OK;
}


// After the streams are idle: the out-of-ring map is emptied into the exact host-side
// list once it is a quarter full (so it never fills across launches: the side list
// grows on demand), and counts the device could not place anywhere (the map full
// within one launch AND the fallback list full) fail the call -- results would no
// longer be exact.  The loss is sticky until ysb_reset.
static int check_capacity(ysb_ctx* c) {
    unsigned long long v[ST_COUNT_ + 1];
    HIPCHK(c, hipMemcpy(v, c->d_stats, sizeof v, hipMemcpyDeviceToHost));
    const u32 used = (u32)v[ST_COUNT_];
    if ((u64)used * 4 > c->side_slots) {
        int rc = pull_side_list(c);
        if (rc) return rc;
    }
    if (v[ST_OVF_DROPPED])
        return fail(c, YSB_ERR_CAPACITY,
                    "%llu joined views outside the window ring were lost: the out-of-ring map and its "
                    "fallback list (overflow_capacity %llu) filled; counts are not exact "
                    "until ysb_reset (raise overflow_capacity or window_ring, or submit smaller batches)",
                    (unsigned long long)v[ST_OVF_DROPPED], (unsigned long long)c->cfg.overflow_capacity);
    if ((c->cfg.flags & YSB_F_STRICT) && (v[ST_PARSE_ERR] || v[ST_TIME_ERR] || v[ST_FOREIGN]))
        return fail(c, YSB_ERR_DATA,
                    "strict mode: %llu lines JSONObject/getString would throw on, %llu event_times "
                    "Long.parseLong rejects, %llu views of another rank's ad shard (routing does not match "
                    "the sharded join table); sticky until ysb_reset",
                    (unsigned long long)v[ST_PARSE_ERR], (unsigned long long)v[ST_TIME_ERR],
                    (unsigned long long)v[ST_FOREIGN]);
    return YSB_OK;
}

int ysb_sync(ysb_ctx* c) {
    if (!c) return YSB_ERR_ARG;
    int rc = sync_streams(c);
    if (rc) return rc;
    return check_capacity(c);
}

// ---- results --------------------------------------------------------------------------------

int read_ring(ysb_ctx* c) {
    i64 r[2];
    HIPCHK(c, hipMemcpy(r, c->d_ring, 16, hipMemcpyDeviceToHost));
    if (r[1]) { c->ring_known = true; c->ring_lo = r[0]; }
    c->ring_query_pending = false;
    return YSB_OK;
}

int pull_side_list(ysb_ctx* c) {
    u32 cnt = 0;
    HIPCHK(c, hipMemcpy(&cnt, c->d_ovf_count, 4, hipMemcpyDeviceToHost));
    const u32 m = (u32)std::min<u64>(cnt, c->cfg.overflow_capacity);
    if (m) {
        std::vector<OvfEntry> v(m);
        HIPCHK(c, hipMemcpy(v.data(), c->d_ovf, (u64)m * sizeof(OvfEntry), hipMemcpyDeviceToHost));
        for (const auto& e : v) c->side[{e.campaign, e.bucket}] += e.count;
    }
    if (cnt) HIPCHK(c, hipMemset(c->d_ovf_count, 0, 4));
    // the out-of-ring map: every occupied slot to the host map, then the map is emptied
    u32 used = 0;
    HIPCHK(c, hipMemcpy(&used, c->d_side_used, 4, hipMemcpyDeviceToHost));
    if (used) {
        if (!c->d_rows_n) HIPCHK(c, hipMalloc(&c->d_rows_n, 8));
        u32 k = 0;
        HIPCHK(c, hipMemsetAsync(c->d_rows_n, 0, 4, c->s_comp));
        launch_side_compact(c->d_side, c->side_slots, c->side_cbits, true, nullptr, c->d_rows_n, 0, c->s_comp);
        HIPCHK(c, hipMemcpyAsync(&k, c->d_rows_n, 4, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        if (k > c->rows_cap) {
            hipFree(c->d_rows);
            c->d_rows = nullptr;
            const u64 cap = std::max<u64>(k, 4096);
            HIPCHK(c, hipMalloc(&c->d_rows, cap * sizeof(TableRow)));
            c->rows_cap = cap;
        }
        if (k) {
            std::vector<TableRow> h(k);
            HIPCHK(c, hipMemsetAsync(c->d_rows_n, 0, 4, c->s_comp));
            launch_side_compact(c->d_side, c->side_slots, c->side_cbits, false, c->d_rows, c->d_rows_n, k, c->s_comp);
            HIPCHK(c, hipMemcpyAsync(h.data(), c->d_rows, (u64)k * sizeof(TableRow), hipMemcpyDeviceToHost, c->s_comp));
            HIPCHK(c, hipStreamSynchronize(c->s_comp));
            for (const TableRow& r : h) c->side[{r.campaign, r.bucket}] += r.count;
        }
        launch_side_clear(c->d_side, c->side_slots, c->s_comp);
        HIPCHK(c, hipMemsetAsync(c->d_side_used, 0, 4, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
    }
    return YSB_OK;
}

// Non-zero ring cells of buckets [blo, bhi) (rank-local table + owned block), compacted
// on the device (two passes: count, then rows), added to `into`; clear zeroes them.
static int ring_rows(ysb_ctx* c, i64 blo, i64 bhi, bool clear, std::map<std::pair<u32, i64>, u64>& into) {
    HIPCHK(c, hipSetDevice(c->device));
    int frc = fold_delta(c);
    if (frc) return frc;
    if (!c->ring_known) return YSB_OK;
    const u32 W = c->cfg.window_ring;
    const i64 lo = c->ring_lo;
    const i64 a = std::max<i64>(blo, lo), b = std::min<i64>(bhi, lo + (i64)W);
    if (a >= b) return YSB_OK;
    const u32 nb = (u32)(b - a);
    if ((frc = fold_owned(c))) return frc;
    struct Tab { unsigned long long* t; u32 rows, off; };
    std::vector<Tab> tabs{{c->d_counts, c->cfg.n_campaigns, 0u}};
    if (c->d_owned) {
        u32 olo = 0, ohi = 0;
        ysb_group_block(c->cfg.n_campaigns, c->rank, c->nranks, &olo, &ohi);
        if (ohi > olo) tabs.push_back({c->d_owned, ohi - olo, olo});
    }
    if (!c->d_rows_n) HIPCHK(c, hipMalloc(&c->d_rows_n, 8));
    for (const Tab& t : tabs) {
        u32 n = 0;
        HIPCHK(c, hipMemsetAsync(c->d_rows_n, 0, 4, c->s_comp));
        launch_compact(t.t, t.rows, W, a, nb, t.off, true, false, nullptr, c->d_rows_n, 0, c->s_comp);
        HIPCHK(c, hipMemcpyAsync(&n, c->d_rows_n, 4, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        if (!n) continue;
        if (n > c->rows_cap) {
            hipFree(c->d_rows);
            c->d_rows = nullptr;
            const u64 cap = std::max<u64>(n, 4096);
            HIPCHK(c, hipMalloc(&c->d_rows, cap * sizeof(TableRow)));
            c->rows_cap = cap;
        }
        std::vector<TableRow> h(n);
        u32 m = 0;
        HIPCHK(c, hipMemsetAsync(c->d_rows_n, 0, 4, c->s_comp));
        launch_compact(t.t, t.rows, W, a, nb, t.off, false, clear, c->d_rows, c->d_rows_n, n, c->s_comp);
        HIPCHK(c, hipMemcpyAsync(&m, c->d_rows_n, 4, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipMemcpyAsync(h.data(), c->d_rows, (u64)n * sizeof(TableRow), hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        if (m != n) return fail(c, YSB_ERR_STATE, "table changed during drain (%u vs %u cells)", m, n);
        for (const TableRow& r : h) into[{r.campaign, r.bucket}] += r.count;
    }
    return YSB_OK;
}

// ---- asynchronous flush (CampaignProcessorCommon's flusher thread, :35-55, 91-98) --------------

constexpr u64 FLUSH_MAX_ROWS = 1u << 20;

int ysb_flush_begin(ysb_ctx* c, int64_t blo, int64_t bhi) {
    if (!c) return YSB_ERR_ARG;
    if (grouped(c)) return fail(c, YSB_ERR_STATE, "ysb_flush_begin after ysb_group_init: use ysb_drain");
    if (c->fl_n == ysb_ctx::FLUSH_SLOTS)
        return fail(c, YSB_ERR_STATE, "%d flushes outstanding: ysb_flush_end first", ysb_ctx::FLUSH_SLOTS);
    int rc = launch_pending_raw(c);   // every batch submitted so far is counted before the compaction
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    const u32 W = c->cfg.window_ring;
    const int k = (c->fl_head + c->fl_n) % ysb_ctx::FLUSH_SLOTS;
    auto& f = c->fl[k];
    if (!c->d_fl_n) {
        HIPCHK(c, hipMalloc(&c->d_fl_n, 4 * ysb_ctx::FLUSH_SLOTS));
        HIPCHK(c, hipMemset(c->d_fl_n, 0, 4 * ysb_ctx::FLUSH_SLOTS));
    }
    if (!f.h_rows) {   // every nonzero cell of the ring fits (up to FLUSH_MAX_ROWS)
        f.cap = std::min<u64>((u64)c->cfg.n_campaigns * W, FLUSH_MAX_ROWS);
        HIPCHK(c, hipHostMalloc(&f.h_rows, f.cap * sizeof(TableRow)));
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&f.hd_rows), f.h_rows, 0));
        HIPCHK(c, hipHostMalloc(&f.h_n, 16));
        HIPCHK(c, hipEventCreateWithFlags(&f.ev, hipEventDisableTiming));
    }
    // the ring's base: known once the first launch's auto-base is back (a copy of 16 bytes)
    poll_ring(c);
    if (!c->ring_known && c->ring_query_pending) {
        HIPCHK(c, hipEventSynchronize(c->ev_ring));
        poll_ring(c);
    }
    if ((rc = fold_delta(c))) return rc;   // record mode's pending bytes into the u64 ring (stream order)
    HIPCHK(c, hipMemsetAsync(c->d_fl_n + k, 0, 4, c->s_comp));
    if (c->ring_known) {
        const i64 a = std::max<i64>(blo, c->ring_lo), b = std::min<i64>(bhi, c->ring_lo + (i64)W);
        if (a < b)   // straight into the pinned rows; a cell past cap keeps its count (next flush)
            launch_compact(c->d_counts, c->cfg.n_campaigns, W, a, (u32)(b - a), 0, false, true, f.hd_rows,
                           c->d_fl_n + k, (u32)f.cap, c->s_comp);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipMemcpyAsync(f.h_n, c->d_fl_n + k, 4, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipEventRecord(f.ev, c->s_comp));
    c->fl_n++;
    return YSB_OK;
}

int ysb_flush_end(ysb_ctx* c, int wait, ysb_count* out, uint64_t cap, uint64_t* n_out, int* more) {
    if (!c || !n_out) return c ? fail(c, YSB_ERR_ARG, "n_out is NULL") : YSB_ERR_ARG;
    if (!c->fl_n) return fail(c, YSB_ERR_STATE, "no flush begun");
    HIPCHK(c, hipSetDevice(c->device));
    auto& f = c->fl[c->fl_head];
    if (!wait) {
        const hipError_t q = hipEventQuery(f.ev);
        if (q == hipErrorNotReady) return YSB_PENDING;
        if (q != hipSuccess) return fail(c, YSB_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(q));
    }
    HIPCHK(c, hipEventSynchronize(f.ev));
    const u64 written = *f.h_n;
    const u64 n = std::min<u64>(written, f.cap);
    *n_out = n;
    if (more) *more = written > f.cap ? 1 : 0;
    if (!out) return YSB_OK;   // (the rows stay: call again with a buffer)
    if (cap < n) return fail(c, YSB_ERR_CAPACITY, "flush needs %llu rows, cap %llu", (unsigned long long)n,
                             (unsigned long long)cap);
    std::vector<TableRow> rows(f.h_rows, f.h_rows + n);
    std::sort(rows.begin(), rows.end(), [](const TableRow& x, const TableRow& y) {
        return x.campaign != y.campaign ? x.campaign < y.campaign : x.bucket < y.bucket;
    });
    for (u64 i = 0; i < n; ++i) {
        out[i].campaign = rows[i].campaign;
        out[i].reserved = 0;
        out[i].window_ms = rows[i].bucket * c->cfg.time_divisor_ms;
        out[i].count = rows[i].count;
    }
    c->fl_head = (c->fl_head + 1) % ysb_ctx::FLUSH_SLOTS;
    c->fl_n--;
    return YSB_OK;
}

int ysb_drain(ysb_ctx* c, int64_t blo, int64_t bhi, int clear, ysb_count* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return c ? fail(c, YSB_ERR_ARG, "n_out is NULL") : YSB_ERR_ARG;
    int rc = ysb_sync(c);
    if (rc) return rc;
    if ((rc = read_ring(c))) return rc;
    if ((rc = pull_side_list(c))) return rc;
    std::map<std::pair<u32, i64>, u64> rows;
    if (clear && out) {
        // move the ring range into the host map first: nothing is lost if `cap` is short
        if ((rc = ring_rows(c, blo, bhi, true, c->side))) return rc;
    } else if ((rc = ring_rows(c, blo, bhi, false, rows))) {
        return rc;
    }
    for (auto it = c->side.begin(); it != c->side.end(); ++it)
        if (it->first.second >= blo && it->first.second < bhi && it->second) rows[it->first] += it->second;
    *n_out = rows.size();
    if (!out) return YSB_OK;
    if (cap < rows.size()) return fail(c, YSB_ERR_CAPACITY, "drain needs %llu rows, cap %llu", (unsigned long long)rows.size(), (unsigned long long)cap);
    u64 k = 0;
    for (const auto& r : rows) {
        out[k].campaign = r.first.first;
        out[k].reserved = 0;
        out[k].window_ms = r.first.second * c->cfg.time_divisor_ms;
        out[k].count = r.second;
        ++k;
    }
    if (clear) {
        for (auto it = c->side.begin(); it != c->side.end();) {
            if (it->first.second >= blo && it->first.second < bhi) it = c->side.erase(it);
            else ++it;
        }
    }
    return YSB_OK;
}

// Moves the ring to [new_lo, new_lo + W): buckets of the old range that the new range
// does not hold go to the exact host-side list (both the rank-local table and, after an
// exchange, the owned block); cells are indexed by bucket mod W, so the rest stays put.
int move_ring(ysb_ctx* c, i64 new_lo) {
    int rc;
    if (c->ring_known && new_lo != c->ring_lo) {
        const i64 lo = c->ring_lo, W = (i64)c->cfg.window_ring;
        const i64 a = new_lo > lo ? lo : std::max<i64>(new_lo + W, lo);
        const i64 b = new_lo > lo ? std::min<i64>(new_lo, lo + W) : lo + W;
        if (a < b && (rc = ring_rows(c, a, b, true, c->side))) return rc;
    }
    i64 r[2] = {new_lo, 1};
    HIPCHK(c, hipMemcpy(c->d_ring, r, 16, hipMemcpyHostToDevice));
    c->ring_known = true;
    c->ring_lo = new_lo;
    c->ring_query_pending = false;
    return YSB_OK;
}

int ysb_ring_advance(ysb_ctx* c, int64_t new_lo) {
    if (!c) return YSB_ERR_ARG;
    // (no capacity check here: after ysb_group_init this is a collective, and a rank must
    // not leave before the others' all-reduce; ysb_sync / ysb_drain report a loss)
    int rc = sync_streams(c);
    if (rc) return rc;
    if ((rc = read_ring(c))) return rc;
    if (grouped(c)) {
        // collective after ysb_group_init: every rank's ring moves together (all ranks call
        // it with the same new_lo; a disagreement fails on every rank alike)
        if (!c->ring_agreed && (rc = agree_ring(c))) return rc;
        i64 h[2] = {new_lo, -new_lo};
        if ((rc = allreduce_max(c, h, 2))) return rc;
        if (h[0] != -h[1]) return fail(c, YSB_ERR_ARG, "ysb_ring_advance: ranks asked for different ring bases");
        c->x_have_plan = false;   // the plan's slots held other buckets
    }
    if (new_lo <= INT64_MIN / 2 || new_lo >= INT64_MAX / 2) return fail(c, YSB_ERR_ARG, "ring base out of range");
    return move_ring(c, new_lo);
}

int ysb_stats_get(ysb_ctx* c, ysb_stats* s) {
    if (!c || !s) return c ? fail(c, YSB_ERR_ARG, "NULL stats") : YSB_ERR_ARG;
    int rc = sync_streams(c);   // readable after a capacity loss (overflow_dropped tells it)
    if (rc) return rc;
    unsigned long long v[ST_COUNT_];
    HIPCHK(c, hipMemcpy(v, c->d_stats, sizeof v, hipMemcpyDeviceToHost));
    s->events = v[ST_EVENTS];
    s->views = v[ST_VIEWS];
    s->joined = v[ST_JOINED];
    s->join_misses = v[ST_MISSES];
    s->parse_errors = v[ST_PARSE_ERR];
    s->time_errors = v[ST_TIME_ERR];
    s->out_of_ring = v[ST_OUT_OF_RING];
    s->overflow_dropped = v[ST_OVF_DROPPED];
    s->batches = c->batches;
    s->deferred = v[ST_DEFERRED];
    s->foreign_shard = v[ST_FOREIGN];
    return YSB_OK;
}

int ysb_reset(ysb_ctx* c) {
    if (!c) return YSB_ERR_ARG;
    c->raw_fail = 0;   // a raw batch that could not launch was dropped: counting starts over
    int rc = sync_streams(c);
    if (rc) return rc;
    c->fl_head = c->fl_n = 0;   // outstanding asynchronous flushes are dropped
    const u64 cells = (u64)c->c_pad * c->cfg.window_ring;
    HIPCHK(c, hipMemset(c->d_counts, 0, cells * 8));
    if (c->d_delta) HIPCHK(c, hipMemset(c->d_delta, 0, c->delta_cells));
    c->delta_bound = 0;
    HIPCHK(c, hipMemset(c->d_dirty, 0, 4));
    c->pend_u64 = false;
    c->x_have_plan = false;
    if (c->d_owned) HIPCHK(c, hipMemset(c->d_owned, 0, cells / c->nranks * 8));
    if (c->d_owned8) HIPCHK(c, hipMemset(c->d_owned8, 0, cells / c->nranks));
    c->owned8_dirty = false;
    if (c->d_truth) HIPCHK(c, hipMemset(c->d_truth, 0, cells * 8));
    if (c->d_truth_out) HIPCHK(c, hipMemset(c->d_truth_out, 0, 8));
    HIPCHK(c, hipMemset(c->d_ovf_count, 0, 16));
    launch_side_clear(c->d_side, c->side_slots, c->s_comp);
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    HIPCHK(c, hipMemset(c->d_side_used, 0, 4));
    HIPCHK(c, hipMemset(c->d_stats, 0, ST_COUNT_ * 8));
    c->side.clear();
    c->batches = 0;
    return YSB_OK;
}

int ysb_ring_range(ysb_ctx* c, int64_t* lo, uint32_t* width) {
    if (!c) return YSB_ERR_ARG;
    int rc = ysb_sync(c);
    if (rc) return rc;
    if ((rc = read_ring(c))) return rc;
    if (!c->ring_known) return fail(c, YSB_ERR_STATE, "ring base not set yet");
    if (lo) *lo = c->ring_lo;
    if (width) *width = c->cfg.window_ring;
    return YSB_OK;
}

int ysb_kernel_time(ysb_ctx* c, double* total_ms, uint64_t* launches) {
    if (!c) return YSB_ERR_ARG;
    int rc = sync_streams(c);
    if (rc) return rc;
    double t = c->tev_ms_fold, tp = c->tev_path_fold;
    for (size_t i = 0; i < c->tev_used; ++i) {
        float ms = 0, mp = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->tev[i][0], c->tev[i][1]));
        HIPCHK(c, hipEventElapsedTime(&mp, c->tev[i][0], c->tev[i][2]));
        t += ms;
        tp += mp;
    }
    const u64 n = c->tev_folded + c->tev_used;
    if (total_ms) *total_ms = t;
    if (launches) *launches = n;
    c->path_ms_acc = tp;
    c->path_launches_acc = n;
    c->tev_used = 0;
    c->tev_ms_fold = c->tev_path_fold = 0;
    c->tev_folded = 0;
    return YSB_OK;
}

int ysb_path_time(ysb_ctx* c, double* total_ms, uint64_t* launches, uint64_t* record_launches) {
    if (!c) return YSB_ERR_ARG;
    if (total_ms) *total_ms = c->path_ms_acc;
    if (launches) *launches = c->path_launches_acc;
    if (record_launches) *record_launches = c->rec_launches;
    return YSB_OK;
}

int ysb_launch_info(ysb_ctx* c, ysb_launch_desc* out) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    int rc = launch_pending_raw(c);
    if (rc) return rc;
    *out = c->last_launch;
    return YSB_OK;
}

void* ysb_stream(ysb_ctx* c) {
    if (!c) return nullptr;
    // work the caller orders after it follows every submitted batch; NULL if one could not
    // launch (ysb_last_error says why)
    if (launch_pending_raw(c)) return nullptr;
    return (void*)c->s_comp;
}

// ---- device memory ----------------------------------------------------------------------------

int ysb_device_alloc(ysb_ctx* c, uint64_t bytes, void** p) {
    if (!c || !p) return YSB_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMalloc(p, bytes ? bytes : 16));
    return YSB_OK;
}
int ysb_device_free(ysb_ctx* c, void* p) {
    if (!c) return YSB_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipFree(p));
    return YSB_OK;
}
int ysb_memcpy_h2d(ysb_ctx* c, void* d, const void* h, uint64_t bytes) {
    if (!c) return YSB_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return YSB_OK;
}
int ysb_memcpy_d2h(ysb_ctx* c, void* h, const void* d, uint64_t bytes) {
    if (!c) return YSB_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
    return YSB_OK;
}

#if defined(YSB_STAMPS) || defined(YSB_WGTIME)
// Diagnostic build only: the deferred-line list of the last batch.
int ysb_debug_defer_list(ysb_ctx* c, uint32_t* out, uint64_t cap) {
    if (!c) return YSB_ERR_ARG;
    int rc = ysb_sync(c);
    if (rc) return rc;
    if (!c->d_defer) return YSB_OK;
    HIPCHK(c, hipMemcpy(out, c->d_defer, std::min<u64>(cap, c->defer_cap) * 4, hipMemcpyDeviceToHost));
    return YSB_OK;
}

// Diagnostic build only: per-wave phase cycles of the scan kernel since the last call.
int ysb_debug_stamps(ysb_ctx* c, uint64_t* out, uint64_t cap, uint64_t* n) {
    if (!c || !n) return YSB_ERR_ARG;
    int rc = ysb_sync(c);
    if (rc) return rc;
    *n = c->dbg_words;
    if (!out || !c->d_dbg) return YSB_OK;
    HIPCHK(c, hipMemcpy(out, c->d_dbg, std::min<u64>(cap, c->dbg_words) * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemset(c->d_dbg, 0, c->dbg_words * 8));
    return YSB_OK;
}
#endif

}  // extern "C"
