// ysb_capi.cpp -- the C ABI of include/ysb_hip.h: context lifecycle, the device
// ad -> campaign table, double-buffered batch submission, result drain, the RCCL
// group step and the host side of the synthetic generator.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ysb_hip.h"
#include "ysb_kernels.h"

using namespace ysb;

namespace ysb {
int scan_lds_bytes();
}

constexpr size_t XEV_KEEP = 64;   // exchange timing pairs pending before they are folded into x_ms

// HBM-resident join table (bucket layout): buckets per key, x4 (8: 2 per key, a 4 GiB
// table at 10M ads; fewer buckets -> a smaller table, more keys in their second bucket)
#ifndef YSB_BUCKETS_X4
#define YSB_BUCKETS_X4 8
#endif

// A key order read off a batch's first line (layout 3, learn_layout).
struct LearnDesc {
    u32 order[8];
    u32 n;
    u32 cp;
};

struct ysb_ctx {
    int device = 0;
    ysb_config cfg{};
    std::string err;
    int cus = 256;
    hipStream_t s_comp = nullptr, s_copy = nullptr;
    // ad table
    u32* d_table = nullptr;
    u64 table_slots = 0;
    u32* d_ctable = nullptr;   // 36-byte-key cuckoo table
    u64 ctable_slots = 0;      // slots, or buckets when ctable_buckets
    bool ctable_buckets = false; // HBM-resident table: 3-entry 128-B buckets (CB_*), serial probes
    int submit_layout = -1;      // the layout a submit read off its batch's first line (-1: the flags')
    LearnDesc submit_learn{};    // ... and, layout 3, the key order
    ysb_launch_desc last_launch{};   // the instantiation of the last launch
    // device batches' first-line samples: written by sample_kernel on the compute stream (so
    // after whatever produced the batch there) into pinned memory, two buffers alternating
    // by launch; ev_sample[k] marks buffer k complete, sample_nseg[k] its segments (0: none)
    u8* h_sample = nullptr;
    hipEvent_t ev_sample[2] = {nullptr, nullptr};
    u32 sample_nseg[2] = {0, 0};
    int sample_cur = 0;
    u32* h_used = nullptr;       // pinned: the out-of-ring map's fill level after a launch ...
    hipEvent_t ev_used = nullptr; // ... readable once this has completed
    bool used_pending = false;
    // raw batches (ysb_submit_raw): the line starts are found on the GPU (ysb_split.hip) on
    // s_split after the slot's H2D, into d_roff[slot]; the scan is launched once the line
    // count is back (launch_pending_raw, at the next call), so the next H2D queues first
    hipStream_t s_split = nullptr;
    u32* d_roff[2] = {nullptr, nullptr};        // max_batch_bytes + 1 starts per slot
    u32* d_split_chunk = nullptr;               // per-chunk counts, then bases
    u64 split_chunk_words = 0;
    unsigned long long* d_rawn = nullptr;       // [2] lines of the slot's raw batch
    unsigned long long* h_rawn = nullptr;       // pinned mirror
    hipEvent_t ev_raw[2] = {nullptr, nullptr};  // split done and its count read back
    int raw_pend = -1;                          // the slot whose raw batch awaits its launch
    u64 raw_nbytes[2] = {0, 0};
    int raw_layout[2] = {-1, -1};               // its first line's layout (sampled on the host)
    LearnDesc raw_learn[2]{};
    // H2D timing (YSB_F_TIMING): {start, end} of each slot copy since the last ysb_copy_time
    std::vector<std::array<hipEvent_t, 2>> cev;
    size_t cev_used = 0;
    u64 copy_bytes = 0;
    CuckooSeed cseed{};
    bool ctable_partial = false;
    bool table_loaded = false;
    u32 shard_rank = 0, shard_n = 1;      // the join table's shard (ysb_load_ad_map_shard)
    // counts
    u32 c_pad = 0;                        // campaigns padded to the group size
    unsigned long long* d_counts = nullptr;   // [c_pad][W]
    unsigned long long* d_owned = nullptr;    // [c_pad / nranks][W] after reduce-scatter
    u8* d_owned8 = nullptr;                   // ... its saturating u8 accumulator (xunpack), folded before reads
    bool owned8_dirty = false;
    unsigned long long* d_rs_tmp = nullptr;
    bool ring_agreed = false;                 // ranks' ring bases checked equal
    TableRow* d_rows = nullptr;               // drain compaction output
    u64 rows_cap = 0;
    u32* d_rows_n = nullptr;
    i64* d_ring = nullptr;                // [lo, set]
    i64* h_ring = nullptr;                // pinned mirror
    hipEvent_t ev_ring = nullptr;
    bool ring_query_pending = false;
    bool ring_known = false;
    i64 ring_lo = 0;
    OvfEntry* d_ovf = nullptr;
    u32* d_ovf_count = nullptr;
    SideSlot* d_side = nullptr;               // out-of-ring cells (device hash map)
    u64 side_slots = 0;
    u32 side_cbits = 1;
    u32* d_side_used = nullptr;               // = (u32*)(d_stats + ST_COUNT_)
    unsigned long long* d_stats = nullptr;    // ST_COUNT_ u64, then the map's slot count
    u64 batches = 0;
    std::map<std::pair<u32, i64>, u64> side;   // drained side-list deltas
    DivMagic div{};
    u32 lds_wl = 0, lds_wl_log2 = 0;
    // slots
    u8* h_bytes[2] = {nullptr, nullptr};
    u32* h_off[2] = {nullptr, nullptr};
    u8* d_bytes[2] = {nullptr, nullptr};
    u32* d_off[2] = {nullptr, nullptr};
    hipEvent_t ev_h2d[2] = {nullptr, nullptr}, ev_kdone[2] = {nullptr, nullptr};
    bool slot_busy[2] = {false, false};
    // timing: per launch {before scan, after scan, after the last kernel of the launch}
    std::vector<std::array<hipEvent_t, 3>> tev;
    size_t tev_used = 0;
    double path_ms_acc = 0;                // ysb_path_time's share, collected by ysb_kernel_time
    u64 path_launches_acc = 0;
    // record mode (ysb_count.hip)
    u32* d_rec = nullptr;
    u64 rec_words = 0;
    u32* d_rec_n = nullptr;
    u64 rec_n_words = 0;
    u32* d_part = nullptr;
    u64 part_words = 0;
    u32* d_runs = nullptr;
    u64 runs_words = 0;
    u64 rec_launches = 0;
    // record mode counts into a saturating u8 delta ring with the u64 ring's layout (a cell
    // passing 255 goes to the u64 ring, ysb_count.hip add16); fold_delta adds it to the u64
    // ring before anything reads that.  delta_bound: events counted into it since the last
    // fold; YSB_DELTA_FOLD_EVENTS (test hook) folds before a launch once it would pass that
    u8* d_delta = nullptr;
    u64 delta_cells = 0;
    u64 delta_bound = 0;
    u64 delta_limit = ~0ull;
    // pending counts since the last exchange: the u64 ring holds some once a launch without
    // record mode ran or a fold moved the delta there (pend_u64), or a record-mode path
    // wrote it (*d_dirty, set on the device)
    bool pend_u64 = true;
    u32* d_dirty = nullptr;
    // group: an RCCL communicator, or the caller's host collectives (ysb_group_init_host)
    ncclComm_t comm = nullptr;
    bool host_coll = false;
    ysb_collectives hops{};
    int rank = 0, nranks = 1;
    // the range-limited exchange: per-slot maxima (all-reduced), the plan's slots, the packed
    // send / receive buffers, and its accounting (HIP event pairs, collected on request)
    // Two plan buffers (device maxima; pinned host maxima + slots): a pipelined exchange
    // packs with the previous call's plan (buffer xb, ready at xplan_ev[xb]) while its own
    // plan is reduced into the other one.
    unsigned long long* d_xmax = nullptr;   // [2][W]
    unsigned long long* h_xmax = nullptr;   // [2][W] maxima, then [2][W] u32 slots
    hipEvent_t xplan_ev[2] = {nullptr, nullptr};
    int xb = 0;
    bool x_have_plan = false;
    // plan -> pack run on the compute stream (in order with the scans that add to the rings);
    // the reduce-scatter on s_x, beside the next launch (at N ranks: the xGMI transfer); the
    // unpack into the owned table on the compute stream again, at the next exchange (or before
    // anything reads the owned table) -- beside a running scan it starved it (round 4 A/B).
    // Two buffer sets (slots, send, receive) alternate; a pack into set k waits for the
    // reduce-scatter that last used it (ev_xdone[k]), the exchange stream for the pack
    // (ev_xpacked[k]).
    hipStream_t s_x = nullptr;
    u32* d_xslots = nullptr;                // [2][W]
    void* d_xsend[2] = {nullptr, nullptr};
    void* d_xrecv[2] = {nullptr, nullptr};
    u64 xsend_bytes[2] = {0, 0}, xrecv_bytes[2] = {0, 0};
    hipEvent_t ev_xpacked[2] = {nullptr, nullptr}, ev_xdone[2] = {nullptr, nullptr};
    bool xset_used[2] = {false, false};
    int xk = 0;
    // the pipelined exchange whose unpack is still to run: its set, slots, width, timing entry
    int unpack_set = -1;
    u32 unpack_R = 0, unpack_width = 0;
    size_t unpack_entry = 0;
    u64 x_count = 0, x_bytes = 0;
    u32 x_last_slots = 0, x_last_width = 0;
    double x_ms = 0, x_crit_ms = 0;
    // per exchange {start, packed (compute stream), reduce-scatter done (exchange stream),
    // unpack start, unpack end (compute stream)}
    std::vector<std::array<hipEvent_t, 5>> xev;
    size_t xev_used = 0;
    // truth
    unsigned long long* d_truth = nullptr;
    unsigned long long* d_truth_out = nullptr;
    unsigned long long* d_cmp = nullptr;
    u32* d_subset = nullptr;
    u32 d_subset_n = 0;
    u32* d_defer = nullptr;                // deferred (general-path) line indices
    u64 defer_cap = 0;
    u32* d_defer_ctr = nullptr;            // [count, done, pad, pad, dynamic-claim counters[MAX_SEGS]]
    u32 dyn_pct = 0;                       // % of a large segment's tiles claimed dynamically (YSB_DYN_PCT; measured neutral, off)
    u32 dyn_chunk = 16;                    // tiles per claim (YSB_DYN_CHUNK)
    unsigned long long* d_dbg = nullptr;   // YSB_STAMPS diagnostic build
    u64 dbg_words = 0;
};

static thread_local std::string g_open_err;

static int fail(ysb_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    else g_open_err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(ctx, YSB_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                \
    } while (0)

static bool is_pow2(u64 x) { return x && !(x & (x - 1)); }
static u32 log2u(u64 x) { u32 l = 0; while (((u64)1 << l) < x) ++l; return l; }

extern "C" {

static int agree_ring(ysb_ctx* c);
static int allreduce_max(ysb_ctx* c, i64* h, int n);
static int sync_streams(ysb_ctx* c);
static int pull_side_list(ysb_ctx* c);
static bool grouped(const ysb_ctx* c);
static int launch_pending_raw(ysb_ctx* c);
static int finish_unpack(ysb_ctx* c);

int ysb_abi_version(void) { return YSB_ABI_VERSION; }

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
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, YSB_ERR_HIP, "no HIP device available");
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

// ---- batches ---------------------------------------------------------------------------

// segs: 1..MAX_SEGS batches, none empty
static ScanParams make_params(ysb_ctx* c, const ysb_segment* segs, u32 nseg) {
    ScanParams p{};
    p.tbl = (c->cfg.flags & YSB_F_FORMAT_TBL) ? 1u : 0u;
    p.bytes = segs[0].d_bytes;
    p.nbytes = segs[0].nbytes;
    p.off = segs[0].d_line_off;
    p.n = segs[0].n_events;
    p.line_base = 0;
    p.table = c->d_table;
    p.table_mask = (u32)(c->table_slots - 1);
    p.ctable = c->d_ctable;
    p.ctable_mask = (u32)(c->ctable_slots - 1);
    p.cseed = c->cseed;
    // a sharded table's misses go to the deferred-line kernel, which tells a foreign-shard
    // key from a real miss (the scan kernels themselves carry no shard logic)
    p.ctable_partial = (c->ctable_partial || c->shard_n > 1) ? 1u : 0u;
    p.shard_rank = c->shard_rank;
    p.shard_n = c->shard_n;
    p.pend_dirty = c->d_dirty;
    // HBM-resident table: buckets, the second one read only after a miss in a full first
    p.probe_serial = c->ctable_buckets ? 1u : 0u;
    p.layout = (c->cfg.flags & YSB_F_FLAT_FIRST) ? 2u : (c->cfg.flags & YSB_F_COMPACT_FIRST) ? 1u : 0u;
    if (c->submit_layout >= 0) p.layout = (u32)c->submit_layout;
    if (p.layout == 3 || p.layout == 4) {   // (4: learn_n 0 when the sample named no learned order)
        p.learn_code = 0;
        for (u32 i = 0; i < c->submit_learn.n; ++i) p.learn_code |= c->submit_learn.order[i] << (3 * i);
        p.learn_n = c->submit_learn.n;
        p.learn_cp = c->submit_learn.cp;
    }
    p.n_campaigns = c->cfg.n_campaigns;
    p.counts = c->d_counts;
    p.ring_w = c->cfg.window_ring;
    p.lds_wl = c->lds_wl;
    p.lds_wl_log2 = c->lds_wl_log2;
    p.require_mask = (c->cfg.flags & YSB_F_REQUIRE_IP) ? 0x7Fu : 0x3Fu;
    p.ring = c->d_ring;
    p.div = c->div;
    p.side = c->d_side;
    p.side_used = c->d_side_used;
    p.side_mask = (u32)(c->side_slots - 1);
    p.side_cbits = c->side_cbits;
    p.ovf = c->d_ovf;
    p.ovf_count = c->d_ovf_count;
    p.ovf_cap = (u32)c->cfg.overflow_capacity;
    p.stats = c->d_stats;
    // Each segment's tiles: a static share split evenly over the grid, and for large
    // segments (>= 8 tiles per resident workgroup) a dynamic share of dyn_pct % claimed in
    // chunks by the workgroups that finish first.  The grid is whole rounds of resident
    // workgroups (a partial last round would idle most CUs), enough that no static run
    // exceeds MAX_TILES_PER_BLOCK tiles (the LDS copy of a run's tile bounds).
    const u64 resident = (u64)c->cus * (p.tbl ? Geom<true>::WG_PER_CU : Geom<false>::WG_PER_CU);
    const u32 chunk = std::min<u32>(c->dyn_chunk, MAX_TILES_PER_BLOCK);
    u64 line_base = 0, max_static = 0;
    bool any_dyn = false;
    p.n_segs = nseg;
    for (u32 i = 0; i < nseg; ++i) {
        ScanSeg& sg = p.seg[i];
        sg.bytes = segs[i].d_bytes;
        sg.off = segs[i].d_line_off;
        sg.n = segs[i].n_events;
        sg.nbytes = segs[i].nbytes;
        sg.line_base = line_base;
        line_base += sg.n;
        sg.n_tiles = (sg.n + TILE_LINES - 1) / TILE_LINES;
        const bool dyn = chunk && c->dyn_pct && sg.n_tiles >= 8 * resident;
        sg.n_static = dyn ? sg.n_tiles - sg.n_tiles * std::min<u32>(c->dyn_pct, 100) / 100 : sg.n_tiles;
        any_dyn |= sg.n_static < sg.n_tiles;
        max_static = std::max(max_static, sg.n_static);
    }
    const u64 rounds = std::max<u64>(1, (max_static + resident * MAX_TILES_PER_BLOCK - 1) / (resident * MAX_TILES_PER_BLOCK));
    const u64 grid = std::max<u64>(1, std::min<u64>(max_static, rounds * resident));
    for (u32 i = 0; i < nseg; ++i) {
        ScanSeg& sg = p.seg[i];
        sg.tiles_per_block = (u32)(sg.n_static / grid);
        sg.static_rem = (u32)(sg.n_static % grid);
    }
    p.dyn_chunk = any_dyn ? chunk : 0u;
    p.n_tiles = p.seg[0].n_tiles;
    p.tiles_per_block = p.seg[0].tiles_per_block;
    p.grid = (u32)grid;
    return p;
}

static void poll_ring(ysb_ctx* c) {
    if (c->ring_known || !c->ring_query_pending) return;
    if (hipEventQuery(c->ev_ring) == hipSuccess) {
        c->ring_query_pending = false;
        if (c->h_ring[1]) { c->ring_known = true; c->ring_lo = c->h_ring[0]; }
    }
}

// Grows a device u32 buffer to at least `words` (contents not kept).
static int grow_u32(ysb_ctx* c, u32** buf, u64* have, u64 words) {
    if (*have >= words) return YSB_OK;
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    HIPCHK(c, hipMalloc(buf, words * 4));
    *have = words;
    return YSB_OK;
}

// The owned table's u8 accumulator into it (queued on the compute stream), cleared.
static int fold_owned(ysb_ctx* c) {
    if (!c->d_owned8 || !c->owned8_dirty) return YSB_OK;
    launch_fold(c->d_owned, c->d_owned8, (u64)c->c_pad / (u64)c->nranks * c->cfg.window_ring, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->owned8_dirty = false;
    return YSB_OK;
}

// The delta ring into the u64 ring (queued on the compute stream), delta cleared.
static int fold_delta(ysb_ctx* c) {
    if (!c->d_delta || c->delta_bound == 0) return YSB_OK;
    launch_fold(c->d_counts, c->d_delta, c->delta_cells, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->delta_bound = 0;
    c->pend_u64 = true;   // pending counts now sit in the u64 ring
    return YSB_OK;
}

// Record mode (ysb_count.hip) for this launch: large count tables without LDS window
// counters (configs[2]), where one global atomic per joined view is the bottleneck.
// Auto: ring >= 1M cells and launch >= 1M events; YSB_F_RECORD_COUNT forces it on
// wherever it is possible, YSB_F_NO_RECORD_COUNT off.
static int plan_records(ysb_ctx* c, ScanParams& p, u64 n_events, RecParams& r) {
    p.rec_on = 0;
    const u32 W = c->cfg.window_ring;
    const u64 cells = (u64)c->c_pad * W;
    const bool force = (c->cfg.flags & YSB_F_RECORD_COUNT) != 0;
    // (the record-mode kernels are the HBM-table instantiations: bucket-layout join table)
    if ((c->cfg.flags & YSB_F_NO_RECORD_COUNT) || c->lds_wl || p.dyn_chunk || cells >= (1ull << 32) ||
        W > (u32)REC_BLOCK_CELLS || !c->ctable_buckets)
        return YSB_OK;
    if (!force && (cells < (1ull << 20) || n_events < (1ull << 20))) return YSB_OK;
    r.ring_w = W;
    r.w_log2 = log2u(W);
    r.blk_shift = log2u(REC_BLOCK_CELLS / W);
    r.c_pad = c->c_pad;
    r.n_blocks = (u32)((c->c_pad + (1u << r.blk_shift) - 1) >> r.blk_shift);
    const u32 sub = (r.n_blocks + REC_BINS_MAX - 1) / REC_BINS_MAX;
    r.sub_log2 = log2u(sub);
    if ((1u << r.sub_log2) > (u32)REC_SUB_MAX) return YSB_OK;   // beyond 8 x 512 blocks: atomics
    r.bins = (r.n_blocks + (1u << r.sub_log2) - 1) >> r.sub_log2;
    r.grid = p.grid;
    if ((r.grid + REC_QUARTERS - 1) / REC_QUARTERS > 128) return YSB_OK;   // REC_SLICE_MAX
    // lines one workgroup scans at most in this launch; ~1/3 are joined views on generator
    // data; 3/4 of the lines spread over the bins leaves room for skew (a full sub-buffer
    // sends the rest of its views to the atomics: slower, still exact)
    u64 tiles = 0;
    for (u32 i = 0; i < p.n_segs; ++i) tiles += p.seg[i].tiles_per_block + (p.seg[i].static_rem ? 1 : 0);
    const u64 lines = tiles * TILE_LINES;
    u64 cap = (lines * 3 / 4 + r.bins - 1) / r.bins;
    cap = std::max<u64>(32, (cap + 31) / 32 * 32);
    // one (bin, slice) output area: the slice's sub-buffers plus a 32-record alignment pad per block
    const u64 area = ((u64)((r.grid + REC_QUARTERS - 1) / REC_QUARTERS) * cap + 32ull * (1u << r.sub_log2) + 31) / 32 * 32;
    const u64 part = (u64)r.bins * REC_QUARTERS * area;
    if (cap > 0xFFFFFFFFull || part >= (1ull << 32)) return YSB_OK;
    r.cap = (u32)cap;
    r.area = area;
    int rc;
    if ((rc = grow_u32(c, &c->d_rec, &c->rec_words, (u64)r.grid * r.bins * cap))) return rc;
    if ((rc = grow_u32(c, &c->d_rec_n, &c->rec_n_words, (u64)r.grid * r.bins))) return rc;
    if ((rc = grow_u32(c, &c->d_part, &c->part_words, part))) return rc;
    if ((rc = grow_u32(c, &c->d_runs, &c->runs_words, (u64)r.n_blocks * REC_QUARTERS * 2))) return rc;
    if (c->delta_cells != cells) {   // the delta ring: the u64 ring's layout, one byte a cell, zeroed
        if ((rc = fold_delta(c))) return rc;
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        hipFree(c->d_delta);
        c->d_delta = nullptr;
        c->delta_cells = 0;
        HIPCHK(c, hipMalloc(&c->d_delta, cells));
        HIPCHK(c, hipMemset(c->d_delta, 0, cells));
        c->delta_cells = cells;
    }
    // the delta saturates instead of wrapping, so it needs no fold between launches; the
    // test hook YSB_DELTA_FOLD_EVENTS folds anyway once the events since the last fold
    // would reach its bound
    if (c->delta_bound + n_events >= c->delta_limit && (rc = fold_delta(c))) return rc;
    c->delta_bound += n_events;
    r.delta = c->d_delta;
    r.counts = c->d_counts;
    r.dirty = c->d_dirty;
    r.rec = c->d_rec;
    r.rec_n = c->d_rec_n;
    r.part = c->d_part;
    r.runs = c->d_runs;
    p.rec_on = 1;
    p.rec_bins = r.bins;
    p.rec_shift = r.blk_shift + r.sub_log2;
    p.rec_cap = r.cap;
    p.rec = c->d_rec;
    p.rec_n = c->d_rec_n;
    return YSB_OK;
}

static int enqueue_scan(ysb_ctx* c, const ysb_segment* in, u32 nin) {
    if (!c->table_loaded) return fail(c, YSB_ERR_STATE, "ysb_load_ad_map has not been called");
    ysb_segment segs[MAX_SEGS];
    u32 nseg = 0;
    u64 n = 0;
    for (u32 i = 0; i < nin; ++i)
        if (in[i].n_events) { segs[nseg++] = in[i]; n += in[i].n_events; }
    if (n == 0) { c->batches += nin; return YSB_OK; }
    if (n >= (1ull << 31)) return fail(c, YSB_ERR_CAPACITY, "at most 2^31-1 events per launch");
    if (n > c->defer_cap) {   // the deferred-line list can hold every line of a batch
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        hipFree(c->d_defer);
        c->d_defer = nullptr;
        const u64 cap = std::max<u64>(n, 1u << 16);
        HIPCHK(c, hipMalloc(&c->d_defer, cap * 4));
        c->defer_cap = cap;
    }
    if (!c->d_defer_ctr) {
        HIPCHK(c, hipMalloc(&c->d_defer_ctr, 16 + 4 * MAX_SEGS));
        HIPCHK(c, hipMemset(c->d_defer_ctr, 0, 16 + 4 * MAX_SEGS));
    }
    // the out-of-ring map's fill level after an earlier launch (read without waiting): a
    // quarter full empties it into the exact host list before this launch adds to it
    if (c->used_pending && hipEventQuery(c->ev_used) == hipSuccess) {
        c->used_pending = false;
        if ((u64)*c->h_used * 4 > c->side_slots) {
            int rc = sync_streams(c);
            if (!rc) rc = pull_side_list(c);
            if (rc) return rc;
        }
    }
    ScanParams p = make_params(c, segs, nseg);
    p.used_out = c->used_pending ? nullptr : c->h_used;
    p.defer = c->d_defer;
    p.defer_count = c->d_defer_ctr;
    p.defer_done = c->d_defer_ctr + 1;
    p.dyn_ctr = c->d_defer_ctr + 4;
    p.defer_cap = (u32)c->defer_cap;
#if defined(YSB_STAMPS) || defined(YSB_WGTIME)
    const u64 words = (u64)c->cus * std::max(Geom<true>::WG_PER_CU, Geom<false>::WG_PER_CU) * (SCAN_TPB / 64) * N_STAMPS;
    if (!c->d_dbg) {
        HIPCHK(c, hipMalloc(&c->d_dbg, words * 8));
        HIPCHK(c, hipMemset(c->d_dbg, 0, words * 8));
        c->dbg_words = words;
    }
    p.dbg = c->d_dbg;
#endif
    poll_ring(c);
    const bool tbl = (c->cfg.flags & YSB_F_FORMAT_TBL) != 0;
    if (!c->ring_known) {
        if (tbl) launch_tbl_ring_autobase(p, c->s_comp);
        else launch_ring_autobase(p, c->s_comp);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->h_ring, c->d_ring, 16, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipEventRecord(c->ev_ring, c->s_comp));
        c->ring_query_pending = true;
    }
    // dynamic claims (off by default) count from zero in every launch
    if (p.dyn_chunk) HIPCHK(c, hipMemsetAsync(p.dyn_ctr, 0, 4 * MAX_SEGS, c->s_comp));
    RecParams rp{};
    int rc = plan_records(c, p, n, rp);
    if (rc) return rc;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (c->cfg.flags & YSB_F_TIMING) {
        if (c->tev_used == c->tev.size()) {
            std::array<hipEvent_t, 3> ev{};
            for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
            c->tev.push_back(ev);
        }
        e0 = c->tev[c->tev_used][0];
        e1 = c->tev[c->tev_used][1];
        e2 = c->tev[c->tev_used][2];
        c->tev_used++;
        HIPCHK(c, hipEventRecord(e0, c->s_comp));
    }
    launch_scan(p, c->s_comp);
    HIPCHK(c, hipGetLastError());
    if (!p.rec_on) c->pend_u64 = true;   // this launch counts into the u64 ring
    // (launch_scan: the layout instantiations exist for every JSON table layout)
    c->last_launch.layout = p.tbl ? 0u : p.layout;
    c->last_launch.record_mode = p.rec_on ? 1u : 0u;
    c->last_launch.hbm_table = p.probe_serial ? 1u : 0u;
    c->last_launch.tbl = p.tbl ? 1u : 0u;
    if (e1) HIPCHK(c, hipEventRecord(e1, c->s_comp));
    launch_defer(p, c->cus, c->s_comp);
    HIPCHK(c, hipGetLastError());
    if (p.rec_on) {
        launch_rec_partition(rp, c->s_comp);
        HIPCHK(c, hipGetLastError());
        launch_rec_count(rp, c->s_comp);
        HIPCHK(c, hipGetLastError());
        c->rec_launches++;
    }
    if (e2) HIPCHK(c, hipEventRecord(e2, c->s_comp));
    if (p.used_out) {   // defer_kernel wrote the map's fill level into h_used
        HIPCHK(c, hipEventRecord(c->ev_used, c->s_comp));
        c->used_pending = true;
    }
    c->batches += nin;   // each segment counts as the batch it is
    return YSB_OK;
}

// The JSON layout of a batch's first line l[0, len): 0 the generator's (core.clj:90-96), 1
// the generator's keys in its order as compact JSON, 3 another key order or subset of
// DeserializeBolt's keys with one consistent spacing (", " / ": " or "," / ":") and plain
// string values (36 bytes for the three ids) -- d then holds the order for the scan's
// learned-order instantiation -- and 2 anything else (the flat-object tier first).  Only a
// choice of instantiation: every instantiation counts every line exactly.
static int learn_layout(const u8* l, u64 len, u32 require_mask, LearnDesc* d) {
    static const char* keys[7] = {"user_id", "page_id", "ad_id", "ad_type", "event_type", "event_time", "ip_address"};
    if (len < 2 || l[0] != '{' || l[1] != '"') return 2;
    auto plain_end = [&](u64 q) {   // the closing quote of a plain string from q (len: none)
        while (q < len && l[q] != '"' && l[q] != '\\' && l[q] >= 0x20) ++q;
        return (q < len && l[q] == '"') ? q : len;
    };
    u64 p = 2;
    int cp = -1;
    u32 seen = 0, n = 0, order[8] = {0};
    for (;;) {
        u64 q = plain_end(p);
        if (q >= len) return 2;
        int id = -1;
        for (int i = 0; i < 7; ++i)
            if (std::strlen(keys[i]) == q - p && std::memcmp(l + p, keys[i], q - p) == 0) id = i;
        if (id < 0 || ((seen >> id) & 1u) || n >= 7) return 2;
        seen |= 1u << id;
        order[n++] = (u32)id;
        p = q + 1;
        int c1;
        if (p + 2 < len && l[p] == ':' && l[p + 1] == ' ' && l[p + 2] == '"') { c1 = 0; p += 3; }
        else if (p + 1 < len && l[p] == ':' && l[p + 1] == '"') { c1 = 1; p += 2; }
        else return 2;
        if (cp < 0) cp = c1;
        else if (cp != c1) return 2;
        q = plain_end(p);
        if (q >= len || (id <= 2 && q - p != 36)) return 2;
        p = q + 1;
        if (p < len && l[p] == '}') break;
        if (cp == 0 && p + 2 < len && l[p] == ',' && l[p + 1] == ' ' && l[p + 2] == '"') p += 3;
        else if (cp == 1 && p + 1 < len && l[p] == ',' && l[p + 1] == '"') p += 2;
        else return 2;
    }
    // key index i is bit i of the required-key mask (ysb_scan.hip K_*)
    if ((seen & require_mask) != require_mask || !((seen >> 2) & 1u) || !((seen >> 4) & 1u) || !((seen >> 5) & 1u))
        return 2;
    bool gen_order = n == 7;
    for (u32 i = 0; i < n; ++i) gen_order &= order[i] == i;
    if (gen_order) return cp ? 1 : 0;
    d->n = n;
    d->cp = (u32)cp;
    for (u32 i = 0; i < 8; ++i) d->order[i] = order[i];
    return 3;
}

// The batch's layout from SAMPLE_LINES of its lines (round 4; until round 3 the first line
// only): line 0 and one line at a hashed position in each of the other strata of
// [0, n).  If at least SAMPLE_AGREE of them name the same layout (for 3 the same key order
// and spacing), that one; otherwise several producers are interleaved and the flat-object
// tier, which takes every layout alike, runs first (2).  Only a choice of instantiation:
// every instantiation counts every line exactly.
// 46 of 64 (72 %): a producer writing most of the batch keeps its instantiation (its lines at
// full speed, the others through the tiers); a batch half of one layout (four producers, two
// of them in the generator's layout) reaches 46 of 64 in ~0.03 % of samples (with 32 lines
// and 23 of them: 0.4 %, which a bench seed hit)
constexpr u32 SAMPLE_LINES = 64, SAMPLE_AGREE = 46;
static_assert(SAMPLE_LINES <= (u32)SAMPLE_MAX, "device samples: one SampleSegs entry per line");
#ifndef YSB_MIXED_TILE
#define YSB_MIXED_TILE 1   // round 4: a sample without a majority layout takes the per-tile dispatch (4), not the flat tier (2)
#endif

// Sample line j: pairs of adjacent lines, one pair per stratum of [0, n) in SAMPLE_LINES / 2
// strata (lines 0 and 1, then a hashed position in each other stratum and the line after it)
// -- so the sample also tells producers writing in runs (adjacent lines alike) from a
// line-by-line interleave.
static u64 sample_index(u64 n, u32 j) {
    if (n <= SAMPLE_LINES) return std::min<u64>(j, n ? n - 1 : 0);
    const u64 P = SAMPLE_LINES / 2, q = j >> 1;
    const u64 a = n * q / P, b = n * (q + 1) / P;   // stratum q
    const u64 base = q == 0 ? 0 : a + mix64(0x51ED27u + q) % std::max<u64>(1, b - a - 1);
    return std::min<u64>(base + (j & 1u), n - 1);
}

static int decide_layout(const ysb_ctx* c, const std::vector<std::pair<const u8*, u64>>& lines, LearnDesc* d) {
    const u32 req = (c->cfg.flags & YSB_F_REQUIRE_IP) ? 0x7Fu : 0x3Fu;
    std::vector<std::pair<int, LearnDesc>> got;
    for (const auto& l : lines) {
        LearnDesc di{};
        const int lay = learn_layout(l.first, l.second, req, &di);
        got.push_back({lay, lay == 3 ? di : LearnDesc{}});
    }
    if (got.empty()) return 0;
    u32 best_learned = 0;
    for (const auto& g : got) {   // the most frequent (layout, order) of the sample
        u32 k = 0;
        for (const auto& h : got) k += h.first == g.first && std::memcmp(&h.second, &g.second, sizeof(LearnDesc)) == 0;
        if (k >= std::min<u32>(SAMPLE_AGREE, (u32)got.size())) {
            *d = g.second;
            return g.first;
        }
        if (g.first == 3 && k > best_learned) {   // the most frequent learned order, for layout 4
            best_learned = k;
            *d = g.second;
        }
    }
#if YSB_MIXED_TILE
    // several producers.  Writing in runs (3 of 4 adjacent sample pairs alike): the per-tile
    // dispatch (4) -- tiles of one producer take its path (the learned order: the sample's
    // most frequent one), mixed tiles the flat tier; interleaved line by line: every tile
    // would be mixed, so the flat tier without the dispatch (2)
    u32 pairs = 0, alike = 0;
    for (size_t i = 0; i + 1 < got.size(); i += 2, ++pairs)
        alike += got[i].first == got[i + 1].first &&
                 std::memcmp(&got[i].second, &got[i + 1].second, sizeof(LearnDesc)) == 0;
    if (4 * alike >= 3 * pairs) {
        if (!best_learned) *d = LearnDesc{};
        return 4;
    }
#endif
    return 2;
}

// A host batch (held in the pinned slot).
static int sniff_layout(const ysb_ctx* c, const uint8_t* bytes, u64 nbytes, const u32* off, u64 n, LearnDesc* d) {
    std::vector<std::pair<const u8*, u64>> lines;
    for (u32 j = 0; j < SAMPLE_LINES && j < n; ++j) {
        const u64 i = sample_index(n, j);
        const u64 s = off[i], e = i + 1 < n ? (u64)off[i + 1] : nbytes;
        if (s >= e || e > nbytes) return 0;   // bad offsets: the scan defers them anyway
        lines.push_back({bytes + s, std::min<u64>(e - s, SAMPLE_BYTES)});
    }
    return decide_layout(c, lines, d);
}

// Whether batches pick the scan instantiation from their first line (the default): not
// with YSB_F_COMPACT_FIRST or YSB_F_LAYOUT_FIXED, and only where the layout instantiations
// exist (JSON: the cache-resident table's and, since round 4, the HBM-resident table's
// serial-probe and record-mode kernels).  Under YSB_F_FLAT_FIRST the sample only tells
// whether the batch has one learnable key order (hinted_layout).
static bool layout_sampling(const ysb_ctx* c) {
    const u32 f = c->cfg.flags;
    return !(f & (YSB_F_LAYOUT_FIXED | YSB_F_COMPACT_FIRST | YSB_F_FORMAT_TBL));
}

// The sampled layout under the flags' hint: YSB_F_FLAT_FIRST keeps the flat-object tier
// first unless the first line names a key order (3: the learned-order instantiation, whose
// lines off that order go to the same flat tier).
static int hinted_layout(const ysb_ctx* c, int sampled) {
    if ((c->cfg.flags & YSB_F_FLAT_FIRST) && sampled >= 0 && sampled != 3 && sampled != 4) return 2;
    return sampled;
}

// Device batches: SAMPLE_LINES lines spread over the launch's segments (as sniff_layout
// spreads them over a host batch), copied by sample_kernel on the compute stream -- in
// stream order, so after whatever produced the batch there (the caller's contract: a device
// batch is complete when submitted, or its producer is ordered before ysb_stream(ctx)) --
// into one of two pinned buffers.  Which sample decides: this launch's own when the compute
// stream was idle at the submit (the copy finishes in microseconds) or no earlier sample
// exists; otherwise the previous launch's, read without waiting for the device (one launch
// late: a producer writes one layout, and counts do not depend on the choice).
static int sample_device_layout(ysb_ctx* c, const ysb_segment* segs, u32 nseg, LearnDesc* d) {
    const u64 buf = (u64)SAMPLE_LINES * SAMPLE_STRIDE;
    if (!c->h_sample) {
        HIPCHK(c, hipHostMalloc(&c->h_sample, 2 * buf));
        for (hipEvent_t& e : c->ev_sample) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const bool idle = hipStreamQuery(c->s_comp) == hipSuccess;
    const int k = c->sample_cur;
    c->sample_cur ^= 1;
    u64 total = 0;
    for (u32 i = 0; i < nseg; ++i) total += segs[i].n_events;
    SampleSegs ss{};
    u32 n = 0;
    for (u32 j = 0; j < SAMPLE_LINES && j < total; ++j) {
        u64 g = sample_index(total, j), i = 0;   // global line -> (segment, line)
        while (g >= segs[i].n_events) g -= segs[i++].n_events;
        ss.bytes[n] = segs[i].d_bytes;
        ss.off[n] = segs[i].d_line_off;
        ss.nbytes[n] = segs[i].nbytes;
        ss.n[n] = segs[i].n_events;
        ss.line[n] = g;
        ++n;
    }
    launch_sample(ss, n, c->h_sample + (u64)k * buf, c->s_comp);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev_sample[k], c->s_comp));
    c->sample_nseg[k] = n;
    const int use = (!idle && c->sample_nseg[k ^ 1]) ? k ^ 1 : k;
    HIPCHK(c, hipEventSynchronize(c->ev_sample[use]));
    const u8* h = c->h_sample + (u64)use * buf;
    std::vector<std::pair<const u8*, u64>> lines;
    for (u32 i = 0; i < c->sample_nseg[use]; ++i) {
        const u8* sp = h + (u64)i * SAMPLE_STRIDE;
        u32 hd[3];
        std::memcpy(hd, sp, 12);
        if (!hd[2]) return 0;   // bad offsets: the scan defers them anyway
        lines.push_back({sp + 16, hd[1]});
    }
    return decide_layout(c, lines, d);
}

// With YSB_F_TIMING: an event pair around a slot's H2D copy (ysb_copy_time), else none.
static int copy_events(ysb_ctx* c, hipEvent_t** out, u64 bytes) {
    *out = nullptr;
    if (!(c->cfg.flags & YSB_F_TIMING)) return YSB_OK;
    if (c->cev_used == c->cev.size()) {
        std::array<hipEvent_t, 2> ev{};
        for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
        c->cev.push_back(ev);
    }
    *out = c->cev[c->cev_used++].data();
    c->copy_bytes += bytes;
    return YSB_OK;
}

static int ensure_slots(ysb_ctx* c) {
    if (c->h_bytes[0]) return YSB_OK;
    HIPCHK(c, hipSetDevice(c->device));
    for (int s = 0; s < 2; ++s) {
        HIPCHK(c, hipHostMalloc(&c->h_bytes[s], c->cfg.max_batch_bytes + 64));
        HIPCHK(c, hipHostMalloc(&c->h_off[s], c->cfg.max_batch_events * 4 + 64));
        HIPCHK(c, hipMalloc(&c->d_bytes[s], c->cfg.max_batch_bytes + 64));
        HIPCHK(c, hipMalloc(&c->d_off[s], c->cfg.max_batch_events * 4 + 64));
    }
    return YSB_OK;
}

int ysb_slot_buffers(ysb_ctx* c, int slot, uint8_t** bytes, uint32_t** line_off) {
    if (!c || slot < 0 || slot > 1) return c ? fail(c, YSB_ERR_ARG, "slot must be 0 or 1") : YSB_ERR_ARG;
    int rc = ensure_slots(c);
    if (rc) return rc;
    if (bytes) *bytes = c->h_bytes[slot];
    if (line_off) *line_off = c->h_off[slot];
    return YSB_OK;
}

int ysb_submit(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes, const uint32_t* line_off,
               uint64_t n) {
    if (!c) return YSB_ERR_ARG;
    if (slot < 0 || slot > 1) return fail(c, YSB_ERR_ARG, "slot must be 0 or 1");
    if (nbytes > c->cfg.max_batch_bytes || n > c->cfg.max_batch_events)
        return fail(c, YSB_ERR_CAPACITY, "batch (%llu B, %llu events) exceeds max_batch_bytes/max_batch_events",
                    (unsigned long long)nbytes, (unsigned long long)n);
    if ((nbytes && !bytes) || (n && !line_off)) return fail(c, YSB_ERR_ARG, "NULL batch buffers");
    int rc = launch_pending_raw(c);   // batches launch in submission order
    if (!rc) rc = ensure_slots(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    // the slot's previous H2D must be done before its pinned buffers are rewritten
    HIPCHK(c, hipEventSynchronize(c->ev_h2d[slot]));
    if (bytes != c->h_bytes[slot] && nbytes) std::memcpy(c->h_bytes[slot], bytes, nbytes);
    if (line_off != c->h_off[slot] && n) std::memcpy(c->h_off[slot], line_off, n * 4);
    // ... and the slot's previous kernel must be done before its device buffers are
    HIPCHK(c, hipStreamWaitEvent(c->s_copy, c->ev_kdone[slot], 0));
    hipEvent_t* ce = nullptr;
    if ((rc = copy_events(c, &ce, nbytes + n * 4))) return rc;
    if (ce) HIPCHK(c, hipEventRecord(ce[0], c->s_copy));
    if (nbytes) HIPCHK(c, hipMemcpyAsync(c->d_bytes[slot], c->h_bytes[slot], nbytes, hipMemcpyHostToDevice, c->s_copy));
    if (n) HIPCHK(c, hipMemcpyAsync(c->d_off[slot], c->h_off[slot], n * 4, hipMemcpyHostToDevice, c->s_copy));
    if (ce) HIPCHK(c, hipEventRecord(ce[1], c->s_copy));
    HIPCHK(c, hipEventRecord(c->ev_h2d[slot], c->s_copy));
    HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_h2d[slot], 0));
    const ysb_segment sg{c->d_bytes[slot], nbytes, c->d_off[slot], n};
    // the scan instantiation named by the batch's first line, which the host holds in the
    // pinned slot (counts are the same whichever runs)
    if (layout_sampling(c) && n)
        c->submit_layout =
            hinted_layout(c, sniff_layout(c, c->h_bytes[slot], nbytes, c->h_off[slot], n, &c->submit_learn));
    rc = enqueue_scan(c, &sg, 1);
    c->submit_layout = -1;
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(c->ev_kdone[slot], c->s_comp));
    return YSB_OK;
}

int ysb_wait(ysb_ctx* c, int slot) {
    if (!c) return YSB_ERR_ARG;
    if (slot < 0 || slot > 1) return fail(c, YSB_ERR_ARG, "slot must be 0 or 1");
    if (!c->h_bytes[0]) return YSB_OK;
    HIPCHK(c, hipEventSynchronize(c->ev_h2d[slot]));
    return YSB_OK;
}

// ---- raw batches (ysb_submit_raw): the line split on the GPU ----------------------------------

static int ensure_raw(ysb_ctx* c) {
    if (c->h_rawn) return YSB_OK;
    HIPCHK(c, hipSetDevice(c->device));
    for (int s = 0; s < 2; ++s) {   // (a failed earlier attempt may have left some of these)
        hipFree(c->d_roff[s]);
        c->d_roff[s] = nullptr;
        HIPCHK(c, hipMalloc(&c->d_roff[s], (c->cfg.max_batch_bytes + 1) * 4));   // n <= nbytes lines
        if (!c->ev_raw[s]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_raw[s], hipEventDisableTiming));
    }
    if (!c->s_split) HIPCHK(c, hipStreamCreateWithFlags(&c->s_split, hipStreamNonBlocking));
    const u64 words = split_chunks(c->cfg.max_batch_bytes) + 1;
    if (c->split_chunk_words < words) {
        hipFree(c->d_split_chunk);
        c->d_split_chunk = nullptr;
        c->split_chunk_words = 0;
        HIPCHK(c, hipMalloc(&c->d_split_chunk, words * 4));
        c->split_chunk_words = words;
    }
    HIPCHK(c, hipHostMalloc(&c->h_rawn, 16));
    return YSB_OK;
}

// The raw batch waiting for its launch (if any): its line count is back from the device
// (ev_raw), so its scan is enqueued now -- the order of submission is kept.
static int launch_pending_raw(ysb_ctx* c) {
    if (c->raw_pend < 0) return YSB_OK;
    const int slot = c->raw_pend;
    c->raw_pend = -1;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipEventSynchronize(c->ev_raw[slot]));
    HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_raw[slot], 0));
    const ysb_segment sg{c->d_bytes[slot], c->raw_nbytes[slot], c->d_roff[slot], c->h_rawn[slot]};
    c->submit_layout = c->raw_layout[slot];
    c->submit_learn = c->raw_learn[slot];
    const int rc = enqueue_scan(c, &sg, 1);
    c->submit_layout = -1;
    // the slot's device buffers are free again once this launch has run
    HIPCHK(c, hipEventRecord(c->ev_kdone[slot], c->s_comp));
    return rc;
}

// The layout of a raw batch (host bytes): its first line and the first complete line after
// each of SAMPLE_LINES - 1 spread byte positions, decided as sniff_layout decides.
static int sniff_raw(const ysb_ctx* c, const u8* b, u64 nbytes, LearnDesc* d) {
    auto line_at = [&](u64 p) -> std::pair<const u8*, u64> {   // the line starting at p
        const u64 lim = std::min<u64>(nbytes, p + SAMPLE_BYTES);
        u64 e = p;
        while (e < lim && b[e] != '\n' && b[e] != '\r') ++e;
        return {b + p, std::min<u64>(e + 1, nbytes) - p};
    };
    // pairs of adjacent lines (as sample_index): the first two, then the two after a '\n' at
    // each other stratum's start (a lone '\r' only ends lines elsewhere)
    auto next_start = [&](u64 p) -> u64 {   // past the '\n' at or after p (nbytes: none near)
        const u64 lim = std::min<u64>(nbytes, p + 4096);
        while (p < lim && b[p] != '\n') ++p;
        return p + 1 < lim ? p + 1 : nbytes;
    };
    std::vector<std::pair<const u8*, u64>> lines;
    for (u32 q = 0; q < SAMPLE_LINES / 2; ++q) {
        const u64 s0 = q == 0 ? 0 : next_start(nbytes * q / (SAMPLE_LINES / 2));
        if (s0 >= nbytes) continue;
        const u64 s1 = next_start(s0);
        if (s1 >= nbytes) continue;   // a pair or nothing
        lines.push_back(line_at(s0));
        lines.push_back(line_at(s1));
    }
    if (lines.empty()) lines.push_back(line_at(0));
    return decide_layout(c, lines, d);
}

int ysb_submit_raw(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes) {
    if (!c) return YSB_ERR_ARG;
    if (slot < 0 || slot > 1) return fail(c, YSB_ERR_ARG, "slot must be 0 or 1");
    if (nbytes > c->cfg.max_batch_bytes)
        return fail(c, YSB_ERR_CAPACITY, "raw batch of %llu B exceeds max_batch_bytes", (unsigned long long)nbytes);
    if (nbytes && !bytes) return fail(c, YSB_ERR_ARG, "NULL batch buffer");
    if (!c->table_loaded) return fail(c, YSB_ERR_STATE, "ysb_load_ad_map has not been called");
    // the slot's own earlier batch launches first (its device buffers are about to be reused)
    int rc = c->raw_pend == slot ? launch_pending_raw(c) : YSB_OK;
    if (!rc) rc = ensure_slots(c);
    if (!rc) rc = ensure_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    // the slot's previous H2D must be done before its pinned buffer is rewritten
    HIPCHK(c, hipEventSynchronize(c->ev_h2d[slot]));
    if (bytes != c->h_bytes[slot] && nbytes) std::memcpy(c->h_bytes[slot], bytes, nbytes);
    c->raw_layout[slot] = -1;
    if (layout_sampling(c) && nbytes)
        c->raw_layout[slot] = hinted_layout(c, sniff_raw(c, c->h_bytes[slot], nbytes, &c->raw_learn[slot]));
    // H2D once the slot's previous kernel has run; the split on a stream of its own, so the
    // next slot's copy queues right behind this one
    HIPCHK(c, hipStreamWaitEvent(c->s_copy, c->ev_kdone[slot], 0));
    hipEvent_t* ce = nullptr;
    if ((rc = copy_events(c, &ce, nbytes))) return rc;
    if (ce) HIPCHK(c, hipEventRecord(ce[0], c->s_copy));
    if (nbytes) HIPCHK(c, hipMemcpyAsync(c->d_bytes[slot], c->h_bytes[slot], nbytes, hipMemcpyHostToDevice, c->s_copy));
    if (ce) HIPCHK(c, hipEventRecord(ce[1], c->s_copy));
    HIPCHK(c, hipEventRecord(c->ev_h2d[slot], c->s_copy));
    HIPCHK(c, hipStreamWaitEvent(c->s_split, c->ev_h2d[slot], 0));
    if (nbytes) {
        // the line count goes straight to pinned memory (read at the launch)
        HIPCHK(c, launch_split_lines(c->d_bytes[slot], nbytes, c->d_split_chunk, c->d_roff[slot],
                                     c->cfg.max_batch_bytes + 1, c->h_rawn + slot, c->s_split));
    } else {
        c->h_rawn[slot] = 0;
    }
    HIPCHK(c, hipEventRecord(c->ev_raw[slot], c->s_split));
    c->raw_nbytes[slot] = nbytes;
    // the other slot's batch, submitted before this one, launches now; this one at the next call
    rc = launch_pending_raw(c);
    c->raw_pend = slot;
    return rc;
}

int ysb_split_lines_device(ysb_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, uint32_t* d_off, uint64_t cap,
                           uint64_t* n) {
    if (!c || !n) return c ? fail(c, YSB_ERR_ARG, "n is NULL") : YSB_ERR_ARG;
    if (nbytes > (4ull << 30) - 64) return fail(c, YSB_ERR_CAPACITY, "batch larger than 4 GiB (u32 offsets)");
    if ((nbytes && !d_bytes) || (cap && !d_off)) return fail(c, YSB_ERR_ARG, "NULL buffers");
    if (reinterpret_cast<uintptr_t>(d_bytes) & 15) return fail(c, YSB_ERR_ARG, "d_bytes must be 16-byte aligned");
    int rc = launch_pending_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    const u64 words = split_chunks(nbytes) + 1;
    if (c->split_chunk_words < words) {
        if (c->s_split) HIPCHK(c, hipStreamSynchronize(c->s_split));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        hipFree(c->d_split_chunk);
        c->d_split_chunk = nullptr;
        c->split_chunk_words = 0;
        HIPCHK(c, hipMalloc(&c->d_split_chunk, words * 4));
        c->split_chunk_words = words;
    }
    if (!c->d_cmp) HIPCHK(c, hipMalloc(&c->d_cmp, 32));
    unsigned long long* d_n = c->d_cmp + 3;
    HIPCHK(c, launch_split_lines(d_bytes, nbytes, c->d_split_chunk, d_off, cap, d_n, c->s_comp));
    unsigned long long got = 0;
    HIPCHK(c, hipMemcpyAsync(&got, d_n, 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    *n = got;
    if (got > cap) return fail(c, YSB_ERR_CAPACITY, "%llu lines, cap %llu", (unsigned long long)got, (unsigned long long)cap);
    return YSB_OK;
}

int ysb_slot_capacity(ysb_ctx* c, uint64_t* max_bytes, uint64_t* max_events) {
    if (!c) return YSB_ERR_ARG;
    if (max_bytes) *max_bytes = c->cfg.max_batch_bytes;
    if (max_events) *max_events = c->cfg.max_batch_events;
    return YSB_OK;
}

int ysb_copy_time(ysb_ctx* c, double* total_ms, uint64_t* copies, uint64_t* bytes) {
    if (!c) return YSB_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->s_copy));
    double t = 0;
    for (size_t i = 0; i < c->cev_used; ++i) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->cev[i][0], c->cev[i][1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (copies) *copies = c->cev_used;
    if (bytes) *bytes = c->copy_bytes;
    c->cev_used = 0;
    c->copy_bytes = 0;
    return YSB_OK;
}

// Device batches: the layout sampled from their first lines (unless fixed), then the launch.
static int enqueue_device(ysb_ctx* c, const ysb_segment* segs, u32 nseg) {
    int prc = launch_pending_raw(c);   // batches launch in submission order
    if (prc) return prc;
    if (c->table_loaded && layout_sampling(c)) {
        const int lay = sample_device_layout(c, segs, nseg, &c->submit_learn);
        if (lay < 0) return lay;
        c->submit_layout = hinted_layout(c, lay);
    }
    const int rc = enqueue_scan(c, segs, nseg);
    c->submit_layout = -1;
    return rc;
}

int ysb_submit_device(ysb_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const uint32_t* d_off, uint64_t n) {
    if (!c) return YSB_ERR_ARG;
    if (nbytes > (4ull << 30) - 64) return fail(c, YSB_ERR_CAPACITY, "device batch larger than 4 GiB (u32 offsets)");
    if ((nbytes && !d_bytes) || (n && !d_off)) return fail(c, YSB_ERR_ARG, "NULL batch buffers");
    if (reinterpret_cast<uintptr_t>(d_bytes) & 15) return fail(c, YSB_ERR_ARG, "d_bytes must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->device));
    const ysb_segment sg{d_bytes, nbytes, d_off, n};
    return enqueue_device(c, &sg, 1);
}

int ysb_submit_device_segments(ysb_ctx* c, const ysb_segment* segs, uint32_t n_segs) {
    if (!c) return YSB_ERR_ARG;
    if (n_segs > (u32)MAX_SEGS) return fail(c, YSB_ERR_CAPACITY, "at most %d segments per launch", MAX_SEGS);
    if (n_segs && !segs) return fail(c, YSB_ERR_ARG, "NULL segment list");
    for (u32 i = 0; i < n_segs; ++i) {
        const ysb_segment& s = segs[i];
        if (s.nbytes > (4ull << 30) - 64)
            return fail(c, YSB_ERR_CAPACITY, "segment %u larger than 4 GiB (u32 offsets)", i);
        if ((s.nbytes && !s.d_bytes) || (s.n_events && !s.d_line_off))
            return fail(c, YSB_ERR_ARG, "NULL buffers in segment %u", i);
        if (reinterpret_cast<uintptr_t>(s.d_bytes) & 15)
            return fail(c, YSB_ERR_ARG, "segment %u: d_bytes must be 16-byte aligned", i);
    }
    HIPCHK(c, hipSetDevice(c->device));
    return enqueue_device(c, segs, n_segs);
}

static int sync_streams(ysb_ctx* c) {
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

static int pull_side_list(ysb_ctx* c);

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

static int read_ring(ysb_ctx* c) {
    i64 r[2];
    HIPCHK(c, hipMemcpy(r, c->d_ring, 16, hipMemcpyDeviceToHost));
    if (r[1]) { c->ring_known = true; c->ring_lo = r[0]; }
    c->ring_query_pending = false;
    return YSB_OK;
}

static int pull_side_list(ysb_ctx* c) {
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
static int move_ring(ysb_ctx* c, i64 new_lo) {
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
    int rc = sync_streams(c);
    if (rc) return rc;
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
    double t = 0, tp = 0;
    for (size_t i = 0; i < c->tev_used; ++i) {
        float ms = 0, mp = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->tev[i][0], c->tev[i][1]));
        HIPCHK(c, hipEventElapsedTime(&mp, c->tev[i][0], c->tev[i][2]));
        t += ms;
        tp += mp;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = c->tev_used;
    c->path_ms_acc = tp;
    c->path_launches_acc = c->tev_used;
    c->tev_used = 0;
    return YSB_OK;
}

int ysb_path_time(ysb_ctx* c, double* total_ms, uint64_t* launches, uint64_t* record_launches) {
    if (!c) return YSB_ERR_ARG;
    if (total_ms) *total_ms = c->path_ms_acc;
    if (launches) *launches = c->path_launches_acc;
    if (record_launches) *record_launches = c->rec_launches;
    return YSB_OK;
}

int ysb_layout_of_line(const uint8_t* line, uint64_t len, int require_ip, uint32_t order[8], uint32_t* n,
                       uint32_t* compact) {
    if (!line && len) return YSB_ERR_ARG;
    LearnDesc d{};
    const int l = learn_layout(line, len, require_ip ? 0x7Fu : 0x3Fu, &d);
    if (order) for (int i = 0; i < 8; ++i) order[i] = d.order[i];
    if (n) *n = l == 3 ? d.n : 0;
    if (compact) *compact = l == 3 ? d.cp : (l == 1 ? 1u : 0u);
    return l;
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
    launch_pending_raw(c);   // work the caller orders after it follows every submitted batch
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

// ---- multi-GPU ---------------------------------------------------------------------------------

static bool grouped(const ysb_ctx* c) { return c->comm != nullptr || c->host_coll; }

// d[0..n) <- elementwise max over the ranks, in place: one RCCL all-reduce on the compute
// stream, or (host collectives) the buffer through host memory and the caller's all-reduce.
static int coll_max_u64(ysb_ctx* c, unsigned long long* d, u64 n) {
    if (c->comm) {
        ncclResult_t r = ncclAllReduce(d, d, n, ncclUint64, ncclMax, c->comm, c->s_comp);
        if (r != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
        return YSB_OK;
    }
    std::vector<uint64_t> h(n);
    HIPCHK(c, hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (c->hops.allreduce_max_u64(c->hops.user, h.data(), n))
        return fail(c, YSB_ERR_RCCL, "host all-reduce(max) failed");
    HIPCHK(c, hipMemcpyAsync(d, h.data(), n * 8, hipMemcpyHostToDevice, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    return YSB_OK;
}

// recv[0..count) <- sum over the ranks of their send blocks [rank * count, (rank + 1) * count),
// cells of `width` bytes (1, 4 or 8, unsigned).
static int coll_reduce_scatter(ysb_ctx* c, const void* d_send, void* d_recv, u64 count, u32 width, hipStream_t st) {
    if (c->comm) {
        const ncclDataType_t ty = width == 1 ? ncclUint8 : width == 4 ? ncclUint32 : ncclUint64;
        ncclResult_t r = ncclReduceScatter(d_send, d_recv, (size_t)count, ty, ncclSum, c->comm, st);
        if (r != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclReduceScatter: %s", ncclGetErrorString(r));
        return YSB_OK;
    }
    const u64 nb = count * width;
    std::vector<u8> hs(nb * (u64)c->nranks), hr(nb);
    HIPCHK(c, hipMemcpyAsync(hs.data(), d_send, hs.size(), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (c->hops.reduce_scatter_sum(c->hops.user, hs.data(), hr.data(), count, width))
        return fail(c, YSB_ERR_RCCL, "host reduce-scatter failed");
    HIPCHK(c, hipMemcpyAsync(d_recv, hr.data(), nb, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return YSB_OK;
}

// h[0..n) <- elementwise max over the ranks (signed: mapped to unsigned by the sign bit).
static int allreduce_max(ysb_ctx* c, i64* h, int n) {
    unsigned long long* d = nullptr;
    HIPCHK(c, hipMalloc(&d, 8 * (u64)n));
    std::vector<u64> u(n);
    for (int i = 0; i < n; ++i) u[i] = (u64)h[i] ^ (1ull << 63);
    hipError_t e = hipMemcpy(d, u.data(), 8 * (u64)n, hipMemcpyHostToDevice);
    int rc = e == hipSuccess ? coll_max_u64(c, d, (u64)n) : YSB_OK;
    if (e == hipSuccess && !rc) e = hipMemcpyAsync(u.data(), d, 8 * (u64)n, hipMemcpyDeviceToHost, c->s_comp);
    if (e == hipSuccess && !rc) e = hipStreamSynchronize(c->s_comp);
    hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return fail(c, YSB_ERR_HIP, "%s", hipGetErrorString(e));
    for (int i = 0; i < n; ++i) h[i] = (i64)(u[i] ^ (1ull << 63));
    return YSB_OK;
}

// Ring-base agreement (collective: every rank calls it at the same point and takes the
// same decision from the reduced values, so no rank skips a collective the others
// enter).  The common base is the smallest base any rank holds.  A rank whose ring
// starts later moves the buckets the common range no longer holds, [common + W, lo + W),
// to its exact host-side list (cells are indexed by bucket mod W, so the rest stays in
// place); a rank without a base takes the common one.  Skewed per-rank streams
// (core.clj:166-174) that auto-based differently therefore still exchange.
static int agree_ring(ysb_ctx* c) {
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    int rc = read_ring(c);
    if (rc) return rc;
    i64 h[2] = {c->ring_known ? -c->ring_lo : INT64_MIN + 1, c->ring_known ? 1 : 0};
    if ((rc = allreduce_max(c, h, 2))) return rc;
    if (!h[1]) return YSB_OK;   // no rank has a base yet: agreed at the next exchange
    if ((rc = move_ring(c, -h[0]))) return rc;
    c->ring_agreed = true;
    return YSB_OK;
}

int ysb_group_unique_id(uint8_t uid[YSB_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == YSB_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail(nullptr, YSB_ERR_RCCL, "ncclGetUniqueId failed");
    std::memcpy(uid, &id, sizeof id);
    return YSB_OK;
}

static int group_setup(ysb_ctx* c, int rank, int nranks);
static void ungroup(ysb_ctx* c);

int ysb_group_init(ysb_ctx* c, int rank, int nranks, const uint8_t uid[YSB_UNIQUE_ID_BYTES]) {
    if (!c || !uid) return YSB_ERR_ARG;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, YSB_ERR_ARG, "bad rank %d / %d", rank, nranks);
    if (grouped(c)) return fail(c, YSB_ERR_STATE, "group already initialised");
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return fail(c, YSB_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    const int rc = group_setup(c, rank, nranks);
    if (rc) ungroup(c);
    return rc;
}

int ysb_group_init_host(ysb_ctx* c, int rank, int nranks, const ysb_collectives* ops) {
    if (!c || !ops || !ops->allreduce_max_u64 || !ops->reduce_scatter_sum) return YSB_ERR_ARG;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, YSB_ERR_ARG, "bad rank %d / %d", rank, nranks);
    if (grouped(c)) return fail(c, YSB_ERR_STATE, "group already initialised");
    HIPCHK(c, hipSetDevice(c->device));
    c->hops = *ops;
    c->host_coll = true;
    const int rc = group_setup(c, rank, nranks);
    if (rc) ungroup(c);
    return rc;
}

// A failed group init leaves the context ungrouped (and a later ysb_group_init possible):
// the communicator, the exchange buffers and the owned table go; the counts stay.
static void ungroup(ysb_ctx* c) {
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->host_coll = false;
    c->hops = ysb_collectives{};
    hipFree(c->d_owned);
    c->d_owned = nullptr;
    hipFree(c->d_owned8);
    c->d_owned8 = nullptr;
    c->owned8_dirty = false;
    hipFree(c->d_xmax);
    c->d_xmax = nullptr;
    hipHostFree(c->h_xmax);
    c->h_xmax = nullptr;
    hipFree(c->d_xslots);
    c->d_xslots = nullptr;
    for (hipEvent_t& e : c->xplan_ev) {
        if (e) hipEventDestroy(e);
        e = nullptr;
    }
    for (int k = 0; k < 2; ++k) {
        if (c->ev_xpacked[k]) hipEventDestroy(c->ev_xpacked[k]);
        if (c->ev_xdone[k]) hipEventDestroy(c->ev_xdone[k]);
        c->ev_xpacked[k] = c->ev_xdone[k] = nullptr;
        c->xset_used[k] = false;
    }
    c->unpack_set = -1;
    c->rank = 0;
    c->nranks = 1;
    c->ring_agreed = false;
    c->x_have_plan = false;
}

static int group_setup(ysb_ctx* c, int rank, int nranks) {
    int prc = launch_pending_raw(c);
    if (prc) return prc;
    c->rank = rank;
    c->nranks = nranks;
    // pad campaigns to a multiple of nranks; keep the current counts
    const u32 cp = (c->cfg.n_campaigns + nranks - 1) / nranks * nranks;
    if (cp != c->c_pad) {
        int frc = fold_delta(c);   // the delta ring has the old layout: fold it, drop it
        if (frc) return frc;
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        hipFree(c->d_delta);
        c->d_delta = nullptr;
        c->delta_cells = 0;
        unsigned long long* old = c->d_counts;
        const u64 W = c->cfg.window_ring;
        c->d_counts = nullptr;
        HIPCHK(c, hipMalloc(&c->d_counts, (u64)cp * W * 8));
        HIPCHK(c, hipMemset(c->d_counts, 0, (u64)cp * W * 8));
        HIPCHK(c, hipMemcpy(c->d_counts, old, (u64)c->c_pad * W * 8, hipMemcpyDeviceToDevice));
        hipFree(old);
        if (c->d_truth) {   // the generator-truth table has the ring's layout: grow it too
            unsigned long long* ot = c->d_truth;
            c->d_truth = nullptr;
            HIPCHK(c, hipMalloc(&c->d_truth, (u64)cp * W * 8));
            HIPCHK(c, hipMemset(c->d_truth, 0, (u64)cp * W * 8));
            HIPCHK(c, hipMemcpy(c->d_truth, ot, (u64)c->c_pad * W * 8, hipMemcpyDeviceToDevice));
            hipFree(ot);
        }
        c->c_pad = cp;
    }
    const u64 per = (u64)c->c_pad / nranks * c->cfg.window_ring;
    HIPCHK(c, hipMalloc(&c->d_owned, per * 8));
    HIPCHK(c, hipMemset(c->d_owned, 0, per * 8));
    HIPCHK(c, hipMalloc(&c->d_owned8, per));
    HIPCHK(c, hipMemset(c->d_owned8, 0, per));
    const u32 W = c->cfg.window_ring;
    HIPCHK(c, hipMalloc(&c->d_xmax, 2 * (u64)W * 8));
    HIPCHK(c, hipHostMalloc(&c->h_xmax, 2 * ((u64)W * 8 + (u64)W * 4)));   // maxima, then the plans' slots
    HIPCHK(c, hipMalloc(&c->d_xslots, 2 * (u64)W * 4));
    for (hipEvent_t& e : c->xplan_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int k = 0; k < 2; ++k) {
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_xpacked[k], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_xdone[k], hipEventDisableTiming));
        c->xset_used[k] = false;
    }
    if (!c->s_x) HIPCHK(c, hipStreamCreateWithFlags(&c->s_x, hipStreamNonBlocking));
    c->x_have_plan = false;
    // every rank's ring must start at the same bucket (the tables are summed cell by
    // cell): agreed here if any rank already knows its base, else at the first exchange
    return agree_ring(c);
}

static int grow_bytes(ysb_ctx* c, void** buf, u64* have, u64 bytes) {
    if (*have >= bytes) return YSB_OK;
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (c->s_x) HIPCHK(c, hipStreamSynchronize(c->s_x));
    hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    const u64 b = std::max<u64>(bytes, 1ull << 16);
    HIPCHK(c, hipMalloc(buf, b));
    *have = b;
    return YSB_OK;
}

int ysb_exchange_plan(const uint64_t* slot_max, uint32_t W, uint32_t nranks, uint32_t* slots, uint32_t* n_slots,
                      uint32_t* width) {
    if (!slot_max || !slots || !n_slots || !width || nranks == 0 || W == 0) return YSB_ERR_ARG;
    u32 n = 0;
    u64 mx = 0;
    for (u32 s = 0; s < W; ++s)
        if (slot_max[s]) {
            slots[n++] = s;
            mx = std::max<u64>(mx, slot_max[s]);
        }
    // the narrowest cell whose sum over the ranks cannot wrap: nranks * max < 2^(8 width)
    // (RCCL has no 16-bit integer type)
    const unsigned __int128 bound = (unsigned __int128)mx * nranks;
    *width = bound <= 0xFFu ? 1u : bound <= 0xFFFFFFFFull ? 4u : 8u;
    if (bound > ~0ull) return YSB_ERR_CAPACITY;
    *n_slots = n;
    return YSB_OK;
}

// The keyBy(0) exchange (AdvertisingTopologyNative.java:118-119), range-limited: only the
// ring slots that hold a pending count on some rank travel, in the narrowest cell width
// that cannot wrap, as the reference's keyed shuffle carries only the touched (campaign,
// window) pairs.  Steps on the compute stream: per-slot maxima of the pending counts
// (xplan) -> one W-element all-reduce(max) -> read back -> plan (ysb_exchange_plan: the
// same on every rank) -> pack the slots' cells [C_pad][R] and zero them (xpack) ->
// ncclReduceScatter -> add the owner block into the owned table (xunpack).
//
// Complete (pipelined false): the plan is this call's, read back with a host wait; every
// pending count travels.  Pipelined: this call's plan is only enqueued (reduced into the
// other buffer, read back by an async copy) and the pack uses the previous call's plan,
// whose read-back finished while the step's scan ran -- no host wait, so the next launch
// queues behind the exchange without a gap.  Counts in slots outside that plan, or above
// what its width sums over the ranks (cap), stay pending for a later exchange; the first
// call after group init / reset / ring advance is complete.
// The recorded exchange timing pairs into x_ms (waits for the last of them).
// The unpack of the last exchange (owner block += received cells), on the compute stream
// once its reduce-scatter is done; a no-op when none is pending.
static int finish_unpack(ysb_ctx* c) {
    if (c->unpack_set < 0) return YSB_OK;
    const int k = c->unpack_set;
    c->unpack_set = -1;
    const u32 W = c->cfg.window_ring, per = c->c_pad / (u32)c->nranks;
    const auto& ev = c->xev[c->unpack_entry];
    HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_xdone[k], 0));
    HIPCHK(c, hipEventRecord(ev[3], c->s_comp));
    launch_xunpack(c->d_owned, c->d_owned8, W, per, c->d_xslots + (u64)k * W, c->unpack_R, c->d_xrecv[k],
                   c->unpack_width, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->owned8_dirty = true;
    HIPCHK(c, hipEventRecord(ev[4], c->s_comp));
    return YSB_OK;
}

// The recorded exchange timing into x_ms (plan to the end of the reduce-scatter, plus the
// unpack) and x_crit_ms (the compute stream's share: plan to pack, plus the unpack); waits
// for the last of them.  Call after finish_unpack.
static int collect_xev(ysb_ctx* c) {
    for (size_t i = 0; i < c->xev_used; ++i) {
        float ms = 0, mc = 0, mu = 0;
        const auto& ev = c->xev[i];
        HIPCHK(c, hipEventSynchronize(ev[2]));
        HIPCHK(c, hipEventSynchronize(ev[4]));
        HIPCHK(c, hipEventElapsedTime(&ms, ev[0], ev[2]));
        HIPCHK(c, hipEventElapsedTime(&mc, ev[0], ev[1]));
        HIPCHK(c, hipEventElapsedTime(&mu, ev[3], ev[4]));
        c->x_ms += ms + mu;
        c->x_crit_ms += mc + mu;
    }
    c->xev_used = 0;
    return YSB_OK;
}

// The plan's ascending slot list widened to whole aligned groups of four: every run of
// consecutive slots grows to [floor4(first), ceil4(last + 1)) (W is a power of two >= 16, so
// the groups never pass W), so the u8 pack / unpack move each group as one u32 of the ring
// (ysb_table.hip xpack8_kernel: a group that is not four consecutive aligned slots takes
// per-cell steps).  An added slot held no pending count anywhere when the plan was made: it
// sends zeros -- or, in a pipelined exchange whose plan is one call old, a count that arrived
// since, within the width's cap like any planned slot.  At most three extra slots per run
// end.  In place (the list has W entries); returns the new length, a multiple of 4.
static u32 align_slot_runs(u32* slots, u32 R, u32 W) {
    std::vector<u32> out;
    out.reserve(R + 8);
    for (u32 i = 0; i < R;) {
        u32 j = i + 1;
        while (j < R && slots[j] == slots[j - 1] + 1) ++j;
        const u32 a = slots[i] & ~3u, b = std::min<u32>((slots[j - 1] + 4) & ~3u, W);
        for (u32 sl = std::max<u32>(a, out.empty() ? 0u : out.back() + 1); sl < b; ++sl) out.push_back(sl);
        i = j;
    }
    std::copy(out.begin(), out.end(), slots);
    return (u32)out.size();
}

static int exchange(ysb_ctx* c, bool pipelined) {
    if (!grouped(c)) return fail(c, YSB_ERR_STATE, "ysb_group_init has not been called");
    int prc = launch_pending_raw(c);
    if (!prc) prc = finish_unpack(c);   // the previous (pipelined) exchange's owner block first
    if (prc) return prc;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->ring_agreed) {
        int rc = agree_ring(c);
        if (rc) return rc;
    }
    if (!c->x_have_plan) pipelined = false;
    const u32 W = c->cfg.window_ring;
    const u64 cells = (u64)c->c_pad * W;
    const u8* delta = c->delta_bound ? c->d_delta : nullptr;   // (delta_bound 0: the delta ring is all zero)
    // timing pairs: folded into x_ms once XEV_KEEP are pending (a streaming caller may never
    // ask for ysb_group_exchange_info); a pair counts only once both events were recorded
    int urc = YSB_OK;
    if (c->xev_used >= XEV_KEEP) {
        int rc = collect_xev(c);
        if (rc) return rc;
    }
    if (c->xev_used == c->xev.size()) {
        std::array<hipEvent_t, 5> ev{};
        for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
        c->xev.push_back(ev);
    }
    const auto ev = c->xev[c->xev_used];
    HIPCHK(c, hipEventRecord(ev[0], c->s_comp));
    // this call's plan into buffer nb
    const int nb = c->xb ^ 1;
    unsigned long long* dmax = c->d_xmax + (u64)nb * W;
    unsigned long long* hmax = c->h_xmax + (u64)nb * W;
    HIPCHK(c, hipMemsetAsync(dmax, 0, (u64)W * 8, c->s_comp));
    launch_xplan(c->d_counts, delta, W, cells, c->pend_u64 ? 1 : 0, c->d_dirty, dmax, c->s_comp);
    HIPCHK(c, hipGetLastError());
    int crc = coll_max_u64(c, dmax, W);
    if (crc) return crc;
    HIPCHK(c, hipMemcpyAsync(hmax, dmax, (u64)W * 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipEventRecord(c->xplan_ev[nb], c->s_comp));
    // the plan the pack uses: this one (complete) or the previous call's (pipelined)
    const int pb = pipelined ? c->xb : nb;
    HIPCHK(c, hipEventSynchronize(c->xplan_ev[pb]));
    c->xb = nb;
    c->x_have_plan = true;
    u32* slots = reinterpret_cast<u32*>(c->h_xmax + 2 * (u64)W) + (u64)pb * W;
    u32 R = 0, width = 8;
    if (ysb_exchange_plan(reinterpret_cast<const uint64_t*>(c->h_xmax + (u64)pb * W), W, (u32)c->nranks, slots, &R,
                          &width))
        return fail(c, YSB_ERR_CAPACITY, "pending counts too large to sum over %d ranks", c->nranks);
    const unsigned long long cap = width == 8 ? ~0ull / (u64)c->nranks : ((1ull << (8 * width)) - 1) / (u64)c->nranks;
    const u32 rows = c->c_pad, per = c->c_pad / (u32)c->nranks;
    const u32 nslots = R;
    R = align_slot_runs(slots, R, W);
    if (R) {
        const int k = c->xk;
        c->xk ^= 1;
        // set k was last used two exchanges ago: its unpack must be done before it is rewritten
        if (c->xset_used[k]) HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_xdone[k], 0));
        int rc = grow_bytes(c, &c->d_xsend[k], &c->xsend_bytes[k], (u64)rows * R * width);
        if (!rc) rc = grow_bytes(c, &c->d_xrecv[k], &c->xrecv_bytes[k], (u64)per * R * width);
        if (rc) return rc;
        u32* dslots = c->d_xslots + (u64)k * W;
        // (the slots' pinned area is rewritten two calls later, after xplan_ev of the call
        // in between: this copy has run by then)
        HIPCHK(c, hipMemcpyAsync(dslots, slots, (u64)R * 4, hipMemcpyHostToDevice, c->s_comp));
        launch_xpack(c->d_counts, delta ? c->d_delta : nullptr, W, rows, dslots, R, c->pend_u64 ? 1 : 0,
                     c->d_dirty, c->d_xsend[k], width, pipelined ? cap : ~0ull, c->s_comp);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev_xpacked[k], c->s_comp));
        // the transfer on the exchange stream, beside the next launch; the unpack follows on
        // the compute stream (finish_unpack)
        HIPCHK(c, hipStreamWaitEvent(c->s_x, c->ev_xpacked[k], 0));
        if ((rc = coll_reduce_scatter(c, c->d_xsend[k], c->d_xrecv[k], (u64)per * R, width, c->s_x))) return rc;
        HIPCHK(c, hipEventRecord(c->ev_xdone[k], c->s_x));
        c->xset_used[k] = true;
        c->unpack_set = k;
        c->unpack_R = R;
        c->unpack_width = width;
        c->unpack_entry = c->xev_used;
    }
    if (!pipelined) {
        // every pending count sat in an exchanged slot: nothing is pending any more
        HIPCHK(c, hipMemsetAsync(c->d_dirty, 0, 4, c->s_comp));
        c->pend_u64 = false;
        c->delta_bound = 0;
    }
    HIPCHK(c, hipEventRecord(ev[1], c->s_comp));
    HIPCHK(c, hipEventRecord(ev[2], R ? c->s_x : c->s_comp));
    if (!R) {   // nothing to unpack: an empty unpack interval
        HIPCHK(c, hipEventRecord(ev[3], c->s_comp));
        HIPCHK(c, hipEventRecord(ev[4], c->s_comp));
    }
    c->xev_used++;
    // complete: the owners' tables hold everything once the call's work has run
    if (!pipelined && (urc = finish_unpack(c))) return urc;
    c->x_count++;
    c->x_bytes += (u64)rows * R * width;
    c->x_last_slots = nslots;
    c->x_last_width = R ? width : 0;
    return YSB_OK;
}

int ysb_group_reduce_scatter(ysb_ctx* c) { return c ? exchange(c, false) : YSB_ERR_ARG; }

int ysb_group_exchange_pipelined(ysb_ctx* c) { return c ? exchange(c, true) : YSB_ERR_ARG; }

int ysb_group_exchange_info(ysb_ctx* c, ysb_exchange_info* out, int reset) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    int rc = sync_streams(c);
    if (!rc) rc = collect_xev(c);
    if (rc) return rc;
    out->exchanges = c->x_count;
    out->bytes = c->x_bytes;
    out->ms = c->x_ms;
    out->critical_ms = c->x_crit_ms;
    out->last_buckets = c->x_last_slots;
    out->last_width = c->x_last_width;
    out->full_ring_bytes = (u64)c->c_pad * c->cfg.window_ring * 8;
    if (reset) {
        c->x_count = 0;
        c->x_bytes = 0;
        c->x_ms = 0;
        c->x_crit_ms = 0;
    }
    return YSB_OK;
}

int ysb_group_checksum(ysb_ctx* c, int what, uint32_t nranks, uint64_t* out) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    if (nranks == 0) return fail(c, YSB_ERR_ARG, "nranks must be >= 1");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = launch_pending_raw(c);
    if (!rc) rc = fold_delta(c);   // the checksums read the u64 ring
    if (!rc) rc = sync_streams(c);
    if (!rc) rc = read_ring(c);
    if (rc) return rc;
    if (!c->ring_known) return fail(c, YSB_ERR_STATE, "ring base not set yet");
    const u32 W = c->cfg.window_ring, C = c->cfg.n_campaigns;
    if (!c->d_cmp) HIPCHK(c, hipMalloc(&c->d_cmp, 32));
    unsigned long long* acc = c->d_cmp;
    auto sum = [&](const unsigned long long* t, u32 rows, u32 c_off, u32 lo, u32 hi, uint64_t* o) -> int {
        HIPCHK(c, hipMemsetAsync(acc, 0, 8, c->s_comp));
        launch_checksum(t, rows, W, c->ring_lo, c_off, lo, hi, acc, c->s_comp);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(o, acc, 8, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        return YSB_OK;
    };
    if (what == YSB_SUM_TRUTH_BLOCKS || what == YSB_SUM_PENDING_BLOCKS) {
        const unsigned long long* t = what == YSB_SUM_TRUTH_BLOCKS ? c->d_truth : c->d_counts;
        if (!t) return fail(c, YSB_ERR_STATE, "no truth accumulated");
        for (u32 r = 0; r < nranks; ++r) {
            u32 lo = 0, hi = 0;
            ysb_group_block(C, (int)r, (int)nranks, &lo, &hi);
            if ((rc = sum(t, c->c_pad, 0, lo, hi, &out[r]))) return rc;
        }
        return YSB_OK;
    }
    if (what == YSB_SUM_OWNED) {
        if (!c->d_owned) { out[0] = 0; return YSB_OK; }
        u32 lo = 0, hi = 0;
        ysb_group_block(C, c->rank, c->nranks, &lo, &hi);
        const u32 per = c->c_pad / (u32)c->nranks;   // row i of the owned table: campaign rank * per + i
        if ((rc = fold_owned(c))) return rc;
        return sum(c->d_owned, per, (u32)c->rank * per, lo, hi, &out[0]);
    }
    return fail(c, YSB_ERR_ARG, "unknown checksum %d", what);
}

int ysb_group_info(ysb_ctx* c, int* rank, int* nranks) {
    if (!c) return YSB_ERR_ARG;
    if (!grouped(c)) return fail(c, YSB_ERR_STATE, "ysb_group_init has not been called");
    if (c->host_coll) {   // the caller's collectives: the ranks it declared
        if (rank) *rank = c->rank;
        if (nranks) *nranks = c->nranks;
        return YSB_OK;
    }
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(c->comm, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
    if (e != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclCommCount: %s", ncclGetErrorString(e));
    if (rank) *rank = r;
    if (nranks) *nranks = n;
    return YSB_OK;
}

int ysb_group_owned(ysb_ctx* c, uint32_t* lo, uint32_t* hi) {
    if (!c) return YSB_ERR_ARG;
    const u32 per = c->c_pad / c->nranks;
    const u32 l = std::min<u32>(c->cfg.n_campaigns, (u32)c->rank * per);
    if (lo) *lo = l;
    if (hi) *hi = std::min<u32>(c->cfg.n_campaigns, l + per);
    return YSB_OK;
}

uint32_t ysb_ad_shard(const char* ad_id, uint32_t len, uint32_t nranks) {
    if (nranks <= 1) return 0;
    u32 kw[KEY_WORDS] = {0};
    std::memcpy(kw, ad_id, std::min<u32>(len, MAX_KEY_BYTES));
    const u32 h = key_hash(kw, std::min<u32>(len, MAX_KEY_BYTES));
    return (u32)(((u64)mix64(h) >> 32) * nranks >> 32);
}

// ---- generator -----------------------------------------------------------------------------------

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
    return p && p->n_campaigns && p->ads_per_campaign && p->events_per_sec && p->format <= YSB_GEN_TBL &&
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
