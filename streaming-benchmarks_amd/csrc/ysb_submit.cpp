// ysb_submit.cpp -- batches into launches: the pinned double-buffered slots (ysb_submit),
// raw lines split on the GPU (ysb_submit_raw), device batches (ysb_submit_device*), the
// layout sampling that picks the scan instantiation, record-mode planning and the launch
// sequence itself (scan, deferred lines, record partition + count).
#include "ysb_ctx.h"

using namespace ysb;

extern "C" {

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

// s waits for e -- unless e has completed already: the slot copies' wait for the slot's last
// scan is normally long satisfied, and a cross-queue barrier packet costs the copy queue time
// between copies even when it has nothing to wait for.
static hipError_t wait_unless_done(hipStream_t s, hipEvent_t e) {
    if (hipEventQuery(e) == hipSuccess) return hipSuccess;
    return hipStreamWaitEvent(s, e, 0);
}

// YSB_F_TIMING keeps HIP events per launch and per slot copy until ysb_kernel_time /
// ysb_copy_time read them.  A caller that never does (a streaming job) would grow them without
// bound: once TIMING_KEEP are pending, the older half is folded into running totals (those
// launches are TIMING_KEEP / 2 launches old -- normally long done; else this waits for them)
// and their events are reused.
static int fold_launch_events(ysb_ctx* c) {
    const size_t half = TIMING_KEEP / 2;
    for (size_t i = 0; i < half; ++i) {
        float ms = 0, mp = 0;
        HIPCHK(c, hipEventSynchronize(c->tev[i][2]));
        HIPCHK(c, hipEventElapsedTime(&ms, c->tev[i][0], c->tev[i][1]));
        HIPCHK(c, hipEventElapsedTime(&mp, c->tev[i][0], c->tev[i][2]));
        c->tev_ms_fold += ms;
        c->tev_path_fold += mp;
        ++c->tev_folded;
    }
    std::rotate(c->tev.begin(), c->tev.begin() + (ptrdiff_t)half, c->tev.begin() + (ptrdiff_t)c->tev_used);
    c->tev_used -= half;
    return YSB_OK;
}

static int fold_copy_events(ysb_ctx* c) {
    const size_t half = TIMING_KEEP / 2;
    for (size_t i = 0; i < half; ++i) {
        float ms = 0;
        HIPCHK(c, hipEventSynchronize(c->cev[i][1]));
        HIPCHK(c, hipEventElapsedTime(&ms, c->cev[i][0], c->cev[i][1]));
        c->cev_ms_fold += ms;
        ++c->cev_folded;
    }
    std::rotate(c->cev.begin(), c->cev.begin() + (ptrdiff_t)half, c->cev.begin() + (ptrdiff_t)c->cev_used);
    c->cev_used -= half;
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
        if (c->tev_used == TIMING_KEEP && (rc = fold_launch_events(c))) return rc;
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
// into one of two pinned buffers, alternating by launch.  Which layout runs:
//  * compute stream idle at the submit: this launch's own sample (the copy takes microseconds);
//  * busy: the previous launch's sample (queued behind the launch before it, so the host waits
//    for that one, never for the launch it is queueing behind) -- if it and the sample before
//    it decided the same layout (or there is no decided sample before it), that one; if they
//    disagree (producers alternating by batch,
//    or a producer that just changed its layout), the per-tile dispatch (4), which takes every
//    producer's tiles at that producer's speed, until two samples agree again;
//  * busy with no earlier sample (the first launch queued behind other work): the per-tile
//    dispatch, without a wait.
// So a producer that changes its layout costs one launch of the wrong instantiation and then
// dispatch launches until it settles; counts never depend on the choice.
static bool same_decision(int a, const LearnDesc& la, int b, const LearnDesc& lb) {
    return a == b && (a != 3 || std::memcmp(&la, &lb, sizeof(LearnDesc)) == 0);
}

static int decide_sample(ysb_ctx* c, int k) {
    if (c->sample_dec[k] >= 0) return YSB_OK;
    HIPCHK(c, hipEventSynchronize(c->ev_sample[k]));
    const u8* h = c->h_sample + (u64)k * SAMPLE_LINES * SAMPLE_STRIDE;
    std::vector<std::pair<const u8*, u64>> lines;
    LearnDesc d{};
    int lay = -1;
    for (u32 i = 0; i < c->sample_nseg[k]; ++i) {
        const u8* sp = h + (u64)i * SAMPLE_STRIDE;
        u32 hd[3];
        std::memcpy(hd, sp, 12);
        if (!hd[2]) { lay = 0; break; }   // bad offsets: the scan defers them anyway
        lines.push_back({sp + 16, hd[1]});
    }
    if (lay < 0) lay = decide_layout(c, lines, &d);
    c->sample_dec[k] = lay;
    c->sample_learn[k] = lay == 3 || lay == 4 ? d : LearnDesc{};
    return YSB_OK;
}

static int sample_device_layout(ysb_ctx* c, const ysb_segment* segs, u32 nseg, LearnDesc* d) {
    const u64 buf = (u64)SAMPLE_LINES * SAMPLE_STRIDE;
    if (!c->h_sample) {
        HIPCHK(c, hipHostMalloc(&c->h_sample, 2 * buf));
        for (hipEvent_t& e : c->ev_sample) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const bool idle = hipStreamQuery(c->s_comp) == hipSuccess;
    const int k = c->sample_cur;
    c->sample_cur ^= 1;
    // buffer k still holds the sample of the launch before the previous one: its decision (if
    // the copy is done -- it is whenever the previous launch waited for a sample) is the
    // older of the two the busy rule compares
    if (c->sample_nseg[k] && c->sample_dec[k] < 0 && hipEventQuery(c->ev_sample[k]) == hipSuccess) {
        int rc = decide_sample(c, k);
        if (rc) return rc;
    }
    const int older = c->sample_nseg[k] ? c->sample_dec[k] : -1;
    const LearnDesc older_learn = c->sample_learn[k];
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
    c->sample_dec[k] = -1;
    int rc;
    if (idle) {   // this launch's own sample
        if ((rc = decide_sample(c, k))) return rc;
        *d = c->sample_learn[k];
        return c->sample_dec[k];
    }
    const int p = k ^ 1;   // the previous launch's sample
    if (!c->sample_nseg[p]) {   // none: no wait, the dispatch
        *d = LearnDesc{};
        return 4;
    }
    if ((rc = decide_sample(c, p))) return rc;
    // (no older decision -- the first two launches -- trusts the previous sample alone)
    if (older < 0 || same_decision(older, older_learn, c->sample_dec[p], c->sample_learn[p])) {
        *d = c->sample_learn[p];
        return c->sample_dec[p];
    }
    // two samples disagree: the per-tile dispatch (with the newer sample's learned order, if any)
    *d = c->sample_dec[p] == 3 || c->sample_dec[p] == 4 ? c->sample_learn[p] : LearnDesc{};
    return 4;
}

// With YSB_F_TIMING: an event pair around a slot's H2D copy (ysb_copy_time), else none.
static int copy_events(ysb_ctx* c, hipEvent_t** out, u64 bytes) {
    *out = nullptr;
    if (!(c->cfg.flags & YSB_F_TIMING)) return YSB_OK;
    if (c->cev_used == TIMING_KEEP) {
        const int rc = fold_copy_events(c);
        if (rc) return rc;
    }
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
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hd_bytes[s]), c->h_bytes[s], 0));
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hd_off[s]), c->h_off[s], 0));
    }
    return YSB_OK;
}

// A slot's host -> device copy on the copy stream: by the CUs from the pinned slot's device
// address (launch_h2d_copy, the default: ysb_split.hip says why; a mapped batch that does not
// start on a 16-byte boundary by launch_h2d_copy_unaligned), or by the DMA engine with
// YSB_F_H2D_SDMA.
static hipError_t h2d(ysb_ctx* c, void* dst, const void* dsrc, const void* hsrc, u64 bytes) {
    if (c->cfg.flags & YSB_F_H2D_SDMA) return hipMemcpyAsync(dst, hsrc, bytes, hipMemcpyHostToDevice, c->s_copy);
    const int wgs = c->h2d_grid ? c->h2d_grid : c->cus * c->h2d_wg;
    if (reinterpret_cast<uintptr_t>(dsrc) & 15) launch_h2d_copy_unaligned(dst, dsrc, bytes, wgs, c->s_copy);
    else launch_h2d_copy(dst, dsrc, bytes, wgs, c->s_copy, c->h2d_prio);
    return hipGetLastError();
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
    HIPCHK(c, wait_unless_done(c->s_copy, c->ev_kdone[slot]));
    hipEvent_t* ce = nullptr;
    if ((rc = copy_events(c, &ce, nbytes + n * 4))) return rc;
    if (ce) HIPCHK(c, hipEventRecord(ce[0], c->s_copy));
    if (nbytes) HIPCHK(c, h2d(c, c->d_bytes[slot], c->hd_bytes[slot], c->h_bytes[slot], nbytes));
    if (n) HIPCHK(c, h2d(c, c->d_off[slot], c->hd_off[slot], c->h_off[slot], n * 4));
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

// Lines a raw batch may hold: max_batch_events, or one per 32 bytes of the slot if that is
// more (an event line is > 60 bytes; the device's line-start array is 4 B per line, not per
// byte); at most one per byte.  A batch with more lines fails its launch (YSB_ERR_CAPACITY).
static u64 raw_line_cap(const ysb_config& cfg) {
    return std::min<u64>(cfg.max_batch_bytes + 1, std::max<u64>(cfg.max_batch_events, cfg.max_batch_bytes / 32) + 1);
}

static int ensure_raw(ysb_ctx* c) {
    if (c->h_rawn) return YSB_OK;
    HIPCHK(c, hipSetDevice(c->device));
    c->raw_lines_cap = raw_line_cap(c->cfg);
    for (int s = 0; s < 2; ++s) {   // (a failed earlier attempt may have left some of these)
        hipFree(c->d_roff[s]);
        c->d_roff[s] = nullptr;
        HIPCHK(c, hipMalloc(&c->d_roff[s], c->raw_lines_cap * 4));
        if (!c->ev_raw[s]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_raw[s], hipEventDisableTiming));
    }
    if (!c->s_split) HIPCHK(c, hipStreamCreateWithFlags(&c->s_split, hipStreamNonBlocking));
    if (const char* e = getenv("YSB_SPLIT_STREAM")) c->split_place = std::atoi(e);
    if (const char* e = getenv("YSB_H2D_WG")) c->h2d_wg = std::max(1, std::atoi(e));
    if (const char* e = getenv("YSB_H2D_PRIO")) c->h2d_prio = std::atoi(e) != 0;
    if (const char* e = getenv("YSB_H2D_GRID")) c->h2d_grid = std::max(0, std::atoi(e));
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
// (ev_raw), so its scan is enqueued now -- the order of submission is kept.  A batch that
// cannot launch (more lines than raw_lines_cap, a failed enqueue) is dropped and its error
// is sticky: every later call on the context that would order work after it returns it,
// until ysb_reset -- counts after a lost batch are not the stream's.
int launch_pending_raw(ysb_ctx* c) {
    if (c->raw_fail) return fail(c, c->raw_fail, "%s", c->raw_fail_msg.c_str());
    if (c->raw_pend < 0) return YSB_OK;
    const int slot = c->raw_pend;
    int rc = YSB_OK;
    if (hipSetDevice(c->device) != hipSuccess || hipEventSynchronize(c->ev_raw[slot]) != hipSuccess ||
        hipStreamWaitEvent(c->s_comp, c->ev_raw[slot], 0) != hipSuccess) {
        rc = fail(c, YSB_ERR_HIP, "raw batch (slot %d): waiting for its line split failed", slot);
    } else if (c->raw_rebase_on[slot] && c->h_rawn[slot] > c->rebase_n - c->raw_rebase[slot].first_line) {
        rc = fail(c, YSB_ERR_ARG, "raw batch (slot %d): %llu lines, more than the rebase table holds from line %llu",
                  slot, (unsigned long long)c->h_rawn[slot], (unsigned long long)c->raw_rebase[slot].first_line);
    } else if (c->h_rawn[slot] > c->raw_lines_cap) {
        rc = fail(c, YSB_ERR_CAPACITY, "raw batch (slot %d): %llu lines, more than the %llu its slot holds "
                  "(max(max_batch_events, max_batch_bytes / 32))", slot, (unsigned long long)c->h_rawn[slot],
                  (unsigned long long)c->raw_lines_cap);
    } else {
        const ysb_segment sg{c->d_bytes[slot], c->raw_nbytes[slot], c->d_roff[slot], c->h_rawn[slot]};
        c->submit_layout = c->raw_layout[slot];
        c->submit_learn = c->raw_learn[slot];
        rc = enqueue_scan(c, &sg, 1);
        c->submit_layout = -1;
    }
    // the slot's device buffers are free again once this launch (or nothing) has run
    if (hipEventRecord(c->ev_kdone[slot], c->s_comp) != hipSuccess && !rc)
        rc = fail(c, YSB_ERR_HIP, "hipEventRecord failed");
    c->raw_pend = -1;
    if (rc) {
        c->raw_fail = rc;
        c->raw_fail_msg = c->err;
    }
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

static int raw_args(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes) {
    if (slot < 0 || slot > 1) return fail(c, YSB_ERR_ARG, "slot must be 0 or 1");
    if (nbytes > c->cfg.max_batch_bytes)
        return fail(c, YSB_ERR_CAPACITY, "raw batch of %llu B exceeds max_batch_bytes", (unsigned long long)nbytes);
    if (nbytes && !bytes) return fail(c, YSB_ERR_ARG, "NULL batch buffer");
    if (!c->table_loaded) return fail(c, YSB_ERR_STATE, "ysb_load_ad_map has not been called");
    return YSB_OK;
}

// A raw batch from hsrc (host address: the layout sample, the DMA engine) / dsrc (its device
// address: the copy kernel) into the slot's device buffer, split, optionally rebased; its scan
// launches at the next call.  The caller has waited for the slot's previous copy.
static int enqueue_raw(ysb_ctx* c, int slot, const u8* hsrc, const u8* dsrc, u64 nbytes, const ysb_rebase* rb) {
    int rc;
    c->raw_layout[slot] = -1;
    if (layout_sampling(c) && nbytes)
        c->raw_layout[slot] = hinted_layout(c, sniff_raw(c, hsrc, nbytes, &c->raw_learn[slot]));
    // H2D once the slot's previous kernel has run.  The split on a stream of its own behind its
    // copy, so the next slot's copy queues right behind this one.  Round 5 kept it on the copy
    // stream: beside a copy kernel of one workgroup per CU the split was starved (its 32 us
    // count took 2.7 ms, and the slot's scan waited behind it).  The copy kernel's grid is now 32
    // workgroups (h2d_grid): still far more bytes in flight than PCIe's bandwidth x latency, and
    // the HBM work beside it (split, scan) no longer queues behind its slow requests.  Same-box
    // A/B (gpurun_out/r6r, r6s): raw host-staged 210 -> 214-218 M events/s, the raw streaming
    // replay 197 -> 206-209 (copy queue busy 0.958 -> 0.986).  (YSB_SPLIT_STREAM: 0 the copy
    // stream, 2 the compute stream -- A/B only.)
    const bool sdma = (c->cfg.flags & YSB_F_H2D_SDMA) != 0u;
    hipStream_t ss = sdma || c->split_place == 1 ? c->s_split : c->split_place == 2 ? c->s_comp : c->s_copy;
    HIPCHK(c, wait_unless_done(c->s_copy, c->ev_kdone[slot]));
    hipEvent_t* ce = nullptr;
    if ((rc = copy_events(c, &ce, nbytes))) return rc;
    if (ce) HIPCHK(c, hipEventRecord(ce[0], c->s_copy));
    if (nbytes) HIPCHK(c, h2d(c, c->d_bytes[slot], dsrc, hsrc, nbytes));
    if (ce) HIPCHK(c, hipEventRecord(ce[1], c->s_copy));
    HIPCHK(c, hipEventRecord(c->ev_h2d[slot], c->s_copy));
    if (ss != c->s_copy) HIPCHK(c, hipStreamWaitEvent(ss, c->ev_h2d[slot], 0));
    c->raw_rebase_on[slot] = rb != nullptr;
    if (rb) c->raw_rebase[slot] = *rb;
    if (nbytes) {
        // the line count goes straight to pinned memory (read at the launch)
        HIPCHK(c, launch_split_lines(c->d_bytes[slot], nbytes, c->d_split_chunk, c->d_roff[slot],
                                     c->raw_lines_cap, c->h_rawn + slot, ss));
        if (rb) {
            launch_rebase(c->d_bytes[slot], nbytes, c->d_roff[slot], c->raw_lines_cap, c->h_rawn + slot, 0,
                          c->d_rebase + rb->first_line, c->rebase_n - rb->first_line,
                          c->rebase_base + rb->lead_shift, c->cus, ss);
            HIPCHK(c, hipGetLastError());
        }
    } else {
        c->h_rawn[slot] = 0;
    }
    HIPCHK(c, hipEventRecord(c->ev_raw[slot], ss));
    c->raw_nbytes[slot] = nbytes;
    // the other slot's batch, submitted before this one, launches now; this one at the next call
    rc = launch_pending_raw(c);
    c->raw_pend = slot;
    return rc;
}

int ysb_submit_raw(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes) {
    if (!c) return YSB_ERR_ARG;
    int rc = raw_args(c, slot, bytes, nbytes);
    if (rc) return rc;
    // the slot's own earlier batch launches first (its device buffers are about to be reused)
    rc = c->raw_pend == slot ? launch_pending_raw(c) : YSB_OK;
    if (!rc) rc = ensure_slots(c);
    if (!rc) rc = ensure_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    // the slot's previous H2D must be done before its pinned buffer is rewritten
    HIPCHK(c, hipEventSynchronize(c->ev_h2d[slot]));
    if (bytes != c->h_bytes[slot] && nbytes) std::memcpy(c->h_bytes[slot], bytes, nbytes);
    return enqueue_raw(c, slot, c->h_bytes[slot], c->hd_bytes[slot], nbytes, nullptr);
}

// ---- zero-copy raw batches from registered caller memory (ABI 5) ----------------------------

int ysb_host_register(ysb_ctx* c, void* host, uint64_t bytes) {
    if (!c) return YSB_ERR_ARG;
    if (!host || !bytes) return fail(c, YSB_ERR_ARG, "empty host range");
    const uintptr_t a = reinterpret_cast<uintptr_t>(host);
    for (const auto& r : c->host_ranges)
        if (a < r.first + r.second.bytes && r.first < a + bytes) return fail(c, YSB_ERR_ARG, "host range overlaps a registered one");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostRegister(host, bytes, hipHostRegisterMapped));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        hipHostUnregister(host);
        return fail(c, YSB_ERR_HIP, "hipHostGetDevicePointer of a registered range failed");
    }
    if ((reinterpret_cast<uintptr_t>(d) ^ a) & 15) {   // the copy's 16-byte widening assumes it
        hipHostUnregister(host);
        return fail(c, YSB_ERR_HIP, "the device alias of a registered range is not 16-byte congruent to it");
    }
    c->host_ranges[a] = {bytes, static_cast<u8*>(d)};
    return YSB_OK;
}

int ysb_host_unregister(ysb_ctx* c, void* host) {
    if (!c) return YSB_ERR_ARG;
    auto it = c->host_ranges.find(reinterpret_cast<uintptr_t>(host));
    if (it == c->host_ranges.end()) return fail(c, YSB_ERR_ARG, "not a registered range");
    // nothing queued may still read it
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->s_copy));
    HIPCHK(c, hipHostUnregister(host));
    c->host_ranges.erase(it);
    return YSB_OK;
}

int ysb_rebase_table(ysb_ctx* c, const uint32_t* time_at, uint64_t n_lines, int64_t lead_base) {
    if (!c) return YSB_ERR_ARG;
    if (n_lines && !time_at) return fail(c, YSB_ERR_ARG, "NULL table");
    HIPCHK(c, hipSetDevice(c->device));
    // batches queued with the old table must be done with it
    HIPCHK(c, hipStreamSynchronize(c->s_copy));
    if (c->s_split) HIPCHK(c, hipStreamSynchronize(c->s_split));
    hipFree(c->d_rebase);
    c->d_rebase = nullptr;
    c->rebase_n = 0;
    if (!n_lines) return YSB_OK;
    u32 kmax = 0;
    for (u64 i = 0; i < n_lines; ++i) kmax = std::max(kmax, time_at[i] >> 16);
    if (lead_base < 0 || lead_base + kmax >= 1000000000LL) return fail(c, YSB_ERR_ARG, "leading digits out of [0, 10^9)");
    HIPCHK(c, hipMalloc(&c->d_rebase, n_lines * 4));
    HIPCHK(c, hipMemcpy(c->d_rebase, time_at, n_lines * 4, hipMemcpyHostToDevice));
    c->rebase_n = n_lines;
    c->rebase_base = lead_base;
    c->rebase_kmax = kmax;
    return YSB_OK;
}

// The device alias of a mapped batch, or NULL when the batch widened to 16-byte boundaries on
// both sides (what the copy reads: launch_h2d_copy / launch_h2d_copy_unaligned) is not inside
// one registered range.
static const u8* mapped_src(const ysb_ctx* c, const uint8_t* bytes, u64 nbytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(bytes);
    auto it = c->host_ranges.upper_bound(a);
    if (it == c->host_ranges.begin()) return nullptr;
    --it;
    const uintptr_t lo = a & ~uintptr_t(15), hi = (a + nbytes + 15) & ~uintptr_t(15);
    if (lo < it->first || hi > it->first + it->second.bytes) return nullptr;
    return it->second.dptr + (a - it->first);
}

int ysb_submit_raw_mapped(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes, const ysb_rebase* rb) {
    if (!c) return YSB_ERR_ARG;
    int rc = raw_args(c, slot, bytes, nbytes);
    if (rc) return rc;
    const u8* dsrc = mapped_src(c, bytes, nbytes);
    if (nbytes && !dsrc)
        return fail(c, YSB_ERR_ARG, "the batch (widened to 16-byte boundaries) is not inside a registered range");
    if (rb) {
        if (!c->d_rebase) return fail(c, YSB_ERR_STATE, "no rebase table (ysb_rebase_table)");
        if (rb->first_line >= c->rebase_n) return fail(c, YSB_ERR_ARG, "first_line beyond the rebase table");
        const i64 lo = c->rebase_base + rb->lead_shift;
        if (lo < 0 || lo + (i64)c->rebase_kmax >= 1000000000LL)
            return fail(c, YSB_ERR_ARG, "rebased leading digits out of [0, 10^9)");
    }
    rc = c->raw_pend == slot ? launch_pending_raw(c) : YSB_OK;
    if (!rc) rc = ensure_slots(c);
    if (!rc) rc = ensure_raw(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    return enqueue_raw(c, slot, bytes, dsrc, nbytes, rb);
}

// A mapped batch whose line offsets are already in HBM: nothing waits for a line count, so the
// copy queue holds copies only (a raw batch's split and rebase between copies cost the copy
// queue ~4 % of its time: DESIGN.md section 11) and the scan is enqueued at once behind the
// copy on the compute stream.
int ysb_submit_mapped(ysb_ctx* c, int slot, const uint8_t* bytes, uint64_t nbytes, const uint32_t* d_line_off,
                      uint64_t n, const ysb_rebase* rb) {
    if (!c) return YSB_ERR_ARG;
    int rc = raw_args(c, slot, bytes, nbytes);
    if (rc) return rc;
    if (n > 0x7FFFFFFFull) return fail(c, YSB_ERR_CAPACITY, "at most 2^31-1 events per batch");
    if (n && !d_line_off) return fail(c, YSB_ERR_ARG, "NULL line offsets");
    const u8* dsrc = mapped_src(c, bytes, nbytes);
    if (nbytes && !dsrc)
        return fail(c, YSB_ERR_ARG, "the batch (widened to 16-byte boundaries) is not inside a registered range");
    if (rb) {
        if (!c->d_rebase) return fail(c, YSB_ERR_STATE, "no rebase table (ysb_rebase_table)");
        if (rb->first_line > c->rebase_n || n > c->rebase_n - rb->first_line)
            return fail(c, YSB_ERR_ARG, "the batch's lines run past the rebase table");
        const i64 lo = c->rebase_base + rb->lead_shift;
        if (lo < 0 || lo + (i64)c->rebase_kmax >= 1000000000LL)
            return fail(c, YSB_ERR_ARG, "rebased leading digits out of [0, 10^9)");
    }
    if (!n) return YSB_OK;
    rc = launch_pending_raw(c);   // batches launch in submission order
    if (!rc) rc = ensure_slots(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    // at most two copies in flight: the slot's previous one must be done (its device buffer is
    // then only still read by its scan, which the copy waits for on the device)
    HIPCHK(c, hipEventSynchronize(c->ev_h2d[slot]));
    if (layout_sampling(c)) c->submit_layout = hinted_layout(c, sniff_raw(c, bytes, nbytes, &c->submit_learn));
    HIPCHK(c, wait_unless_done(c->s_copy, c->ev_kdone[slot]));
    hipEvent_t* ce = nullptr;
    if ((rc = copy_events(c, &ce, nbytes))) return rc;
    if (ce) HIPCHK(c, hipEventRecord(ce[0], c->s_copy));
    HIPCHK(c, h2d(c, c->d_bytes[slot], dsrc, bytes, nbytes));
    if (ce) HIPCHK(c, hipEventRecord(ce[1], c->s_copy));
    HIPCHK(c, hipEventRecord(c->ev_h2d[slot], c->s_copy));
    HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_h2d[slot], 0));
    if (rb) {
        launch_rebase(c->d_bytes[slot], nbytes, d_line_off, n, nullptr, n, c->d_rebase + rb->first_line,
                      c->rebase_n - rb->first_line, c->rebase_base + rb->lead_shift, c->cus, c->s_comp);
        HIPCHK(c, hipGetLastError());
    }
    const ysb_segment sg{c->d_bytes[slot], nbytes, d_line_off, n};
    rc = enqueue_scan(c, &sg, 1);
    c->submit_layout = -1;
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(c->ev_kdone[slot], c->s_comp));
    return YSB_OK;
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
    double t = c->cev_ms_fold;
    for (size_t i = 0; i < c->cev_used; ++i) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->cev[i][0], c->cev[i][1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (copies) *copies = c->cev_folded + c->cev_used;
    if (bytes) *bytes = c->copy_bytes;
    c->cev_used = 0;
    c->cev_ms_fold = 0;
    c->cev_folded = 0;
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

}  // extern "C"
