// ysb_ctx.h -- the library context behind the C ABI (include/ysb_hip.h), shared by the
// library's host translation units:
//   ysb_capi.cpp    context lifecycle, the ad -> campaign tables, sync / drain / ring / stats
//   ysb_submit.cpp  batches: slots, raw lines, device batches, layout sampling, the launches
//   ysb_group.cpp   multi-GPU: the RCCL / host-collective group and the keyBy exchange
//   ysb_gen_api.cpp the synthetic generator (host and device) and its truth tables
// Internal: nothing here is part of the ABI (the shared helpers have hidden visibility).
#pragma once
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

using namespace ysb;   // (an internal header of the library's own units)


namespace ysb {
int scan_lds_bytes();
}

constexpr size_t XEV_KEEP = 64;   // exchange timing pairs pending before they are folded into x_ms
// YSB_F_TIMING: launch / copy event records pending before the older half is folded into
// running totals (a streaming caller may never call ysb_kernel_time / ysb_copy_time)
constexpr size_t TIMING_KEEP = 256;

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
    // the layout decided from buffer k's sample (-1: not decided yet) and its key order
    int sample_dec[2] = {-1, -1};
    LearnDesc sample_learn[2]{};
    u32* h_used = nullptr;       // pinned: the out-of-ring map's fill level after a launch ...
    hipEvent_t ev_used = nullptr; // ... readable once this has completed
    bool used_pending = false;
    // raw batches (ysb_submit_raw): the line starts are found on the GPU (ysb_split.hip) on
    // s_split after the slot's H2D, into d_roff[slot]; the scan is launched once the line
    // count is back (launch_pending_raw, at the next call), so the next H2D queues first
    hipStream_t s_split = nullptr;
    u32* d_roff[2] = {nullptr, nullptr};        // raw_lines_cap starts per slot
    u64 raw_lines_cap = 0;                      // lines a raw batch may hold (raw_line_cap)
    u32* d_split_chunk = nullptr;               // per-chunk counts, then bases
    u64 split_chunk_words = 0;
    unsigned long long* d_rawn = nullptr;       // [2] lines of the slot's raw batch
    unsigned long long* h_rawn = nullptr;       // pinned mirror
    hipEvent_t ev_raw[2] = {nullptr, nullptr};  // split done and its count read back
    int raw_pend = -1;                          // the slot whose raw batch awaits its launch
    int raw_fail = 0;                           // a raw batch that could not launch: sticky until ysb_reset
    std::string raw_fail_msg;
    u64 raw_nbytes[2] = {0, 0};
    int raw_layout[2] = {-1, -1};               // its first line's layout (sampled on the host)
    LearnDesc raw_learn[2]{};
    // H2D timing (YSB_F_TIMING): {start, end} of each slot copy since the last ysb_copy_time
    std::vector<std::array<hipEvent_t, 2>> cev;
    size_t cev_used = 0;
    u64 copy_bytes = 0;
    double cev_ms_fold = 0;                     // pairs folded into totals (TIMING_KEEP)
    u64 cev_folded = 0;
    // caller host ranges registered for zero-copy raw batches (ysb_host_register): base ->
    // {bytes, device address}
    struct HostRange {
        u64 bytes;
        u8* dptr;
    };
    std::map<uintptr_t, HostRange> host_ranges;
    // the replay's rebase table (ysb_rebase_table) and each slot's pending rebase
    u32* d_rebase = nullptr;
    u64 rebase_n = 0;
    i64 rebase_base = 0;
    u32 rebase_kmax = 0;                        // the largest bucket index in it
    bool raw_rebase_on[2] = {false, false};
    int split_place = 1;                        // raw split on: 1 s_split (default), 0 the copy stream, 2 s_comp (A/B)
    int h2d_wg = 1;                             // copy-kernel workgroups per CU (A/B)
    bool h2d_prio = false;                      // copy kernel at raised wave priority (A/B)
    int h2d_grid = 32;                          // copy-kernel workgroups (0: one per CU; YSB_H2D_GRID A/B)
    ysb_rebase raw_rebase[2]{};
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
    u8* hd_bytes[2] = {nullptr, nullptr};      // the pinned slots' device-visible addresses (the CU copy)
    u32* hd_off[2] = {nullptr, nullptr};
    u8* d_bytes[2] = {nullptr, nullptr};
    u32* d_off[2] = {nullptr, nullptr};
    hipEvent_t ev_h2d[2] = {nullptr, nullptr}, ev_kdone[2] = {nullptr, nullptr};
    bool slot_busy[2] = {false, false};
    // timing: per launch {before scan, after scan, after the last kernel of the launch}
    std::vector<std::array<hipEvent_t, 3>> tev;
    size_t tev_used = 0;
    double tev_ms_fold = 0, tev_path_fold = 0;   // launches folded into totals (TIMING_KEEP)
    u64 tev_folded = 0;
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
    double x_ms = 0, x_crit_ms = 0, x_rs_ms = 0, x_exposed_ms = 0;
    // per exchange {start, packed (compute stream), reduce-scatter done (exchange stream),
    // unpack start, unpack end (compute stream)}
    std::vector<std::array<hipEvent_t, 6>> xev;
    size_t xev_used = 0;
    // asynchronous flushes (ysb_flush_begin / ysb_flush_end): a ring of FLUSH_SLOTS pinned row
    // buffers the compaction kernel writes straight into, each with its device-side count
    // copied back and an event; fl_head the oldest outstanding, fl_n how many
    struct FlushSlot {
        TableRow* h_rows = nullptr;   // pinned (device-visible: written by the kernel)
        TableRow* hd_rows = nullptr;  // ... its device address
        u32* h_n = nullptr;           // pinned: the rows the kernel wrote
        u64 cap = 0;
        hipEvent_t ev = nullptr;
    };
    static constexpr int FLUSH_SLOTS = 4;
    FlushSlot fl[FLUSH_SLOTS];
    int fl_head = 0, fl_n = 0;
    u32* d_fl_n = nullptr;                 // [FLUSH_SLOTS] device counters
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

#define YSB_INTERNAL __attribute__((visibility("hidden")))

// an error message for ysb_last_error (the context's, or the thread's when c is NULL)
YSB_INTERNAL int fail(ysb_ctx* c, int code, const char* fmt, ...);
extern thread_local std::string g_open_err;

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(ctx, YSB_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                \
    } while (0)

inline bool is_pow2(u64 x) { return x && !(x & (x - 1)); }
inline u32 log2u(u64 x) { u32 l = 0; while (((u64)1 << l) < x) ++l; return l; }

extern "C" {
// ysb_capi.cpp
YSB_INTERNAL int sync_streams(ysb_ctx* c);       // every queued launch / copy / exchange done
YSB_INTERNAL int pull_side_list(ysb_ctx* c);     // the out-of-ring map into the host side list
YSB_INTERNAL void poll_ring(ysb_ctx* c);         // the auto-based ring's base, if known by now
YSB_INTERNAL int read_ring(ysb_ctx* c);          // ... read with a wait
YSB_INTERNAL int move_ring(ysb_ctx* c, i64 new_lo);
YSB_INTERNAL int fold_delta(ysb_ctx* c);         // record mode's u8 delta ring into the u64 ring
// ysb_submit.cpp
YSB_INTERNAL int launch_pending_raw(ysb_ctx* c); // the raw batch awaiting its launch
// ysb_group.cpp
YSB_INTERNAL bool grouped(const ysb_ctx* c);
YSB_INTERNAL int agree_ring(ysb_ctx* c);
YSB_INTERNAL int allreduce_max(ysb_ctx* c, i64* h, int n);
YSB_INTERNAL int finish_unpack(ysb_ctx* c);      // a pipelined exchange's owner-block unpack
YSB_INTERNAL int fold_owned(ysb_ctx* c);         // the owned table's u8 accumulator into it
}
