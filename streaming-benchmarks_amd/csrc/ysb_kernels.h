// ysb_kernels.h -- launch interface between the C-ABI layer (ysb_capi.cpp) and the
// gfx950 kernels (ysb_scan.hip, ysb_gen.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "ysb_common.h"

namespace ysb {

// Geometry of the fused scan kernel (see DESIGN.md "Kernel 1").
// One wave per workgroup: no intra-workgroup barrier ever waits for a slower wave,
// and the two waves of a SIMD drift into different phases (one classifying while the
// other parses), which hides each other's LDS latency.
constexpr int SCAN_TPB = 64;                  // threads per scan workgroup (one wave)
#ifndef YSB_TILE_LINES
#define YSB_TILE_LINES 64
#endif
// lines per tile: one per lane (fewer than 64 leaves lanes idle but shrinks the LDS tile,
// so more workgroups fit a CU)
constexpr int TILE_LINES = YSB_TILE_LINES;
static_assert(TILE_LINES >= 1 && TILE_LINES <= SCAN_TPB, "one line per lane at most");
#ifndef YSB_WG_PER_CU
#define YSB_WG_PER_CU 8
#endif
#ifndef YSB_MAX_TILES
#define YSB_MAX_TILES 128
#endif
constexpr int SCAN_WG_PER_CU = YSB_WG_PER_CU; // resident scan workgroups per CU (LDS-bound)
#ifndef YSB_TILE_LINE_BYTES
#define YSB_TILE_LINE_BYTES 272
#endif
constexpr int TILE_CAP = TILE_LINES * YSB_TILE_LINE_BYTES;   // LDS bytes of one tile (per-line average cap)
constexpr int TILE_CHUNKS = TILE_CAP / 16;    // 16-byte chunks per tile
constexpr int CHUNKS_PER_THREAD = (TILE_CHUNKS + SCAN_TPB - 1) / SCAN_TPB;  // 17
constexpr int LCNT_CAP = 256;                 // u32 per-workgroup (campaign, window) counters
constexpr int MAX_TILES_PER_BLOCK = YSB_MAX_TILES;   // tile bounds preloaded into LDS
// .tbl rows are ~140 B (JSON lines ~254 B): smaller tiles, so more workgroups fit a CU's
// LDS and the bytes in flight per CU stay comparable.
#ifndef YSB_TBL_LINE_BYTES
#define YSB_TBL_LINE_BYTES 160
#endif
#ifndef YSB_TBL_WG_PER_CU
#define YSB_TBL_WG_PER_CU 12
#endif

// Per-input-format geometry of the scan kernel: tile capacity, prefetch registers and
// the LDS carve (tile | slack | window counters | misc | tile bounds).
// Record mode (REC): the window-counter area holds the record staging lines instead --
// REC_BINS_MAX level-1 bins x a 64-record ring each (2 KiB).
constexpr int REC_BINS_MAX = 8;       // level-1 bins of the scan's record staging
constexpr int REC_RING = 64;          // staged records per bin (two 128-B lines)
template <bool TBL, bool REC = false>
struct Geom {
    static constexpr int WG_PER_CU = TBL ? YSB_TBL_WG_PER_CU : SCAN_WG_PER_CU;
    // (.tbl record mode: 8 B less per row, so its record staging lines fit 12 workgroups per
    // CU in whole LDS granules; the generator's rows average 140 B, at most 151)
    static constexpr int CAP = TILE_LINES * (TBL ? YSB_TBL_LINE_BYTES - (REC ? 8 : 0) : YSB_TILE_LINE_BYTES);
    static constexpr int CHUNKS = CAP / 16;
    static constexpr int CPT = (CHUNKS + SCAN_TPB - 1) / SCAN_TPB;   // 16-byte chunks per thread
    static constexpr int OFF_TILE = 0;
    static constexpr int OFF_LCNT = OFF_TILE + CAP + 64;             // 64 B slack for reads past a tile
    static constexpr int LCNT_BYTES = REC ? REC_BINS_MAX * REC_RING * 4 : LCNT_CAP * 4;
    static constexpr int OFF_MISC = OFF_LCNT + LCNT_BYTES;
    static constexpr int OFF_TB = OFF_MISC + 64;
    static constexpr int LDS = OFF_TB + (MAX_TILES_PER_BLOCK + 4) * 4;
    static_assert(OFF_LCNT % 16 == 0 && OFF_MISC % 16 == 0 && OFF_TB % 16 == 0 && LDS % 16 == 0,
                  "LDS carve must stay 16-byte aligned");
    // LDS is allocated per workgroup in 1280-byte granules (measured round 3: a .tbl geometry
    // of 13,232 B ran 12 per CU at 2/3 speed, 12,656 B at full; 163,840 / 128 = 1280)
    static constexpr int LDS_ALLOC = (LDS + 1279) / 1280 * 1280;
    static_assert(LDS_ALLOC * WG_PER_CU <= 163840, "WG_PER_CU workgroups must fit one CU's 160 KiB of LDS");
};
constexpr int AUX_TPB = 256;                  // threads per workgroup of the other kernels

// One batch of a multi-batch launch (ysb_submit_device_segments): each keeps its own
// u32 line offsets (so each stays under 4 GiB), and one launch scans them all -- every
// workgroup walks its run of tiles in segment 0, then in segment 1, ..., without a
// grid-wide drain between batches (one launch tail per step instead of one per batch).
constexpr int MAX_SEGS = 16;
struct ScanSeg {
    const u8* bytes;            // 16-byte aligned
    const u32* off;
    u64 n;
    u64 nbytes;
    u64 line_base;              // index of the segment's first line among all segments
    u64 n_tiles;
    u64 n_static;               // tiles [0, n_static) split over the grid, the rest claimed in chunks
    u32 tiles_per_block;        // static tiles per workgroup (q) ...
    u32 static_rem;             // ... plus one for workgroups b < static_rem
};

struct ScanParams {
    // the batch being scanned: segment 0 on the host side; scan_kernel sets them to each
    // segment in turn, defer_kernel to the segment of each deferred line
    const u8* bytes;            // batch bytes (16-byte aligned)
    u64 nbytes;
    const u32* off;             // n line offsets
    u64 n;
    u64 line_base;              // segment's first line among all segments (defer list indices)
    const u32* table;           // ad table, SLOT_WORDS u32 per slot (every key)
    u32 table_mask;             // slots - 1
    const u32* ctable;          // 36-byte-key cuckoo table, CSLOT_WORDS u32 per slot
    u32 ctable_mask;
    u32 ctable_partial;         // 1: some 36-byte key missed the cuckoo build (misses defer)
    u32 probe_serial;           // 1: probe the second cuckoo slot only after a first-slot miss
    u32 tbl;                    // 1: the fork's .tbl rows (YSB_F_FORMAT_TBL) instead of JSON lines
    CuckooSeed cseed;
    u32 n_campaigns;
    unsigned long long* counts; // [c_pad][W] u64, campaign-major
    u32 ring_w;                 // W (power of two)
    u32 lds_wl;                 // per-WG window slots in LDS (power of two), 0 = off
    u32 lds_wl_log2;
    u32 require_mask;           // required-key bit mask
    const i64* ring;            // ring[0] = first bucket, ring[1] = 1 when set
    DivMagic div;
    SideSlot* side;             // out-of-ring cells (hash map)
    u32* side_used;             // slots taken
    u32 side_mask;              // slots - 1
    u32 side_cbits;             // campaign bits of a key
    OvfEntry* ovf;              // fallback list: buckets a key cannot express, or a full map
    u32* ovf_count;
    u32 ovf_cap;
    u32 tiles_per_block;
    u64 n_tiles;
    u32 grid;                   // scan workgroups: max over segments of ceil(n_tiles / tiles_per_block)
    u32 n_segs;                 // >= 1
    u32 dyn_chunk;              // tiles per dynamic claim (0: all static)
    u32* dyn_ctr;               // [MAX_SEGS] claim counters, zero at launch
    ScanSeg seg[MAX_SEGS];
    unsigned long long* stats;  // ST_COUNT_ u64
    unsigned long long* dbg;    // diagnostic build only (YSB_STAMPS): per-wave phase cycles
    u32* defer;                 // line indices for the general path (defer_kernel)
    u32* defer_count;           // [0] entries, reset by defer_kernel
    u32* defer_done;            // workgroup ticket of defer_kernel
    u32 defer_cap;
    // Record mode (large count tables, no LDS window counters: configs[2]): a joined
    // in-ring view is not an HBM atomic but a u32 record (its ring cell index) appended
    // to the sub-buffer of (workgroup, campaign range); partition_kernel and
    // count_kernel then sum the records per campaign block in LDS and add each touched
    // ring cell once (RecParams).  A full sub-buffer falls back to the atomic.
    u32 rec_on;
    u32 rec_bins;               // level-1 bins (campaign >> rec_shift), <= REC_BINS_MAX
    u32 rec_shift;
    u32 rec_cap;                // records per (workgroup, bin) sub-buffer
    u32* rec;                   // [grid][rec_bins][rec_cap]
    u32* rec_n;                 // [grid][rec_bins] records written
    u32 layout;                 // JSON layout tried first: 0 generator, 1 YSB_F_COMPACT_FIRST, 2 YSB_F_FLAT_FIRST
    // the join table's shard (ysb_load_ad_map_shard): a miss of a key whose shard is not
    // shard_rank counts as ST_FOREIGN (shard_n 1: unsharded).  Sharded contexts defer the
    // scan's misses (ctable_partial) so that only the deferred-line kernel classifies them.
    u32 shard_rank;
    u32 shard_n;
    // record mode: set when a view went to the u64 ring instead of a record (the exchange
    // then reads that ring too; ysb_capi.cpp exchange)
    u32* pend_dirty;
    // pinned host word (or null): defer_kernel stores the out-of-ring map's fill level there
    // (the host checks it at the next submit without waiting)
    u32* used_out;
    // layout 3 (a learned key order): the batch's key order as key indices (0 user_id,
    // 1 page_id, 2 ad_id, 3 ad_type, 4 event_type, 5 event_time, 6 ip_address), 3 bits per
    // key (key k in bits 3k..3k+2: no array, so no indexed private memory), read off its
    // first line by the host (ysb_capi.cpp learn_layout); learn_cp: compact separators
    u32 learn_code;
    u32 learn_n;
    u32 learn_cp;
};

// Record-mode pipeline after the scan (ysb_count.hip).  Level-2 bins ("blocks") are
// L2C = 32768 / W campaigns, so a block's L2C x W cells fit one workgroup's LDS as u32.
// Every stage writes whole 128-B lines from LDS staging: a partial-line store costs a
// memory write of its own (the XCD L2s are write-through for stores), which made scattered
// 4-B record stores as slow as the atomics they replace (tools/mb_scatter.hip).
constexpr int REC_BLOCK_CELLS = 32768;  // u32 LDS counters per count workgroup (128 KiB)
#ifndef YSB_REC_QUARTERS
#define YSB_REC_QUARTERS 64
#endif
constexpr int REC_QUARTERS = YSB_REC_QUARTERS;   // partition workgroups per level-1 bin (each a slice of the scan workgroups)
constexpr int REC_SUB_MAX = 512;      // level-2 blocks per level-1 bin (the partition's staging rings)
struct RecParams {
    const u32* rec;             // the scan's sub-buffers
    const u32* rec_n;
    u32 grid;                   // scan workgroups
    u32 bins;                   // level-1 bins
    u32 cap;                    // records per sub-buffer
    u32 sub_log2;               // level-2 blocks per level-1 bin = 1 << sub_log2
    u32 blk_shift;              // block = campaign >> blk_shift (L2C = 1 << blk_shift)
    u32 n_blocks;               // ceil(c_pad / L2C)
    u32 ring_w;
    u32 w_log2;
    u32 c_pad;
    u64 area;                   // u32 words of one (bin, quarter) output area
    u32* part;                  // partitioned records: [bins * QUARTERS][area], runs 32-record aligned
    u32* runs;                  // [n_blocks][QUARTERS] {offset, count} into part
    u8* delta;                  // the u8 delta ring [c_pad][W] (saturating: a cell that would pass
                                // 255 adds its whole value to the u64 ring instead and restarts at 0)
    unsigned long long* counts; // the u64 ring
    u32* dirty;                 // set when the count kernel added to the u64 ring
};
void launch_rec_partition(const RecParams& r, hipStream_t s);
void launch_rec_count(const RecParams& r, hipStream_t s);
// counts[i] += delta[i], delta[i] = 0 (cells: a multiple of 16)
void launch_fold(unsigned long long* counts, u8* delta, u64 cells, hipStream_t s);

// Range-limited exchange (ysb_group_reduce_scatter).  A rank's pending counts are its u64
// ring (read when force_u64 or *dirty) plus, in record mode, its u8 delta ring.
// xplan: slot_max[s] = max over campaigns of the pending count in ring slot s (atomicMax:
// zero slot_max first).  xpack: the pending cells of slots[0..R) as a dense [rows][R] array
// of `width`-byte cells (1, 4 or 8), the sources zeroed.  xunpack: owned[c][slots[k]] +=
// in[c][k] for the owner block's rows (through the saturating u8 accumulator owned8).
void launch_xplan(const unsigned long long* counts, const u8* delta, u32 W, u64 cells, int force_u64,
                  const u32* dirty, unsigned long long* slot_max, hipStream_t s);
void launch_xpack(unsigned long long* counts, u8* delta, u32 W, u32 rows, const u32* slots, u32 R, int force_u64,
                  const u32* dirty, void* out, u32 width, unsigned long long cap, hipStream_t s);
void launch_xunpack(unsigned long long* owned, u8* owned8, u32 W, u32 rows, const u32* slots, u32 R, const void* in,
                    u32 width, hipStream_t s);
// Linear checksum of a campaign-major [rows][W] u64 table (row i = campaign c_off + i) over
// the campaigns [c_lo, c_hi): *out += SUM count * cell_weight(campaign, bucket) (mod 2^64).
void launch_checksum(const unsigned long long* table, u32 rows, u32 W, i64 ring_lo, u32 c_off, u32 c_lo, u32 c_hi,
                     unsigned long long* out, hipStream_t s);

// BufferedReader.readLine's line split of raw bytes (ysb_split.hip): off[0..min(n, cap)) <-
// the line starts of b[0, nbytes) (b 16-byte aligned, nbytes < 4 GiB), *d_n <- n.  chunk:
// split_chunks(nbytes) u32 of scratch.  Asynchronous on s.
u64 split_chunks(u64 nbytes);
// the slots' host -> device copy by a kernel (ysb_split.hip): src a device-visible pinned host pointer
void launch_h2d_copy(void* dst, const void* src, u64 bytes, int cus, hipStream_t s, bool prio = false);
// the same from a device-visible host address at any byte alignment (reads up to 31 bytes
// past src + bytes, from the 16-byte boundary below src)
void launch_h2d_copy_unaligned(void* dst, const void* src, u64 bytes, int wgs, hipStream_t s);
hipError_t launch_split_lines(const u8* b, u64 nbytes, u32* chunk, u32* off, u64 cap, unsigned long long* d_n,
                              hipStream_t s);
// The replay's event-time rebasing (ysb_split.hip, ysb_submit_raw_mapped): for the first
// min(*d_n, tab_n, cap) lines of a split raw batch (starts off[0..cap)), the nine digits at line
// start + (tab[i] & 0xFFFF) <- lead + (tab[i] >> 16), zero-padded; writes stay inside [0, nbytes).
void launch_rebase(u8* b, u64 nbytes, const u32* off, u64 cap, const unsigned long long* d_n, u64 n_val,
                   const u32* tab, u64 tab_n, i64 lead, int cus, hipStream_t s);   // d_n NULL: n_val lines
// Layout sampling of device launches: sampled lines (spread over the launch's segments),
// copied on the device (in stream order after the batch's producer) into pinned host memory,
// SAMPLE_STRIDE bytes per line: u32 {line start, sampled length, valid, 0}, then
// <= SAMPLE_BYTES line bytes.
constexpr u32 SAMPLE_BYTES = 288;   // a line of the scan's tile capacity
constexpr u32 SAMPLE_STRIDE = 16 + SAMPLE_BYTES;
constexpr int SAMPLE_MAX = 64;
struct SampleSegs {                  // per sampled line: its batch and its index there
    const u8* bytes[SAMPLE_MAX];
    const u32* off[SAMPLE_MAX];
    u64 nbytes[SAMPLE_MAX];
    u64 n[SAMPLE_MAX];   // >= 1
    u64 line[SAMPLE_MAX];
};
void launch_sample(const SampleSegs& s, u32 nseg, u8* out, hipStream_t st);

constexpr int N_STAMPS = 8;     // phases timed by the YSB_STAMPS diagnostic build

void launch_scan(const ScanParams& p, hipStream_t s);
// The general-path lines the scan deferred (same stream, right after launch_scan).
void launch_defer(const ScanParams& p, int blocks, hipStream_t s);
// Sets ring[0..1] from the first lines of a batch if ring[1] == 0.
void launch_ring_autobase(const ScanParams& p, hipStream_t s);
// The pipe-delimited .tbl input format (YSB_F_FORMAT_TBL): scan + ring auto-base.
void launch_tbl_ring_autobase(const ScanParams& p, hipStream_t s);

// Generator kernels (ysb_gen.hip).
hipError_t gen_events_device(const GenSpec& spec, u64 first, u64 n, u8* d_out, u64 cap,
                             u32* d_off, u64* nbytes, hipStream_t s);
void launch_truth(const GenSpec& spec, u64 first, u64 n, const DivMagic& div,
                  unsigned long long* truth, u32 ring_w, const i64* ring,
                  unsigned long long* truth_outside, hipStream_t s);
// out[0] += #cells differing, out[1] += sum(truth), out[2] += sum(counts)
void launch_compare(const unsigned long long* a, const unsigned long long* b, u64 cells,
                    unsigned long long* out, hipStream_t s);
void launch_add_u64(unsigned long long* dst, const unsigned long long* src, u64 n, hipStream_t s);

// Table maintenance (ysb_table.hip): the non-zero cells of buckets [blo, blo + nb) of a
// campaign-major [rows][W] table as rows (campaign + c_off), optionally cleared.  With
// count_only only *out_n is incremented (by the number of such cells).
struct TableRow {
    u32 campaign;
    u32 pad;
    i64 bucket;
    unsigned long long count;
};
void launch_compact(unsigned long long* table, u32 rows, u32 W, i64 blo, u32 nb, u32 c_off, bool count_only,
                    bool clear, TableRow* out, u32* out_n, u32 cap, hipStream_t s);
// Empties the out-of-ring map (keys SIDE_EMPTY, counts 0).
void launch_side_clear(SideSlot* t, u64 slots, hipStream_t s);
// Every occupied slot of the out-of-ring map as rows (count_only: just the number).
void launch_side_compact(const SideSlot* t, u64 slots, u32 cbits, bool count_only, TableRow* out, u32* out_n,
                         u32 cap, hipStream_t s);

}  // namespace ysb
