/*
 * ysb_hip.h -- C ABI of the MI355X-native YSB advertising hot path.
 *
 * One library (libysb_hip.so) replaces the Flink operator chain
 *   DeserializeBolt -> EventFilterBolt -> project(ad_id, event_time)
 *   -> RedisJoinBolt -> keyBy(campaign) -> CampaignProcessor/CampaignProcessorCommon
 * of the reference (flink-benchmarks/src/main/java/flink/benchmark/
 * AdvertisingTopologyNative.java:111-138) with hand-written gfx950 kernels.
 * Every entry point below names the reference interface it stands in for.
 *
 * Conventions
 *   - plain C, no exceptions cross the ABI; every call returns an int status,
 *     0 = YSB_OK, negative = error; ysb_last_error(ctx) explains the last one.
 *   - one ysb_ctx per Flink subtask and per GPU; calls on one ctx are not
 *     concurrent (the reference's operators are single-threaded per subtask).
 *   - counts are exact 64-bit integers (the reference's Window.seenCount is a
 *     java.lang.Long, streaming-benchmark-common/.../Window.java:9).
 */
#ifndef YSB_HIP_H
#define YSB_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ysb_stats.foreign_shard, YSB_F_STRICT, ysb_load_ad_map(_packed)_shard, the
 *    range-limited exchange (ysb_group_exchange_info / ysb_exchange_plan),
 *    ysb_group_checksum, layout selection on by default (YSB_F_LAYOUT_FIXED turns it off),
 *    ysb_sync's sticky YSB_ERR_CAPACITY, the collective ysb_ring_advance after
 *    ysb_group_init, ysb_gen_params.variant
 * 3: raw batches with the line split on the GPU (ysb_submit_raw, ysb_split_lines_device),
 *    ysb_slot_capacity, ysb_copy_time; device batches' layout sampled in stream order
 * 4: ysb_device_count; a busy stream's device batches take the sampled layout only when two
 *    samples agree (else the per-tile dispatch, never a host wait for the launch queued
 *    last); a raw batch that cannot launch is a sticky error (ysb_stream returns NULL);
 *    raw batches hold at most max(max_batch_events, max_batch_bytes / 32) lines
 * 5: ysb_device_sync, ysb_device_numa_node; batches read in place from caller-registered host
 *    memory (ysb_host_register; raw lines: ysb_submit_raw_mapped; offsets in device memory:
 *    ysb_submit_mapped) with the replay's event-time rebasing on the device
 *    (ysb_rebase_table); ysb_exchange_info_size (the struct grew in ABI 4: a caller
 *    checks the size it was built with); YSB_F_TIMING's event records are folded into running
 *    totals, so a caller that never reads them keeps a bounded number */
#define YSB_ABI_VERSION 5

/* status codes */
#define YSB_OK            0
#define YSB_ERR_ARG      (-1)  /* bad argument / size                      */
#define YSB_ERR_HIP      (-2)  /* HIP runtime failure                      */
#define YSB_ERR_STATE    (-3)  /* call not valid in the current state      */
#define YSB_ERR_CAPACITY (-4)  /* batch, table or output buffer too small  */
#define YSB_ERR_FORMAT   (-5)  /* malformed ad map / config                */
#define YSB_ERR_RCCL     (-6)  /* RCCL failure                             */
#define YSB_ERR_NOMEM    (-7)  /* host or device allocation failed         */
#define YSB_ERR_DATA     (-8)  /* strict mode: the batch held records the
                                  reference would have thrown on           */
#define YSB_PENDING        1   /* ysb_flush_end(wait = 0): not complete yet (not an error) */

/* ysb_config.flags */
#define YSB_F_TIMING       0x1u /* record HIP events around every scan launch */
#define YSB_F_REQUIRE_IP   0x2u /* also require a string "ip_address" (the Storm/
                                   Spark deserializers read 7 fields:
                                   storm-benchmarks/.../AdvertisingTopology.java:56-62,
                                   AdvertisingSpark.scala:124-134; Flink reads 6:
                                   AdvertisingTopologyNative.java:267-272)      */
#define YSB_F_NO_LDS_COUNT 0x4u /* disable the per-workgroup LDS window counters
                                   (every joined view becomes a global atomic)   */
#define YSB_F_FORMAT_TBL  0x10u /* batches are the fork's pipe-delimited .tbl lines
                                   user_id|page_id|ad_id|ad_type|event_type|event_time
                                   (MockWindowedFlatMap, AdvertisingTopologyNative.java:
                                   197-226) instead of JSON                       */
#define YSB_F_RECORD_COUNT 0x20u /* count joined views in record mode wherever possible (the
                                   default: only for rings >= 1M cells and launches >= 1M
                                   events without LDS window counters; ysb_path_time).
                                   Record mode needs the HBM-resident join table (the
                                   bucket layout ysb_load_ad_map builds for tables beyond
                                   64 MB): with a cache-resident table the flag has no
                                   effect.  ysb_path_time's record_launches tells which
                                   launches used it.                                    */
#define YSB_F_NO_RECORD_COUNT 0x40u /* never: one global atomic per joined view             */
#define YSB_F_COMPACT_FIRST 0x80u /* layout hint: JSON lines are expected as compact JSON
                                   ({"user_id":"...","page_id":...} -- no space after ':'
                                   or ','); the scan tries that layout first and the
                                   generator's (core.clj:90-96) as a later tier.  Counts
                                   are identical either way; only the speed differs.
                                   Every join-table layout (since ABI 3 also the HBM-
                                   resident table's serial-probe / record-mode kernels). */
#define YSB_F_FLAT_FIRST 0x100u /* layout hint: JSON lines are flat objects in any key
                                   order or spacing (another producer's serializer); the
                                   scan parses every line with its flat-object tier first
                                   (generator-layout lines too, a little slower than their
                                   own path) -- unless a batch's first line names one key
                                   order of DeserializeBolt's keys with one spacing: then
                                   the learned-order instantiation, which sends lines off
                                   that order to the same flat tier (without
                                   YSB_F_LAYOUT_FIXED).  Counts are identical; takes
                                   precedence over YSB_F_COMPACT_FIRST.  Every join-table
                                   layout (since ABI 3). */
#define YSB_F_LAYOUT_AUTO 0x200u /* (the default since ABI 2; the bit is accepted and
                                   ignored) layout read from the data: every submit picks
                                   the scan instantiation from 64 stratified lines of the
                                   launch (since ABI 3; ABI 2: the first line) -- host
                                   batches from the pinned slot, device batches from
                                   <= 288-byte samples taken on the device in stream order
                                   (ysb_submit_device) -- the generator's layout, compact
                                   JSON, a learned key order (the sampled order and
                                   spacing, checked in place on every line), when 46 of
                                   the 64 agree; else (several producers) the per-tile
                                   dispatch (layout 4) when the sample's adjacent lines
                                   are mostly alike (producers writing in runs), the
                                   flat-object tier (2) when they are not.  Counts
                                   are identical whichever runs.  The explicit hints above
                                   take precedence.  Every join-table layout: since ABI 3
                                   the HBM-resident table's serial-probe and record-mode
                                   kernels (configs[2]) have the layout instantiations
                                   too. */
#define YSB_F_LAYOUT_FIXED 0x800u /* no layout sampling: the generator's layout first (or
                                   the explicit hint); device batches are then never read
                                   by the host before their launch */
#define YSB_F_H2D_SDMA 0x1000u   /* the slots' host-to-device copies by the DMA engine
                                   (hipMemcpyAsync) instead of a copy kernel reading the
                                   pinned slot (the default since ABI 4): on this pool DMA
                                   copies run at half rate in episodes after the GPU idled
                                   ("H2D") */
#define YSB_F_STRICT 0x400u      /* ysb_sync (and the calls built on it) return YSB_ERR_DATA
                                   once a record the reference would have thrown on was seen
                                   (parse_errors / time_errors: JSONObject / getString /
                                   Long.parseLong exceptions fail the Flink task,
                                   AdvertisingTopologyNative.java:263-272,
                                   CampaignProcessorCommon.java:58) or a view whose ad_id
                                   belongs to another rank's shard (foreign_shard: input
                                   routed by another hash than the join table's).  Sticky
                                   until ysb_reset; the counts of the other records stay
                                   exact and readable through ysb_stats_get. */
#define YSB_F_SPARSE_FAST_JOIN 0x8u /* test hook: leave every other 36-byte key out of
                                   the fast-path cuckoo table, as a failed cuckoo
                                   placement would; its misses then take the
                                   general path (results unchanged)              */

typedef struct ysb_ctx ysb_ctx;

typedef struct ysb_config {
    int64_t  time_divisor_ms;    /* 10000: CampaignProcessorCommon.java:28           */
    uint32_t n_campaigns;        /* campaign index space [0, n_campaigns)            */
    uint32_t window_ring;        /* W: live (campaign, bucket) slots per campaign,
                                    power of two >= 16 (the reference keeps <= 9 live
                                    buckets: LRUHashMap(10), CampaignProcessorCommon.java:37) */
    uint64_t max_ads;            /* capacity of the device ad -> campaign table      */
    uint64_t max_batch_events;   /* per ysb_submit                                   */
    uint64_t max_batch_bytes;    /* per ysb_submit, <= 4 GiB (u32 line offsets)      */
    int64_t  ring_base_bucket;   /* first bucket of the ring; INT64_MIN = take it from
                                    the first event of the first batch              */
    uint64_t overflow_capacity;  /* (campaign, bucket) deltas outside the ring that
                                    are kept exactly in a side list                  */
    uint32_t flags;              /* YSB_F_*                                          */
    uint32_t reserved;
} ysb_config;

/* Running totals since ysb_open / ysb_reset. */
typedef struct ysb_stats {
    uint64_t events;       /* lines scanned                                          */
    uint64_t views;        /* parsed lines with event_type == "view"
                              (EventFilterBolt, AdvertisingTopologyNative.java:434)   */
    uint64_t joined;       /* views whose ad_id is in the map (RedisJoinBolt :464)   */
    uint64_t join_misses;  /* views dropped on a map miss (:465-467)                 */
    uint64_t parse_errors; /* lines org.json's JSONObject/getString would throw on
                              (:263-272)                                             */
    uint64_t time_errors;  /* joined views whose event_time Long.parseLong rejects
                              (CampaignProcessorCommon.java:58)                       */
    uint64_t out_of_ring;  /* joined views counted through the overflow side list    */
    uint64_t overflow_dropped; /* side-list entries lost for lack of capacity (must be 0) */
    uint64_t batches;      /* submits                                                */
    uint64_t deferred;     /* lines the fast path handed to the general tokenizer    */
    uint64_t foreign_shard; /* views dropped on a map miss whose ad_id belongs to another
                              rank's shard (ysb_load_ad_map_shard): mis-routed input, not a
                              miss of the reference's map; join_misses excludes them      */
} ysb_stats;

/* One (campaign, window) delta: the unit the Redis writer HINCRBYs into
 * <windowUUID>.seen_count (AdvertisingSpark.scala:184-208,
 * CampaignProcessorCommon.java:70-88 (commented in the fork)). */
typedef struct ysb_count {
    uint32_t campaign;     /* campaign index                                         */
    uint32_t reserved;
    int64_t  window_ms;    /* bucket * time_divisor_ms = Redis window timestamp
                              (CampaignProcessorCommon.java:103)                      */
    uint64_t count;
} ysb_count;

/* ---- lifecycle ---------------------------------------------------------------- */

int         ysb_abi_version(void);
void        ysb_config_default(ysb_config* cfg);
/* The HIP devices this process sees (hipGetDeviceCount; 0 when there is none or the runtime
 * fails).  A launcher maps rank -> device with it (one context per GPU, the reference's one
 * subtask per slot) without a framework's device query. */
int         ysb_device_count(void);
/* hipDeviceSynchronize on `device` through the library's own HIP runtime (ABI 5): a host
 * (bench.py, a JVM) that must wait for the whole GPU without loading a framework's HIP
 * runtime.  A process may hold only one working HIP/HSA runtime: if another one (e.g. the
 * libamdhip64 a framework bundles) opens the GPU first, this library's runtime may see no
 * device, and ysb_open / ysb_device_sync fail with a message that says so (INTEGRATION.md
 * section 1.4a: load order). */
int         ysb_device_sync(int device);
/* The NUMA node of `device`'s PCI function (sysfs numa_node of hipDeviceGetPCIBusId's address;
 * -1 when unknown), ABI 5: where a caller's registered batches and feeder threads for this GPU
 * belong (each Flink source instance NUMA-local to the GPU its chain runs on). */
int         ysb_device_numa_node(int device);

/* Replaces CampaignProcessorCommon(String)/prepare() (CampaignProcessorCommon.java:30-55)
 * and RedisJoinBolt.open() (AdvertisingTopologyNative.java:451-458). */
int         ysb_open(ysb_ctx** out, int device, const ysb_config* cfg);
int         ysb_close(ysb_ctx* ctx);
/* ctx may be NULL: then the last error of a failed ysb_open on this thread. */
const char* ysb_last_error(const ysb_ctx* ctx);

/* Replaces getAdCampaignMap + RedisJoinBolt(Map) (AdvertisingTopologyNative.java:47-56,
 * 443-448) and RedisAdCampaignCache (RedisAdCampaignCache.java:23-35): builds the
 * GPU-resident open-addressing ad_id -> campaign table.  ad_ids[i] points at
 * ad_id_lens[i] bytes (NULL lens = 36 each, the UUID length); a later duplicate
 * wins, as HashMap.put does.  Keys are matched as exact byte strings (<= 56 B). */
int         ysb_load_ad_map(ysb_ctx* ctx, const char* const* ad_ids,
                            const uint32_t* ad_id_lens, const uint32_t* campaign_idx,
                            uint64_t n);
/* Same for n keys of key_len bytes packed back to back (a JNI byte[] of UUIDs; config 3
 * loads 10M ads this way). */
int         ysb_load_ad_map_packed(ysb_ctx* ctx, const char* keys, uint32_t key_len,
                                   const uint32_t* campaign_idx, uint64_t n);
/* The join table sharded 1/nranks per GPU: of the n entries only
 * those with ysb_ad_shard(ad_id, nranks) == rank are loaded, and the context remembers its
 * shard.  A view whose ad_id misses the table is then classified on the miss path only:
 * an ad of another shard counts as foreign_shard (input routed by another hash -- with
 * YSB_F_STRICT ysb_sync fails with YSB_ERR_DATA), any other as a join miss that the
 * reference's RedisJoinBolt would drop too (AdvertisingTopologyNative.java:443-448,
 * 465-467).  nranks = 1 is ysb_load_ad_map. */
int         ysb_load_ad_map_shard(ysb_ctx* ctx, const char* const* ad_ids,
                                  const uint32_t* ad_id_lens, const uint32_t* campaign_idx,
                                  uint64_t n, uint32_t rank, uint32_t nranks);
int         ysb_load_ad_map_packed_shard(ysb_ctx* ctx, const char* keys, uint32_t key_len,
                                         const uint32_t* campaign_idx, uint64_t n,
                                         uint32_t rank, uint32_t nranks);

/* ---- batches --------------------------------------------------------------------
 * A batch is n_events JSON lines packed back to back in `bytes`; line i spans
 * [line_off[i], line_off[i+1]) (the last one ends at nbytes).  This replaces the
 * per-record FlatMapFunction.flatMap calls of the chain
 * (AdvertisingTopologyNative.java:111-119 / 122-138). */

/* Library-owned pinned staging buffers for double-buffered slots 0 and 1, each
 * max_batch_bytes / max_batch_events large.  Fill, then ysb_submit the slot. */
int         ysb_slot_buffers(ysb_ctx* ctx, int slot, uint8_t** bytes, uint32_t** line_off);
/* Asynchronous: H2D copy on the copy stream, kernel on the compute stream.
 * bytes/line_off may be the slot's own buffers (zero-copy staging) or any host
 * memory (copied into the slot first).  The caller must not touch the slot's
 * buffers until ysb_wait(ctx, slot). */
int         ysb_submit(ysb_ctx* ctx, int slot, const uint8_t* bytes, uint64_t nbytes,
                       const uint32_t* line_off, uint64_t n_events);
int         ysb_wait(ysb_ctx* ctx, int slot);
/* The capacity the context was opened with (ysb_config.max_batch_bytes / max_batch_events):
 * the size of each slot's pinned buffers from ysb_slot_buffers, for a caller (e.g. a JNI
 * NewDirectByteBuffer over them) that must not write past them. */
int         ysb_slot_capacity(ysb_ctx* ctx, uint64_t* max_bytes, uint64_t* max_events);
/* A raw batch: whole lines as bytes, no offsets.  The line starts are found on the GPU
 * (ysb_split.hip) where BufferedReader.readLine ends a line -- '\n', "\r\n" or a lone '\r';
 * a last line without a terminator is a line, a terminator that ends the batch starts none --
 * so the caller (FileBasedDataSource.run, AdvertisingTopologyNative.java:144-165) only reads
 * the file into the pinned slot (max_batch_bytes bytes, at most max(max_batch_events,
 * max_batch_bytes / 32) lines: the device keeps 4 B per line start, not per byte).
 * Asynchronous and double-buffered like ysb_submit: H2D on the copy stream, the split right
 * behind it on the same stream (with YSB_F_H2D_SDMA: on a stream of its own); the batch's scan
 * is launched once its line count is back, at the next call on the context (the next submit,
 * ysb_sync, ...), so a caller that fills the other slot in between keeps the copies going;
 * ysb_wait(ctx, slot) before the slot's pinned buffer is rewritten.  A batch that cannot
 * launch (more lines than the slot holds: YSB_ERR_CAPACITY, or a HIP failure) is dropped, and
 * its error is returned by the call that performs the launch and by every later call that
 * orders work after it, until ysb_reset. */
int         ysb_submit_raw(ysb_ctx* ctx, int slot, const uint8_t* bytes, uint64_t nbytes);
/* Zero-copy raw batches (ABI 5).  ysb_host_register pins and maps caller host memory (a JNI
 * DirectByteBuffer, a replay file read into memory) for this context's device, so that
 * ysb_submit_raw_mapped reads a batch in place over PCIe -- no copy into the pinned slot, no
 * host pass over the bytes (the streaming replay's ingest: FileBasedDataSource.run,
 * AdvertisingTopologyNative.java:144-165, with the source's buffer itself pinned).  Ranges
 * must not overlap; ysb_close unregisters what is left. */
int         ysb_host_register(ysb_ctx* ctx, void* host, uint64_t bytes);
int         ysb_host_unregister(ysb_ctx* ctx, void* host);
/* The replay's event-time rebasing on the device (the data/ generator's batch replay output,
 * core.clj:166-174 played past its first cycle).  A replay cycle's line i holds its 13-digit
 * event_time at byte time_at[i] & 0xFFFF of the line, and its leading nine digits (the
 * 10-second bucket) equal lead_base + (time_at[i] >> 16).  The table (4 B per line) is copied
 * into HBM; n_lines = 0 drops it. */
int         ysb_rebase_table(ysb_ctx* ctx, const uint32_t* time_at, uint64_t n_lines, int64_t lead_base);
typedef struct ysb_rebase {
    uint64_t first_line;   /* the batch's first line is the table's line first_line         */
    int64_t  lead_shift;   /* added to every line's leading nine digits (cycle k of a cycle of
                              c ms: k * c / 10000); the result must lie in [0, 10^9)         */
} ysb_rebase;
/* ysb_submit_raw of a batch that lies in a registered range: at any byte address (a file
 * mapping's batch starts where the previous one's last line ended), the range holding the batch
 * widened to 16-byte boundaries on both sides (the copy reads whole 16-byte vectors).  The copy
 * kernel (or, YSB_F_H2D_SDMA, the DMA
 * engine) reads it in place into the slot's device buffer, the GPU splits the lines, and with
 * rebase != NULL every line's leading event_time digits are rewritten from the rebase table
 * before the scan (YSB_ERR_ARG at the launch if the batch has more lines than the table holds
 * from first_line).  Asynchronous like ysb_submit_raw; the caller must not rewrite the bytes
 * until ysb_wait(ctx, slot).  The slot's pinned host buffer is not used. */
int         ysb_submit_raw_mapped(ysb_ctx* ctx, int slot, const uint8_t* bytes, uint64_t nbytes,
                                  const ysb_rebase* rebase);
/* The same for a batch whose record boundaries the source already knows (a Kafka source's
 * messages; a replay cycle's line offsets, computed once and kept in HBM for every cycle):
 * d_line_off holds n_events u32 offsets into `bytes` in device memory.  No line split: the copy
 * kernel reads the bytes in place, the scan (after the rebase, with rebase != NULL: lines
 * [first_line, first_line + n_events) of the table) is enqueued behind it on the compute stream
 * at once.  The call first waits for the slot's previous copy (at most two in flight); the
 * caller must not rewrite the bytes until ysb_wait(ctx, slot). */
int         ysb_submit_mapped(ysb_ctx* ctx, int slot, const uint8_t* bytes, uint64_t nbytes,
                              const uint32_t* d_line_off, uint64_t n_events, const ysb_rebase* rebase);
/* The same split of a device-resident batch (16-byte aligned, < 4 GiB): d_off[0..*n) <- its
 * line starts (YSB_ERR_CAPACITY, *n = the lines, if more than cap).  Synchronous. */
int         ysb_split_lines_device(ysb_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes, uint32_t* d_off,
                                   uint64_t cap, uint64_t* n);
/* Device-resident batch (HBM pointers, e.g. from ysb_device_alloc). Asynchronous.  The batch
 * must be complete when submitted, or its producer ordered before the compute stream
 * (hipStreamWaitEvent(ysb_stream(ctx), ...), or produced on that stream).  Unless
 * YSB_F_LAYOUT_FIXED, 64 stratified lines of the launch (ABI 2: each segment's first line) are
 * copied into pinned memory by a small kernel on the compute stream (so after that producer)
 * to pick the scan's instantiation (46 of 64 must agree, else the per-tile dispatch or the flat
 * tier): the launch's own sample when the compute stream is idle at the submit (the host waits
 * for that copy, microseconds); else the previous launch's sample if the one before it decided
 * the same (the host waits for that copy, which is queued behind the launch before the
 * previous one -- never for the launch just queued), and the per-tile dispatch when the two
 * disagree (producers alternating by batch: every producer's tiles still take its own path) or
 * no earlier sample exists.  A producer that changes its layout on a busy stream therefore
 * runs one launch through the old instantiation, then the dispatch until two samples agree;
 * counts never depend on the choice (ysb_launch_info tells which ran). */
int         ysb_submit_device(ysb_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes,
                              const uint32_t* d_line_off, uint64_t n_events);
/* Several device-resident batches in ONE kernel launch.  Each segment is a batch as
 * for ysb_submit_device (its own u32 line offsets, so each stays under 4 GiB); every
 * scan workgroup walks its run of tiles in segment 0, then segment 1, ..., so a step
 * over many batches pays one launch tail instead of one per batch.  Results are the
 * same as n_segs ysb_submit_device calls in order.  At most 16 segments and 2^31-1
 * events per call.  Replaces the same flatMap chain as ysb_submit (:111-119), for a
 * replay file larger than 4 GiB (FileBasedDataSource.run, :144-165). */
typedef struct ysb_segment {
    const uint8_t*  d_bytes;       /* HBM, 16-byte aligned */
    uint64_t        nbytes;        /* < 4 GiB */
    const uint32_t* d_line_off;    /* HBM, n_events offsets into d_bytes */
    uint64_t        n_events;
} ysb_segment;
int         ysb_submit_device_segments(ysb_ctx* ctx, const ysb_segment* segs, uint32_t n_segs);
/* Wait for every submitted batch.  YSB_ERR_CAPACITY if joined views were lost because
 * the out-of-ring map and its fallback list (overflow_capacity) both filled (stats.
 * overflow_dropped > 0): counts are then not exact, and every ysb_sync / ysb_drain reports
 * it until ysb_reset.  The map is emptied into the exact host-side list once it is a
 * quarter full: here, and at every submit from its fill level after the launch before
 * the previous one (read without waiting).  So a chain of submits without ysb_sync loses
 * counts only if ONE or two launches fill the map from below a quarter to full
 * (overflow_capacity distinct out-of-ring cells).  With YSB_F_STRICT, YSB_ERR_DATA once a
 * record the reference would have thrown on (or a foreign-shard view) was seen. */
int         ysb_sync(ysb_ctx* ctx);

/* ---- results ------------------------------------------------------------------------
 * Replaces CampaignProcessorCommon.flushWindows/writeWindow
 * (CampaignProcessorCommon.java:41-54, 69-98): returns the nonzero
 * (campaign, window) deltas with bucket in [bucket_lo, bucket_hi) (ring + side
 * list), sorted by (campaign, window).  clear != 0 zeroes what was returned (a
 * flush: the next drain reports only new deltas).  out == NULL: *n_out = rows
 * needed.  After ysb_group_reduce_scatter the ring part covers only this rank's
 * campaign block (every rank still reports its own side-list deltas; deltas are
 * additive, exactly like the HINCRBY they feed). */
int         ysb_drain(ysb_ctx* ctx, int64_t bucket_lo, int64_t bucket_hi, int clear,
                      ysb_count* out, uint64_t cap, uint64_t* n_out);
/* Asynchronous flush for streaming callers: CampaignProcessorCommon's flusher thread
 * (CampaignProcessorCommon.java:35-55, 91-98) writes every second while records keep flowing.
 * ysb_flush_begin enqueues, behind every batch submitted so far (a pending raw batch is launched
 * first), the compaction of the ring's nonzero (campaign, bucket) cells of [bucket_lo,
 * bucket_hi) straight into pinned host rows, clearing them on the device, and returns without
 * waiting: the stream keeps running.  Up to 4 flushes may be outstanding.  ysb_flush_end
 * returns the oldest one's rows sorted by (campaign, window): with wait = 0 it returns
 * YSB_PENDING if the device has not reached it yet; out = NULL: *n_out = rows needed (the rows
 * stay until they are taken).  A flush holds at most min(n_campaigns * window_ring, 2^20) rows:
 * cells beyond that keep their counts for the next flush (*more = 1).  Counts outside the ring
 * (the out-of-ring map and the side list) are not part of an asynchronous flush -- ysb_drain
 * reports them; deltas are additive, so a caller that sums flushes and drains has every count
 * exactly once.  Not after ysb_group_init (YSB_ERR_STATE). */
int         ysb_flush_begin(ysb_ctx* ctx, int64_t bucket_lo, int64_t bucket_hi);
int         ysb_flush_end(ysb_ctx* ctx, int wait, ysb_count* out, uint64_t cap, uint64_t* n_out, int* more);
int         ysb_stats_get(ysb_ctx* ctx, ysb_stats* out);
/* Zero counts, side list and stats; the ad table is kept. */
int         ysb_reset(ysb_ctx* ctx);
/* Bucket range currently held by the ring: [*lo, *lo + window_ring). */
int         ysb_ring_range(ysb_ctx* ctx, int64_t* lo, uint32_t* width);
/* Moves the ring to [new_lo, new_lo + window_ring) (streaming: follow the watermark).
 * Counts of buckets leaving the ring move to the exact host-side list and are reported
 * by later drains; events of buckets outside the new range keep going to the side list.
 * Replaces the LRU eviction of old buckets (LRUHashMap(10), CampaignProcessorCommon.java:37,
 * LRUHashMap.java:18-19) without its loss of counts.  After ysb_group_init this is a
 * collective: every rank calls it with the same new_lo (YSB_ERR_ARG on every rank if they
 * differ). */
int         ysb_ring_advance(ysb_ctx* ctx, int64_t new_lo);

/* ---- measurement -------------------------------------------------------------------- */
/* With YSB_F_TIMING: total device time of the scan kernel launches (HIP events on
 * the compute stream) and the number of launches since the last call (resets). */
int         ysb_kernel_time(ysb_ctx* ctx, double* total_ms, uint64_t* launches);
/* With YSB_F_TIMING: device time of the host-to-device copies of ysb_submit / ysb_submit_raw
 * (HIP events on the copy stream), their number and bytes since the last call (resets). */
int         ysb_copy_time(ysb_ctx* ctx, double* total_ms, uint64_t* copies, uint64_t* bytes);
/* The same launches' whole device sequence -- scan, general-path and (record mode)
 * partition + count kernels -- as measured by the last ysb_kernel_time call (which
 * collects both), and the launches so far that used record mode. */
int         ysb_path_time(ysb_ctx* ctx, double* total_ms, uint64_t* launches, uint64_t* record_launches);
/* The scan instantiation the last launch ran: the JSON layout tried first (0 the
 * generator's, 1 compact JSON, 2 the flat-object tier, 3 a learned key order, 4 the per-tile
 * dispatch for several producers in one batch; what layout sampling or a hint chose), record-mode counting, the HBM-resident join table (bucket layout, serial
 * probes), the .tbl format -- each 0 or 1. */
typedef struct ysb_launch_desc {
    uint32_t layout;
    uint32_t record_mode;
    uint32_t hbm_table;
    uint32_t tbl;
} ysb_launch_desc;
int         ysb_launch_info(ysb_ctx* ctx, ysb_launch_desc* out);
/* The layout sampling's decision for one line (host function; what every submit applies
 * to its batch's first line): 0 the generator's layout (core.clj:90-96), 1 its keys in its
 * order as compact JSON, 3 another order or subset of DeserializeBolt's keys with one
 * consistent spacing -- order[0..*n) then receives the key indices (0 user_id, 1 page_id,
 * 2 ad_id, 3 ad_type, 4 event_type, 5 event_time, 6 ip_address) and *compact the spacing
 * -- or 2 anything else (the flat-object tier first).  require_ip: YSB_F_REQUIRE_IP's
 * rule (ip_address must be among the keys). */
int         ysb_layout_of_line(const uint8_t* line, uint64_t len, int require_ip, uint32_t order[8],
                               uint32_t* n, uint32_t* compact);
/* The compute stream (hipStream_t) for callers that want to order work with it (a pending
 * raw batch is launched first); NULL if that launch failed (ysb_last_error). */
void*       ysb_stream(ysb_ctx* ctx);

/* ---- device memory helpers (so host code needs no framework for HBM buffers) ----------- */
int         ysb_device_alloc(ysb_ctx* ctx, uint64_t bytes, void** d_ptr);
int         ysb_device_free(ysb_ctx* ctx, void* d_ptr);
int         ysb_memcpy_h2d(ysb_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes);
int         ysb_memcpy_d2h(ysb_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes);

/* ---- multi-GPU: replaces the keyBy(0) shuffle (AdvertisingTopologyNative.java:118) ----
 * Events are sharded by ad_id hash across ranks; the per-rank (campaign, window)
 * tables are summed with one RCCL reduce-scatter over xGMI, leaving rank r the
 * owner of campaigns [r*Cp/N, (r+1)*Cp/N), Cp = n_campaigns padded to N. */
#define YSB_UNIQUE_ID_BYTES 128
int         ysb_group_unique_id(uint8_t uid[YSB_UNIQUE_ID_BYTES]);
/* Collective.  Also agrees on the ring base (every rank's ring must start at the same
 * bucket: the tables are summed cell by cell): the smallest base any rank holds wins; a
 * rank whose ring starts later moves the buckets the common range does not hold to its
 * exact side list.  If no rank has a base yet, the first ysb_group_reduce_scatter agrees.
 * After ysb_group_init, ysb_ring_advance is collective too (same new_lo on every rank). */
int         ysb_group_init(ysb_ctx* ctx, int rank, int nranks,
                           const uint8_t uid[YSB_UNIQUE_ID_BYTES]);
/* The same group over the caller's own collectives instead of RCCL (a job whose ranks
 * already share a transport; the test rehearsal of N ranks on one GPU, where RCCL refuses
 * two ranks per device).  Both callbacks run on the calling thread, on host memory, and
 * must be collective over the nranks ranks; nonzero = failure:
 *   allreduce_max_u64: buf[0..n) <- elementwise max over the ranks, in place;
 *   reduce_scatter_sum: recv[0..count) <- sum over the ranks of their send blocks
 *     [rank * count, (rank + 1) * count), cells of `width` bytes (1, 4 or 8), unsigned. */
typedef struct ysb_collectives {
    int (*allreduce_max_u64)(void* user, uint64_t* buf, uint64_t n);
    int (*reduce_scatter_sum)(void* user, const void* send, void* recv, uint64_t count, uint32_t width);
    void* user;
} ysb_collectives;
int         ysb_group_init_host(ysb_ctx* ctx, int rank, int nranks, const ysb_collectives* ops);
/* Collective: sums the ranks' pending counts (everything counted since the previous call)
 * into the owner ranks' tables and zeroes them.  Range-limited, like the reference's keyed
 * shuffle, which carries only the touched (campaign, window) pairs: per ring bucket the
 * largest pending count on any rank is agreed by one W-element all-reduce(max) (the call's
 * only wait for the device), and only the buckets holding a count travel, as a dense
 * [C_pad][buckets] array of the narrowest cell width that cannot wrap in the sum (1 byte
 * while nranks * max <= 255, else 4, else 8) through one ncclReduceScatter.  The rest is
 * asynchronous on the compute stream.  Record mode's u8 delta ring is read directly (no
 * fold): configs[2]'s 1M campaigns x 100 live buckets move 100 MB per rank and exchange
 * instead of the whole 1 GB u64 ring. */
int         ysb_group_reduce_scatter(ysb_ctx* ctx);
/* Collective, the streaming form of ysb_group_reduce_scatter: no wait for the device.  This
 * call's per-bucket maxima are only enqueued (all-reduced and read back asynchronously);
 * the buckets and width that travel are the PREVIOUS call's plan, read back while the
 * step's scan ran.  Counts in buckets outside that plan, or larger than its width sums over
 * the ranks, stay pending for a later exchange (nothing is lost or double counted; the
 * owners' tables lag by at most one call).  The first call after ysb_group_init, ysb_reset
 * or ysb_ring_advance is a complete ysb_group_reduce_scatter; a complete call settles
 * everything (do one before reading the owned tables).  Every rank must use the same
 * sequence of the two calls. */
int         ysb_group_exchange_pipelined(ysb_ctx* ctx);
/* Exchange accounting: exchanges run, reduce-scatter input bytes this rank contributed
 * (campaign rows x the planned buckets, each run widened to aligned groups of 4 ring slots,
 * x the cell width), device
 * time of the exchanges (HIP events: plan, all-reduce(max), read-back, pack, reduce-scatter,
 * unpack), of their part on the compute stream (critical_ms: plan to pack, plus the unpack --
 * what the launches queue behind; the reduce-scatter runs on a stream of its own beside the
 * next launch, and the unpack is enqueued on the compute stream at the next exchange or read),
 * the last exchange's bucket count and cell width (0: nothing was pending), what one
 * whole-ring u64 exchange would move, the reduce-scatters' own time (rs_ms: pack done to
 * reduce-scatter done, on the exchange stream, waiting for the peers included) and the part of
 * it the compute stream stood waiting for at the unpack (exposed_ms; rs_ms - exposed_ms ran
 * hidden beside the launches queued since -- a complete exchange exposes all of it).  reset != 0
 * zeroes the totals after reading them.  (ABI 4 appended rs_ms and exposed_ms.) */
typedef struct ysb_exchange_info {
    uint64_t exchanges;
    uint64_t bytes;
    double   ms;
    uint32_t last_buckets;
    uint32_t last_width;
    uint64_t full_ring_bytes;
    double   critical_ms;
    double   rs_ms;
    double   exposed_ms;
} ysb_exchange_info;
int         ysb_group_exchange_info(ysb_ctx* ctx, ysb_exchange_info* out, int reset);
/* sizeof(ysb_exchange_info) as this library writes it (ABI 5): a caller built against an older
 * header (ABI 3: 48 bytes) must not pass its smaller struct to ysb_group_exchange_info. */
uint64_t    ysb_exchange_info_size(void);
/* The plan every rank derives from the all-reduced per-bucket maxima (host function):
 * slots[0..*n_slots) = the ring slots with slot_max > 0, ascending; *width = the cell width
 * above.  YSB_ERR_CAPACITY if nranks * max does not fit 64 bits. */
int         ysb_exchange_plan(const uint64_t* slot_max, uint32_t W, uint32_t nranks, uint32_t* slots,
                              uint32_t* n_slots, uint32_t* width);
/* Linear checksums for a multi-rank check that moves no tables (sum over cells of count x
 * an odd 64-bit weight of (campaign, bucket), mod 2^64, so checksums add like the tables):
 *   YSB_SUM_TRUTH_BLOCKS   out[r], r < nranks: the generator truth's cells of owner block r
 *   YSB_SUM_PENDING_BLOCKS out[r], r < nranks: this rank's pending (not yet exchanged) cells
 *   YSB_SUM_OWNED          out[0]: this rank's owned table (its block, after exchanges)
 * After ysb_group_reduce_scatter on every rank: OWNED of rank r + SUM over ranks of
 * PENDING[r] == SUM over ranks of TRUTH[r]. */
#define YSB_SUM_TRUTH_BLOCKS   0
#define YSB_SUM_PENDING_BLOCKS 1
#define YSB_SUM_OWNED          2
int         ysb_group_checksum(ysb_ctx* ctx, int what, uint32_t nranks, uint64_t* out);
int         ysb_group_owned(ysb_ctx* ctx, uint32_t* campaign_lo, uint32_t* campaign_hi);
/* The communicator as RCCL sees it (ncclCommUserRank / ncclCommCount): a check that the
 * exchange really spans the ranks the launcher started. */
int         ysb_group_info(ysb_ctx* ctx, int* rank, int* nranks);
/* Shard of an ad_id under the partitioning above (host function). */
uint32_t    ysb_ad_shard(const char* ad_id, uint32_t len, uint32_t nranks);
/* Campaign block [*lo, *hi) that rank `rank` of `nranks` owns after
 * ysb_group_reduce_scatter (host function, no context needed; ysb_group_owned of an
 * initialised context reports the same block).  Replaces the key -> subtask mapping of
 * Flink's keyBy(0) hash partitioner (AdvertisingTopologyNative.java:118-119). */
int         ysb_group_block(uint32_t n_campaigns, int rank, int nranks, uint32_t* lo, uint32_t* hi);
/* Host router for batches that are not pre-sharded: out_shard[i] = ysb_ad_shard of line
 * i's top-level "ad_id" string, its escapes decoded to UTF-8 as org.json and the device
 * decode them (an escaped key name is found too; generator lines: bytes 113..148; other
 * layouts: a key scan); lines without one go to shard 0.  shard_counts (nranks
 * entries, may be NULL) receives the lines per shard.  Routing must match the join table:
 * with a sharded table (ysb_load_ad_map_shard) only this hash is exact -- a view routed
 * elsewhere misses and is counted as foreign_shard (an error under YSB_F_STRICT); with the
 * whole map on every rank (ysb_load_ad_map) any deterministic routing is exact. */
int         ysb_route_lines(const uint8_t* bytes, uint64_t nbytes, const uint32_t* line_off,
                            uint64_t n, uint32_t nranks, uint32_t* out_shard,
                            uint64_t* shard_counts);

/* ---- synthetic input: the data/ generator's event format (core.clj:61-98, 163-181)
 * restated as a seeded, counter-based generator with a file-dump mode.  Host and
 * device produce byte-identical lines for the same parameters. */
typedef struct ysb_gen_params {
    uint64_t seed;
    uint32_t n_campaigns;       /* 100 (core.clj:15)                                  */
    uint32_t ads_per_campaign;  /* 10 ((partition 10 ads), core.clj:52)               */
    int64_t  t0_ms;             /* event_time of event 0                              */
    uint64_t events_per_sec;    /* event time advances 1000/rate ms per event;
                                   100 reproduces catch-up mode (10 ms, core.clj:95)   */
    uint32_t with_skew;         /* 1: +-50 ms skew, 1e-5 late by <60 s (core.clj:166-174);
                                   2: the skew only (out of order, never late)         */
    uint32_t n_users;           /* 0: a fresh user/page UUID per event (core.clj:79-80);
                                   k: draw from a pool of k (core.clj:187-188)         */
    const uint32_t* ad_subset;  /* optional: draw ads only from these indices (shards) */
    uint32_t n_ad_subset;
    uint32_t event_stream;      /* 0: the single-stream generator; k > 0: an independent
                                   event stream over the SAME campaign/ad ids (one per
                                   rank of a sharded run); ids depend on seed only     */
    uint32_t format;            /* YSB_GEN_JSON (core.clj:90-97 lines) or YSB_GEN_TBL (the
                                   fork's .tbl rows of the same events, :197-226)       */
    uint32_t variant;           /* 0: the generator's own lines; YSB_GEN_RANDOM_IP /
                                   YSB_GEN_MORE_AD_TYPES / YSB_GEN_COMPACT / YSB_GEN_REORDER:
                                   the same events as other producers would write them (a
                                   random dotted-quad ip_address, 8 ad_types, no space after
                                   ':' and ',', the keys in another fixed order) --
                                   lines the vocabulary fast path does not take; the views,
                                   ads and times (and so the truth) are unchanged except that
                                   YSB_GEN_MORE_AD_TYPES draws the ad_type from 8           */
} ysb_gen_params;
#define YSB_GEN_JSON 0u
#define YSB_GEN_TBL  1u
#define YSB_GEN_RANDOM_IP     1u
#define YSB_GEN_MORE_AD_TYPES 2u
#define YSB_GEN_COMPACT       4u
#define YSB_GEN_REORDER       8u
#define YSB_GEN_MIXED        16u  /* four producers interleaved line by line: each event's layout drawn
                                     from {the generator's, compact, reordered keys, random ip with 8
                                     ad_types}; the same events and truth */
#define YSB_GEN_MIXED_BLOCKS 32u  /* the same four producers in runs of 256 events (drawn per run) */

void        ysb_gen_default(ysb_gen_params* p);
/* Campaign and ad UUIDs, 36 bytes each, no separators (ad a -> campaign a / ads_per_campaign). */
int         ysb_gen_ids(const ysb_gen_params* p, char* campaign_ids, char* ad_ids);
/* Events [first, first+n) into out (cap bytes); line offsets relative to out. */
int         ysb_gen_events_host(const ysb_gen_params* p, uint64_t first, uint64_t n,
                                uint8_t* out, uint64_t cap, uint32_t* line_off,
                                uint64_t* nbytes);
/* The same with `threads` host threads (lengths, their prefix, then the lines in place): a
 * real-time producer fast enough to load the streaming path (configs[4] under load). */
int         ysb_gen_events_host_mt(const ysb_gen_params* p, uint64_t first, uint64_t n, uint8_t* out,
                                   uint64_t cap, uint32_t* line_off, uint64_t* nbytes, uint32_t threads);
/* Same on the device (d_out / d_line_off are HBM); synchronous. */
int         ysb_gen_events_device(ysb_ctx* ctx, const ysb_gen_params* p, uint64_t first,
                                  uint64_t n, uint8_t* d_out, uint64_t cap,
                                  uint32_t* d_line_off, uint64_t* nbytes);
/* Upper bound of one generated line in bytes. */
uint64_t    ysb_gen_max_line_bytes(const ysb_gen_params* p);
/* Generator truth, independent of any parsing: adds the (campaign, bucket) view
 * counts of events [first, first+n) to a second device table ("truth") laid out
 * like the ring; ysb_truth_compare counts ring/truth cells that differ. */
int         ysb_truth_accumulate(ysb_ctx* ctx, const ysb_gen_params* p, uint64_t first,
                                 uint64_t n);
int         ysb_truth_compare(ysb_ctx* ctx, uint64_t* mismatched_cells,
                              uint64_t* truth_total, uint64_t* ring_total);
/* The truth table itself: n_campaigns x window_ring u64, campaign-major, cell (c, b mod W)
 * holding bucket b of [*ring_lo, *ring_lo + W) (cells >= n_campaigns * window_ring).  Lets
 * a multi-rank check sum the ranks' truths and compare them with the owners' drains. */
int         ysb_truth_read(ysb_ctx* ctx, uint64_t* out, uint64_t cells, int64_t* ring_lo);
/* Writes the generator's files into dir: campaign-ids.txt, ad-ids.txt (core.clj:24-34),
 * ad-to-campaign-ids.txt ({ "AD": "CAMPAIGN"} lines, core.clj:58), ad-to-campaign.csv
 * (ad,campaign lines, AdvertisingTopologyNative.java:52) and kafka-json.txt with
 * n_events events (core.clj:76-97). */
int         ysb_gen_dump(const ysb_gen_params* p, uint64_t n_events, const char* dir);
/* The fork's events.tbl rows from generator-format JSON lines (the external tool that
 * wrote conf/benchmarkConf.yaml:6's events.tbl is not in the reference):
 * user_id|page_id|ad_id|ad_type|event_type|event_time\n per line, values copied raw.
 * YSB_ERR_FORMAT for a line that is not 7 unescaped "key": "value" pairs in the
 * generator's key order (core.clj:90-96); YSB_ERR_CAPACITY if out (cap bytes) is short. */
int         ysb_json_to_tbl(const uint8_t* bytes, uint64_t nbytes, const uint32_t* line_off,
                            uint64_t n, uint8_t* out, uint64_t cap, uint32_t* out_off,
                            uint64_t* out_nbytes);
/* Sharded file-dump mode (config 4's pre-sharded replay files): the id and map files
 * as ysb_gen_dump, and events [0, n_events) split by ysb_route_lines into
 * kafka-json.<r>.txt for r in [0, nranks). */
int         ysb_gen_dump_shards(const ysb_gen_params* p, uint64_t n_events, const char* dir,
                                uint32_t nranks);

#ifdef __cplusplus
}
#endif
#endif /* YSB_HIP_H */
