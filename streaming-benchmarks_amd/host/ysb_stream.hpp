// ysb_stream.hpp -- the streaming mode of the native runner (BASELINE configs[4]): the
// reference's job running unbounded, as CampaignProcessorCommon runs it
// (streaming-benchmark-common/.../CampaignProcessorCommon.java:35-67, 91-98): records flow
// through the chain while a flusher writes every (campaign, window) delta once per second,
// and get-stats (data/src/setup/core.clj:130-149) reads time_updated - window_ms back as
// the latency of each window.
//
// A StreamingJob drives one context per shard (GPU).  Like the reference, where every parallel
// source instance feeds its own operator chain (AdvertisingTopologyNative.java:97-99,114-119),
// every shard has a feeder thread of its own, pinned to its GPU's NUMA node, that owns the
// shard's context: it releases the shard's batches on the replay clock, begins and takes the
// shard's flushes, and moves the shard's ring.  The main thread only runs the flusher's clock,
// merges the shards' flushes and hands them to the sink thread.
//
//   * event time   the replay's: the data/ generator's lines over one cycle of event time,
//                  cycled with every event_time moved by the cycle length; the lines of a cycle
//                  are released no earlier than their nominal emission time on the replay clock,
//                  which runs `speedup` times faster than the wall clock (a recorded stream
//                  played fast: every time relation of the reference -- 10 s windows, the 1 s
//                  flusher, the +-50 ms skew, the 100 ms buffer timeout -- holds in event time);
//   * ingest       (mapped, the default) the cycle sits in host memory laid out batch by batch
//                  (each batch 64-byte aligned), registered with the shard's context once
//                  (ysb_host_register), its line offsets in HBM (computed once: every cycle
//                  reuses them, as a Kafka source knows its message boundaries); a batch is
//                  handed over in place (ysb_submit_mapped): the GPU's copy kernel reads it over
//                  PCIe and the nine leading event_time digits are rewritten on the GPU for the
//                  cycle being played (ysb_rebase_table) -- no host pass over the bytes, and
//                  nothing but copies on the copy queue.  (mapped-raw: the same with the line
//                  split on the GPU, ysb_submit_raw_mapped; copy, round 5's path: the feeder
//                  copies the batch into the pinned slot and patches the digits itself.)
//   * watermark    per shard the largest event_time submitted minus the out-of-orderness bound;
//                  a merged flush's watermark is the minimum over the shards at their begins
//                  (Flink's watermark at a keyed operator);
//   * flushes      every flushMs of event time each shard begins a flush (ysb_flush_begin, no
//                  drain of the stream) and takes it when ready (ysb_flush_end without waiting);
//                  the merged flush is written by a sink thread (Redis in the reference's schema,
//                  time_updated from the replay clock; and/or the CSV totals);
//   * windows      a window is closed by the first flush whose watermark has passed its end;
//                  its close latency is that flush's write time minus the window end, and each
//                  (campaign, window)'s time_updated - window_ms at that point is the sample
//                  get-stats reports;
//   * the ring     each shard's follows its own watermark (ysb_ring_advance, synchronous, rare:
//                  W - 16 buckets of event time apart), the buckets it leaves reported by a drain.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "ysb_topology.hpp"

namespace ysb {
namespace topology {

struct StreamOptions {
    int shards = 1;
    int device = 0;                   // shard s runs on device (device + s) % ysb_device_count()
    uint64_t seed = 42;               // the generator (core.clj:61-98, ysb_gen_params)
    uint32_t campaigns = 100, adsPerCampaign = 10;
    int skew = 2;                     // with_skew: 1 the reference's (+-50 ms, 1e-5 late < 60 s), 2 skew only
    double eventRate = 5e6;           // events per second of event time, per shard
    double speedup = 32;              // event-time ms per wall-clock ms
    int64_t cycleMs = 10000;          // replay cycle, a multiple of 10 000 ms
    int64_t flushMs = 1000;           // CampaignProcessorCommon's flusher period (:45), event time
    int64_t batchMs = 100;            // setBufferTimeout(100) (AdvertisingTopologyNative.java:79), event time
    int64_t oooMs = 100;              // max out-of-orderness of the watermark
    double seconds = 12;              // wall seconds of input
    uint64_t slotBytes = 256ull << 20;
    uint32_t windowRing = 64;
    unsigned threads = 0;             // host threads per shard for preparing (and, copy mode, filling) (0: 16 / shards)
    int64_t t0Ms = 1700000000000LL;   // nominal time of event 0 (a multiple of 10 000)
    bool timing = true;               // YSB_F_TIMING: the slots' copy time (folded by the library)
    // ingest: MAPPED in place from the registered cycle, its line offsets kept in HBM
    // (ysb_submit_mapped); MAPPED_RAW in place with the line split on the GPU
    // (ysb_submit_raw_mapped); COPY round 5's host copy into the pinned slot (ysb_submit_raw)
    enum Replay { MAPPED = 0, MAPPED_RAW = 1, COPY = 2 };
    int replay = MAPPED;
    bool pinNuma = true;              // feeder threads (and the cycle's pages) on the GPU's NUMA node
};

// One flush as the sink sees it: every shard's deltas, the watermark at its begin and the
// replay-clock time it is written at (the writer's "now", CampaignProcessorCommon.java:84).
struct FlushRows {
    int64_t index = 0;
    int64_t watermarkMs = 0;
    std::vector<WindowDelta> rows;
};

struct ShardReport {
    int device = 0, numaNode = -1;
    bool pinned = false;              // the feeder ran on its GPU's node's CPUs
    uint64_t events = 0, batches = 0, cycles = 0, partialLines = 0;
    double submitMs = 0;              // wall time inside the submit calls (incl. the wait for the line count)
    double feederCpuS = 0;            // the feeder thread's CPU time
    double maxBehindMs = 0;           // how late (wall ms) a batch was released after its time
    uint64_t ringAdvances = 0;
    double replayGB = 0, prepareS = 0, registerS = 0;
};

struct StreamReport {
    uint64_t events = 0, batches = 0, flushes = 0, rowsWritten = 0;
    // wall time from the first submit to the last batch counted (every shard's ysb_sync) and
    // events / that; the submit-side rate (first to last submit) separately
    double wallSeconds = 0, eventsPerSecond = 0, submitEventsPerSecond = 0, targetEventsPerSecond = 0;
    double copyMs = 0, copyGBs = 0, copyBusyFrac = 0;
    uint64_t copyBytes = 0;
    uint64_t slotWaits = 0;           // submits that took > 1 ms (the copy queue was full)
    double slotWaitMs = 0, slotWaitMaxMs = 0;
    double maxBehindMs = 0;
    uint64_t ringAdvances = 0;
    std::vector<uint64_t> cycles;     // per shard: whole replay cycles submitted ...
    std::vector<uint64_t> partialLines;   // ... and the lines of the next one
    uint64_t linesPerCycle = 0;
    std::vector<ShardReport> shards;
    // windows closed by the watermark: close latency (write time - window end)
    std::vector<double> closeReplayMs;
    // per (campaign, window) of those windows: time_updated - window_ms at the close (get-stats)
    std::vector<double> cwReplayMs;
    uint64_t openAtEnd = 0;
    int64_t finalWatermarkMs = 0;     // the watermark at the last flush: windows ending by it are closed
    uint64_t overflowDropped = 0, parseErrors = 0, joinMisses = 0;
};

// sink(flush, nowMs): writes one flush's rows with the replay clock's now (ms).
using FlushSink = std::function<void(const FlushRows&, int64_t nowMs)>;

class StreamingJob {
public:
    explicit StreamingJob(const StreamOptions& o);
    // Opens the contexts and generates the replay cycles (one per shard, each on its own
    // thread on its GPU's NUMA node).  The campaign and ad ids are the generator's
    // (ysb_gen_ids): campaignIds()[i] is campaign index i's UUID.
    void prepare();
    StreamReport run(const FlushSink& sink);
    const std::vector<std::string>& campaignIds() const { return campaigns_; }
    // CPU check of the replay (no GPU): a cycle from the host generator, each batch of each of
    // `cycles` rebased into a buffer (the host restatement of the device rebase) and compared
    // byte for byte with the host generator's own lines of that cycle (t0 moved by cycle *
    // cycleMs).  A JSON summary.
    static std::string replaySelfCheck(const StreamOptions& o, const std::vector<uint64_t>& cycles);
    // CPU measurement of the copy feeders (no GPU): `shards` host cycles, each shard's feeder on
    // a thread of its own filling its slot buffer as fast as it can for `seconds` (round 5's fill:
    // memcpy + digit patch).  A JSON summary with the aggregate events/s.  (The mapped feeder has
    // no per-byte host work: its cost per batch is the submit call, measured by the GPU run.)
    static std::string feedCheck(const StreamOptions& o, double seconds);
    // CPU check of the shards' flush merge (no GPU): `shards` threads deliver `flushes` flushes
    // each, at random moments, with jittered watermarks and one delta row per flush, through the
    // runner's own merger and sink thread.  Checks: the sink sees every index once, in order,
    // with every shard's rows and the minimum of the shards' watermarks; the windows it closes
    // are exactly those the merged watermarks pass.  A JSON summary ("ok": true|false).
    static std::string mergeCheck(int shards, int flushes, uint64_t seed);
    ~StreamingJob();

private:
    struct Shard;
    StreamOptions o_;
    std::vector<std::string> campaigns_, ads_;
    std::vector<Shard*> shards_;
};

// The NUMA node of a GPU (its PCI device's numa_node; -1 unknown) and the CPUs of a node this
// process may run on (empty: none / unknown).
int gpuNumaNode(int device);
std::vector<int> nodeCpus(int node);

}  // namespace topology
}  // namespace ysb
