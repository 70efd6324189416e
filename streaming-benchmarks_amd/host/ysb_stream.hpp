// ysb_stream.hpp -- the streaming mode of the native runner (BASELINE configs[4]): the
// reference's job running unbounded, as CampaignProcessorCommon runs it
// (streaming-benchmark-common/.../CampaignProcessorCommon.java:35-67, 91-98): records flow
// through the chain while a flusher writes every (campaign, window) delta once per second,
// and get-stats (data/src/setup/core.clj:130-149) reads time_updated - window_ms back as
// the latency of each window.
//
// Here a StreamingJob drives one context per shard (GPU), each fed through its pinned
// double-buffered slots (ysb_submit_raw) from a replay of pre-generated event lines, with
//   * event time   the replay's: the data/ generator's lines over one cycle of event time,
//                  cycled with every event_time moved by the cycle length (only the nine
//                  leading digits of a 13-digit time change: patched while the lines are
//                  copied into the slot); the lines of a cycle are released no earlier than
//                  their nominal emission time on the replay clock, which runs `speedup`
//                  times faster than the wall clock (a recorded stream played fast: every
//                  time relation of the reference -- 10 s windows, the 1 s flusher, the
//                  +-50 ms skew, the 100 ms buffer timeout -- holds in event time);
//   * watermark    the largest event_time submitted minus the out-of-orderness bound, the
//                  minimum over the shards (Flink's watermark at a keyed operator);
//   * flushes      every flushMs of event time, ysb_flush_begin on every shard (no drain of
//                  the stream), the rows taken by ysb_flush_end without waiting and written by
//                  a sink thread (Redis in the reference's schema, time_updated from the replay
//                  clock; and/or the CSV totals);
//   * windows      a window is closed by the first flush whose watermark has passed its end;
//                  its close latency is that flush's write time minus the window end, and each
//                  (campaign, window)'s time_updated - window_ms at that point is the sample
//                  get-stats reports (no event of a closed window can arrive later: skew +-50 ms
//                  under a 100 ms bound, and the late-by events are off unless asked for);
//   * the ring     follows the watermark (ysb_ring_advance, synchronous, rare: W - 16 buckets
//                  of event time apart), the buckets it leaves reported by a drain.
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
    unsigned threads = 0;             // copy threads (0: min(16, hardware))
    int64_t t0Ms = 1700000000000LL;   // nominal time of event 0 (a multiple of 10 000)
    bool timing = true;               // YSB_F_TIMING: the slots' copy time
};

// One flush as the sink sees it: every shard's deltas, the watermark at its begin and the
// replay-clock time it is written at (the writer's "now", CampaignProcessorCommon.java:84).
struct FlushRows {
    int64_t index = 0;
    int64_t watermarkMs = 0;
    std::vector<WindowDelta> rows;
};

struct StreamReport {
    uint64_t events = 0, batches = 0, flushes = 0, rowsWritten = 0;
    double wallSeconds = 0, eventsPerSecond = 0, targetEventsPerSecond = 0;
    double copyMs = 0, copyGBs = 0, copyBusyFrac = 0;
    uint64_t copyBytes = 0;
    uint64_t slotWaits = 0;           // submits that waited > 0.1 ms for the other slot's copy
    double slotWaitMs = 0, slotWaitMaxMs = 0;
    double maxBehindMs = 0;           // how late (wall ms) a batch was released after its time
    uint64_t ringAdvances = 0;
    std::vector<uint64_t> cycles;     // per shard: whole replay cycles submitted ...
    std::vector<uint64_t> partialLines;   // ... and the lines of the next one
    uint64_t linesPerCycle = 0;
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
    // Generates the replay cycles (one per shard) and opens the contexts.  The campaign and ad
    // ids are the generator's (ysb_gen_ids): campaignIds()[i] is campaign index i's UUID.
    void prepare();
    StreamReport run(const FlushSink& sink);
    const std::vector<std::string>& campaignIds() const { return campaigns_; }
    // CPU check of the replay (no GPU): a cycle from the host generator, each batch of each of
    // `cycles` rebased into a buffer and compared byte for byte with the host generator's own
    // lines of that cycle (t0 moved by cycle * cycleMs).  A JSON summary.
    static std::string replaySelfCheck(const StreamOptions& o, const std::vector<uint64_t>& cycles);
    ~StreamingJob();

private:
    struct Shard;
    StreamOptions o_;
    std::vector<std::string> campaigns_, ads_;
    std::vector<Shard*> shards_;
};

}  // namespace topology
}  // namespace ysb
