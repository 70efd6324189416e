// ysb_topology.hpp -- the C++ host side above the C ABI (include/ysb_hip.h): the
// reference's Flink job (flink-benchmarks/src/main/java/flink/benchmark/
// AdvertisingTopologyNative.java:58-142) restated with the reference's class names,
// argument meanings and error behaviour, driving the GPU operator instead of the
// per-record Java chain.
//
//   Config::findAndReadConfigFile   benchmark.common.Utils.findAndReadConfigFile (Utils.java:29-63)
//   AdCampaignMap                   AdvertisingTopologyNative.getAdCampaignMap (:47-56) and the
//                                   generator's JSON map lines (data/src/setup/core.clj:58)
//   FileBasedDataSource             FileBasedDataSource.run (:144-165): readLine over events_path
//   GpuAdCampaignOperator           DeserializeBolt -> EventFilterBolt -> project -> RedisJoinBolt
//                                   -> keyBy -> CampaignProcessor (:111-119 / :122-138), one operator
//   RedisWindowWriter               CampaignProcessorCommon.writeWindow (CampaignProcessorCommon.java:69-89)
//                                   / AdvertisingSpark.writeWindow (AdvertisingSpark.scala:184-208)
//
// Errors surface as exceptions (std::runtime_error) where the reference's Java code
// throws; records the reference would have dropped are dropped and counted.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "ysb_hip.h"

namespace ysb {
namespace topology {

// ---- configuration ---------------------------------------------------------------------
// The YAML subset conf/benchmarkConf.yaml uses: `key: scalar`, `key:` followed by
// `- item` lines, `#` comments, single/double-quoted scalars.
class Config {
public:
    static Config findAndReadConfigFile(const std::string& path, bool mustExist);
    static Config parse(const std::string& text);
    bool has(const std::string& key) const;
    const std::string& get(const std::string& key) const;          // throws when missing
    std::string get(const std::string& key, const std::string& dflt) const;
    long long getLong(const std::string& key) const;               // throws when missing / not a number
    const std::vector<std::string>& getList(const std::string& key) const;
    const std::map<std::string, std::string>& scalars() const { return scalars_; }
    const std::map<std::string, std::vector<std::string>>& lists() const { return lists_; }

private:
    std::map<std::string, std::string> scalars_;
    std::map<std::string, std::vector<std::string>> lists_;
};

// java.io.BufferedReader.readLine over a whole text: "\n", "\r\n" and "\r" end a line.
std::vector<std::string> readLines(const std::string& text);
// java.lang.String.split(one literal char, limit 0): trailing empty items dropped.
std::vector<std::string> javaSplit(const std::string& s, char sep);
std::string readFile(const std::string& path);

// ---- ad -> campaign map -------------------------------------------------------------------
struct AdCampaignMap {
    std::vector<std::string> campaigns;                 // campaign index -> UUID
    std::vector<std::string> ads;                       // distinct ads, first-appearance order
    std::vector<uint32_t> adCampaign;                   // ads[i] -> campaign index
    // CSV `ad,campaign` (split(","); kv[0] -> kv[1]; a later duplicate wins; a line with
    // fewer than two items throws, as ArrayIndexOutOfBounds does) or JSON map lines
    // `{ "AD": "CAMPAIGN"}` (merged left to right, core.clj:104-106): chosen by content.
    static AdCampaignMap fromFile(const std::string& path);
    static AdCampaignMap fromCsv(const std::string& text);
    static AdCampaignMap fromJsonLines(const std::string& text);

private:
    std::unordered_map<std::string, uint32_t> campaignIndex_, adIndex_;
    void put(const std::string& ad, const std::string& campaign);
};

// ---- event source ----------------------------------------------------------------------------
// Threads that stay up for the source's lifetime: run(n, f) calls f(t) for t in [0, n) on
// n threads (the caller's is t = 0) and returns when all are done.
class WorkerPool;

// The events file as complete lines ('\n'-terminated; the last line may lack it), read
// in large blocks straight into a caller buffer, by parallel preads of a persistent pool;
// a partial line at the end of a block is carried into the next one.  Empty lines are
// records, as readLine returns them.
class FileBasedDataSource {
public:
    // threads: readers/splitters per block (0 = min(16, hardware threads)).  mmap: read by
    // parallel copies out of a read-only mapping of the file (no syscall per piece) instead of
    // parallel preads.
    explicit FileBasedDataSource(const std::string& path, unsigned threads = 0, bool mmap = true);
    ~FileBasedDataSource();
    FileBasedDataSource(const FileBasedDataSource&) = delete;
    FileBasedDataSource& operator=(const FileBasedDataSource&) = delete;
    // Fills buf (cap bytes) with whole lines and off (maxLines) with their offsets;
    // returns the number of lines (0 = end of file).  Throws if one line exceeds cap.
    uint64_t fill(uint8_t* buf, uint64_t cap, uint32_t* off, uint64_t maxLines, uint64_t* nbytes);
    // The same without the line split: buf receives whole lines, the return value is their
    // bytes (0 = end of file); the GPU finds the line starts (ysb_submit_raw).
    uint64_t fillRaw(uint8_t* buf, uint64_t cap);
    // Zero-copy (mmap mode only): the next whole lines, at most cap bytes, where they lie in the
    // mapping -- *p points into it, the return value is their bytes (0 = end of file).  The
    // GPU reads them in place (ysb_submit_raw_mapped) once the mapping is registered.
    uint64_t nextMapped(uint64_t cap, const uint8_t** p);
    // The mapping (NULL without mmap) and its registrable length (whole pages).
    const uint8_t* mapping() const { return map_; }
    uint64_t mappingBytes() const;
    // Back to the file's start (a replay source read again).
    void rewind();
    uint64_t linesRead() const { return lines_; }
    uint64_t bytesRead() const { return bytes_; }

private:
    int fd_ = -1;
    const uint8_t* map_ = nullptr;      // the file mapped read-only (mmap mode)
    uint64_t size_ = 0;
    uint64_t pos_ = 0;                  // file offset of the next read
    unsigned threads_ = 1;
    std::unique_ptr<WorkerPool> pool_;
    std::vector<uint8_t> carry_;
    bool eof_ = false;
    uint64_t lines_ = 0, bytes_ = 0;
    uint64_t readBlock(uint8_t* buf, uint64_t cap);   // carry + file bytes into buf: bytes held
    uint64_t completeEnd(const uint8_t* buf, uint64_t have, bool anyCr) const;
};

// One (campaign, window) delta: what writeWindow HINCRBYs into seen_count.
struct WindowDelta {
    std::string campaign;
    int64_t windowMs;
    uint64_t count;
};

// ---- the operator -------------------------------------------------------------------------------
class GpuAdCampaignOperator {
public:
    struct Options {
        int device = 0;
        int64_t timeDivisorMs = 10000;      // CampaignProcessorCommon.java:28
        uint32_t windowRing = 1024;
        uint64_t batchBytes = 256ull << 20;
        uint64_t batchEvents = 1ull << 20;
        bool tbl = false;                   // MockWindowedFlatMap's .tbl rows (:197-226)
        bool requireIp = false;             // Storm/Spark's 7-field deserializer
        bool gpuSplit = true;               // fillFromRaw + ysb_submit_raw: line starts found on the GPU
        bool h2dSdma = false;               // YSB_F_H2D_SDMA: the slot's H2D by the DMA engine (default: a copy kernel)
        bool mappedIo = false;              // the source's mapping registered, batches read in place (--io mapped)
    };
    GpuAdCampaignOperator(const AdCampaignMap& map, const Options& o);
    ~GpuAdCampaignOperator();
    GpuAdCampaignOperator(const GpuAdCampaignOperator&) = delete;
    GpuAdCampaignOperator& operator=(const GpuAdCampaignOperator&) = delete;

    void open();                                           // RichFlatMapFunction.open
    void flatMap(const char* line, uint64_t len);          // one record
    uint64_t fillFrom(FileBasedDataSource& src);           // a slot's worth of records, zero-copy
    uint64_t fillFromRaw(FileBasedDataSource& src);        // the same as raw lines (bytes returned)
    void registerSource(FileBasedDataSource& src);         // pin + map the source's mapping (mappedIo)
    uint64_t submitMapped(FileBasedDataSource& src);       // the next whole lines, read in place: bytes
    void submit();                                         // hand the open slot to the GPU
    std::vector<WindowDelta> flushWindows();               // CampaignProcessorCommon.flushWindows (:91-98)
    void close();                                          // RichFlatMapFunction.close
    ysb_stats stats();
    uint64_t submittedEvents() const { return submitted_; }
    // host seconds spent filling slots (fillFrom / fillFromRaw) and waiting for a slot's H2D
    double fillSeconds() const { return fillS_; }
    double waitSeconds() const { return waitS_; }
    // the slots' H2D: total ms, copies and bytes (YSB_F_TIMING, ysb_copy_time)
    void copyTime(double* ms, uint64_t* copies, uint64_t* bytes);

private:
    const AdCampaignMap& map_;
    Options o_;
    ysb_ctx* ctx_ = nullptr;
    double fillS_ = 0, waitS_ = 0;
    uint8_t* bytes_[2] = {nullptr, nullptr};
    uint32_t* off_[2] = {nullptr, nullptr};
    int cur_ = 0;
    uint64_t fillBytes_ = 0, fillEvents_ = 0, submitted_ = 0, rawBytes_ = 0;
    void check(int rc, const char* what);
};

// ---- output -------------------------------------------------------------------------------------------
class RespClient;   // RESP2 over a TCP socket

class RedisWindowWriter {
public:
    RedisWindowWriter(const std::string& host, int port);
    ~RedisWindowWriter();
    // writeWindow for every delta of one flush, in two pipelined round trips; time_updated is
    // nowMs (the wall clock when negative; a streaming replay passes its replay clock).
    void writeWindows(const std::vector<WindowDelta>& rows, int64_t nowMs = -1);
    uint64_t roundTrips() const { return trips_; }

private:
    std::unique_ptr<RespClient> r_;
    std::map<std::pair<std::string, std::string>, std::string> windowUuid_;
    std::map<std::string, std::string> listUuid_;
    uint64_t trips_ = 0;
};

// Totals per (campaign, window) written as `campaign_id,window_ms,count` lines.
class CsvWindowSink {
public:
    void add(const std::vector<WindowDelta>& rows);
    void write(const std::string& path) const;
    uint64_t windows() const { return totals_.size(); }

private:
    std::map<std::pair<std::string, int64_t>, uint64_t> totals_;
};

std::string randomUuid();

}  // namespace topology
}  // namespace ysb
