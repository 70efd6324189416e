// ysb_topology -- the native drop-in for `flink run ... AdvertisingTopologyNative
// --confPath conf/benchmarkConf.yaml` (flink-benchmarks/.../AdvertisingTopologyNative.java:
// 58-142): reads the same YAML keys, the same ad map and events files, runs the chain on
// one GPU, and writes the (campaign, window) counts to Redis in the reference's schema
// (or to a CSV file).
//
//   ysb_topology --confPath PATH [--device N] [--sink none|csv:FILE|redis[:HOST[:PORT]]]
//                [--format json|tbl] [--flush-ms MS] [--batch-mb MB | --batch-bytes B] [--batch-events N]
//                [--window-ring W] [--require-ip] [--dry-run] [--print-config]
//                [--replay-rows CSV] [--host-split] [--repeat K] [--io-threads T] [--io mmap|pread]
//
// --dry-run reads the config, the map and the events file (FileBasedDataSource) without a
// GPU and reports what it found; --replay-rows writes the (campaign_id,window_ms,count)
// rows of a CSV through the sink without a GPU (the Redis writer on its own).  The events
// file is read as raw lines and the GPU finds the line starts (ysb_submit_raw); --host-split
// splits the lines on the host instead (ysb_submit with offsets).  --repeat K reads the file
// K times (a replay source; the counts are K times the file's).  The last stdout line is a
// JSON summary.
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ysb_stream.hpp"
#include "ysb_topology.hpp"

using namespace ysb::topology;

namespace {

struct Args {
    std::string conf, sink = "none", format, replay;
    int device = 0;
    long long flush_ms = 1000;                  // CampaignProcessorCommon's flusher period (:45)
    long long batch_bytes = 256ll << 20, batch_events = 1 << 20;
    unsigned window_ring = 1024;
    bool require_ip = false, dry = false, print_config = false, host_split = false;
    long long repeat = 1;
    unsigned io_threads = 0;
    bool io_mmap = true;
    // --io mapped: the mapping registered, batches read in place by the GPU; auto (the default):
    // that whenever the GPU splits the lines and the slots' copy is the copy kernel's, with
    // slot copies out of the mapping if the registration is refused
    std::string io = "auto";
    bool h2d_sdma = false;
    // streaming mode (configs[4]): --stream plus its options (ysb_stream.hpp)
    bool stream = false;
    StreamOptions so;
    std::string stream_csv;   // per-(campaign, window) totals of everything written
    bool self_check = false;  // --stream-self-check: the replay's rebasing on the CPU, no GPU
    bool feed_check = false;  // --stream-feed-check: the feeders' host rate on the CPU, no GPU
    bool merge_check = false; // --stream-merge-check: the shards' flush merge on the CPU, no GPU
    int merge_flushes = 400;
    double feed_seconds = 2;
};

void usage() {
    std::fprintf(stderr,
                 "usage: ysb_topology --confPath PATH [--device N] [--sink none|csv:FILE|redis[:HOST[:PORT]]]\n"
                 "       [--format json|tbl] [--flush-ms MS] [--batch-mb MB | --batch-bytes B] [--batch-events N]\n"
                 "       [--window-ring W] [--require-ip] [--dry-run] [--print-config] [--replay-rows CSV]\n"
                 "       [--host-split] [--repeat K] [--io-threads T] [--io auto|mapped|mmap|pread]\n"
                 "       [--h2d-sdma]\n"
                 "   or: ysb_topology --stream [--sink none|csv:FILE|redis[:HOST[:PORT]]] [--shards N] [--device D]\n"
                 "       [--seed S] [--campaigns C] [--ads-per-campaign A] [--event-rate E] [--speedup F]\n"
                 "       [--cycle-ms MS] [--flush-ms MS] [--batch-ms MS] [--ooo-ms MS] [--seconds S]\n"
                 "       [--batch-mb MB] [--window-ring W] [--skew 0|1|2] [--io-threads T] [--totals CSV]\n"
                 "       [--replay mapped|mapped-raw|copy] [--no-numa] [--no-timing]\n"
                 "   or: ysb_topology --stream-self-check | --stream-feed-check [--shards N] [--feed-seconds S] ...\n"
                 "   or: ysb_topology --stream-merge-check [--shards N] [--merge-flushes F] [--seed S]\n");
}

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        if (k == "--confPath") a.conf = val();
        else if (k == "--device") a.device = std::atoi(val().c_str());
        else if (k == "--sink") a.sink = val();
        else if (k == "--format") a.format = val();
        else if (k == "--flush-ms") a.flush_ms = std::atoll(val().c_str());
        else if (k == "--batch-mb") a.batch_bytes = (long long)std::atoll(val().c_str()) << 20;
        else if (k == "--batch-bytes") a.batch_bytes = std::atoll(val().c_str());
        else if (k == "--batch-events") a.batch_events = std::atoll(val().c_str());
        else if (k == "--window-ring") a.window_ring = (unsigned)std::atoll(val().c_str());
        else if (k == "--require-ip") a.require_ip = true;
        else if (k == "--dry-run") a.dry = true;
        else if (k == "--print-config") a.print_config = true;
        else if (k == "--replay-rows") a.replay = val();
        else if (k == "--host-split") a.host_split = true;
        else if (k == "--repeat") a.repeat = std::max(1ll, std::atoll(val().c_str()));
        else if (k == "--io-threads") a.io_threads = (unsigned)std::atoll(val().c_str());
        else if (k == "--io") {
            const std::string m = val();
            if (m != "mmap" && m != "pread" && m != "mapped" && m != "auto") { usage(); std::exit(2); }
            a.io_mmap = m != "pread";
            a.io = m;
        }
        else if (k == "--h2d-sdma") a.h2d_sdma = true;
        else if (k == "--stream") a.stream = true;
        else if (k == "--stream-self-check") { a.stream = true; a.self_check = true; }
        else if (k == "--shards") a.so.shards = std::atoi(val().c_str());
        else if (k == "--seed") a.so.seed = std::strtoull(val().c_str(), nullptr, 10);
        else if (k == "--campaigns") a.so.campaigns = (uint32_t)std::atoll(val().c_str());
        else if (k == "--ads-per-campaign") a.so.adsPerCampaign = (uint32_t)std::atoll(val().c_str());
        else if (k == "--event-rate") a.so.eventRate = std::atof(val().c_str());
        else if (k == "--speedup") a.so.speedup = std::atof(val().c_str());
        else if (k == "--cycle-ms") a.so.cycleMs = std::atoll(val().c_str());
        else if (k == "--batch-ms") a.so.batchMs = std::atoll(val().c_str());
        else if (k == "--ooo-ms") a.so.oooMs = std::atoll(val().c_str());
        else if (k == "--seconds") a.so.seconds = std::atof(val().c_str());
        else if (k == "--skew") a.so.skew = std::atoi(val().c_str());
        else if (k == "--totals") a.stream_csv = val();
        else if (k == "--stream-feed-check") { a.stream = true; a.feed_check = true; }
        else if (k == "--feed-seconds") a.feed_seconds = std::atof(val().c_str());
        else if (k == "--stream-merge-check") { a.stream = true; a.merge_check = true; }
        else if (k == "--merge-flushes") a.merge_flushes = std::atoi(val().c_str());
        else if (k == "--no-numa") a.so.pinNuma = false;
        else if (k == "--no-timing") a.so.timing = false;
        else if (k == "--replay") {
            const std::string m = val();
            if (m != "mapped" && m != "mapped-raw" && m != "copy") { usage(); std::exit(2); }
            a.so.replay = m == "mapped" ? StreamOptions::MAPPED : m == "mapped-raw" ? StreamOptions::MAPPED_RAW
                                                                                    : StreamOptions::COPY;
        }
        else { usage(); std::exit(2); }
    }
    if (a.stream) {   // the generator's ids and events: no config file needed
        a.so.device = a.device;
        a.so.flushMs = a.flush_ms;
        a.so.slotBytes = (uint64_t)a.batch_bytes;
        a.so.windowRing = a.window_ring == 1024 ? 64 : a.window_ring;
        a.so.threads = a.io_threads;
        return a;
    }
    if (a.conf.empty()) {   // ParameterTool.getRequired("confPath")
        std::fprintf(stderr, "No data for required key 'confPath'\n");
        std::exit(2);
    }
    return a;
}

std::string json_str(const std::string& s) {
    std::string o = "\"";
    for (char c : s) {
        if (c == '"' || c == '\\') o += '\\';
        if ((unsigned char)c < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", c); o += b; continue; }
        o += c;
    }
    return o + "\"";
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int run(const Args& a) {
    const Config conf = Config::findAndReadConfigFile(a.conf, true);
    if (a.print_config) {
        std::string o = "{";
        bool first = true;
        for (const auto& kv : conf.scalars()) {
            o += (first ? "" : ", ") + json_str(kv.first) + ": " + json_str(kv.second);
            first = false;
        }
        for (const auto& kv : conf.lists()) {
            o += (first ? "" : ", ") + json_str(kv.first) + ": [";
            for (size_t i = 0; i < kv.second.size(); ++i) o += (i ? ", " : "") + json_str(kv.second[i]);
            o += "]";
            first = false;
        }
        std::printf("%s}\n", o.c_str());
    }
    // getAdCampaignMap(conf.get("ad_to_campaign_path")) (:67)
    const AdCampaignMap map = AdCampaignMap::fromFile(conf.get("ad_to_campaign_path"));
    const std::string events = conf.get("events_path");
    const bool tbl = a.format.empty() ? (events.size() > 4 && events.compare(events.size() - 4, 4, ".tbl") == 0)
                                      : a.format == "tbl";
    if (!a.format.empty() && a.format != "json" && a.format != "tbl") { usage(); return 2; }

    GpuAdCampaignOperator::Options o;
    o.device = a.device;
    o.windowRing = a.window_ring;
    o.batchBytes = (uint64_t)a.batch_bytes;
    o.batchEvents = (uint64_t)a.batch_events;
    o.tbl = tbl;
    o.requireIp = a.require_ip;
    o.gpuSplit = !a.host_split;
    o.h2dSdma = a.h2d_sdma;
    o.mappedIo = a.io == "mapped" || (a.io == "auto" && o.gpuSplit && !o.h2dSdma);
    if (a.io == "mapped" && !o.gpuSplit) {
        std::fprintf(stderr, "--io mapped reads raw lines in place: not with --host-split\n");
        return 2;
    }

    FileBasedDataSource src(events, a.io_threads, a.io_mmap);
    const double t0 = now_s();
    if (a.dry && a.io == "mapped") {   // the mapped source's ranges alone: whole lines, every byte once
        uint64_t nb, bytes = 0, batches = 0, cut = 0;
        const uint8_t* p = nullptr;
        while ((nb = src.nextMapped(o.batchBytes, &p)) > 0) {
            if (p != src.mapping() + bytes) throw std::runtime_error("mapped ranges not back to back");
            const uint8_t last = p[nb - 1];
            if (last != '\n' && last != '\r') ++cut;   // only the file's last line may lack its terminator
            bytes += nb;
            ++batches;
        }
        std::printf("{\"mode\": \"dry-run\", \"io\": \"mapped\", \"bytes\": %llu, \"batches\": %llu, "
                    "\"unterminated\": %llu}\n",
                    (unsigned long long)bytes, (unsigned long long)batches, (unsigned long long)cut);
        return 0;
    }
    if (a.dry) {   // host half only: map + source, no device
        std::vector<uint8_t> buf(o.batchBytes);
        std::vector<uint32_t> off(o.batchEvents);
        uint64_t n, nb, bytes = 0, batches = 0;
        while ((n = src.fill(buf.data(), buf.size(), off.data(), off.size(), &nb)) > 0) {
            bytes += nb;
            ++batches;
        }
        std::printf("{\"mode\": \"dry-run\", \"ads\": %zu, \"campaigns\": %zu, \"events\": %llu, \"bytes\": %llu, "
                    "\"batches\": %llu, \"format\": \"%s\"}\n",
                    map.ads.size(), map.campaigns.size(), (unsigned long long)src.linesRead(),
                    (unsigned long long)bytes, (unsigned long long)batches, tbl ? "tbl" : "json");
        return 0;
    }

    std::unique_ptr<RedisWindowWriter> redis;
    CsvWindowSink csv;
    std::string csv_path;
    if (a.sink.rfind("redis", 0) == 0) {
        std::string host = conf.get("redis.host", "localhost");
        int port = 6379;
        const std::string rest = a.sink.size() > 6 ? a.sink.substr(6) : "";
        if (!rest.empty()) {
            const size_t c = rest.rfind(':');
            host = c == std::string::npos ? rest : rest.substr(0, c);
            if (c != std::string::npos) port = std::atoi(rest.c_str() + c + 1);
        }
        redis.reset(new RedisWindowWriter(host, port));
    } else if (a.sink.rfind("csv:", 0) == 0) {
        csv_path = a.sink.substr(4);
    } else if (a.sink != "none") {
        usage();
        return 2;
    }

    if (!a.replay.empty()) {   // the sink alone: rows from a CSV, one flush
        std::vector<WindowDelta> d;
        const std::vector<std::string> lines = readLines(readFile(a.replay));
        for (size_t i = 1; i < lines.size(); ++i) {
            const std::vector<std::string> f = javaSplit(lines[i], ',');
            if (f.size() != 3) throw std::runtime_error("bad row line " + std::to_string(i + 1));
            d.push_back({f[0], std::stoll(f[1]), std::stoull(f[2])});
        }
        if (redis) redis->writeWindows(d);
        if (!csv_path.empty()) {
            csv.add(d);
            csv.write(csv_path);
        }
        std::printf("{\"mode\": \"replay-rows\", \"rows\": %zu, \"round_trips\": %llu}\n", d.size(),
                    (unsigned long long)(redis ? redis->roundTrips() : 0));
        return 0;
    }

    GpuAdCampaignOperator op(map, o);
    op.open();
    if (o.mappedIo && a.io == "auto" && !src.mapping()) o.mappedIo = false;   // nothing mapped (empty file)
    if (o.mappedIo) {
        try {
            op.registerSource(src);
        } catch (const std::exception& e) {
            if (a.io == "mapped") throw;
            std::fprintf(stderr, "note: the events file's mapping cannot be read in place (%s): slot copies\n",
                         e.what());
            o.mappedIo = false;
        }
    }
    const double t_open = now_s();   // the stream itself: from the first read to close
    uint64_t rows = 0, flushes = 0;
    auto flush = [&]() {
        const std::vector<WindowDelta> d = op.flushWindows();
        rows += d.size();
        ++flushes;
        if (redis) redis->writeWindows(d);
        if (!csv_path.empty()) csv.add(d);
    };
    double last_flush = now_s();
    for (long long rep = 0; rep < a.repeat; ++rep) {
        if (rep) src.rewind();
        while (o.mappedIo ? op.submitMapped(src) > 0 : (o.gpuSplit ? op.fillFromRaw(src) : op.fillFrom(src)) > 0) {
            if (!o.mappedIo) op.submit();
            if (a.flush_ms > 0 && (now_s() - last_flush) * 1000.0 >= (double)a.flush_ms) {
                flush();
                last_flush = now_s();
            }
        }
        op.submit();   // a last partial slot
    }
    op.close();
    const double el_stream = now_s() - t_open;
    flush();
    const double el = now_s() - t0;
    if (!csv_path.empty()) csv.write(csv_path);
    const ysb_stats s = op.stats();
    double copy_ms = 0;
    uint64_t copies = 0, copy_bytes = 0;
    op.copyTime(&copy_ms, &copies, &copy_bytes);
    std::printf("{\"mode\": \"gpu\", \"events\": %llu, \"views\": %llu, \"joined\": %llu, \"join_misses\": %llu, "
                "\"parse_errors\": %llu, \"time_errors\": %llu, \"out_of_ring\": %llu, \"overflow_dropped\": %llu, "
                "\"batches\": %llu, \"rows_written\": %llu, \"flushes\": %llu, \"seconds\": %.3f, "
                "\"events_per_s\": %.1f, \"stream_seconds\": %.3f, \"stream_events_per_s\": %.1f, "
                "\"bytes\": %llu, \"stream_GBs\": %.2f, \"line_split\": \"%s\", \"repeat\": %lld, "
                "\"format\": \"%s\", \"sink\": %s, \"h2d\": \"%s\", \"copy_GBs\": %.2f, \"copy_busy_frac\": %.4f, "
                "\"fill_s\": %.3f, \"slot_wait_s\": %.3f}\n",
                (unsigned long long)s.events, (unsigned long long)s.views, (unsigned long long)s.joined,
                (unsigned long long)s.join_misses, (unsigned long long)s.parse_errors,
                (unsigned long long)s.time_errors, (unsigned long long)s.out_of_ring,
                (unsigned long long)s.overflow_dropped, (unsigned long long)s.batches, (unsigned long long)rows,
                (unsigned long long)flushes, el, el > 0 ? (double)s.events / el : 0.0, el_stream,
                el_stream > 0 ? (double)s.events / el_stream : 0.0, (unsigned long long)src.bytesRead(),
                el_stream > 0 ? (double)src.bytesRead() / el_stream / 1e9 : 0.0, o.gpuSplit ? "gpu" : "host",
                a.repeat, tbl ? "tbl" : "json",
                json_str(a.sink).c_str(), a.h2d_sdma ? "sdma" : o.mappedIo ? "mapped" : "kernel",
                copy_ms > 0 ? (double)copy_bytes / (copy_ms * 1e-3) / 1e9 : 0.0,
                el_stream > 0 ? copy_ms * 1e-3 / el_stream : 0.0, op.fillSeconds(), op.waitSeconds());
    return s.overflow_dropped ? 3 : 0;
}

double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    const double pos = q / 100.0 * (double)(v.size() - 1);
    const size_t lo = (size_t)pos, hi = std::min(v.size() - 1, lo + 1);
    return v[lo] + (v[hi] - v[lo]) * (pos - (double)lo);
}

std::string dist(const std::vector<double>& v, double scale) {
    char b[256];
    std::snprintf(b, sizeof b, "{\"n\": %zu, \"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}", v.size(),
                  pct(v, 50) * scale, pct(v, 99) * scale, v.empty() ? 0.0 : *std::max_element(v.begin(), v.end()) * scale);
    return b;
}

// Streaming mode (BASELINE configs[4]): ysb_stream.hpp.
int run_stream(const Args& a) {
    StreamingJob job(a.so);
    const double t0 = now_s();
    job.prepare();
    const double prep_s = now_s() - t0;
    std::unique_ptr<RedisWindowWriter> redis;
    if (a.sink.rfind("redis", 0) == 0) {
        std::string host = "localhost";
        int port = 6379;
        const std::string rest = a.sink.size() > 6 ? a.sink.substr(6) : "";
        if (!rest.empty()) {
            const size_t c = rest.rfind(':');
            host = c == std::string::npos ? rest : rest.substr(0, c);
            if (c != std::string::npos) port = std::atoi(rest.c_str() + c + 1);
        }
        redis.reset(new RedisWindowWriter(host, port));
    } else if (a.sink != "none" && a.sink.rfind("csv:", 0) != 0) {
        usage();
        return 2;
    }
    CsvWindowSink totals;
    const std::string csv_path = a.sink.rfind("csv:", 0) == 0 ? a.sink.substr(4) : a.stream_csv;
    const StreamReport r = job.run([&](const FlushRows& f, int64_t now) {
        if (redis) redis->writeWindows(f.rows, now);
        totals.add(f.rows);
    });
    if (!csv_path.empty()) totals.write(csv_path);
    const double f = 1.0 / a.so.speedup;   // replay ms -> wall ms
    std::string cyc = "[", part = "[";
    for (size_t i = 0; i < r.cycles.size(); ++i) {
        cyc += (i ? ", " : "") + std::to_string(r.cycles[i]);
        part += (i ? ", " : "") + std::to_string(r.partialLines[i]);
    }
    cyc += "]";
    part += "]";
    std::string per = "[";
    for (size_t i = 0; i < r.shards.size(); ++i) {
        const ShardReport& s = r.shards[i];
        char b[512];
        std::snprintf(b, sizeof b, "%s{\"device\": %d, \"numa_node\": %d, \"feeder_pinned\": %s, \"events\": %llu, "
                      "\"batches\": %llu, \"submit_ms\": %.1f, \"feeder_cpu_s\": %.3f, \"max_behind_ms\": %.2f, "
                      "\"ring_advances\": %llu, \"replay_GB\": %.2f, \"prepare_s\": %.2f, \"register_s\": %.2f}",
                      i ? ", " : "", s.device, s.numaNode, s.pinned ? "true" : "false", (unsigned long long)s.events,
                      (unsigned long long)s.batches, s.submitMs, s.feederCpuS, s.maxBehindMs,
                      (unsigned long long)s.ringAdvances, s.replayGB, s.prepareS, s.registerS);
        per += b;
    }
    per += "]";
    std::printf("{\"mode\": \"stream\", \"replay\": \"%s\", \"shards\": %d, \"events\": %llu, \"batches\": %llu, "
                "\"wall_s\": %.3f, \"submit_events_per_s\": %.1f, \"per_shard\": %s, "
                "\"events_per_s\": %.1f, \"target_events_per_s\": %.1f, \"copy_GBs\": %.2f, \"copy_busy_frac\": %.4f, "
                "\"slot_waits\": %llu, \"slot_wait_ms\": %.2f, \"slot_wait_max_ms\": %.3f, \"max_behind_ms\": %.2f, "
                "\"flushes\": %llu, \"rows_written\": %llu, \"ring_advances\": %llu, "
                "\"window_close_ms\": %s, \"window_close_wall_ms\": %s, \"get_stats_ms\": %s, "
                "\"get_stats_wall_ms_after_window_end\": %s, \"open_at_end\": %llu, \"final_watermark_ms\": %lld, "
                "\"speedup\": %.3f, \"event_rate\": %.1f, \"cycle_ms\": %lld, \"flush_ms\": %lld, \"batch_ms\": %lld, "
                "\"ooo_ms\": %lld, \"skew\": %d, \"seed\": %llu, \"campaigns\": %u, \"ads_per_campaign\": %u, "
                "\"t0_ms\": %lld, \"lines_per_cycle\": %llu, \"cycles\": %s, \"partial_lines\": %s, "
                "\"overflow_dropped\": %llu, \"parse_errors\": %llu, \"join_misses\": %llu, \"prepare_s\": %.2f, "
                "\"sink\": %s}\n",
                a.so.replay == StreamOptions::MAPPED ? "mapped" : a.so.replay == StreamOptions::MAPPED_RAW ? "mapped-raw" : "copy",
                a.so.shards, (unsigned long long)r.events, (unsigned long long)r.batches,
                r.wallSeconds, r.submitEventsPerSecond, per.c_str(), r.eventsPerSecond,
                r.targetEventsPerSecond, r.copyGBs, r.copyBusyFrac, (unsigned long long)r.slotWaits, r.slotWaitMs,
                r.slotWaitMaxMs, r.maxBehindMs, (unsigned long long)r.flushes, (unsigned long long)r.rowsWritten,
                (unsigned long long)r.ringAdvances, dist(r.closeReplayMs, 1.0).c_str(), dist(r.closeReplayMs, f).c_str(),
                dist(r.cwReplayMs, 1.0).c_str(),
                dist([&] { std::vector<double> v; for (double x : r.cwReplayMs) v.push_back(x - 10000.0); return v; }(), f).c_str(),
                (unsigned long long)r.openAtEnd, (long long)r.finalWatermarkMs, a.so.speedup, a.so.eventRate, (long long)a.so.cycleMs,
                (long long)a.so.flushMs, (long long)a.so.batchMs, (long long)a.so.oooMs, a.so.skew,
                (unsigned long long)a.so.seed, a.so.campaigns, a.so.adsPerCampaign, (long long)a.so.t0Ms,
                (unsigned long long)r.linesPerCycle, cyc.c_str(), part.c_str(), (unsigned long long)r.overflowDropped,
                (unsigned long long)r.parseErrors, (unsigned long long)r.joinMisses, prep_s, json_str(a.sink).c_str());
    return r.overflowDropped ? 3 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    const Args a = parse(argc, argv);
    if (ysb_abi_version() != YSB_ABI_VERSION || ysb_exchange_info_size() != sizeof(ysb_exchange_info)) {
        std::fprintf(stderr, "ysb_topology: libysb_hip.so has ABI %d, this runner was built for ABI %d: rebuild\n",
                     ysb_abi_version(), YSB_ABI_VERSION);
        return 2;
    }
    try {
        if (a.self_check) {
            std::printf("%s\n", StreamingJob::replaySelfCheck(a.so, {0, 1, 2, 7, 1000}).c_str());
            return 0;
        }
        if (a.feed_check) {
            std::printf("%s\n", StreamingJob::feedCheck(a.so, a.feed_seconds).c_str());
            return 0;
        }
        if (a.merge_check) {
            const std::string r = StreamingJob::mergeCheck(a.so.shards, a.merge_flushes, a.so.seed);
            std::printf("%s\n", r.c_str());
            return r.find("\"ok\": true") != std::string::npos ? 0 : 1;
        }
        if (a.stream) return run_stream(a);
        return run(a);
    } catch (const std::exception& e) {   // the job fails, as the reference's uncaught exceptions do
        std::fprintf(stderr, "ysb_topology: %s\n", e.what());
        return 1;
    }
}
