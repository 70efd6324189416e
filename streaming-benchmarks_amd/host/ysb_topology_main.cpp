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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

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
};

void usage() {
    std::fprintf(stderr,
                 "usage: ysb_topology --confPath PATH [--device N] [--sink none|csv:FILE|redis[:HOST[:PORT]]]\n"
                 "       [--format json|tbl] [--flush-ms MS] [--batch-mb MB | --batch-bytes B] [--batch-events N]\n"
                 "       [--window-ring W] [--require-ip] [--dry-run] [--print-config] [--replay-rows CSV]\n"
                 "       [--host-split] [--repeat K] [--io-threads T] [--io mmap|pread]\n");
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
        else if (k == "--io") a.io_mmap = val() != "pread";
        else { usage(); std::exit(2); }
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

    FileBasedDataSource src(events, a.io_threads, a.io_mmap);
    const double t0 = now_s();
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
        while ((o.gpuSplit ? op.fillFromRaw(src) : op.fillFrom(src)) > 0) {
            op.submit();
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
    std::printf("{\"mode\": \"gpu\", \"events\": %llu, \"views\": %llu, \"joined\": %llu, \"join_misses\": %llu, "
                "\"parse_errors\": %llu, \"time_errors\": %llu, \"out_of_ring\": %llu, \"overflow_dropped\": %llu, "
                "\"batches\": %llu, \"rows_written\": %llu, \"flushes\": %llu, \"seconds\": %.3f, "
                "\"events_per_s\": %.1f, \"stream_seconds\": %.3f, \"stream_events_per_s\": %.1f, "
                "\"bytes\": %llu, \"stream_GBs\": %.2f, \"line_split\": \"%s\", \"repeat\": %lld, "
                "\"format\": \"%s\", \"sink\": %s}\n",
                (unsigned long long)s.events, (unsigned long long)s.views, (unsigned long long)s.joined,
                (unsigned long long)s.join_misses, (unsigned long long)s.parse_errors,
                (unsigned long long)s.time_errors, (unsigned long long)s.out_of_ring,
                (unsigned long long)s.overflow_dropped, (unsigned long long)s.batches, (unsigned long long)rows,
                (unsigned long long)flushes, el, el > 0 ? (double)s.events / el : 0.0, el_stream,
                el_stream > 0 ? (double)s.events / el_stream : 0.0, (unsigned long long)src.bytesRead(),
                el_stream > 0 ? (double)src.bytesRead() / el_stream / 1e9 : 0.0, o.gpuSplit ? "gpu" : "host",
                a.repeat, tbl ? "tbl" : "json",
                json_str(a.sink).c_str());
    return s.overflow_dropped ? 3 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    const Args a = parse(argc, argv);
    try {
        return run(a);
    } catch (const std::exception& e) {   // the job fails, as the reference's uncaught exceptions do
        std::fprintf(stderr, "ysb_topology: %s\n", e.what());
        return 1;
    }
}
