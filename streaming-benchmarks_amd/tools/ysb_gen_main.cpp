// ysb_gen -- file-dump mode of the data/ generator (data/src/setup/core.clj:239-248
// -s, and write-to-kafka :61-98 which the reference leaves unwired at :246).
//
//   ysb_gen -d DIR [-n EVENTS] [--seed S] [--campaigns C] [--ads-per-campaign A]
//           [--rate EVENTS_PER_SEC] [--t0 MS] [--with-skew] [--users K]
//           [--shards K] [--tbl]
//
// Writes campaign-ids.txt, ad-ids.txt, ad-to-campaign-ids.txt (JSON map lines),
// ad-to-campaign.csv (the fork's CSV map) and kafka-json.txt into DIR; with --shards K
// kafka-json.<r>.txt per ad_id-hash shard instead; with --tbl also events.tbl, the
// fork's pipe-delimited rows (conf/benchmarkConf.yaml:6).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ysb_hip.h"

int main(int argc, char** argv) {
    ysb_gen_params p;
    ysb_gen_default(&p);
    p.events_per_sec = 100;   // catch-up mode: one event per 10 ms (core.clj:95)
    unsigned long long n = 10000000ULL;   // kafka-event-count (core.clj:17)
    const char* dir = nullptr;
    unsigned shards = 0;
    bool tbl = false;
    for (int i = 1; i < argc; ++i) {
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", argv[i]); std::exit(2); }
            return argv[++i];
        };
        if (!std::strcmp(argv[i], "-d")) dir = val();
        else if (!std::strcmp(argv[i], "-n")) n = std::strtoull(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--seed")) p.seed = std::strtoull(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--campaigns")) p.n_campaigns = (unsigned)std::strtoul(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--ads-per-campaign")) p.ads_per_campaign = (unsigned)std::strtoul(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--rate")) p.events_per_sec = std::strtoull(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--t0")) p.t0_ms = std::strtoll(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--with-skew")) p.with_skew = 1;
        else if (!std::strcmp(argv[i], "--users")) p.n_users = (unsigned)std::strtoul(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--shards")) shards = (unsigned)std::strtoul(val(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--tbl")) tbl = true;
        else { std::fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    if (!dir) { std::fprintf(stderr, "usage: ysb_gen -d DIR [-n EVENTS] [options]\n"); return 2; }
    int rc = shards > 1 ? ysb_gen_dump_shards(&p, n, dir, shards) : ysb_gen_dump(&p, n, dir);
    if (rc) { std::fprintf(stderr, "ysb_gen: %s\n", ysb_last_error(nullptr)); return 1; }
    if (tbl) {   // events.tbl: the same events as .tbl rows, in chunks
        FILE* f = std::fopen((std::string(dir) + "/events.tbl").c_str(), "wb");
        if (!f) { std::fprintf(stderr, "ysb_gen: cannot write events.tbl\n"); return 1; }
        const unsigned long long chunk = 1 << 16;
        const unsigned long long cap = chunk * ysb_gen_max_line_bytes(&p);
        std::vector<unsigned char> js(cap), tb(cap);
        std::vector<unsigned> off(chunk), toff(chunk);
        for (unsigned long long first = 0; first < n; first += chunk) {
            const unsigned long long m = n - first < chunk ? n - first : chunk;
            uint64_t nb = 0, tnb = 0;
            if (ysb_gen_events_host(&p, first, m, js.data(), cap, off.data(), &nb) ||
                ysb_json_to_tbl(js.data(), nb, off.data(), m, tb.data(), cap, toff.data(), &tnb)) {
                std::fprintf(stderr, "ysb_gen: .tbl conversion failed\n");
                std::fclose(f);
                return 1;
            }
            std::fwrite(tb.data(), 1, tnb, f);
        }
        std::fclose(f);
    }
    return 0;
}
