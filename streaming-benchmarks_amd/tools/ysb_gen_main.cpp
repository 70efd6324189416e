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
    if (tbl) {   // events.tbl: the same events as .tbl rows (generator format YSB_GEN_TBL)
        ysb_gen_params q = p;
        q.format = YSB_GEN_TBL;
        rc = ysb_gen_dump(&q, n, dir);
        if (rc) { std::fprintf(stderr, "ysb_gen: %s\n", ysb_last_error(nullptr)); return 1; }
    }
    return 0;
}
