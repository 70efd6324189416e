// ysb_stream.cpp -- implementation of ysb_stream.hpp (the runner's streaming mode).
#include "ysb_stream.hpp"

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <stdexcept>
#include <thread>

#include "worker_pool.hpp"

namespace ysb {
namespace topology {

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double thread_cpu_s() {
    timespec ts{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

constexpr int64_t BUCKET_MS = 10000;       // CampaignProcessorCommon.java:28 (time_divisor)
constexpr uint64_t GEN_PIECE = 2u << 20;   // events per generator call
constexpr uint64_t BATCH_ALIGN = 64;       // each batch's first byte (ysb_submit_raw_mapped: >= 16)
constexpr int64_t LEAD_SLACK = 16;         // buckets below t0's a line may fall in (skew, late events)
const char ET_KEY[] = "\"event_time\"";

void check_ctx(int rc, ysb_ctx* c, const char* what) {
    if (rc != YSB_OK) throw std::runtime_error(std::string(what) + ": " + ysb_last_error(c));
}

unsigned default_threads(const StreamOptions& o) {
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    return o.threads ? o.threads : std::max(1u, hw / (unsigned)std::max(1, o.shards));
}

// Pins the calling thread to `cpus` (threads it creates inherit the mask); false if it could not.
bool pin_to(const std::vector<int>& cpus) {
    if (cpus.empty()) return false;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    return pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0;
}

}  // namespace

int gpuNumaNode(int device) { return ysb_device_numa_node(device); }

std::vector<int> nodeCpus(int node) {
    std::vector<int> out;
    if (node < 0) return out;
    FILE* f = std::fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return out;
    char buf[4096] = {0};
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
    for (char* p = buf; *p;) {   // "0-23,96-119"
        char* e = nullptr;
        const long a = std::strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        if (*e == '-') {
            p = e + 1;
            b = std::strtol(p, &e, 10);
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET((int)c, &allowed)) out.push_back((int)c);
        p = *e == ',' ? e + 1 : e;
        if (*p == '\n') break;
    }
    return out;
}

// One cycle of the replay: the generator's lines over cycleMs of event time, laid out batch by
// batch in one anonymous mapping (each batch 64-byte aligned, the lines of a batch back to
// back), each line's event_time digits located, and the batches the cycle is released in.
struct ReplayCycle {
    uint8_t* bytes = nullptr;
    uint64_t reserved = 0;           // bytes mapped (virtual)
    uint64_t used = 0;               // bytes written, slack included (what is registered)
    std::vector<uint64_t> start;     // n line starts in `bytes`
    // per line: offset of its 13 time digits within the line | (leading nine digits - upperMin) << 16
    std::vector<uint32_t> timeAt;
    int64_t upperMin = 0;
    uint32_t nUpper = 0;
    struct Batch {
        uint64_t a, b;               // lines [a, b)
        uint64_t off, nbytes;        // its bytes: [off, off + nbytes) of `bytes`
        int64_t releaseMs;           // nominal emission time of line b - 1 (cycle 0)
        int64_t maxTimeMs;           // the largest event_time in it (cycle 0)
    };
    std::vector<Batch> batches;
    uint64_t lines() const { return start.size(); }
    ReplayCycle() = default;
    ReplayCycle(const ReplayCycle&) = delete;
    ReplayCycle& operator=(const ReplayCycle&) = delete;
    ~ReplayCycle() {
        if (bytes) munmap(bytes, reserved);
    }
};

struct StreamingJob::Shard {
    int index = 0, device = 0, node = -1;
    std::vector<int> cpus;
    bool pinned = false;
    ysb_ctx* ctx = nullptr;
    uint8_t* slot[2] = {nullptr, nullptr};
    ysb_gen_params gen{};
    std::vector<uint32_t> subset;
    ReplayCycle cyc;
    bool registered = false;
    uint32_t* d_lineOff = nullptr;   // (mapped) every line's offset within its batch, in HBM
    double prepareS = 0, registerS = 0;
    // feeder state (the feeder thread's own)
    uint64_t cycle = 0, next = 0;    // the next batch: cyc.batches[next] of cycle `cycle`
    int cur = 0;
    int64_t maxTime = INT64_MIN;
    uint64_t events = 0, batches = 0;
    std::deque<std::pair<int64_t, int64_t>> flushes;   // outstanding: (flush index, watermark at its begin)
    int64_t flushBegun = 0;
    int64_t ringLo = 0;
    uint64_t ringAdvances = 0, slowSubmits = 0;
    double submitMs = 0, slowMs = 0, slowMaxMs = 0, maxBehindMs = 0, cpuS = 0;
    double firstSubmit = 0, lastSubmit = 0, doneAt = 0;
    std::atomic<bool> synced{false};
    std::thread th;
    std::string error;
    ~Shard() {
        if (th.joinable()) th.join();
        if (ctx && d_lineOff) ysb_device_free(ctx, d_lineOff);
        if (ctx) ysb_close(ctx);   // (unregisters the cycle before it is unmapped)
    }
};

StreamingJob::StreamingJob(const StreamOptions& o) : o_(o) {
    if (o_.cycleMs <= 0 || o_.cycleMs % BUCKET_MS) throw std::runtime_error("the replay cycle must be a multiple of 10 000 ms");
    if (o_.t0Ms % BUCKET_MS) throw std::runtime_error("t0 must be a multiple of 10 000 ms");
    if (o_.shards < 1 || o_.eventRate < 1 || o_.speedup <= 0) throw std::runtime_error("bad stream options");
    if (o_.skew < 0 || o_.skew > 2) throw std::runtime_error("skew must be 0 (off), 1 (skew + late events) or 2 (skew only)");
}

StreamingJob::~StreamingJob() {
    for (Shard* s : shards_) delete s;
}

// The shard's replay cycle: generated on its GPU (ysb_gen_events_device, the data/ generator)
// in pieces -- or, ctx NULL (the CPU checks), by the host generator -- and laid out batch by
// batch: batches close at batchMs of nominal emission time or a slot's bytes, whichever comes
// first; each starts 64-byte aligned.  The pages are written by the calling thread (first touch:
// on its NUMA node).
static void build_cycle(ysb_ctx* ctx, const ysb_gen_params& g, const StreamOptions& o, ReplayCycle& c,
                        WorkerPool& pool) {
    const uint64_t n = (uint64_t)(o.eventRate * (double)o.cycleMs / 1000.0);
    if (n == 0) throw std::runtime_error("empty replay cycle");
    const uint64_t maxLine = ysb_gen_max_line_bytes(&g);
    c.reserved = n * (maxLine + BATCH_ALIGN) + (1u << 20);
    void* m = mmap(nullptr, c.reserved, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) throw std::runtime_error("replay cycle: mmap failed");
    c.bytes = static_cast<uint8_t*>(m);
    madvise(c.bytes, c.reserved, MADV_HUGEPAGE);
    c.start.assign(n, 0);
    c.timeAt.assign(n, 0);
    const int64_t base = g.t0_ms / BUCKET_MS - LEAD_SLACK;
    c.upperMin = base;
    auto nominal = [&](uint64_t i) { return g.t0_ms + (int64_t)((i * 1000ull) / g.events_per_sec); };
    const uint64_t piece = std::min<uint64_t>(n, GEN_PIECE);
    void *d_b = nullptr, *d_o = nullptr;
    if (ctx) {
        check_ctx(ysb_device_alloc(ctx, piece * maxLine + 64, &d_b), ctx, "ysb_device_alloc");
        check_ctx(ysb_device_alloc(ctx, piece * 4 + 64, &d_o), ctx, "ysb_device_alloc");
    }
    std::vector<uint8_t> hbuf(piece * maxLine + 64);
    std::vector<uint32_t> off(piece + 1);
    std::vector<std::string> err(pool.size());
    std::vector<uint32_t> kmax(pool.size(), 0);
    uint64_t pos = 0;                 // write position in c.bytes
    bool open = false;
    ReplayCycle::Batch cur{};
    int64_t lim = 0;
    auto close_batch = [&](uint64_t b) {
        cur.b = b;
        cur.nbytes = pos - cur.off;
        cur.releaseMs = nominal(b - 1);
        c.batches.push_back(cur);
        open = false;
    };
    for (uint64_t first = 0; first < n; first += piece) {
        const uint64_t mcount = std::min(piece, n - first);
        uint64_t nb = 0;
        if (ctx) {
            check_ctx(ysb_gen_events_device(ctx, &g, first, mcount, (uint8_t*)d_b, piece * maxLine, (uint32_t*)d_o, &nb),
                      ctx, "ysb_gen_events_device");
            check_ctx(ysb_memcpy_d2h(ctx, hbuf.data(), d_b, nb), ctx, "ysb_memcpy_d2h");
            check_ctx(ysb_memcpy_d2h(ctx, off.data(), d_o, mcount * 4), ctx, "ysb_memcpy_d2h");
        } else if (ysb_gen_events_host_mt(&g, first, mcount, hbuf.data(), hbuf.size(), off.data(), &nb, pool.size()) != YSB_OK) {
            throw std::runtime_error(std::string("ysb_gen_events_host_mt: ") + ysb_last_error(nullptr));
        }
        off[mcount] = (uint32_t)nb;
        // the layout: sequential (batch boundaries depend on the lines before), positions only
        for (uint64_t j = 0; j < mcount; ++j) {
            const uint64_t i = first + j, len = off[j + 1] - off[j];
            if (open && (nominal(i) >= lim || pos + len - cur.off > o.slotBytes)) close_batch(i);
            if (!open) {
                pos = (pos + BATCH_ALIGN - 1) / BATCH_ALIGN * BATCH_ALIGN;
                cur = ReplayCycle::Batch{i, i, pos, 0, 0, INT64_MIN};
                lim = nominal(i) + o.batchMs;
                open = true;
                if (len > o.slotBytes) throw std::runtime_error("a replay line is longer than the slot");
            }
            c.start[i] = pos;
            pos += len;
        }
        // the bytes and the time index: in parallel
        pool.run(pool.size(), [&](unsigned t) {
            const uint64_t ja = mcount * t / pool.size(), jb = mcount * (t + 1) / pool.size();
            uint32_t km = 0;
            for (uint64_t j = ja; j < jb && err[t].empty(); ++j) {
                const uint64_t i = first + j, len = off[j + 1] - off[j];
                const uint8_t* l = hbuf.data() + off[j];
                std::memcpy(c.bytes + c.start[i], l, len);
                const void* k = memmem(l, len, ET_KEY, sizeof ET_KEY - 1);
                uint64_t p = k ? (uint64_t)((const uint8_t*)k - l) + sizeof ET_KEY - 1 : len;
                while (p < len && (l[p] == ' ' || l[p] == ':')) ++p;
                if (p < len && l[p] == '"') ++p;
                if (p + 13 >= len || l[p + 13] != '"' || p > 0xFFFF) { err[t] = "line " + std::to_string(i) + ": no 13-digit event_time"; break; }
                int64_t v = 0;
                for (int d = 0; d < 13; ++d) {
                    if (l[p + d] < '0' || l[p + d] > '9') { err[t] = "line " + std::to_string(i) + ": event_time"; break; }
                    v = v * 10 + (l[p + d] - '0');
                }
                const int64_t kk = v / BUCKET_MS - base;
                if (kk < 0 || kk > 0xFFFF) { err[t] = "line " + std::to_string(i) + ": event_time out of the cycle's range"; break; }
                c.timeAt[i] = (uint32_t)p | ((uint32_t)kk << 16);
                km = std::max(km, (uint32_t)kk);
            }
            kmax[t] = std::max(kmax[t], km);
        });
        for (const auto& e : err)
            if (!e.empty()) throw std::runtime_error("replay cycle: " + e);
    }
    if (open) close_batch(n);
    c.used = pos + BATCH_ALIGN;       // slack: a batch's copy reads up to 15 bytes past its end
    c.nUpper = 1 + *std::max_element(kmax.begin(), kmax.end());
    // each batch's largest event_time (cycle 0): from the index, in parallel over batches
    pool.run(pool.size(), [&](unsigned t) {
        for (size_t k = t; k < c.batches.size(); k += pool.size()) {
            ReplayCycle::Batch& b = c.batches[k];
            int64_t mx = INT64_MIN;
            for (uint64_t i = b.a; i < b.b; ++i) {
                const uint8_t* d = c.bytes + c.start[i] + (c.timeAt[i] & 0xFFFFu);
                int64_t v = 0;
                for (int q = 0; q < 13; ++q) v = v * 10 + (d[q] - '0');
                mx = std::max(mx, v);
            }
            b.maxTimeMs = mx;
        }
    });
    if (ctx) {
        ysb_device_free(ctx, d_b);
        ysb_device_free(ctx, d_o);
    }
}

// The host restatement of the device rebase (ysb_split.hip rebase_kernel): batch b of cycle
// `cycle` copied into dst with every line's nine leading event_time digits moved by
// cycle * cycleMs / 10 000 buckets (the four trailing digits do not change).  Round 5's fill and
// the CPU checks.
static uint64_t fill_batch(const ReplayCycle& c, const ReplayCycle::Batch& b, uint64_t cycle, int64_t cycleMs,
                           uint8_t* dst, WorkerPool& pool, unsigned T) {
    const int64_t shift = (int64_t)cycle * (cycleMs / BUCKET_MS);
    std::vector<char> table(9ull * c.nUpper);
    for (uint32_t k = 0; k < c.nUpper; ++k) {
        int64_t v = c.upperMin + k + shift;
        for (int d = 8; d >= 0; --d) {
            table[9ull * k + d] = (char)('0' + v % 10);
            v /= 10;
        }
    }
    const uint64_t lines = b.b - b.a;
    const unsigned tn = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(std::min(T, pool.size()), b.nbytes >> 22));
    pool.run(tn, [&](unsigned t) {
        const uint64_t la = b.a + lines * t / tn, lb = b.a + lines * (t + 1) / tn;
        const uint64_t pa = c.start[la], pb = lb < b.b ? c.start[lb] : b.off + b.nbytes;
        std::memcpy(dst + (pa - b.off), c.bytes + pa, pb - pa);
        if (shift)
            for (uint64_t i = la; i < lb; ++i)
                std::memcpy(dst + (c.start[i] - b.off) + (c.timeAt[i] & 0xFFFFu), &table[9ull * (c.timeAt[i] >> 16)], 9);
    });
    return b.nbytes;
}

static ysb_gen_params shard_gen(const StreamOptions& o, uint32_t stream) {
    ysb_gen_params g;
    ysb_gen_default(&g);
    g.seed = o.seed;
    g.n_campaigns = o.campaigns;
    g.ads_per_campaign = o.adsPerCampaign;
    g.t0_ms = o.t0Ms;
    g.events_per_sec = (uint64_t)o.eventRate;
    g.with_skew = (uint32_t)o.skew;
    g.event_stream = stream;
    return g;
}

std::string StreamingJob::replaySelfCheck(const StreamOptions& o, const std::vector<uint64_t>& cycles) {
    const ysb_gen_params g = shard_gen(o, 1);
    const unsigned T = o.threads ? o.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    WorkerPool pool(T);
    ReplayCycle c;
    build_cycle(nullptr, g, o, c, pool);
    std::vector<uint8_t> buf(o.slotBytes + 64), ref(o.slotBytes + 64);
    std::vector<uint32_t> off(c.lines() + 1);
    uint64_t lines = 0, bad = 0, batches = 0, misaligned = 0;
    for (uint64_t cy : cycles) {
        ysb_gen_params gc = g;
        gc.t0_ms = o.t0Ms + (int64_t)cy * o.cycleMs;   // the generator's own lines of that cycle
        for (const auto& b : c.batches) {
            const uint64_t nb = fill_batch(c, b, cy, o.cycleMs, buf.data(), pool, T);
            uint64_t rb = 0;
            if (ysb_gen_events_host(&gc, b.a, b.b - b.a, ref.data(), ref.size(), off.data(), &rb) != YSB_OK)
                throw std::runtime_error("ysb_gen_events_host failed");
            if (rb != nb || std::memcmp(buf.data(), ref.data(), nb) != 0) ++bad;
            misaligned += (b.off % BATCH_ALIGN) != 0;
            lines += b.b - b.a;
            ++batches;
        }
    }
    char o2[320];
    std::snprintf(o2, sizeof o2, "{\"mode\": \"stream-self-check\", \"lines_per_cycle\": %llu, \"batches\": %llu, "
                  "\"lines\": %llu, \"mismatched_batches\": %llu, \"misaligned_batches\": %llu, \"upper_values\": %u}",
                  (unsigned long long)c.lines(), (unsigned long long)batches, (unsigned long long)lines,
                  (unsigned long long)bad, (unsigned long long)misaligned, c.nUpper);
    return o2;
}

std::string StreamingJob::feedCheck(const StreamOptions& o, double seconds) {
    // every shard: its own cycle (its own event stream), built and fed on a thread of its own
    const int S = o.shards;
    std::vector<std::unique_ptr<ReplayCycle>> cyc(S);
    std::vector<std::thread> th;
    std::vector<std::string> err(S);
    for (int s = 0; s < S; ++s)
        th.emplace_back([&, s] {
            try {
                WorkerPool pool(default_threads(o));
                cyc[s].reset(new ReplayCycle());
                build_cycle(nullptr, shard_gen(o, 1 + (uint32_t)s), o, *cyc[s], pool);
            } catch (const std::exception& e) {
                err[s] = e.what();
            }
        });
    for (auto& t : th) t.join();
    th.clear();
    for (const auto& e : err)
        if (!e.empty()) throw std::runtime_error(e);
    // every feeder fills its own slot buffer as fast as it can (one thread each)
    std::vector<uint64_t> ev(S, 0);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<double> el(S, 0);
    for (int s = 0; s < S; ++s)
        th.emplace_back([&, s] {
            const ReplayCycle& c = *cyc[s];
            std::vector<uint8_t> slot(o.slotBytes + 64);
            WorkerPool pool(1);
            ++ready;
            while (!go.load()) std::this_thread::yield();
            const double t0 = now_s();
            uint64_t cycle = 0, next = 0, events = 0;
            while (now_s() - t0 < seconds) {
                const ReplayCycle::Batch& b = c.batches[next];
                fill_batch(c, b, cycle, o.cycleMs, slot.data(), pool, 1);
                events += b.b - b.a;
                if (++next == c.batches.size()) {
                    next = 0;
                    ++cycle;
                }
            }
            el[s] = now_s() - t0;
            ev[s] = events;
        });
    while (ready.load() < S) std::this_thread::yield();
    go = true;
    for (auto& t : th) t.join();
    uint64_t total = 0;
    double mx = 0;
    for (int s = 0; s < S; ++s) {
        total += ev[s];
        mx = std::max(mx, el[s]);
    }
    const double rate = mx > 0 ? (double)total / mx : 0;
    const double lineBytes = (double)(cyc[0]->used) / (double)cyc[0]->lines();
    char out[512];
    std::snprintf(out, sizeof out, "{\"mode\": \"stream-feed-check\", \"shards\": %d, \"seconds\": %.2f, "
                  "\"lines_per_cycle\": %llu, \"batches_per_cycle\": %zu, \"copy_events_per_s\": %.1f, "
                  "\"copy_GBs\": %.2f, \"hardware_threads\": %u}",
                  S, seconds, (unsigned long long)cyc[0]->lines(), cyc[0]->batches.size(), rate,
                  rate * lineBytes / 1e9, std::thread::hardware_concurrency());
    return out;
}

void StreamingJob::prepare() {
    ysb_gen_params g = shard_gen(o_, 0);
    std::vector<char> cid(36ull * o_.campaigns), aid(36ull * o_.campaigns * o_.adsPerCampaign);
    if (ysb_gen_ids(&g, cid.data(), aid.data()) != YSB_OK) throw std::runtime_error("ysb_gen_ids failed");
    const uint64_t A = (uint64_t)o_.campaigns * o_.adsPerCampaign;
    for (uint32_t c = 0; c < o_.campaigns; ++c) campaigns_.emplace_back(&cid[36ull * c], 36);
    for (uint64_t a = 0; a < A; ++a) ads_.emplace_back(&aid[36 * a], 36);
    const int ndev = std::max(1, ysb_device_count());
    std::vector<const char*> keys(A);
    std::vector<uint32_t> camp(A);
    for (uint64_t a = 0; a < A; ++a) {
        keys[a] = ads_[a].data();
        camp[a] = (uint32_t)(a / o_.adsPerCampaign);
    }
    for (int s = 0; s < o_.shards; ++s) {
        Shard* sh = new Shard();
        shards_.push_back(sh);
        sh->index = s;
        sh->device = (o_.device + s) % ndev;
        sh->node = gpuNumaNode(sh->device);
        if (o_.pinNuma) sh->cpus = nodeCpus(sh->node);
    }
    // every shard prepared on a thread of its own, on its GPU's NUMA node: the context, the
    // cycle (generated on its GPU, its pages first touched there), registered with the context
    std::vector<std::thread> th;
    for (Shard* sh : shards_)
        th.emplace_back([&, sh] {
            try {
                const double t0 = now_s();
                sh->pinned = pin_to(sh->cpus);
                WorkerPool pool(default_threads(o_));
                ysb_config cfg;
                ysb_config_default(&cfg);
                cfg.n_campaigns = o_.campaigns;
                cfg.window_ring = o_.windowRing;
                cfg.max_batch_bytes = o_.slotBytes;
                cfg.max_batch_events = o_.slotBytes / 64;
                cfg.ring_base_bucket = o_.t0Ms / BUCKET_MS - 8;
                cfg.flags = o_.timing ? YSB_F_TIMING : 0u;
                if (ysb_open(&sh->ctx, sh->device, &cfg) != YSB_OK)
                    throw std::runtime_error(std::string("ysb_open: ") + ysb_last_error(nullptr));
                sh->ringLo = cfg.ring_base_bucket;
                check_ctx(ysb_load_ad_map(sh->ctx, keys.data(), nullptr, camp.data(), A), sh->ctx, "ysb_load_ad_map");
                for (int k = 0; k < 2; ++k)
                    check_ctx(ysb_slot_buffers(sh->ctx, k, &sh->slot[k], nullptr), sh->ctx, "ysb_slot_buffers");
                // the shard's own event stream over its ad_id shard (ysb_ad_shard), as bench.py's ranks
                sh->gen = shard_gen(o_, 1 + (uint32_t)sh->index);
                if (o_.shards > 1) {
                    for (uint64_t a = 0; a < A; ++a)
                        if (ysb_ad_shard(ads_[a].data(), 36, (uint32_t)o_.shards) == (uint32_t)sh->index)
                            sh->subset.push_back((uint32_t)a);
                    sh->gen.ad_subset = sh->subset.data();
                    sh->gen.n_ad_subset = (uint32_t)sh->subset.size();
                }
                build_cycle(sh->ctx, sh->gen, o_, sh->cyc, pool);
                const double t1 = now_s();
                if (o_.replay != StreamOptions::COPY) {
                    check_ctx(ysb_host_register(sh->ctx, sh->cyc.bytes, (sh->cyc.used + 4095) / 4096 * 4096), sh->ctx,
                              "ysb_host_register");
                    sh->registered = true;
                    check_ctx(ysb_rebase_table(sh->ctx, sh->cyc.timeAt.data(), sh->cyc.lines(), sh->cyc.upperMin),
                              sh->ctx, "ysb_rebase_table");
                }
                if (o_.replay == StreamOptions::MAPPED) {   // the line offsets, once for every cycle
                    std::vector<uint32_t> lo(sh->cyc.lines());
                    for (const auto& b : sh->cyc.batches)
                        for (uint64_t i = b.a; i < b.b; ++i) lo[i] = (uint32_t)(sh->cyc.start[i] - b.off);
                    void* d = nullptr;
                    check_ctx(ysb_device_alloc(sh->ctx, lo.size() * 4 + 64, &d), sh->ctx, "ysb_device_alloc");
                    sh->d_lineOff = static_cast<uint32_t*>(d);
                    check_ctx(ysb_memcpy_h2d(sh->ctx, d, lo.data(), lo.size() * 4), sh->ctx, "ysb_memcpy_h2d");
                }
                sh->registerS = now_s() - t1;
                sh->prepareS = now_s() - t0;
            } catch (const std::exception& e) {
                sh->error = e.what();
            }
        });
    for (auto& t : th) t.join();
    for (Shard* sh : shards_)
        if (!sh->error.empty()) throw std::runtime_error("shard " + std::to_string(sh->index) + ": " + sh->error);
}

namespace {

// The sink side: merged flushes, written in order by one thread (the flusher's writes), with
// the window bookkeeping of the latency figures.
class SinkThread {
public:
    SinkThread(const FlushSink& sink, std::function<int64_t()> clock) : sink_(sink), clock_(std::move(clock)) {
        th_ = std::thread([this] { loop(); });
    }
    ~SinkThread() {
        try {
            finish();
        } catch (...) {   // (an error already reported by the explicit finish)
        }
    }
    void push(FlushRows&& f) {
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }
    void finish() {
        {
            std::lock_guard<std::mutex> g(m_);
            if (done_) return;
            done_ = true;
        }
        cv_.notify_one();
        th_.join();
        if (!error_.empty()) throw std::runtime_error("sink: " + error_);
    }
    std::vector<double> closeMs, cwMs;
    uint64_t rows = 0, flushes = 0;
    std::set<int64_t> seen, closed;

private:
    FlushSink sink_;
    std::function<int64_t()> clock_;
    std::thread th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<FlushRows> q_;
    bool done_ = false;
    std::string error_;
    std::map<std::pair<std::string, int64_t>, int64_t> lastWrite_;   // (campaign, window_ms) -> time_updated
    std::map<int64_t, std::set<std::string>> windowCampaigns_;
    void loop() {
        for (;;) {
            FlushRows f;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [this] { return done_ || !q_.empty(); });
                if (q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            try {
                const int64_t now = clock_();
                if (!f.rows.empty()) sink_(f, now);
                rows += f.rows.size();
                ++flushes;
                for (const WindowDelta& d : f.rows) {
                    lastWrite_[{d.campaign, d.windowMs}] = now;
                    windowCampaigns_[d.windowMs].insert(d.campaign);
                    seen.insert(d.windowMs);
                }
                // windows whose end the watermark has passed: closed by this flush
                for (int64_t w : seen) {
                    if (closed.count(w) || w + BUCKET_MS > f.watermarkMs) continue;
                    closed.insert(w);
                    closeMs.push_back((double)(now - (w + BUCKET_MS)));
                    for (const std::string& c : windowCampaigns_[w]) cwMs.push_back((double)(lastWrite_[{c, w}] - w));
                }
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> g(m_);
                error_ = e.what();
                q_.clear();
                return;
            }
        }
    }
};

// The shards' flushes merged by index: a flush goes to the sink once every shard delivered it,
// in index order, its watermark the minimum of the shards' (each taken at that shard's begin).
class FlushMerger {
public:
    FlushMerger(SinkThread& st, int shards) : st_(st), shards_(shards) {}
    void deliver(int64_t index, int64_t watermark, std::vector<WindowDelta>&& rows) {
        std::lock_guard<std::mutex> g(m_);
        Pending& p = pend_[index];
        if (p.left < 0) {
            p.left = shards_;
            p.f.index = index;
            p.f.watermarkMs = INT64_MAX;
        }
        p.f.watermarkMs = std::min(p.f.watermarkMs, watermark);
        for (auto& r : rows) p.f.rows.push_back(std::move(r));
        --p.left;
        while (!pend_.empty() && pend_.begin()->first == next_ && pend_.begin()->second.left == 0) {
            st_.push(std::move(pend_.begin()->second.f));
            pend_.erase(pend_.begin());
            ++next_;
        }
    }
    bool empty() {
        std::lock_guard<std::mutex> g(m_);
        return pend_.empty();
    }

private:
    struct Pending {
        int left = -1;
        FlushRows f;
    };
    SinkThread& st_;
    const int shards_;
    std::mutex m_;
    std::map<int64_t, Pending> pend_;
    int64_t next_ = 0;
};

}  // namespace

std::string StreamingJob::mergeCheck(int shards, int flushes, uint64_t seed) {
    if (shards < 1 || flushes < 1) throw std::runtime_error("mergeCheck: shards and flushes must be >= 1");
    const int64_t W0 = 1700000000000LL, STEP = 2500;
    std::vector<std::vector<int64_t>> wm(shards, std::vector<int64_t>(flushes));
    std::mt19937_64 rng(seed);
    for (int s = 0; s < shards; ++s)
        for (int i = 0; i < flushes; ++i) wm[s][i] = W0 + i * STEP - (int64_t)(rng() % 3001);
    std::vector<FlushRows> got;
    std::mutex gm;
    int64_t fake_now = W0;
    std::set<int64_t> closed;
    {
        SinkThread st([&](const FlushRows& f, int64_t) {
            std::lock_guard<std::mutex> g(gm);
            got.push_back(f);
        }, [&]() { return fake_now; });
        FlushMerger merger(st, shards);
        std::vector<std::thread> th;
        for (int s = 0; s < shards; ++s)
            th.emplace_back([&, s]() {
                std::mt19937_64 r(seed * 977 + (uint64_t)s);
                for (int i = 0; i < flushes; ++i) {
                    std::this_thread::sleep_for(std::chrono::microseconds(r() % 300));
                    const int64_t w = (W0 + i * STEP) / BUCKET_MS * BUCKET_MS;
                    std::vector<WindowDelta> rows{{"c" + std::to_string(s), w, (uint64_t)(s + 1)}};
                    merger.deliver(i, wm[s][i], std::move(rows));
                }
            });
        for (auto& t : th) t.join();
        st.finish();
        closed = st.closed;
    }
    // the expectation: in index order, min watermark, every shard's row; windows closed by the
    // first flush (at or after the one that first shows them) whose watermark passes their end
    bool inOrder = (int)got.size() == flushes, wmMin = true, rowsOk = true;
    std::set<int64_t> seen, want;
    for (int i = 0; i < (int)got.size(); ++i) {
        const FlushRows& f = got[i];
        inOrder = inOrder && f.index == i;
        int64_t m = INT64_MAX;
        for (int s = 0; s < shards; ++s) m = std::min(m, wm[s][std::min<int64_t>(f.index, flushes - 1)]);
        wmMin = wmMin && f.watermarkMs == m;
        std::set<std::string> cs;
        for (const WindowDelta& d : f.rows) cs.insert(d.campaign);
        rowsOk = rowsOk && (int)f.rows.size() == shards && (int)cs.size() == shards;
        for (const WindowDelta& d : f.rows) seen.insert(d.windowMs);
        for (int64_t w : seen)
            if (w + BUCKET_MS <= f.watermarkMs) want.insert(w);
    }
    const bool ok = inOrder && wmMin && rowsOk && closed == want && !want.empty();
    char b[320];
    std::snprintf(b, sizeof b,
                  "{\"mode\": \"stream-merge-check\", \"shards\": %d, \"flushes\": %d, \"delivered\": %zu, "
                  "\"in_order\": %s, \"watermark_min\": %s, \"rows\": %s, \"closed\": %zu, \"closed_expected\": %zu, "
                  "\"ok\": %s}",
                  shards, flushes, got.size(), inOrder ? "true" : "false", wmMin ? "true" : "false",
                  rowsOk ? "true" : "false", closed.size(), want.size(), ok ? "true" : "false");
    return b;
}

StreamReport StreamingJob::run(const FlushSink& sink) {
    StreamReport rep;
    const unsigned T = default_threads(o_);
    const double wall0 = now_s() + 0.1;   // the replay clock starts 100 ms from now (feeders started)
    auto clock = [&]() -> int64_t { return o_.t0Ms + (int64_t)((now_s() - wall0) * 1000.0 * o_.speedup); };
    auto wallOf = [&](int64_t eventMs) { return wall0 + (double)(eventMs - o_.t0Ms) / (1000.0 * o_.speedup); };
    SinkThread st(sink, clock);
    FlushMerger merger(st, (int)shards_.size());
    rep.linesPerCycle = shards_[0]->cyc.lines();
    const double stopAt = wall0 + o_.seconds;
    std::atomic<int64_t> flushReq{0};
    std::atomic<bool> stop{false}, final{false}, failed{false};

    // ---- one feeder per shard: it owns the shard's context ------------------------------
    auto feed = [&](Shard* s) {
        const double cpu0 = thread_cpu_s();
        try {
            pin_to(s->cpus);
            WorkerPool pool(o_.replay == StreamOptions::COPY ? T : 1u);
            ysb_copy_time(s->ctx, nullptr, nullptr, nullptr);   // reset the copy timing
            check_ctx(ysb_wait(s->ctx, 0), s->ctx, "ysb_wait");
            auto takeFlushes = [&](bool wait) {
                while (!s->flushes.empty()) {
                    uint64_t n = 0;
                    int more = 0;
                    int rc = ysb_flush_end(s->ctx, wait ? 1 : 0, nullptr, 0, &n, &more);
                    if (rc == YSB_PENDING) break;
                    check_ctx(rc, s->ctx, "ysb_flush_end");
                    std::vector<ysb_count> rows(std::max<uint64_t>(n, 1));
                    check_ctx(ysb_flush_end(s->ctx, 1, rows.data(), n, &n, &more), s->ctx, "ysb_flush_end");
                    std::vector<WindowDelta> d;
                    d.reserve(n);
                    for (uint64_t i = 0; i < n; ++i) d.push_back({campaigns_[rows[i].campaign], rows[i].window_ms, rows[i].count});
                    merger.deliver(s->flushes.front().first, s->flushes.front().second, std::move(d));
                    s->flushes.pop_front();
                }
            };
            auto beginFlushes = [&]() {
                const int64_t want = flushReq.load();
                while (s->flushBegun < want) {
                    if (s->flushes.size() == 4) takeFlushes(true);   // at most 4 outstanding: the oldest first
                    check_ctx(ysb_flush_begin(s->ctx, INT64_MIN, INT64_MAX), s->ctx, "ysb_flush_begin");
                    s->flushes.push_back({s->flushBegun++, s->maxTime == INT64_MIN ? INT64_MIN : s->maxTime - o_.oooMs});
                }
            };
            // the ring follows this shard's watermark: when the newest bucket nears the ring's
            // end, a synchronous move (rare) -- only when it moves the base
            auto followRing = [&]() {
                if (s->maxTime == INT64_MIN) return;
                if (s->maxTime / BUCKET_MS + 8 < s->ringLo + (int64_t)o_.windowRing) return;
                const int64_t lo = (s->maxTime - o_.oooMs) / BUCKET_MS - 8;
                if (lo <= s->ringLo) return;
                takeFlushes(true);
                check_ctx(ysb_ring_advance(s->ctx, lo), s->ctx, "ysb_ring_advance");
                s->ringLo = lo;
                ++s->ringAdvances;
            };
            while (!stop.load()) {
                const double w = now_s();
                bool any = false;
                const ReplayCycle::Batch& b = s->cyc.batches[s->next];
                const double due = wallOf(b.releaseMs + (int64_t)s->cycle * o_.cycleMs);
                if (w >= due && w < stopAt) {
                    s->maxBehindMs = std::max(s->maxBehindMs, (w - due) * 1e3);
                    const double t0 = now_s();
                    const ysb_rebase rb{b.a, (int64_t)s->cycle * (o_.cycleMs / BUCKET_MS)};
                    if (o_.replay == StreamOptions::MAPPED) {
                        check_ctx(ysb_submit_mapped(s->ctx, s->cur, s->cyc.bytes + b.off, b.nbytes, s->d_lineOff + b.a,
                                                    b.b - b.a, &rb), s->ctx, "ysb_submit_mapped");
                    } else if (o_.replay == StreamOptions::MAPPED_RAW) {
                        check_ctx(ysb_submit_raw_mapped(s->ctx, s->cur, s->cyc.bytes + b.off, b.nbytes, &rb), s->ctx,
                                  "ysb_submit_raw_mapped");
                    } else {
                        check_ctx(ysb_wait(s->ctx, s->cur), s->ctx, "ysb_wait");   // the slot's last copy is done
                        const uint64_t nb = fill_batch(s->cyc, b, s->cycle, o_.cycleMs, s->slot[s->cur], pool, T);
                        check_ctx(ysb_submit_raw(s->ctx, s->cur, s->slot[s->cur], nb), s->ctx, "ysb_submit_raw");
                    }
                    const double t1 = now_s(), dt = (t1 - t0) * 1e3;
                    s->submitMs += dt;
                    if (dt > 1.0) {
                        ++s->slowSubmits;
                        s->slowMs += dt;
                        s->slowMaxMs = std::max(s->slowMaxMs, dt);
                    }
                    if (!s->firstSubmit) s->firstSubmit = t0;
                    s->lastSubmit = t1;
                    s->maxTime = std::max(s->maxTime, b.maxTimeMs + (int64_t)s->cycle * o_.cycleMs);
                    s->events += b.b - b.a;
                    ++s->batches;
                    s->cur ^= 1;
                    if (++s->next == s->cyc.batches.size()) {
                        s->next = 0;
                        ++s->cycle;
                    }
                    any = true;
                }
                beginFlushes();
                takeFlushes(false);
                followRing();
                if (!any) {
                    // sleep until the next batch is due (at most 200 us: flushes to begin / take)
                    const double nd = wallOf(s->cyc.batches[s->next].releaseMs + (int64_t)s->cycle * o_.cycleMs) - now_s();
                    if (nd > 20e-6) std::this_thread::sleep_for(std::chrono::microseconds((int64_t)std::min(200.0, nd * 1e6 - 10)));
                }
            }
            // end of input: every batch counted, then the final flushes the coordinator asks for
            check_ctx(ysb_sync(s->ctx), s->ctx, "ysb_sync");
            s->doneAt = now_s();
            s->synced = true;
            while (!final.load() && !failed.load()) std::this_thread::sleep_for(std::chrono::microseconds(100));
            if (!failed.load()) {
                beginFlushes();
                takeFlushes(true);
            }
        } catch (const std::exception& e) {
            s->error = e.what();
            failed = true;
            s->synced = true;
        }
        s->cpuS = thread_cpu_s() - cpu0;
    };
    for (Shard* s : shards_) s->th = std::thread(feed, s);

    // ---- the flusher's clock (CampaignProcessorCommon.java:45: every flushMs) ----------------
    int64_t nextFlush = o_.t0Ms + o_.flushMs;
    while (now_s() < stopAt && !failed.load()) {
        if (clock() >= nextFlush) {
            ++flushReq;
            nextFlush += o_.flushMs;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    stop = true;
    for (Shard* s : shards_)
        while (!s->synced.load()) std::this_thread::sleep_for(std::chrono::microseconds(100));
    ++flushReq;   // the last flush: everything submitted
    final = true;
    for (Shard* s : shards_) s->th.join();
    for (Shard* s : shards_)
        if (!s->error.empty()) throw std::runtime_error("shard " + std::to_string(s->index) + ": " + s->error);
    if (!merger.empty()) throw std::runtime_error("a flush was not delivered by every shard");

    // a drain for anything outside the ring (the side list); the watermark stays where the input stopped
    FlushRows last;
    last.index = flushReq.load();
    last.watermarkMs = INT64_MAX;
    for (Shard* s : shards_) {
        last.watermarkMs = std::min(last.watermarkMs, s->maxTime == INT64_MIN ? INT64_MIN : s->maxTime - o_.oooMs);
        uint64_t n = 0;
        check_ctx(ysb_drain(s->ctx, INT64_MIN, INT64_MAX, 0, nullptr, 0, &n), s->ctx, "ysb_drain");
        std::vector<ysb_count> rows(std::max<uint64_t>(n, 1));
        check_ctx(ysb_drain(s->ctx, INT64_MIN, INT64_MAX, 1, rows.data(), n, &n), s->ctx, "ysb_drain");
        for (uint64_t i = 0; i < n; ++i) last.rows.push_back({campaigns_[rows[i].campaign], rows[i].window_ms, rows[i].count});
    }
    const int64_t finalWm = last.watermarkMs;
    st.push(std::move(last));
    st.finish();

    double first = 0, lastSubmit = 0, done = 0;
    for (Shard* s : shards_) {
        ShardReport sr;
        sr.device = s->device;
        sr.numaNode = s->node;
        sr.pinned = s->pinned;
        sr.events = s->events;
        sr.batches = s->batches;
        sr.cycles = s->cycle;
        sr.partialLines = s->next ? s->cyc.batches[s->next].a : 0;
        sr.submitMs = s->submitMs;
        sr.feederCpuS = s->cpuS;
        sr.maxBehindMs = s->maxBehindMs;
        sr.ringAdvances = s->ringAdvances;
        sr.replayGB = (double)s->cyc.used / 1e9;
        sr.prepareS = s->prepareS;
        sr.registerS = s->registerS;
        rep.shards.push_back(sr);
        rep.events += s->events;
        rep.batches += s->batches;
        rep.cycles.push_back(s->cycle);
        rep.partialLines.push_back(sr.partialLines);
        rep.slotWaits += s->slowSubmits;
        rep.slotWaitMs += s->slowMs;
        rep.slotWaitMaxMs = std::max(rep.slotWaitMaxMs, s->slowMaxMs);
        rep.maxBehindMs = std::max(rep.maxBehindMs, s->maxBehindMs);
        rep.ringAdvances += s->ringAdvances;
        if (s->firstSubmit && (!first || s->firstSubmit < first)) first = s->firstSubmit;
        lastSubmit = std::max(lastSubmit, s->lastSubmit);
        done = std::max(done, s->doneAt);
        double ms = 0;
        uint64_t copies = 0, bytes = 0;
        check_ctx(ysb_copy_time(s->ctx, &ms, &copies, &bytes), s->ctx, "ysb_copy_time");
        rep.copyMs += ms;
        rep.copyBytes += bytes;
        ysb_stats x;
        check_ctx(ysb_stats_get(s->ctx, &x), s->ctx, "ysb_stats_get");
        rep.overflowDropped += x.overflow_dropped;
        rep.parseErrors += x.parse_errors;
        rep.joinMisses += x.join_misses;
    }
    // every submitted event counted, from the first submit to the last shard's ysb_sync
    rep.wallSeconds = first ? done - first : 0;
    rep.eventsPerSecond = rep.wallSeconds > 0 ? (double)rep.events / rep.wallSeconds : 0;
    rep.submitEventsPerSecond = lastSubmit > first ? (double)rep.events / (lastSubmit - first) : 0;
    rep.targetEventsPerSecond = o_.eventRate * o_.speedup * (double)shards_.size();
    rep.copyGBs = rep.copyMs > 0 ? (double)rep.copyBytes / (rep.copyMs * 1e-3) / 1e9 : 0;
    rep.copyBusyFrac = rep.wallSeconds > 0 ? rep.copyMs * 1e-3 / rep.wallSeconds / (double)shards_.size() : 0;
    rep.flushes = st.flushes;
    rep.rowsWritten = st.rows;
    rep.closeReplayMs = st.closeMs;
    rep.cwReplayMs = st.cwMs;
    rep.openAtEnd = st.seen.size() - st.closed.size();
    rep.finalWatermarkMs = finalWm;
    return rep;
}

}  // namespace topology
}  // namespace ysb
