// ysb_stream.cpp -- implementation of ysb_stream.hpp (the runner's streaming mode).
#include "ysb_stream.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
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

constexpr int64_t BUCKET_MS = 10000;      // CampaignProcessorCommon.java:28 (time_divisor)
constexpr uint64_t GEN_PIECE = 8u << 20;  // events per device generator call
const char ET_KEY[] = "\"event_time\"";

void check_ctx(int rc, ysb_ctx* c, const char* what) {
    if (rc != YSB_OK) throw std::runtime_error(std::string(what) + ": " + ysb_last_error(c));
}

}  // namespace

// One cycle of the replay: the generator's lines over cycleMs of event time, each line's 13
// time digits located, and the slot-sized batches it is released in.
struct ReplayCycle {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> start;     // n + 1 line starts
    std::vector<uint16_t> timePos;   // the 13 time digits' offset within the line
    std::vector<uint16_t> upper;     // their leading 9 digits, minus upperMin
    int64_t upperMin = 0;
    uint32_t nUpper = 0;
    struct Batch {
        uint64_t a, b;               // lines [a, b)
        int64_t releaseMs;           // nominal emission time of line b - 1 (cycle 0)
        int64_t maxTimeMs;           // the largest event_time in it (cycle 0)
    };
    std::vector<Batch> batches;
    uint64_t lines() const { return start.size() - 1; }
};

struct StreamingJob::Shard {
    int index = 0, device = 0;
    ysb_ctx* ctx = nullptr;
    uint8_t* slot[2] = {nullptr, nullptr};
    ysb_gen_params gen{};
    std::vector<uint32_t> subset;
    ReplayCycle cyc;
    // progress
    uint64_t cycle = 0, next = 0;    // the next batch: cyc.batches[next] of cycle `cycle`
    int cur = 0;
    int64_t maxTime = INT64_MIN;
    uint64_t events = 0, batches = 0;
    std::deque<int64_t> flushes;     // indices of this shard's outstanding asynchronous flushes
    int64_t ringLo = 0;
    ~Shard() {
        if (ctx) ysb_close(ctx);
    }
};

StreamingJob::StreamingJob(const StreamOptions& o) : o_(o) {
    if (o_.cycleMs <= 0 || o_.cycleMs % BUCKET_MS) throw std::runtime_error("the replay cycle must be a multiple of 10 000 ms");
    if (o_.t0Ms % BUCKET_MS) throw std::runtime_error("t0 must be a multiple of 10 000 ms");
    if (o_.shards < 1 || o_.eventRate < 1 || o_.speedup <= 0) throw std::runtime_error("bad stream options");
}

StreamingJob::~StreamingJob() {
    for (Shard* s : shards_) delete s;
}

// The shard's replay cycle: generated on its GPU (ysb_gen_events_device, the data/ generator)
// in pieces and copied to host memory -- or, ctx NULL (the CPU self-check), by the host
// generator -- then indexed.
static void build_cycle(ysb_ctx* ctx, const ysb_gen_params& g, const StreamOptions& o,
                        ReplayCycle& c, WorkerPool& pool) {
    const uint64_t n = (uint64_t)(o.eventRate * (double)o.cycleMs / 1000.0);
    if (n == 0) throw std::runtime_error("empty replay cycle");
    const uint64_t maxLine = ysb_gen_max_line_bytes(&g);
    c.bytes.reserve(n * 256);
    c.start.assign(n + 1, 0);
    void *d_b = nullptr, *d_o = nullptr;
    const uint64_t piece = std::min<uint64_t>(n, GEN_PIECE);
    std::vector<uint8_t> hbuf;
    if (ctx) {
        check_ctx(ysb_device_alloc(ctx, piece * maxLine + 64, &d_b), ctx, "ysb_device_alloc");
        check_ctx(ysb_device_alloc(ctx, piece * 4 + 64, &d_o), ctx, "ysb_device_alloc");
    } else {
        hbuf.resize(piece * maxLine + 64);
    }
    std::vector<uint32_t> off(piece);
    for (uint64_t first = 0; first < n; first += piece) {
        const uint64_t m = std::min(piece, n - first);
        uint64_t nb = 0;
        const uint64_t base = c.bytes.size();
        if (ctx) {
            check_ctx(ysb_gen_events_device(ctx, &g, first, m, (uint8_t*)d_b, piece * maxLine, (uint32_t*)d_o, &nb), ctx,
                      "ysb_gen_events_device");
            c.bytes.resize(base + nb);
            check_ctx(ysb_memcpy_d2h(ctx, c.bytes.data() + base, d_b, nb), ctx, "ysb_memcpy_d2h");
            check_ctx(ysb_memcpy_d2h(ctx, off.data(), d_o, m * 4), ctx, "ysb_memcpy_d2h");
        } else {
            if (ysb_gen_events_host_mt(&g, first, m, hbuf.data(), hbuf.size(), off.data(), &nb, pool.size()) != YSB_OK)
                throw std::runtime_error(std::string("ysb_gen_events_host_mt: ") + ysb_last_error(nullptr));
            c.bytes.insert(c.bytes.end(), hbuf.begin(), hbuf.begin() + (ptrdiff_t)nb);
        }
        for (uint64_t i = 0; i < m; ++i) c.start[first + i] = base + off[i];
    }
    c.start[n] = c.bytes.size();
    if (ctx) {
        ysb_device_free(ctx, d_b);
        ysb_device_free(ctx, d_o);
    }
    // each line's 13 time digits: their offset and the leading nine as a number
    c.timePos.assign(n, 0);
    std::vector<int64_t> up(n), tm(n);
    std::vector<std::string> err(pool.size());
    pool.run(pool.size(), [&](unsigned t) {
        const uint64_t a = n * t / pool.size(), b = n * (t + 1) / pool.size();
        for (uint64_t i = a; i < b && err[t].empty(); ++i) {
            const uint8_t* l = c.bytes.data() + c.start[i];
            const uint64_t len = c.start[i + 1] - c.start[i];
            const void* k = memmem(l, len, ET_KEY, sizeof ET_KEY - 1);
            uint64_t p = k ? (uint64_t)((const uint8_t*)k - l) + sizeof ET_KEY - 1 : len;
            while (p < len && (l[p] == ' ' || l[p] == ':')) ++p;
            if (p < len && l[p] == '"') ++p;
            if (p + 13 >= len || l[p + 13] != '"') { err[t] = "line " + std::to_string(i) + ": no 13-digit event_time"; break; }
            int64_t v = 0;
            for (int d = 0; d < 13; ++d) {
                if (l[p + d] < '0' || l[p + d] > '9') { err[t] = "line " + std::to_string(i) + ": event_time"; break; }
                v = v * 10 + (l[p + d] - '0');
            }
            c.timePos[i] = (uint16_t)p;
            up[i] = v / BUCKET_MS;
            tm[i] = v;
        }
    });
    for (const auto& e : err)
        if (!e.empty()) throw std::runtime_error("replay cycle: " + e);
    c.upperMin = *std::min_element(up.begin(), up.end());
    const int64_t umax = *std::max_element(up.begin(), up.end());
    if (umax - c.upperMin >= 65535) throw std::runtime_error("replay cycle spans too many windows");
    c.nUpper = (uint32_t)(umax - c.upperMin + 1);
    c.upper.resize(n);
    for (uint64_t i = 0; i < n; ++i) c.upper[i] = (uint16_t)(up[i] - c.upperMin);
    // batches: at most a slot's bytes and batchMs of nominal emission time each
    auto nominal = [&](uint64_t i) { return g.t0_ms + (int64_t)((i * 1000ull) / g.events_per_sec); };
    for (uint64_t a = 0; a < n;) {
        uint64_t b = a;
        int64_t mx = INT64_MIN;
        const int64_t lim = nominal(a) + o.batchMs;
        while (b < n && c.start[b + 1] - c.start[a] <= o.slotBytes && (b == a || nominal(b) < lim)) {
            mx = std::max(mx, tm[b]);
            ++b;
        }
        if (b == a) throw std::runtime_error("a replay line is longer than the slot");
        c.batches.push_back({a, b, nominal(b - 1), mx});
        a = b;
    }
}

// Batch b of cycle `cycle` into dst: its lines copied in parallel pieces, every event_time moved
// by cycle * cycleMs -- the nine leading digits replaced from a per-cycle table of the few
// values they take (the four trailing digits do not change: cycleMs is a multiple of 10 000).
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
    const uint64_t base = c.start[b.a], nb = c.start[b.b] - base;
    const uint64_t lines = b.b - b.a;
    const unsigned tn = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(std::min(T, pool.size()), nb >> 22));
    pool.run(tn, [&](unsigned t) {
        const uint64_t la = b.a + lines * t / tn, lb = b.a + lines * (t + 1) / tn;
        const uint64_t pa = c.start[la], pb = c.start[lb];
        std::memcpy(dst + (pa - base), c.bytes.data() + pa, pb - pa);
        if (shift)
            for (uint64_t i = la; i < lb; ++i)
                std::memcpy(dst + (c.start[i] - base) + c.timePos[i], &table[9ull * c.upper[i]], 9);
    });
    return nb;
}

std::string StreamingJob::replaySelfCheck(const StreamOptions& o, const std::vector<uint64_t>& cycles) {
    ysb_gen_params g;
    ysb_gen_default(&g);
    g.seed = o.seed;
    g.n_campaigns = o.campaigns;
    g.ads_per_campaign = o.adsPerCampaign;
    g.t0_ms = o.t0Ms;
    g.events_per_sec = (uint64_t)o.eventRate;
    g.with_skew = (uint32_t)o.skew;
    g.event_stream = 1;
    const unsigned T = o.threads ? o.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    WorkerPool pool(T);
    ReplayCycle c;
    build_cycle(nullptr, g, o, c, pool);
    std::vector<uint8_t> buf(o.slotBytes + 64), ref(o.slotBytes + 64);
    std::vector<uint32_t> off(c.lines() + 1);
    uint64_t lines = 0, bad = 0, batches = 0;
    for (uint64_t cy : cycles) {
        ysb_gen_params gc = g;
        gc.t0_ms = o.t0Ms + (int64_t)cy * o.cycleMs;   // the generator's own lines of that cycle
        for (const auto& b : c.batches) {
            const uint64_t nb = fill_batch(c, b, cy, o.cycleMs, buf.data(), pool, T);
            uint64_t rb = 0;
            if (ysb_gen_events_host(&gc, b.a, b.b - b.a, ref.data(), ref.size(), off.data(), &rb) != YSB_OK)
                throw std::runtime_error("ysb_gen_events_host failed");
            if (rb != nb || std::memcmp(buf.data(), ref.data(), nb) != 0) ++bad;
            lines += b.b - b.a;
            ++batches;
        }
    }
    char o2[256];
    std::snprintf(o2, sizeof o2, "{\"mode\": \"stream-self-check\", \"lines_per_cycle\": %llu, \"batches\": %llu, "
                  "\"lines\": %llu, \"mismatched_batches\": %llu, \"upper_values\": %u}",
                  (unsigned long long)c.lines(), (unsigned long long)batches, (unsigned long long)lines,
                  (unsigned long long)bad, c.nUpper);
    return o2;
}

void StreamingJob::prepare() {
    ysb_gen_params g;
    ysb_gen_default(&g);
    g.seed = o_.seed;
    g.n_campaigns = o_.campaigns;
    g.ads_per_campaign = o_.adsPerCampaign;
    std::vector<char> cid(36ull * o_.campaigns), aid(36ull * o_.campaigns * o_.adsPerCampaign);
    if (ysb_gen_ids(&g, cid.data(), aid.data()) != YSB_OK) throw std::runtime_error("ysb_gen_ids failed");
    const uint64_t A = (uint64_t)o_.campaigns * o_.adsPerCampaign;
    for (uint32_t c = 0; c < o_.campaigns; ++c) campaigns_.emplace_back(&cid[36ull * c], 36);
    for (uint64_t a = 0; a < A; ++a) ads_.emplace_back(&aid[36 * a], 36);
    const int ndev = std::max(1, ysb_device_count());
    WorkerPool pool(o_.threads ? o_.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
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
        for (int k = 0; k < 2; ++k) check_ctx(ysb_slot_buffers(sh->ctx, k, &sh->slot[k], nullptr), sh->ctx, "ysb_slot_buffers");
        // the shard's own event stream over its ad_id shard (ysb_ad_shard), as bench.py's ranks
        sh->gen = g;
        sh->gen.t0_ms = o_.t0Ms;
        sh->gen.events_per_sec = (uint64_t)o_.eventRate;
        sh->gen.with_skew = (uint32_t)o_.skew;
        sh->gen.event_stream = 1 + (uint32_t)s;
        if (o_.shards > 1) {
            for (uint64_t a = 0; a < A; ++a)
                if (ysb_ad_shard(ads_[a].data(), 36, (uint32_t)o_.shards) == (uint32_t)s) sh->subset.push_back((uint32_t)a);
            sh->gen.ad_subset = sh->subset.data();
            sh->gen.n_ad_subset = (uint32_t)sh->subset.size();
        }
        build_cycle(sh->ctx, sh->gen, o_, sh->cyc, pool);
    }
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

}  // namespace

StreamReport StreamingJob::run(const FlushSink& sink) {
    StreamReport rep;
    const unsigned T = o_.threads ? o_.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    WorkerPool pool(T);
    const double wall0 = now_s() + 0.05;   // the replay clock starts 50 ms from now (warm threads)
    auto clock = [&]() -> int64_t { return o_.t0Ms + (int64_t)((now_s() - wall0) * 1000.0 * o_.speedup); };
    auto wallOf = [&](int64_t eventMs) { return wall0 + (double)(eventMs - o_.t0Ms) / (1000.0 * o_.speedup); };
    SinkThread st(sink, clock);
    rep.linesPerCycle = shards_[0]->cyc.lines();
    for (Shard* s : shards_) {
        ysb_copy_time(s->ctx, nullptr, nullptr, nullptr);   // reset the copy timing
        check_ctx(ysb_wait(s->ctx, 0), s->ctx, "ysb_wait");
    }
    std::deque<FlushRows> pending;   // begun on every shard, not yet taken from all
    std::deque<int> pendingLeft;
    int64_t nextFlush = o_.t0Ms + o_.flushMs, flushIndex = 0;
    const double stopAt = wall0 + o_.seconds;
    double firstSubmit = 0, lastSubmit = 0;

    auto fill = [&](Shard* s, const ReplayCycle::Batch& b, uint8_t* dst) -> uint64_t {
        return fill_batch(s->cyc, b, s->cycle, o_.cycleMs, dst, pool, T);
    };

    auto takeFlushes = [&](bool wait) {
        for (Shard* s : shards_) {
            while (!s->flushes.empty()) {
                uint64_t n = 0;
                int more = 0;
                int rc = ysb_flush_end(s->ctx, wait ? 1 : 0, nullptr, 0, &n, &more);
                if (rc == YSB_PENDING) break;
                check_ctx(rc, s->ctx, "ysb_flush_end");
                std::vector<ysb_count> rows(std::max<uint64_t>(n, 1));
                check_ctx(ysb_flush_end(s->ctx, 1, rows.data(), n, &n, &more), s->ctx, "ysb_flush_end");
                const int64_t idx = s->flushes.front();
                s->flushes.pop_front();
                const size_t at = (size_t)(idx - pending.front().index);
                for (uint64_t i = 0; i < n; ++i)
                    pending[at].rows.push_back({campaigns_[rows[i].campaign], rows[i].window_ms, rows[i].count});
                --pendingLeft[at];
            }
        }
        while (!pending.empty() && pendingLeft.front() == 0) {
            st.push(std::move(pending.front()));
            pending.pop_front();
            pendingLeft.pop_front();
        }
    };

    auto watermark = [&]() {
        int64_t wm = INT64_MAX;
        for (Shard* s : shards_) wm = std::min(wm, s->maxTime == INT64_MIN ? INT64_MIN : s->maxTime - o_.oooMs);
        return wm;
    };

    auto beginFlush = [&]() {
        FlushRows f;
        f.index = flushIndex++;
        f.watermarkMs = watermark();
        for (Shard* s : shards_) {
            if (s->flushes.size() == 4) {   // at most 4 outstanding: take the oldest first
                takeFlushes(true);
            }
            check_ctx(ysb_flush_begin(s->ctx, INT64_MIN, INT64_MAX), s->ctx, "ysb_flush_begin");
            s->flushes.push_back(f.index);
        }
        pending.push_back(std::move(f));
        pendingLeft.push_back((int)shards_.size());
    };

    // the ring follows the watermark: when it nears the ring's end, a synchronous move (rare)
    auto followRing = [&](Shard* s) {
        const int64_t wmB = s->maxTime / BUCKET_MS;
        if (wmB + 8 < s->ringLo + (int64_t)o_.windowRing) return;
        takeFlushes(true);
        const int64_t lo = std::max(s->ringLo, watermark() / BUCKET_MS - 8);
        check_ctx(ysb_ring_advance(s->ctx, lo), s->ctx, "ysb_ring_advance");
        s->ringLo = lo;
        ++rep.ringAdvances;
    };

    while (true) {
        const double w = now_s();
        bool any = false, running = w < stopAt;
        for (Shard* s : shards_) {
            if (!running) break;
            const ReplayCycle::Batch& b = s->cyc.batches[s->next];
            const int64_t rel = b.releaseMs + (int64_t)s->cycle * o_.cycleMs;
            const double due = wallOf(rel);
            if (w < due) continue;
            rep.maxBehindMs = std::max(rep.maxBehindMs, (w - due) * 1e3);
            const uint64_t nb = fill(s, b, s->slot[s->cur]);
            check_ctx(ysb_submit_raw(s->ctx, s->cur, s->slot[s->cur], nb), s->ctx, "ysb_submit_raw");
            if (!firstSubmit) firstSubmit = now_s();
            lastSubmit = now_s();
            s->maxTime = std::max(s->maxTime, b.maxTimeMs + (int64_t)s->cycle * o_.cycleMs);
            s->events += b.b - b.a;
            ++s->batches;
            s->cur ^= 1;
            const double t0 = now_s();
            check_ctx(ysb_wait(s->ctx, s->cur), s->ctx, "ysb_wait");   // the other slot's copy: refill it
            const double wt = (now_s() - t0) * 1e3;
            if (wt > 0.1) {
                ++rep.slotWaits;
                rep.slotWaitMs += wt;
                rep.slotWaitMaxMs = std::max(rep.slotWaitMaxMs, wt);
            }
            if (++s->next == s->cyc.batches.size()) {
                s->next = 0;
                ++s->cycle;
            }
            followRing(s);
            any = true;
        }
        if (clock() >= nextFlush && running) {
            beginFlush();
            nextFlush += o_.flushMs;
            any = true;
        }
        takeFlushes(false);
        if (!running) break;
        if (!any) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    // end of input: every batch counted, the last flush, then a drain for anything outside the
    // ring (the side list); the watermark stays where the input stopped
    for (Shard* s : shards_) check_ctx(ysb_sync(s->ctx), s->ctx, "ysb_sync");
    beginFlush();
    takeFlushes(true);
    FlushRows last;
    last.index = flushIndex++;
    last.watermarkMs = watermark();
    for (Shard* s : shards_) {
        uint64_t n = 0;
        check_ctx(ysb_drain(s->ctx, INT64_MIN, INT64_MAX, 0, nullptr, 0, &n), s->ctx, "ysb_drain");
        std::vector<ysb_count> rows(std::max<uint64_t>(n, 1));
        check_ctx(ysb_drain(s->ctx, INT64_MIN, INT64_MAX, 1, rows.data(), n, &n), s->ctx, "ysb_drain");
        for (uint64_t i = 0; i < n; ++i) last.rows.push_back({campaigns_[rows[i].campaign], rows[i].window_ms, rows[i].count});
    }
    st.push(std::move(last));
    st.finish();

    rep.wallSeconds = lastSubmit - firstSubmit;
    for (Shard* s : shards_) {
        rep.events += s->events;
        rep.batches += s->batches;
        rep.cycles.push_back(s->cycle);
        rep.partialLines.push_back(s->next ? s->cyc.batches[s->next].a : 0);
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
    // (the last batch's events count over the interval up to its submit: close enough at
    // hundreds of batches; the report also carries the wall time)
    rep.eventsPerSecond = rep.wallSeconds > 0 ? (double)rep.events / rep.wallSeconds : 0;
    rep.targetEventsPerSecond = o_.eventRate * o_.speedup * (double)shards_.size();
    rep.copyGBs = rep.copyMs > 0 ? (double)rep.copyBytes / (rep.copyMs * 1e-3) / 1e9 : 0;
    rep.copyBusyFrac = rep.wallSeconds > 0 ? rep.copyMs * 1e-3 / rep.wallSeconds / (double)shards_.size() : 0;
    rep.flushes = st.flushes;
    rep.rowsWritten = st.rows;
    rep.closeReplayMs = st.closeMs;
    rep.cwReplayMs = st.cwMs;
    rep.openAtEnd = st.seen.size() - st.closed.size();
    rep.finalWatermarkMs = watermark();
    return rep;
}

}  // namespace topology
}  // namespace ysb
