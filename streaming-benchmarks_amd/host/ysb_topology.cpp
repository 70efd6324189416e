// ysb_topology.cpp -- implementation of ysb_topology.hpp (see there for what each class
// restates from the reference).
#include "ysb_topology.hpp"
#include "worker_pool.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <fstream>
#include <random>
#include <set>
#include <sstream>
#include <thread>

namespace ysb {
namespace topology {

// ---- text helpers ----------------------------------------------------------------------------

std::string readFile(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) throw std::runtime_error("java.io.FileNotFoundException: " + path);
    std::ostringstream ss;
    ss << in.rdbuf();
    return ss.str();
}

std::vector<std::string> readLines(const std::string& t) {
    std::vector<std::string> out;
    size_t p = 0;
    while (p < t.size()) {
        size_t q = p;
        while (q < t.size() && t[q] != '\n' && t[q] != '\r') ++q;
        out.emplace_back(t, p, q - p);
        if (q < t.size() && t[q] == '\r' && q + 1 < t.size() && t[q + 1] == '\n') ++q;
        p = q + 1;
    }
    return out;
}

std::vector<std::string> javaSplit(const std::string& s, char sep) {
    std::vector<std::string> out;
    size_t p = 0;
    while (true) {
        const size_t q = s.find(sep, p);
        out.emplace_back(s, p, (q == std::string::npos ? s.size() : q) - p);
        if (q == std::string::npos) break;
        p = q + 1;
    }
    // "If the expression does not match any part of the input then the resulting array
    // has just one element, namely this string" -- otherwise drop trailing empties
    if (out.size() > 1)
        while (!out.empty() && out.back().empty()) out.pop_back();
    return out;
}

static std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
    return s.substr(a, b - a);
}

static std::string unquote(const std::string& v) {
    if (v.size() >= 2 && ((v.front() == '"' && v.back() == '"') || (v.front() == '\'' && v.back() == '\'')))
        return v.substr(1, v.size() - 2);
    return v;
}

// A '#' that starts a comment (at the line start or after blank, outside quotes).
static std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (q) {
            if (c == q) q = 0;
        } else if (c == '"' || c == '\'') {
            q = c;
        } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
            return s.substr(0, i);
        }
    }
    return s;
}

// ---- Config ---------------------------------------------------------------------------------

Config Config::parse(const std::string& text) {
    Config c;
    std::string list_key;
    int line_no = 0;
    for (const std::string& raw : readLines(text)) {
        ++line_no;
        const std::string ln = trim(strip_comment(raw));
        if (ln.empty() || ln == "---") continue;
        if (ln[0] == '-') {
            if (list_key.empty())
                throw std::runtime_error("config line " + std::to_string(line_no) + ": list item without a key");
            c.lists_[list_key].push_back(unquote(trim(ln.substr(1))));
            continue;
        }
        size_t colon = std::string::npos;
        for (size_t i = 0; i < ln.size(); ++i)
            if (ln[i] == ':' && (i + 1 == ln.size() || ln[i + 1] == ' ' || ln[i + 1] == '\t')) { colon = i; break; }
        if (colon == std::string::npos)
            throw std::runtime_error("config line " + std::to_string(line_no) + ": expected `key: value`");
        const std::string key = unquote(trim(ln.substr(0, colon)));
        const std::string val = trim(ln.substr(colon + 1));
        if (val.empty()) {
            list_key = key;
            c.lists_[key];
            c.scalars_.erase(key);
        } else {
            list_key.clear();
            c.scalars_[key] = unquote(val);
            c.lists_.erase(key);
        }
    }
    return c;
}

Config Config::findAndReadConfigFile(const std::string& path, bool mustExist) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        if (mustExist) throw std::runtime_error("Could not find config file on classpath " + path);
        return Config();
    }
    std::ostringstream ss;
    ss << in.rdbuf();
    Config c = parse(ss.str());
    if (mustExist && c.scalars_.empty() && c.lists_.empty())
        throw std::runtime_error("Config file " + path + " doesn't have any valid storm configs");
    return c;
}

bool Config::has(const std::string& k) const { return scalars_.count(k) || lists_.count(k); }

const std::string& Config::get(const std::string& k) const {
    auto it = scalars_.find(k);
    if (it == scalars_.end()) throw std::runtime_error("No data for required key '" + k + "'");
    return it->second;
}

std::string Config::get(const std::string& k, const std::string& dflt) const {
    auto it = scalars_.find(k);
    return it == scalars_.end() ? dflt : it->second;
}

long long Config::getLong(const std::string& k) const {
    const std::string& v = get(k);
    char* end = nullptr;
    errno = 0;
    const long long x = std::strtoll(v.c_str(), &end, 10);
    if (errno || end == v.c_str() || *end) throw std::runtime_error("java.lang.NumberFormatException: " + v);
    return x;
}

const std::vector<std::string>& Config::getList(const std::string& k) const {
    auto it = lists_.find(k);
    if (it == lists_.end()) throw std::runtime_error("No list for required key '" + k + "'");
    return it->second;
}

// ---- AdCampaignMap ----------------------------------------------------------------------------

void AdCampaignMap::put(const std::string& ad, const std::string& campaign) {
    auto ci = campaignIndex_.find(campaign);
    uint32_t c;
    if (ci == campaignIndex_.end()) {
        c = (uint32_t)campaigns.size();
        campaignIndex_.emplace(campaign, c);
        campaigns.push_back(campaign);
    } else {
        c = ci->second;
    }
    auto ai = adIndex_.find(ad);
    if (ai == adIndex_.end()) {   // HashMap.put: a later duplicate wins
        adIndex_.emplace(ad, (uint32_t)ads.size());
        ads.push_back(ad);
        adCampaign.push_back(c);
    } else {
        adCampaign[ai->second] = c;
    }
}

AdCampaignMap AdCampaignMap::fromCsv(const std::string& text) {
    AdCampaignMap m;
    uint64_t n = 0;
    for (const std::string& ln : readLines(text)) {
        ++n;
        const std::vector<std::string> kv = javaSplit(ln, ',');
        if (kv.size() < 2)
            throw std::runtime_error("java.lang.ArrayIndexOutOfBoundsException: 1 (ad map line " + std::to_string(n) + ")");
        m.put(kv[0], kv[1]);
    }
    return m;
}

AdCampaignMap AdCampaignMap::fromJsonLines(const std::string& text) {
    AdCampaignMap m;
    uint64_t n = 0;
    for (const std::string& ln : readLines(text)) {
        ++n;
        if (trim(ln).empty()) continue;
        // `{ "AD": "CAMPAIGN"}`: the two strings of a one-entry object (no escapes)
        std::vector<std::string> str;
        size_t p = 0;
        while ((p = ln.find('"', p)) != std::string::npos) {
            const size_t q = ln.find('"', p + 1);
            if (q == std::string::npos) break;
            str.push_back(ln.substr(p + 1, q - p - 1));
            p = q + 1;
        }
        if (str.size() != 2 || ln.find('\\') != std::string::npos)
            throw std::runtime_error("ad map line " + std::to_string(n) + " is not { \"AD\": \"CAMPAIGN\"}");
        m.put(str[0], str[1]);
    }
    return m;
}

AdCampaignMap AdCampaignMap::fromFile(const std::string& path) {
    const std::string t = readFile(path);
    size_t p = 0;
    while (p < t.size() && (t[p] == ' ' || t[p] == '\n' || t[p] == '\r' || t[p] == '\t')) ++p;
    return (p < t.size() && t[p] == '{') ? fromJsonLines(t) : fromCsv(t);
}

// ---- FileBasedDataSource -----------------------------------------------------------------------

FileBasedDataSource::FileBasedDataSource(const std::string& path, unsigned threads, bool mmap) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("java.io.FileNotFoundException: " + path);
    threads_ = threads ? threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    pool_.reset(new WorkerPool(threads_));
    struct stat st;
    if (mmap && ::fstat(fd_, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
        void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd_, 0);
        if (m != MAP_FAILED) {
            ::madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
            map_ = static_cast<const uint8_t*>(m);
            size_ = (uint64_t)st.st_size;
        }
    }
}

FileBasedDataSource::~FileBasedDataSource() {
    pool_.reset();
    if (map_) ::munmap(const_cast<uint8_t*>(map_), size_);
    if (fd_ >= 0) ::close(fd_);
}

void FileBasedDataSource::rewind() {
    pos_ = 0;
    eof_ = false;
    carry_.clear();
}

// The carried partial line, then parallel preads of disjoint pieces (>= 4 MiB each) straight
// into the buffer: the bytes buf holds.
uint64_t FileBasedDataSource::readBlock(uint8_t* buf, uint64_t cap) {
    if (carry_.size() > cap) throw std::runtime_error("a line is longer than the batch buffer");
    uint64_t have = carry_.size();
    std::memcpy(buf, carry_.data(), have);
    carry_.clear();
    if (!eof_ && have < cap && map_) {   // parallel copies out of the mapping (>= 4 MiB each)
        const uint64_t want = std::min<uint64_t>(cap - have, size_ - std::min(pos_, size_));
        const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads_, want >> 22));
        pool_->run(T, [&](unsigned t) {
            const uint64_t a = want * t / T, b = want * (t + 1) / T;
            std::memcpy(buf + have + a, map_ + pos_ + a, b - a);
        });
        pos_ += want;
        have += want;
        if (pos_ >= size_) eof_ = true;
    } else if (!eof_ && have < cap) {
        const uint64_t want = cap - have;
        const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads_, want >> 22));
        std::vector<uint64_t> got(T, 0);
        std::vector<int> err(T, 0);
        pool_->run(T, [&](unsigned t) {
            const uint64_t a = want * t / T, b = want * (t + 1) / T;
            uint64_t p = a;
            while (p < b) {
                const ssize_t r = ::pread(fd_, buf + have + p, b - p, (off_t)(pos_ + p));
                if (r < 0) { if (errno == EINTR) continue; err[t] = errno; break; }
                if (r == 0) break;
                p += (uint64_t)r;
            }
            got[t] = p - a;
        });
        uint64_t read = 0;
        for (unsigned t = 0; t < T; ++t) {
            if (err[t]) throw std::runtime_error(std::string("read: ") + std::strerror(err[t]));
            read += got[t];
            if (got[t] < want * (t + 1) / T - want * t / T) { eof_ = true; break; }   // short piece: file end
        }
        pos_ += read;
        have += read;
    }
    return have;
}

// BufferedReader.readLine's terminators: "\n", "\r\n" and a lone "\r" (:153-159).  The end
// of the complete lines among buf[0, have): up to the last terminator (at end of file,
// everything); a '\r' that ends the buffer may still be followed by '\n', so it waits.
uint64_t FileBasedDataSource::completeEnd(const uint8_t* buf, uint64_t have, bool anyCr) const {
    if (eof_) return have;
    uint64_t end = 0;
    for (uint64_t q = have; q > 0; --q) {
        const uint8_t c = buf[q - 1];
        if (c == '\n' || (c == '\r' && q < have)) { end = q; break; }
        if (!anyCr) {   // only '\n' can end a line: jump to it
            const void* nl = memrchr(buf, '\n', q);
            end = nl ? (uint64_t)((const uint8_t*)nl - buf) + 1 : 0;
            break;
        }
    }
    if (end == 0) throw std::runtime_error("a line is longer than the batch buffer");
    return end;
}

uint64_t FileBasedDataSource::fillRaw(uint8_t* buf, uint64_t cap) {
    if (!cap) return 0;
    const uint64_t have = readBlock(buf, cap);
    if (have == 0) return 0;
    // only the tail decides where the complete lines end: a '\r' there needs the slow walk
    const uint64_t tail = std::min<uint64_t>(have, 1u << 16);
    const bool anyCr = std::memchr(buf + have - tail, '\r', tail) != nullptr;
    const uint64_t end = completeEnd(buf, have, anyCr);
    carry_.assign(buf + end, buf + have);
    bytes_ += end;
    return end;
}

uint64_t FileBasedDataSource::mappingBytes() const {
    const uint64_t page = (uint64_t)::sysconf(_SC_PAGESIZE);
    return map_ ? (size_ + page - 1) / page * page : 0;
}

uint64_t FileBasedDataSource::nextMapped(uint64_t cap, const uint8_t** p) {
    if (!map_) throw std::runtime_error("nextMapped needs the file mapped (--io mmap)");
    *p = map_ + pos_;
    if (!cap || pos_ >= size_) return 0;
    const uint64_t have = std::min(cap, size_ - pos_);
    uint64_t end = have;
    if (pos_ + have < size_) {   // not the file's last bytes: up to the last complete line
        const uint64_t tail = std::min<uint64_t>(have, 1u << 16);
        const bool anyCr = std::memchr(map_ + pos_ + have - tail, '\r', tail) != nullptr;
        end = completeEnd(map_ + pos_, have, anyCr);
    }
    pos_ += end;
    bytes_ += end;
    return end;
}

uint64_t FileBasedDataSource::fill(uint8_t* buf, uint64_t cap, uint32_t* off, uint64_t maxLines, uint64_t* nbytes) {
    *nbytes = 0;
    if (!maxLines || !cap) return 0;
    const uint64_t have = readBlock(buf, cap);
    if (have == 0) return 0;
    // A line keeps its terminator bytes in the batch (the parsers ignore them).
    const bool any_cr = std::memchr(buf, '\r', have) != nullptr;   // generator files: none
    const uint64_t end = completeEnd(buf, have, any_cr);
    // line starts: 0 and every byte after a terminator below `end`, in parallel pieces
    const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads_, end >> 22));
    std::vector<std::vector<uint32_t>> starts(T);
    pool_->run(T, [&](unsigned t) {
        const uint64_t a = end * t / T, b = end * (t + 1) / T;
        auto& v = starts[t];
        v.reserve((b - a) / 200 + 16);
        if (t == 0) v.push_back(0);
        if (!any_cr) {
            for (uint64_t p = a; p < b;) {
                const void* q = std::memchr(buf + p, '\n', b - p);
                if (!q) break;
                const uint64_t s = (uint64_t)((const uint8_t*)q - buf) + 1;
                if (s < end) v.push_back((uint32_t)s);
                p = s;
            }
        } else {
            for (uint64_t p = a; p < b; ++p) {
                const uint8_t c = buf[p];
                const bool term = c == '\n' || (c == '\r' && (p + 1 >= have || buf[p + 1] != '\n'));
                if (term && p + 1 < end) v.push_back((uint32_t)(p + 1));
            }
        }
    });
    uint64_t n = 0, p_end = end;
    for (unsigned t = 0; t < T && n < maxLines; ++t)
        for (uint32_t s : starts[t]) {
            if (n == maxLines) { p_end = s; break; }
            off[n++] = s;
        }
    // the rest (lines beyond maxLines, then the partial line) waits for the next call
    carry_.assign(buf + p_end, buf + have);
    *nbytes = p_end;
    lines_ += n;
    bytes_ += p_end;
    return n;
}

// ---- GpuAdCampaignOperator -----------------------------------------------------------------------

GpuAdCampaignOperator::GpuAdCampaignOperator(const AdCampaignMap& map, const Options& o) : map_(map), o_(o) {}

GpuAdCampaignOperator::~GpuAdCampaignOperator() {
    if (ctx_) ysb_close(ctx_);
}

void GpuAdCampaignOperator::check(int rc, const char* what) {
    if (rc != YSB_OK) throw std::runtime_error(std::string(what) + ": " + ysb_last_error(ctx_));
}

void GpuAdCampaignOperator::open() {
    ysb_config cfg;
    ysb_config_default(&cfg);
    cfg.time_divisor_ms = o_.timeDivisorMs;
    cfg.n_campaigns = (uint32_t)std::max<size_t>(1, map_.campaigns.size());
    cfg.window_ring = o_.windowRing;
    cfg.max_ads = map_.ads.size();
    cfg.max_batch_bytes = o_.batchBytes;
    cfg.max_batch_events = o_.batchEvents;
    // the replay file's producer is not known here: each host batch picks its scan from its
    // first line (YSB_F_LAYOUT_AUTO; the counts do not depend on it)
    cfg.flags = (o_.tbl ? YSB_F_FORMAT_TBL : 0u) | (o_.requireIp ? YSB_F_REQUIRE_IP : 0u) | YSB_F_LAYOUT_AUTO |
                YSB_F_TIMING | (o_.h2dSdma ? YSB_F_H2D_SDMA : 0u);
    if (ysb_open(&ctx_, o_.device, &cfg) != YSB_OK)
        throw std::runtime_error(std::string("ysb_open: ") + ysb_last_error(nullptr));
    // RedisJoinBolt(Map) (:443-448): the whole map on the device
    std::vector<const char*> keys(map_.ads.size());
    std::vector<uint32_t> lens(map_.ads.size());
    for (size_t i = 0; i < map_.ads.size(); ++i) {
        keys[i] = map_.ads[i].data();
        lens[i] = (uint32_t)map_.ads[i].size();
    }
    check(ysb_load_ad_map(ctx_, keys.data(), lens.data(), map_.adCampaign.data(), map_.ads.size()), "ysb_load_ad_map");
    for (int s = 0; s < 2; ++s) check(ysb_slot_buffers(ctx_, s, &bytes_[s], &off_[s]), "ysb_slot_buffers");
}

void GpuAdCampaignOperator::flatMap(const char* line, uint64_t len) {
    const bool nl = len && line[len - 1] == '\n';
    const uint64_t need = len + (nl ? 0 : 1);
    if (need > o_.batchBytes) throw std::runtime_error("record larger than the batch buffer");
    if (fillBytes_ + need > o_.batchBytes || fillEvents_ == o_.batchEvents) submit();
    off_[cur_][fillEvents_++] = (uint32_t)fillBytes_;
    std::memcpy(bytes_[cur_] + fillBytes_, line, len);
    fillBytes_ += len;
    if (!nl) bytes_[cur_][fillBytes_++] = '\n';
}

uint64_t GpuAdCampaignOperator::fillFromRaw(FileBasedDataSource& src) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t nb = src.fillRaw(bytes_[cur_] + fillBytes_, o_.batchBytes - fillBytes_);
    fillS_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fillBytes_ += nb;
    rawBytes_ += nb;
    return nb;
}

uint64_t GpuAdCampaignOperator::fillFrom(FileBasedDataSource& src) {
    uint64_t nb = 0;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t n = src.fill(bytes_[cur_] + fillBytes_, o_.batchBytes - fillBytes_, off_[cur_] + fillEvents_,
                                o_.batchEvents - fillEvents_, &nb);
    fillS_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (uint64_t i = 0; i < n; ++i) off_[cur_][fillEvents_ + i] += (uint32_t)fillBytes_;
    fillBytes_ += nb;
    fillEvents_ += n;
    return n;
}

void GpuAdCampaignOperator::registerSource(FileBasedDataSource& src) {
    if (!src.mapping()) throw std::runtime_error("--io mapped needs the events file mapped");
    check(ysb_host_register(ctx_, const_cast<uint8_t*>(src.mapping()), src.mappingBytes()), "ysb_host_register");
}

// FileBasedDataSource.run's batch without the copy into a slot: the lines stay in the page
// cache, the copy kernel reads them over PCIe into the slot's device buffer (any byte alignment:
// launch_h2d_copy_unaligned) and the GPU splits them.
uint64_t GpuAdCampaignOperator::submitMapped(FileBasedDataSource& src) {
    const uint8_t* p = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t nb = src.nextMapped(o_.batchBytes, &p);
    fillS_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!nb) return 0;
    check(ysb_submit_raw_mapped(ctx_, cur_, p, nb, nullptr), "ysb_submit_raw_mapped");
    cur_ ^= 1;
    const auto t1 = std::chrono::steady_clock::now();
    check(ysb_wait(ctx_, cur_), "ysb_wait");   // at most two batches in flight
    waitS_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    return nb;
}

void GpuAdCampaignOperator::submit() {
    if (rawBytes_) {   // raw lines (fillFromRaw): the GPU finds the line starts
        check(ysb_submit_raw(ctx_, cur_, bytes_[cur_], fillBytes_), "ysb_submit_raw");
        rawBytes_ = 0;
    } else {
        if (!fillEvents_) return;
        check(ysb_submit(ctx_, cur_, bytes_[cur_], fillBytes_, off_[cur_], fillEvents_), "ysb_submit");
    }
    submitted_ += fillEvents_;
    fillBytes_ = fillEvents_ = 0;
    cur_ ^= 1;
    const auto t0 = std::chrono::steady_clock::now();
    check(ysb_wait(ctx_, cur_), "ysb_wait");   // the other slot's H2D is done: refill it
    waitS_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void GpuAdCampaignOperator::copyTime(double* ms, uint64_t* copies, uint64_t* bytes) {
    check(ysb_copy_time(ctx_, ms, copies, bytes), "ysb_copy_time");
}

std::vector<WindowDelta> GpuAdCampaignOperator::flushWindows() {
    uint64_t n = 0;
    check(ysb_drain(ctx_, INT64_MIN, INT64_MAX, 0, nullptr, 0, &n), "ysb_drain");
    std::vector<ysb_count> rows(n ? n : 1);
    check(ysb_drain(ctx_, INT64_MIN, INT64_MAX, 1, rows.data(), n, &n), "ysb_drain");
    std::vector<WindowDelta> out;
    out.reserve(n);
    for (uint64_t i = 0; i < n; ++i)
        out.push_back({map_.campaigns[rows[i].campaign], rows[i].window_ms, rows[i].count});
    return out;
}

void GpuAdCampaignOperator::close() {
    submit();
    check(ysb_sync(ctx_), "ysb_sync");
}

ysb_stats GpuAdCampaignOperator::stats() {
    ysb_stats s;
    check(ysb_stats_get(ctx_, &s), "ysb_stats_get");
    return s;
}

// ---- RESP2 client and the Redis writer -----------------------------------------------------------

class RespClient {
public:
    RespClient(const std::string& host, int port) {
        addrinfo hints{}, *res = nullptr;
        hints.ai_socktype = SOCK_STREAM;
        if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) || !res)
            throw std::runtime_error("redis: cannot resolve " + host);
        fd_ = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
        const int rc = fd_ < 0 ? -1 : connect(fd_, res->ai_addr, res->ai_addrlen);
        freeaddrinfo(res);
        if (rc != 0) throw std::runtime_error("redis: cannot connect to " + host + ":" + std::to_string(port));
        const int one = 1;   // a pipeline goes out at once, not held back by Nagle's algorithm
        setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    }
    ~RespClient() {
        if (fd_ >= 0) ::close(fd_);
    }
    struct Reply {
        bool nil = false;
        std::string str;
        long long num = 0;
    };
    // Sends every command, then reads every reply in order.
    std::vector<Reply> pipeline(const std::vector<std::vector<std::string>>& cmds) {
        std::string out;
        for (const auto& c : cmds) {
            out += "*" + std::to_string(c.size()) + "\r\n";
            for (const auto& a : c) out += "$" + std::to_string(a.size()) + "\r\n" + a + "\r\n";
        }
        for (size_t p = 0; p < out.size();) {
            const ssize_t w = ::send(fd_, out.data() + p, out.size() - p, 0);
            if (w <= 0) throw std::runtime_error("redis: send failed");
            p += (size_t)w;
        }
        std::vector<Reply> r;
        r.reserve(cmds.size());
        for (size_t i = 0; i < cmds.size(); ++i) r.push_back(reply());
        return r;
    }

private:
    int fd_ = -1;
    std::string buf_;
    size_t pos_ = 0;
    void more() {
        char tmp[65536];
        const ssize_t n = ::recv(fd_, tmp, sizeof tmp, 0);
        if (n <= 0) throw std::runtime_error("redis: connection closed");
        buf_.erase(0, pos_);
        pos_ = 0;
        buf_.append(tmp, (size_t)n);
    }
    std::string line() {
        size_t e;
        while ((e = buf_.find("\r\n", pos_)) == std::string::npos) more();
        std::string s = buf_.substr(pos_, e - pos_);
        pos_ = e + 2;
        return s;
    }
    Reply reply() {
        const std::string ln = line();
        Reply r;
        if (ln.empty()) throw std::runtime_error("redis: empty reply");
        const std::string rest = ln.substr(1);
        switch (ln[0]) {
        case '+': r.str = rest; break;
        case '-': throw std::runtime_error("redis: " + rest);
        case ':': r.num = std::stoll(rest); break;
        case '$': {
            const long long n = std::stoll(rest);
            if (n < 0) { r.nil = true; break; }
            while (buf_.size() - pos_ < (size_t)n + 2) more();
            r.str = buf_.substr(pos_, (size_t)n);
            pos_ += (size_t)n + 2;
            break;
        }
        case '*': {
            const long long n = std::stoll(rest);
            for (long long i = 0; i < n; ++i) reply();   // not used by the writer
            break;
        }
        default: throw std::runtime_error("redis: bad reply " + ln);
        }
        return r;
    }
};

std::string randomUuid() {
    static thread_local std::mt19937_64 rng(std::random_device{}());
    const uint64_t hi = (rng() & ~0xF000ull) | 0x4000ull;                        // version 4
    const uint64_t lo = (rng() & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;   // IETF variant
    char b[40];
    std::snprintf(b, sizeof b, "%08llx-%04llx-%04llx-%04llx-%012llx", (unsigned long long)(hi >> 32),
                  (unsigned long long)((hi >> 16) & 0xFFFF), (unsigned long long)(hi & 0xFFFF),
                  (unsigned long long)(lo >> 48), (unsigned long long)(lo & 0xFFFFFFFFFFFFull));
    return b;
}

RedisWindowWriter::RedisWindowWriter(const std::string& host, int port) : r_(new RespClient(host, port)) {}
RedisWindowWriter::~RedisWindowWriter() = default;

void RedisWindowWriter::writeWindows(const std::vector<WindowDelta>& rows, int64_t nowMs) {
    // the (campaign, window) keys and campaigns not cached yet, each once, in first-seen
    // order (sets beside the vectors: a config-3 flush holds millions of rows)
    std::vector<std::pair<std::string, std::string>> need_w;
    std::vector<std::string> need_l;
    std::set<std::pair<std::string, std::string>> seen_w;
    std::set<std::string> seen_l;
    for (const WindowDelta& d : rows) {
        if (!d.count) continue;
        auto k = std::make_pair(d.campaign, std::to_string(d.windowMs));
        if (!windowUuid_.count(k) && seen_w.insert(k).second) {
            need_w.push_back(std::move(k));
            if (!listUuid_.count(d.campaign) && seen_l.insert(d.campaign).second) need_l.push_back(d.campaign);
        }
    }
    // round trip 1: the window / list UUIDs not cached yet (hmget campaign ts, :70)
    std::vector<std::vector<std::string>> reads;
    for (const auto& k : need_w) reads.push_back({"HGET", k.first, k.second});
    for (const auto& c : need_l) reads.push_back({"HGET", c, "windows"});
    std::vector<RespClient::Reply> got;
    if (!reads.empty()) {
        got = r_->pipeline(reads);
        ++trips_;
    }
    for (size_t i = 0; i < need_l.size(); ++i)
        if (!got[need_w.size() + i].nil) listUuid_[need_l[i]] = got[need_w.size() + i].str;
    std::vector<std::vector<std::string>> writes;
    for (size_t i = 0; i < need_w.size(); ++i) {
        if (!got[i].nil) {
            windowUuid_[need_w[i]] = got[i].str;
            continue;
        }
        const std::string w = randomUuid();                                          // :72-73
        windowUuid_[need_w[i]] = w;
        writes.push_back({"HSET", need_w[i].first, need_w[i].second, w});
        auto l = listUuid_.find(need_w[i].first);
        if (l == listUuid_.end()) {                                                  // :75-79
            l = listUuid_.emplace(need_w[i].first, randomUuid()).first;
            writes.push_back({"HSET", need_w[i].first, "windows", l->second});
        }
        writes.push_back({"LPUSH", l->second, need_w[i].second});                    // :80
    }
    // round trip 2: the deltas (:84, :87-88)
    const std::string now = std::to_string(
        nowMs >= 0 ? nowMs
                   : (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                         std::chrono::system_clock::now().time_since_epoch()).count());
    for (const WindowDelta& d : rows) {
        if (!d.count) continue;
        const std::string& w = windowUuid_[std::make_pair(d.campaign, std::to_string(d.windowMs))];
        writes.push_back({"HINCRBY", w, "seen_count", std::to_string(d.count)});
        writes.push_back({"HSET", w, "time_updated", now});
        writes.push_back({"LPUSH", "time_updated", now});
    }
    if (!writes.empty()) {
        r_->pipeline(writes);
        ++trips_;
    }
}

// ---- CSV sink --------------------------------------------------------------------------------------

void CsvWindowSink::add(const std::vector<WindowDelta>& rows) {
    for (const WindowDelta& d : rows) totals_[{d.campaign, d.windowMs}] += d.count;
}

void CsvWindowSink::write(const std::string& path) const {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fprintf(f, "campaign_id,window_ms,count\n");
    for (const auto& t : totals_)
        if (t.second)
            std::fprintf(f, "%s,%lld,%llu\n", t.first.first.c_str(), (long long)t.first.second,
                         (unsigned long long)t.second);
    std::fclose(f);
}

}  // namespace topology
}  // namespace ysb
