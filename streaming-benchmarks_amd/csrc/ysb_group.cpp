// ysb_group.cpp -- multi-GPU (the keyBy(0) shuffle, AdvertisingTopologyNative.java:118-119):
// the group over RCCL or the caller's host collectives, ring-base agreement, the
// range-limited (pipelined) reduce-scatter of the (campaign, window) tables and its
// checksums.
#include "ysb_ctx.h"

using namespace ysb;

extern "C" {

// The owned table's u8 accumulator into it (queued on the compute stream), cleared.
int fold_owned(ysb_ctx* c) {
    if (!c->d_owned8 || !c->owned8_dirty) return YSB_OK;
    launch_fold(c->d_owned, c->d_owned8, (u64)c->c_pad / (u64)c->nranks * c->cfg.window_ring, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->owned8_dirty = false;
    return YSB_OK;
}

bool grouped(const ysb_ctx* c) { return c->comm != nullptr || c->host_coll; }

// d[0..n) <- elementwise max over the ranks, in place: one RCCL all-reduce on the compute
// stream, or (host collectives) the buffer through host memory and the caller's all-reduce.
static int coll_max_u64(ysb_ctx* c, unsigned long long* d, u64 n) {
    if (c->comm) {
        ncclResult_t r = ncclAllReduce(d, d, n, ncclUint64, ncclMax, c->comm, c->s_comp);
        if (r != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
        return YSB_OK;
    }
    std::vector<uint64_t> h(n);
    HIPCHK(c, hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (c->hops.allreduce_max_u64(c->hops.user, h.data(), n))
        return fail(c, YSB_ERR_RCCL, "host all-reduce(max) failed");
    HIPCHK(c, hipMemcpyAsync(d, h.data(), n * 8, hipMemcpyHostToDevice, c->s_comp));
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    return YSB_OK;
}

// recv[0..count) <- sum over the ranks of their send blocks [rank * count, (rank + 1) * count),
// cells of `width` bytes (1, 4 or 8, unsigned).
static int coll_reduce_scatter(ysb_ctx* c, const void* d_send, void* d_recv, u64 count, u32 width, hipStream_t st) {
    if (c->comm) {
        const ncclDataType_t ty = width == 1 ? ncclUint8 : width == 4 ? ncclUint32 : ncclUint64;
        ncclResult_t r = ncclReduceScatter(d_send, d_recv, (size_t)count, ty, ncclSum, c->comm, st);
        if (r != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclReduceScatter: %s", ncclGetErrorString(r));
        return YSB_OK;
    }
    const u64 nb = count * width;
    std::vector<u8> hs(nb * (u64)c->nranks), hr(nb);
    HIPCHK(c, hipMemcpyAsync(hs.data(), d_send, hs.size(), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (c->hops.reduce_scatter_sum(c->hops.user, hs.data(), hr.data(), count, width))
        return fail(c, YSB_ERR_RCCL, "host reduce-scatter failed");
    HIPCHK(c, hipMemcpyAsync(d_recv, hr.data(), nb, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return YSB_OK;
}

// h[0..n) <- elementwise max over the ranks (signed: mapped to unsigned by the sign bit).
int allreduce_max(ysb_ctx* c, i64* h, int n) {
    unsigned long long* d = nullptr;
    HIPCHK(c, hipMalloc(&d, 8 * (u64)n));
    std::vector<u64> u(n);
    for (int i = 0; i < n; ++i) u[i] = (u64)h[i] ^ (1ull << 63);
    hipError_t e = hipMemcpy(d, u.data(), 8 * (u64)n, hipMemcpyHostToDevice);
    int rc = e == hipSuccess ? coll_max_u64(c, d, (u64)n) : YSB_OK;
    if (e == hipSuccess && !rc) e = hipMemcpyAsync(u.data(), d, 8 * (u64)n, hipMemcpyDeviceToHost, c->s_comp);
    if (e == hipSuccess && !rc) e = hipStreamSynchronize(c->s_comp);
    hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return fail(c, YSB_ERR_HIP, "%s", hipGetErrorString(e));
    for (int i = 0; i < n; ++i) h[i] = (i64)(u[i] ^ (1ull << 63));
    return YSB_OK;
}

// Ring-base agreement (collective: every rank calls it at the same point and takes the
// same decision from the reduced values, so no rank skips a collective the others
// enter).  The common base is the smallest base any rank holds.  A rank whose ring
// starts later moves the buckets the common range no longer holds, [common + W, lo + W),
// to its exact host-side list (cells are indexed by bucket mod W, so the rest stays in
// place); a rank without a base takes the common one.  Skewed per-rank streams
// (core.clj:166-174) that auto-based differently therefore still exchange.
int agree_ring(ysb_ctx* c) {
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    int rc = read_ring(c);
    if (rc) return rc;
    i64 h[2] = {c->ring_known ? -c->ring_lo : INT64_MIN + 1, c->ring_known ? 1 : 0};
    if ((rc = allreduce_max(c, h, 2))) return rc;
    if (!h[1]) return YSB_OK;   // no rank has a base yet: agreed at the next exchange
    if ((rc = move_ring(c, -h[0]))) return rc;
    c->ring_agreed = true;
    return YSB_OK;
}

int ysb_group_unique_id(uint8_t uid[YSB_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == YSB_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail(nullptr, YSB_ERR_RCCL, "ncclGetUniqueId failed");
    std::memcpy(uid, &id, sizeof id);
    return YSB_OK;
}

static int group_setup(ysb_ctx* c, int rank, int nranks);
static void ungroup(ysb_ctx* c);

int ysb_group_init(ysb_ctx* c, int rank, int nranks, const uint8_t uid[YSB_UNIQUE_ID_BYTES]) {
    if (!c || !uid) return YSB_ERR_ARG;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, YSB_ERR_ARG, "bad rank %d / %d", rank, nranks);
    if (grouped(c)) return fail(c, YSB_ERR_STATE, "group already initialised");
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return fail(c, YSB_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    const int rc = group_setup(c, rank, nranks);
    if (rc) ungroup(c);
    return rc;
}

int ysb_group_init_host(ysb_ctx* c, int rank, int nranks, const ysb_collectives* ops) {
    if (!c || !ops || !ops->allreduce_max_u64 || !ops->reduce_scatter_sum) return YSB_ERR_ARG;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, YSB_ERR_ARG, "bad rank %d / %d", rank, nranks);
    if (grouped(c)) return fail(c, YSB_ERR_STATE, "group already initialised");
    HIPCHK(c, hipSetDevice(c->device));
    c->hops = *ops;
    c->host_coll = true;
    const int rc = group_setup(c, rank, nranks);
    if (rc) ungroup(c);
    return rc;
}

// A failed group init leaves the context ungrouped (and a later ysb_group_init possible):
// the communicator, the exchange buffers and the owned table go; the counts stay.
static void ungroup(ysb_ctx* c) {
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->host_coll = false;
    c->hops = ysb_collectives{};
    hipFree(c->d_owned);
    c->d_owned = nullptr;
    hipFree(c->d_owned8);
    c->d_owned8 = nullptr;
    c->owned8_dirty = false;
    hipFree(c->d_xmax);
    c->d_xmax = nullptr;
    hipHostFree(c->h_xmax);
    c->h_xmax = nullptr;
    hipFree(c->d_xslots);
    c->d_xslots = nullptr;
    for (hipEvent_t& e : c->xplan_ev) {
        if (e) hipEventDestroy(e);
        e = nullptr;
    }
    for (int k = 0; k < 2; ++k) {
        if (c->ev_xpacked[k]) hipEventDestroy(c->ev_xpacked[k]);
        if (c->ev_xdone[k]) hipEventDestroy(c->ev_xdone[k]);
        c->ev_xpacked[k] = c->ev_xdone[k] = nullptr;
        c->xset_used[k] = false;
    }
    c->unpack_set = -1;
    c->rank = 0;
    c->nranks = 1;
    c->ring_agreed = false;
    c->x_have_plan = false;
}

static int group_setup(ysb_ctx* c, int rank, int nranks) {
    int prc = launch_pending_raw(c);
    if (prc) return prc;
    c->rank = rank;
    c->nranks = nranks;
    // pad campaigns to a multiple of nranks; keep the current counts
    const u32 cp = (c->cfg.n_campaigns + nranks - 1) / nranks * nranks;
    if (cp != c->c_pad) {
        int frc = fold_delta(c);   // the delta ring has the old layout: fold it, drop it
        if (frc) return frc;
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        hipFree(c->d_delta);
        c->d_delta = nullptr;
        c->delta_cells = 0;
        unsigned long long* old = c->d_counts;
        const u64 W = c->cfg.window_ring;
        c->d_counts = nullptr;
        HIPCHK(c, hipMalloc(&c->d_counts, (u64)cp * W * 8));
        HIPCHK(c, hipMemset(c->d_counts, 0, (u64)cp * W * 8));
        HIPCHK(c, hipMemcpy(c->d_counts, old, (u64)c->c_pad * W * 8, hipMemcpyDeviceToDevice));
        hipFree(old);
        if (c->d_truth) {   // the generator-truth table has the ring's layout: grow it too
            unsigned long long* ot = c->d_truth;
            c->d_truth = nullptr;
            HIPCHK(c, hipMalloc(&c->d_truth, (u64)cp * W * 8));
            HIPCHK(c, hipMemset(c->d_truth, 0, (u64)cp * W * 8));
            HIPCHK(c, hipMemcpy(c->d_truth, ot, (u64)c->c_pad * W * 8, hipMemcpyDeviceToDevice));
            hipFree(ot);
        }
        c->c_pad = cp;
    }
    const u64 per = (u64)c->c_pad / nranks * c->cfg.window_ring;
    HIPCHK(c, hipMalloc(&c->d_owned, per * 8));
    HIPCHK(c, hipMemset(c->d_owned, 0, per * 8));
    HIPCHK(c, hipMalloc(&c->d_owned8, per));
    HIPCHK(c, hipMemset(c->d_owned8, 0, per));
    const u32 W = c->cfg.window_ring;
    HIPCHK(c, hipMalloc(&c->d_xmax, 2 * (u64)W * 8));
    HIPCHK(c, hipHostMalloc(&c->h_xmax, 2 * ((u64)W * 8 + (u64)W * 4)));   // maxima, then the plans' slots
    HIPCHK(c, hipMalloc(&c->d_xslots, 2 * (u64)W * 4));
    for (hipEvent_t& e : c->xplan_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int k = 0; k < 2; ++k) {
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_xpacked[k], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_xdone[k], hipEventDisableTiming));
        c->xset_used[k] = false;
    }
    if (!c->s_x) HIPCHK(c, hipStreamCreateWithFlags(&c->s_x, hipStreamNonBlocking));
    c->x_have_plan = false;
    // every rank's ring must start at the same bucket (the tables are summed cell by
    // cell): agreed here if any rank already knows its base, else at the first exchange
    return agree_ring(c);
}

static int grow_bytes(ysb_ctx* c, void** buf, u64* have, u64 bytes) {
    if (*have >= bytes) return YSB_OK;
    HIPCHK(c, hipStreamSynchronize(c->s_comp));
    if (c->s_x) HIPCHK(c, hipStreamSynchronize(c->s_x));
    hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    const u64 b = std::max<u64>(bytes, 1ull << 16);
    HIPCHK(c, hipMalloc(buf, b));
    *have = b;
    return YSB_OK;
}

int ysb_exchange_plan(const uint64_t* slot_max, uint32_t W, uint32_t nranks, uint32_t* slots, uint32_t* n_slots,
                      uint32_t* width) {
    if (!slot_max || !slots || !n_slots || !width || nranks == 0 || W == 0) return YSB_ERR_ARG;
    u32 n = 0;
    u64 mx = 0;
    for (u32 s = 0; s < W; ++s)
        if (slot_max[s]) {
            slots[n++] = s;
            mx = std::max<u64>(mx, slot_max[s]);
        }
    // the narrowest cell whose sum over the ranks cannot wrap: nranks * max < 2^(8 width)
    // (RCCL has no 16-bit integer type)
    const unsigned __int128 bound = (unsigned __int128)mx * nranks;
    *width = bound <= 0xFFu ? 1u : bound <= 0xFFFFFFFFull ? 4u : 8u;
    if (bound > ~0ull) return YSB_ERR_CAPACITY;
    *n_slots = n;
    return YSB_OK;
}

// The keyBy(0) exchange (AdvertisingTopologyNative.java:118-119), range-limited: only the
// ring slots that hold a pending count on some rank travel, in the narrowest cell width
// that cannot wrap, as the reference's keyed shuffle carries only the touched (campaign,
// window) pairs.  Steps on the compute stream: per-slot maxima of the pending counts
// (xplan) -> one W-element all-reduce(max) -> read back -> plan (ysb_exchange_plan: the
// same on every rank) -> pack the slots' cells [C_pad][R] and zero them (xpack) ->
// ncclReduceScatter -> add the owner block into the owned table (xunpack).
//
// Complete (pipelined false): the plan is this call's, read back with a host wait; every
// pending count travels.  Pipelined: this call's plan is only enqueued (reduced into the
// other buffer, read back by an async copy) and the pack uses the previous call's plan,
// whose read-back finished while the step's scan ran -- no host wait, so the next launch
// queues behind the exchange without a gap.  Counts in slots outside that plan, or above
// what its width sums over the ranks (cap), stay pending for a later exchange; the first
// call after group init / reset / ring advance is complete.
// The recorded exchange timing pairs into x_ms (waits for the last of them).
// The unpack of the last exchange (owner block += received cells), on the compute stream
// once its reduce-scatter is done; a no-op when none is pending.
int finish_unpack(ysb_ctx* c) {
    if (c->unpack_set < 0) return YSB_OK;
    const int k = c->unpack_set;
    c->unpack_set = -1;
    const u32 W = c->cfg.window_ring, per = c->c_pad / (u32)c->nranks;
    const auto& ev = c->xev[c->unpack_entry];
    HIPCHK(c, hipEventRecord(ev[5], c->s_comp));   // ev[5] -> ev[3]: the compute stream's wait
    HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_xdone[k], 0));
    HIPCHK(c, hipEventRecord(ev[3], c->s_comp));
    launch_xunpack(c->d_owned, c->d_owned8, W, per, c->d_xslots + (u64)k * W, c->unpack_R, c->d_xrecv[k],
                   c->unpack_width, c->s_comp);
    HIPCHK(c, hipGetLastError());
    c->owned8_dirty = true;
    HIPCHK(c, hipEventRecord(ev[4], c->s_comp));
    return YSB_OK;
}

// The recorded exchange timing into x_ms (plan to the end of the reduce-scatter, plus the
// unpack), x_crit_ms (the compute stream's share: plan to pack, plus the unpack), x_rs_ms
// (pack done to reduce-scatter done, on the exchange stream) and x_exposed_ms (how long the
// compute stream stood at the unpack's wait for that reduce-scatter: the part of it the
// launches queued since did not hide; a complete exchange exposes all of it).  Call
// after finish_unpack.  wait: every entry, waiting for the last of them (an info request);
// otherwise only the entries whose events have completed -- the rest stay pending, so the
// host never waits behind the launches it has queued (the pipelined exchange's periodic fold).
static int collect_xev(ysb_ctx* c, bool wait) {
    size_t keep = 0;
    for (size_t i = 0; i < c->xev_used; ++i) {
        const auto& ev = c->xev[i];
        if (!wait && (hipEventQuery(ev[2]) != hipSuccess || hipEventQuery(ev[4]) != hipSuccess)) {
            std::swap(c->xev[keep++], c->xev[i]);   // pending entries keep their order
            continue;
        }
        float ms = 0, mc = 0, mu = 0, mr = 0, mx = 0;
        HIPCHK(c, hipEventSynchronize(ev[2]));
        HIPCHK(c, hipEventSynchronize(ev[4]));
        HIPCHK(c, hipEventElapsedTime(&ms, ev[0], ev[2]));
        HIPCHK(c, hipEventElapsedTime(&mc, ev[0], ev[1]));
        HIPCHK(c, hipEventElapsedTime(&mu, ev[3], ev[4]));
        HIPCHK(c, hipEventElapsedTime(&mr, ev[1], ev[2]));
        HIPCHK(c, hipEventElapsedTime(&mx, ev[5], ev[3]));
        c->x_ms += ms + mu;
        c->x_crit_ms += mc + mu;
        c->x_rs_ms += mr;
        c->x_exposed_ms += mx;
    }
    c->xev_used = keep;
    return YSB_OK;
}

// The plan's ascending slot list widened to whole aligned groups of four: every run of
// consecutive slots grows to [floor4(first), ceil4(last + 1)) (W is a power of two >= 16, so
// the groups never pass W), so the u8 pack / unpack move each group as one u32 of the ring
// (ysb_table.hip xpack8_kernel: a group that is not four consecutive aligned slots takes
// per-cell steps).  An added slot held no pending count anywhere when the plan was made: it
// sends zeros -- or, in a pipelined exchange whose plan is one call old, a count that arrived
// since, within the width's cap like any planned slot.  At most three extra slots per run
// end.  In place (the list has W entries); returns the new length, a multiple of 4.
static u32 align_slot_runs(u32* slots, u32 R, u32 W) {
    std::vector<u32> out;
    out.reserve(R + 8);
    for (u32 i = 0; i < R;) {
        u32 j = i + 1;
        while (j < R && slots[j] == slots[j - 1] + 1) ++j;
        const u32 a = slots[i] & ~3u, b = std::min<u32>((slots[j - 1] + 4) & ~3u, W);
        for (u32 sl = std::max<u32>(a, out.empty() ? 0u : out.back() + 1); sl < b; ++sl) out.push_back(sl);
        i = j;
    }
    std::copy(out.begin(), out.end(), slots);
    return (u32)out.size();
}

static int exchange(ysb_ctx* c, bool pipelined) {
    if (!grouped(c)) return fail(c, YSB_ERR_STATE, "ysb_group_init has not been called");
    int prc = launch_pending_raw(c);
    if (!prc) prc = finish_unpack(c);   // the previous (pipelined) exchange's owner block first
    if (prc) return prc;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->ring_agreed) {
        int rc = agree_ring(c);
        if (rc) return rc;
    }
    if (!c->x_have_plan) pipelined = false;
    const u32 W = c->cfg.window_ring;
    const u64 cells = (u64)c->c_pad * W;
    const u8* delta = c->delta_bound ? c->d_delta : nullptr;   // (delta_bound 0: the delta ring is all zero)
    // timing pairs: folded into x_ms once XEV_KEEP are pending (a streaming caller may never
    // ask for ysb_group_exchange_info); a pair counts only once both events were recorded
    int urc = YSB_OK;
    if (c->xev_used >= XEV_KEEP) {
        int rc = collect_xev(c, false);
        if (rc) return rc;
    }
    if (c->xev_used == c->xev.size()) {
        std::array<hipEvent_t, 6> ev{};
        for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
        c->xev.push_back(ev);
    }
    const auto ev = c->xev[c->xev_used];
    HIPCHK(c, hipEventRecord(ev[0], c->s_comp));
    // this call's plan into buffer nb
    const int nb = c->xb ^ 1;
    unsigned long long* dmax = c->d_xmax + (u64)nb * W;
    unsigned long long* hmax = c->h_xmax + (u64)nb * W;
    HIPCHK(c, hipMemsetAsync(dmax, 0, (u64)W * 8, c->s_comp));
    launch_xplan(c->d_counts, delta, W, cells, c->pend_u64 ? 1 : 0, c->d_dirty, dmax, c->s_comp);
    HIPCHK(c, hipGetLastError());
    int crc = coll_max_u64(c, dmax, W);
    if (crc) return crc;
    HIPCHK(c, hipMemcpyAsync(hmax, dmax, (u64)W * 8, hipMemcpyDeviceToHost, c->s_comp));
    HIPCHK(c, hipEventRecord(c->xplan_ev[nb], c->s_comp));
    // the plan the pack uses: this one (complete) or the previous call's (pipelined)
    const int pb = pipelined ? c->xb : nb;
    HIPCHK(c, hipEventSynchronize(c->xplan_ev[pb]));
    c->xb = nb;
    c->x_have_plan = true;
    u32* slots = reinterpret_cast<u32*>(c->h_xmax + 2 * (u64)W) + (u64)pb * W;
    u32 R = 0, width = 8;
    if (ysb_exchange_plan(reinterpret_cast<const uint64_t*>(c->h_xmax + (u64)pb * W), W, (u32)c->nranks, slots, &R,
                          &width))
        return fail(c, YSB_ERR_CAPACITY, "pending counts too large to sum over %d ranks", c->nranks);
    const unsigned long long cap = width == 8 ? ~0ull / (u64)c->nranks : ((1ull << (8 * width)) - 1) / (u64)c->nranks;
    const u32 rows = c->c_pad, per = c->c_pad / (u32)c->nranks;
    const u32 nslots = R;
    R = align_slot_runs(slots, R, W);
    if (R) {
        const int k = c->xk;
        c->xk ^= 1;
        // set k was last used two exchanges ago: its unpack must be done before it is rewritten
        if (c->xset_used[k]) HIPCHK(c, hipStreamWaitEvent(c->s_comp, c->ev_xdone[k], 0));
        int rc = grow_bytes(c, &c->d_xsend[k], &c->xsend_bytes[k], (u64)rows * R * width);
        if (!rc) rc = grow_bytes(c, &c->d_xrecv[k], &c->xrecv_bytes[k], (u64)per * R * width);
        if (rc) return rc;
        u32* dslots = c->d_xslots + (u64)k * W;
        // (the slots' pinned area is rewritten two calls later, after xplan_ev of the call
        // in between: this copy has run by then)
        HIPCHK(c, hipMemcpyAsync(dslots, slots, (u64)R * 4, hipMemcpyHostToDevice, c->s_comp));
        launch_xpack(c->d_counts, delta ? c->d_delta : nullptr, W, rows, dslots, R, c->pend_u64 ? 1 : 0,
                     c->d_dirty, c->d_xsend[k], width, pipelined ? cap : ~0ull, c->s_comp);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev_xpacked[k], c->s_comp));
        // the transfer on the exchange stream, beside the next launch; the unpack follows on
        // the compute stream (finish_unpack)
        HIPCHK(c, hipStreamWaitEvent(c->s_x, c->ev_xpacked[k], 0));
        if ((rc = coll_reduce_scatter(c, c->d_xsend[k], c->d_xrecv[k], (u64)per * R, width, c->s_x))) return rc;
        HIPCHK(c, hipEventRecord(c->ev_xdone[k], c->s_x));
        c->xset_used[k] = true;
        c->unpack_set = k;
        c->unpack_R = R;
        c->unpack_width = width;
        c->unpack_entry = c->xev_used;
    }
    if (!pipelined) {
        // every pending count sat in an exchanged slot: nothing is pending any more
        HIPCHK(c, hipMemsetAsync(c->d_dirty, 0, 4, c->s_comp));
        c->pend_u64 = false;
        c->delta_bound = 0;
    }
    HIPCHK(c, hipEventRecord(ev[1], c->s_comp));
    HIPCHK(c, hipEventRecord(ev[2], R ? c->s_x : c->s_comp));
    if (!R) {   // nothing to unpack: an empty unpack interval, no wait
        HIPCHK(c, hipEventRecord(ev[5], c->s_comp));
        HIPCHK(c, hipEventRecord(ev[3], c->s_comp));
        HIPCHK(c, hipEventRecord(ev[4], c->s_comp));
    }
    c->xev_used++;
    // complete: the owners' tables hold everything once the call's work has run
    if (!pipelined && (urc = finish_unpack(c))) return urc;
    c->x_count++;
    c->x_bytes += (u64)rows * R * width;
    c->x_last_slots = nslots;
    c->x_last_width = R ? width : 0;
    return YSB_OK;
}

int ysb_group_reduce_scatter(ysb_ctx* c) { return c ? exchange(c, false) : YSB_ERR_ARG; }

int ysb_group_exchange_pipelined(ysb_ctx* c) { return c ? exchange(c, true) : YSB_ERR_ARG; }

uint64_t ysb_exchange_info_size(void) { return sizeof(ysb_exchange_info); }

int ysb_group_exchange_info(ysb_ctx* c, ysb_exchange_info* out, int reset) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    int rc = sync_streams(c);
    if (!rc) rc = collect_xev(c, true);
    if (rc) return rc;
    out->exchanges = c->x_count;
    out->bytes = c->x_bytes;
    out->ms = c->x_ms;
    out->critical_ms = c->x_crit_ms;
    out->rs_ms = c->x_rs_ms;
    out->exposed_ms = c->x_exposed_ms;
    out->last_buckets = c->x_last_slots;
    out->last_width = c->x_last_width;
    out->full_ring_bytes = (u64)c->c_pad * c->cfg.window_ring * 8;
    if (reset) {
        c->x_count = 0;
        c->x_bytes = 0;
        c->x_ms = 0;
        c->x_crit_ms = 0;
        c->x_rs_ms = 0;
        c->x_exposed_ms = 0;
    }
    return YSB_OK;
}

int ysb_group_checksum(ysb_ctx* c, int what, uint32_t nranks, uint64_t* out) {
    if (!c || !out) return c ? fail(c, YSB_ERR_ARG, "NULL output") : YSB_ERR_ARG;
    if (nranks == 0) return fail(c, YSB_ERR_ARG, "nranks must be >= 1");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = launch_pending_raw(c);
    if (!rc) rc = fold_delta(c);   // the checksums read the u64 ring
    if (!rc) rc = sync_streams(c);
    if (!rc) rc = read_ring(c);
    if (rc) return rc;
    if (!c->ring_known) return fail(c, YSB_ERR_STATE, "ring base not set yet");
    const u32 W = c->cfg.window_ring, C = c->cfg.n_campaigns;
    if (!c->d_cmp) HIPCHK(c, hipMalloc(&c->d_cmp, 32));
    unsigned long long* acc = c->d_cmp;
    auto sum = [&](const unsigned long long* t, u32 rows, u32 c_off, u32 lo, u32 hi, uint64_t* o) -> int {
        HIPCHK(c, hipMemsetAsync(acc, 0, 8, c->s_comp));
        launch_checksum(t, rows, W, c->ring_lo, c_off, lo, hi, acc, c->s_comp);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(o, acc, 8, hipMemcpyDeviceToHost, c->s_comp));
        HIPCHK(c, hipStreamSynchronize(c->s_comp));
        return YSB_OK;
    };
    if (what == YSB_SUM_TRUTH_BLOCKS || what == YSB_SUM_PENDING_BLOCKS) {
        const unsigned long long* t = what == YSB_SUM_TRUTH_BLOCKS ? c->d_truth : c->d_counts;
        if (!t) return fail(c, YSB_ERR_STATE, "no truth accumulated");
        for (u32 r = 0; r < nranks; ++r) {
            u32 lo = 0, hi = 0;
            ysb_group_block(C, (int)r, (int)nranks, &lo, &hi);
            if ((rc = sum(t, c->c_pad, 0, lo, hi, &out[r]))) return rc;
        }
        return YSB_OK;
    }
    if (what == YSB_SUM_OWNED) {
        if (!c->d_owned) { out[0] = 0; return YSB_OK; }
        u32 lo = 0, hi = 0;
        ysb_group_block(C, c->rank, c->nranks, &lo, &hi);
        const u32 per = c->c_pad / (u32)c->nranks;   // row i of the owned table: campaign rank * per + i
        if ((rc = fold_owned(c))) return rc;
        return sum(c->d_owned, per, (u32)c->rank * per, lo, hi, &out[0]);
    }
    return fail(c, YSB_ERR_ARG, "unknown checksum %d", what);
}

int ysb_group_info(ysb_ctx* c, int* rank, int* nranks) {
    if (!c) return YSB_ERR_ARG;
    if (!grouped(c)) return fail(c, YSB_ERR_STATE, "ysb_group_init has not been called");
    if (c->host_coll) {   // the caller's collectives: the ranks it declared
        if (rank) *rank = c->rank;
        if (nranks) *nranks = c->nranks;
        return YSB_OK;
    }
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(c->comm, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
    if (e != ncclSuccess) return fail(c, YSB_ERR_RCCL, "ncclCommCount: %s", ncclGetErrorString(e));
    if (rank) *rank = r;
    if (nranks) *nranks = n;
    return YSB_OK;
}

int ysb_group_owned(ysb_ctx* c, uint32_t* lo, uint32_t* hi) {
    if (!c) return YSB_ERR_ARG;
    const u32 per = c->c_pad / c->nranks;
    const u32 l = std::min<u32>(c->cfg.n_campaigns, (u32)c->rank * per);
    if (lo) *lo = l;
    if (hi) *hi = std::min<u32>(c->cfg.n_campaigns, l + per);
    return YSB_OK;
}

uint32_t ysb_ad_shard(const char* ad_id, uint32_t len, uint32_t nranks) {
    if (nranks <= 1) return 0;
    u32 kw[KEY_WORDS] = {0};
    std::memcpy(kw, ad_id, std::min<u32>(len, MAX_KEY_BYTES));
    const u32 h = key_hash(kw, std::min<u32>(len, MAX_KEY_BYTES));
    return (u32)(((u64)mix64(h) >> 32) * nranks >> 32);
}

}  // extern "C"
