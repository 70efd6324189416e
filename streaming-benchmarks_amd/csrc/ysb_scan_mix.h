// ysb_scan_mix.h -- Kernel 1m (round 5): the scan for batches whose producers interleave line
// by line (layout 2 with LDS window counters).  Part of the scan kernel's translation unit:
// included by ysb_scan.hip after scan_kernel, whose device functions it reuses.
//
// In layout 2 every 64-line tile mixes four producers, so each lane's walk through the flat
// tier diverges from its neighbours' at every pair, and the wave pays for every branch any
// lane takes.  Here a four-wave workgroup stages four consecutive tiles (256 lines) into LDS,
// classes every line by its first 12 bytes (the generator's `{"user_id": `, compact
// `{"user_id":"`, anything else), and re-deals the lines so that each wave takes 64 lines
// sorted by class.  A wave then runs, for each class present among its lanes, that class's
// own path with only those lanes active: the generator's vocabulary path (then its canonical
// tier), compact JSON's, the learned order (when the sample learned one).  Any lane a path
// rejects, and the third class without a learned order, takes the flat tier.  Most waves
// hold one class and run one uniform path; a wave at a class boundary runs two.  The counts,
// the deferred lines and every decision are the scan kernel's: the same parse functions on
// the same staged bytes, only the lane a line lands on changes.
#pragma once

// (included inside namespace ysb)

// The workgroup barrier the step needs: every wave's LDS writes visible to the others, with
// no wait for global loads -- __syncthreads() is also a global fence (s_waitcnt vmcnt(0)),
// which would expose the next tile's prefetch at every step.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr int MIX_WAVES = YSB_MIX_WAVES;
constexpr int MIX_TPB = 64 * MIX_WAVES;

// LDS carve: four tiles (each with the 64-B read slack), the window counters, the misc
// words, the run's tile bounds, the dealt lines, the class counts and the key table.
struct GeomMix {
    static constexpr int WG_PER_CU = MIX_WG_PER_CU;
    static constexpr int CAP = TILE_CAP;
    static constexpr int CPT = (CAP / 16 + 63) / 64;                  // 16-byte chunks per lane
    static constexpr int TILE_STRIDE = CAP + 64;
    static constexpr int OFF_TILE = 0;
    static constexpr int OFF_LCNT = MIX_WAVES * TILE_STRIDE;
    static constexpr int OFF_MISC = OFF_LCNT + LCNT_CAP * 4;         // [0..1] window requests, [2] claim
    static constexpr int OFF_TB = OFF_MISC + 64;
    static constexpr int OFF_DEAL = OFF_TB + (MIX_MAX_TILES + 4) * 4;   // uint4 per line
    static constexpr int OFF_CNT = OFF_DEAL + MIX_TPB * 16;          // u32 [wave][8]: class counts
    static constexpr int OFF_KT = OFF_CNT + MIX_WAVES * 8 * 4;
    static constexpr int LDS = OFF_KT + KEYTAB_BYTES;
    static_assert(TILE_STRIDE % 16 == 0 && OFF_LCNT % 16 == 0 && OFF_DEAL % 16 == 0 && OFF_KT % 16 == 0,
                  "LDS carve must stay 16-byte aligned");
    static constexpr int LDS_ALLOC = (LDS + 1279) / 1280 * 1280;
    static_assert(LDS_ALLOC * WG_PER_CU <= 163840, "MIX_WG_PER_CU multi-wave workgroups must fit one CU's LDS");
};

// The line classes (the order in which lines are dealt): 1 the generator's layout, 2 compact
// JSON, 3 anything else, 4 a line to defer without a parse (offsets outside its tile), 5 no line.
constexpr u32 MIX_CLASSES = 6;

// issue_tile_loads for one wave of a multi-wave workgroup: chunk j * 64 + lane of the tile,
// lane's own line's offsets (line = lane).
template <int CPT>
__device__ __forceinline__ void mix_tile_loads(const ScanParams& P, const TileInfo& ti, uint4 (&pre)[CPT], u32& my_off,
                                               u32& my_end, int lane) {
    const u8* tbase = P.bytes + (ti.s0 - ti.delta);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(tbase), 0, (int)((ti.len + 15u) & ~15u), 0x00020000);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * (j * 64 + lane), 0, AUX_NT);
        pre[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    const u64 left = P.n - min(ti.first, P.n);
    const u32 nrec = (u32)min<u64>((u64)ti.count + 1u, left) * 4u;
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u32*>(P.off + min(ti.first, P.n)), 0, (int)nrec, 0x00020000);
    my_off = __builtin_amdgcn_raw_buffer_load_b32(ro, 4 * lane, 0, 0);
    my_end = __builtin_amdgcn_raw_buffer_load_b32(ro, 4 * lane + 4, 0, 0);
}

template <bool SERIAL>
__global__ __launch_bounds__(MIX_TPB) __attribute__((amdgpu_waves_per_eu(2))) void mix_scan_kernel(const ScanParams P0) {
    using G = GeomMix;
    constexpr int CPT = G::CPT;
    extern __shared__ __attribute__((aligned(16))) u8 smem[];
    u32* tile32 = reinterpret_cast<u32*>(smem + G::OFF_TILE);
    u32* lcnt = reinterpret_cast<u32*>(smem + G::OFF_LCNT);
    i64* misc64 = reinterpret_cast<i64*>(smem + G::OFF_MISC);
    u32* tb = reinterpret_cast<u32*>(smem + G::OFF_TB);
    uint4* deal = reinterpret_cast<uint4*>(smem + G::OFF_DEAL);
    u32* cnt = reinterpret_cast<u32*>(smem + G::OFF_CNT);
    u32* keytab = reinterpret_cast<u32*>(smem + G::OFF_KT);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    ScanParams P = P0;
    const i64 ring_lo = P.ring[0];
    const bool ring_set = P.ring[1] != 0;
    const u32 WL = P.lds_wl;
    const u32 ncells = WL ? P.n_campaigns * WL : 0u;
    for (u32 i = tid; i < ncells; i += MIX_TPB) lcnt[i] = 0;
    if (tid < 2) misc64[tid] = INT64_MIN;
    if (tid < 64) keytab[tid] = KEYTAB.w[tid];

    Tally tl{0, 0, 0, 0, 0, 0, 0, 0};
    u64 t_begin = 0, t_end = 0, n_run = 0;
    TileInfo none{0, 0u, 0u, 0u, 0u, 0u, true};
    uint4 pre[CPT];
    u32 pre_off = 0, pre_end = 0;
    TileInfo inf = none;
    u32 tseq = 0;
    i64 lbase = 0;
    bool lset = false;
    const LdsSrc lsrc{tile32};
    const uint4* ct4 = reinterpret_cast<const uint4*>(P.ctable);
    // static priority for every other workgroup, as scan_kernel (two waves per SIMD)
    if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);

    // One step: this wave's tile t of the run's four (its bytes in pre since the step before).
    auto mix_step = [&](u64 t0) __attribute__((always_inline)) {
        const TileInfo cur = inf;
        const u32 my_off = pre_off;
        const u32 li = (u32)lane;
        const u32 my_end = (cur.first + li + 1 < P.n) ? pre_end : (u32)P.nbytes;
        const int tbase = wave * G::TILE_STRIDE;
        // ---- Phase A: registers -> this wave's tile in LDS -------------------------------
        if (!cur.oversize) {
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
                const u32 k = (u32)(j * 64 + lane);
                if (j * 64 + 64 <= G::CAP / 16 || k < (u32)(G::CAP / 16))
                    reinterpret_cast<uint4*>(tile32 + tbase / 4)[k] = pre[j];
            }
        }
        const int par = (int)(tseq++ & 1);
        if (WL) {
            const i64 req = misc64[par ^ 1];
            if (req != INT64_MIN) {
                if (lset) {
                    for (u32 i = tid; i < ncells; i += MIX_TPB) {   // flush_window over the workgroup
                        const u32 v = lcnt[i];
                        if (v) {
                            lcnt[i] = 0;
                            global_add(P, ring_lo, ring_set, i >> P.lds_wl_log2, lbase + (i64)(i & (WL - 1)), v, tl);
                        }
                    }
                }
                lbase = req - (i64)(WL / 2) + 1;
                lset = true;
            }
        }
        // ---- the line's class, then the deal: lines sorted by class over the four waves --
        // (a wave classes only the tile it staged itself: its own LDS writes are in order,
        // no barrier before; the one after the counts also publishes the four tiles)
        const bool has = li < cur.count;
        const bool elig = has && !cur.oversize && my_off >= cur.s0 && my_end >= my_off && my_end <= cur.e;
        const int ls0 = tbase + (int)(my_off - cur.s0 + cur.delta);
        const int le0 = tbase + (int)(my_end - cur.s0 + cur.delta);
        u32 cls = has ? 4u : 5u;
        if (elig) {
            const u32 h2 = lsrc.load4(ls0 + 8);
            const bool up = lsrc.load4(ls0) == w4('{', '"', 'u', 's') && lsrc.load4(ls0 + 4) == w4('e', 'r', '_', 'i') &&
                            (h2 & 0xFFFFFFu) == (w4('d', '"', ':', 0) & 0xFFFFFFu);
            cls = up && (h2 >> 24) == ' ' ? 1u : up && (h2 >> 24) == '"' ? 2u : 3u;
        }
        u64 mine = 0;
#pragma unroll
        for (u32 k = 1; k < MIX_CLASSES; ++k) {
            const u64 m = __ballot(cls == k);
            if (cls == k) mine = m;
            if (lane == 0) cnt[wave * 8 + k] = (u32)__popcll(m);
        }
        lds_barrier();
        if (tid == 0) misc64[par ^ 1] = INT64_MIN;   // every thread has read the request
        // position: every line of a lower class, then this class's lines in lower waves, then
        // the lanes below this one in the wave
        u32 pos = __builtin_amdgcn_mbcnt_hi((u32)(mine >> 32), __builtin_amdgcn_mbcnt_lo((u32)mine, 0u));
#pragma unroll
        for (u32 k = 1; k < MIX_CLASSES; ++k) {
#pragma unroll
            for (int w = 0; w < MIX_WAVES; ++w) {
                const u32 c = cnt[w * 8 + k];
                pos += (k < cls || (k == cls && w < wave)) ? c : 0u;
            }
        }
#ifdef YSB_MIX_NODEAL   // diagnostic: every line stays on its own lane (the deal's cost alone)
        pos = (u32)tid;
#endif
        deal[pos] = make_uint4((u32)ls0, (u32)le0, (u32)(P.line_base + cur.first + li), cls);
        lds_barrier();
        // (a wave's 64 dealt lines interleaved over its lanes as scan_kernel's lane_line does:
        // a 32-lane half takes every other line, so the lines' start banks spread)
        const uint4 d = deal[wave * 64 + (int)lane_line(lane)];
        const int ls = (int)d.x, le = (int)d.y;
        const u32 line = d.z;
        const u32 dc = d.w;   // the dealt line's class
        // ---- Phase B1: each class present in the wave through its own path ----------------
        CanonA ca;
#pragma unroll
        for (int k = 0; k < 9; ++k) ca.kw[k] = 0u;
        ca.t0 = 0;
        CanonB cb;
        cb.view = false;
        bool ok2 = false;
        // (the scan kernel's tiers in the same order, each from fresh state as there: the
        // vocabulary path on the zeroed ca, a canonical tier or the flat tier on new ones)
        if (__ballot(dc == 1u) && dc == 1u) {   // the generator's layout: vocabulary path, then its canonical tier
            ok2 = vocab_stage1<false>(lsrc, ls, le, ca) && vocab_stage2<false>(lsrc, ls, le, ca, cb);
            if (!ok2) {
                CanonA a2;
                CanonB b2;
                b2.view = false;
                if (canon_stage1<false>(lsrc, ls, le, a2) && canon_stage2<false>(lsrc, ls, le, a2, b2)) {
                    ca = a2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        if (__ballot(dc == 2u) && dc == 2u) {   // compact JSON: its vocabulary path, then its canonical tier
            ok2 = vocab_stage1<true>(lsrc, ls, le, ca) && vocab_stage2<true>(lsrc, ls, le, ca, cb);
            if (!ok2) {
                CanonA a2;
                CanonB b2;
                b2.view = false;
                if (canon_stage1<true>(lsrc, ls, le, a2) && canon_stage2<true>(lsrc, ls, le, a2, b2)) {
                    ca = a2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        if (P.learn_n && __ballot(dc == 3u) && dc == 3u)   // another producer: the sample's learned order
            ok2 = P.learn_cp ? learned_parse<true>(lsrc, ls, le, P, ca, cb) : learned_parse<false>(lsrc, ls, le, P, ca, cb);
        // every eligible line no path took: the flat tier (any key order or spacing)
        const bool fl = dc <= 3u && !ok2;
        if (__ballot(fl)) {
            if (fl) {
                CanonA a2;
                CanonB b2;
                b2.view = false;
                if (flat_tier<LdsSrc, true>(lsrc, ls, le, P.require_mask, a2, b2, keytab)) {
                    ca = a2;
                    cb = b2;
                    ok2 = true;
                }
            }
        }
        const bool dfr = dc <= 4u && !ok2;   // bad offsets, escapes, other forms: Kernel 1b
        const bool pend = ok2 && cb.view;    // EventFilterBolt
        bool tok = false;
        i64 bucket = 0;
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0, a2 = a0, b0 = a0, b1 = a0, b2 = a0;
        uint4 q[CB_Q];
#pragma unroll
        for (int j = 0; j < (int)CB_Q; ++j) q[j] = a0;
        u32 ib_s = 0;
        if (pend) {   // RedisJoinBolt's lookup, as scan_kernel issues it
            u32 ia, ib;
            cuckoo_slots36(ca.kw, P.cseed, P.ctable_mask, &ia, &ib);
            if constexpr (SERIAL) {
#pragma unroll
                for (int j = 0; j < (int)CB_Q; ++j) q[j] = ct4[CB_Q * (u64)ia + j];
                ib_s = ib;
            } else {
                a0 = ct4[CSLOT_Q * (u64)ia]; a1 = ct4[CSLOT_Q * (u64)ia + 1]; a2 = ct4[CSLOT_Q * (u64)ia + 2];
                b0 = ct4[CSLOT_Q * (u64)ib]; b1 = ct4[CSLOT_Q * (u64)ib + 1]; b2 = ct4[CSLOT_Q * (u64)ib + 2];
            }
        }
        if (ok2) {
            tl.ev++;
            if (pend) {
                tl.view++;
                tok = canonical_bucket<false>(lsrc, cb, ls + ca.t0, P, bucket);   // Long.parseLong
            }
        }
        defer_append(P, dfr, line, lane);
        // ---- prefetch this wave's tile of the next step ------------------------------------
        const u64 tn = t0 + MIX_WAVES + (u64)wave;
        inf = tn < t_end ? tile_info<G::CAP>(P, tn, t_begin, tb) : none;
        mix_tile_loads(P, inf, pre, pre_off, pre_end, lane);
        // ---- Phase B2: join result, count ------------------------------------------------
        bool valid = false, dfr2 = false;
        u32 campaign = 0;
        if (pend) {
            const u32* k = ca.kw;
            u32 ci;
            if constexpr (SERIAL) {
                bool full;
                ci = bucket_find(q, k, full);
                if (ci == EMPTY_SLOT && full) {
#pragma unroll
                    for (int j = 0; j < (int)CB_Q; ++j) q[j] = ct4[CB_Q * (u64)ib_s + j];
                    ci = bucket_find(q, k, full);
                }
            } else {
                const u32 da = (a0.x ^ k[0]) | (a0.y ^ k[1]) | (a0.z ^ k[2]) | (a0.w ^ k[3]) | (a1.x ^ k[4]) |
                               (a1.y ^ k[5]) | (a1.z ^ k[6]) | (a1.w ^ k[7]) | (a2.x ^ k[8]);
                const u32 db = (b0.x ^ k[0]) | (b0.y ^ k[1]) | (b0.z ^ k[2]) | (b0.w ^ k[3]) | (b1.x ^ k[4]) |
                               (b1.y ^ k[5]) | (b1.z ^ k[6]) | (b1.w ^ k[7]) | (b2.x ^ k[8]);
                ci = (da == 0u && a2.y != EMPTY_SLOT) ? a2.y : (db == 0u ? b2.y : EMPTY_SLOT);
            }
            if (ci == EMPTY_SLOT) {
                if (P.ctable_partial) {
                    dfr2 = true;
                    tl.ev--;
                    tl.view--;
                } else {
                    tl.miss++;
                }
            } else {
                tl.join++;
                campaign = ci;
                valid = tok;
                if (!tok) tl.terr++;
            }
        }
        if (P.ctable_partial) defer_append(P, dfr2, line, lane);
        if (valid) {
            const i64 rel = bucket - lbase;
            if (lset && rel >= 0 && rel < (i64)WL) {
                atomicAdd(&lcnt[(campaign << P.lds_wl_log2) + (u32)rel], 1u);
            } else {
                global_add(P, ring_lo, ring_set, campaign, bucket, 1u, tl);
                if (!lset || rel >= (i64)WL) atomicMax(reinterpret_cast<long long*>(&misc64[par]), (long long)bucket);
            }
        }
        lds_barrier();
    };
    auto run_tiles = [&]() __attribute__((always_inline)) {
        n_run += t_end - t_begin;
        for (u32 i = tid; i <= (u32)(t_end - t_begin); i += MIX_TPB) {
            const u64 f = (t_begin + i) * TILE_LINES;
            tb[i] = f < P.n ? P.off[f] : (u32)P.nbytes;
        }
        lds_barrier();
        const u64 tw = t_begin + (u64)wave;
        inf = tw < t_end ? tile_info<G::CAP>(P, tw, t_begin, tb) : none;
        mix_tile_loads(P, inf, pre, pre_off, pre_end, lane);
        for (u64 t0 = t_begin; t0 < t_end; t0 += MIX_WAVES) mix_step(t0);
    };
    auto use_segment = [&](const ScanSeg& sg) __attribute__((always_inline)) {
        P.bytes = sg.bytes;
        P.off = sg.off;
        P.n = sg.n;
        P.nbytes = sg.nbytes;
        P.line_base = sg.line_base;
        none.first = sg.n;
    };
    // the runs, one call site (one inlined copy of the step): each segment's static share,
    // then the dynamic share claimed by the workgroup (thread 0) and shared through LDS
    const u64 wg = blockIdx.x;
    u32* claim_lds = reinterpret_cast<u32*>(misc64 + 2);
    u32 sgi = 0;
    bool dyn = false;
    for (;;) {
        bool have = false;
        if (!dyn) {
            for (; sgi < P0.n_segs && !have; ++sgi) {
                const ScanSeg& sg = P0.seg[sgi];
                t_begin = wg * sg.tiles_per_block + (wg < sg.static_rem ? wg : (u64)sg.static_rem);
                t_end = t_begin + sg.tiles_per_block + (wg < sg.static_rem ? 1u : 0u);
                if (t_begin < t_end) {
                    use_segment(sg);
                    have = true;
                }
            }
            if (!have) {
                if (!P0.dyn_chunk) break;
                dyn = true;
                sgi = 0;
                while (sgi < P0.n_segs && P0.seg[sgi].n_static >= P0.seg[sgi].n_tiles) ++sgi;
            }
        }
        if (!have) {   // a dynamic claim
            while (sgi < P0.n_segs && !have) {
                lds_barrier();   // every wave has read the previous claim
                if (tid == 0) *claim_lds = atomicAdd(&P0.dyn_ctr[sgi], 1u);
                lds_barrier();
                const u32 c = (u32)__builtin_amdgcn_readfirstlane(*claim_lds);
                const ScanSeg& sg = P0.seg[sgi];
                t_begin = sg.n_static + (u64)c * P0.dyn_chunk;
                if (t_begin >= sg.n_tiles) {
                    ++sgi;
                    while (sgi < P0.n_segs && P0.seg[sgi].n_static >= P0.seg[sgi].n_tiles) ++sgi;
                    continue;
                }
                t_end = min<u64>(t_begin + P0.dyn_chunk, sg.n_tiles);
                use_segment(sg);
                have = true;
            }
            if (!have) break;
        }
        run_tiles();
    }
    if (n_run == 0) return;   // (uniform over the workgroup: every wave saw the same runs)
    if (WL && lset) {
        for (u32 i = tid; i < ncells; i += MIX_TPB) {
            const u32 v = lcnt[i];
            if (v) {
                lcnt[i] = 0;
                global_add(P, ring_lo, ring_set, i >> P.lds_wl_log2, lbase + (i64)(i & (WL - 1)), v, tl);
            }
        }
    }
    flush_tally(P, tl, lane);
}

