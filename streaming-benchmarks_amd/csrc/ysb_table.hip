// ysb_table.hip -- maintenance kernels of the device (campaign, window) count table:
// compaction of the non-zero cells of a bucket range (what ysb_drain returns and what
// ysb_ring_advance evicts from the ring).  The table is campaign-major [rows][W] u64,
// cell (c, b & (W-1)) holding bucket b of the live range [ring_lo, ring_lo + W).
//
// This is CampaignProcessorCommon.flushWindows' walk over the dirty windows
// (streaming-benchmark-common/.../CampaignProcessorCommon.java:91-98) done on the
// device: only non-zero cells cross PCIe, so a 1M-campaign table (config 3) drains in
// O(active windows), not O(table).
#include "ysb_kernels.h"

namespace ysb {

// Pass 1 (count_only) counts the non-zero cells with bucket in [blo, bhi); pass 2
// writes them as rows {campaign + c_off, bucket, count} (order unspecified) and, when
// clear, zeroes them.  One thread per cell of the buckets' columns.
__global__ __launch_bounds__(AUX_TPB) void compact_kernel(unsigned long long* table, u32 rows, u32 W, i64 blo, u32 nb, u32 c_off, int count_only, int clear,
                                                          TableRow* out, u32* out_n, u32 cap) {
    const u64 cells = (u64)rows * nb;
    u32 mine = 0;
    for (u64 i = (u64)blockIdx.x * AUX_TPB + threadIdx.x; i < cells; i += (u64)gridDim.x * AUX_TPB) {
        const u32 c = (u32)(i / nb);
        const i64 b = blo + (i64)(i % nb);
        unsigned long long* cell = &table[(u64)c * W + (u64)(b & (i64)(W - 1))];
        const unsigned long long v = *cell;
        if (!v) continue;
        if (count_only) { ++mine; continue; }
        const u32 k = atomicAdd(out_n, 1u);
        if (k < cap) {
            TableRow r;
            r.campaign = c + c_off;
            r.pad = 0;
            r.bucket = b;
            r.count = v;
            out[k] = r;
            // cleared only once written out: a cell past cap keeps its count (the host
            // reports "table changed during drain" and nothing is lost)
            if (clear) *cell = 0;
        }
    }
    if (count_only) {
        // one atomic per wave
        u32 s = mine;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(out_n, s);
    }
}

void launch_compact(unsigned long long* table, u32 rows, u32 W, i64 blo, u32 nb, u32 c_off,
                    bool count_only, bool clear, TableRow* out, u32* out_n, u32 cap, hipStream_t s) {
    const u64 cells = (u64)rows * nb;
    if (!cells) return;
    const u64 blocks = std::min<u64>((cells + AUX_TPB - 1) / AUX_TPB, 4096);
    hipLaunchKernelGGL(compact_kernel, dim3((unsigned)blocks), dim3(AUX_TPB), 0, s, table, rows, W, blo, nb,
                       c_off, count_only ? 1 : 0, clear ? 1 : 0, out, out_n, cap);
}

__global__ __launch_bounds__(AUX_TPB) void side_compact_kernel(const SideSlot* t, u64 slots, u32 cbits,
                                                               int count_only, TableRow* out, u32* out_n, u32 cap) {
    u32 mine = 0;
    const i64 half = (i64)1 << (63 - cbits);
    for (u64 i = (u64)blockIdx.x * AUX_TPB + threadIdx.x; i < slots; i += (u64)gridDim.x * AUX_TPB) {
        const SideSlot sl = t[i];
        if (sl.key == SIDE_EMPTY || sl.count == 0) continue;
        if (count_only) { ++mine; continue; }
        const u32 k = atomicAdd(out_n, 1u);
        if (k < cap) {
            TableRow r;
            r.campaign = (u32)(sl.key & ((1ull << cbits) - 1));
            r.pad = 0;
            r.bucket = (i64)(sl.key >> cbits) - half;
            r.count = sl.count;
            out[k] = r;
        }
    }
    if (count_only) {
        u32 s = mine;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(out_n, s);
    }
}

__global__ __launch_bounds__(AUX_TPB) void side_clear_kernel(SideSlot* t, u64 slots) {
    for (u64 i = (u64)blockIdx.x * AUX_TPB + threadIdx.x; i < slots; i += (u64)gridDim.x * AUX_TPB) {
        SideSlot e;
        e.key = SIDE_EMPTY;
        e.count = 0;
        t[i] = e;
    }
}

void launch_side_clear(SideSlot* t, u64 slots, hipStream_t s) {
    if (!slots) return;
    const u64 blocks = std::min<u64>((slots + AUX_TPB - 1) / AUX_TPB, 4096);
    hipLaunchKernelGGL(side_clear_kernel, dim3((unsigned)blocks), dim3(AUX_TPB), 0, s, t, slots);
}

void launch_side_compact(const SideSlot* t, u64 slots, u32 cbits, bool count_only, TableRow* out, u32* out_n,
                         u32 cap, hipStream_t s) {
    if (!slots) return;
    const u64 blocks = std::min<u64>((slots + AUX_TPB - 1) / AUX_TPB, 4096);
    hipLaunchKernelGGL(side_compact_kernel, dim3((unsigned)blocks), dim3(AUX_TPB), 0, s, t, slots, cbits,
                       count_only ? 1 : 0, out, out_n, cap);
}

// ---- the range-limited exchange (keyBy(0), AdvertisingTopologyNative.java:118-119) -------
// A rank's pending counts since its last exchange are its u64 ring plus (record mode) its
// u8 delta ring.  The u64 ring is read only when a launch without record mode ran
// (force_u64) or a record-mode path wrote it (*dirty): configs[2]'s exchange then reads a
// 1-byte delta per cell instead of an 8-byte one.

constexpr u32 XPLAN_LDS_W = 4096;   // ring slots whose maxima a plan workgroup keeps in LDS

__device__ __forceinline__ bool read_u64(int force_u64, const u32* dirty) { return force_u64 || (dirty && *dirty); }

// slot_max[s] = max pending count of ring slot s over this rank's campaigns; 16 cells
// (one campaign's consecutive slots) per thread.
__global__ __launch_bounds__(AUX_TPB) void xplan_kernel(const unsigned long long* counts, const u8* delta, u32 W,
                                                        u64 vecs, int force_u64, const u32* dirty,
                                                        unsigned long long* slot_max) {
    __shared__ unsigned long long lmax[XPLAN_LDS_W];
    const bool in_lds = W <= XPLAN_LDS_W;
    if (in_lds)
        for (u32 s = threadIdx.x; s < W; s += AUX_TPB) lmax[s] = 0;
    __syncthreads();
    const bool r64 = read_u64(force_u64, dirty);
    if (!r64 && in_lds && delta) {
        // Round 4: the grid stride (a multiple of W / 16 vectors: AUX_TPB = 256 >= 4096 / 16)
        // keeps a thread on the same 16 slots, so their maxima stay in registers and reach
        // LDS once per thread -- not an LDS atomic per nonzero cell (configs[2]: ~30 %).
        u32 m[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) m[j] = 0;
        const u64 q0 = (u64)blockIdx.x * AUX_TPB + threadIdx.x, st = (u64)gridDim.x * AUX_TPB;
        const uint4* dv = reinterpret_cast<const uint4*>(delta);
        auto fold = [&](const uint4 d) {
            const u32 dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) m[j] = max(m[j], (dw[j >> 2] >> (8 * (j & 3))) & 0xFFu);
        };
        u64 q = q0;
        for (; q + 7 * st < vecs; q += 8 * st) {   // eight loads in flight
            uint4 d[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = dv[q + u * st];
#pragma unroll
            for (int u = 0; u < 8; ++u) fold(d[u]);
        }
        for (; q < vecs; q += st) fold(dv[q]);
        const u32 s0 = (u32)((16 * q0) & (u64)(W - 1));
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (m[j]) atomicMax(&lmax[s0 + j], (unsigned long long)m[j]);
        __syncthreads();
        for (u32 s = threadIdx.x; s < W; s += AUX_TPB)
            if (lmax[s]) atomicMax(&slot_max[s], lmax[s]);
        return;
    }
    for (u64 q = (u64)blockIdx.x * AUX_TPB + threadIdx.x; q < vecs; q += (u64)gridDim.x * AUX_TPB) {
        const u64 i0 = 16 * q;
        const u32 s0 = (u32)(i0 & (u64)(W - 1));
        u32 dw[4] = {0u, 0u, 0u, 0u};
        if (delta) {
            const uint4 d = reinterpret_cast<const uint4*>(delta)[q];
            dw[0] = d.x; dw[1] = d.y; dw[2] = d.z; dw[3] = d.w;
        }
        if (!r64 && (dw[0] | dw[1] | dw[2] | dw[3]) == 0u) continue;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            unsigned long long v = (dw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            if (r64) v += counts[i0 + j];
            if (!v) continue;
            if (in_lds) atomicMax(&lmax[s0 + j], v);
            else atomicMax(&slot_max[s0 + j], v);
        }
    }
    if (!in_lds) return;
    __syncthreads();
    for (u32 s = threadIdx.x; s < W; s += AUX_TPB)
        if (lmax[s]) atomicMax(&slot_max[s], lmax[s]);
}

// The pack and unpack walk the [rows][R] cell array two-dimensionally: one wave per campaign
// row (grid-stride over rows), its lanes over the plan's slots (a few hundred bytes, cached) --
// no 64-bit division or modulo per cell, and the packed cells of a row are written contiguously.
constexpr int XROW_WAVES = AUX_TPB / 64;

template <class T>
__device__ __forceinline__ void put_cell(void* out, u64 i, unsigned long long v) { static_cast<T*>(out)[i] = (T)v; }

// The host widens the plan's runs of slots to aligned groups of four (ysb_capi.cpp
// align_slot_runs), so a packed u8 row is whole words; a slot >= W in the list would be a
// cell that sends 0 and receives nothing.

// out[c][k] = pending(c, slots[k]) as `width`-byte cells, the sources zeroed -- except a
// cell above `cap` (a pipelined exchange whose plan is one call old: the cell grew past what
// the width can sum over the ranks), which stays pending for a later exchange and sends 0.
// (On the compute stream, in order with the scans that add to the rings.)
template <class T>
__global__ __launch_bounds__(AUX_TPB) void xpack_kernel(unsigned long long* counts, u8* delta, u32 W, u32 rows,
                                                        const u32* slots, u32 R, int force_u64, const u32* dirty,
                                                        void* out, unsigned long long cap) {
    const bool r64 = read_u64(force_u64, dirty);
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (u32 c = blockIdx.x * XROW_WAVES + wave; c < rows; c += gridDim.x * XROW_WAVES) {
        const u64 row = (u64)c * W, orow = (u64)c * R;
        for (u32 k = lane; k < R; k += 64) {
            if (slots[k] >= W) {
                put_cell<T>(out, orow + k, 0);
                continue;
            }
            const u64 cell = row + slots[k];
            const unsigned long long d = delta ? delta[cell] : 0ull;
            const unsigned long long x = r64 ? counts[cell] : 0ull;
            unsigned long long v = d + x;
            if (v > cap) {
                v = 0;
            } else {
                if (d) delta[cell] = 0;
                if (x) counts[cell] = 0;
            }
            put_cell<T>(out, orow + k, v);
        }
    }
}

// owned[c][slots[k]] += in[c][k], through a u8 accumulator of the owned table's layout
// (saturating, as the record-mode delta ring: a cell whose byte would pass 255 adds the whole
// sum to the u64 owned table and restarts at 0; launch_fold moves the bytes into it before the
// owned table is read).  configs[2]'s ~0.3 views per cell and exchange then cost a byte of
// read-modify-write per cell instead of 8 (the owned table's 1.6 GB per exchange at one rank).
// The unpack is the owned table's only writer (one thread per cell: plain adds).
template <class T>
__global__ __launch_bounds__(AUX_TPB) void xunpack_kernel(unsigned long long* owned, u8* owned8, u32 W, u32 rows,
                                                          const u32* slots, u32 R, const void* in) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T* src = static_cast<const T*>(in);
    for (u32 c = blockIdx.x * XROW_WAVES + wave; c < rows; c += gridDim.x * XROW_WAVES) {
        const u64 row = (u64)c * W, irow = (u64)c * R;
        for (u32 k = lane; k < R; k += 64) {
            const unsigned long long v = src[irow + k];
            if (!v || slots[k] >= W) continue;
            const u64 cell = row + slots[k];
            const unsigned long long sum = owned8[cell] + v;
            if (sum > 255u) {
                owned[cell] += sum;
                owned8[cell] = 0;
            } else {
                owned8[cell] = (u8)sum;
            }
        }
    }
}

// Round 4: the u8 pack and unpack (configs[2]: ~100 slots x 1M campaigns per exchange) a word
// of 4 cells per lane: a row's L = R / 4 words over L lanes, 64 / L rows per wave.  Four
// consecutive, aligned slots (the common case: the plan is the live bucket range) move as one
// u32 load / store of the ring; any other group, a cell above cap, or the u64 ring in play
// (r64) takes the per-cell steps of xpack_kernel / xunpack_kernel for its 4 cells.
struct XLanes {
    u32 L, rpw, sub, j;
    __device__ XLanes(u32 R, u32 lane) : L(R / 4) {
        rpw = L <= 64 ? 64 / L : 1;
        sub = L <= 64 ? lane / L : 0;
        j = lane - sub * (L <= 64 ? L : 0);
    }
};

__device__ __forceinline__ bool run4(const uint4 sk) {
    return (sk.x & 3u) == 0u && sk.y == sk.x + 1 && sk.z == sk.x + 2 && sk.w == sk.x + 3;
}

__global__ __launch_bounds__(AUX_TPB) void xpack8_kernel(unsigned long long* counts, u8* delta, u32 W, u32 rows,
                                                         const u32* slots, u32 R, int force_u64, const u32* dirty,
                                                         u32* out, unsigned long long cap) {
    const bool r64 = read_u64(force_u64, dirty);
    const XLanes X(R, threadIdx.x & 63);
    if (X.sub >= X.rpw) return;
    const u32 wave = threadIdx.x >> 6;
    const u32 c8 = cap < 255ull ? (u32)cap : 255u;
    const u32 c0 = (blockIdx.x * XROW_WAVES + wave) * X.rpw + X.sub, cst = gridDim.x * XROW_WAVES * X.rpw;
    if (X.L <= 64 && !r64) {
        // the common case: a lane keeps one word of the row (its slots loaded once), four
        // rows' loads in flight per step
        const uint4 sk = reinterpret_cast<const uint4*>(slots)[X.j];
        if (run4(sk)) {
            u32 c = c0;
            for (; c < rows; c += 4 * cst) {
                u32 d[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const u32 cu = c + u * cst;
                    d[u] = cu < rows ? *reinterpret_cast<const u32*>(delta + (u64)cu * W + sk.x) : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const u32 cu = c + u * cst;
                    if (cu >= rows) continue;
                    u32 word = d[u];
                    const u32 hi = max(max(word & 0xFFu, (word >> 8) & 0xFFu), max((word >> 16) & 0xFFu, word >> 24));
                    if (hi <= c8) {
                        if (word) *reinterpret_cast<u32*>(delta + (u64)cu * W + sk.x) = 0;
                    } else {   // a cell above cap stays pending and sends 0
                        u32 keep = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            const u32 v = (word >> (8 * b)) & 0xFFu;
                            if (v > c8) keep |= v << (8 * b);
                        }
                        *reinterpret_cast<u32*>(delta + (u64)cu * W + sk.x) = keep;
                        word &= ~keep;
                    }
                    out[(u64)cu * X.L + X.j] = word;
                }
            }
            return;
        }
    }
    for (u32 c = c0; c < rows; c += cst) {
        const u64 row = (u64)c * W;
        for (u32 j = X.j; j < X.L; j += (X.L <= 64 ? X.L : 64)) {
            const uint4 sk = reinterpret_cast<const uint4*>(slots)[j];
            u32 word = 0;
            bool done = false;
            if (!r64 && run4(sk)) {
                u32* dp = reinterpret_cast<u32*>(delta + row + sk.x);
                const u32 d = *dp;
                const u32 hi = max(max(d & 0xFFu, (d >> 8) & 0xFFu), max((d >> 16) & 0xFFu, d >> 24));
                if (hi <= c8) {
                    word = d;
                    if (d) *dp = 0;
                    done = true;
                }
            }
            if (!done) {
                const u32 sl[4] = {sk.x, sk.y, sk.z, sk.w};
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    if (sl[b] >= W) continue;
                    const u64 cell = row + sl[b];
                    const unsigned long long d = delta[cell];
                    const unsigned long long x = r64 ? counts[cell] : 0ull;
                    const unsigned long long v = d + x;
                    if (v > cap) continue;   // stays pending, sends 0
                    if (d) delta[cell] = 0;
                    if (x) counts[cell] = 0;
                    word |= (u32)v << (8 * b);
                }
            }
            out[(u64)c * X.L + j] = word;
        }
    }
}

// Bytes of o + v (four u8 lanes) that carry out of their lane: bit 7 of each byte set where
// the byte sum passes 255.  t holds the sums of the low seven bits, so bit 7 of t is the carry
// INTO bit 7; the carry out of bit 7 is the majority of o7, v7 and that carry.
__device__ __forceinline__ u32 byte_carry(u32 o, u32 v) {
    const u32 t = (o & 0x7F7F7F7Fu) + (v & 0x7F7F7F7Fu);
    return ((o & v) | ((o ^ v) & t)) & 0x80808080u;
}

__global__ __launch_bounds__(AUX_TPB) void xunpack8_kernel(unsigned long long* owned, u8* owned8, u32 W, u32 rows,
                                                           const u32* slots, u32 R, const u32* in) {
    const XLanes X(R, threadIdx.x & 63);
    if (X.sub >= X.rpw) return;
    const u32 wave = threadIdx.x >> 6;
    const u32 c0 = (blockIdx.x * XROW_WAVES + wave) * X.rpw + X.sub, cst = gridDim.x * XROW_WAVES * X.rpw;
    if (X.L <= 64) {
        // the common case: a lane keeps one word of the row, four rows' loads in flight per step
        const uint4 sk = reinterpret_cast<const uint4*>(slots)[X.j];
        if (run4(sk)) {
            for (u32 c = c0; c < rows; c += 4 * cst) {
                u32 v[4], o[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const u32 cu = c + u * cst;
                    v[u] = cu < rows ? in[(u64)cu * X.L + X.j] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const u32 cu = c + u * cst;
                    o[u] = v[u] ? *reinterpret_cast<const u32*>(owned8 + (u64)cu * W + sk.x) : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (!v[u]) continue;
                    const u64 row = (u64)(c + u * cst) * W;
                    if (!byte_carry(o[u], v[u])) {
                        *reinterpret_cast<u32*>(owned8 + row + sk.x) = o[u] + v[u];
                        continue;
                    }
#pragma unroll
                    for (int b = 0; b < 4; ++b) {   // a byte would pass 255: its sum to the u64 table
                        const u32 vb = (v[u] >> (8 * b)) & 0xFFu;
                        const u64 cell = row + sk.x + b;
                        const u32 sum = ((o[u] >> (8 * b)) & 0xFFu) + vb;
                        if (sum > 255u) {
                            owned[cell] += sum;
                            owned8[cell] = 0;
                        } else {
                            owned8[cell] = (u8)sum;
                        }
                    }
                }
            }
            return;
        }
    }
    for (u32 c = c0; c < rows; c += cst) {
        const u64 row = (u64)c * W;
        for (u32 j = X.j; j < X.L; j += (X.L <= 64 ? X.L : 64)) {
            const u32 v = in[(u64)c * X.L + j];
            if (!v) continue;
            const uint4 sk = reinterpret_cast<const uint4*>(slots)[j];
            if (run4(sk)) {
                u32* op = reinterpret_cast<u32*>(owned8 + row + sk.x);
                const u32 o = *op;
                // no byte of o + v carries out: the bytes add as one word
                if (!byte_carry(o, v)) {
                    *op = o + v;
                    continue;
                }
            }
            const u32 sl[4] = {sk.x, sk.y, sk.z, sk.w};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const u32 vb = (v >> (8 * b)) & 0xFFu;
                if (!vb || sl[b] >= W) continue;
                const u64 cell = row + sl[b];
                const u32 sum = owned8[cell] + vb;
                if (sum > 255u) {
                    owned[cell] += sum;
                    owned8[cell] = 0;
                } else {
                    owned8[cell] = (u8)sum;
                }
            }
        }
    }
}

// *out += SUM over rows whose campaign is in [c_lo, c_hi) of count * cell_weight (mod 2^64)
__global__ __launch_bounds__(AUX_TPB) void checksum_kernel(const unsigned long long* table, u32 rows, u32 W,
                                                           i64 ring_lo, u32 c_off, u32 c_lo, u32 c_hi,
                                                           unsigned long long* out) {
    unsigned long long acc = 0;
    const u64 cells = (u64)rows * W;
    for (u64 i = (u64)blockIdx.x * AUX_TPB + threadIdx.x; i < cells; i += (u64)gridDim.x * AUX_TPB) {
        const unsigned long long v = table[i];
        if (!v) continue;
        const u32 c = c_off + (u32)(i / W);
        if (c < c_lo || c >= c_hi) continue;
        const i64 slot = (i64)(i & (u64)(W - 1));
        const i64 b = ring_lo + ((slot - ring_lo) & (i64)(W - 1));
        acc += v * cell_weight(c, b);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

static u64 grid_for(u64 items, u64 cap = 8192) { return std::max<u64>(1, std::min<u64>((items + AUX_TPB - 1) / AUX_TPB, cap)); }

void launch_xplan(const unsigned long long* counts, const u8* delta, u32 W, u64 cells, int force_u64,
                  const u32* dirty, unsigned long long* slot_max, hipStream_t s) {
    const u64 vecs = cells / 16;
    if (!vecs) return;
    // 512 workgroups: each ends with one global atomicMax per live slot (configs[2]: ~100 slots)
    hipLaunchKernelGGL(xplan_kernel, dim3((unsigned)grid_for(vecs, 512)), dim3(AUX_TPB), 0, s, counts, delta, W, vecs,
                       force_u64, dirty, slot_max);
}

static u64 row_grid(u32 rows, u32 rpw = 1) {
    const u64 waves = ((u64)rows + rpw - 1) / rpw;
    return std::max<u64>(1, std::min<u64>((waves + XROW_WAVES - 1) / XROW_WAVES, 8192));
}
static u32 rows_per_wave(u32 R) { return R / 4 <= 64 ? 64 / (R / 4) : 1; }

void launch_xpack(unsigned long long* counts, u8* delta, u32 W, u32 rows, const u32* slots, u32 R, int force_u64,
                  const u32* dirty, void* out, u32 width, unsigned long long cap, hipStream_t s) {
    if (!rows || !R) return;
    const dim3 g((unsigned)row_grid(rows)), b(AUX_TPB);
    if (width == 1 && delta && R % 4 == 0)
        hipLaunchKernelGGL(xpack8_kernel, dim3((unsigned)row_grid(rows, rows_per_wave(R))), b, 0, s, counts, delta, W,
                           rows, slots, R, force_u64, dirty, static_cast<u32*>(out), cap);
    else if (width == 1) hipLaunchKernelGGL(xpack_kernel<u8>, g, b, 0, s, counts, delta, W, rows, slots, R, force_u64, dirty, out, cap);
    else if (width == 4) hipLaunchKernelGGL(xpack_kernel<u32>, g, b, 0, s, counts, delta, W, rows, slots, R, force_u64, dirty, out, cap);
    else hipLaunchKernelGGL(xpack_kernel<unsigned long long>, g, b, 0, s, counts, delta, W, rows, slots, R, force_u64, dirty, out, cap);
}

void launch_xunpack(unsigned long long* owned, u8* owned8, u32 W, u32 rows, const u32* slots, u32 R, const void* in,
                    u32 width, hipStream_t s) {
    if (!rows || !R) return;
    const dim3 g((unsigned)row_grid(rows)), b(AUX_TPB);
    if (width == 1 && R % 4 == 0)
        hipLaunchKernelGGL(xunpack8_kernel, dim3((unsigned)row_grid(rows, rows_per_wave(R))), b, 0, s, owned, owned8, W,
                           rows, slots, R, static_cast<const u32*>(in));
    else if (width == 1) hipLaunchKernelGGL(xunpack_kernel<u8>, g, b, 0, s, owned, owned8, W, rows, slots, R, in);
    else if (width == 4) hipLaunchKernelGGL(xunpack_kernel<u32>, g, b, 0, s, owned, owned8, W, rows, slots, R, in);
    else hipLaunchKernelGGL(xunpack_kernel<unsigned long long>, g, b, 0, s, owned, owned8, W, rows, slots, R, in);
}

void launch_checksum(const unsigned long long* table, u32 rows, u32 W, i64 ring_lo, u32 c_off, u32 c_lo, u32 c_hi,
                     unsigned long long* out, hipStream_t s) {
    const u64 cells = (u64)rows * W;
    if (!cells) return;
    hipLaunchKernelGGL(checksum_kernel, dim3((unsigned)grid_for(cells, 4096)), dim3(AUX_TPB), 0, s, table, rows, W,
                       ring_lo, c_off, c_lo, c_hi, out);
}

}  // namespace ysb
