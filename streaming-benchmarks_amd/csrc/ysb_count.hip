// ysb_count.hip -- record mode of the window count for large count tables (configs[2]:
// 1M campaigns x W buckets, no LDS window counters).
//
// CampaignProcessorCommon.execute's windows[bucket][campaign].seenCount++
// (streaming-benchmark-common/.../CampaignProcessorCommon.java:57-67) as one global
// atomic per joined view costs a memory-side atomic request per view: 64 lanes in 64
// different rows run ~17x below the contiguous rate (MI355X_MICROARCH.md, "Global float
// atomics"), and config 3's 33M views per 100M events took 2.4 ms of a 6.9 ms launch.
// Record mode sums them first:
//
//   scan_kernel   a joined in-ring view appends its ring cell index (u32) to a 64-record
//                 LDS ring of its level-1 bin (campaign >> rec_shift, 8 bins); every full
//                 32-record line goes to the (workgroup, bin) HBM sub-buffer as ONE 128-B
//                 store (a partial-line store costs a memory write of its own: scattered
//                 4-B stores were as slow as the atomics, tools/mb_scatter.hip);
//   partition     per (level-1 bin, slice of the scan workgroups): LDS histogram over the
//                 bin's level-2 blocks, 32-aligned runs, records staged per block in LDS
//                 rings and written out as whole lines;
//   count         per level-2 block (32768 / W campaigns, whose L2C x W cells are one
//                 contiguous slab of the campaign-major ring): LDS u32 counters, then
//                 every counted line of cells added ONCE with a plain load/add/store to
//                 the u8 DELTA ring (the block's slab belongs to this workgroup alone;
//                 consecutive lanes take consecutive cells, so the loads and stores
//                 coalesce) -- an eighth of the bytes of the u64 ring's read-modify-write;
//                 a cell whose sum would pass 255 adds it to the u64 ring with one atomic
//                 and restarts at 0 (saturation, never a wrap);
//   fold          before anything reads the u64 ring (drain, ring advance, truth compare,
//                 checksums) delta is added to the ring and cleared (ysb_capi.cpp
//                 fold_delta); the exchange reads the delta ring itself (ysb_table.hip).
//
// Exact: the same additions, reordered (integer sums commute).
#include "ysb_kernels.h"
#include <algorithm>

namespace ysb {

constexpr int REC_TPB = 1024;
// the partition's staged records per level-2 block: one 128-B line (72 KiB of LDS, two
// workgroups per CU; 64 measured slower, profiles/r03t_partition_ab.txt)
constexpr int PART_RING = 32;
constexpr int REC_WAVES = REC_TPB / 64;
constexpr int REC_UNROLL = 8;        // records in flight per lane (loads issued together)
constexpr u32 REC_NONE = 0xFFFFFFFFu;

// One partition workgroup: level-1 bin b, the sub-buffers of scan workgroups
// [w_lo, w_hi) (one of REC_QUARTERS slices).  Each wave walks its own sub-buffers (wave,
// wave + 16, ...) 512 records per round, 8 loads in flight per lane.  Sweep 1 counts
// the records per level-2 block; each block's run starts 32-record aligned in this
// workgroup's output area.  Sweep 2 stages every record in its block's 64-record LDS ring
// (a record arriving when its ring is full goes straight to its final slot) and after
// every round each block's full 128-B lines are written out by one thread.
// (a 32-record ring keeps the workgroup under 80 KiB of LDS: two per CU, so 8 waves per
// SIMD, which the register budget must allow)
__global__ __launch_bounds__(REC_TPB) __attribute__((amdgpu_waves_per_eu(PART_RING == 32 ? 8 : 4)))
void rec_partition_kernel(const RecParams R) {
    __shared__ __attribute__((aligned(16))) u32 stage[REC_SUB_MAX * PART_RING];
    __shared__ u32 hist[REC_SUB_MAX];
    __shared__ u32 boff[REC_SUB_MAX];
    __shared__ u32 cur[REC_SUB_MAX];
    __shared__ u32 fl[REC_SUB_MAX];
    __shared__ u32 rounds_sh;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 b = blockIdx.x / REC_QUARTERS, q = blockIdx.x % REC_QUARTERS;
    const u32 S = 1u << R.sub_log2;
    for (u32 i = tid; i < S; i += REC_TPB) { hist[i] = 0; cur[i] = 0; fl[i] = 0; }
    if (tid == 0) rounds_sh = 0;
    const u32 w_lo = (u32)((u64)q * R.grid / REC_QUARTERS), w_hi = (u32)((u64)(q + 1) * R.grid / REC_QUARTERS);
    const u32 first_blk = b << R.sub_log2;
    const u32 sh = R.w_log2 + R.blk_shift;   // cell -> block
    constexpr u32 CH = 64 * REC_UNROLL;      // records per wave and round
    // this wave's rounds: its sub-buffers in chunks of CH
    u32 my_rounds = 0;
    for (u32 w = w_lo + wave; w < w_hi; w += REC_WAVES) my_rounds += (R.rec_n[(u64)w * R.bins + b] + CH - 1) / CH;
    __syncthreads();
    if (lane == 0) atomicMax(&rounds_sh, my_rounds);
    // cursor over this wave's sub-buffers: (sub-buffer, offset)
    u32 cw = w_lo + wave, coff = 0, cn = cw < w_hi ? R.rec_n[(u64)cw * R.bins + b] : 0u;
    auto next_chunk = [&](u32 (&v)[REC_UNROLL]) {
        while (cw < w_hi && coff >= cn) {
            cw += REC_WAVES;
            coff = 0;
            cn = cw < w_hi ? R.rec_n[(u64)cw * R.bins + b] : 0u;
        }
        const u32* src = R.rec + ((u64)(cw < w_hi ? cw : w_lo) * R.bins + b) * R.cap;
#pragma unroll
        for (int u = 0; u < REC_UNROLL; ++u) {
            const u32 i = coff + u * 64 + lane;
            v[u] = (cw < w_hi && i < cn) ? src[i] : REC_NONE;
        }
        coff += CH;
    };
    // sweep 1: per-block histogram
    for (u32 r = 0; r < my_rounds; ++r) {
        u32 v[REC_UNROLL];
        next_chunk(v);
#pragma unroll
        for (int u = 0; u < REC_UNROLL; ++u)
            if (v[u] != REC_NONE) atomicAdd(&hist[(v[u] >> sh) - first_blk], 1u);
    }
    __syncthreads();
    const u32 rounds = rounds_sh;
    // block runs: 32-record aligned offsets in this workgroup's area
    const u64 base = ((u64)b * REC_QUARTERS + q) * R.area;
    if (wave == 0) {
        const u32 per = (S + 63) / 64;
        const u32 k0 = min(S, lane * per), k1 = min(S, k0 + per);
        u32 sum = 0;
        for (u32 k = k0; k < k1; ++k) sum += (hist[k] + 31u) & ~31u;
        u32 incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if ((int)lane >= o) incl += y;
        }
        u32 run = incl - sum;
        for (u32 k = k0; k < k1; ++k) {
            boff[k] = run;
            const u32 blk = first_blk + k;
            if (blk < R.n_blocks) {
                R.runs[((u64)blk * REC_QUARTERS + q) * 2] = (u32)(base + run);
                R.runs[((u64)blk * REC_QUARTERS + q) * 2 + 1] = hist[k];
            }
            run += (hist[k] + 31u) & ~31u;
        }
    }
    __syncthreads();
    u32* out = R.part + base;
    // writes staged positions [fl, fl + n) of block k (n <= 32: one line or a tail)
    auto write_line = [&](u32 k, u32 n) {
        const u32 f = fl[k];
        u32* dst = out + boff[k] + f;
        const u32* src = stage + k * PART_RING;
        if (n == 32 && (f & 31u) == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const u32 o = (f + 4 * j) & (PART_RING - 1);
                reinterpret_cast<uint4*>(dst)[j] = make_uint4(src[o], src[o + 1], src[o + 2], src[o + 3]);
            }
        } else {
            for (u32 j = 0; j < n; ++j) dst[j] = src[(f + j) & (PART_RING - 1)];
        }
        fl[k] = f + n;
    };
    // sweep 2: stage + write full lines, every wave one chunk per round
    cw = w_lo + wave;
    coff = 0;
    cn = cw < w_hi ? R.rec_n[(u64)cw * R.bins + b] : 0u;
    for (u32 r = 0; r < rounds; ++r) {
        if (r < my_rounds) {
            u32 v[REC_UNROLL];
            next_chunk(v);
#pragma unroll
            for (int u = 0; u < REC_UNROLL; ++u) {
                if (v[u] == REC_NONE) continue;
                const u32 k = (v[u] >> sh) - first_blk;
                const u32 pos = atomicAdd(&cur[k], 1u);
                if (pos - fl[k] < (u32)PART_RING) stage[k * PART_RING + (pos & (PART_RING - 1))] = v[u];
                else out[boff[k] + pos] = v[u];   // its ring is full this round: straight to its slot
            }
        }
        __syncthreads();
        for (u32 k = tid; k < S; k += REC_TPB) {
            const u32 f0 = fl[k], c = cur[k];
            // staged this round: positions [f0, f0 + 64); beyond that they went direct
            const u32 lines = min(c - f0, (u32)PART_RING) / 32;
            for (u32 l = 0; l < lines; ++l) write_line(k, 32);
            if (c - f0 > (u32)PART_RING) fl[k] = c;   // direct positions are written already
        }
        __syncthreads();
    }
    for (u32 k = tid; k < S; k += REC_TPB)   // tails
        if (cur[k] > fl[k]) write_line(k, cur[k] - fl[k]);
}

// 16 cells of the u8 delta ring (one 16-B vector) plus their LDS counts.  A cell whose sum
// passes 255 adds the whole sum to its u64 ring cell (one atomic; rare: ~0.3 views per cell
// per launch on configs[2]) and restarts at 0, so the delta never wraps.
__device__ __forceinline__ uint4 add16(uint4 d, const u32* cnt16, unsigned long long* ring16, u32* dirty) {
    const u32 dw[4] = {d.x, d.y, d.z, d.w};
    u32 o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 c = reinterpret_cast<const uint4*>(cnt16)[k];
        const u32 cc[4] = {c.x, c.y, c.z, c.w};
        u32 w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 s = ((dw[k] >> (8 * j)) & 0xFFu) + cc[j];
            if (s > 255u) {
                atomicAdd(&ring16[4 * k + j], (unsigned long long)s);
                *dirty = 1u;
            } else {
                w |= s << (8 * j);
            }
        }
        o[k] = w;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// One count workgroup: level-2 block j (campaigns [j*L2C, (j+1)*L2C), the slab of
// L2C x W ring cells).  The block's QUARTERS runs flattened, 8 records per lane in flight
// -> LDS u32 counters; then the slab is read, added to and written back whole (16-B
// accesses, all issued before any is used: the sweep is a stream, not a chain of
// dependent loads; whole lines written back, no partial-line writes).
__global__ __launch_bounds__(REC_TPB) void rec_count_kernel(const RecParams R) {
    __shared__ __attribute__((aligned(16))) u32 cnt[REC_BLOCK_CELLS];
    __shared__ u32 roff[REC_QUARTERS + 1];
    __shared__ u32 rbeg[REC_QUARTERS];
    const u32 tid = threadIdx.x;
    const u32 j = blockIdx.x;
    const u32 c0 = j << R.blk_shift;
    const u32 nc = min(1u << R.blk_shift, R.c_pad - c0);
    const u32 cells = nc << R.w_log2;            // <= REC_BLOCK_CELLS, a multiple of 16
    for (u32 i = tid; i < cells / 4; i += REC_TPB) reinterpret_cast<uint4*>(cnt)[i] = make_uint4(0, 0, 0, 0);
    if (tid < 64) {   // the runs' sizes, prefix
        const u32 n = tid < (u32)REC_QUARTERS ? R.runs[((u64)j * REC_QUARTERS + tid) * 2 + 1] : 0u;
        if (tid < (u32)REC_QUARTERS) rbeg[tid] = R.runs[((u64)j * REC_QUARTERS + tid) * 2];
        u32 incl = n;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if ((int)tid >= o) incl += y;
        }
        if (tid < (u32)REC_QUARTERS) roff[tid] = incl - n;
        if (tid == (u32)REC_QUARTERS - 1) roff[REC_QUARTERS] = incl;
    }
    __syncthreads();
    const u32 total = roff[REC_QUARTERS];
    const u32 base_cell = c0 << R.w_log2;
    // the slab of the u8 delta ring: [base_cell, base_cell + cells) bytes, as 16-cell
    // vectors (16 B); 8 consecutive threads cover one 128-B line; vectors <= REC_TPB * SU,
    // so each thread holds at most SU of them.  A cell whose sum would pass 255 adds it to
    // the u64 ring instead (add16), so no cell ever wraps and nothing needs folding between
    // launches: per launch the slab costs a quarter of a u32 delta ring's bytes.
    uint4* dr = reinterpret_cast<uint4*>(R.delta + base_cell);
    const u32 quads = cells / 16;  // 16-cell vectors (cells: a multiple of 16); lines of 8
    constexpr int SU = REC_BLOCK_CELLS / 16 / REC_TPB;
    static_assert(SU * REC_TPB * 16 == REC_BLOCK_CELLS, "one slab vector set per thread");
    unsigned long long* ring = R.counts + base_cell;
    // Dense block (at least one record per 16 cells: nearly every line is counted): the
    // whole slab is read up front, its round trip under the record loads and LDS atomics,
    // and written back whole.  Sparse block: after the counts, only the lines holding a
    // count are read and written (the ring slots this launch's buckets do not reach).
    const bool dense = (u64)total * 16u >= cells;
    uint4 r[SU];
    if (dense) {
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const u32 p = u * REC_TPB + tid;
            r[u] = p < quads ? dr[p] : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    // TPS threads per partition slice (REC_TPB = TPS x REC_QUARTERS): thread (q, k) reads
    // records k, k + TPS, ... of run q -- coalesced lines, no search for the run
    constexpr u32 TPS = REC_TPB / REC_QUARTERS;
    static_assert(TPS * REC_QUARTERS == REC_TPB && TPS >= 16, "one thread group per partition slice");
    const u32 q = tid / TPS, k = tid % TPS;
    const u32 nq = roff[q + 1] - roff[q];
    const u32* src = R.part + rbeg[q];
    for (u32 j0 = 0; j0 < nq; j0 += TPS * REC_UNROLL) {
        u32 v[REC_UNROLL];
#pragma unroll
        for (int u = 0; u < REC_UNROLL; ++u) {
            const u32 jj = j0 + u * TPS + k;
            v[u] = jj < nq ? src[jj] : REC_NONE;
        }
#pragma unroll
        for (int u = 0; u < REC_UNROLL; ++u)
            if (v[u] != REC_NONE) atomicAdd(&cnt[v[u] - base_cell], 1u);
    }
    __syncthreads();
    if (dense) {
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const u32 p = u * REC_TPB + tid;
            if (p < quads) dr[p] = add16(r[u], cnt + 16 * p, ring + 16 * (u64)p, R.dirty);
        }
        return;
    }
    bool live[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const u32 p = u * REC_TPB + tid;
        u32 any = 0;
        if (p < quads) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 c = reinterpret_cast<const uint4*>(cnt)[4 * p + j];
                any |= c.x | c.y | c.z | c.w;
            }
        }
        any |= __shfl_xor(any, 1, 64);
        any |= __shfl_xor(any, 2, 64);
        any |= __shfl_xor(any, 4, 64);
        live[u] = p < quads && any != 0u;
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const u32 p = u * REC_TPB + tid;
        if (live[u]) r[u] = dr[p];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const u32 p = u * REC_TPB + tid;
        if (live[u]) dr[p] = add16(r[u], cnt + 16 * p, ring + 16 * (u64)p, R.dirty);
    }
}

// counts[i] += delta[i], delta[i] = 0 for every cell (16 per thread; all-zero vectors skipped)
__global__ __launch_bounds__(256) void fold_kernel(unsigned long long* counts, u8* delta, u64 vecs) {
    for (u64 q = (u64)blockIdx.x * 256 + threadIdx.x; q < vecs; q += (u64)gridDim.x * 256) {
        const uint4 d = reinterpret_cast<const uint4*>(delta)[q];
        if ((d.x | d.y | d.z | d.w) == 0u) continue;
        const u32 dw[4] = {d.x, d.y, d.z, d.w};
        ulonglong2* c2 = reinterpret_cast<ulonglong2*>(counts + 16 * q);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (((dw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) == 0u) continue;
            ulonglong2 a = c2[j];
            a.x += (dw[j >> 1] >> (16 * (j & 1))) & 0xFFu;
            a.y += (dw[j >> 1] >> (16 * (j & 1) + 8)) & 0xFFu;
            c2[j] = a;
        }
        reinterpret_cast<uint4*>(delta)[q] = make_uint4(0u, 0u, 0u, 0u);
    }
}

void launch_rec_partition(const RecParams& r, hipStream_t s) {
    hipLaunchKernelGGL(rec_partition_kernel, dim3(r.bins * REC_QUARTERS), dim3(REC_TPB), 0, s, r);
}

void launch_fold(unsigned long long* counts, u8* delta, u64 cells, hipStream_t s) {
    const u64 vecs = cells / 16;   // cells: c_pad * W, W a power of two >= 16
    if (!vecs) return;
    const u64 blocks = std::min<u64>((vecs + 255) / 256, 65536);
    hipLaunchKernelGGL(fold_kernel, dim3((u32)blocks), dim3(256), 0, s, counts, delta, vecs);
}

void launch_rec_count(const RecParams& r, hipStream_t s) {
    hipLaunchKernelGGL(rec_count_kernel, dim3(r.n_blocks), dim3(REC_TPB), 0, s, r);
}

}  // namespace ysb
