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

}  // namespace ysb
