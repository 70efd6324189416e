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
//   scan_kernel   a joined in-ring view appends its ring cell index (u32) to the
//                 sub-buffer of (its workgroup, campaign >> rec_shift) -- 64 level-1
//                 bins, LDS cursors, plain stores that fill whole lines in L2;
//   partition     per level-1 bin (x4 quarters of the scan workgroups): LDS histogram
//                 over the bin's level-2 blocks, prefix, scatter into contiguous runs;
//   count         per level-2 block (32768 / W campaigns, whose L2C x W cells are one
//                 contiguous slab of the campaign-major ring): LDS u32 counters, then
//                 every non-zero cell added to the ring ONCE with a plain load/add/store
//                 (the block's slab belongs to this workgroup alone; consecutive lanes
//                 take consecutive cells, so the loads and stores coalesce).
//
// Exact: the same additions, reordered (integer sums commute).
#include "ysb_kernels.h"

namespace ysb {

constexpr int REC_TPB = 1024;
constexpr u32 REC_SUB_MAX = 4096;   // level-2 blocks per level-1 bin (host keeps it below)

__global__ __launch_bounds__(REC_TPB) void rec_partition_kernel(const RecParams R) {
    __shared__ u32 hist[REC_SUB_MAX];
    __shared__ u32 cur[REC_SUB_MAX];
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 b = blockIdx.x / REC_QUARTERS, q = blockIdx.x % REC_QUARTERS;
    const u32 S = 1u << R.sub_log2;
    for (u32 i = tid; i < S; i += REC_TPB) hist[i] = 0;
    __syncthreads();
    const u32 w_lo = (u32)((u64)q * R.grid / REC_QUARTERS), w_hi = (u32)((u64)(q + 1) * R.grid / REC_QUARTERS);
    const u32 first_blk = b << R.sub_log2;
    const u32 sh = R.w_log2 + R.blk_shift;   // cell -> block
    // sweep 1: level-2 histogram (one wave per sub-buffer)
    for (u32 w = w_lo + wave; w < w_hi; w += REC_TPB / 64) {
        const u64 sb = (u64)w * R.bins + b;
        const u32 n = R.rec_n[sb];
        const u32* src = R.rec + sb * R.cap;
        for (u32 i = lane; i < n; i += 64) atomicAdd(&hist[(src[i] >> sh) - first_blk], 1u);
    }
    __syncthreads();
    // exclusive prefix over the S blocks: wave 0, each lane a chunk
    const u64 area = (u64)((R.grid + REC_QUARTERS - 1) / REC_QUARTERS) * R.cap;
    const u64 base = ((u64)b * REC_QUARTERS + q) * area;
    if (wave == 0) {
        const u32 per = (S + 63) / 64;
        const u32 k0 = min(S, lane * per), k1 = min(S, k0 + per);
        u32 sum = 0;
        for (u32 k = k0; k < k1; ++k) sum += hist[k];
        u32 incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if ((int)lane >= o) incl += y;
        }
        u32 run = incl - sum;
        for (u32 k = k0; k < k1; ++k) {
            const u32 h = hist[k];
            cur[k] = run;
            const u32 blk = first_blk + k;
            if (blk < R.n_blocks) {
                R.runs[((u64)blk * REC_QUARTERS + q) * 2] = (u32)(base + run);
                R.runs[((u64)blk * REC_QUARTERS + q) * 2 + 1] = h;
            }
            run += h;
        }
    }
    __syncthreads();
    // sweep 2: scatter into the blocks' runs
    u32* out = R.part + base;
    for (u32 w = w_lo + wave; w < w_hi; w += REC_TPB / 64) {
        const u64 sb = (u64)w * R.bins + b;
        const u32 n = R.rec_n[sb];
        const u32* src = R.rec + sb * R.cap;
        for (u32 i = lane; i < n; i += 64) {
            const u32 cell = src[i];
            out[atomicAdd(&cur[(cell >> sh) - first_blk], 1u)] = cell;
        }
    }
}

__global__ __launch_bounds__(REC_TPB) void rec_count_kernel(const RecParams R) {
    __shared__ __attribute__((aligned(16))) u32 cnt[REC_BLOCK_CELLS];
    const u32 tid = threadIdx.x;
    const u32 j = blockIdx.x;
    const u32 c0 = j << R.blk_shift;
    const u32 nc = min(1u << R.blk_shift, R.c_pad - c0);
    const u32 cells = nc << R.w_log2;            // <= REC_BLOCK_CELLS, a multiple of 16
    for (u32 i = tid; i < cells / 4; i += REC_TPB) reinterpret_cast<uint4*>(cnt)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const u32 base_cell = c0 << R.w_log2;
    for (u32 q = 0; q < (u32)REC_QUARTERS; ++q) {
        const u32 off = R.runs[((u64)j * REC_QUARTERS + q) * 2];
        const u32 n = R.runs[((u64)j * REC_QUARTERS + q) * 2 + 1];
        const u32* src = R.part + off;
        for (u32 i = tid; i < n; i += REC_TPB) atomicAdd(&cnt[src[i] - base_cell], 1u);
    }
    __syncthreads();
    unsigned long long* ring = R.counts + base_cell;
    for (u32 i = tid; i < cells; i += REC_TPB) {
        const u32 v = cnt[i];
        if (v) ring[i] += v;
    }
}

void launch_rec_partition(const RecParams& r, hipStream_t s) {
    hipLaunchKernelGGL(rec_partition_kernel, dim3(r.bins * REC_QUARTERS), dim3(REC_TPB), 0, s, r);
}

void launch_rec_count(const RecParams& r, hipStream_t s) {
    hipLaunchKernelGGL(rec_count_kernel, dim3(r.n_blocks), dim3(REC_TPB), 0, s, r);
}

}  // namespace ysb
