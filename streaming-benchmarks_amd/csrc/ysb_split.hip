// ysb_split.hip -- FileBasedDataSource's line split on the GPU (ysb_submit_raw,
// ysb_split_lines_device).
//
// The reference reads the replay file with BufferedReader.readLine and hands each line to
// the chain (flink-benchmarks/.../AdvertisingTopologyNative.java:144-165).  A raw batch is
// whole lines as bytes: the host only reads the file into the pinned slot, and the u32 line
// starts the scan kernel needs are found here, at HBM speed, instead of by a host pass over
// every byte (the native runner's bound until round 4: 54 M events/s).
//
// readLine's terminators: '\n', "\r\n" and a lone '\r'.  Line i starts at position 0 or right
// after a terminator; a terminator that ends the batch starts no line, and a last line
// without a terminator is a line.  So the starts are {0} and every s in [1, nbytes) with
//     b[s-1] == '\n'  ||  (b[s-1] == '\r' && b[s] != '\n').
//
// Three kernels, all on the byte stream in 64 KiB chunks (one 256-thread workgroup each,
// every thread one 16-byte vector per step, so each load instruction of a wave covers 1 KiB):
// count (starts per chunk), prefix (chunk bases, one workgroup), write (each chunk's starts in
// order: a block-wide exclusive scan of the per-vector counts per step).  Algorithmic bytes:
// the batch read twice plus 4 B per line written -- for a 256 MiB slot ~0.1 ms, against the
// ~5 ms its PCIe copy takes.
#include <hipcub/hipcub.hpp>
#include "ysb_kernels.h"

namespace ysb {

constexpr int SPLIT_TPB = 256;
constexpr int SPLIT_STEPS = 16;                                   // 16-byte vectors per thread and chunk
constexpr u64 SPLIT_CHUNK = (u64)SPLIT_TPB * 16 * SPLIT_STEPS;    // 64 KiB
constexpr int SPLIT_PREFIX_TPB = 1024;

// ---- host -> device copy by the CUs (the slots' H2D) ---------------------------------------
// A pinned host slot is visible to the device at its own address (hipHostMalloc); this kernel
// streams it into HBM with 16-byte nontemporal loads and stores, H2D_UNROLL vectors in flight
// per lane.  Why not the DMA engine (hipMemcpyAsync): measured on this pool
// (profiles/r05_h2d_*), SDMA copies of a slot run at 56.5 GB/s or at exactly half that in
// episodes that follow a stretch of GPU idleness and last until compute work wakes the chip
// (the drop-in path's one short scan per 4.5 ms copy does not); a copy done by the CUs keeps
// the GPU active and ran at 55-56 GB/s in every measurement, episodes included.
constexpr int H2D_TPB = 256, H2D_UNROLL = 4;

typedef u32 h2d_v4 __attribute__((ext_vector_type(4)));

template <bool PRIO>
__global__ __launch_bounds__(H2D_TPB) void h2d_copy_kernel(const h2d_v4* __restrict__ src, h2d_v4* __restrict__ dst,
                                                           u64 vecs) {
    if (PRIO) __builtin_amdgcn_s_setprio(3);   // issue ahead of a concurrent scan's waves on the SIMD
    const u64 stride = (u64)gridDim.x * H2D_TPB;
    u64 i = (u64)blockIdx.x * H2D_TPB + threadIdx.x;
    for (; i + (H2D_UNROLL - 1) * stride < vecs; i += H2D_UNROLL * stride) {
        h2d_v4 v[H2D_UNROLL];
#pragma unroll
        for (int u = 0; u < H2D_UNROLL; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < H2D_UNROLL; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
    }
    for (; i < vecs; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// bytes rounded up to whole 16-byte vectors: both buffers have >= 64 bytes of slack
void launch_h2d_copy(void* dst, const void* src, u64 bytes, int cus, hipStream_t s, bool prio) {
    const u64 vecs = (bytes + 15) / 16;
    if (!vecs) return;
    // `cus` workgroups: the caller's choice (32: 512 KiB in flight, well above PCIe's bandwidth
    // x latency, and few enough slow PCIe requests that HBM work beside the copy is not starved;
    // ysb_submit.cpp enqueue_raw)
    const u64 grid = std::max<u64>(1, std::min<u64>((u64)cus, (vecs + H2D_TPB - 1) / H2D_TPB));
    if (prio)
        hipLaunchKernelGGL(h2d_copy_kernel<true>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s,
                           static_cast<const h2d_v4*>(src), static_cast<h2d_v4*>(dst), vecs);
    else
        hipLaunchKernelGGL(h2d_copy_kernel<false>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s,
                           static_cast<const h2d_v4*>(src), static_cast<h2d_v4*>(dst), vecs);
}

// The same from a source at any byte address (a file mapping's batch starts where the previous
// batch's last line ended): output vector i = bytes [16 i + sh, 16 i + sh + 16) of the 16-byte
// aligned `src`, whose first nsrc vectors are read (to the 16-byte boundary at or above the
// batch's end, never further: the same bound the aligned copy keeps).  Each wave copies one
// contiguous run of steps of H2D_UNROLL x 64 vectors (4 KB).  A lane loads one source vector;
// the next one is its right neighbour's (a lane shuffle) or, at lane 63, the next slice's lane
// 0's (a lane read), and the next step's loads are issued before the current step's shifts
// and stores: the step's last vector comes from them (no extra load) and the loop's own
// instructions overlap the PCIe round trip.  Measured against two simpler forms (a grid
// stride of steps with one extra load per step: -2 %; one extra load per wave slice and the
// word shift picked at run time: -10 %), profiles/AB_LOG.md round 6.
// bytes [4 Q + r, 4 Q + r + 16) of the 32 bytes a:b (Q = shift / 4 a template argument: the
// word selection costs nothing, the byte shift is one v_alignbyte per word)
template <int Q>
__device__ __forceinline__ h2d_v4 shift_bytes(const h2d_v4& a, const h2d_v4& b, u32 r) {
    const u32 w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    h2d_v4 o;
    o.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q + 0], r);
    o.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], r);
    o.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], r);
    o.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], r);
    return o;
}

__device__ __forceinline__ h2d_v4 lane_down(const h2d_v4& v) {
    return h2d_v4{(u32)__shfl_down((int)v.x, 1), (u32)__shfl_down((int)v.y, 1), (u32)__shfl_down((int)v.z, 1),
                  (u32)__shfl_down((int)v.w, 1)};
}

__device__ __forceinline__ h2d_v4 lane0(const h2d_v4& v) {
    return h2d_v4{(u32)__builtin_amdgcn_readlane((int)v.x, 0), (u32)__builtin_amdgcn_readlane((int)v.y, 0),
                  (u32)__builtin_amdgcn_readlane((int)v.z, 0), (u32)__builtin_amdgcn_readlane((int)v.w, 0)};
}

template <int Q>
__global__ __launch_bounds__(H2D_TPB) void h2d_copy_unaligned_kernel(const h2d_v4* __restrict__ src,
                                                                          h2d_v4* __restrict__ dst, u64 vecs,
                                                                          u64 nsrc, u32 r) {
    constexpr u64 STEP = 64 * H2D_UNROLL;
    const u32 lane = threadIdx.x & 63u;
    const u64 waves = (u64)gridDim.x * (H2D_TPB / 64);
    const u64 wave = (u64)blockIdx.x * (H2D_TPB / 64) + (threadIdx.x >> 6);
    const u64 steps = (vecs + STEP - 1) / STEP;
    const u64 s0 = steps * wave / waves, s1 = steps * (wave + 1) / waves;   // wave-uniform
    if (s0 >= s1) return;
    auto load = [&](u64 i) { return i < nsrc ? __builtin_nontemporal_load(src + i) : h2d_v4{0, 0, 0, 0}; };
    h2d_v4 cur[H2D_UNROLL], nxt[H2D_UNROLL];
#pragma unroll
    for (int u = 0; u < H2D_UNROLL; ++u) cur[u] = load(s0 * STEP + u * 64 + lane);
    for (u64 st = s0; st < s1; ++st) {
        const u64 b = st * STEP;
        if (st + 1 < s1) {
#pragma unroll
            for (int u = 0; u < H2D_UNROLL; ++u) nxt[u] = load(b + STEP + u * 64 + lane);
        } else {   // the run's end: only the vector after it
            nxt[0] = load(b + STEP + lane);
#pragma unroll
            for (int u = 1; u < H2D_UNROLL; ++u) nxt[u] = h2d_v4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < H2D_UNROLL; ++u) {
            const u64 i = b + u * 64 + lane;
            // both cross-lane reads in every lane (a ?: evaluates one operand only: a shuffle
            // under lane != 63 would give lane 62 an inactive lane's 0)
            const h2d_v4 down = lane_down(cur[u]);
            const h2d_v4 nx = lane0(u + 1 < H2D_UNROLL ? cur[u + 1 < H2D_UNROLL ? u + 1 : u] : nxt[0]);
            h2d_v4 n = down;
            if (lane == 63u) n = nx;
            if (i < vecs) __builtin_nontemporal_store(shift_bytes<Q>(cur[u], n, r), dst + i);
        }
#pragma unroll
        for (int u = 0; u < H2D_UNROLL; ++u) cur[u] = nxt[u];
    }
}

void launch_h2d_copy_unaligned(void* dst, const void* src, u64 bytes, int wgs, hipStream_t s) {
    const u64 vecs = (bytes + 15) / 16;
    if (!vecs) return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    const u64 nsrc = ((a & 15) + bytes + 15) / 16;
    const u64 per_wg = (u64)(H2D_TPB / 64) * 64 * H2D_UNROLL;
    const u64 grid = std::max<u64>(1, std::min<u64>((u64)wgs, (vecs + per_wg - 1) / per_wg));
    const h2d_v4* s16 = reinterpret_cast<const h2d_v4*>(a & ~(uintptr_t)15);
    h2d_v4* d16 = static_cast<h2d_v4*>(dst);
    const u32 r = (u32)(a & 3);
    switch ((a >> 2) & 3) {
    case 0: hipLaunchKernelGGL(h2d_copy_unaligned_kernel<0>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s, s16, d16, vecs, nsrc, r); break;
    case 1: hipLaunchKernelGGL(h2d_copy_unaligned_kernel<1>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s, s16, d16, vecs, nsrc, r); break;
    case 2: hipLaunchKernelGGL(h2d_copy_unaligned_kernel<2>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s, s16, d16, vecs, nsrc, r); break;
    default: hipLaunchKernelGGL(h2d_copy_unaligned_kernel<3>, dim3((unsigned)grid), dim3(H2D_TPB), 0, s, s16, d16, vecs, nsrc, r); break;
    }
}

u64 split_chunks(u64 nbytes) { return (nbytes + SPLIT_CHUNK - 1) / SPLIT_CHUNK; }

// high bit of every zero byte of x (exact, no carries between bytes)
__device__ __forceinline__ u32 zero_bytes(u32 x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu); }

// the four zero-byte flags of zero_bytes() as bits 0..3
__device__ __forceinline__ u32 flag4(u32 z) {
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// Byte by byte (a vector holding a '\r', or the batch's last partial vector): bit j set when
// s = p + j + 1 starts a line.
__device__ __noinline__ u32 start_mask_bytes(const u8* b, u64 nbytes, u64 p) {
    u32 m = 0;
    for (u32 j = 0; j < 16; ++j) {
        const u64 q = p + j;
        if (q + 1 >= nbytes) break;   // a start must lie inside the batch (and b[q + 1] exists)
        const u8 c = b[q];
        if (c == '\n' || (c == '\r' && b[q + 1] != '\n')) m |= 1u << j;
    }
    return m;
}

// Line starts s = p + j + 1 (bit j) of the 16-byte vector at p (16-byte aligned, p < nbytes).
__device__ __forceinline__ u32 start_mask16(const u8* b, u64 nbytes, u64 p) {
    if (p + 17 > nbytes) return start_mask_bytes(b, nbytes, p);   // the last vector: bounds per byte
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(b + p));
    const u32 w[4] = {v.x, v.y, v.z, v.w};
    u32 m = 0, cr = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m |= flag4(zero_bytes(w[k] ^ 0x0A0A0A0Au)) << (4 * k);
        cr |= zero_bytes(w[k] ^ 0x0D0D0D0Du);
    }
    if (cr) return start_mask_bytes(b, nbytes, p);   // a '\r': its next byte decides (never on generator data)
    return m;
}

__global__ __launch_bounds__(SPLIT_TPB) void split_count_kernel(const u8* b, u64 nbytes, u32* chunk_cnt) {
    typedef hipcub::BlockReduce<u32, SPLIT_TPB> Reduce;
    __shared__ typename Reduce::TempStorage tmp;
    const u64 base = (u64)blockIdx.x * SPLIT_CHUNK;
    u32 cnt = 0;
#pragma unroll 4
    for (int it = 0; it < SPLIT_STEPS; ++it) {
        const u64 p = base + ((u64)it * SPLIT_TPB + threadIdx.x) * 16;
        if (p < nbytes) cnt += __popc(start_mask16(b, nbytes, p));
    }
    const u32 total = Reduce(tmp).Sum(cnt);
    if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = total;
}

// chunk_cnt[0..nchunks) -> exclusive bases in place; *n = lines of the batch (0 when empty)
__global__ __launch_bounds__(SPLIT_PREFIX_TPB) void split_prefix_kernel(u32* chunk, u64 nchunks, u64 nbytes,
                                                                        unsigned long long* n) {
    typedef hipcub::BlockScan<unsigned long long, SPLIT_PREFIX_TPB> Scan;
    __shared__ typename Scan::TempStorage tmp;
    const u64 per = (nchunks + SPLIT_PREFIX_TPB - 1) / SPLIT_PREFIX_TPB;
    const u64 a = (u64)threadIdx.x * per, e = a + per < nchunks ? a + per : nchunks;
    unsigned long long s = 0;
    for (u64 i = a; i < e; ++i) s += chunk[i];
    unsigned long long pre = 0, total = 0;
    Scan(tmp).ExclusiveSum(s, pre, total);
    for (u64 i = a; i < e; ++i) {
        const u32 c = chunk[i];
        chunk[i] = (u32)pre;   // < nbytes < 2^32
        pre += c;
    }
    if (threadIdx.x == 0) *n = nbytes ? 1ull + total : 0ull;
}

__global__ __launch_bounds__(SPLIT_TPB) void split_write_kernel(const u8* b, u64 nbytes, const u32* chunk_base,
                                                                u32* off, u64 cap) {
    typedef hipcub::BlockScan<u32, SPLIT_TPB> Scan;
    __shared__ typename Scan::TempStorage tmp;
    const u64 base = (u64)blockIdx.x * SPLIT_CHUNK;
    u64 run = (u64)chunk_base[blockIdx.x] + 1;   // off index of the chunk's first start (off[0] = 0)
    if (blockIdx.x == 0 && threadIdx.x == 0 && cap) off[0] = 0;
    for (int it = 0; it < SPLIT_STEPS; ++it) {
        const u64 p = base + ((u64)it * SPLIT_TPB + threadIdx.x) * 16;
        u32 m = p < nbytes ? start_mask16(b, nbytes, p) : 0u;
        u32 pre = 0, agg = 0;
        Scan(tmp).ExclusiveSum((u32)__popc(m), pre, agg);
        u64 o = run + pre;
        while (m) {
            const u32 j = __builtin_ctz(m);
            if (o < cap) off[o] = (u32)(p + j + 1);
            ++o;
            m &= m - 1;
        }
        run += agg;
        __syncthreads();   // the scan's storage is reused by the next step
    }
}

// The sampled lines of a device launch, for the host's layout sampling (ysb_capi.cpp
// sample_device_layout): block i copies line s.line[i] of its batch: out[i * SAMPLE_STRIDE] = {line start,
// sampled length, valid} and then the line's first <= SAMPLE_BYTES bytes.  It runs on the
// compute stream, so it reads the batch after whatever produced it there; out is pinned host
// memory (no copy of its own).
__global__ __launch_bounds__(64) void sample_kernel(SampleSegs s, u8* out) {
    __shared__ u32 hdr[2];
    const u32 i = blockIdx.x;
    u8* o = out + (u64)i * SAMPLE_STRIDE;
    if (threadIdx.x == 0) {
        const u64 li = s.line[i];
        const u32 o0 = s.off[i][li];
        const u64 end = li + 1 < s.n[i] ? (u64)s.off[i][li + 1] : s.nbytes[i];
        const bool valid = o0 <= end && end <= s.nbytes[i];
        const u32 len = valid ? (u32)(end - o0 < SAMPLE_BYTES ? end - o0 : SAMPLE_BYTES) : 0u;
        hdr[0] = o0;
        hdr[1] = len;
        u32* h = reinterpret_cast<u32*>(o);
        h[0] = o0;
        h[1] = len;
        h[2] = valid ? 1u : 0u;
        h[3] = 0;
    }
    __syncthreads();
    for (u32 j = threadIdx.x; j < hdr[1]; j += 64) o[16 + j] = s.bytes[i][(u64)hdr[0] + j];
}

void launch_sample(const SampleSegs& s, u32 nseg, u8* out, hipStream_t st) {
    if (nseg) hipLaunchKernelGGL(sample_kernel, dim3(nseg), dim3(64), 0, st, s, out);
}

// ---- the replay's event-time rebasing (ysb_submit_raw_mapped with a ysb_rebase) ------------
// A replay cycle is played again with every event_time moved by whole 10-second buckets: only
// the nine leading digits of the 13-digit time change.  One lane per
// line, after the split: the line's start from off[], the digits' position and bucket index
// from the cycle's table (4 B per line, HBM), nine byte stores.  ~9 B written + 8 B read per
// line against the line's ~254 B copied over PCIe: the kernel is a few microseconds per batch.
constexpr int REBASE_TPB = 256;

__global__ __launch_bounds__(REBASE_TPB) void rebase_kernel(u8* __restrict__ b, u64 nbytes, const u32* __restrict__ off,
                                                            const unsigned long long* d_n, u64 n_val,
                                                            const u32* __restrict__ tab, u64 tab_n, u64 cap, i64 lead) {
    const u64 nl = d_n ? *d_n : n_val;
    u64 n = nl < tab_n ? nl : tab_n;
    if (n > cap) n = cap;   // (more lines than off[] holds: the launch fails on the host)
    for (u64 i = (u64)blockIdx.x * REBASE_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * REBASE_TPB) {
        const u32 t = tab[i];
        const u64 p = (u64)off[i] + (t & 0xFFFFu);
        if (p + 9 > nbytes) continue;
        u64 v = (u64)(lead + (i64)(t >> 16));
#pragma unroll
        for (int d = 8; d >= 0; --d) {
            b[p + d] = (u8)('0' + v % 10);
            v /= 10;
        }
    }
}

void launch_rebase(u8* b, u64 nbytes, const u32* off, u64 cap, const unsigned long long* d_n, u64 n_val,
                   const u32* tab, u64 tab_n, i64 lead, int cus, hipStream_t s) {
    if (!nbytes || !tab_n) return;
    // (a raw batch's lines are unknown until the split's count is read on the device: a
    // grid-stride loop either way)
    const u64 lines = d_n ? tab_n : std::min(n_val, tab_n);
    const u64 grid = std::max<u64>(1, std::min<u64>((u64)cus * 4, (lines + REBASE_TPB - 1) / REBASE_TPB));
    hipLaunchKernelGGL(rebase_kernel, dim3((unsigned)grid), dim3(REBASE_TPB), 0, s, b, nbytes, off, d_n, n_val, tab,
                       tab_n, cap, lead);
}

hipError_t launch_split_lines(const u8* b, u64 nbytes, u32* chunk, u32* off, u64 cap, unsigned long long* d_n,
                              hipStream_t s) {
    if (nbytes == 0) return hipMemsetAsync(d_n, 0, 8, s);
    const u64 nch = split_chunks(nbytes);
    hipLaunchKernelGGL(split_count_kernel, dim3((unsigned)nch), dim3(SPLIT_TPB), 0, s, b, nbytes, chunk);
    hipLaunchKernelGGL(split_prefix_kernel, dim3(1), dim3(SPLIT_PREFIX_TPB), 0, s, chunk, nch, nbytes, d_n);
    hipLaunchKernelGGL(split_write_kernel, dim3((unsigned)nch), dim3(SPLIT_TPB), 0, s, b, nbytes, chunk, off, cap);
    return hipGetLastError();
}

}  // namespace ysb
