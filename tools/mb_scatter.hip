// mb_scatter.hip -- microbenchmark (never used for results): what does a stream of
// scattered per-view updates cost next to a nontemporal byte stream shaped like the scan
// kernel's?  One-wave workgroups, 8 per CU, each walks a run of 64-line "tiles" of a
// 25.8 GB buffer with 17 x 16-B nontemporal buffer loads per lane per tile (issued one
// tile ahead), and per tile 21 lanes do one of:
//   mode 0: nothing                       (the stream alone)
//   mode 1: no-return u64 atomicAdd into a random cell of a 1 GiB table
//   mode 2: plain u32 store to a random word of a 1 GiB table
//   mode 3: u32 record appended to an LDS line; every full 32-record line written out as
//           one 128-B store (the record-mode staging)
//   mode 4: like 1, but the atomics of tile t issued after tile t+1's loads are waited for
//           (deferred by one tile)
//   mode 5: u64 atomicAdd into a random cell of a 16 MiB table
//   mode 6: 48-B random reads of a 4 GiB table, consumed in the same tile (probe)
//   mode 7: like 6, consumed one tile later (pipelined probe)
//   mode 10: 128-B bucket reads (one 128-B line per probe); 11: 48-B probes plus, for 1 in
//   13 lanes, a dependent second probe (serial cuckoo); 12: 64-B probes; 13 (argument 13): 128-B
//   bucket probes vs table size, 64 MiB .. 4 GiB (does a table that fits the 256 MiB Infinity
//   Cache stay resident beside the nontemporal stream?)
//
//   hipcc --offload-arch=gfx950 -O3 -o mb_scatter tools/mb_scatter.hip && ./mb_scatter
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32;
typedef unsigned long long u64;

constexpr int CPT = 17;          // 16-B chunks per lane per tile (~260 B per line)
constexpr int TILE_BYTES = CPT * 64 * 16;

__device__ __forceinline__ u64 mix(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

template <int MODE>
__global__ __launch_bounds__(64) void k(const unsigned char* __restrict__ buf, u64 tiles_per_wg, u64* table,
                                        u32* words, u64 table_mask, u32* rec_out, u64 rec_cap, u32* sink,
                                        const uint4* probe_tab, u64 probe_mask) {
    __shared__ u32 stage[64];
    __shared__ u32 sum_sh[64];
    const int lane = threadIdx.x;
    const u64 t0 = blockIdx.x * tiles_per_wg;
    u32 acc = 0;
    uint4 pre[CPT];
    auto issue = [&](u64 t) {
        const unsigned char* base = buf + t * TILE_BYTES;
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(base), 0, TILE_BYTES, 0x00020000);
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * (j * 64 + lane), 0, 2);
            pre[j] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    issue(t0);
    u32 rcur = 0;
    u64 rout = 0;
    bool pend_v = false;
    u64 pend_i = 0;
    uint4 pa = make_uint4(0, 0, 0, 0), pb = pa, pc = pa;
    bool pprobe = false;
    for (u64 t = t0; t < t0 + tiles_per_wg; ++t) {
        u32 x = 0;
#pragma unroll
        for (int j = 0; j < CPT; ++j) x ^= pre[j].x + pre[j].y + pre[j].z + pre[j].w;
        acc += x;
        const u64 h = mix(t * 64 + lane);
        const bool act = lane < 21;
        if (MODE == 4 && pend_v) atomicAdd(&table[pend_i], 1ull);
        if (MODE == 6 && act) {
            const uint4* p = probe_tab + 4 * (h & probe_mask);
            const uint4 a = p[0], b = p[1], c = p[2];
            acc += a.x ^ b.y ^ c.z;
        }
        if (MODE == 8) {   // the same 21 x 48 B as ONE instruction: lanes 3r..3r+2 load view r's parts
            const u32 r = lane / 3, part = lane % 3;
            if (lane < 63) {
                const u64 hr = mix(t * 64 + r);
                const uint4 a = probe_tab[4 * (hr & probe_mask) + part];
                acc += a.x ^ a.y;
            }
        }
        if (MODE == 9 && act) {   // 2 loads (32 B) per view
            const uint4* p = probe_tab + 4 * (h & probe_mask);
            const uint4 a = p[0], b = p[1];
            acc += a.x ^ b.y;
        }
        if (MODE == 10 && act) {   // a 128-B bucket: 8 x 16 B of one 128-B line
            const uint4* p = probe_tab + 8 * (h & (probe_mask >> 1));
            uint4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = p[q];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc += v[q].x ^ v[q].w;
        }
        if (MODE == 11 && act) {   // 48-B probe, then (1 in 13 lanes) a dependent second one
            const uint4* p = probe_tab + 4 * (h & probe_mask);
            const uint4 a = p[0], b = p[1], c = p[2];
            acc += a.x ^ b.y ^ c.z;
            if ((h >> 40) % 13 == 0) {
                const uint4* p2 = probe_tab + 4 * (((h >> 20) ^ a.x) & probe_mask);
                const uint4 a2 = p2[0], b2 = p2[1], c2 = p2[2];
                acc += a2.x ^ b2.y ^ c2.z;
            }
        }
        if (MODE == 13 && act) {   // a 128-B bucket of a table of probe_mask buckets (any count)
            const uint4* p = probe_tab + 8 * (((h >> 32) * probe_mask) >> 32);   // multiply-shift range reduction
            uint4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = p[q];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc += v[q].x ^ v[q].w;
        }
        if (MODE >= 14 && MODE <= 17 && act) {   // 48-B probes of one 64-B slot, other cache policies
            const uint4* p = probe_tab + 4 * (h & probe_mask);
            uint4 a, b, c;
            if constexpr (MODE == 14) {   // nontemporal (global_load ... nt)
                typedef u32 v4u __attribute__((ext_vector_type(4)));
                const v4u* pv = reinterpret_cast<const v4u*>(p);
                const v4u x = __builtin_nontemporal_load(pv), y = __builtin_nontemporal_load(pv + 1),
                          z = __builtin_nontemporal_load(pv + 2);
                a = make_uint4(x[0], x[1], x[2], x[3]); b = make_uint4(y[0], y[1], y[2], y[3]); c = make_uint4(z[0], z[1], z[2], z[3]);
            } else {                      // buffer loads with cache-policy bits sc0 / sc1 / sc0|sc1
                constexpr int AUX = MODE == 15 ? 1 : MODE == 16 ? 2 : 3;
                const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, 64, 0x00020000);
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(rb, 0, 0, AUX);
                const auto y = __builtin_amdgcn_raw_buffer_load_b128(rb, 16, 0, AUX);
                const auto z = __builtin_amdgcn_raw_buffer_load_b128(rb, 32, 0, AUX);
                a = make_uint4(x[0], x[1], x[2], x[3]); b = make_uint4(y[0], y[1], y[2], y[3]); c = make_uint4(z[0], z[1], z[2], z[3]);
            }
            acc += a.x ^ b.y ^ c.z;
        }
        if (MODE == 12 && act) {   // 64-B probe: 4 x 16 B of one 64-B slot
            const uint4* p = probe_tab + 4 * (h & probe_mask);
            const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
            acc += a.x ^ b.y ^ c.z ^ d.w;
        }
        if (MODE == 7) {
            if (pprobe) acc += pa.x ^ pb.y ^ pc.z;
            pprobe = act;
            if (act) {
                const uint4* p = probe_tab + 4 * (h & probe_mask);
                pa = p[0]; pb = p[1]; pc = p[2];
            }
        }
        if (t + 1 < t0 + tiles_per_wg) issue(t + 1);
        if (MODE == 1 && act) atomicAdd(&table[h & table_mask], 1ull);
        if (MODE == 5 && act) atomicAdd(&table[h & (table_mask >> 6)], 1ull);
        if (MODE == 2 && act) words[h & (2 * table_mask + 1)] = (u32)h;
        if (MODE == 4) { pend_v = act; pend_i = h & table_mask; }
        if (MODE == 3) {
            const unsigned long long m = __ballot(act);
            const u32 r = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
            if (act) stage[(rcur + r) & 63] = (u32)h;
            rcur += (u32)__popcll(m);
            while (rcur - (u32)rout >= 32) {
                if (lane < 32) {
                    const u32 v = stage[((u32)rout + lane) & 63];
                    rec_out[(blockIdx.x * rec_cap + rout + lane) % (rec_cap * gridDim.x)] = v;
                }
                rout += 32;
            }
        }
    }
    if (MODE == 4 && pend_v) atomicAdd(&table[pend_i], 1ull);
    if (MODE == 7 && pprobe) acc += pa.x ^ pb.y ^ pc.z;
    sum_sh[lane] = acc;
    if (acc == 0x12345678u) sink[blockIdx.x] = sum_sh[(lane + 1) & 63];   // keep the loads alive
}

int main(int argc, char** argv) {
    int cus = 256;
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
    const u64 grid = (u64)cus * 8;
    const u64 total = 25806623508ull;
    const u64 tiles = total / TILE_BYTES;
    const u64 tpw = tiles / grid;
    unsigned char* buf;
    u64* table;
    u32* rec;
    u32* sink;
    uint4* probe;
    const u64 cells = 1ull << 27;   // 1 GiB of u64
    const u64 rec_cap = tpw * 64;
    const u64 probe_slots = 1ull << 26;   // 4 GiB of 64-B slots
    if (hipMalloc(&buf, tiles * TILE_BYTES + 4096) || hipMalloc(&table, cells * 8) ||
        hipMalloc(&rec, rec_cap * grid * 4) || hipMalloc(&sink, grid * 4) || hipMalloc(&probe, probe_slots * 64)) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, tiles * TILE_BYTES);
    hipMemset(table, 0, cells * 8);
    hipMemset(probe, 3, probe_slots * 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"stream only", "u64 atomics, 1 GiB", "u32 scattered stores, 1 GiB",
                           "LDS-staged 128-B record lines", "u64 atomics deferred one tile",
                           "u64 atomics, 16 MiB", "48-B probes, same tile", "48-B probes, next tile",
                           "48-B probes as one 63-lane load", "32-B probes (2 loads)",
                           "128-B bucket probes (8 loads)", "48-B probes + 1/13 dependent 2nd",
                           "64-B probes (4 loads)", "(table sweep)", "48-B probes, nontemporal",
                           "48-B probes, buffer sc0", "48-B probes, buffer sc1", "48-B probes, buffer sc0|sc1"};
    int only = argc > 1 ? atoi(argv[1]) : -1;
    if (only == 13) {   // 128-B bucket probes beside the stream vs table size (Infinity Cache residency)
        for (u64 mib : {64ull, 128ull, 192ull, 224ull, 256ull, 320ull, 512ull, 1024ull, 4096ull}) {
            const u64 nb = mib << 13;   // 128-B buckets
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k<13>, dim3(grid), dim3(64), 0, 0, buf, tpw, table, (u32*)table, cells - 1, rec, rec_cap, sink, probe, nb);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (rep > 0 && ms < best) best = ms;
            }
            printf("128-B bucket probes into %llu MiB beside the stream: %.3f ms\n", mib, best);
        }
        only = 0;   // and the stream alone
    }
    if (only == 6) {   // probe cost vs table size
        for (u64 sz : {1ull << 26, 1ull << 24, 1ull << 22, 1ull << 21, 1ull << 20}) {
            float best = 1e9;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k<6>, dim3(grid), dim3(64), 0, 0, buf, tpw, table, (u32*)table, cells - 1, rec, rec_cap, sink, probe, sz - 1);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (rep > 0 && ms < best) best = ms;
            }
            printf("probes into %llu MiB: %.3f ms\n", sz * 64 >> 20, best);
        }
        return 0;
    }
    for (int mode = 0; mode < 18; ++mode) {
        if (mode == 13) continue;   // (13: the table-size sweep above)
        if (only >= 0 && mode != only && !(only == 100 && (mode == 0 || mode == 6 || mode == 8 || mode == 9)) &&
            !(only == 101 && (mode == 0 || mode == 6 || mode >= 10)) &&
            !(only == 102 && (mode == 0 || mode == 6 || mode == 10 || mode == 12 || mode >= 14))) continue;
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(a);
#define L(M) hipLaunchKernelGGL(k<M>, dim3(grid), dim3(64), 0, 0, buf, tpw, table, (u32*)table, cells - 1, rec, rec_cap, sink, probe, probe_slots - 1)
            switch (mode) {
                case 0: L(0); break; case 1: L(1); break; case 2: L(2); break; case 3: L(3); break;
                case 4: L(4); break; case 5: L(5); break; case 6: L(6); break; case 7: L(7); break;
                case 8: L(8); break; case 9: L(9); break; case 10: L(10); break; case 11: L(11); break;
                case 12: L(12); break; case 14: L(14); break; case 15: L(15); break; case 16: L(16); break;
                case 17: L(17); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep > 0 && ms < best) best = ms;
        }
        printf("mode %d %-34s %.3f ms  (%.2f TB/s stream, %.2f G updates/s)\n", mode, names[mode], best,
               (double)tiles * TILE_BYTES / best / 1e9, (double)grid * tpw * 21 / best / 1e6);
    }
    return 0;
}
