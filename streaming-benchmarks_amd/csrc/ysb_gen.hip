// ysb_gen.hip -- device side of the synthetic input: the seeded generator that
// writes the data/ generator's JSON line format (core.clj:90-97) straight into HBM,
// the generator-truth counter (independent of any parsing), and small helpers.
#include <hipcub/hipcub.hpp>
#include "ysb_kernels.h"

namespace ysb {

// Line lengths, plus their exact 64-bit total (the u32 offsets of a batch must not wrap).
__global__ void gen_len_kernel(GenSpec s, u64 first, u64 n, u32* len, unsigned long long* total) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    u32 l = 0;
    if (i < n) {
        l = gen_line_len(s, first + i, gen_event(s, first + i));
        len[i] = l;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
    if ((threadIdx.x & 63) == 0 && l) atomicAdd(total, (unsigned long long)l);
}

// One line per thread, assembled in registers and written as bytes.
__global__ void gen_write_kernel(GenSpec s, u64 first, u64 n, const u32* off, u8* out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    char line[288];
    const GenEvent e = gen_event(s, first + i);
    const u32 len = gen_line_write(s, first + i, e, line);
    u8* o = out + off[i];
    for (u32 k = 0; k < len; ++k) o[k] = (u8)line[k];
}

hipError_t gen_events_device(const GenSpec& spec, u64 first, u64 n, u8* d_out, u64 cap, u32* d_off,
                             u64* nbytes, hipStream_t s) {
    if (n == 0) { *nbytes = 0; return hipSuccess; }
    const unsigned blocks = (unsigned)((n + 255) / 256);
    unsigned long long* d_total = nullptr;
    hipError_t err = hipMalloc(&d_total, 8);
    if (err != hipSuccess) return err;
    err = hipMemsetAsync(d_total, 0, 8, s);
    hipLaunchKernelGGL(gen_len_kernel, dim3(blocks), dim3(256), 0, s, spec, first, n, d_off, d_total);
    unsigned long long total64 = 0;
    if (err == hipSuccess) err = hipMemcpyAsync(&total64, d_total, 8, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    hipFree(d_total);
    if (err != hipSuccess) return err;
    if (total64 > cap) {   // includes every total the u32 offsets cannot express
        *nbytes = total64;
        return hipErrorInvalidValue;
    }
    size_t temp = 0;
    err = hipcub::DeviceScan::ExclusiveSum(nullptr, temp, d_off, d_off, (int)n, s);
    if (err != hipSuccess) return err;
    void* d_temp = nullptr;
    err = hipMalloc(&d_temp, temp ? temp : 16);
    if (err != hipSuccess) return err;
    err = hipcub::DeviceScan::ExclusiveSum(d_temp, temp, d_off, d_off, (int)n, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    hipFree(d_temp);
    if (err != hipSuccess) return err;
    *nbytes = total64;
    hipLaunchKernelGGL(gen_write_kernel, dim3(blocks), dim3(256), 0, s, spec, first, n, d_off, d_out);
    return hipStreamSynchronize(s);
}

// Generator truth: per event, straight from the RNG (no bytes), the view count per
// (campaign, bucket) -- the dostats oracle's arithmetic (core.clj:107-126) on the
// generator's own choices.
__global__ void truth_kernel(GenSpec s, u64 first, u64 n, DivMagic div, unsigned long long* truth, u32 W,
                             const i64* ring, unsigned long long* outside) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GenEvent e = gen_event(s, first + i);
    if (e.event_type != 0) return;
    const u32 c = e.ad / s.ads_per_campaign;
    if (c >= s.n_campaigns) return;
    const i64 b = div_trunc(e.time_ms, div);
    const i64 rel = b - ring[0];
    if (ring[1] && rel >= 0 && rel < (i64)W) atomicAdd(&truth[(u64)c * W + (u64)(b & (i64)(W - 1))], 1ull);
    else atomicAdd(outside, 1ull);
}

void launch_truth(const GenSpec& spec, u64 first, u64 n, const DivMagic& div, unsigned long long* truth,
                  u32 ring_w, const i64* ring, unsigned long long* truth_outside, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(truth_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, spec, first, n, div,
                       truth, ring_w, ring, truth_outside);
}

__global__ void compare_kernel(const unsigned long long* a, const unsigned long long* b, u64 cells,
                               unsigned long long* out) {
    u32 diff = 0;
    unsigned long long sa = 0, sb = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += (u64)gridDim.x * blockDim.x) {
        diff += a[i] != b[i];
        sa += a[i];
        sb += b[i];
    }
    if (diff) atomicAdd(&out[0], (unsigned long long)diff);
    if (sa) atomicAdd(&out[1], sa);
    if (sb) atomicAdd(&out[2], sb);
}

void launch_compare(const unsigned long long* a, const unsigned long long* b, u64 cells, unsigned long long* out,
                    hipStream_t s) {
    if (cells == 0) return;
    hipLaunchKernelGGL(compare_kernel, dim3(1024), dim3(256), 0, s, a, b, cells, out);
}

__global__ void add_u64_kernel(unsigned long long* dst, const unsigned long long* src, u64 n) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        dst[i] += src[i];
}

void launch_add_u64(unsigned long long* dst, const unsigned long long* src, u64 n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(add_u64_kernel, dim3(1024), dim3(256), 0, s, dst, src, n);
}

}  // namespace ysb
