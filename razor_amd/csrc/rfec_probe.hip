// rfec_probe.hip -- HBM ceiling probes for the roofline report (measurement
// only; not on the FEC data path).  Streaming read / copy / write of 16-byte
// vectors in the same access shape the FEC kernels use (one dwordx4 per lane,
// consecutive lanes on consecutive chunks), so bench.py can state a measured
// ceiling beside the 8 TB/s spec peak.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "razor_fec.h"

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT>
__device__ __forceinline__ void st(v4u* p, v4u v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <bool NT, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_read(const v4u* __restrict__ src, size_t n, v4u* __restrict__ sink)
{
    const size_t lanes = (size_t)gridDim.x * kBlock;
    const size_t t0 = (size_t)blockIdx.x * kBlock + threadIdx.x;
    v4u acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const size_t i = t0 + u * lanes;
        if (i < n)
            acc ^= ld<NT>(src + i);
    }
    // keep the loads live; sink is written only when the XOR is a magic value
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u)
        sink[t0 & 1023] = acc;
}

template <bool NT, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n)
{
    const size_t lanes = (size_t)gridDim.x * kBlock;
    const size_t t0 = (size_t)blockIdx.x * kBlock + threadIdx.x;
    v4u v[ITEMS];
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const size_t i = t0 + u * lanes;
        if (i < n)
            v[u] = ld<NT>(src + i);
    }
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const size_t i = t0 + u * lanes;
        if (i < n)
            st<NT>(dst + i, v[u]);
    }
}

template <bool NT, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_write(v4u* __restrict__ dst, size_t n)
{
    const size_t lanes = (size_t)gridDim.x * kBlock;
    const size_t t0 = (size_t)blockIdx.x * kBlock + threadIdx.x;
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const size_t i = t0 + u * lanes;
        if (i < n)
            st<NT>(dst + i, v4u{(uint32_t)i, 0, 0, 0});
    }
}

// R read streams : W write streams (the FEC kernels' read / write mixes:
// 10 : 3 for the row encode, 10 : 7 for the full 3 x 4 plan, 4 : 1 for rows
// of 4 as at k = 32): lane i loads
// chunk i of each read stream (all in flight), stores their XOR to chunk i of
// each write stream; non-temporal both ways.
template <int R, int W>
__global__ __launch_bounds__(kBlock) void k_mix(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    v4u v[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
        v[r] = ld<true>(src + r * n + i);
    v4u acc = v[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
        acc ^= v[r];
#pragma unroll
    for (int w = 0; w < W; ++w)
        st<true>(dst + w * n + i, acc);
}

inline dim3 grid_for(size_t n, int items)
{
    const size_t lanes = (n + items - 1) / items;
    return dim3((unsigned)((lanes + kBlock - 1) / kBlock));
}

} // namespace

extern "C" {

/* flags: bit0 = non-temporal, bit1 = 4 vectors per lane */
int rfec_probe_read(const void* src, size_t bytes, void* sink, unsigned flags, void* stream)
{
    const size_t n = bytes / 16;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const v4u* p = reinterpret_cast<const v4u*>(src);
    v4u* k = reinterpret_cast<v4u*>(sink);
    const int items = (flags & 2) ? 4 : 1;
    if (flags & 1) {
        if (items == 4)
            hipLaunchKernelGGL((k_read<true, 4>), grid_for(n, 4), dim3(kBlock), 0, s, p, n, k);
        else
            hipLaunchKernelGGL((k_read<true, 1>), grid_for(n, 1), dim3(kBlock), 0, s, p, n, k);
    } else {
        if (items == 4)
            hipLaunchKernelGGL((k_read<false, 4>), grid_for(n, 4), dim3(kBlock), 0, s, p, n, k);
        else
            hipLaunchKernelGGL((k_read<false, 1>), grid_for(n, 1), dim3(kBlock), 0, s, p, n, k);
    }
    return (int)hipGetLastError();
}

int rfec_probe_copy(const void* src, void* dst, size_t bytes, unsigned flags, void* stream)
{
    const size_t n = bytes / 16;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const v4u* a = reinterpret_cast<const v4u*>(src);
    v4u* b = reinterpret_cast<v4u*>(dst);
    const int items = (flags & 2) ? 4 : 1;
    if (flags & 1) {
        if (items == 4)
            hipLaunchKernelGGL((k_copy<true, 4>), grid_for(n, 4), dim3(kBlock), 0, s, a, b, n);
        else
            hipLaunchKernelGGL((k_copy<true, 1>), grid_for(n, 1), dim3(kBlock), 0, s, a, b, n);
    } else {
        if (items == 4)
            hipLaunchKernelGGL((k_copy<false, 4>), grid_for(n, 4), dim3(kBlock), 0, s, a, b, n);
        else
            hipLaunchKernelGGL((k_copy<false, 1>), grid_for(n, 1), dim3(kBlock), 0, s, a, b, n);
    }
    return (int)hipGetLastError();
}

int rfec_probe_write(void* dst, size_t bytes, unsigned flags, void* stream)
{
    const size_t n = bytes / 16;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    v4u* b = reinterpret_cast<v4u*>(dst);
    const int items = (flags & 2) ? 4 : 1;
    if (flags & 1) {
        if (items == 4)
            hipLaunchKernelGGL((k_write<true, 4>), grid_for(n, 4), dim3(kBlock), 0, s, b, n);
        else
            hipLaunchKernelGGL((k_write<true, 1>), grid_for(n, 1), dim3(kBlock), 0, s, b, n);
    } else {
        if (items == 4)
            hipLaunchKernelGGL((k_write<false, 4>), grid_for(n, 4), dim3(kBlock), 0, s, b, n);
        else
            hipLaunchKernelGGL((k_write<false, 1>), grid_for(n, 1), dim3(kBlock), 0, s, b, n);
    }
    return (int)hipGetLastError();
}

/* R : W streaming mix (see k_mix), stream_bytes per stream; (r, w) in
   {(10, 3), (10, 7), (4, 1), (1, 1)}; -1 for another pair */
int rfec_probe_mix(const void* src, void* dst, size_t stream_bytes, unsigned r, unsigned w, void* stream)
{
    const size_t n = stream_bytes / 16;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const v4u* a = reinterpret_cast<const v4u*>(src);
    v4u* b = reinterpret_cast<v4u*>(dst);
    const dim3 g = grid_for(n, 1);
    if (r == 10 && w == 3)
        hipLaunchKernelGGL((k_mix<10, 3>), g, dim3(kBlock), 0, s, a, b, n);
    else if (r == 10 && w == 7)
        hipLaunchKernelGGL((k_mix<10, 7>), g, dim3(kBlock), 0, s, a, b, n);
    else if (r == 4 && w == 1)
        hipLaunchKernelGGL((k_mix<4, 1>), g, dim3(kBlock), 0, s, a, b, n);
    else if (r == 1 && w == 1)
        hipLaunchKernelGGL((k_mix<1, 1>), g, dim3(kBlock), 0, s, a, b, n);
    else
        return -1;
    return (int)hipGetLastError();
}

} // extern "C"
