// encode_lab.hip -- A/B lab for the k = 10 / 1,200-B row encode (payload
// only, no headers): which lane -> byte mapping and cache policy moves the
// 10:3 read:write stream closest to the HBM ceiling.  Measurement only; not
// on the product path.  Rotates NSETS disjoint buffer sets so no launch finds
// its operands in the 256 MB MALL.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/encode_lab.hip -o tools/bin/encode_lab
// run:   tools/bin/encode_lab [groups=65536] [rounds=7] [reps=10]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int K = 10, R = 3, COL = 4, CH = 75; // 1200 B = 75 chunks of 16 B

template <int L>
__device__ __forceinline__ v4u ld(const v4u* p)
{
    if constexpr (L == 1)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// 0 plain, 1 nt, 2 write-through (sc0 sc1), 3 sc0 sc1 nt
template <int S>
__device__ __forceinline__ void st(v4u* p, v4u v)
{
    if constexpr (S == 1)
        __builtin_nontemporal_store(v, p);
    else if constexpr (S == 2)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (S == 3)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        *p = v;
}

// A: flat (group, chunk) lanes: 10 loads, 3 stores per lane
template <int L, int S, int BS>
__global__ __launch_bounds__(BS) void k_flat(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t total)
{
    const uint32_t t = blockIdx.x * BS + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / CH, c = t - g * CH;
    const v4u* s = sh + (size_t)g * K * CH + c;
    v4u v[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        v[i] = ld<L>(s + i * CH);
    v4u* d = par + (size_t)g * R * CH + c;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v4u a = v[r * COL];
#pragma unroll
        for (int q = 1; q < COL; ++q)
            if (r * COL + q < K)
                a ^= v[r * COL + q];
        st<S>(d + r * CH, a);
    }
}

// B: output-mapped lanes, one per parity chunk (g, r, c): every wave's store
// is 1 KiB of consecutive, line-aligned parity bytes
template <int L, int S, int BS>
__global__ __launch_bounds__(BS) void k_out(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t total)
{
    const uint32_t t = blockIdx.x * BS + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / (R * CH), rem = t - g * (R * CH);
    const uint32_t r = rem / CH, c = rem - r * CH;
    const v4u* s = sh + ((size_t)g * K + r * COL) * CH + c;
    v4u a = ld<L>(s), b = ld<L>(s + CH);
    if (r < 2) {
        const v4u x = ld<L>(s + 2 * CH), y = ld<L>(s + 3 * CH);
        a ^= x;
        b ^= y;
    }
    st<S>(par + t, a ^ b);
}

// C: output-mapped, grid-stride persistent (grid = nblk)
template <int L, int S, int BS>
__global__ __launch_bounds__(BS) void k_out_gs(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t total)
{
    for (uint32_t t = blockIdx.x * BS + threadIdx.x; t < total; t += gridDim.x * BS) {
        const uint32_t g = t / (R * CH), rem = t - g * (R * CH);
        const uint32_t r = rem / CH, c = rem - r * CH;
        const v4u* s = sh + ((size_t)g * K + r * COL) * CH + c;
        v4u a = ld<L>(s), b = ld<L>(s + CH);
        if (r < 2) {
            const v4u x = ld<L>(s + 2 * CH), y = ld<L>(s + 3 * CH);
            a ^= x;
            b ^= y;
        }
        st<S>(par + t, a ^ b);
    }
}

// D: flat, grid-stride persistent
template <int L, int S, int BS>
__global__ __launch_bounds__(BS) void k_flat_gs(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t total)
{
    for (uint32_t t = blockIdx.x * BS + threadIdx.x; t < total; t += gridDim.x * BS) {
        const uint32_t g = t / CH, c = t - g * CH;
        const v4u* s = sh + (size_t)g * K * CH + c;
        v4u v[K];
#pragma unroll
        for (int i = 0; i < K; ++i)
            v[i] = ld<L>(s + i * CH);
        v4u* d = par + (size_t)g * R * CH + c;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            v4u a = v[r * COL];
#pragma unroll
            for (int q = 1; q < COL; ++q)
                if (r * COL + q < K)
                    a ^= v[r * COL + q];
            st<S>(d + r * CH, a);
        }
    }
}

// E: ceiling probe for the same mix on contiguous streams: lane t reads
// stream i at t (i < 10) and writes stream j at t (j < 3)
template <int L, int S, int BS>
__global__ __launch_bounds__(BS) void k_mix(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t n)
{
    const uint32_t t = blockIdx.x * BS + threadIdx.x;
    if (t >= n)
        return;
    v4u v[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        v[i] = ld<L>(sh + (size_t)i * n + t);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v4u a = v[r * COL];
#pragma unroll
        for (int q = 1; q < COL; ++q)
            if (r * COL + q < K)
                a ^= v[r * COL + q];
        st<S>(par + (size_t)r * n + t, a);
    }
}

template <int L, int BS>
__global__ __launch_bounds__(BS) void k_copy(const v4u* __restrict__ a, v4u* __restrict__ b, uint32_t n)
{
    const uint32_t t = blockIdx.x * BS + threadIdx.x;
    if (t < n)
        st<1>(b + t, ld<L>(a + t));
}

struct Set {
    v4u *sh, *par;
};

typedef void (*Launch)(const Set&, uint32_t G, hipStream_t);

template <int L, int S, int BS>
void run_flat(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t total = G * CH;
    hipLaunchKernelGGL((k_flat<L, S, BS>), dim3((total + BS - 1) / BS), dim3(BS), 0, st, s.sh, s.par, total);
}
template <int L, int S, int BS>
void run_out(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t total = G * R * CH;
    hipLaunchKernelGGL((k_out<L, S, BS>), dim3((total + BS - 1) / BS), dim3(BS), 0, st, s.sh, s.par, total);
}
template <int L, int S, int BS, int NB>
void run_out_gs(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t total = G * R * CH;
    hipLaunchKernelGGL((k_out_gs<L, S, BS>), dim3(NB), dim3(BS), 0, st, s.sh, s.par, total);
}
template <int L, int S, int BS, int NB>
void run_flat_gs(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t total = G * CH;
    hipLaunchKernelGGL((k_flat_gs<L, S, BS>), dim3(NB), dim3(BS), 0, st, s.sh, s.par, total);
}
template <int L, int S, int BS>
void run_mix(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t n = G * CH;
    hipLaunchKernelGGL((k_mix<L, S, BS>), dim3((n + BS - 1) / BS), dim3(BS), 0, st, s.sh, s.par, n);
}
template <int L, int BS>
void run_copy(const Set& s, uint32_t G, hipStream_t st)
{
    const uint32_t n = G * CH * 5; // 5 of the 10 source slots' bytes -> copy read+write = encode-sized
    hipLaunchKernelGGL((k_copy<L, BS>), dim3((n + BS - 1) / BS), dim3(BS), 0, st, s.sh, s.sh + (size_t)n, n);
}

struct Var {
    const char* name;
    Launch fn;
    int check; // output comparable to the reference parity
    double bpg = 13 * 1200.0; // algorithmic bytes per group
};

int main(int argc, char** argv)
{
    const uint32_t G = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int NSETS = 3;
    const size_t shb = (size_t)G * K * CH * 16, pb = (size_t)G * R * CH * 16;
    std::vector<Set> sets(NSETS);
    std::vector<uint8_t> h(shb);
    uint64_t x = 0x52415A4F52464543ull;
    for (size_t i = 0; i < shb; i += 8) {
        x ^= x >> 12;
        x ^= x << 25;
        x ^= x >> 27;
        uint64_t v = x * 2685821657736338717ull;
        memcpy(&h[i], &v, 8);
    }
    for (auto& s : sets) {
        CK(hipMalloc(&s.sh, shb));
        CK(hipMalloc(&s.par, pb));
        CK(hipMemcpy(s.sh, h.data(), shb, hipMemcpyHostToDevice));
    }
    // reference parity on the host
    std::vector<uint8_t> ref(pb);
    for (uint32_t g = 0; g < G; ++g)
        for (int r = 0; r < R; ++r)
            for (int b = 0; b < 1200; ++b) {
                uint8_t a = 0;
                for (int q = 0; q < COL && r * COL + q < K; ++q)
                    a ^= h[((size_t)g * K + r * COL + q) * 1200 + b];
                ref[((size_t)g * R + r) * 1200 + b] = a;
            }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<Var> vars = {
        {"flat nt_ld wt_st (product)", run_flat<1, 2, 256>, 1},
        {"flat nt_ld nt_st", run_flat<1, 1, 256>, 1},
        {"flat nt_ld plain_st", run_flat<1, 0, 256>, 1},
        {"flat plain_ld wt_st", run_flat<0, 2, 256>, 1},
        {"flat nt_ld wt_st bs512", run_flat<1, 2, 512>, 1},
        {"flat nt_ld wt_st bs1024", run_flat<1, 2, 1024>, 1},
        {"flat_gs nt wt 256x2048", run_flat_gs<1, 2, 256, 2048>, 1},
        {"flat_gs nt wt 256x1024", run_flat_gs<1, 2, 256, 1024>, 1},
        {"out nt_ld wt_st", run_out<1, 2, 256>, 1},
        {"out nt_ld nt_st", run_out<1, 1, 256>, 1},
        {"out nt_ld plain_st", run_out<1, 0, 256>, 1},
        {"out nt_ld wtnt_st", run_out<1, 3, 256>, 1},
        {"out plain_ld nt_st", run_out<0, 1, 256>, 1},
        {"out nt_ld nt_st bs512", run_out<1, 1, 512>, 1},
        {"out_gs nt nt 256x2048", run_out_gs<1, 1, 256, 2048>, 1},
        {"out_gs nt nt 256x4096", run_out_gs<1, 1, 256, 4096>, 1},
        {"out_gs nt wt 256x2048", run_out_gs<1, 2, 256, 2048>, 1},
        {"mix (contiguous) nt wt", run_mix<1, 2, 256>, 0},
        {"mix (contiguous) nt nt", run_mix<1, 1, 256>, 0},
        {"copy nt", run_copy<1, 256>, 0, 10 * 1200.0},
    };
    std::vector<uint8_t> out(pb);
    for (auto& v : vars) { // warm + verify
        for (auto& s : sets)
            v.fn(s, G, st);
        CK(hipStreamSynchronize(st));
        if (v.check) {
            CK(hipMemcpy(out.data(), sets[0].par, pb, hipMemcpyDeviceToHost));
            if (memcmp(out.data(), ref.data(), pb) != 0) {
                fprintf(stderr, "MISMATCH %s\n", v.name);
                return 2;
            }
        }
    }
    std::vector<std::vector<float>> ts(vars.size());
    hipEvent_t e[64];
    for (int i = 0; i < 64; ++i)
        CK(hipEventCreate(&e[i]));
    int si = 0;
    for (int rd = 0; rd < rounds; ++rd)
        for (size_t vi = 0; vi < vars.size(); ++vi) {
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e[2 * r], st));
                vars[vi].fn(sets[si], G, st);
                CK(hipEventRecord(e[2 * r + 1], st));
                si = (si + 1) % NSETS;
            }
            CK(hipStreamSynchronize(st));
            for (int r = 0; r < reps; ++r) {
                float ms;
                CK(hipEventElapsedTime(&ms, e[2 * r], e[2 * r + 1]));
                ts[vi].push_back(ms * 1e3f);
            }
        }
    printf("%-32s %9s %9s %9s %7s\n", "variant", "med_us", "min_us", "GB/s", "frac8T");
    for (size_t vi = 0; vi < vars.size(); ++vi) {
        auto t = ts[vi];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2], mn = t[0];
        const double bytes = (double)G * vars[vi].bpg;
        printf("%-32s %9.1f %9.1f %9.1f %7.4f\n", vars[vi].name, med, mn, bytes / med / 1e3, bytes / med / 1e3 / 8000);
    }
    fflush(stdout);
    return 0;
}
