// svc_probe.hip -- measurement only (GPU box): host <-> device hand-off costs
// behind the drop-in's resident service (rfec_service.hip).
//
// NWG persistent workgroups poll a doorbell in pinned, host-coherent memory;
// on a ring each stages its 1/NWG of a payload the host has just rewritten
// (plain loads behind a system-scope acquire), XOR-folds it, writes the fold
// and its answer with system-coherent stores; the host spins until every
// answer is in and checks every fold (fresh data, no stale cache lines).
// Round trip per ring, for payload sizes and NWG = 1, 2, 4, 8.
//
// Prints one JSON object.  Build: hipcc --offload-arch=gfx950 -O3 tools/svc_probe.hip -o tools/bin/svc_probe
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Ctl {
    uint32_t bell, stop, pad0[14];
    uint32_t ans[16];
    uint32_t fold[16][4];
};

static double now_us()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

__global__ __launch_bounds__(256) void k_probe(Ctl* c, const v4u* pay, uint32_t nchunks, uint64_t life)
{
    __shared__ v4u red[256];
    __shared__ uint32_t s_cmd;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t w = blockIdx.x, nw = gridDim.x;
    const uint32_t lo = nchunks * w / nw, hi = nchunks * (w + 1) / nw;
    uint32_t done = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t cmd = 0xFFFFFFFFu;
            for (;;) {
                const uint32_t b = __hip_atomic_load(&c->bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (__hip_atomic_load(&c->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
                    break;
                if (b != done) {
                    cmd = b;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > life)
                    break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_cmd = cmd;
        }
        __syncthreads();
        const uint32_t cmd = s_cmd;
        if (cmd == 0xFFFFFFFFu)
            return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        constexpr int U = 16;
        v4u v[U];
        v4u x = v4u{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = lo + u * 256u + threadIdx.x;
            v[u] = pay[i < hi ? i : lo];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lo + u * 256u + threadIdx.x < hi)
                x ^= v[u];
        red[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t s = 128; s; s >>= 1) {
            if (threadIdx.x < s)
                red[threadIdx.x] ^= red[threadIdx.x + s];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const v4u f = red[0];
            for (int k = 0; k < 4; ++k)
                __hip_atomic_store(&c->fold[w][k], f[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(&c->ans[w], cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        done = cmd;
        __syncthreads();
    }
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd()
{
    rng ^= rng >> 12;
    rng ^= rng << 25;
    rng ^= rng >> 27;
    return (uint32_t)((rng * 2685821657736338717ull) >> 32);
}

int main()
{
    const size_t pay_max = 64 * 1024;
    uint8_t* h = nullptr;
    if (hipHostMalloc((void**)&h, 4096 + pay_max, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return 1;
    memset(h, 0, 4096 + pay_max);
    uint8_t* hd = nullptr;
    if (hipHostGetDevicePointer((void**)&hd, h, 0) != hipSuccess)
        return 1;
    Ctl* c = (Ctl*)h;
    uint32_t* pay = (uint32_t*)(h + 4096);
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return 1;
    printf("{");
    int first = 1, bad = 0;
    for (uint32_t nw : {1u, 2u, 4u, 8u}) {
        for (uint32_t bytes : {1024u, 12288u, 24576u}) {
            const uint32_t nch = bytes / 16;
            memset(c, 0, sizeof(Ctl));
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            hipLaunchKernelGGL(k_probe, dim3(nw), dim3(256), 0, s, (Ctl*)hd, (const v4u*)(hd + 4096), nch,
                               (uint64_t)200000000);
            if (hipGetLastError() != hipSuccess)
                return 1;
            double sum = 0, best = 1e30;
            int n = 0;
            for (uint32_t i = 1; i <= 2000; ++i) {
                for (uint32_t k = 0; k < bytes / 4; ++k)
                    pay[k] = rnd();
                const double t0 = now_us();
                __atomic_store_n(&c->bell, i, __ATOMIC_RELEASE);
                for (uint32_t w = 0; w < nw; ++w)
                    while (__atomic_load_n(&c->ans[w], __ATOMIC_ACQUIRE) != i)
                        if (now_us() - t0 > 1e6) {
                            fprintf(stderr, "no answer\n");
                            c->stop = 1;
                            (void)hipStreamSynchronize(s);
                            return 1;
                        }
                const double t1 = now_us();
                for (uint32_t w = 0; w < nw; ++w) { // fresh data: each workgroup's fold
                    const uint32_t lo = nch * w / nw, hi = nch * (w + 1) / nw;
                    uint32_t f[4] = {0, 0, 0, 0};
                    for (uint32_t q = lo; q < hi; ++q)
                        for (int k = 0; k < 4; ++k)
                            f[k] ^= pay[4 * q + k];
                    for (int k = 0; k < 4; ++k)
                        bad += f[k] != c->fold[w][k];
                }
                if (i > 20) {
                    sum += t1 - t0;
                    best = t1 - t0 < best ? t1 - t0 : best;
                    ++n;
                }
            }
            __atomic_store_n(&c->stop, 1u, __ATOMIC_RELEASE);
            (void)hipStreamSynchronize(s);
            printf("%s\"wg%u_%u\": {\"mean_us\": %.3f, \"min_us\": %.3f}", first ? "" : ",\n ", nw, bytes, sum / n,
                   best);
            first = 0;
        }
    }
    printf(",\n \"stale_folds\": %d}\n", bad);
    return bad ? 2 : 0;
}
