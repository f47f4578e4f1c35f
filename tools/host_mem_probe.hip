// CPU read cost of pinned host memory the device wrote, by allocation flag (hipHostMalloc Default / Mapped /
// Mapped|NonCoherent / Mapped|Coherent, hipHostRegister'd malloc, plain malloc): a kernel writes the buffer,
// then the host reads it with 8-byte loads (a dependent-free sum) and with memcpy into a private buffer.
// Build: hipcc --offload-arch=gfx950 -O2 tools/host_mem_probe.hip -o /tmp/host_mem_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void fill(uint64_t* p, size_t n, uint64_t v)
{
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v + i;
}
static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void probe(const char* name, uint64_t* h, uint64_t* d, size_t bytes)
{
    const size_t n = bytes / 8;
    std::vector<uint64_t> priv(n);
    double best_sum = 1e30, best_cpy = 1e30, best_cached = 1e30;
    uint64_t acc = 0;
    for (int rep = 0; rep < 5; ++rep) {
        if (d) {
            fill<<<256, 256>>>(d, n, rep);
            (void)hipDeviceSynchronize();
        } else {
            for (size_t i = 0; i < n; ++i)
                h[i] = rep + i;
        }
        double t = now_us();
        for (size_t i = 0; i < n; ++i)
            acc += h[i];
        best_sum = std::min(best_sum, now_us() - t);
        t = now_us();
        for (size_t i = 0; i < n; ++i) // again: whatever the first pass left in the caches
            acc += h[i];
        best_cached = std::min(best_cached, now_us() - t);
        if (d) {
            fill<<<256, 256>>>(d, n, rep + 1);
            (void)hipDeviceSynchronize();
        }
        t = now_us();
        memcpy(priv.data(), h, bytes);
        best_cpy = std::min(best_cpy, now_us() - t);
        acc += priv[n / 2];
    }
    printf("%-28s %8zu B: 8-B loads %8.1f us (%6.2f GB/s), again %8.1f us, memcpy %8.1f us (%6.2f GB/s)  [%llu]\n",
           name, bytes, best_sum, bytes / best_sum / 1e3, best_cached, best_cpy, bytes / best_cpy / 1e3,
           (unsigned long long)(acc & 1));
}
int main()
{
    for (size_t bytes : {(size_t)32768, (size_t)262144, (size_t)4 << 20}) {
        struct { const char* name; unsigned flags; } kinds[] = {
            {"hipHostMalloc Default", hipHostMallocDefault},
            {"hipHostMalloc Mapped", hipHostMallocMapped},
            {"Mapped|NonCoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
            {"Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent},
        };
        for (auto& k : kinds) {
            void* h = nullptr;
            void* d = nullptr;
            if (hipHostMalloc(&h, bytes, k.flags) != hipSuccess || hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
                printf("%s: alloc failed\n", k.name);
                continue;
            }
            probe(k.name, (uint64_t*)h, (uint64_t*)d, bytes);
            (void)hipHostFree(h);
        }
        void* m = aligned_alloc(4096, bytes);
        memset(m, 1, bytes);
        void* d = nullptr;
        if (hipHostRegister(m, bytes, hipHostRegisterMapped) == hipSuccess && hipHostGetDevicePointer(&d, m, 0) == hipSuccess) {
            probe("malloc + hipHostRegister", (uint64_t*)m, (uint64_t*)d, bytes);
            (void)hipHostUnregister(m);
        }
        probe("malloc (CPU-written)", (uint64_t*)m, nullptr, bytes);
        free(m);
    }
    return 0;
}
