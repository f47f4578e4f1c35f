// sclk_probe.hip -- measurement only (GPU box): the shader clock a lone
// resident workgroup runs at, the situation of the drop-in's service kernel
// (one workgroup on an otherwise idle GPU).  s_memtime counts shader clocks,
// s_memrealtime a constant 100 MHz; their ratio over a burst of dependent VALU
// work is the clock.  Bursts after 0, 10 us, 100 us and 1 ms of s_sleep
// polling, one workgroup; then the same while a second stream keeps the GPU
// busy with a streaming kernel.
//
// Prints one JSON object.  Build: hipcc --offload-arch=gfx950 -O3 tools/sclk_probe.hip -o tools/bin/sclk_probe
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(64) void k_clock(uint64_t* out, uint32_t reps)
{
    const uint64_t idle_ticks[4] = {0, 1000, 10000, 100000}; // 100 MHz ticks: 0, 10 us, 100 us, 1 ms
    float x = threadIdx.x;
    for (int k = 0; k < 4; ++k) {
        const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - w0 < idle_ticks[k])
            __builtin_amdgcn_s_sleep(2);
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
        for (uint32_t i = 0; i < reps; ++i)
            x = __builtin_fmaf(x, 1.000001f, 0.5f);
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) {
            out[2 * k] = r1 - r0;
            out[2 * k + 1] = c1 - c0;
        }
    }
    // latency of a dependent chain of 64 s_memrealtime / s_memtime (shader clocks each)
    uint64_t acc = 0;
    const uint64_t m0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) { // each value consumed before the next is read
        const uint64_t v = __builtin_amdgcn_s_memrealtime();
        __asm__ volatile("; use %0" ::"s"(v));
        acc += v & 1u;
    }
    const uint64_t m1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) {
        const uint64_t v = __builtin_amdgcn_s_memtime();
        __asm__ volatile("; use %0" ::"s"(v));
        acc += v & 1u;
    }
    const uint64_t m2 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[8] = (m1 - m0) / 64;
        out[9] = (m2 - m1) / 64;
    }
    if (x == 12345.f || acc == 12345)
        out[15] = 1;
}

__global__ void k_stream(float4* p, size_t n, int iters)
{
    for (int it = 0; it < iters; ++it)
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
            p[i] = make_float4(p[i].x + 1.f, p[i].y, p[i].z, p[i].w);
}

int main()
{
    uint64_t* d = nullptr;
    if (hipMalloc(&d, 16 * sizeof(uint64_t)) != hipSuccess)
        return 1;
    float4* buf = nullptr;
    const size_t n = (size_t)1 << 26; // 1 GiB
    if (hipMalloc(&buf, n * sizeof(float4)) != hipSuccess)
        return 1;
    (void)hipMemset(buf, 0, n * sizeof(float4));
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    printf("{");
    const char* names[4] = {"after_0us", "after_10us", "after_100us", "after_1ms"};
    for (int busy = 0; busy < 2; ++busy) {
        (void)hipDeviceSynchronize();
        if (busy)
            hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, s2, buf, n, 20);
        hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, s1, d, 20000u);
        uint64_t h[16];
        if (hipStreamSynchronize(s1) != hipSuccess || hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
            return 1;
        (void)hipDeviceSynchronize();
        printf("%s\"%s\": {", busy ? ", " : "", busy ? "gpu_busy" : "gpu_idle");
        for (int k = 0; k < 4; ++k)
            printf("%s\"%s_MHz\": %.0f", k ? ", " : "", names[k],
                   h[2 * k] ? 100.0 * (double)h[2 * k + 1] / (double)h[2 * k] : 0.0);
        printf(", \"memrealtime_clk\": %llu, \"memtime_clk\": %llu}", (unsigned long long)h[8],
               (unsigned long long)h[9]);
    }
    printf("}\n");
    return 0;
}
