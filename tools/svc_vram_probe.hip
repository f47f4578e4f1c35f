// svc_vram_probe.hip -- measurement only (GPU box): does staging a service job
// in device memory the HOST writes (through the BAR mapping of a fine-grained
// VRAM allocation) beat the service's current hand-off, where the device reads
// the job from pinned host memory (one PCIe read round trip per job)?
//
// One persistent workgroup polls a doorbell; on a ring it loads the payload
// (plain loads behind a system-scope acquire, as rfec_service.hip), XOR-folds
// it and writes fold + answer with system-coherent stores to pinned host
// memory.  The host rewrites the payload (random words), then rings.  Modes:
//   bell host / vram  x  payload host / vram
// Per mode: the host's write of the payload (memcpy + sfence), the doorbell ->
// answer round trip, their sum, and stale folds (must be 0).
//
// First it probes which VRAM allocations the host can write at all (a
// SIGSEGV handler turns a fault into "no").
//
// Prints one JSON object.  Build: hipcc --offload-arch=gfx950 -O3 tools/svc_vram_probe.hip -o tools/bin/svc_vram_probe
#include <hip/hip_runtime.h>

#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Bell {
    uint32_t bell, stop, pad[14];
};
struct Ans {
    uint32_t ans, pad0[15];
    uint32_t fold[4], pad1[12];
};

static double now_us()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

__global__ __launch_bounds__(256) void k_probe(const Bell* b, Ans* a, const v4u* pay, uint32_t nchunks, uint64_t life)
{
    __shared__ v4u red[256];
    __shared__ uint32_t s_cmd;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t done = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t cmd = 0xFFFFFFFFu;
            for (;;) {
                const uint32_t v = __hip_atomic_load(&b->bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (__hip_atomic_load(&b->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
                    break;
                if (v != done) {
                    cmd = v;
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
        constexpr int U = 4;
        v4u v[U];
        v4u x = v4u{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = u * 256u + threadIdx.x;
            v[u] = pay[i < nchunks ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u * 256u + threadIdx.x < nchunks)
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
                __hip_atomic_store(&a->fold[k], f[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(&a->ans, cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// 1 when the host can write and read back `p` (a VRAM allocation)
static int host_can_write(volatile uint32_t* p)
{
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    int ok = 0;
    if (sigsetjmp(g_jb, 1) == 0) {
        p[0] = 0x5A5A1234u;
        __builtin_ia32_sfence();
        ok = p[0] == 0x5A5A1234u;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

int main(int argc, char** argv)
{
    const int want = argc > 1 ? atoi(argv[1]) : -1; // VRAM allocation to use: 0 hipMalloc, 1 fine-grained, 2 uncached
    const uint32_t bytes = 12288, nch = bytes / 16;
    // host side: bell, answer, payload
    uint8_t* h = nullptr;
    if (hipHostMalloc((void**)&h, 8192 + bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return 1;
    memset(h, 0, 8192 + bytes);
    uint8_t* hd = nullptr;
    if (hipHostGetDevicePointer((void**)&hd, h, 0) != hipSuccess)
        return 1;
    Bell* hb = (Bell*)h;
    Ans* ha = (Ans*)(h + 4096);
    uint32_t* hpay = (uint32_t*)(h + 8192);

    // VRAM candidates
    struct Cand {
        const char* name;
        uint8_t* p;
        int ok;
    } cand[3] = {{"hipMalloc", nullptr, 0}, {"finegrained", nullptr, 0}, {"uncached", nullptr, 0}};
    (void)hipMalloc((void**)&cand[0].p, 8192 + bytes);
    (void)hipExtMallocWithFlags((void**)&cand[1].p, 8192 + bytes, hipDeviceMallocFinegrained);
    (void)hipExtMallocWithFlags((void**)&cand[2].p, 8192 + bytes, hipDeviceMallocUncached);
    (void)hipGetLastError();
    printf("{\"alloc\": {");
    int pick = -1;
    for (int c = 0; c < 3; ++c) {
        int hostp = 0;
        if (cand[c].p) {
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, cand[c].p) == hipSuccess)
                hostp = at.hostPointer != nullptr;
            (void)hipGetLastError();
            cand[c].ok = host_can_write((volatile uint32_t*)cand[c].p);
        }
        printf("%s\"%s\": {\"allocated\": %d, \"host_pointer_attr\": %d, \"host_write\": %d}", c ? ", " : "",
               cand[c].name, cand[c].p != nullptr, hostp, cand[c].ok);
        if (cand[c].ok && pick < 0 && (want < 0 ? c > 0 : c == want))
            pick = c;
    }
    printf("}");
    if (pick < 0) {
        printf(", \"vram_host_write\": false}\n");
        return 0;
    }
    printf(", \"vram\": \"%s\"", cand[pick].name);
    uint8_t* v = cand[pick].p;
    memset(v, 0, 8192 + bytes);
    __builtin_ia32_sfence();
    Bell* vb = (Bell*)v;
    uint32_t* vpay = (uint32_t*)(v + 8192);

    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return 1;
    static uint32_t src[12288 / 4];
    int bad_total = 0;
    for (int mode = 0; mode < 4; ++mode) {
        const int bell_vram = mode & 1, pay_vram = (mode >> 1) & 1;
        Bell* b = bell_vram ? vb : hb;            // host view (VRAM: same address)
        const Bell* bdev = bell_vram ? vb : (Bell*)hd;
        uint32_t* pay = pay_vram ? vpay : hpay;
        const v4u* pdev = pay_vram ? (const v4u*)vpay : (const v4u*)(hd + 8192);
        memset(b, 0, sizeof(Bell));
        memset(ha, 0, sizeof(Ans));
        __builtin_ia32_sfence();
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(256), 0, s, bdev, (Ans*)(hd + 4096), pdev, nch,
                           (uint64_t)300000000);
        if (hipGetLastError() != hipSuccess)
            return 1;
        double sw = 0, sr = 0, best = 1e30;
        int n = 0, bad = 0;
        static double rt[3000];
        for (uint32_t i = 1; i <= 3000; ++i) {
            for (uint32_t k = 0; k < bytes / 4; ++k)
                src[k] = rnd();
            const double t0 = now_us();
            memcpy(pay, src, bytes);
            __builtin_ia32_sfence();
            const double t1 = now_us();
            __atomic_store_n(&b->bell, i, __ATOMIC_RELEASE);
            __builtin_ia32_sfence();
            while (__atomic_load_n(&ha->ans, __ATOMIC_ACQUIRE) != i)
                if (now_us() - t1 > 1e6) {
                    fprintf(stderr, "no answer (mode %d)\n", mode);
                    b->stop = 1;
                    hb->stop = 1;
                    __builtin_ia32_sfence();
                    (void)hipStreamSynchronize(s);
                    return 1;
                }
            const double t2 = now_us();
            uint32_t f[4] = {0, 0, 0, 0};
            for (uint32_t q = 0; q < nch; ++q)
                for (int k = 0; k < 4; ++k)
                    f[k] ^= src[4 * q + k];
            for (int k = 0; k < 4; ++k)
                bad += f[k] != ha->fold[k];
            if (i > 50) {
                sw += t1 - t0;
                sr += t2 - t1;
                rt[n] = t2 - t0;
                best = t2 - t0 < best ? t2 - t0 : best;
                ++n;
            }
        }
        __atomic_store_n(&b->stop, 1u, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();
        (void)hipStreamSynchronize(s);
        // median of the totals
        for (int i = 1; i < n; ++i)
            for (int j = i; j > 0 && rt[j - 1] > rt[j]; --j) {
                const double t = rt[j];
                rt[j] = rt[j - 1];
                rt[j - 1] = t;
            }
        printf(",\n \"bell_%s_pay_%s\": {\"write_us\": %.3f, \"ring_us\": %.3f, \"total_mean_us\": %.3f, "
               "\"total_median_us\": %.3f, \"total_min_us\": %.3f, \"stale_folds\": %d}",
               bell_vram ? "vram" : "host", pay_vram ? "vram" : "host", sw / n, sr / n, (sw + sr) / n, rt[n / 2],
               best, bad);
        bad_total += bad;
    }
    printf("}\n");
    return bad_total ? 2 : 0;
}
