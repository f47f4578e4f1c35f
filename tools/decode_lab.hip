// decode_lab.hip -- A/B lab for the k = 10 / 1,200-B row decode (payload
// only, 2 erasures per group in distinct rows): which lane mapping and store
// shape brings the scattered in-place recovery closest to the HBM ceiling.
// Measurement only; not on the product path.  The parity operand is cold:
// NSETS disjoint sets are rotated, so nothing is MALL-resident.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/decode_lab.hip -o tools/bin/decode_lab
// run:   tools/bin/decode_lab [groups=65536] [rounds=7] [reps=10]
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

constexpr int K = 10, R = 3, COL = 4, CH = 75;

__device__ __forceinline__ v4u ld(const v4u* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(v4u* p, v4u v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ uint32_t row_mask(uint32_t r) { return r < 2 ? 0xFu << (4 * r) : 0x300u; }

// D0: flat (group, chunk) lanes, both fired rows' loads in flight
__global__ __launch_bounds__(256) void k_flat(v4u* __restrict__ sh, const v4u* __restrict__ par,
                                              const uint32_t* __restrict__ pres, uint32_t total)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / CH, c = t - g * CH;
    const uint32_t h = pres[g];
    v4u* s = sh + (size_t)g * K * CH + c;
    const v4u* p = par + (size_t)g * R * CH + c;
    v4u acc[2], mv[2][COL];
    uint32_t tg[2];
    bool on[2];
    uint32_t fire = 0;
    for (uint32_t r = 0; r < R; ++r)
        if (__popc(row_mask(r) & ~h) == 1)
            fire |= 1u << r;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        on[b] = fire != 0;
        const uint32_t r = on[b] ? __ffs(fire) - 1 : 0;
        fire &= fire - 1;
        acc[b] = on[b] ? ld(p + r * CH) : v4u{0, 0, 0, 0};
        tg[b] = r * COL;
#pragma unroll
        for (int q = 0; q < COL; ++q) {
            const uint32_t i = r * COL + q;
            mv[b][q] = v4u{0, 0, 0, 0};
            if (!on[b] || i >= K)
                continue;
            if ((h >> i) & 1)
                mv[b][q] = ld(s + i * CH);
            else
                tg[b] = i;
        }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int q = 0; q < COL; ++q)
            acc[b] ^= mv[b][q];
        if (on[b])
            st(s + tg[b] * CH, acc[b]);
    }
}

// D1: output-mapped, one lane per (group, row, chunk); rows that do not fire exit
template <int MODE> // 0 in place, 1 dense output [G][2][CH], 2 no store (reads only)
__global__ __launch_bounds__(256) void k_out(v4u* __restrict__ sh, const v4u* __restrict__ par,
                                             const uint32_t* __restrict__ pres, v4u* __restrict__ dense,
                                             uint32_t total)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / (R * CH), rem = t - g * (R * CH);
    const uint32_t r = rem / CH, c = rem - r * CH;
    const uint32_t h = pres[g];
    const uint32_t miss = row_mask(r) & ~h;
    if (__popc(miss) != 1)
        return;
    const uint32_t tgt = __ffs(miss) - 1;
    v4u* s = sh + ((size_t)g * K + r * COL) * CH + c;
    v4u acc = ld(par + t);
    v4u mv[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q) {
        mv[q] = v4u{0, 0, 0, 0};
        if (r * COL + q < K && ((h >> (r * COL + q)) & 1))
            mv[q] = ld(s + q * CH);
    }
#pragma unroll
    for (int q = 0; q < COL; ++q)
        acc ^= mv[q];
    if constexpr (MODE == 0) {
        st(sh + ((size_t)g * K + tgt) * CH + c, acc);
    } else if constexpr (MODE == 1) {
        const uint32_t e = __popc(~h & 0x3FFu & ((1u << tgt) - 1)); // which erasure of the group
        st(dense + ((size_t)g * 2 + e) * CH + c, acc);
    } else {
        if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u)
            dense[t & 1023] = acc;
    }
}

// D2: output-mapped over the line-aligned span of the target slot: lanes
// outside the slot write the neighbour's bytes back unchanged (when the
// neighbour is present), so every line of the span is written whole
constexpr int SPAN = 88; // chunks of the widest line-aligned span of a 1,200-B slot (11 lines)
__global__ __launch_bounds__(256) void k_aligned(v4u* __restrict__ sh, const v4u* __restrict__ par,
                                                 const uint32_t* __restrict__ pres, uint32_t total, uint32_t G)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / (R * SPAN), rem = t - g * (R * SPAN);
    const uint32_t r = rem / SPAN, i = rem - r * SPAN;
    const uint32_t h = pres[g];
    const uint32_t miss = row_mask(r) & ~h;
    if (__popc(miss) != 1)
        return;
    const uint32_t tgt = __ffs(miss) - 1;
    const uint64_t slot = (uint64_t)g * K + tgt;
    const uint64_t base = slot * CH; // chunk index of the slot's first chunk
    const uint64_t a0 = (base * 16) & ~127ull;
    const uint64_t a = a0 / 16 + i; // this lane's chunk
    const uint64_t a1 = (base * 16 + 1200 + 127) & ~127ull;
    if (a * 16 >= a1)
        return;
    if (a < base || a >= base + CH) { // neighbour's chunk of an edge line
        const uint64_t ns = a < base ? slot - 1 : slot + 1;
        if (ns >= (uint64_t)G * K)
            return;
        const uint32_t ng = (uint32_t)(ns / K), ni = (uint32_t)(ns - (uint64_t)ng * K);
        if (!((pres[ng] >> ni) & 1))
            return; // the neighbour is being recovered too: leave it a partial write
        st(sh + a, ld(sh + a));
        return;
    }
    const uint32_t c = (uint32_t)(a - base);
    v4u* s = sh + ((size_t)g * K + r * COL) * CH + c;
    v4u acc = ld(par + ((size_t)g * R + r) * CH + c);
    v4u mv[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q) {
        mv[q] = v4u{0, 0, 0, 0};
        if (r * COL + q < K && ((h >> (r * COL + q)) & 1))
            mv[q] = ld(s + q * CH);
    }
#pragma unroll
    for (int q = 0; q < COL; ++q)
        acc ^= mv[q];
    st(sh + a, acc);
}

__global__ void k_encode(const v4u* __restrict__ sh, v4u* __restrict__ par, uint32_t total)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = t / (R * CH), rem = t - g * (R * CH);
    const uint32_t r = rem / CH, c = rem - r * CH;
    v4u a = {0, 0, 0, 0};
    for (int q = 0; q < COL; ++q)
        if (r * COL + q < K)
            a ^= sh[((size_t)g * K + r * COL + q) * CH + c];
    par[t] = a;
}

__global__ void k_copy(const v4u* __restrict__ a, v4u* __restrict__ b, uint32_t n)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t < n)
        st(b + t, ld(a + t));
}

struct Set {
    v4u *orig, *rx, *par, *dense;
    uint32_t* pres;
};

int main(int argc, char** argv)
{
    const uint32_t G = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int NSETS = 3;
    const size_t shb = (size_t)G * K * CH * 16, pb = (size_t)G * R * CH * 16, db = (size_t)G * 2 * CH * 16;
    std::vector<uint8_t> h(shb);
    uint64_t x = 0x52415A4F52464543ull;
    for (size_t i = 0; i < shb; i += 8) {
        x ^= x >> 12;
        x ^= x << 25;
        x ^= x >> 27;
        uint64_t v = x * 2685821657736338717ull;
        memcpy(&h[i], &v, 8);
    }
    // two erasures per group in distinct rows
    std::vector<uint32_t> pres(G);
    const int rows[3][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {8, 9, -1, -1}};
    std::vector<std::pair<int, int>> pairs;
    for (int r1 = 0; r1 < 3; ++r1)
        for (int r2 = r1 + 1; r2 < 3; ++r2)
            for (int a : rows[r1])
                for (int b : rows[r2])
                    if (a >= 0 && b >= 0)
                        pairs.push_back({a, b});
    uint64_t y = 12345;
    double alg = 0;
    for (uint32_t g = 0; g < G; ++g) {
        y ^= y << 13;
        y ^= y >> 7;
        y ^= y << 17;
        auto pr = pairs[y % pairs.size()];
        pres[g] = 0x3FFu & ~(1u << pr.first) & ~(1u << pr.second);
        for (int e : {pr.first, pr.second})
            alg += ((e < 8) ? 5 : 3) * 1200.0;
    }
    std::vector<Set> sets(NSETS);
    hipStream_t st_;
    CK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    for (auto& s : sets) {
        CK(hipMalloc(&s.orig, shb));
        CK(hipMalloc(&s.rx, shb));
        CK(hipMalloc(&s.par, pb));
        CK(hipMalloc(&s.dense, db));
        CK(hipMalloc(&s.pres, G * 4));
        CK(hipMemcpy(s.orig, h.data(), shb, hipMemcpyHostToDevice));
        CK(hipMemcpy(s.rx, h.data(), shb, hipMemcpyHostToDevice));
        CK(hipMemcpy(s.pres, pres.data(), G * 4, hipMemcpyHostToDevice));
        const uint32_t tot = G * R * CH;
        hipLaunchKernelGGL(k_encode, dim3((tot + 255) / 256), dim3(256), 0, st_, s.orig, s.par, tot);
    }
    CK(hipStreamSynchronize(st_));
    struct Var {
        const char* name;
        int kind;
        double bytes;
    };
    std::vector<Var> vars = {{"flat (product shape)", 0, alg},   {"out in place", 1, alg},
                             {"out line-aligned spans", 2, alg}, {"out dense output", 3, alg},
                             {"out reads only", 4, alg * 0.0},   {"copy nt", 5, (double)G * 2 * 5400}};
    for (auto& v : vars)
        if (v.kind == 4)
            v.bytes = alg - (double)G * 2 * 1200; // reads of the two fired rows
    auto launch = [&](int kind, Set& s) {
        switch (kind) {
        case 0: {
            const uint32_t tot = G * CH;
            hipLaunchKernelGGL(k_flat, dim3((tot + 255) / 256), dim3(256), 0, st_, s.rx, s.par, s.pres, tot);
            break;
        }
        case 1:
        case 3:
        case 4: {
            const uint32_t tot = G * R * CH;
            if (kind == 1)
                hipLaunchKernelGGL(k_out<0>, dim3((tot + 255) / 256), dim3(256), 0, st_, s.rx, s.par, s.pres, s.dense, tot);
            else if (kind == 3)
                hipLaunchKernelGGL(k_out<1>, dim3((tot + 255) / 256), dim3(256), 0, st_, s.rx, s.par, s.pres, s.dense, tot);
            else
                hipLaunchKernelGGL(k_out<2>, dim3((tot + 255) / 256), dim3(256), 0, st_, s.rx, s.par, s.pres, s.dense, tot);
            break;
        }
        case 2: {
            const uint32_t tot = G * R * SPAN;
            hipLaunchKernelGGL(k_aligned, dim3((tot + 255) / 256), dim3(256), 0, st_, s.rx, s.par, s.pres, tot, G);
            break;
        }
        case 5: {
            const uint32_t n = G * 2 * 5400 / 32;
            hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, st_, s.orig, s.rx, n);
            break;
        }
        }
    };
    // verify the in-place variants: rx must equal orig after a decode (erased slots start as garbage)
    for (int kind : {0, 1, 2}) {
        Set& s = sets[0];
        CK(hipMemset(s.rx, 0xA5, shb));
        // restore the present slots
        std::vector<uint8_t> rxh(h);
        for (uint32_t g = 0; g < G; ++g)
            for (int i = 0; i < K; ++i)
                if (!((pres[g] >> i) & 1))
                    memset(&rxh[((size_t)g * K + i) * 1200], 0xA5, 1200);
        CK(hipMemcpy(s.rx, rxh.data(), shb, hipMemcpyHostToDevice));
        launch(kind, s);
        CK(hipStreamSynchronize(st_));
        CK(hipMemcpy(rxh.data(), s.rx, shb, hipMemcpyDeviceToHost));
        if (memcmp(rxh.data(), h.data(), shb) != 0) {
            fprintf(stderr, "MISMATCH kind %d\n", kind);
            return 2;
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
                CK(hipEventRecord(e[2 * r], st_));
                launch(vars[vi].kind, sets[si]);
                CK(hipEventRecord(e[2 * r + 1], st_));
                si = (si + 1) % NSETS;
            }
            CK(hipStreamSynchronize(st_));
            for (int r = 0; r < reps; ++r) {
                float ms;
                CK(hipEventElapsedTime(&ms, e[2 * r], e[2 * r + 1]));
                ts[vi].push_back(ms * 1e3f);
            }
        }
    printf("%-28s %9s %9s %9s %7s\n", "variant", "med_us", "min_us", "GB/s", "frac8T");
    for (size_t vi = 0; vi < vars.size(); ++vi) {
        auto t = ts[vi];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2], mn = t[0];
        printf("%-28s %9.1f %9.1f %9.1f %7.4f\n", vars[vi].name, med, mn, vars[vi].bytes / med / 1e3,
               vars[vi].bytes / med / 1e3 / 8000);
    }
    printf("algorithmic decode bytes %.0f (%.1f per group)\n", alg, alg / G);
    return 0;
}
