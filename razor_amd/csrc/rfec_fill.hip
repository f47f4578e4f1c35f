// rfec_fill.hip -- synthetic payload generator of SURVEY.md §8(d) on the
// device (bench and test inputs only; not on the FEC data path).
//
// Spec: xorshift64* (test/common_test.c:10-16): x ^= x >> 12; x ^= x << 25;
// x ^= x >> 27; out = x * 2685821657736338717.  State seeded with
// 0x52415A4F52464543 ("RAZORFEC") ^ config_id; payload bytes are the
// successive outputs, 8 little-endian bytes each (a slot of S bytes takes
// ceil(S / 8) outputs, the last one truncated), filled group-major,
// shard-major; bytes [S, stride) are zero.
//
// The state update is linear over GF(2), so the state n outputs ahead is
// T^n x: the host builds the 64 x 64 bit matrices J_j = T^(W * 2^j) (W =
// outputs per slot) by repeated squaring and the state at the launch's first
// slot; each device lane (one per slot) reaches its own slot's state with
// popcount(slot) matrix-vector products and then streams its W outputs.  A
// rank's slice [g0, g0 + groups) is therefore generated without the outputs
// before it (multi-GPU split, razor_amd/dist.py).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include "razor_fec.h"

namespace {

constexpr uint64_t kSeed = 0x52415A4F52464543ull;
constexpr uint64_t kMul = 2685821657736338717ull;
constexpr int kJumps = 40; // slot indices < 2^40
constexpr int kBlock = 256;

struct Mat {
    uint64_t col[64]; // col[b] = M * e_b
};

__host__ __device__ inline uint64_t mat_vec(const uint64_t* col, uint64_t x)
{
    uint64_t y = 0;
    for (int b = 0; b < 64; ++b)
        y ^= col[b] & (0ull - ((x >> b) & 1ull));
    return y;
}

inline uint64_t xs_step(uint64_t x)
{
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    return x;
}

inline Mat mat_mul(const Mat& a, const Mat& b) // a * b
{
    Mat c;
    for (int i = 0; i < 64; ++i)
        c.col[i] = mat_vec(a.col, b.col[i]);
    return c;
}

inline Mat mat_identity()
{
    Mat m;
    for (int i = 0; i < 64; ++i)
        m.col[i] = 1ull << i;
    return m;
}

inline Mat mat_pow(Mat m, uint64_t n)
{
    Mat r = mat_identity();
    while (n) {
        if (n & 1)
            r = mat_mul(m, r);
        m = mat_mul(m, m);
        n >>= 1;
    }
    return r;
}

inline Mat mat_step()
{
    Mat t;
    for (int i = 0; i < 64; ++i)
        t.col[i] = xs_step(1ull << i);
    return t;
}

__global__ __launch_bounds__(kBlock) void k_fill(uint8_t* __restrict__ shards, const uint64_t* __restrict__ jumps,
                                                 uint64_t x0, uint32_t slots, uint32_t S, uint32_t stride)
{
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= slots)
        return;
    uint64_t x = x0;
    for (int j = 0; j < 32; ++j)
        if ((s >> j) & 1u)
            x = mat_vec(jumps + (size_t)j * 64, x);
    uint8_t* d = shards + (size_t)s * stride;
    uint32_t b = 0;
    if ((stride & 7u) == 0) { // 8-byte aligned slots: one dwordx2 store per output
        for (; b + 8 <= S; b += 8) {
            x ^= x >> 12;
            x ^= x << 25;
            x ^= x >> 27;
            *reinterpret_cast<uint64_t*>(d + b) = x * kMul;
        }
    }
    for (; b < S; b += 8) {
        x ^= x >> 12;
        x ^= x << 25;
        x ^= x >> 27;
        const uint64_t v = x * kMul;
        for (uint32_t q = 0; q < 8 && b + q < S; ++q)
            d[b + q] = (uint8_t)(v >> (8 * q));
    }
    for (b = S; b < stride; ++b)
        d[b] = 0;
}

} // namespace

extern "C" {

uint64_t rfec_xorshift_jump(uint64_t x, uint64_t n) { return mat_vec(mat_pow(mat_step(), n).col, x); }

int rfec_fill_xorshift(uint8_t* shards, uint64_t config_id, uint64_t g0, uint32_t groups, uint32_t k, uint32_t S,
                       uint32_t stride, void* stream)
{
    if (!shards || !k || !S || stride < S || (uint64_t)groups * k >= (1ull << 32) ||
        (g0 + groups) * (uint64_t)k >= (1ull << kJumps))
        return RFEC_EINVAL;
    if (!groups)
        return RFEC_OK;
    const uint64_t W = (S + 7) / 8;
    const Mat t = mat_step();
    Mat jw = mat_pow(t, W);
    static_assert(sizeof(Mat) == 512, "matrix layout");
    uint64_t hj[32 * 64];
    for (int j = 0; j < 32; ++j) {
        memcpy(hj + (size_t)j * 64, jw.col, sizeof(jw.col));
        jw = mat_mul(jw, jw);
    }
    const uint64_t x0 = mat_vec(mat_pow(t, W * g0 * k).col, kSeed ^ config_id);
    uint64_t* dj = nullptr;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (hipMallocAsync(reinterpret_cast<void**>(&dj), sizeof(hj), st) != hipSuccess)
        return RFEC_EDEVICE;
    hipError_t e = hipMemcpyAsync(dj, hj, sizeof(hj), hipMemcpyHostToDevice, st);
    const uint32_t slots = groups * k;
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_fill, dim3((slots + kBlock - 1) / kBlock), dim3(kBlock), 0, st, shards, dj, x0, slots, S,
                           stride);
        e = hipGetLastError();
    }
    // the host copy of the matrices must outlive the async H2D
    const hipError_t e2 = hipStreamSynchronize(st);
    hipFreeAsync(dj, st);
    return (e == hipSuccess && e2 == hipSuccess) ? RFEC_OK : RFEC_EDEVICE;
}

} // extern "C"
