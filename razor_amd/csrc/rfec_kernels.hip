// rfec_kernels.hip -- CDNA4 (gfx950) kernels of the flex-FEC engine, plus the
// thin extern "C" launch shim the C host layer (rfec_host.c) calls.
//
// Arithmetic restated from the reference (yuanrongxi/razor):
//   parity payload  = XOR of zero-padded member payloads  flex_fec_xor.c:30-32, 46-49
//   parity meta     = XOR of member headers, max data_size flex_fec_xor.c:13-26, 37-44
//   recovery        = parity ^ XOR of present members      flex_fec_xor.c:64-95
//   peeling order / conditions                             flex_fec_receiver.c:105-206
//
// Device layout (include/razor_fec.h): payload slots of `stride` bytes
// (multiple of 16), zero beyond data_size; one lane owns one 16-byte chunk
// column of one group and walks every line of that group, so all arithmetic
// is wave64 v_xor_b32 on dwordx4 registers: no LDS, no MFMA (XOR is the only
// operation, ~0.06 op/B -> HBM-bound).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rfec_internal.h"

namespace {

constexpr int kBlock = 256;

// CUTLASS-style fast unsigned division for dividends < 2^31.
struct FastDiv {
    uint32_t d, m, s;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f)
{
    uint64_t hi = __umulhi(n, f.m);
    return (uint32_t)((hi + n) >> f.s);
}

// native 16-byte vector (the nontemporal builtins need a clang vector type)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u xor4(v4u a, v4u b) { return a ^ b; }

template <bool NT>
__device__ __forceinline__ v4u ld16(const v4u* p)
{
    if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

template <bool NT>
__device__ __forceinline__ void st16(v4u* p, v4u v)
{
    if constexpr (NT) {
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

struct Hdr5 {
    uint32_t w[5];
};

__device__ __forceinline__ Hdr5 ldh(const rfec_hdr* h)
{
    const uint32_t* p = reinterpret_cast<const uint32_t*>(h);
    Hdr5 r;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        r.w[i] = p[i];
    return r;
}

__device__ __forceinline__ void sth(rfec_hdr* h, const Hdr5& r)
{
    uint32_t* p = reinterpret_cast<uint32_t*>(h);
#pragma unroll
    for (int i = 0; i < 5; ++i)
        p[i] = r.w[i];
}

__device__ __forceinline__ uint32_t hsize(const Hdr5& h) { return h.w[4] >> 16; }

// Parity meta of line l of group g: XOR of the member headers as five dwords
// (field-wise XOR, flex_fec_xor.c:13-20, 37-44) and L = max data_size
// (:22-26); status -1 where flex_fec_generate fails (:9-10, :27-28).
__device__ __forceinline__ void encode_meta(const rfec_hdr* __restrict__ hdr, rfec_hdr* __restrict__ meta,
                                            uint16_t* __restrict__ fsize, int8_t* __restrict__ status,
                                            uint32_t g, uint32_t l, const rfec_kplan& P, uint32_t capacity)
{
    const rfec_line ln = P.line[l];
    const rfec_hdr* hg = hdr + (size_t)g * P.k;
    Hdr5 m = {{0, 0, 0, 0, 0}};
    uint32_t L = 0;
    for (uint32_t q = 0; q < ln.count; ++q) {
        Hdr5 h = ldh(hg + ln.first + q * ln.stride);
#pragma unroll
        for (int i = 0; i < 5; ++i)
            m.w[i] ^= h.w[i];
        L = max(L, hsize(h));
    }
    const size_t o = (size_t)g * P.n_lines + l;
    sth(meta + o, m);
    fsize[o] = (uint16_t)L;
    if (status)
        status[o] = (ln.count <= 1 || L > capacity) ? (int8_t)-1 : (int8_t)0;
}

// ---------------------------------------------------------------------------
// Encode, generic plan: one lane per (group, 16-B chunk column).
// ---------------------------------------------------------------------------
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_encode(const v4u* __restrict__ shards,
                                                   const rfec_hdr* __restrict__ hdr, v4u* __restrict__ parity,
                                                   rfec_hdr* __restrict__ meta, uint16_t* __restrict__ fsize,
                                                   int8_t* __restrict__ status, uint32_t total, uint32_t C,
                                                   FastDiv divC, uint32_t capacity, rfec_kplan P)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * C;
    const v4u* src = shards + (size_t)g * P.k * C + j;
    v4u* dst = parity + (size_t)g * P.n_lines * C + j;
    for (uint32_t l = 0; l < P.n_lines; ++l) {
        const rfec_line ln = P.line[l];
        const v4u* s = src + (size_t)ln.first * C;
        const size_t step = (size_t)ln.stride * C;
        v4u acc = ld16<NT>(s);
        for (uint32_t q = 1; q < ln.count; ++q)
            acc = xor4(acc, ld16<NT>(s + q * step));
        st16<NT>(dst + (size_t)l * C, acc);
    }
    if (j < P.n_lines)
        encode_meta(hdr, meta, fsize, status, g, j, P, capacity);
}

// ---------------------------------------------------------------------------
// Encode, rows-of-COL fast path (the k=10 / rows {4,4,2} and k=32 / 8x4
// configurations): every member offset is a compile-time constant, so all K
// dwordx4 loads of a lane issue back to back before the first XOR.
// ---------------------------------------------------------------------------
template <int K, int COL, bool NT>
__global__ __launch_bounds__(kBlock) void k_encode_rows(const v4u* __restrict__ shards,
                                                        const rfec_hdr* __restrict__ hdr,
                                                        v4u* __restrict__ parity, rfec_hdr* __restrict__ meta,
                                                        uint16_t* __restrict__ fsize, int8_t* __restrict__ status,
                                                        uint32_t total, uint32_t C, FastDiv divC,
                                                        uint32_t capacity, rfec_kplan P)
{
    constexpr int R = (K + COL - 1) / COL;
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * C;
    const v4u* src = shards + (size_t)g * K * C + j;
    v4u* dst = parity + (size_t)g * R * C + j;
    v4u v[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        v[i] = ld16<NT>(src + (size_t)i * C);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v4u acc = v[r * COL];
#pragma unroll
        for (int q = 1; q < COL; ++q)
            if (r * COL + q < K)
                acc = xor4(acc, v[r * COL + q]);
        st16<NT>(dst + (size_t)r * C, acc);
    }
    if (j < (uint32_t)R)
        encode_meta(hdr, meta, fsize, status, g, j, P, capacity);
}

// ---------------------------------------------------------------------------
// Peeling schedule: one lane per group.  Fixpoint of flex_recover_row/col
// (flex_fec_receiver.c:105-206) with the cascade of sim_receiver.c:780-804,
// lines in plan order, repeated until nothing fires.  Writes the recovered
// headers (flex_fec_xor.c:64-85) and the step list the XOR kernel replays.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_peel(rfec_hdr* __restrict__ hdr, const uint64_t* __restrict__ present,
                                                 const rfec_hdr* __restrict__ meta,
                                                 const uint16_t* __restrict__ fsize,
                                                 const uint64_t* __restrict__ parity_present,
                                                 uint64_t* __restrict__ recovered, rfec_step* __restrict__ ws,
                                                 uint32_t groups, uint32_t ws_stride, uint32_t capacity,
                                                 rfec_kmask M)
{
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= groups)
        return;
    const rfec_kplan& P = M.plan;
    uint64_t have0 = present[2 * g], have1 = present[2 * g + 1];
    const uint64_t pp = parity_present[g];
    uint64_t rec0 = 0, rec1 = 0;
    rfec_hdr* hg = hdr + (size_t)g * P.k;
    rfec_step* steps = ws + (size_t)g * ws_stride;
    uint32_t n_steps = 0;
    bool progress = true;
    while (progress) {
        progress = false;
        for (uint32_t l = 0; l < P.n_lines; ++l) {
            if (!((pp >> l) & 1ull))
                continue;
            const uint64_t m0 = M.mask[l][0], m1 = M.mask[l][1];
            const uint64_t x0 = m0 & ~have0, x1 = m1 & ~have1;
            if (__popcll(x0) + __popcll(x1) != 1)
                continue;
            if (((m0 & have0) | (m1 & have1)) == 0)
                continue; // count == 0 (:134, :190)
            const uint32_t t = x0 ? (uint32_t)__ffsll((long long)x0) - 1 : 64u + (uint32_t)__ffsll((long long)x1) - 1;
            const size_t o = (size_t)g * P.n_lines + l;
            const uint32_t L = fsize[o];
            if (L > capacity)
                continue;
            const rfec_line ln = P.line[l];
            Hdr5 r = ldh(meta + o);
            bool ok = true;
            for (uint32_t q = 0; q < ln.count; ++q) {
                const uint32_t i = ln.first + q * ln.stride;
                if (i == t)
                    continue;
                Hdr5 h = ldh(hg + i);
#pragma unroll
                for (int w = 0; w < 5; ++w)
                    r.w[w] ^= h.w[w];
                ok = ok && hsize(h) <= L; // flex_fec_xor.c:88-89
            }
            if (!ok || hsize(r) > L) // :98-99
                continue;
            sth(hg + t, r);
            rfec_step st;
            st.first = ln.first;
            st.stride = ln.stride;
            st.count = ln.count;
            st.q = (uint8_t)((t - ln.first) / ln.stride);
            st.line = (uint8_t)l;
            st.target = (uint8_t)t;
            st.pad[0] = st.pad[1] = 0;
            steps[1 + n_steps] = st;
            ++n_steps;
            if (t < 64) {
                have0 |= 1ull << t;
                rec0 |= 1ull << t;
            } else {
                have1 |= 1ull << (t - 64);
                rec1 |= 1ull << (t - 64);
            }
            progress = true;
        }
    }
    rfec_step head = {};
    head.first = (uint8_t)n_steps; // step 0 slot carries the count
    head.count = 0;
    steps[0] = head;
    recovered[2 * g] = rec0;
    recovered[2 * g + 1] = rec1;
}

// ---------------------------------------------------------------------------
// Recovery XOR: one lane per (group, chunk column) replays the group's steps;
// a member recovered by an earlier step was written by this same lane.
// ---------------------------------------------------------------------------
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_recover(v4u* shards, const v4u* __restrict__ parity,
                                                    const rfec_step* __restrict__ ws, uint32_t total, uint32_t C,
                                                    FastDiv divC, uint32_t k, uint32_t n_lines,
                                                    uint32_t ws_stride)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * C;
    const rfec_step* steps = ws + (size_t)g * ws_stride;
    const uint32_t n = steps[0].first;
    v4u* grp = shards + (size_t)g * k * C + j;
    const v4u* par = parity + (size_t)g * n_lines * C + j;
    for (uint32_t s = 0; s < n; ++s) {
        const rfec_step st = steps[1 + s];
        v4u acc = ld16<NT>(par + (size_t)st.line * C);
        const v4u* base = grp + (size_t)st.first * C;
        const size_t step = (size_t)st.stride * C;
        for (uint32_t q = 0; q < st.count; ++q) {
            if (q == st.q)
                continue;
            acc = xor4(acc, base[q * step]);
        }
        grp[(size_t)st.target * C] = acc;
    }
}

// Zero bytes [data_size, stride) of every slot.
__global__ __launch_bounds__(kBlock) void k_zero_tails(v4u* shards, const rfec_hdr* __restrict__ hdr,
                                                       uint32_t total, uint32_t C, FastDiv divC)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t slot = fdiv(t, divC);
    const uint32_t j = t - slot * C;
    const uint32_t size = hdr[slot].size;
    const uint32_t b0 = j * 16;
    if (b0 + 16 <= size)
        return;
    v4u* p = shards + (size_t)slot * C + j;
    if (b0 >= size) {
        *p = v4u{0, 0, 0, 0};
        return;
    }
    v4u v = *p;
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lo = b0 + 4 * i;
        if (lo >= size)
            w[i] = 0;
        else if (lo + 4 > size)
            w[i] &= (1u << (8 * (size - lo))) - 1u;
    }
    *p = v4u{w[0], w[1], w[2], w[3]};
}

FastDiv make_fastdiv(uint32_t d)
{
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d)
        ++s;
    f.s = s;
    f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    return f;
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

template <bool NT>
hipError_t launch_encode_t(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                           const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                           uint16_t* fsize, int8_t* status, hipStream_t stream, int force_generic)
{
    const uint32_t C = stride / 16;
    const uint32_t total = groups * C;
    const FastDiv f = make_fastdiv(C);
    const dim3 grid(blocks_for(total)), block(kBlock);
    const v4u* s = reinterpret_cast<const v4u*>(shards);
    v4u* p = reinterpret_cast<v4u*>(parity);
    // fast paths: pure row layouts, rows of COL consecutive members
    const uint32_t col = P->n_lines ? P->line[0].count : 0;
    bool full_rows = col >= 2 && P->n_lines == (P->k + col - 1) / col;
    for (uint32_t l = 0; l < P->n_lines && full_rows; ++l) {
        const uint32_t first = l * col;
        const uint32_t count = P->k - first < col ? P->k - first : col;
        full_rows = P->line[l].stride == 1 && P->line[l].first == first && P->line[l].count == count;
    }
    if (!force_generic && full_rows) {
        if (P->k == 10 && col == 4) {
            hipLaunchKernelGGL((k_encode_rows<10, 4, NT>), grid, block, 0, stream, s, hdr, p, meta, fsize, status,
                               total, C, f, capacity, *P);
            return hipGetLastError();
        }
        if (P->k == 32 && col == 4) {
            hipLaunchKernelGGL((k_encode_rows<32, 4, NT>), grid, block, 0, stream, s, hdr, p, meta, fsize, status,
                               total, C, f, capacity, *P);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_encode<NT>), grid, block, 0, stream, s, hdr, p, meta, fsize, status, total, C, f, capacity,
                       *P);
    return hipGetLastError();
}

} // namespace

extern "C" {

int rfec_launch_encode(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                       const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                       uint16_t* fsize, int8_t* status, void* stream, unsigned flags)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int generic = (flags & RFEC_KFLAG_GENERIC) != 0;
    hipError_t e = (flags & RFEC_KFLAG_TEMPORAL)
                       ? launch_encode_t<false>(P, groups, stride, capacity, shards, hdr, parity, meta, fsize,
                                                status, st, generic)
                       : launch_encode_t<true>(P, groups, stride, capacity, shards, hdr, parity, meta, fsize,
                                               status, st, generic);
    return (int)e;
}

int rfec_launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                        uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fsize, const uint64_t* parity_present,
                        uint64_t* recovered, void* ws, uint32_t ws_stride, void* stream, unsigned flags)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint32_t C = stride / 16;
    hipLaunchKernelGGL(k_peel, dim3(blocks_for(groups)), dim3(kBlock), 0, st, hdr, present, meta, fsize,
                       parity_present, recovered, reinterpret_cast<rfec_step*>(ws), groups, ws_stride, capacity,
                       *M);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return (int)e;
    const uint32_t total = groups * C;
    const FastDiv f = make_fastdiv(C);
    if (flags & RFEC_KFLAG_TEMPORAL)
        hipLaunchKernelGGL(k_recover<false>, dim3(blocks_for(total)), dim3(kBlock), 0, st,
                           reinterpret_cast<v4u*>(shards), reinterpret_cast<const v4u*>(parity),
                           reinterpret_cast<const rfec_step*>(ws), total, C, f, (uint32_t)M->plan.k,
                           (uint32_t)M->plan.n_lines, ws_stride);
    else
        hipLaunchKernelGGL(k_recover<true>, dim3(blocks_for(total)), dim3(kBlock), 0, st,
                           reinterpret_cast<v4u*>(shards), reinterpret_cast<const v4u*>(parity),
                           reinterpret_cast<const rfec_step*>(ws), total, C, f, (uint32_t)M->plan.k,
                           (uint32_t)M->plan.n_lines, ws_stride);
    return (int)hipGetLastError();
}

int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream)
{
    const uint32_t C = stride / 16;
    const uint32_t total = slots * C;
    hipLaunchKernelGGL(k_zero_tails, dim3(blocks_for(total)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<v4u*>(shards), hdr, total, C,
                       make_fastdiv(C));
    return (int)hipGetLastError();
}

const char* rfec_hip_error_string(int code) { return hipGetErrorString((hipError_t)code); }

} // extern "C"
