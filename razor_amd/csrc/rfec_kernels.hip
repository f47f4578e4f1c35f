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
// (multiple of 16), zero beyond data_size.  All arithmetic is wave64
// v_xor_b32 on dwordx4 registers (no MFMA: XOR is ~0.06 op/B, HBM-bound).
//
//  encode: one launch, two kinds of workgroups.
//    * payload blocks: one lane per (group, 16-B chunk column); a lane loads
//      the chunk of every member (all loads in flight before the first XOR)
//      and stores one chunk per parity line -- a pure streaming pass.
//    * meta blocks (the first ones in the grid): copy the headers of up to
//      64 groups into LDS with coalesced dword loads, then one lane per
//      (group, line) XORs its members' 20-byte records out of LDS.
//  recover (rfec_launch_recover picks by plan):
//    * disjoint lines (row layer, strip mode): k_decode_disjoint, one launch --
//      header lanes (one per group and line) at the head of the grid, then one
//      lane per (group, chunk column) XORing every line with one missing member;
//    * lines that cascade (rows + columns), up to 8 members: k_decode_cascade, one
//      launch -- the exact peel in header blocks, a mask-only replay of the
//      same canonical schedule in the payload lanes -- plus k_decode_fixup for
//      the groups whose header checks disagree with the masks;
//    * otherwise k_peel_lds (schedule records) + k_recover_flat (replay);
//      k_recover (one wave per group, schedule and XOR interleaved) stays as
//      an A/B variant.
#include <hip/hip_runtime.h>

#include <atomic>
#include <ctime>
#include <unistd.h>
#include <stdint.h>

#include "rfec_internal.h"

#include "rfec_launch.h"

static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
static thread_local uint32_t t_launches = 0; // launches since rfec_timing_events

bool rfec_timing_take(hipEvent_t* start, hipEvent_t* stop)
{
    ++t_launches;
    if (!t_ev_start && !t_ev_stop)
        return false;
    *start = t_ev_start;
    *stop = t_ev_stop;
    t_ev_start = t_ev_stop = nullptr;
    return true;
}

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMetaDwords = 4096; // 16 KiB of LDS for the meta blocks' header stage

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

template <bool NT>
__device__ __forceinline__ v4u ld16(const v4u* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// Store cache policy: 0 plain, 1 non-temporal, 2 write-through (sc0 sc1),
// 3 write-through + non-temporal.  2 and 3 are emitted as inline asm (hipcc
// has no builtin for them).  hipcc neither counts nor pads an asm statement
// (cdna_hip_programming.md §5.7): the trailing `s_nop 1` keeps the next VALU
// from overwriting the store-data VGPRs before the dwordx4 store reads them;
// no s_waitcnt is needed (nothing of ours waits on a store, and a later load
// of the same address by the same lane is ordered behind it by the memory pipe).
template <int SP>
__device__ __forceinline__ void st16(v4u* p, v4u v)
{
    if constexpr (SP == 1)
        __builtin_nontemporal_store(v, p);
    else if constexpr (SP == 2)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 3)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        *p = v;
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// Payload-block index, optionally XCD-swizzled.  Workgroups are dispatched
// round-robin over the 8 XCDs (block b runs on XCD b % 8, each XCD with its
// own L2); the swizzle gives every XCD one contiguous range of logical blocks,
// so a cache line shared by neighbouring blocks is fetched into one L2.  The
// tail beyond the last multiple of 8 keeps the identity mapping (a bijection).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t swz)
{
    const uint32_t nb8 = nb & ~7u;
    if (!swz || b >= nb8)
        return b;
    return (b & 7u) * (nb8 >> 3) + (b >> 3);
}

// Copies n dwords global -> LDS with the whole block, several loads in flight
// per lane (a plain strided loop would wait on each load before the next).
// `lds` must be 16-byte aligned; 16-byte loads are used when `src` is too.
__device__ __forceinline__ void stage_dwords(uint32_t* lds, const uint32_t* __restrict__ src, uint32_t n)
{
    constexpr int U = 4;
    const uint32_t nv = ((reinterpret_cast<uintptr_t>(src) & 15) == 0) ? n / 4 : 0;
    const v4u* s4 = reinterpret_cast<const v4u*>(src);
    v4u* d4 = reinterpret_cast<v4u*>(lds);
    for (uint32_t base = 0; base < nv; base += U * kBlock) {
        v4u tmp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = base + u * kBlock + threadIdx.x;
            if (i < nv)
                tmp[u] = s4[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = base + u * kBlock + threadIdx.x;
            if (i < nv)
                d4[i] = tmp[u];
        }
    }
    for (uint32_t base = nv * 4; base < n; base += 4 * U * kBlock) {
        uint32_t tmp[4 * U];
#pragma unroll
        for (int u = 0; u < 4 * U; ++u) {
            const uint32_t i = base + u * kBlock + threadIdx.x;
            if (i < n)
                tmp[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < 4 * U; ++u) {
            const uint32_t i = base + u * kBlock + threadIdx.x;
            if (i < n)
                lds[i] = tmp[u];
        }
    }
}

// ---------------------------------------------------------------------------
// Encode meta blocks: fec_meta = XOR of the member headers taken as five
// dwords (field-wise XOR, flex_fec_xor.c:13-20, 37-44), fec_data_size = max
// data_size (:22-26), status -1 where flex_fec_generate fails (:9-10, :27-28).
// ---------------------------------------------------------------------------
__device__ void meta_block(uint32_t mb, const uint32_t* __restrict__ hdr_dw, uint32_t* __restrict__ meta_dw,
                           uint16_t* __restrict__ fsize, int8_t* __restrict__ status, uint32_t groups,
                           uint32_t capacity, uint32_t gpb, const rfec_kplan& P)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kMetaDwords];
    const uint32_t K = P.k, NL = P.n_lines;
    const uint32_t g0 = mb * gpb;
    const uint32_t ng = min(gpb, groups - g0);
    stage_dwords(lds, hdr_dw + (size_t)g0 * K * 5, ng * K * 5);
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < ng * NL; o += kBlock) {
        const uint32_t gl = o / NL, l = o - gl * NL;
        const rfec_line ln = P.line[l];
        const uint32_t* h = lds + gl * K * 5;
        uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, L = 0;
        for (uint32_t q = 0; q < ln.count; ++q) {
            const uint32_t* r = h + (ln.first + q * ln.stride) * 5;
            m0 ^= r[0];
            m1 ^= r[1];
            m2 ^= r[2];
            m3 ^= r[3];
            m4 ^= r[4];
            L = max(L, r[4] >> 16);
        }
        const size_t out = (size_t)g0 * NL + o;
        uint32_t* d = meta_dw + out * 5;
        d[0] = m0;
        d[1] = m1;
        d[2] = m2;
        d[3] = m3;
        d[4] = m4;
        fsize[out] = (uint16_t)L;
        if (status)
            status[out] = (ln.count <= 1 || L > capacity) ? (int8_t)-1 : (int8_t)0;
    }
}

struct EncMeta {
    const uint32_t* hdr_dw;
    uint32_t* meta_dw;
    uint16_t* fsize;
    int8_t* status;
    uint32_t groups, capacity, gpb, n_meta_blocks;
};

// ---------------------------------------------------------------------------
// Encode payload, generic plan.
// ---------------------------------------------------------------------------
template <bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_encode(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                   uint32_t total, uint32_t C, FastDiv divC, EncMeta E,
                                                   rfec_kplan P)
{
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    const uint32_t t = (blockIdx.x - E.n_meta_blocks) * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
    const v4u* src = shards + (size_t)g * P.k * C + j;
    v4u* dst = parity + (size_t)g * P.n_lines * C + j;
    for (uint32_t l = 0; l < P.n_lines; ++l) {
        const rfec_line ln = P.line[l];
        const v4u* s = src + (size_t)ln.first * C;
        const size_t step = (size_t)ln.stride * C;
        v4u acc = ld16<NTL>(s);
        for (uint32_t q = 1; q < ln.count; ++q)
            acc ^= ld16<NTL>(s + q * step);
        st16<NTS>(dst + (size_t)l * C, acc);
    }
}

// ---------------------------------------------------------------------------
// Encode payload, the reference sender's full matrix plan at small k
// (flex_fec_sender.c:166-233: rows of COL consecutive segments, then columns
// strided by COL, lines with fewer than 2 members dropped), member offsets
// and line order compile-time: all K loads in flight, every line's XOR from
// registers.  K = 6..16 (COL = 3 or 4, as flex_fec_sender_num_packets picks).
// ---------------------------------------------------------------------------
template <int K, int COL>
struct MatrixShape {
    static constexpr int R = (K + COL - 1) / COL;
    static constexpr int row_count(int r) { return (r * COL + COL <= K) ? COL : K - r * COL; }
    static constexpr int col_count(int c) { return (K - c + COL - 1) / COL; }
    static constexpr int n_rows()
    {
        int n = 0;
        for (int r = 0; r < R; ++r)
            n += row_count(r) >= 2;
        return n;
    }
    static constexpr int n_lines()
    {
        int n = n_rows();
        for (int c = 0; c < COL; ++c)
            n += col_count(c) >= 2;
        return n;
    }
};

template <int K, int COL, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_encode_matrix(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                          uint32_t total, uint32_t C, FastDiv divC, EncMeta E,
                                                          rfec_kplan P)
{
    using Sh = MatrixShape<K, COL>;
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    const uint32_t t = (blockIdx.x - E.n_meta_blocks) * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d;
    const v4u* src = shards + (size_t)g * K * C + j;
    v4u* dst = parity + (size_t)g * Sh::n_lines() * C + j;
    v4u v[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        v[i] = ld16<NTL>(src + (size_t)i * C);
    int l = 0;
#pragma unroll
    for (int r = 0; r < Sh::R; ++r) {
        if (Sh::row_count(r) < 2)
            continue;
        v4u acc = v[r * COL];
#pragma unroll
        for (int q = 1; q < COL; ++q)
            if (q < Sh::row_count(r))
                acc ^= v[r * COL + q];
        st16<NTS>(dst + (size_t)(l++) * C, acc);
    }
#pragma unroll
    for (int c = 0; c < COL; ++c) {
        if (Sh::col_count(c) < 2)
            continue;
        v4u acc = v[c];
#pragma unroll
        for (int q = 1; q < (K + COL - 1) / COL; ++q)
            if (q < Sh::col_count(c))
                acc ^= v[c + q * COL];
        st16<NTS>(dst + (size_t)(l++) * C, acc);
    }
}

// ---------------------------------------------------------------------------
// Encode payload, any plan over k <= 16 segments (e.g. the reference sender's
// full row + column plan, flex_fec_sender.c:166-233): a lane loads the chunk
// of every member once, all k loads in flight, and forms each line's XOR from
// registers; the lines come as wave-uniform 16-bit member masks, so the
// member selection is scalar control flow, not per-lane work.
// ---------------------------------------------------------------------------
struct LineMasks16 {
    uint32_t n;
    uint16_t m[RFEC_MAX_LINES];
};

template <bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_encode_k16(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                       uint32_t total, uint32_t C, FastDiv divC, EncMeta E,
                                                       rfec_kplan P, LineMasks16 LM)
{
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    const uint32_t t = (blockIdx.x - E.n_meta_blocks) * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d;
    const uint32_t K = P.k;
    const v4u* src = shards + (size_t)g * K * C + j;
    v4u* dst = parity + (size_t)g * LM.n * C + j;
    v4u v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = v4u{0, 0, 0, 0};
        if ((uint32_t)i < K)
            v[i] = ld16<NTL>(src + (size_t)i * C);
    }
    for (uint32_t l = 0; l < LM.n; ++l) {
        const uint32_t m = LM.m[l];
        v4u acc = v4u{0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u)
                acc ^= v[i];
        st16<NTS>(dst + (size_t)l * C, acc);
    }
}

// ---------------------------------------------------------------------------
// Encode payload, rows-of-COL fast path (k=10 rows {4,4,2}; k=32 8x4): member
// offsets are compile-time constants, so all K x ITEMS dwordx4 loads of a lane
// issue back to back.  Item u of a lane is chunk t0 + u*(payload lanes), so
// every wave instruction still covers 1 KiB of consecutive chunks.
// ---------------------------------------------------------------------------
template <int K, int COL, bool NTL, int NTS, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_encode_rows(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                        uint32_t total, uint32_t C, FastDiv divC, EncMeta E,
                                                        rfec_kplan P)
{
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    constexpr int R = (K + COL - 1) / COL;
    const uint32_t lanes = (gridDim.x - E.n_meta_blocks) * kBlock;
    const uint32_t t0 = (blockIdx.x - E.n_meta_blocks) * kBlock + threadIdx.x;
    v4u v[ITEMS][K];
    uint32_t gi[ITEMS], ji[ITEMS];
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        const uint32_t t = t0 + u * lanes;
        gi[u] = fdiv(t, divC);
        ji[u] = t - gi[u] * divC.d;
        if (t < total) {
            const v4u* src = shards + (size_t)gi[u] * K * C + ji[u];
#pragma unroll
            for (int i = 0; i < K; ++i)
                v[u][i] = ld16<NTL>(src + (size_t)i * C);
        }
    }
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        if (t0 + u * lanes >= total)
            continue;
        v4u* dst = parity + (size_t)gi[u] * R * C + ji[u];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            v4u acc = v[u][r * COL];
#pragma unroll
            for (int q = 1; q < COL; ++q)
                if (r * COL + q < K)
                    acc ^= v[u][r * COL + q];
            st16<NTS>(dst + (size_t)r * C, acc);
        }
    }
}

// ---------------------------------------------------------------------------
// Encode payload, rows-of-COL, output-mapped (default for row layouts): one
// lane per PARITY chunk (group, row, chunk column), the lane loads its row's
// COL (last row: K - (R-1)*COL) member chunks and stores one chunk.  Lane t
// writes parity chunk t when the slots are packed (stride == capacity), so
// every wave's store is 1 KiB of consecutive, 128-B-aligned parity bytes:
// whole lines, never two partial writes of one line from two waves on two
// XCDs, which the flat (group, chunk) mapping makes at every 1,200-B slot
// edge.  Row layouts have no member in two lines, so no chunk is loaded twice.
// tools/encode_lab.hip: 165-171 us vs 178-211 us flat at k = 10 / 1,200 B,
// equal to a 10-read : 3-write probe over contiguous streams.
// Meta blocks sit at the head of the grid, or at its tail (META_TAIL).
// ---------------------------------------------------------------------------
template <int K, int COL, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_encode_out(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                       uint32_t total, uint32_t C, FastDiv divC, FastDiv divRC,
                                                       uint32_t meta_first, uint32_t swz_head, EncMeta E, rfec_kplan P)
{
    const uint32_t mb = blockIdx.x - meta_first; // meta_first: 0 (head) or the payload block count (tail)
    if (mb < E.n_meta_blocks) {
        meta_block(mb, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    constexpr int R = (K + COL - 1) / COL;
    constexpr int LAST = K - (R - 1) * COL;
    uint32_t b = meta_first ? blockIdx.x : blockIdx.x - E.n_meta_blocks;
    if (swz_head) { // XCD swizzle (A/B): swz_head = meta + padding blocks, a multiple of 8
        if (blockIdx.x < swz_head)
            return;
        b = xcd_block(blockIdx.x - swz_head, gridDim.x - swz_head, 1);
    }
    const uint32_t t = b * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divRC);
    const uint32_t rem = t - g * divRC.d;
    const uint32_t r = fdiv(rem, divC);
    const uint32_t j = rem - r * divC.d;
    const v4u* s = shards + ((size_t)g * K + (size_t)r * COL) * C + j;
    v4u v[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q)
        if (q < LAST || r < (uint32_t)(R - 1))
            v[q] = ld16<NTL>(s + (size_t)q * C);
    v4u acc = v[0];
#pragma unroll
    for (int q = 1; q < COL; ++q)
        if (q < LAST || r < (uint32_t)(R - 1))
            acc ^= v[q];
    st16<NTS>(parity + ((size_t)g * R + r) * C + j, acc);
}

// The same for any row layout with rows of at most CMAX members (k, col
// runtime: the strip-mode plans of flex_fec_sender_num_packets, :112-132);
// the lane's member loads stay unrolled, predicated on the row's size.
template <int CMAX, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_encode_out_rt(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                          uint32_t total, uint32_t C, FastDiv divC, FastDiv divRC,
                                                          uint32_t K, uint32_t COL, uint32_t swz_head, EncMeta E,
                                                          rfec_kplan P)
{
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    uint32_t b = blockIdx.x - E.n_meta_blocks;
    if (swz_head) { // XCD swizzle: swz_head = meta + padding blocks, a multiple of 8
        if (blockIdx.x < swz_head)
            return;
        b = xcd_block(blockIdx.x - swz_head, gridDim.x - swz_head, 1);
    }
    const uint32_t t = b * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t R = divRC.d / divC.d;
    const uint32_t g = fdiv(t, divRC);
    const uint32_t rem = t - g * divRC.d;
    const uint32_t r = fdiv(rem, divC);
    const uint32_t j = rem - r * divC.d;
    const uint32_t cnt = r + 1 < R ? COL : K - (R - 1) * COL;
    const v4u* s = shards + ((size_t)g * K + (size_t)r * COL) * C + j;
    v4u v[CMAX];
#pragma unroll
    for (int q = 0; q < CMAX; ++q) {
        v[q] = v4u{0, 0, 0, 0};
        if ((uint32_t)q < cnt)
            v[q] = ld16<NTL>(s + (size_t)q * C);
    }
    v4u acc = v[0];
#pragma unroll
    for (int q = 1; q < CMAX; ++q)
        acc ^= v[q];
    st16<NTS>(parity + ((size_t)g * R + r) * C + j, acc);
}

// ---------------------------------------------------------------------------
// Encode payload, rows-of-COL, group-per-wave mapping.  Every wave covers
// whole groups (gpw = max(1, 64 / cd) of them, NI items per lane): a slot's
// last chunk and the next slot's first chunk, which share a 128-B line when
// the slot size is not a line multiple (1200 = 9.375 lines), are loaded by
// the same wave, so the line is fetched from HBM once.  Under the flat
// mapping those two chunks fall in different waves (often different XCDs)
// and the line is fetched twice.
// ---------------------------------------------------------------------------
template <int K, int COL, bool NTL, int NTS, int NI>
__global__ __launch_bounds__(kBlock) void k_encode_rows_gw(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                           uint32_t groups, uint32_t C, FastDiv divC, uint32_t gpw,
                                                           uint32_t swz, EncMeta E, rfec_kplan P)
{
    if (blockIdx.x < E.n_meta_blocks) {
        meta_block(blockIdx.x, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return;
    }
    constexpr int R = (K + COL - 1) / COL;
    const uint32_t b = xcd_block(blockIdx.x - E.n_meta_blocks, gridDim.x - E.n_meta_blocks, swz);
    const uint32_t wave = b * (kBlock / kWave) + threadIdx.x / kWave;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t g0 = wave * gpw;
    const uint32_t span = gpw * divC.d;
    v4u v[NI][K];
    uint32_t gi[NI], ji[NI];
    bool on[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        const uint32_t x = lane + u * kWave;
        const uint32_t gl = fdiv(x, divC);
        gi[u] = g0 + gl;
        ji[u] = x - gl * divC.d;
        on[u] = x < span && gi[u] < groups;
        if (on[u]) {
            const v4u* src = shards + (size_t)gi[u] * K * C + ji[u];
#pragma unroll
            for (int i = 0; i < K; ++i)
                v[u][i] = ld16<NTL>(src + (size_t)i * C);
        }
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        if (!on[u])
            continue;
        v4u* dst = parity + (size_t)gi[u] * R * C + ji[u];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            v4u acc = v[u][r * COL];
#pragma unroll
            for (int q = 1; q < COL; ++q)
                if (r * COL + q < K)
                    acc ^= v[u][r * COL + q];
            st16<NTS>(dst + (size_t)r * C, acc);
        }
    }
}

// ---------------------------------------------------------------------------
// Recover: one wave per group.
//
// Peeling = the fixpoint reached by flex_recover_row / flex_recover_col
// (flex_fec_receiver.c:105-206) as segments, parities and recovered segments
// (sim_receiver.c:780-804) arrive; canonical order: lines in plan order,
// repeated until nothing fires.  A line fires when its parity is present,
// exactly one member is missing, at least one is present (:133-140,
// :189-196) and flex_fec_recover would succeed: fec_data_size within the
// capacity, every member's data_size <= fec_data_size (flex_fec_xor.c:88-89)
// and the recovered data_size <= fec_data_size (:98-99).
// ---------------------------------------------------------------------------
struct RecArgs {
    v4u* shards;
    rfec_hdr* hdr;
    const uint64_t* present;
    const v4u* parity;
    const rfec_hdr* meta;
    const uint16_t* fsize;
    const uint64_t* parity_present;
    uint64_t* recovered;
    uint32_t groups, C, Cd, capacity;
};

template <bool NTL>
__global__ __launch_bounds__(kBlock) void k_recover(RecArgs A, rfec_kmask M)
{
    const uint32_t g = __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) / kWave);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    if (g >= A.groups)
        return;
    const rfec_kplan& P = M.plan;
    const uint32_t K = P.k, NL = P.n_lines, C = A.C;

    // ---- lane-parallel loads of the group's bookkeeping -------------------
    uint64_t have0 = A.present[2 * g], have1 = A.present[2 * g + 1];
    const uint64_t ppm = A.parity_present[g];
    const uint32_t* hdr_dw = reinterpret_cast<const uint32_t*>(A.hdr + (size_t)g * K);
    const uint32_t* meta_dw = reinterpret_cast<const uint32_t*>(A.meta + (size_t)g * NL);
    uint32_t hA[5] = {0, 0, 0, 0, 0}, hB[5] = {0, 0, 0, 0, 0}; // headers of segments lane, lane+64
    uint32_t mL[5] = {0, 0, 0, 0, 0}, fL = 0;                  // meta / fec_data_size of line `lane`
    if (lane < K) {
#pragma unroll
        for (int w = 0; w < 5; ++w)
            hA[w] = hdr_dw[lane * 5 + w];
    }
    if (lane + kWave < K) {
#pragma unroll
        for (int w = 0; w < 5; ++w)
            hB[w] = hdr_dw[(lane + kWave) * 5 + w];
    }
    if (lane < NL) {
#pragma unroll
        for (int w = 0; w < 5; ++w)
            mL[w] = meta_dw[lane * 5 + w];
        fL = A.fsize[(size_t)g * NL + lane];
    }
    v4u* grp = A.shards + (size_t)g * K * C;
    const v4u* par = A.parity + (size_t)g * NL * C;
    uint64_t rec0 = 0, rec1 = 0;

    bool progress = true;
    while (progress) {
        progress = false;
        for (uint32_t l = 0; l < NL; ++l) {
            if (!((ppm >> l) & 1ull))
                continue;
            const uint64_t m0 = M.mask[l][0], m1 = M.mask[l][1];
            const uint64_t x0 = m0 & ~have0, x1 = m1 & ~have1;
            if (__popcll(x0) + __popcll(x1) != 1)
                continue;
            if (((m0 & have0) | (m1 & have1)) == 0)
                continue; // count == 0
            const uint32_t t = x0 ? (uint32_t)__ffsll((long long)x0) - 1
                                  : 64u + (uint32_t)__ffsll((long long)x1) - 1;
            const uint32_t L = rl(fL, l);
            if (L > A.capacity)
                continue;
            const rfec_line ln = P.line[l];
            uint32_t r0 = rl(mL[0], l), r1 = rl(mL[1], l), r2 = rl(mL[2], l), r3 = rl(mL[3], l), r4 = rl(mL[4], l);
            bool ok = true;
            for (uint32_t q = 0; q < ln.count; ++q) {
                const uint32_t i = ln.first + q * ln.stride;
                if (i == t)
                    continue;
                const bool hi = i >= kWave;
                const uint32_t src = i & (kWave - 1);
                r0 ^= rl(hi ? hB[0] : hA[0], src);
                r1 ^= rl(hi ? hB[1] : hA[1], src);
                r2 ^= rl(hi ? hB[2] : hA[2], src);
                r3 ^= rl(hi ? hB[3] : hA[3], src);
                const uint32_t w4 = rl(hi ? hB[4] : hA[4], src);
                r4 ^= w4;
                ok = ok && (w4 >> 16) <= L;
            }
            if (!ok || (r4 >> 16) > L)
                continue;

            // payload: this lane's chunk columns j = lane, lane+64, ...
            for (uint32_t j0 = 0; j0 < A.Cd; j0 += 2 * kWave) {
                const uint32_t ja = j0 + lane, jb = j0 + kWave + lane;
                const bool oka = ja < A.Cd, okb = jb < A.Cd;
                v4u a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
                const v4u* pl = par + (size_t)l * C;
                if (oka)
                    a = ld16<NTL>(pl + ja);
                if (okb)
                    b = ld16<NTL>(pl + jb);
                for (uint32_t q = 0; q < ln.count; ++q) {
                    const uint32_t i = ln.first + q * ln.stride;
                    if (i == t)
                        continue;
                    const v4u* s = grp + (size_t)i * C;
                    if (oka)
                        a ^= s[ja];
                    if (okb)
                        b ^= s[jb];
                }
                v4u* d = grp + (size_t)t * C;
                if (oka)
                    d[ja] = a;
                if (okb)
                    d[jb] = b;
            }
            // recovered header (flex_fec_xor.c:64-85): lanes 0-4 store one dword
            // each; the holder lane of segment t keeps it for cascaded lines
            const uint32_t rw = lane == 0 ? r0 : lane == 1 ? r1 : lane == 2 ? r2 : lane == 3 ? r3 : r4;
            if (lane < 5)
                reinterpret_cast<uint32_t*>(A.hdr + (size_t)g * K + t)[lane] = rw;
            if ((t & (kWave - 1)) == lane) {
                if (t >= kWave) {
                    hB[0] = r0, hB[1] = r1, hB[2] = r2, hB[3] = r3, hB[4] = r4;
                } else {
                    hA[0] = r0, hA[1] = r1, hA[2] = r2, hA[3] = r3, hA[4] = r4;
                }
            }
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
    if (lane == 0) {
        A.recovered[2 * g] = rec0;
        A.recovered[2 * g + 1] = rec1;
    }
}

// ---------------------------------------------------------------------------
// Recover, two-kernel form (default).
//
// k_peel_lds: the same peeling schedule as k_recover, one lane per group, over
// the group's headers / line metadata staged in LDS by coalesced dword loads.
// Writes the recovered headers and a schedule record per group:
//   byte 0 = steps, byte 1 = 1 when no step reads a segment recovered by an
//   earlier step (single level), then (line, target) byte pairs.
// k_recover_flat: one lane per (group, 16-B chunk column) replays the record;
// single-level schedules run BATCH steps with every load in flight at once.
// ---------------------------------------------------------------------------
constexpr int kPeelDwords = 8192; // 32 KiB of LDS per peel block
constexpr int kFusedPeelDwords = 4096; // fused decodes: 16 KiB, the payload blocks carry this allocation too

struct PeelArgs {
    rfec_hdr* hdr;
    const uint64_t* present;
    const rfec_hdr* meta;
    const uint16_t* fsize;
    const uint64_t* parity_present;
    uint64_t* recovered;
    uint8_t* sched;
    uint32_t groups, capacity, gpb, rec_bytes, disjoint;
    uint32_t nlp_log2; // fused decode: > 0 = header lanes (line_headers), 0 = LDS-staged peel blocks
    // one-launch cascade decode: groups whose header checks rejected a line
    // the masks alone would fire go to fixlist; fixc = (gen << 32) | count,
    // a counter left from another launch (other gen) reads as 0
    unsigned long long* fixc;
    uint32_t* fixlist;
    uint32_t gen;
    // dense output (rfec_recover_batch_out): recovered segment e of group g
    // (the e-th erased one in index order, e < out_per_group) goes to
    // out_hdr[g * out_per_group + e]; out_per_group == 0: in place
    rfec_hdr* out_hdr;
    uint8_t* out_index;
    uint32_t out_per_group;
};

// Payload side of the dense output: out slot (g * E + e) of `sh` (E == 0: in place).
struct DenseOut {
    v4u* sh;
    uint32_t E;
};

// rank of erased segment t among the group's erased segments (index order)
__device__ __forceinline__ uint32_t missing_rank(uint64_t h0, uint64_t h1, uint32_t t)
{
    return t < 64 ? (uint32_t)__popcll(~h0 & ((1ull << t) - 1ull))
                  : (uint32_t)__popcll(~h0) + (uint32_t)__popcll(~h1 & ((1ull << (t - 64)) - 1ull));
}

__device__ __forceinline__ void fix_append(const PeelArgs& A, uint32_t g)
{
    unsigned long long old = *reinterpret_cast<volatile unsigned long long*>(A.fixc);
    for (;;) {
        const uint32_t idx = (uint32_t)(old >> 32) == A.gen ? (uint32_t)old : 0u;
        const unsigned long long nw = ((unsigned long long)A.gen << 32) | (idx + 1u);
        const unsigned long long seen = atomicCAS(A.fixc, old, nw);
        if (seen == old) {
            if (idx < A.groups)
                A.fixlist[idx] = g;
            return;
        }
        old = seen;
    }
}

// One peel block: groups [blk*gpb, ...).  With WRITE_SCHED false (fused
// decode of disjoint plans) only the recovered headers and masks are written.
template <bool WRITE_SCHED, int LDSD, bool FIXUP = false>
__device__ void peel_block(const PeelArgs& A, const rfec_kmask& M, uint32_t blk)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[LDSD];
    const rfec_kplan& P = M.plan;
    const uint32_t K = P.k, NL = P.n_lines;
    const uint32_t g0 = blk * A.gpb;
    const uint32_t ng = min(A.gpb, A.groups - g0);
    const uint32_t g = g0 + threadIdx.x;
    // this lane's masks first, so their latency overlaps the staging below
    uint64_t have0 = 0, have1 = 0, ppm = 0;
    if (threadIdx.x < ng) {
        have0 = A.present[2 * g];
        have1 = A.present[2 * g + 1];
        ppm = A.parity_present[g];
    }
    const uint32_t nh = ng * K * 5, nm = ng * NL * 5, nf = ng * NL;
    uint32_t* Lh = lds;                            // [ng][K][5]
    uint32_t* Lm = Lh + ((nh + 3) & ~3u);          // [ng][NL][5]
    uint16_t* Lf = reinterpret_cast<uint16_t*>(Lm + ((nm + 3) & ~3u)); // [ng][NL]
    stage_dwords(Lh, reinterpret_cast<const uint32_t*>(A.hdr + (size_t)g0 * K), nh);
    stage_dwords(Lm, reinterpret_cast<const uint32_t*>(A.meta + (size_t)g0 * NL), nm);
    const uint16_t* fsrc = A.fsize + (size_t)g0 * NL;
    if ((reinterpret_cast<uintptr_t>(fsrc) & 3) == 0) {
        stage_dwords(reinterpret_cast<uint32_t*>(Lf), reinterpret_cast<const uint32_t*>(fsrc), nf / 2);
        if ((nf & 1) && threadIdx.x == 0)
            Lf[nf - 1] = fsrc[nf - 1];
    } else {
        for (uint32_t i = threadIdx.x; i < nf; i += kBlock)
            Lf[i] = fsrc[i];
    }
    __syncthreads();
    if (threadIdx.x >= ng)
        return;
    uint32_t* h = Lh + threadIdx.x * K * 5;
    const uint32_t* m = Lm + threadIdx.x * NL * 5;
    const uint16_t* f = Lf + threadIdx.x * NL;
    uint64_t rec0 = 0, rec1 = 0;
    uint8_t* rec = A.sched + (size_t)g * A.rec_bytes;
    uint32_t n = 0, single = 1;
    bool rejected = false; // a line the masks fire failed the header checks
    // with pairwise-disjoint lines (e.g. the row layer alone) a recovery can
    // never complete another line, so one pass reaches the fixpoint
    bool progress = true;
    for (uint32_t pass = 0; progress && !(A.disjoint && pass > 0); ++pass) {
        progress = false;
        for (uint32_t l = 0; l < NL; ++l) {
            if (!((ppm >> l) & 1ull))
                continue;
            const uint64_t m0 = M.mask[l][0], m1 = M.mask[l][1];
            const uint64_t x0 = m0 & ~have0, x1 = m1 & ~have1;
            if (__popcll(x0) + __popcll(x1) != 1)
                continue;
            if (((m0 & have0) | (m1 & have1)) == 0)
                continue;
            const uint32_t t = x0 ? (uint32_t)__ffsll((long long)x0) - 1
                                  : 64u + (uint32_t)__ffsll((long long)x1) - 1;
            const uint32_t L = f[l];
            if (L > A.capacity) {
                rejected = true;
                continue;
            }
            uint32_t r0 = m[l * 5], r1 = m[l * 5 + 1], r2 = m[l * 5 + 2], r3 = m[l * 5 + 3], r4 = m[l * 5 + 4];
            bool ok = true;
            const bool reads_recovered = ((m0 & rec0) | (m1 & rec1)) != 0;
            const rfec_line ln = P.line[l];
            for (uint32_t q = 0; q < ln.count; ++q) {
                const uint32_t i = ln.first + q * ln.stride;
                if (i == t)
                    continue;
                const uint32_t* r = h + i * 5;
                r0 ^= r[0];
                r1 ^= r[1];
                r2 ^= r[2];
                r3 ^= r[3];
                r4 ^= r[4];
                ok = ok && (r[4] >> 16) <= L;
            }
            if (!ok || (r4 >> 16) > L) {
                rejected = true;
                continue;
            }
            uint32_t* ht = h + t * 5;
            ht[0] = r0, ht[1] = r1, ht[2] = r2, ht[3] = r3, ht[4] = r4;
            uint32_t* gh = reinterpret_cast<uint32_t*>(A.hdr + (size_t)g * K + t);
            gh[0] = r0, gh[1] = r1, gh[2] = r2, gh[3] = r3, gh[4] = r4;
            if (WRITE_SCHED) {
                rec[2 + 2 * n] = (uint8_t)l;
                rec[3 + 2 * n] = (uint8_t)t;
            }
            ++n;
            if (reads_recovered)
                single = 0;
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
    if (WRITE_SCHED) {
        rec[0] = (uint8_t)n;
        rec[1] = (uint8_t)single;
    }
    if (FIXUP && (rejected || n > 7)) // header checks disagree with the masks, or more steps than a record image
        fix_append(A, g);
    A.recovered[2 * g] = rec0;
    A.recovered[2 * g + 1] = rec1;
}

__global__ __launch_bounds__(kBlock) void k_peel_lds(PeelArgs A, rfec_kmask M)
{
    peel_block<true, kPeelDwords>(A, M, blockIdx.x);
}

__device__ __forceinline__ uint32_t rec_byte(const v4u& r, uint32_t b)
{
    return (r[b >> 2] >> (8 * (b & 3))) & 0xffu;
}

// Replays one group's schedule record over one chunk column: grp / par point
// at chunk j of the group's segment / parity slots, r0 = first 16 record bytes.
template <int MAXC, int BATCH, bool NTL, int NTS>
__device__ __forceinline__ void replay(v4u* grp, const v4u* __restrict__ par, const uint8_t* __restrict__ rec,
                                       const v4u r0, uint32_t C, uint32_t fast_ok, const uint32_t* lplan)
{
    const uint32_t n = rec_byte(r0, 0);
    uint32_t s = 0;
    if (fast_ok && rec_byte(r0, 1)) {
        // single level: BATCH steps at a time, all loads in flight together
        const uint32_t nf = n < 7 ? n : 7; // steps carried in the first 16 record bytes
        for (; s < nf; s += BATCH) {
            v4u acc[BATCH], mv[BATCH][MAXC];
            uint32_t tg[BATCH];
            bool on[BATCH];
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
                on[b] = s + b < nf;
                const uint32_t l = on[b] ? rec_byte(r0, 2 + 2 * (s + b)) : 0;
                tg[b] = rec_byte(r0, 3 + 2 * (s + b));
                const uint32_t ln = lplan[l];
                const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
                acc[b] = v4u{0, 0, 0, 0};
                if (on[b])
                    acc[b] = ld16<NTL>(par + (size_t)l * C);
#pragma unroll
                for (int q = 0; q < MAXC; ++q) {
                    const uint32_t i = first + q * stride;
                    mv[b][q] = v4u{0, 0, 0, 0};
                    if (on[b] && (uint32_t)q < count && i != tg[b])
                        mv[b][q] = ld16<NTL>(grp + (size_t)i * C);
                }
            }
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
#pragma unroll
                for (int q = 0; q < MAXC; ++q)
                    acc[b] ^= mv[b][q];
                if (on[b])
                    st16<NTS>(grp + (size_t)tg[b] * C, acc[b]);
            }
        }
        s = nf;
    }
    // remaining / multi-level steps, one at a time in schedule order
    for (; s < n; ++s) {
        const uint32_t l = s < 7 ? rec_byte(r0, 2 + 2 * s) : rec[2 + 2 * s];
        const uint32_t tt = s < 7 ? rec_byte(r0, 3 + 2 * s) : rec[3 + 2 * s];
        const uint32_t ln = lplan[l];
        const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
        v4u acc = ld16<NTL>(par + (size_t)l * C);
        for (uint32_t q = 0; q < count; ++q) {
            const uint32_t i = first + q * stride;
            if (i != tt)
                acc ^= grp[(size_t)i * C];
        }
        st16<NTS>(grp + (size_t)tt * C, acc);
    }
}

__device__ __forceinline__ void stage_plan(uint32_t* lplan, const rfec_kplan& P)
{
    if (threadIdx.x < P.n_lines)
        lplan[threadIdx.x] = reinterpret_cast<const uint32_t*>(P.line)[threadIdx.x];
    __syncthreads();
}

template <int MAXC, int BATCH, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_recover_flat(v4u* shards, const v4u* __restrict__ parity,
                                                         const uint8_t* __restrict__ sched, uint32_t total,
                                                         uint32_t C, FastDiv divC, uint32_t rec_bytes,
                                                         uint32_t fast_ok, rfec_kplan P)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    stage_plan(lplan, P);
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
    // fast_ok bit 1 (RFEC_TUNE_DIAG_CONST_SCHED, timing only): every group
    // replays group 0's record, an L2-hot load instead of a dependent HBM one
    const uint8_t* rec = sched + (size_t)((fast_ok & 2u) ? 0u : g) * rec_bytes;
    const v4u r0 = *reinterpret_cast<const v4u*>(rec);
    replay<MAXC, BATCH, NTL, NTS>(shards + (size_t)g * P.k * C + j, parity + (size_t)g * P.n_lines * C + j, rec, r0, C,
                             fast_ok & 1u, lplan);
}

// Grid-stride form: each lane walks items t, t+T, t+2T, ... and loads the
// next item's schedule record before replaying the current one, so the
// record's latency hides under the current item's payload loads.
template <int MAXC, int BATCH, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_recover_pipe(v4u* shards, const v4u* __restrict__ parity,
                                                         const uint8_t* __restrict__ sched, uint32_t total,
                                                         uint32_t C, FastDiv divC, uint32_t rec_bytes,
                                                         uint32_t fast_ok, rfec_kplan P)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    stage_plan(lplan, P);
    const uint32_t T = gridDim.x * kBlock;
    uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    uint32_t g = fdiv(t, divC);
    v4u r0 = *reinterpret_cast<const v4u*>(sched + (size_t)g * rec_bytes);
    while (t < total) {
        const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
        const uint32_t tn = t + T;
        const uint32_t gn = tn < total ? fdiv(tn, divC) : g;
        const v4u rn = *reinterpret_cast<const v4u*>(sched + (size_t)gn * rec_bytes);
        replay<MAXC, BATCH, NTL, NTS>(shards + (size_t)g * P.k * C + j, parity + (size_t)g * P.n_lines * C + j,
                                 sched + (size_t)g * rec_bytes, r0, C, fast_ok, lplan);
        t = tn;
        g = gn;
        r0 = rn;
    }
}

// ---------------------------------------------------------------------------
// Recover, one-launch form for plans with cascades (rows + columns).  Header
// blocks at the head of the grid run the exact peel (peel_block: headers,
// schedule records, recovered masks); every payload lane (group, chunk column)
// derives the schedule from the received masks alone -- the same canonical
// peel without the header size checks -- and replays up to 7 of its steps.
// The two schedules differ only where a header check rejected a line the masks
// fire; the peel lists those groups, and those with more than 7 steps, and
// k_decode_fixup, launched next, replays their exact records over the
// mask-only writes (which touched only erased slots, so nothing it reads).
// Replaying an exact record is idempotent.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void put_rec_byte(v4u& r, uint32_t pos, uint32_t v)
{
    const uint32_t w = pos >> 2, sh = 8 * (pos & 3);
    r[0] |= w == 0 ? v << sh : 0u;
    r[1] |= w == 1 ? v << sh : 0u;
    r[2] |= w == 2 ? v << sh : 0u;
    r[3] |= w == 3 ? v << sh : 0u;
}

// the canonical peel over the masks (lines in plan order to a fixpoint, as
// peel_block without its header checks) as a record image in registers:
// byte 0 = steps, byte 1 = single level, then (line, target) pairs
template <bool WIDE> // WIDE: k > 64, the second mask word in play
__device__ __forceinline__ v4u mask_schedule(const rfec_kmask& M, uint32_t NL, uint64_t h0, uint64_t h1, uint64_t ppm)
{
    if (!WIDE)
        h1 = 0;
    v4u r = {0, 0, 0, 0};
    uint32_t n = 0, single = 1;
    uint64_t rec0 = 0, rec1 = 0;
    bool progress = true;
    while (progress) {
        progress = false;
        for (uint32_t l = 0; l < NL; ++l) {
            if (!((ppm >> l) & 1ull))
                continue;
            const uint64_t m0 = M.mask[l][0], m1 = WIDE ? M.mask[l][1] : 0;
            const uint64_t x0 = m0 & ~h0, x1 = m1 & ~h1;
            if (__popcll(x0) + (WIDE ? __popcll(x1) : 0) != 1 || ((m0 & h0) | (m1 & h1)) == 0)
                continue;
            const uint32_t t = x0 ? (uint32_t)__ffsll((long long)x0) - 1 : 64u + (uint32_t)__ffsll((long long)x1) - 1;
            if (n == 7) { // the record image holds 7 steps: the peel lists this group for the fix-up
                r[0] |= n | (single << 8);
                return r;
            }
            if ((m0 & rec0) | (m1 & rec1))
                single = 0;
            put_rec_byte(r, 2 + 2 * n, l);
            put_rec_byte(r, 3 + 2 * n, t);
            ++n;
            if (t < 64) {
                h0 |= 1ull << t;
                rec0 |= 1ull << t;
            } else {
                h1 |= 1ull << (t - 64);
                rec1 |= 1ull << (t - 64);
            }
            progress = true;
        }
    }
    r[0] |= n | (single << 8);
    return r;
}

template <int MAXC, int BATCH, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_decode_cascade(v4u* shards, const v4u* __restrict__ parity,
                                                           uint32_t total, uint32_t C, FastDiv divC,
                                                           uint32_t n_hdr_blocks, PeelArgs A, rfec_kmask M)
{
    if (blockIdx.x < n_hdr_blocks) {
        peel_block<true, kFusedPeelDwords, true>(A, M, blockIdx.x);
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    const rfec_kplan& P = M.plan;
    stage_plan(lplan, P);
    const uint32_t t = (blockIdx.x - n_hdr_blocks) * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
    const v4u r0 = P.k <= 64 ? mask_schedule<false>(M, P.n_lines, A.present[2 * g], 0, A.parity_present[g])
                              : mask_schedule<true>(M, P.n_lines, A.present[2 * g], A.present[2 * g + 1],
                                                    A.parity_present[g]);
    if ((r0[0] & 0xffu) == 0)
        return;
    // at most 7 steps (mask_schedule stops there; longer schedules are the
    // fix-up's): every step sits in the 16 bytes of r0, the record pointer
    // (the peel's, being written meanwhile) is valid memory but never read
    replay<MAXC, BATCH, NTL, NTS>(shards + (size_t)g * P.k * C + j, parity + (size_t)g * P.n_lines * C + j,
                                  A.sched + (size_t)g * A.rec_bytes, r0, C, 1u, lplan);
}

// Exact replay of the listed groups (see k_decode_cascade), grid-stride over
// (listed group, chunk column); a counter from another launch counts 0.
template <int MAXC, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_decode_fixup(v4u* shards, const v4u* __restrict__ parity,
                                                         const uint8_t* __restrict__ sched,
                                                         const unsigned long long* __restrict__ fixc,
                                                         const uint32_t* __restrict__ fixlist, uint32_t gen,
                                                         uint32_t groups, uint32_t C, FastDiv divC,
                                                         uint32_t rec_bytes, rfec_kplan P)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    stage_plan(lplan, P);
    const unsigned long long c = *fixc;
    const uint32_t n = (uint32_t)(c >> 32) == gen ? min((uint32_t)c, groups) : 0u;
    const uint32_t total = n * divC.d;
    for (uint32_t it = blockIdx.x * kBlock + threadIdx.x; it < total; it += gridDim.x * kBlock) {
        const uint32_t gi = fdiv(it, divC);
        const uint32_t j = it - gi * divC.d;
        const uint32_t g = fixlist[gi];
        if (g >= groups)
            continue;
        const uint8_t* rec = sched + (size_t)g * rec_bytes;
        replay<MAXC, 1, NTL, NTS>(shards + (size_t)g * P.k * C + j, parity + (size_t)g * P.n_lines * C + j, rec,
                                  *reinterpret_cast<const v4u*>(rec), C, 0u, lplan);
    }
}

// ---------------------------------------------------------------------------
// Recover, fused form for plans whose lines are pairwise disjoint (the row
// layer alone, strip mode).  No recovery there can complete another line, so
// which lines fire follows from the received masks alone and no schedule has
// to travel between kernels.  The first n_hdr blocks do the peel's header
// work (size checks, recovered headers, the recovered mask); every other lane
// is one (group, 16-B chunk column) that XORs each line with exactly one
// missing member and its parity received into that member's slot.  A line the
// header checks reject is still written, into an erased slot whose recovered
// bit stays clear (rfec_recover_batch documents such slots as unspecified).
// ---------------------------------------------------------------------------

__device__ __forceinline__ bool has_bit(uint64_t h0, uint64_t h1, uint32_t i)
{
    return ((i < 64 ? h0 >> i : h1 >> (i - 64)) & 1ull) != 0;
}

// Header work of the fused decode, one lane per (group, line): NLP = 2^nlp_log2
// >= n_lines consecutive lanes per group.  A line fires as in peel_block (one
// member missing, one present, its parity received, sizes within bounds); it
// reads only its own members' headers, so a group costs the fired lines'
// records instead of all K + NL staged.  Lines are pairwise disjoint, so the
// lines of a group are independent; the group's recovered mask is OR-reduced
// over its NLP lanes (all in one wave: NLP <= 64).
__device__ void line_headers(const PeelArgs& A, const rfec_kmask& M, uint32_t blk)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    __shared__ uint64_t lmask[RFEC_MAX_LINES][2];
    const rfec_kplan& P = M.plan;
    if (threadIdx.x < P.n_lines) {
        lmask[threadIdx.x][0] = M.mask[threadIdx.x][0];
        lmask[threadIdx.x][1] = M.mask[threadIdx.x][1];
    }
    stage_plan(lplan, P);
    const uint32_t nlp = 1u << A.nlp_log2;
    const uint32_t hl = blk * kBlock + threadIdx.x;
    const uint32_t g = hl >> A.nlp_log2, l = hl & (nlp - 1);
    uint64_t rec0 = 0, rec1 = 0; // recovered mask (no dynamic register index: no scratch)
    if (g < A.groups && l < P.n_lines && ((A.parity_present[g] >> l) & 1ull)) {
        const uint64_t h0 = A.present[2 * g], h1 = A.present[2 * g + 1];
        const uint64_t m0 = lmask[l][0], m1 = lmask[l][1];
        const uint64_t x0 = m0 & ~h0, x1 = m1 & ~h1;
        if (__popcll(x0) + __popcll(x1) == 1 && ((m0 & h0) | (m1 & h1)) != 0) {
            // one round of loads: fec_data_size, fec_meta and the present
            // members' records together (the size check comes after them)
            const uint32_t t = x0 ? (uint32_t)__ffsll((long long)x0) - 1 : 64u + (uint32_t)__ffsll((long long)x1) - 1;
            const uint32_t L = A.fsize[(size_t)g * P.n_lines + l];
            const uint32_t* mr = reinterpret_cast<const uint32_t*>(A.meta + (size_t)g * P.n_lines + l);
            uint32_t r0 = mr[0], r1 = mr[1], r2 = mr[2], r3 = mr[3], r4 = mr[4];
            const uint32_t ln = lplan[l];
            const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
            const uint32_t* gh = reinterpret_cast<const uint32_t*>(A.hdr + (size_t)g * P.k);
            uint32_t w[8][5];
#pragma unroll
            for (int q = 0; q < 8; ++q) { // fused decodes: lines of at most 8 members
                const uint32_t i = first + q * stride;
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    w[q][d] = 0;
                if ((uint32_t)q < count && i != t) {
                    const uint32_t* r = gh + i * 5;
#pragma unroll
                    for (int d = 0; d < 5; ++d)
                        w[q][d] = r[d];
                }
            }
            bool ok = L <= A.capacity;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                r0 ^= w[q][0];
                r1 ^= w[q][1];
                r2 ^= w[q][2];
                r3 ^= w[q][3];
                r4 ^= w[q][4];
                ok = ok && (w[q][4] >> 16) <= L;
            }
            if (ok && (r4 >> 16) <= L) {
                uint32_t* ht = nullptr;
                if (!A.out_per_group) {
                    ht = reinterpret_cast<uint32_t*>(A.hdr + (size_t)g * P.k + t);
                } else {
                    const uint32_t e = missing_rank(h0, h1, t);
                    if (e < A.out_per_group)
                        ht = reinterpret_cast<uint32_t*>(A.out_hdr + (size_t)g * A.out_per_group + e);
                }
                if (ht) {
                    ht[0] = r0, ht[1] = r1, ht[2] = r2, ht[3] = r3, ht[4] = r4;
                    if (t < 64)
                        rec0 = 1ull << t;
                    else
                        rec1 = 1ull << (t - 64);
                }
            }
        }
    }
    for (uint32_t sh = 1; sh < nlp; sh <<= 1) {
        rec0 |= __shfl_xor(rec0, sh);
        rec1 |= __shfl_xor(rec1, sh);
    }
    if (g < A.groups && l == 0) {
        A.recovered[2 * g] = rec0;
        A.recovered[2 * g + 1] = rec1;
        if (A.out_per_group) {
            // out_index: the e-th erased segment's index where it was recovered, else 0xFF
            const uint32_t K = P.k;
            uint64_t m0 = ~A.present[2 * g] & (K >= 64 ? ~0ull : (1ull << K) - 1ull);
            uint64_t m1 = K <= 64 ? 0ull : ~A.present[2 * g + 1] & (K >= 128 ? ~0ull : (1ull << (K - 64)) - 1ull);
            uint8_t* oi = A.out_index + (size_t)g * A.out_per_group;
            for (uint32_t e = 0; e < A.out_per_group; ++e) {
                uint32_t v = 0xFF;
                if (m0 | m1) {
                    const uint32_t i = m0 ? (uint32_t)__ffsll((long long)m0) - 1 : 64u + (uint32_t)__ffsll((long long)m1) - 1;
                    if (has_bit(rec0, rec1, i))
                        v = i;
                    if (m0)
                        m0 &= m0 - 1;
                    else
                        m1 &= m1 - 1;
                }
                oi[e] = (uint8_t)v;
            }
        }
    }
}

// Header blocks of the fused decodes: the first n_hdr of the grid, or (every
// > 0) every (every + 1)-th block until they run out, spread over the grid so
// their latency-bound chains overlap the payload stream.  Returns true with
// *hb = header block index, else false with *pb = payload block index.
__device__ __forceinline__ bool header_block(uint32_t n_hdr, uint32_t every, uint32_t* hb, uint32_t* pb)
{
    const uint32_t b = blockIdx.x;
    if (!every) {
        *hb = b;
        *pb = b - n_hdr;
        return b < n_hdr;
    }
    const uint32_t per = b / (every + 1);
    *hb = per;
    *pb = b - min(per, n_hdr);
    return per < n_hdr && b - per * (every + 1) == every;
}

// The same spread in rounds of 8 blocks (one per XCD: block b runs on XCD
// b % 8) for the XCD-swizzled decodes: every (every + 1)-th round is a round
// of 8 header blocks until n_hr of them ran, so the payload blocks fill whole
// rounds and payload block p (in payload order) runs on XCD p % 8; it then
// takes logical block xcd_block(p): consecutive logical blocks share an XCD's
// L2 (the 128-B lines split between neighbouring slots are fetched once).
// npay8: payload blocks rounded up to a multiple of 8.
__device__ __forceinline__ bool header_block_xcd(uint32_t n_hr, uint32_t every, uint32_t npay8, uint32_t* hb,
                                                 uint32_t* pb)
{
    const uint32_t R = blockIdx.x >> 3, x = blockIdx.x & 7u;
    uint32_t pr;
    if (!every) {
        if (R < n_hr) {
            *hb = R * 8u + x;
            return true;
        }
        pr = R - n_hr;
    } else {
        const uint32_t per = R / (every + 1);
        if (per < n_hr && R - per * (every + 1) == every) {
            *hb = per * 8u + x;
            return true;
        }
        pr = R - min(per, n_hr);
    }
    *pb = xcd_block(pr * 8u + x, npay8, 1);
    return false;
}

__device__ __forceinline__ void run_header_block(const PeelArgs& A, const rfec_kmask& M, uint32_t hb)
{
    if (A.nlp_log2)
        line_headers(A, M, hb);
    else
        peel_block<false, kFusedPeelDwords>(A, M, hb);
}

template <int MAXC, bool NTL, int NTS, int NI>
__global__ __launch_bounds__(kBlock) void k_decode_disjoint(v4u* shards, const v4u* __restrict__ parity,
                                                            uint32_t total, uint32_t C, FastDiv divC,
                                                            uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                            rfec_kmask M, DenseOut D)
{
    uint32_t hb, pb;
    if (header_block(n_hdr_blocks, hdr_every, &hb, &pb)) {
        run_header_block(A, M, hb);
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    const rfec_kplan& P = M.plan;
    stage_plan(lplan, P);
    // NI items per lane, item u = t0 + u * (payload lanes): every wave
    // instruction still covers consecutive chunks, and the items' dependent
    // mask loads -> payload loads chains overlap
    const uint32_t lanes = (gridDim.x - n_hdr_blocks) * kBlock;
    const uint32_t t0 = pb * kBlock + threadIdx.x;
    uint64_t h0[NI], h1[NI], fire[NI];
    v4u* grp[NI];
    v4u* out[NI]; // dense output: the group's first out slot at this chunk column
    const v4u* par[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        const uint32_t t = t0 + u * lanes;
        h0[u] = h1[u] = fire[u] = 0;
        grp[u] = shards;
        out[u] = D.sh;
        par[u] = parity;
        if (t < total) {
            const uint32_t g = fdiv(t, divC);
            const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
            h0[u] = A.present[2 * g];
            h1[u] = A.present[2 * g + 1];
            fire[u] = A.parity_present[g];
            grp[u] = shards + (size_t)g * P.k * C + j;
            if (D.E)
                out[u] = D.sh + (size_t)g * D.E * C + j;
            par[u] = parity + (size_t)g * P.n_lines * C + j;
        }
    }
    // lines with their parity received and exactly one member missing
    // (uniform loop: the line masks stay scalar kernel-argument loads)
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        uint64_t f = 0;
        for (uint32_t l = 0; l < P.n_lines; ++l) {
            const uint64_t x0 = M.mask[l][0] & ~h0[u], x1 = M.mask[l][1] & ~h1[u];
            if (__popcll(x0) + __popcll(x1) == 1)
                f |= 1ull << l;
        }
        fire[u] &= f;
    }
    bool more = true;
    while (more) {
        // two fired lines per item per round, every load of all of them in flight together
        v4u acc[NI][2], mv[NI][2][MAXC];
        uint32_t tg[NI][2];
        bool on[NI][2];
#pragma unroll
        for (int u = 0; u < NI; ++u) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                on[u][b] = fire[u] != 0;
                const uint32_t l = on[u][b] ? (uint32_t)__ffsll((long long)fire[u]) - 1 : 0;
                fire[u] &= fire[u] - 1;
                const uint32_t ln = lplan[l];
                const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
                acc[u][b] = v4u{0, 0, 0, 0};
                if (on[u][b])
                    acc[u][b] = ld16<NTL>(par[u] + (size_t)l * C);
                tg[u][b] = first;
#pragma unroll
                for (int q = 0; q < MAXC; ++q) {
                    const uint32_t i = first + q * stride;
                    mv[u][b][q] = v4u{0, 0, 0, 0};
                    if (!on[u][b] || (uint32_t)q >= count)
                        continue;
                    if (has_bit(h0[u], h1[u], i))
                        mv[u][b][q] = ld16<NTL>(grp[u] + (size_t)i * C);
                    else
                        tg[u][b] = i;
                }
            }
        }
        more = false;
#pragma unroll
        for (int u = 0; u < NI; ++u) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
#pragma unroll
                for (int q = 0; q < MAXC; ++q)
                    acc[u][b] ^= mv[u][b][q];
                if (on[u][b]) {
                    if (!D.E) {
                        st16<NTS>(grp[u] + (size_t)tg[u][b] * C, acc[u][b]);
                    } else {
                        const uint32_t e = missing_rank(h0[u], h1[u], tg[u][b]);
                        if (e < D.E)
                            st16<NTS>(out[u] + (size_t)e * C, acc[u][b]);
                    }
                }
            }
            more = more || fire[u] != 0;
        }
    }
}

// Fused disjoint-plan decode for small slots (CD = 16 or 32 chunks, a group's
// lanes inside one wave), header work folded into the payload lanes: no
// header blocks.  Lane (g, j) runs the fired lines two at a time as
// k_decode_disjoint does; for line b of the pair, lanes j = 5b .. 5b + 4 also
// take dword j - 5b of its meta and of its present members' header records
// (the record of the erased member is their XOR), lane 5b + 4 the sizes and
// the checks of line_headers / peel_block (fec_data_size <= capacity, every
// present member and the recovered size within fec_data_size).  The verdict
// reaches the group's other lanes by one ds_bpermute, so every lane keeps the
// group's recovered mask and lane j == 0 writes it.
template <int CD, int BATCH, bool WIDE, bool NTL, int NTS>
__global__ __launch_bounds__(kBlock) void k_decode_small(v4u* shards, const v4u* __restrict__ parity, uint32_t C,
                                                         PeelArgs A, rfec_kmask M, DenseOut D)
{
    static_assert(CD == 16 || CD == 32, "a group's lanes must sit in one wave");
    constexpr int MAXC = 4;
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    const rfec_kplan& P = M.plan;
    stage_plan(lplan, P);
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = t / CD, j = t % CD;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t base = lane - j; // the group's first lane in this wave
    const bool valid = g < A.groups;
    const uint32_t gg = valid ? g : 0u;
    const uint64_t h0 = valid ? A.present[2 * gg] : ~0ull;
    const uint64_t h1 = valid && WIDE ? A.present[2 * gg + 1] : ~0ull;
    uint64_t fire = valid ? A.parity_present[gg] : 0ull;
    {
        uint64_t f = 0;
        for (uint32_t l = 0; l < P.n_lines; ++l) {
            const uint64_t m0 = M.mask[l][0], m1 = WIDE ? M.mask[l][1] : 0ull;
            const uint64_t x0 = m0 & ~h0, x1 = m1 & ~h1;
            if (__popcll(x0) + (WIDE ? __popcll(x1) : 0) == 1 && ((m0 & h0) | (m1 & h1)) != 0)
                f |= 1ull << l;
        }
        fire &= f;
    }
    v4u* grp = shards + (size_t)gg * P.k * C + j;
    const v4u* par = parity + (size_t)gg * P.n_lines * C + j;
    const uint32_t* gh = reinterpret_cast<const uint32_t*>(A.hdr + (size_t)gg * P.k);
    const uint32_t hb = j / 5, hd = j - 5 * hb; // header lane of pair slot hb, dword hd
    uint64_t rec0 = 0, rec1 = 0;
    while (fire) { // uniform within the group: all its lanes loop alike
        v4u acc[BATCH], mv[BATCH][MAXC];
        uint32_t tg[BATCH], hx[BATCH], L[BATCH], hsz[BATCH];
        bool on[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
            on[b] = fire != 0;
            const uint32_t l = on[b] ? (uint32_t)__ffsll((long long)fire) - 1 : 0;
            fire &= fire - 1;
            const uint32_t ln = lplan[l];
            const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
            const bool hl = on[b] && hb == (uint32_t)b; // header lane of this line
            acc[b] = v4u{0, 0, 0, 0};
            hx[b] = 0;
            L[b] = 0;
            hsz[b] = 0; // max present member size
            if (on[b]) {
                acc[b] = ld16<NTL>(par + (size_t)l * C);
                if (hl) {
                    hx[b] = reinterpret_cast<const uint32_t*>(A.meta + (size_t)gg * P.n_lines + l)[hd];
                    if (hd == 4)
                        L[b] = A.fsize[(size_t)gg * P.n_lines + l];
                }
            }
            tg[b] = first;
#pragma unroll
            for (int q = 0; q < MAXC; ++q) {
                const uint32_t i = first + q * stride;
                mv[b][q] = v4u{0, 0, 0, 0};
                if (!on[b] || (uint32_t)q >= count)
                    continue;
                if (has_bit(h0, h1, i)) {
                    mv[b][q] = ld16<NTL>(grp + (size_t)i * C);
                    if (hl) {
                        const uint32_t w = gh[i * 5 + hd];
                        hx[b] ^= w;
                        hsz[b] = max(hsz[b], w >> 16);
                    }
                } else {
                    tg[b] = i;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
#pragma unroll
            for (int q = 0; q < MAXC; ++q)
                acc[b] ^= mv[b][q];
            const uint32_t e = D.E ? missing_rank(h0, h1, tg[b]) : 0u;
            if (on[b] && (!D.E || e < D.E))
                st16<NTS>(D.E ? D.sh + ((size_t)gg * D.E + e) * C + j : grp + (size_t)tg[b] * C, acc[b]);
            // the checks in lane 5b + 4 (sizes in the high half of dword 4), to the group's lanes
            const uint32_t okv = (hb == (uint32_t)b && hd == 4 && L[b] <= A.capacity && hsz[b] <= L[b] &&
                                  (hx[b] >> 16) <= L[b]) ? 1u : 0u;
            const uint32_t ok = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * (base + 5u * b + 4u)), (int)okv);
            if (on[b] && ok && (!D.E || e < D.E)) { // (beyond the dense output: not recovered)
                if (tg[b] < 64)
                    rec0 |= 1ull << tg[b];
                else
                    rec1 |= 1ull << (tg[b] - 64);
                if (hb == (uint32_t)b) {
                    uint32_t* ht = D.E ? reinterpret_cast<uint32_t*>(A.out_hdr + (size_t)gg * D.E + e)
                                       : reinterpret_cast<uint32_t*>(A.hdr + (size_t)gg * P.k + tg[b]);
                    ht[hd] = hx[b];
                }
            }
        }
    }
    if (valid && j == 0) {
        A.recovered[2 * g] = rec0;
        A.recovered[2 * g + 1] = rec1;
        if (D.E) {
            const uint32_t K = P.k;
            uint64_t m0 = ~h0 & (K >= 64 ? ~0ull : (1ull << K) - 1ull);
            uint64_t m1 = K <= 64 ? 0ull : ~h1 & (K >= 128 ? ~0ull : (1ull << (K - 64)) - 1ull);
            uint8_t* oi = A.out_index + (size_t)g * D.E;
            for (uint32_t e = 0; e < D.E; ++e) {
                uint32_t v = 0xFF;
                if (m0 | m1) {
                    const uint32_t i = m0 ? (uint32_t)__ffsll((long long)m0) - 1 : 64u + (uint32_t)__ffsll((long long)m1) - 1;
                    if (has_bit(rec0, rec1, i))
                        v = i;
                    if (m0)
                        m0 &= m0 - 1;
                    else
                        m1 &= m1 - 1;
                }
                oi[e] = (uint8_t)v;
            }
        }
    }
}

// Fused disjoint-plan decode, output-mapped (default): one lane per (group,
// line, chunk column).  A lane whose line does not fire (parity missing, or
// not exactly one member missing) exits; the others load the parity chunk
// and the line's present members' chunks, all in flight, and store one
// chunk of the missing member.  A wave's loads and its store each cover 1 KiB
// of one slot, and no lane carries a second line (the flat (group, chunk)
// form serialises two lines' loads per lane).  tools/decode_lab.hip, cold
// parity: 142.7 us vs 157.8 us flat at k = 10 / 1,200 B.
// SLOTS (dense output): one lane per (group, output slot e, chunk column)
// instead: slot e's target is the group's e-th erased segment and its line
// comes from a segment -> line table (disjoint plan), so no lane sits on a
// line that does not fire (divLC divides by E C then).
template <int MAXC, bool NTL, int NTS, bool SLOTS>
__global__ __launch_bounds__(kBlock) void k_decode_out(v4u* shards, const v4u* __restrict__ parity, uint32_t total,
                                                       uint32_t C, FastDiv divC, FastDiv divLC,
                                                       uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                       rfec_kmask M, DenseOut D)
{
    uint32_t hb, pb;
    if (header_block(n_hdr_blocks, hdr_every, &hb, &pb)) {
        run_header_block(A, M, hb);
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    __shared__ uint64_t lmask[RFEC_MAX_LINES][2];
    __shared__ uint8_t sline[SLOTS ? RFEC_MAX_K : 1]; // segment -> its line (0xFF: none)
    const rfec_kplan& P = M.plan;
    if (threadIdx.x < P.n_lines) {
        lmask[threadIdx.x][0] = M.mask[threadIdx.x][0];
        lmask[threadIdx.x][1] = M.mask[threadIdx.x][1];
    }
    if constexpr (SLOTS) {
        if (threadIdx.x < P.k) {
            const uint32_t i = threadIdx.x;
            uint32_t li = 0xFF;
            for (uint32_t q = 0; q < P.n_lines; ++q) { // (uniform loads of the line masks)
                const uint64_t w = i < 64 ? M.mask[q][0] : M.mask[q][1];
                li = (w >> (i & 63)) & 1ull ? q : li;
            }
            sline[i] = (uint8_t)li;
        }
    }
    stage_plan(lplan, P); // ends in a barrier
    const uint32_t t = pb * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divLC);
    const uint32_t rem = t - g * divLC.d;
    const uint32_t q0 = fdiv(rem, divC); // line, or output slot (SLOTS)
    const uint32_t j = rem - q0 * divC.d;
    const uint64_t h0 = A.present[2 * g], h1 = A.present[2 * g + 1];
    uint32_t l = q0, tgt = 0;
    if constexpr (SLOTS) { // the q0-th erased segment among [0, k)
        const uint32_t k = P.k;
        uint64_t m0 = ~h0 & (k >= 64 ? ~0ull : (1ull << k) - 1ull);
        uint64_t m1 = k > 64 ? ~h1 & (k >= 128 ? ~0ull : (1ull << (k - 64)) - 1ull) : 0ull;
        const uint32_t c0 = (uint32_t)__popcll(m0);
        uint64_t m = q0 < c0 ? m0 : m1;
        for (uint32_t u = 0, ue = q0 < c0 ? q0 : q0 - c0; u < ue; ++u)
            m &= m - 1ull;
        if (!m)
            return;
        tgt = (q0 < c0 ? 0u : 64u) + (uint32_t)__ffsll((long long)m) - 1;
        l = sline[tgt];
        if (l == 0xFFu)
            return;
    }
    if (!((A.parity_present[g] >> l) & 1ull))
        return;
    const uint64_t x0 = lmask[l][0] & ~h0, x1 = lmask[l][1] & ~h1;
    if (__popcll(x0) + __popcll(x1) != 1 || ((lmask[l][0] & h0) | (lmask[l][1] & h1)) == 0)
        return;
    if constexpr (!SLOTS)
        tgt = x0 ? (uint32_t)__ffsll((long long)x0) - 1 : 64u + (uint32_t)__ffsll((long long)x1) - 1;
    v4u* grp = shards + (size_t)g * P.k * C + j;
    v4u* dst = grp + (size_t)tgt * C;
    if constexpr (SLOTS) {
        dst = D.sh + ((size_t)g * D.E + q0) * C + j;
    } else if (D.E) {
        const uint32_t e = missing_rank(h0, h1, tgt);
        if (e >= D.E)
            return;
        dst = D.sh + ((size_t)g * D.E + e) * C + j;
    }
    const uint32_t ln = lplan[l];
    const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
    v4u acc = ld16<NTL>(parity + ((size_t)g * P.n_lines + l) * C + j);
    v4u mv[MAXC];
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
        const uint32_t i = first + q * stride;
        mv[q] = v4u{0, 0, 0, 0};
        if ((uint32_t)q < count && i != tgt) // every other member of a firing line is present
            mv[q] = ld16<NTL>(grp + (size_t)i * C);
    }
#pragma unroll
    for (int q = 0; q < MAXC; ++q)
        acc ^= mv[q];
    st16<NTS>(dst, acc);
}

// The same for the row layouts of the encode fast path (rows of COL
// consecutive segments, K <= 64): the line masks and members are arithmetic
// in the row index, so no plan is staged through LDS (no barrier before the
// first load).  SLOTS (dense output): one lane per (group, output slot e,
// chunk) instead of (group, row, chunk): slot e's target is the group's e-th
// erased segment, recovered when its row fires, so no lane sits on a row
// that does not (divRC divides by E C then).
// K = 0: k and col at run time (k_rt <= 64, col_rt <= COL), the member loads
// unrolled to COL and predicated on the row's size (the strip-mode plans).
template <int K, int COL, bool NTL, int NTS, bool SLOTS>
__global__ __launch_bounds__(kBlock) void k_decode_rows(v4u* shards, const v4u* __restrict__ parity, uint32_t total,
                                                        uint32_t C, FastDiv divC, FastDiv divRC,
                                                        uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                        rfec_kmask M, DenseOut D, uint32_t swz_npay8, uint32_t k_rt,
                                                        uint32_t col_rt, FastDiv divCol)
{
    static_assert(K <= 64, "row decode keeps the present mask in one word");
    uint32_t hb, pb;
    if (swz_npay8) { // XCD swizzle: rounds of 8 blocks, header rounds spread (hdr_every in rounds)
        if (header_block_xcd((n_hdr_blocks + 7u) >> 3, hdr_every, swz_npay8, &hb, &pb)) {
            if (hb < n_hdr_blocks)
                run_header_block(A, M, hb);
            return;
        }
    } else if (header_block(n_hdr_blocks, hdr_every, &hb, &pb)) {
        run_header_block(A, M, hb);
        return;
    }
    const uint32_t KK = K ? (uint32_t)K : k_rt, CC = K ? (uint32_t)COL : col_rt;
    const uint32_t R = (KK + CC - 1) / CC, LAST = KK - (R - 1) * CC;
    const uint32_t t = pb * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divRC);
    const uint32_t rem = t - g * divRC.d;
    const uint32_t q0 = fdiv(rem, divC); // row, or output slot (SLOTS)
    const uint32_t j = rem - q0 * divC.d;
    const uint64_t h = A.present[2 * g];
    uint32_t r, tgt;
    if constexpr (SLOTS) {
        uint64_t m = ~h & (KK == 64 ? ~0ull : (1ull << KK) - 1ull);
        for (uint32_t u = 0; u < q0; ++u) // the q0-th erased segment
            m &= m - 1ull;
        if (!m)
            return;
        tgt = (uint32_t)__ffsll((long long)m) - 1;
        r = K ? tgt / (uint32_t)COL : fdiv(tgt, divCol);
    } else {
        r = q0;
    }
    const uint32_t cnt = r + 1 < R ? CC : LAST;
    const uint64_t rm = ((1ull << cnt) - 1ull) << (r * CC);
    const uint64_t miss = rm & ~h;
    if (__popcll(miss) != 1 || !((A.parity_present[g] >> r) & 1ull))
        return;
    if constexpr (!SLOTS)
        tgt = (uint32_t)__ffsll((long long)miss) - 1;
    v4u* dst = shards + ((size_t)g * KK + tgt) * C + j;
    if constexpr (SLOTS) {
        dst = D.sh + ((size_t)g * D.E + q0) * C + j;
    } else if (D.E) {
        const uint32_t e = (uint32_t)__popcll(~h & ((1ull << tgt) - 1ull));
        if (e >= D.E)
            return;
        dst = D.sh + ((size_t)g * D.E + e) * C + j;
    }
    v4u* row = shards + ((size_t)g * KK + r * CC) * C + j;
    v4u acc = ld16<NTL>(parity + ((size_t)g * R + r) * C + j);
    v4u mv[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q) {
        mv[q] = v4u{0, 0, 0, 0};
        if ((uint32_t)q < cnt && r * CC + q != tgt)
            mv[q] = ld16<NTL>(row + (size_t)q * C);
    }
#pragma unroll
    for (int q = 0; q < COL; ++q)
        acc ^= mv[q];
    st16<NTS>(dst, acc);
}

// Fused disjoint-plan decode, group-per-wave mapping (see k_encode_rows_gw):
// each wave covers whole groups, NI chunk items per lane, one item at a time
// with both fired lines' loads in flight together.
template <int MAXC, bool NTL, int NTS, int NI>
__global__ __launch_bounds__(kBlock) void k_decode_disjoint_gw(v4u* shards, const v4u* __restrict__ parity,
                                                               uint32_t C, FastDiv divC, uint32_t gpw, uint32_t swz,
                                                               uint32_t n_hdr_blocks, PeelArgs A, rfec_kmask M)
{
    if (blockIdx.x < n_hdr_blocks) {
        if (A.nlp_log2)
            line_headers(A, M, blockIdx.x);
        else
            peel_block<false, kFusedPeelDwords>(A, M, blockIdx.x);
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    const rfec_kplan& P = M.plan;
    stage_plan(lplan, P);
    const uint32_t b = xcd_block(blockIdx.x - n_hdr_blocks, gridDim.x - n_hdr_blocks, swz);
    const uint32_t wave = b * (kBlock / kWave) + threadIdx.x / kWave;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t g0 = wave * gpw;
    const uint32_t span = gpw * divC.d;
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        const uint32_t x = lane + u * kWave;
        const uint32_t gl = fdiv(x, divC);
        const uint32_t g = g0 + gl;
        const uint32_t j = x - gl * divC.d;
        if (x >= span || g >= A.groups)
            continue;
        const uint64_t h0 = A.present[2 * g], h1 = A.present[2 * g + 1], pm = A.parity_present[g];
        uint64_t fire = 0;
        for (uint32_t l = 0; l < P.n_lines; ++l) {
            const uint64_t x0 = M.mask[l][0] & ~h0, x1 = M.mask[l][1] & ~h1;
            if (__popcll(x0) + __popcll(x1) == 1)
                fire |= 1ull << l;
        }
        fire &= pm;
        v4u* grp = shards + (size_t)g * P.k * C + j;
        const v4u* par = parity + (size_t)g * P.n_lines * C + j;
        while (fire) {
            v4u acc[2], mv[2][MAXC];
            uint32_t tg[2];
            bool onb[2];
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                onb[bb] = fire != 0;
                const uint32_t l = onb[bb] ? (uint32_t)__ffsll((long long)fire) - 1 : 0;
                fire &= fire - 1;
                const uint32_t ln = lplan[l];
                const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
                acc[bb] = v4u{0, 0, 0, 0};
                if (onb[bb])
                    acc[bb] = ld16<NTL>(par + (size_t)l * C);
                tg[bb] = first;
#pragma unroll
                for (int q = 0; q < MAXC; ++q) {
                    const uint32_t i = first + q * stride;
                    mv[bb][q] = v4u{0, 0, 0, 0};
                    if (!onb[bb] || (uint32_t)q >= count)
                        continue;
                    if (has_bit(h0, h1, i))
                        mv[bb][q] = ld16<NTL>(grp + (size_t)i * C);
                    else
                        tg[bb] = i;
                }
            }
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
#pragma unroll
                for (int q = 0; q < MAXC; ++q)
                    acc[bb] ^= mv[bb][q];
                if (onb[bb])
                    st16<NTS>(grp + (size_t)tg[bb] * C, acc[bb]);
            }
        }
    }
}

// dst row r <- src row map[r] (all `C` 16-B chunks), or zeros for map[r] < 0:
// the receiver's scatter of parsed payloads into group slots and its gather
// of recovered segments.  One lane per chunk, streaming.
__global__ __launch_bounds__(kBlock) void k_gather_rows(v4u* __restrict__ dst, const v4u* __restrict__ src,
                                                        const int32_t* __restrict__ map, uint32_t total, uint32_t C,
                                                        FastDiv divC)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t r = fdiv(t, divC);
    const uint32_t j = t - r * C;
    const int32_t s = map[r];
    const v4u v = s >= 0 ? __builtin_nontemporal_load(src + (size_t)s * C + j) : v4u{0, 0, 0, 0};
    __builtin_nontemporal_store(v, dst + (size_t)r * C + j);
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
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lo = b0 + 4 * i;
        if (lo >= size)
            v[i] = 0;
        else if (lo + 4 > size)
            v[i] &= (1u << (8 * (size - lo))) - 1u;
    }
    *p = v;
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

struct EncLaunch {
    const rfec_kplan* P;
    uint32_t groups, stride, cd; // cd = 16-B chunks of work per slot, ceil(capacity / 16)
    const v4u* s;
    v4u* p;
    EncMeta E;
    hipStream_t stream;
};

template <int K, int COL, bool NTL, int NTS, int ITEMS>
hipError_t launch_rows(const EncLaunch& a)
{
    const uint32_t C = a.stride / 16;
    const uint32_t total = a.groups * a.cd;
    const uint32_t lanes = (total + ITEMS - 1) / ITEMS;
    RFEC_LAUNCH((k_encode_rows<K, COL, NTL, NTS, ITEMS>), dim3(a.E.n_meta_blocks + blocks_for(lanes)),
                       dim3(kBlock), 0, a.stream, a.s, a.p, total, C, make_fastdiv(a.cd), a.E, *a.P);
    return hipGetLastError();
}

// group-per-wave geometry: gpw whole groups per wave, ni chunk items per lane
struct GwGeom {
    uint32_t gpw, ni, blocks;
};

GwGeom gw_geom(uint32_t groups, uint32_t cd)
{
    GwGeom g;
    g.gpw = cd >= (uint32_t)kWave ? 1u : (uint32_t)kWave / cd;
    g.ni = (g.gpw * cd + kWave - 1) / kWave;
    const uint64_t waves = ((uint64_t)groups + g.gpw - 1) / g.gpw;
    g.blocks = (uint32_t)((waves + kBlock / kWave - 1) / (kBlock / kWave));
    return g;
}

template <int K, int COL, bool NTL, int NTS, int NI>
hipError_t launch_rows_gw(const EncLaunch& a, const GwGeom& g, uint32_t swz)
{
    const uint32_t C = a.stride / 16;
    RFEC_LAUNCH((k_encode_rows_gw<K, COL, NTL, NTS, NI>), dim3(a.E.n_meta_blocks + g.blocks), dim3(kBlock), 0,
                       a.stream, a.s, a.p, a.groups, C, make_fastdiv(a.cd), g.gpw, swz, a.E, *a.P);
    return hipGetLastError();
}

template <int K, int COL, bool NTL, int NTS>
hipError_t launch_rows_out(const EncLaunch& a, unsigned flags)
{
    constexpr uint32_t R = (K + COL - 1) / COL;
    const uint32_t C = a.stride / 16;
    const uint64_t total = (uint64_t)a.groups * R * a.cd;
    const uint32_t nb = blocks_for(total);
    // XCD-swizzled block order by default (tools/gpu_xcd.sh, cold: 168.1-168.4 vs 172.1 us linear, HBM
    // traffic 1.029 vs 1.059 x algorithmic: a 128-B line split between neighbouring slots is fetched once)
    const bool swz = !(flags & (RFEC_KFLAG_LINEAR_BLOCKS | RFEC_KFLAG_META_TAIL));
    const uint32_t meta_first = (flags & RFEC_KFLAG_META_TAIL) && !swz ? nb : 0u;
    // swizzle: meta blocks at the head, padded to a multiple of 8 so payload block p runs on XCD p % 8
    const uint32_t head = swz ? (a.E.n_meta_blocks + 7u) & ~7u : 0u;
    RFEC_LAUNCH((k_encode_out<K, COL, NTL, NTS>), dim3((swz ? head : a.E.n_meta_blocks) + nb), dim3(kBlock), 0,
                       a.stream, a.s, a.p, (uint32_t)total, C, make_fastdiv(a.cd), make_fastdiv(R * a.cd), meta_first,
                       head, a.E, *a.P);
    return hipGetLastError();
}

template <int CMAX, bool NTL, int NTS>
hipError_t launch_rows_out_rt(const EncLaunch& a, unsigned flags, uint32_t col)
{
    const uint32_t K = a.P->k, R = (K + col - 1) / col;
    const uint64_t total = (uint64_t)a.groups * R * a.cd; // < 2^32: checked by the caller
    const uint32_t nb = blocks_for(total);
    const bool swz = !(flags & RFEC_KFLAG_LINEAR_BLOCKS);
    const uint32_t head = swz ? (a.E.n_meta_blocks + 7u) & ~7u : 0u;
    RFEC_LAUNCH((k_encode_out_rt<CMAX, NTL, NTS>), dim3((swz ? head : a.E.n_meta_blocks) + nb), dim3(kBlock),
                       0, a.stream, a.s, a.p, (uint32_t)total, a.stride / 16, make_fastdiv(a.cd),
                       make_fastdiv(R * a.cd), K, col, head, a.E, *a.P);
    return hipGetLastError();
}

template <int K, int COL, bool NTL, int NTS>
hipError_t launch_rows_v(const EncLaunch& a, unsigned flags)
{
    constexpr uint64_t R = (K + COL - 1) / COL;
    if (!(flags & (RFEC_KFLAG_FLAT_ENCODE | RFEC_KFLAG_GROUP_WAVE | RFEC_KFLAG_ITEMS2)) &&
        (uint64_t)a.groups * R * a.cd < (1ull << 32))
        return launch_rows_out<K, COL, NTL, NTS>(a, flags);
    if (flags & RFEC_KFLAG_GROUP_WAVE) {
        const GwGeom g = gw_geom(a.groups, a.cd);
        const uint32_t swz = (flags & RFEC_KFLAG_XCD_SWIZZLE) ? 1u : 0u;
        if (g.ni == 1)
            return launch_rows_gw<K, COL, NTL, NTS, 1>(a, g, swz);
        if constexpr (K <= 16) { // 2 x K dwordx4 loads in flight per lane
            if (g.ni == 2)
                return launch_rows_gw<K, COL, NTL, NTS, 2>(a, g, swz);
        }
    }
    if (flags & RFEC_KFLAG_ITEMS2)
        return launch_rows<K, COL, NTL, NTS, 2>(a);
    return launch_rows<K, COL, NTL, NTS, 1>(a);
}

struct ReplayArgs {
    v4u* shards;
    const v4u* parity;
    const uint8_t* sched;
    uint32_t total, C;
    FastDiv f;
    uint32_t rec_bytes, fast_ok;
    hipStream_t stream;
};

template <int MAXC, int BATCH, bool PIPE, bool NTL, int NTS>
void launch_replay_t(const ReplayArgs& R, const rfec_kplan& P, dim3 grid)
{
    if constexpr (PIPE)
        RFEC_LAUNCH((k_recover_pipe<MAXC, BATCH, NTL, NTS>), grid, dim3(kBlock), 0, R.stream, R.shards,
                           R.parity, R.sched, R.total, R.C, R.f, R.rec_bytes, R.fast_ok, P);
    else
        RFEC_LAUNCH((k_recover_flat<MAXC, BATCH, NTL, NTS>), grid, dim3(kBlock), 0, R.stream, R.shards,
                           R.parity, R.sched, R.total, R.C, R.f, R.rec_bytes, R.fast_ok, P);
}

template <int MAXC, int BATCH, bool PIPE>
void launch_replay(const ReplayArgs& R, bool ntl, int sp, const rfec_kplan& P, dim3 grid)
{
    if (!ntl) {
        launch_replay_t<MAXC, BATCH, PIPE, false, 1>(R, P, grid); // A/B only: NT stores
        return;
    }
    switch (sp) {
    case 0: launch_replay_t<MAXC, BATCH, PIPE, true, 0>(R, P, grid); break;
    case 2: launch_replay_t<MAXC, BATCH, PIPE, true, 2>(R, P, grid); break;
    case 3: launch_replay_t<MAXC, BATCH, PIPE, true, 3>(R, P, grid); break;
    default: launch_replay_t<MAXC, BATCH, PIPE, true, 1>(R, P, grid); break;
    }
}

struct FusedArgs {
    v4u* shards;
    const v4u* parity;
    uint32_t total, C;
    FastDiv f;
    uint32_t n_hdr;
    hipStream_t stream;
    bool spread; // header blocks spread over the grid (RFEC_TUNE_HDR_SPREAD)
    DenseOut D;  // recovered payloads in place (E == 0) or to the dense output
};

// header_block()'s period for npay payload blocks (0: header blocks first).
// n_hdr periods of (every + 1) blocks must fit the grid: every <= npay / n_hdr,
// so fewer payload than header blocks keeps them at the head.
inline uint32_t hdr_every(const FusedArgs& F, uint32_t npay)
{
    if (!F.spread || !F.n_hdr)
        return 0;
    return npay / F.n_hdr;
}

template <int MAXC, int NI>
void launch_fused_gw(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M, const GwGeom& g,
                     uint32_t swz)
{
    const dim3 grid(F.n_hdr + g.blocks);
#define RFEC_FUSED_GW(NTL, NTS)                                                                                  \
    RFEC_LAUNCH((k_decode_disjoint_gw<MAXC, NTL, NTS, NI>), grid, dim3(kBlock), 0, F.stream, F.shards,    \
                       F.parity, F.C, F.f, g.gpw, swz, F.n_hdr, B, M)
    switch (sp) {
    case -1: RFEC_FUSED_GW(false, 1); break;
    case 0: RFEC_FUSED_GW(true, 0); break;
    case 2: RFEC_FUSED_GW(true, 2); break;
    case 3: RFEC_FUSED_GW(true, 3); break;
    default: RFEC_FUSED_GW(true, 1); break;
    }
#undef RFEC_FUSED_GW
}

// one-launch cascade decode + the fix-up replay (sp as launch_fused)
template <int MAXC, int BATCH>
void launch_cascade(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M)
{
    const dim3 grid(F.n_hdr + blocks_for(F.total));
    // fix-up: a small grid (the list is empty unless headers disagree with the masks)
    const uint32_t fb = blocks_for(F.total) < 128u ? blocks_for(F.total) : 128u;
#define RFEC_CASCADE(NTL, NTS)                                                                                    \
    RFEC_LAUNCH((k_decode_cascade<MAXC, BATCH, NTL, NTS>), grid, dim3(kBlock), 0, F.stream, F.shards,       \
                       F.parity, F.total, F.C, F.f, F.n_hdr, B, M);                                               \
    RFEC_LAUNCH((k_decode_fixup<MAXC, NTL, NTS>), dim3(fb), dim3(kBlock), 0, F.stream, F.shards, F.parity,  \
                       B.sched, B.fixc, B.fixlist, B.gen, B.groups, F.C, F.f, B.rec_bytes, M.plan)
    switch (sp) {
    case -1: RFEC_CASCADE(false, 1); break;
    case 0: RFEC_CASCADE(true, 0); break;
    case 2: RFEC_CASCADE(true, 2); break;
    case 3: RFEC_CASCADE(true, 3); break;
    default: RFEC_CASCADE(true, 1); break;
    }
#undef RFEC_CASCADE
}

// fix-up generation: a per-process sequence from a time/pid seed, so that a
// workspace left by an earlier launch (or process) never matches
uint32_t next_gen()
{
    static std::atomic<uint32_t> g{0};
    uint32_t v = g.fetch_add(1, std::memory_order_relaxed);
    if (v == 0) {
        const uint32_t seed = (uint32_t)time(nullptr) * 2654435761u ^ (uint32_t)getpid() * 40503u;
        uint32_t expect = 1;
        g.compare_exchange_strong(expect, seed | 1u);
        v = g.fetch_add(1, std::memory_order_relaxed);
    }
    return v;
}

// output-mapped fused decode: one lane per (group, line, chunk column)
template <int MAXC>
void launch_fused_out(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M, uint32_t cd, bool slots)
{
    const uint32_t per = slots ? F.D.E : M.plan.n_lines;
    const uint32_t total = B.groups * per * cd; // < 2^32: checked by the caller
    const uint32_t npay = blocks_for(total);
    const dim3 grid(F.n_hdr + npay);
    const FastDiv dC = make_fastdiv(cd), dLC = make_fastdiv(per * cd);
    const uint32_t every = hdr_every(F, npay);
#define RFEC_FUSED_OUT(NTL, NTS)                                                                                 \
    if (slots)                                                                                                   \
        RFEC_LAUNCH((k_decode_out<MAXC, NTL, NTS, true>), grid, dim3(kBlock), 0, F.stream, F.shards,       \
                           F.parity, total, F.C, dC, dLC, F.n_hdr, every, B, M, F.D);                           \
    else                                                                                                         \
        RFEC_LAUNCH((k_decode_out<MAXC, NTL, NTS, false>), grid, dim3(kBlock), 0, F.stream, F.shards,      \
                           F.parity, total, F.C, dC, dLC, F.n_hdr, every, B, M, F.D)
    switch (sp) {
    case -1: RFEC_FUSED_OUT(false, 1); break;
    case 0: RFEC_FUSED_OUT(true, 0); break;
    case 2: RFEC_FUSED_OUT(true, 2); break;
    case 3: RFEC_FUSED_OUT(true, 3); break;
    default: RFEC_FUSED_OUT(true, 1); break;
    }
#undef RFEC_FUSED_OUT
}

// row-layout fused decode: one lane per (group, row, chunk column), or per
// (group, dense output slot, chunk column) when `slots`
template <int K, int COL>
void launch_fused_rows(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M, uint32_t cd, bool swz,
                       bool slots, uint32_t col_rt = 0)
{
    const uint32_t kk = K ? (uint32_t)K : M.plan.k, cc = K ? (uint32_t)COL : col_rt;
    const uint32_t R = (kk + cc - 1) / cc;
    const uint32_t per = slots ? F.D.E : R;
    const uint32_t total = B.groups * per * cd; // < 2^32: checked by the caller
    const uint32_t npay = blocks_for(total), npay8 = (npay + 7u) & ~7u, nhr = (F.n_hdr + 7u) >> 3;
    // swizzled: rounds of 8 blocks, nhr header rounds spread over npay8 / 8 payload rounds
    const dim3 grid(swz ? 8u * nhr + npay8 : F.n_hdr + npay);
    const uint32_t every = swz ? (F.spread && nhr ? (npay8 >> 3) / nhr : 0u) : hdr_every(F, npay);
    const FastDiv dC = make_fastdiv(cd), dRC = make_fastdiv(per * cd), dCol = make_fastdiv(cc);
#define RFEC_FUSED_ROWS(NTL, NTS)                                                                                \
    if (slots)                                                                                                   \
        RFEC_LAUNCH((k_decode_rows<K, COL, NTL, NTS, true>), grid, dim3(kBlock), 0, F.stream, F.shards,    \
                           F.parity, total, F.C, dC, dRC, F.n_hdr, every, B, M, F.D, swz ? npay8 : 0u, kk, cc,   \
                           dCol);                                                                                \
    else                                                                                                         \
        RFEC_LAUNCH((k_decode_rows<K, COL, NTL, NTS, false>), grid, dim3(kBlock), 0, F.stream, F.shards,   \
                           F.parity, total, F.C, dC, dRC, F.n_hdr, every, B, M, F.D, swz ? npay8 : 0u, kk, cc,   \
                           dCol)
    switch (sp) {
    case -1: RFEC_FUSED_ROWS(false, 1); break;
    case 0: RFEC_FUSED_ROWS(true, 0); break;
    case 2: RFEC_FUSED_ROWS(true, 2); break;
    case 3: RFEC_FUSED_ROWS(true, 3); break;
    default: RFEC_FUSED_ROWS(true, 1); break;
    }
#undef RFEC_FUSED_ROWS
}

// small-slot fused decode with the header work in the payload lanes (cd = CD)
template <int CD, int BATCH, bool WIDE>
void launch_small(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M)
{
    const dim3 grid(blocks_for(B.groups * CD)); // groups * CD < 2^31: check_geometry
#define RFEC_SMALL(NTL, NTS)                                                                                     \
    RFEC_LAUNCH((k_decode_small<CD, BATCH, WIDE, NTL, NTS>), grid, dim3(kBlock), 0, F.stream, F.shards,    \
                       F.parity, F.C, B, M, F.D)
    switch (sp) {
    case -1: RFEC_SMALL(false, 1); break;
    case 0: RFEC_SMALL(true, 0); break;
    case 2: RFEC_SMALL(true, 2); break;
    case 3: RFEC_SMALL(true, 3); break;
    default: RFEC_SMALL(true, 1); break;
    }
#undef RFEC_SMALL
}

// sp: store policy, -1 = plain loads + non-temporal stores (A/B only)
template <int MAXC, int NI>
void launch_fused(const FusedArgs& F, int sp, const PeelArgs& B, const rfec_kmask& M)
{
    const dim3 grid(F.n_hdr + blocks_for((F.total + NI - 1) / NI));
#define RFEC_FUSED(NTL, NTS)                                                                                     \
    RFEC_LAUNCH((k_decode_disjoint<MAXC, NTL, NTS, NI>), grid, dim3(kBlock), 0, F.stream, F.shards,       \
                       F.parity, F.total, F.C, F.f, F.n_hdr, hdr_every(F, grid.x - F.n_hdr), B, M, F.D)
    switch (sp) {
    case -1: RFEC_FUSED(false, 1); break;
    case 0: RFEC_FUSED(true, 0); break;
    case 2: RFEC_FUSED(true, 2); break;
    case 3: RFEC_FUSED(true, 3); break;
    default: RFEC_FUSED(true, 1); break;
    }
#undef RFEC_FUSED
}

// flags -> store cache policy of st16<SP>.  Defaults, measured in the
// encode -> decode alternation bench.py runs (tools/ab_encode.py step mode):
// parity stores write-through (sc0 sc1), recovered-segment stores
// non-temporal; a decode that leaves written-back lines behind slows the
// next write-through encode by ~45%, a non-temporal one does not.
constexpr int kEncodeStoreDefault = 2;
constexpr int kRecoverStoreDefault = 1;

int store_policy(unsigned flags, int dflt)
{
    if (flags & RFEC_KFLAG_PLAIN_STORES)
        return 0;
    if (flags & RFEC_KFLAG_WT_STORES)
        return (flags & RFEC_KFLAG_WT_NT) ? 3 : 2;
    if (flags & RFEC_KFLAG_NT_STORES)
        return 1;
    return dflt;
}

// the sender's full plan of a k-segment group in rows of `col`: rows, then
// columns, lines with fewer than 2 members dropped (flex_fec_sender.c:166-233)
bool is_full_matrix(const rfec_kplan* P, uint32_t col)
{
    const uint32_t k = P->k, rows = (k + col - 1) / col;
    uint32_t l = 0;
    for (uint32_t r = 0; r < rows; ++r) {
        const uint32_t cnt = k - r * col < col ? k - r * col : col;
        if (cnt < 2)
            continue;
        if (l >= P->n_lines || P->line[l].first != r * col || P->line[l].stride != 1 || P->line[l].count != cnt)
            return false;
        ++l;
    }
    for (uint32_t c = 0; c < col; ++c) {
        const uint32_t cnt = (k - c + col - 1) / col;
        if (cnt < 2)
            continue;
        if (l >= P->n_lines || P->line[l].first != c || P->line[l].stride != col || P->line[l].count != cnt)
            return false;
        ++l;
    }
    return l == P->n_lines;
}

bool is_row_layout(const rfec_kplan* P, uint32_t* col_out)
{
    const uint32_t col = P->n_lines ? P->line[0].count : 0;
    bool rows = col >= 2 && P->n_lines == (P->k + col - 1) / col;
    for (uint32_t l = 0; l < P->n_lines && rows; ++l) {
        const uint32_t first = l * col;
        const uint32_t count = P->k - first < col ? P->k - first : col;
        rows = P->line[l].stride == 1 && P->line[l].first == first && P->line[l].count == count;
    }
    *col_out = col;
    return rows;
}

template <bool NTL, int NTS>
hipError_t launch_encode_t(const EncLaunch& a, unsigned flags)
{
    const rfec_kplan* P = a.P;
    uint32_t col = 0;
    if (!(flags & RFEC_KFLAG_GENERIC) && is_row_layout(P, &col)) {
        if (P->k == 10 && col == 4)
            return launch_rows_v<10, 4, NTL, NTS>(a, flags);
        if (P->k == 32 && col == 4)
            return launch_rows_v<32, 4, NTL, NTS>(a, flags);
        // other row layouts: the same output-mapped lanes with k and col at run time
        if (!(flags & (RFEC_KFLAG_FLAT_ENCODE | RFEC_KFLAG_GROUP_WAVE | RFEC_KFLAG_ITEMS2)) && col <= 16 &&
            (uint64_t)a.groups * ((P->k + col - 1) / col) * a.cd < (1ull << 32)) {
            // (an 8-wide instantiation compiled to 230 VGPRs, two waves per SIMD: 0.33 of 8 TB/s at k = 20,
            // col = 5, so rows of 5..16 take the 16-wide one, 74 VGPRs)
            if (col <= 4)
                return launch_rows_out_rt<4, NTL, NTS>(a, flags, col);
            return launch_rows_out_rt<16, NTL, NTS>(a, flags, col);
        }
    }
    const uint32_t C = a.stride / 16;
    const uint32_t total = a.groups * a.cd;
    if (!(flags & RFEC_KFLAG_GENERIC) && P->k >= 6 && P->k <= 16 && is_full_matrix(P, P->k <= 9 ? 3 : 4)) {
        const dim3 grid(a.E.n_meta_blocks + blocks_for(total));
#define RFEC_MX(KK, CC)                                                                                           \
    case KK:                                                                                                      \
        RFEC_LAUNCH((k_encode_matrix<KK, CC, NTL, NTS>), grid, dim3(kBlock), 0, a.stream, a.s, a.p, total, C, \
                           make_fastdiv(a.cd), a.E, *P);                                                          \
        return hipGetLastError();
        switch (P->k) {
            RFEC_MX(6, 3) RFEC_MX(7, 3) RFEC_MX(8, 3) RFEC_MX(9, 3) RFEC_MX(10, 4) RFEC_MX(11, 4) RFEC_MX(12, 4)
            RFEC_MX(13, 4) RFEC_MX(14, 4) RFEC_MX(15, 4) RFEC_MX(16, 4)
        default: break;
        }
#undef RFEC_MX
    }
    if (!(flags & RFEC_KFLAG_GENERIC) && P->k <= 16) {
        LineMasks16 LM;
        LM.n = P->n_lines;
        for (uint32_t l = 0; l < P->n_lines; ++l) {
            uint32_t m = 0;
            for (uint32_t q = 0; q < P->line[l].count; ++q)
                m |= 1u << (P->line[l].first + q * P->line[l].stride);
            LM.m[l] = (uint16_t)m;
        }
        RFEC_LAUNCH((k_encode_k16<NTL, NTS>), dim3(a.E.n_meta_blocks + blocks_for(total)), dim3(kBlock), 0,
                           a.stream, a.s, a.p, total, C, make_fastdiv(a.cd), a.E, *P, LM);
        return hipGetLastError();
    }
    RFEC_LAUNCH((k_encode<NTL, NTS>), dim3(a.E.n_meta_blocks + blocks_for(total)), dim3(kBlock), 0, a.stream,
                       a.s, a.p, total, C, make_fastdiv(a.cd), a.E, *P);
    return hipGetLastError();
}

} // namespace

extern "C" int rfec_timing_events(void* start, void* stop)
{
    t_ev_start = reinterpret_cast<hipEvent_t>(start);
    t_ev_stop = reinterpret_cast<hipEvent_t>(stop);
    t_launches = 0;
    return 0;
}

extern "C" uint32_t rfec_timing_launches(void) { return t_launches; }

extern "C" {

int rfec_launch_encode(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                       const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                       uint16_t* fsize, int8_t* status, void* stream, unsigned flags)
{
    EncMeta E;
    E.hdr_dw = reinterpret_cast<const uint32_t*>(hdr);
    E.meta_dw = reinterpret_cast<uint32_t*>(meta);
    E.fsize = fsize;
    E.status = status;
    E.groups = groups;
    E.capacity = capacity;
    uint32_t gpb = kMetaDwords / (5u * P->k);
    gpb = gpb < 1 ? 1 : (gpb > 64 ? 64 : gpb);
    if (gpb >= 4)
        gpb &= ~3u; // keeps every block's header slice 16-byte aligned
    E.gpb = gpb;
    E.n_meta_blocks = (flags & RFEC_KFLAG_DIAG_NO_META) ? 0 : (groups + gpb - 1) / gpb;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    const EncLaunch a = {P, groups, stride, cd, reinterpret_cast<const v4u*>(shards), reinterpret_cast<v4u*>(parity),
                         E, reinterpret_cast<hipStream_t>(stream)};
    if (flags & RFEC_KFLAG_PLAIN_LOADS) // A/B only
        return (int)launch_encode_t<false, 1>(a, flags);
    // default store policy (rotated-buffer benches): write-through (kEncodeStoreDefault) for the row
    // layouts over slots that split 128-B lines (k = 10 / 1,200 B: 173 vs 177 us non-temporal),
    // non-temporal where every parity slot is whole lines (k = 32 / 256 B: 120 vs 136 us) and for the
    // other plans, which write two parities per segment or more (the full row + column plan: 285 vs
    // 312 us at k = 10)
    // The output-mapped row kernel (default) writes whole lines: non-temporal
    // (tools/step_ab.py: 172.7 us vs 185.8 write-through once the decode
    // reads a parity set that is not MALL-resident).
    uint32_t col = 0;
    const int dflt =
        (flags & RFEC_KFLAG_FLAT_ENCODE) && is_row_layout(P, &col) && stride % 128 != 0 ? kEncodeStoreDefault : 1;
    switch (store_policy(flags, dflt)) {
    case 0: return (int)launch_encode_t<true, 0>(a, flags);
    case 2: return (int)launch_encode_t<true, 2>(a, flags);
    case 3: return (int)launch_encode_t<true, 3>(a, flags);
    default: return (int)launch_encode_t<true, 1>(a, flags);
    }
}

} // extern "C"

namespace {

int launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity, uint8_t* shards,
                   rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity, const rfec_hdr* meta,
                   const uint16_t* fsize, const uint64_t* parity_present, uint64_t* recovered, void* ws,
                   void* stream, unsigned flags, const rfec_dense_out* out)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const bool dense = out && out->per_group;
    if (dense) // the dense-output forms: fused decodes, header lanes (the host checks the plan is disjoint)
        flags &= ~(RFEC_KFLAG_WAVE_DECODE | RFEC_KFLAG_TWO_KERNEL_DECODE | RFEC_KFLAG_PIPE_DECODE |
                   RFEC_KFLAG_GROUP_WAVE | RFEC_KFLAG_LDS_HDR_PEEL);
    const bool ntl = !(flags & RFEC_KFLAG_PLAIN_LOADS);
    if (flags & RFEC_KFLAG_WAVE_DECODE) {
        RecArgs A;
        A.shards = reinterpret_cast<v4u*>(shards);
        A.hdr = hdr;
        A.present = present;
        A.parity = reinterpret_cast<const v4u*>(parity);
        A.meta = meta;
        A.fsize = fsize;
        A.parity_present = parity_present;
        A.recovered = recovered;
        A.groups = groups;
        A.C = stride / 16;
        A.Cd = capacity ? (capacity + 15) / 16 : 1;
        A.capacity = capacity;
        const dim3 grid((unsigned)(((uint64_t)groups * kWave + kBlock - 1) / kBlock));
        if (ntl)
            RFEC_LAUNCH(k_recover<true>, grid, dim3(kBlock), 0, st, A, *M);
        else
            RFEC_LAUNCH(k_recover<false>, grid, dim3(kBlock), 0, st, A, *M);
        return (int)hipGetLastError();
    }
    const rfec_kplan& P = M->plan;
    PeelArgs B;
    B.hdr = hdr;
    B.present = present;
    B.meta = meta;
    B.fsize = fsize;
    B.parity_present = parity_present;
    B.recovered = recovered;
    B.sched = reinterpret_cast<uint8_t*>(ws);
    B.groups = groups;
    B.capacity = capacity;
    B.rec_bytes = rfec_sched_record_bytes(P.n_lines);
    B.out_hdr = dense ? out->hdr : nullptr;
    B.out_index = dense ? out->index : nullptr;
    B.out_per_group = dense ? out->per_group : 0u;
    const DenseOut DO = {dense ? reinterpret_cast<v4u*>(out->shards) : nullptr, dense ? out->per_group : 0u};
    uint64_t seen0 = 0, seen1 = 0;
    B.disjoint = 1;
    for (uint32_t l = 0; l < P.n_lines; ++l) {
        if ((seen0 & M->mask[l][0]) | (seen1 & M->mask[l][1]))
            B.disjoint = 0;
        seen0 |= M->mask[l][0];
        seen1 |= M->mask[l][1];
    }
    uint32_t maxc = 0;
    for (uint32_t l = 0; l < P.n_lines; ++l)
        maxc = P.line[l].count > maxc ? P.line[l].count : maxc;
    // disjoint plans (row layer alone, strip mode) decode in one launch
    const bool fused = B.disjoint && maxc <= 8 && !(flags & (RFEC_KFLAG_TWO_KERNEL_DECODE | RFEC_KFLAG_PIPE_DECODE));
    if (dense && !fused)
        return (int)hipErrorInvalidValue; // rfec_recover_batch_out checks this first
    // plans with cascades (the sender's matrix plans): one launch + fix-up
    const bool cascade = !B.disjoint && maxc <= 8 &&
                         !(flags & (RFEC_KFLAG_TWO_KERNEL_DECODE | RFEC_KFLAG_PIPE_DECODE));
    B.fixc = reinterpret_cast<unsigned long long*>(reinterpret_cast<uint8_t*>(ws) + rfec_ws_fix_offset(P.n_lines, groups));
    B.fixlist = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(B.fixc) + 16);
    B.gen = cascade ? next_gen() : 0u;
    // LDS per group: K + NL header records (5 dwords) + NL u16 sizes; block
    // ranges start on 8-group boundaries so the staged slices are 16-B aligned
    const uint32_t per = 5u * P.k + 6u * P.n_lines;
    // (at most 64 groups per block: the peel is one serial chain per lane, so
    // more, smaller blocks give each SIMD more chains to interleave)
    uint32_t gpb = ((fused || cascade ? kFusedPeelDwords : kPeelDwords) - 8) / per;
    gpb = gpb > 64u ? 64u : gpb;
    if (gpb >= 8)
        gpb &= ~7u;
    B.gpb = gpb < 1 ? 1 : gpb;
    uint32_t n_hdr = (groups + B.gpb - 1) / B.gpb;
    // fused decode: header lanes, one per (group, line), unless A/B asks for the LDS peel blocks
    B.nlp_log2 = 0;
    if (fused && !(flags & RFEC_KFLAG_LDS_HDR_PEEL)) {
        uint32_t lg = 1;
        while ((1u << lg) < P.n_lines)
            ++lg;
        B.nlp_log2 = lg;
        n_hdr = (uint32_t)((((uint64_t)groups << lg) + kBlock - 1) / kBlock); // host checks groups << lg < 2^32
    }
    if (fused && (flags & RFEC_KFLAG_DIAG_NO_HDR))
        n_hdr = 0; // timing only: no recovered headers / masks
    const uint32_t C = stride / 16;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    const uint32_t total = groups * cd;
    const dim3 grid(blocks_for(total));
    const FastDiv f = make_fastdiv(cd);
    const v4u* pp = reinterpret_cast<const v4u*>(parity);
    v4u* sh = reinterpret_cast<v4u*>(shards);
    if (fused) {
        // header blocks spread over the grid by default (tools/step_ab.py, cold: k = 32 / 256 B flat
        // 41.6 vs 46.9 us at the head; k = 10 / 1,200 B rows 139.4-141.1 vs 144.0-144.4 us)
        const FusedArgs F = {sh, pp, total, C, f, n_hdr, st, !(flags & RFEC_KFLAG_HDR_HEAD), DO};
        const int sp = ntl ? store_policy(flags, kRecoverStoreDefault) : -1;
        const GwGeom gg = gw_geom(groups, cd);
        const uint32_t swz = (flags & RFEC_KFLAG_XCD_SWIZZLE) ? 1u : 0u;
        if ((flags & RFEC_KFLAG_GROUP_WAVE) && gg.ni <= 2) {
            if (maxc <= 4 && gg.ni == 1)
                launch_fused_gw<4, 1>(F, sp, B, *M, gg, swz);
            else if (maxc <= 4)
                launch_fused_gw<4, 2>(F, sp, B, *M, gg, swz);
            else if (gg.ni == 1)
                launch_fused_gw<8, 1>(F, sp, B, *M, gg, swz);
            else
                launch_fused_gw<8, 2>(F, sp, B, *M, gg, swz);
            return (int)hipGetLastError();
        }
        const bool two = (flags & RFEC_KFLAG_ITEMS2) != 0;
        // A/B: slots of 16 or 32 chunks, lines of <= 4, header work in the payload lanes (k_decode_small).
        // Slower than header blocks + the flat lanes at c5 (k = 32 / 256 B, cold parity, tools/gpu_v4.sh:
        // 40.8 us one line per pass, 48.1 us two, vs 35.9 us), so not the default.
        if ((flags & RFEC_KFLAG_SMALL_FUSED) && !two && (cd == 16 || cd == 32) && maxc <= 4) {
            const bool wide = P.k > 64, b2 = (flags & RFEC_KFLAG_SMALL_B2) != 0;
            if (cd == 16 && !b2)
                wide ? launch_small<16, 1, true>(F, sp, B, *M) : launch_small<16, 1, false>(F, sp, B, *M);
            else if (cd == 16)
                wide ? launch_small<16, 2, true>(F, sp, B, *M) : launch_small<16, 2, false>(F, sp, B, *M);
            else
                wide ? launch_small<32, 1, true>(F, sp, B, *M) : launch_small<32, 1, false>(F, sp, B, *M);
            return (int)hipGetLastError();
        }
        // output-mapped (a lane per (group, line, chunk)) where a line's slot spans at least a wave of
        // chunks; below that most of its lanes would sit on lines that do not fire (k = 32 / 256 B, 2
        // erasures: 6 of 8 rows idle, 60.0 vs 41.6 us flat), so the flat form
        if (!two && !(flags & RFEC_KFLAG_FLAT_DECODE) && (cd >= (uint32_t)kWave || (flags & RFEC_KFLAG_OUT_DECODE)) &&
            (uint64_t)groups * P.n_lines * cd < (1ull << 32)) {
            uint32_t col = 0;
            // dense output: lanes per output slot (no lane on a line that does not fire)
            const bool slots = F.D.E && F.D.E <= P.n_lines && !(flags & RFEC_KFLAG_LINE_LANES);
            if (!(flags & RFEC_KFLAG_GENERIC) && is_row_layout(&P, &col) && col == 4 &&
                (P.k == 10 || P.k == 32)) {
                // XCD-swizzled by default: decode traffic 1.077 vs 1.107 x algorithmic at k = 10 / 1,200 B,
                // time within noise (130.0-130.4 vs 129.2 us, tools/gpu_xcd.sh)
                const bool swz = !(flags & RFEC_KFLAG_LINEAR_BLOCKS);
                if (P.k == 10)
                    launch_fused_rows<10, 4>(F, sp, B, *M, cd, swz, slots);
                else
                    launch_fused_rows<32, 4>(F, sp, B, *M, cd, swz, slots);
                return (int)hipGetLastError();
            }
            // other row layouts of k <= 64, rows of <= 4 members: the same kernel with k and col at run time
            if (!(flags & RFEC_KFLAG_GENERIC) && is_row_layout(&P, &col) && col <= 4 && P.k <= 64) {
                launch_fused_rows<0, 4>(F, sp, B, *M, cd, !(flags & RFEC_KFLAG_LINEAR_BLOCKS), slots, col);
                return (int)hipGetLastError();
            }
            if (maxc <= 4)
                launch_fused_out<4>(F, sp, B, *M, cd, slots);
            else
                launch_fused_out<8>(F, sp, B, *M, cd, slots);
            return (int)hipGetLastError();
        }
        if (maxc <= 4 && two)
            launch_fused<4, 2>(F, sp, B, *M);
        else if (maxc <= 4)
            launch_fused<4, 1>(F, sp, B, *M);
        else
            launch_fused<8, 1>(F, sp, B, *M);
        return (int)hipGetLastError();
    }
    if (cascade) {
        const FusedArgs F = {sh, pp, total, C, f, n_hdr, st, false, DO};
        const int sp = ntl ? store_policy(flags, kRecoverStoreDefault) : -1;
        if (maxc <= 4)
            launch_cascade<4, 2>(F, sp, B, *M);
        else
            launch_cascade<8, 1>(F, sp, B, *M);
        return (int)hipGetLastError();
    }
    RFEC_LAUNCH(k_peel_lds, dim3(n_hdr), dim3(kBlock), 0, st, B, *M);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return (int)e;
    const uint8_t* sc = B.sched;
    const int nts = store_policy(flags, kRecoverStoreDefault);
    const uint32_t fast = (maxc <= 8 ? 1u : 0u) | ((flags & RFEC_TUNE_DIAG_CONST_SCHED) ? 2u : 0u);
    const ReplayArgs R = {sh, pp, sc, total, C, f, B.rec_bytes, fast, st};
    if (maxc <= 4 && (flags & RFEC_KFLAG_PIPE_DECODE))
        launch_replay<4, 2, true>(R, ntl, nts, P, dim3(grid.x < 4096u ? grid.x : 4096u));
    else if (maxc <= 4)
        launch_replay<4, 2, false>(R, ntl, nts, P, grid);
    else
        launch_replay<8, 1, false>(R, ntl, nts, P, grid);
    return (int)hipGetLastError();
}

} // namespace

extern "C" {

int rfec_launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                        uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fsize, const uint64_t* parity_present,
                        uint64_t* recovered, void* ws, void* stream, unsigned flags)
{
    return launch_recover(M, groups, stride, capacity, shards, hdr, present, parity, meta, fsize, parity_present,
                          recovered, ws, stream, flags, nullptr);
}

int rfec_launch_recover_out(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                            const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                            const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                            const uint64_t* parity_present, uint64_t* recovered, void* ws, void* stream,
                            unsigned flags, const rfec_dense_out* out)
{
    // the fused decodes only read the shards and headers when the output is dense
    return launch_recover(M, groups, stride, capacity, const_cast<uint8_t*>(shards), const_cast<rfec_hdr*>(hdr),
                          present, parity, meta, fsize, parity_present, recovered, ws, stream, flags, out);
}

int rfec_launch_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                            void* stream)
{
    const uint32_t C = stride / 16;
    const uint32_t total = rows * C;
    if (!total)
        return 0;
    RFEC_LAUNCH(k_gather_rows, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<v4u*>(dst), reinterpret_cast<const v4u*>(src), map, total, C, make_fastdiv(C));
    return (int)hipGetLastError();
}

int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream)
{
    const uint32_t C = stride / 16;
    const uint32_t total = slots * C;
    RFEC_LAUNCH(k_zero_tails, dim3(blocks_for(total)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<v4u*>(shards), hdr, total, C,
                       make_fastdiv(C));
    return (int)hipGetLastError();
}

const char* rfec_hip_error_string(int code) { return hipGetErrorString((hipError_t)code); }

} // extern "C"
