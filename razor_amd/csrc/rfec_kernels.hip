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
// Every payload load and store is non-temporal (measured best for both
// directions of the encode -> decode alternation).
//
//  encode (one launch; meta blocks at the head of the grid XOR the 20-byte
//  header records of up to 64 groups staged in LDS, one lane per (group, line)):
//    * row layouts (the sender's row layer, strip mode): k_encode_out, one
//      lane per PARITY chunk loading its row's members, XCD-swizzled blocks;
//    * the sender's full rows + columns plan (k = 6..16): k_encode_matrix_out,
//      one lane per PARITY chunk (group, line, chunk), member loads at the
//      default policy so a column's lanes re-read its members from L2 (at the
//      10 : 7 read / write mix's streaming ceiling, rfec_probe_mix);
//    * any other plan: k_encode (plan-driven).
//  recover (rfec_launch_recover picks by plan):
//    * pairwise disjoint lines (row layer, strip mode), one launch: header
//      lanes (one per (group, line)) spread over the grid, then
//      k_decode_rows (row layouts: one lane per (group, row or output slot,
//      chunk)), k_decode_out (other plans, slots of >= 64 chunks) or
//      k_decode_disjoint (one lane per (group, chunk column));
//    * lines that cascade (the sender's rows + columns: k <= 64, <= 8 lines of
//      <= 4 members), one launch: k_decode_cascade, one lane per (group, slot,
//      chunk column) that derives the canonical schedule, runs the header
//      checks of the steps it depends on and recomputes them in registers;
//    * otherwise (and RFEC_TUNE_GENERIC): k_peel_lds (schedule records) +
//      k_recover_flat (replay).
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

// payload streams: non-temporal loads and stores (every byte is touched once)
__device__ __forceinline__ v4u ld16(const v4u* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st16(v4u* p, v4u v) { __builtin_nontemporal_store(v, p); }

// Predicated member loads of the decodes: a buffer descriptor over the wave's
// first group (wave-uniform base, made provably uniform by readfirstlane) and
// per-lane byte offsets; a load that is not wanted takes kNoLoad, past the
// descriptor's range, and returns zeros without touching memory.  No branch
// and no redundant request: with per-load branches hipcc waited on each load
// before the next (c3 decode 130 us), with loads redirected to an address
// already in flight it issued 25-150 % more requests (127 us).
constexpr uint32_t kNoLoad = 0x7FFFFFF0u;
constexpr int kAuxNT = 2; // gfx950 cache-policy bits: nt
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p)
{
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t)hi << 32 | lo), 0, (int)kNoLoad,
                                             0x00020000);
}
__device__ __forceinline__ v4u bld16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxNT));
}
__device__ __forceinline__ v4u bld16_l2(__amdgpu_buffer_rsrc_t r, uint32_t off) // default policy (kept in L2)
{
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// Payload-block index, XCD-swizzled.  Workgroups are dispatched round-robin
// over the 8 XCDs (block b runs on XCD b % 8, each XCD with its own L2); the
// swizzle gives every XCD one contiguous range of logical blocks, so a cache
// line shared by neighbouring blocks is fetched into one L2.  The tail beyond
// the last multiple of 8 keeps the identity mapping (a bijection).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb)
{
    const uint32_t nb8 = nb & ~7u;
    if (b >= nb8)
        return b;
    return (b & 7u) * (nb8 >> 3) + (b >> 3);
}

// Header / meta blocks spread in rounds of 8 blocks (one per XCD: block b runs on XCD
// b % 8) for the XCD-swizzled decodes: the first round of every (every + 1) is
// a round of 8 header blocks until n_hr of them ran, so the payload blocks fill
// whole rounds and payload block p (in payload order) runs on XCD p % 8; it
// then takes logical block xcd_block(p): consecutive logical blocks share an
// XCD's L2 (the 128-B lines split between neighbouring slots are fetched once)
// and XCD x sweeps its eighth of the groups in order.  XCD x's header blocks
// are x n_hr + 0, 1, ...: the groups its own payload rounds reach next, so the
// header blocks' reads of the masks come in through the same L2 just before
// the payload lanes read them (the cascade decode: 128.3-128.8 vs 129.4-130.3
// us with header block per * 8 + x, last in each period).
// npay8: payload blocks rounded up to a multiple of 8.
__device__ __forceinline__ bool header_block_xcd(uint32_t n_hr, uint32_t every, uint32_t npay8, uint32_t* hb,
                                                 uint32_t* pb)
{
    const uint32_t R = blockIdx.x >> 3, x = blockIdx.x & 7u;
    uint32_t pr;
    if (!every) {
        if (R < n_hr) {
            *hb = x * n_hr + R;
            return true;
        }
        pr = R - n_hr;
    } else {
        const uint32_t per = R / (every + 1);
        if (per < n_hr && R == per * (every + 1)) {
            *hb = x * n_hr + per;
            return true;
        }
        pr = R - min(per + 1, n_hr);
    }
    *pb = xcd_block(pr * 8u + x, npay8);
    return false;
}


// Copies n dwords global -> LDS with the whole block (nt lanes), several loads
// in flight per lane: the loads go through a buffer descriptor over exactly
// the n dwords, so a lane past the end reads zeros with no branch around the
// load (hipcc waited on each guarded load before issuing the next).  `lds`
// must be 16-byte aligned; 16-byte loads are used when `src` is too.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const void* p, uint32_t nbytes)
{
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t)hi << 32 | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane((int)nbytes), 0x00020000);
}

__device__ __forceinline__ void stage_dwords(uint32_t* lds, const uint32_t* __restrict__ src, uint32_t n,
                                             uint32_t nt = kBlock)
{
    constexpr int U = 4;
    const __amdgpu_buffer_rsrc_t r = span_rsrc(src, n * 4u);
    const uint32_t nv = ((reinterpret_cast<uintptr_t>(src) & 15) == 0) ? n / 4 : 0;
    v4u* d4 = reinterpret_cast<v4u*>(lds);
    for (uint32_t base = 0; base < nv; base += U * nt) {
        v4u tmp[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            tmp[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(
                                                 r, (base + u * nt + threadIdx.x) * 16u, 0, 0));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = base + u * nt + threadIdx.x;
            if (i < nv)
                d4[i] = tmp[u];
        }
    }
    for (uint32_t base = nv * 4; base < n; base += 4 * U * nt) {
        uint32_t tmp[4 * U];
#pragma unroll
        for (int u = 0; u < 4 * U; ++u)
            tmp[u] = __builtin_amdgcn_raw_buffer_load_b32(r, (base + u * nt + threadIdx.x) * 4u, 0, 0);
#pragma unroll
        for (int u = 0; u < 4 * U; ++u) {
            const uint32_t i = base + u * nt + threadIdx.x;
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
// (lds: kMetaDwords, 16-byte aligned; nt: the block's threads)
__device__ void meta_block_in(uint32_t* lds, uint32_t nt, uint32_t mb, const uint32_t* __restrict__ hdr_dw,
                              uint32_t* __restrict__ meta_dw, uint16_t* __restrict__ fsize,
                              int8_t* __restrict__ status, uint32_t groups, uint32_t capacity, uint32_t gpb,
                              const rfec_kplan& P)
{
    const uint32_t K = P.k, NL = P.n_lines;
    const uint32_t g0 = mb * gpb;
    const uint32_t ng = min(gpb, groups - g0);
    stage_dwords(lds, hdr_dw + (size_t)g0 * K * 5, ng * K * 5, nt);
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < ng * NL; o += nt) {
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

__device__ void meta_block(uint32_t mb, const uint32_t* __restrict__ hdr_dw, uint32_t* __restrict__ meta_dw,
                           uint16_t* __restrict__ fsize, int8_t* __restrict__ status, uint32_t groups,
                           uint32_t capacity, uint32_t gpb, const rfec_kplan& P)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kMetaDwords];
    meta_block_in(lds, kBlock, mb, hdr_dw, meta_dw, fsize, status, groups, capacity, gpb, P);
}

struct EncMeta {
    const uint32_t* hdr_dw;
    uint32_t* meta_dw;
    uint16_t* fsize;
    int8_t* status;
    uint32_t groups, capacity, gpb, n_meta_blocks;
};

// Grid of the swizzled encodes: head / 8 rounds of 8 meta blocks spread over
// the payload rounds (header_block_xcd; the payload part of the grid is whole
// rounds of 8), so the meta blocks' latency-bound header stages overlap the
// payload stream instead of holding the whole GPU at the start of the launch:
// c5 (k = 32 / 256 B, 8 % header bytes) 113.4-113.6 vs 117.9-119.4 us, c3
// 161.7-162.2 vs 162.8-163.4 us (round 5, profiles/r05/ab/enc_meta_spread/).
// Returns false for meta / padding blocks (meta work done), else the logical
// payload block.
__device__ __forceinline__ bool enc_payload_block(const EncMeta& E, uint32_t head, const rfec_kplan& P, uint32_t* b)
{
    const uint32_t n_mr = head >> 3, npay8 = gridDim.x - head;
    const uint32_t every = n_mr ? (npay8 >> 3) / n_mr : 0u;
    uint32_t mb;
    if (header_block_xcd(n_mr, every, npay8, &mb, b)) {
        if (mb < E.n_meta_blocks)
            meta_block(mb, E.hdr_dw, E.meta_dw, E.fsize, E.status, E.groups, E.capacity, E.gpb, P);
        return false;
    }
    return true;
}

// ---------------------------------------------------------------------------
// Encode payload, generic plan: one lane per (group, chunk column), every
// line's members loaded in turn.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_encode(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                   uint32_t total, uint32_t C, FastDiv divC, EncMeta E, rfec_kplan P)
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
        v4u acc = ld16(s);
        uint32_t q = 1;
        for (; q + 4 <= ln.count; q += 4) { // four loads in flight
            const v4u a = ld16(s + q * step), b = ld16(s + (q + 1) * step);
            const v4u c = ld16(s + (q + 2) * step), d = ld16(s + (q + 3) * step);
            acc ^= (a ^ b) ^ (c ^ d);
        }
        for (; q < ln.count; ++q)
            acc ^= ld16(s + q * step);
        st16(dst + (size_t)l * C, acc);
    }
}

// ---------------------------------------------------------------------------
// Encode payload, the reference sender's full matrix plan at small k
// (flex_fec_sender.c:166-233: rows of COL consecutive segments, then columns
// strided by COL, lines with fewer than 2 members dropped), K = 6..16 (COL =
// 3 or 4, as flex_fec_sender_num_packets picks); MatrixShape = its compile-time
// line layout.
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

// Output-mapped form of the full matrix encode: one lane per PARITY chunk
// (group, line, chunk column), as k_encode_out, so that every wave's store is
// 1 KiB of consecutive parity bytes (whole 128-B lines when the slots are
// packed) instead of seven 1 KiB runs that start and end inside lines shared
// with the neighbouring waves.  Each member is loaded by its row's lanes and
// again by its column's lanes one block or so later, on the same XCD, so HBM
// should still see every member once (PMC: 1.018 x algorithmic).  Row l <
// NR: members l COL + q; column c = l - NR: c + q COL (K >= 2 COL here, so no
// column has fewer than 2 members).  Loads take the default policy: the
// column lanes' second reads are meant to hit L2.  At c3 full (10 reads : 7
// writes per group) 228-230 us with the unused member slots predicated off
// through a buffer descriptor (round 5; 234-237 us when they re-read member
// 0; non-temporal loads on the rows, the columns or both: 239-242 us,
// profiles/r05/ab/encode_pred/).
// Measured slower: one lane per (group, chunk) loading each member once, all
// seven parity chunks through LDS and stored as one contiguous run per block
// (238-239 us, round 4); the same with seven direct stores per lane (252-260
// us, round 2: every 1-KiB store run starts and ends inside lines that the
// neighbouring waves write).
template <int K, int COL>
__global__ __launch_bounds__(kBlock) void k_encode_matrix_out(const v4u* __restrict__ shards,
                                                              v4u* __restrict__ parity, uint32_t total, uint32_t C,
                                                              FastDiv divC, FastDiv divLC, uint32_t head, EncMeta E,
                                                              rfec_kplan P)
{
    using Sh = MatrixShape<K, COL>;
    constexpr int NR = Sh::n_rows(), R = Sh::R, M = COL > R ? COL : R;
    static_assert(K >= 2 * COL && Sh::n_lines() == NR + COL, "every column has >= 2 members");
    uint32_t b;
    if (!enc_payload_block(E, head, P, &b))
        return;
    const uint32_t t = b * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divLC);
    const uint32_t rem = t - g * divLC.d;
    const uint32_t l = fdiv(rem, divC);
    const uint32_t j = rem - l * divC.d;
    const bool row = l < (uint32_t)NR;
    const uint32_t c = l - NR;
    const uint32_t first = row ? l * COL : c, step = row ? 1u : (uint32_t)COL;
    const uint32_t count = row ? min((uint32_t)COL, K - l * COL) : (K - c + COL - 1) / COL;
    // member loads through a descriptor over the wave's first group, an unused
    // slot predicated off (kNoLoad reads 0 without a memory access), default
    // policy: the column lanes' second reads are meant to hit L2
    const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
    const __amdgpu_buffer_rsrc_t rs = wave_rsrc(shards + (size_t)gb * K * C);
    const uint32_t o0 = (((g - gb) * K + first) * C + j) * 16u;
    v4u v[M];
#pragma unroll
    for (int q = 0; q < M; ++q)
        v[q] = bld16_l2(rs, (uint32_t)q < count ? o0 + (uint32_t)q * step * C * 16u : kNoLoad);
    v4u acc = v[0];
#pragma unroll
    for (int q = 1; q < M; ++q)
        acc ^= v[q];
    st16(parity + ((size_t)g * (NR + COL) + l) * C + j, acc);
}

// ---------------------------------------------------------------------------
// Encode payload, rows-of-COL, output-mapped (default for row layouts): one
// lane per PARITY chunk (group, row, chunk column), the lane loads its row's
// COL (last row: K - (R-1)*COL) member chunks and stores one chunk.  Lane t
// writes parity chunk t when the slots are packed (stride == capacity), so
// every wave's store is 1 KiB of consecutive, 128-B-aligned parity bytes:
// whole lines, never two partial writes of one line from two waves on two
// XCDs, which a flat (group, chunk) mapping makes at every 1,200-B slot
// edge.  Row layouts have no member in two lines, so no chunk is loaded twice.
// 165-171 us vs 178-211 us flat at k = 10 / 1,200 B, equal to a 10-read :
// 3-write probe over contiguous streams; XCD-swizzled blocks: 168 vs 172 us,
// HBM traffic 1.029 vs 1.059 x algorithmic.  Round 5: the last row's absent
// members predicated off through a buffer descriptor instead of per-load
// branches: 163-166 vs 166-168 us (profiles/r05/ab/encode_pred/).
// ---------------------------------------------------------------------------
template <int K, int COL>
__global__ __launch_bounds__(kBlock) void k_encode_out(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                       uint32_t total, uint32_t C, FastDiv divC, FastDiv divRC,
                                                       uint32_t head, EncMeta E, rfec_kplan P)
{
    constexpr int R = (K + COL - 1) / COL;
    constexpr int LAST = K - (R - 1) * COL;
    uint32_t b;
    if (!enc_payload_block(E, head, P, &b))
        return;
    const uint32_t t = b * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divRC);
    const uint32_t rem = t - g * divRC.d;
    const uint32_t r = fdiv(rem, divC);
    const uint32_t j = rem - r * divC.d;
    // member loads predicated through a descriptor (the last row's missing
    // members read 0 without a memory access), not per-load branches
    const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
    const __amdgpu_buffer_rsrc_t rs = wave_rsrc(shards + (size_t)gb * K * C);
    const uint32_t o0 = (((g - gb) * K + r * COL) * C + j) * 16u;
    v4u v[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q)
        v[q] = bld16(rs, (q < LAST || r < (uint32_t)(R - 1)) ? o0 + (uint32_t)q * C * 16u : kNoLoad);
    v4u acc = v[0];
#pragma unroll
    for (int q = 1; q < COL; ++q)
        acc ^= v[q];
    st16(parity + ((size_t)g * R + r) * C + j, acc);
}

// The same for any row layout with rows of at most CMAX members (k, col
// runtime: the strip-mode plans of flex_fec_sender_num_packets, :112-132);
// the lane's member loads stay unrolled, predicated on the row's size.
template <int CMAX>
__global__ __launch_bounds__(kBlock) void k_encode_out_rt(const v4u* __restrict__ shards, v4u* __restrict__ parity,
                                                          uint32_t total, uint32_t C, FastDiv divC, FastDiv divRC,
                                                          uint32_t K, uint32_t COL, uint32_t head, EncMeta E,
                                                          rfec_kplan P)
{
    uint32_t b;
    if (!enc_payload_block(E, head, P, &b))
        return;
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
            v[q] = ld16(s + (size_t)q * C);
    }
    v4u acc = v[0];
#pragma unroll
    for (int q = 1; q < CMAX; ++q)
        acc ^= v[q];
    st16(parity + ((size_t)g * R + r) * C + j, acc);
}

// ---------------------------------------------------------------------------
// Recover.
//
// Peeling = the fixpoint reached by flex_recover_row / flex_recover_col
// (flex_fec_receiver.c:105-206) as segments, parities and recovered segments
// (sim_receiver.c:780-804) arrive; canonical order: lines in plan order,
// repeated until nothing fires.  A line fires when its parity is present,
// exactly one member is missing, at least one is present (:133-140,
// :189-196) and flex_fec_recover would succeed: fec_data_size within the
// capacity, every member's data_size <= fec_data_size (flex_fec_xor.c:88-89)
// and the recovered data_size <= fec_data_size (:98-99).
//
// Two-kernel form (generic): k_peel_lds runs that peel, one lane per group,
// over the group's headers / line metadata staged in LDS by coalesced dword
// loads, and writes the recovered headers and a schedule record per group:
//   byte 0 = steps, byte 1 = 1 when no step reads a segment recovered by an
//   earlier step (single level), then (line, target) byte pairs.
// k_recover_flat: one lane per (group, 16-B chunk column) replays the record;
// single-level schedules run BATCH steps with every load in flight at once.
// ---------------------------------------------------------------------------
constexpr int kPeelDwords = 8192; // 32 KiB of LDS per peel block

struct PeelArgs {
    rfec_hdr* hdr;
    const uint64_t* present;
    const rfec_hdr* meta;
    const uint16_t* fsize;
    const uint64_t* parity_present;
    uint64_t* recovered;
    uint8_t* sched;
    uint32_t groups, capacity, gpb, rec_bytes, disjoint;
    uint32_t nlp_log2; // fused disjoint decodes: header lanes per group (line_headers)
    // dense output (rfec_recover_batch_out): recovered segment e of group g
    // (the e-th erased one in index order, e < out_per_group) goes to
    // out_hdr[g * out_per_group + e]; out_per_group == 0: in place
    rfec_hdr* out_hdr;
    uint8_t* out_index;
    uint32_t out_per_group;
    // packed erasure records (rfec_recover_packed_out): group g's record at
    // packed + g * pk_stride, slot e's at + 16 + e * pk_slot; null: the batch layout
    const uint8_t* packed;
    uint32_t pk_stride, pk_slot;
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

__device__ __forceinline__ bool has_bit(uint64_t h0, uint64_t h1, uint32_t i)
{
    return ((i < 64 ? h0 >> i : h1 >> (i - 64)) & 1ull) != 0;
}

// One peel block: groups [blk*gpb, ...), one lane per group, records staged in
// LDS.  Dense output (out_per_group = E > 0): only erased segments of rank < E
// are targets; their headers go to out_hdr, the out_index row is written.
template <int LDSD>
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
    const uint32_t E = A.out_per_group;
    const uint64_t er0 = ~have0, er1 = ~have1; // erased (rank order of the dense output)
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
            if (L > A.capacity || (E && missing_rank(~er0, ~er1, t) >= E))
                continue;
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
            if (!ok || (r4 >> 16) > L)
                continue;
            uint32_t* ht = h + t * 5;
            ht[0] = r0, ht[1] = r1, ht[2] = r2, ht[3] = r3, ht[4] = r4;
            uint32_t* gh = E ? reinterpret_cast<uint32_t*>(A.out_hdr + (size_t)g * E + missing_rank(~er0, ~er1, t))
                             : reinterpret_cast<uint32_t*>(A.hdr + (size_t)g * K + t);
            gh[0] = r0, gh[1] = r1, gh[2] = r2, gh[3] = r3, gh[4] = r4;
            rec[2 + 2 * n] = (uint8_t)l;
            rec[3 + 2 * n] = (uint8_t)t;
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
    rec[0] = (uint8_t)n;
    rec[1] = (uint8_t)single;
    A.recovered[2 * g] = rec0;
    A.recovered[2 * g + 1] = rec1;
    if (E) { // out_index: the e-th erased segment's index where it was recovered, else 0xFF
        const uint64_t km0 = K >= 64 ? ~0ull : (1ull << K) - 1ull;
        const uint64_t km1 = K <= 64 ? 0ull : (K >= 128 ? ~0ull : (1ull << (K - 64)) - 1ull);
        uint64_t e0 = er0 & km0, e1 = er1 & km1;
        for (uint32_t e = 0; e < E; ++e) {
            uint32_t v = 0xFF;
            if (e0 | e1) {
                const uint32_t i = e0 ? (uint32_t)__ffsll((long long)e0) - 1 : 64u + (uint32_t)__ffsll((long long)e1) - 1;
                if (has_bit(rec0, rec1, i))
                    v = i;
                if (e0)
                    e0 &= e0 - 1;
                else
                    e1 &= e1 - 1;
            }
            A.out_index[(size_t)g * E + e] = (uint8_t)v;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_peel_lds(PeelArgs A, rfec_kmask M)
{
    peel_block<kPeelDwords>(A, M, blockIdx.x);
}

__device__ __forceinline__ uint32_t rec_byte(const v4u& r, uint32_t b)
{
    return (r[b >> 2] >> (8 * (b & 3))) & 0xffu;
}

// Replays one group's schedule record over one chunk column: grp / par point
// at chunk j of the group's segment / parity slots, r0 = first 16 record bytes.
// Dense output (out != nullptr, the group's first out slot at chunk j): a
// recovered segment goes to out slot rank(t) (h0 / h1: the received masks),
// and a later step reads it back from there (same lane, same address, in order).
template <int MAXC, int BATCH>
__device__ __forceinline__ void replay(v4u* grp, const v4u* __restrict__ par, const uint8_t* __restrict__ rec,
                                       const v4u r0, uint32_t C, uint32_t fast_ok, const uint32_t* lplan,
                                       v4u* out, uint64_t h0, uint64_t h1)
{
    const uint32_t n = rec_byte(r0, 0);
    uint32_t s = 0;
    if (fast_ok && rec_byte(r0, 1)) {
        // single level: BATCH steps at a time, all loads in flight together
        const uint32_t nf = n < 7 ? n : 7; // steps carried in the first 16 record bytes
        for (; s < nf; s += BATCH) {
            // (unconditional loads, see k_decode_rows; an off step re-reads
            // the first step's parity chunk)
            v4u acc[BATCH], mv[BATCH][MAXC];
            uint32_t tg[BATCH], l0 = 0;
            bool on[BATCH], use[BATCH][MAXC];
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
                on[b] = s + b < nf;
                const uint32_t l = on[b] ? rec_byte(r0, 2 + 2 * (s + b)) : l0;
                l0 = l;
                tg[b] = rec_byte(r0, 3 + 2 * (s + b));
                const uint32_t ln = lplan[l];
                const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
                const v4u* pl = par + (size_t)l * C;
                acc[b] = ld16(pl);
                const ptrdiff_t to_par = pl - grp;
#pragma unroll
                for (int q = 0; q < MAXC; ++q) {
                    const uint32_t i = first + q * stride;
                    use[b][q] = on[b] && (uint32_t)q < count && i != tg[b];
                    mv[b][q] = ld16(grp + (use[b][q] ? (ptrdiff_t)i * C : to_par));
                }
            }
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
#pragma unroll
                for (int q = 0; q < MAXC; ++q)
                    acc[b] ^= use[b][q] ? mv[b][q] : v4u{0, 0, 0, 0};
                if (on[b])
                    st16(out ? out + (size_t)missing_rank(h0, h1, tg[b]) * C : grp + (size_t)tg[b] * C, acc[b]);
            }
        }
        s = nf;
    }
    // remaining / multi-level steps, one at a time in schedule order (a step
    // reads what this lane stored before: same address, same lane, in order)
    for (; s < n; ++s) {
        const uint32_t l = s < 7 ? rec_byte(r0, 2 + 2 * s) : rec[2 + 2 * s];
        const uint32_t tt = s < 7 ? rec_byte(r0, 3 + 2 * s) : rec[3 + 2 * s];
        const uint32_t ln = lplan[l];
        const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
        v4u acc = ld16(par + (size_t)l * C);
        for (uint32_t q = 0; q < count; ++q) {
            const uint32_t i = first + q * stride;
            if (i != tt)
                acc ^= (out && !has_bit(h0, h1, i)) ? out[(size_t)missing_rank(h0, h1, i) * C] : grp[(size_t)i * C];
        }
        st16(out ? out + (size_t)missing_rank(h0, h1, tt) * C : grp + (size_t)tt * C, acc);
    }
}

__device__ __forceinline__ void stage_plan(uint32_t* lplan, const rfec_kplan& P)
{
    if (threadIdx.x < P.n_lines)
        lplan[threadIdx.x] = reinterpret_cast<const uint32_t*>(P.line)[threadIdx.x];
    __syncthreads();
}

template <int MAXC, int BATCH>
__global__ __launch_bounds__(kBlock) void k_recover_flat(v4u* shards, const v4u* __restrict__ parity,
                                                         const uint8_t* __restrict__ sched, uint32_t total,
                                                         uint32_t C, FastDiv divC, uint32_t rec_bytes,
                                                         uint32_t fast_ok, rfec_kplan P, DenseOut D,
                                                         const uint64_t* __restrict__ present)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    stage_plan(lplan, P);
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
    const uint8_t* rec = sched + (size_t)g * rec_bytes;
    const v4u r0 = *reinterpret_cast<const v4u*>(rec);
    v4u* out = D.E ? D.sh + (size_t)g * D.E * C + j : nullptr;
    const uint64_t h0 = D.E ? present[2 * g] : 0ull, h1 = D.E ? present[2 * g + 1] : 0ull;
    replay<MAXC, BATCH>(shards + (size_t)g * P.k * C + j, parity + (size_t)g * P.n_lines * C + j, rec, r0, C,
                        fast_ok, lplan, out, h0, h1);
}

// ---------------------------------------------------------------------------
// Recover, plans with cascades (the sender's rows + columns: k <= 64, at most
// 8 lines of at most 4 members, every matrix plan of
// flex_fec_sender_num_packets up to k = 16): one launch, no workspace.
// Lanes (group, slot q, chunk column) in blocks of 256 (XCD-swizzled);
// dense output: slot q = the group's q-th erased segment, written to out slot
// q; in place: slot q = step q of the group's schedule.
// In each block one CHECKER lane per group the block touches runs the exact
// peel of that group: the canonical schedule over the masks (lines in plan
// order, repeated to a fixpoint: flex_fec_receiver.c:105-206 with the cascade
// of sim_receiver.c:780-804), then the header checks of its steps, two steps'
// loads in flight together (fec_data_size within the capacity, every member's
// size and the recovered size within fec_data_size: flex_fec_xor.c:88-89,
// 98-99).  A line that fails them is left out and the schedule recomputed:
// such a line fails every time it fires (same target, same members, same
// headers), so the exact peel is the mask peel without it.  The checker
// writes the recovered header records, the recovered mask and out_index, and
// hands the schedule to its block through LDS; after one barrier every lane
// replays the steps its slot depends on, recovered chunks of earlier steps
// kept in registers (a cascade costs loads, never another launch nor a round
// trip through another lane's output).
// ---------------------------------------------------------------------------

struct CascArgs {
    v4u* shards;              // in place: the erased slots are written; dense: read only
    const v4u* parity;
    uint32_t* hdr_dw;         // [G][K][5]
    const uint32_t* meta_dw;  // [G][NL][5]
    const uint16_t* fsize;    // [G][NL]
    const uint64_t* present;  // [G][2]
    const uint64_t* parity_present;
    uint64_t* recovered;      // [G][2]
    v4u* out_sh;              // dense: [G][E][C]
    uint32_t* out_hdr_dw;     // dense: [G][E][5]
    uint8_t* out_index;       // dense: [G][E]
    uint32_t E;               // dense slots per group; 0 = in place
    uint32_t groups, total, C, capacity;
    FastDiv divC, divQC;      // cd, Q * cd (Q = slots per group)
    uint8_t* ws;              // per group (ws_stride bytes): the schedule record, then Q task words
    uint32_t ws_stride, Q;
};

// A slot's task (the checker writes one per output slot of every group): the
// line and target of the step that recovers the slot's segment (dense: the
// slot's erased segment; in place: the slot-th step), bit 31 = there is one,
// bit 30 = it reads a segment recovered by an earlier step (a cascade: the
// payload lane then replays from the schedule record).
constexpr uint32_t kTaskValid = 1u << 31, kTaskCascade = 1u << 30;

// A schedule: step s = (line, target), packed so that no register array is
// indexed at run time (no scratch).  Which earlier steps a step reads follows
// from its line: its erased members other than its target were recovered
// before it.
struct CSched {
    uint32_t n;     // steps (<= 8)
    uint32_t lines; // line of step s in bits [4s, 4s + 4)
    uint64_t tg;    // target of step s in bits [8s, 8s + 8)
};

__device__ __forceinline__ uint32_t cs_line(const CSched& S, uint32_t s) { return (S.lines >> (4 * s)) & 15u; }
__device__ __forceinline__ uint32_t cs_tg(const CSched& S, uint32_t s) { return (uint32_t)(S.tg >> (8 * s)) & 0xffu; }

// Line records (first | stride << 8 | count << 16) and member masks of a plan:
// from the kernel arguments (any plan; KArgLines), from LDS copies (LdsLines),
// or arithmetic in the line index for the sender's matrix shapes (MatLines).
struct KArgLines {
    const rfec_kmask& M;
    __device__ uint32_t rec(uint32_t l) const { return reinterpret_cast<const uint32_t*>(M.plan.line)[l]; }
    __device__ uint64_t mask(uint32_t l) const { return M.mask[l][0]; }
    __device__ uint32_t nl(uint32_t n) const { return n; }
};

// The canonical schedule over the masks: a line fires with its parity
// received, exactly one member missing and one present; lines in `banned`
// never fire; dense (E > 0): only erased segments of rank < E are targets.
// MT: the mask word, uint32_t for k <= 32 (half the VALU work), else uint64_t.
template <typename MT, class Lines>
__device__ CSched cascade_schedule(const Lines& LL, uint32_t NL, MT have, uint64_t ppm, uint32_t banned, MT erased,
                                   uint32_t E)
{
    CSched S = {0, 0, 0};
    bool progress = true;
    while (progress) {
        progress = false;
        for (uint32_t l = 0; l < NL; ++l) { // uniform: the masks stay scalar kernel-argument loads (or constants)
            const MT m = (MT)LL.mask(l);
            const MT x = m & ~have;
            if (!((ppm >> l) & 1ull) || ((banned >> l) & 1u) || __popcll((uint64_t)x) != 1 || (m & have) == 0)
                continue;
            const uint32_t t = (uint32_t)__ffsll((long long)x) - 1;
            if (E && (uint32_t)__popcll((uint64_t)(erased & ((MT(1) << t) - MT(1)))) >= E)
                continue;
            S.lines |= l << (4 * S.n);
            S.tg |= (uint64_t)t << (8 * S.n);
            ++S.n;
            have |= MT(1) << t;
            progress = true;
        }
    }
    return S;
}

// the record of erased segment i's output: the dense slot of its rank, or its own slot in place
__device__ __forceinline__ uint32_t cs_slot(uint32_t E, uint64_t erased, uint32_t i)
{
    return E ? (uint32_t)__popcll(erased & ((1ull << i) - 1ull)) : i;
}

// The serial exact peel of group g (rare path: a header check failed): its
// header records, recovered mask and out_index written; returns the schedule.
// A step's record goes straight to its output (dense: out_hdr[g][rank], in
// place: hdr[g][t]); a later step of a cascade reads it back from there (same
// lane, same address, in order).  A line that fails its checks is left out and
// the schedule recomputed -- it would fail every time it fires (same target,
// same members, same headers), so the exact peel is the mask peel without it.
__device__ CSched cascade_check(const CascArgs& A, const rfec_kmask& M, uint32_t g)
{
    const rfec_kplan& P = M.plan;
    const uint32_t* lines = reinterpret_cast<const uint32_t*>(P.line);
    const uint32_t K = P.k, NL = P.n_lines;
    const uint64_t kmask = K >= 64 ? ~0ull : (1ull << K) - 1ull;
    const uint64_t have = A.present[2 * g] & kmask;
    const uint64_t erased = ~have & kmask;
    const uint64_t ppm = A.parity_present[g];
    const uint32_t* gh = A.hdr_dw + (size_t)g * K * 5;
    const uint32_t* gm = A.meta_dw + (size_t)g * NL * 5;
    const uint16_t* gf = A.fsize + (size_t)g * NL;
    uint32_t* const ob = A.E ? A.out_hdr_dw + (size_t)g * A.E * 5 : A.hdr_dw + (size_t)g * K * 5;
    uint32_t banned = 0;
    CSched S;
#pragma unroll 1
    for (uint32_t attempt = 0; attempt <= NL; ++attempt) {
        S = cascade_schedule<uint64_t>(KArgLines{M}, NL, have, ppm, banned, erased, A.E);
        int bad = -1;
#pragma unroll 1
        for (uint32_t s = 0; s < S.n; ++s) {
            const uint32_t l = cs_line(S, s), t = cs_tg(S, s), ln = lines[l];
            const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
            const uint32_t L = gf[l];
            uint32_t rec[5], mem[4][5];
#pragma unroll
            for (int d = 0; d < 5; ++d)
                rec[d] = gm[l * 5 + d];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t i = first + u * stride;
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    mem[u][d] = 0;
                if ((uint32_t)u < count && i != t) {
                    const uint32_t* r = ((erased >> i) & 1ull) ? ob + cs_slot(A.E, erased, i) * 5 : gh + i * 5;
#pragma unroll
                    for (int d = 0; d < 5; ++d)
                        mem[u][d] = r[d];
                }
            }
            bool ok = L <= A.capacity;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    rec[d] ^= mem[u][d];
                ok = ok && (mem[u][4] >> 16) <= L;
            }
            if (!ok || (rec[4] >> 16) > L) {
                bad = (int)s;
                break;
            }
            uint32_t* oh = ob + cs_slot(A.E, erased, t) * 5;
#pragma unroll
            for (int d = 0; d < 5; ++d)
                oh[d] = rec[d];
        }
        if (bad < 0)
            break;
        banned |= 1u << cs_line(S, (uint32_t)bad);
    }
    return S;
}

// Replays the steps in `need` (the lane's step ss and the steps it reads) over
// one chunk column; returns the result of step ss.  A step of a cascade (some
// member recovered by an earlier step) reads that member back from the slot
// where the earlier step stored it -- the dense output slot of its rank, or its
// own slot in place -- which this lane writes first (the slot's owner lane
// writes the same bytes; a lane's later load of an address it stored is
// ordered behind the store).
// Line records and masks for the replay: staged in LDS (any plan), or
// arithmetic in the line index (the sender's matrix shapes, MatLines below).
struct LdsLines {
    const uint32_t* lplan;
    const uint64_t* lmask;
    __device__ uint32_t rec(uint32_t l) const { return lplan[l]; }
    __device__ uint64_t mask(uint32_t l) const { return lmask[l]; }
};

template <class Lines>
__device__ __forceinline__ v4u cascade_replay(const CSched& S, uint32_t need, uint32_t ss, uint64_t erased,
                                              const v4u* grp, const v4u* par, v4u* slot0, uint32_t E, uint32_t C,
                                              const Lines& LL)
{
    v4u res = {0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t s = 0; s < 8; ++s) {
        if (!((need >> s) & 1u))
            continue;
        const uint32_t l = cs_line(S, s), t = cs_tg(S, s), ln = LL.rec(l);
        const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
        v4u acc = ld16(par + (size_t)l * C);
        v4u mv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = first + u * stride;
            mv[u] = v4u{0, 0, 0, 0};
            if ((uint32_t)u < count && i != t)
                mv[u] = ld16(((erased >> i) & 1ull) ? slot0 + (size_t)cs_slot(E, erased, i) * C : grp + (size_t)i * C);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            acc ^= mv[u];
        if (s == ss) {
            res = acc;
            break;
        }
        st16(slot0 + (size_t)cs_slot(E, erased, t) * C, acc);
    }
    return res;
}

// The checker kernel, eight lanes per group (step s = lane & 7): every lane
// derives the group's mask schedule (one instruction stream for the wave's 8
// groups), lane s loads and checks step s -- fec_data_size, its meta record
// and its present members' records in one round of loads -- and forms its
// recovered header record; a member recovered by an earlier step comes from
// that step's lane (shuffles, in step order, only in waves holding a
// cascade).  When every step passes, lane s writes its record and lane 0 the
// mask, out_index and the group's schedule record (16 B: lines, targets, n);
// when one fails, lane 0 runs the serial exact peel for the group instead.
__device__ __forceinline__ v4u cs_pack(const CSched& S) { return v4u{S.lines, (uint32_t)S.tg, (uint32_t)(S.tg >> 32), S.n}; }

__device__ __forceinline__ CSched cs_unpack(const v4u r)
{
    CSched S;
    S.lines = r[0];
    S.tg = (uint64_t)r[1] | ((uint64_t)r[2] << 32);
    S.n = r[3] & 15u;
    return S;
}

// The checker, LPG lanes per group (step s = lane % LPG; the group's lanes
// [base, base + LPG) of one wave, every lane of the wave taking part): writes
// the group's header records, recovered mask and out_index, returns its
// schedule packed.  A group of more than LPG steps (more than LPG erasures
// recovered) takes the serial exact peel.  Dead lanes (live false) join the
// shuffles only.
template <typename MT, int LPG, bool kTasks, class Lines>
__device__ v4u cascade_check_lanes(const CascArgs& A, const rfec_kmask& M, const Lines& LL, uint32_t g, bool live,
                                   uint32_t s, uint32_t base)
{
    const uint32_t gg = live ? g : 0u;
    const rfec_kplan& P = M.plan;
    const uint32_t K = P.k, NL = P.n_lines;
    const MT kmask = K >= 8 * sizeof(MT) ? ~MT(0) : (MT(1) << K) - MT(1);
    const MT have = (MT)A.present[2 * gg] & kmask;
    const MT erased = ~have & kmask;
    const uint64_t ppm = A.parity_present[gg];
    const CSched S = cascade_schedule<MT>(LL, LL.nl(NL), have, ppm, 0u, erased, A.E);
    const bool on = live && s < S.n;
    const uint32_t l = on ? cs_line(S, s) : 0u, t = cs_tg(S, s);
    const uint32_t ln = LL.rec(l);
    const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
    const uint32_t* gh = A.hdr_dw + (size_t)gg * K * 5;
    const uint32_t* gm = A.meta_dw + (size_t)gg * NL * 5;
    uint32_t L = 0, rec[5] = {0, 0, 0, 0, 0}, mem[4][5];
    if (on) {
        L = A.fsize[(size_t)gg * NL + l];
#pragma unroll
        for (int d = 0; d < 5; ++d)
            rec[d] = gm[l * 5 + d];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t i = first + u * stride;
#pragma unroll
        for (int d = 0; d < 5; ++d)
            mem[u][d] = 0;
        if (on && (uint32_t)u < count && i != t && ((erased >> i) & MT(1)) == 0) {
#pragma unroll
            for (int d = 0; d < 5; ++d)
                mem[u][d] = gh[i * 5 + d];
        }
    }
    bool ok = L <= A.capacity;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        ok = ok && (mem[u][4] >> 16) <= L;
#pragma unroll
        for (int d = 0; d < 5; ++d)
            rec[d] ^= mem[u][d];
    }
    // cascades: the members recovered by earlier steps, folded in step order (step r's record is
    // final before round r); only waves that hold one take the shuffles
    const MT depm = on ? ((MT)LL.mask(l) & erased & ~(MT(1) << t)) : MT(0);
    if (__ballot(depm != 0)) {
#pragma unroll
        for (int r = 0; r < LPG - 1; ++r) {
            uint32_t w[5];
#pragma unroll
            for (int d = 0; d < 5; ++d)
                w[d] = (uint32_t)__shfl((int)rec[d], (int)(base + r), kWave);
            if ((uint32_t)r < S.n && ((depm >> cs_tg(S, r)) & MT(1))) {
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    rec[d] ^= w[d];
                ok = ok && (w[4] >> 16) <= L;
            }
        }
    }
    ok = !on || (ok && (rec[4] >> 16) <= L);
    uint32_t all = ok && S.n <= (uint32_t)LPG ? 1u : 0u; // every step of the group taken and passed?
#pragma unroll
    for (int m = 1; m < LPG; m <<= 1)
        all &= (uint32_t)__shfl_xor((int)all, m, kWave);
    CSched X = S;
    if (!live)
        return v4u{0, 0, 0, 0};
    if (!all) { // rare: a rejection -- the serial exact peel (it writes the header records)
        if (s != 0)
            return v4u{0, 0, 0, 0};
        X = cascade_check(A, M, g);
    } else if (on) { // the recovered header record (flex_fec_xor.c:64-85)
        uint32_t* oh = (A.E ? A.out_hdr_dw + (size_t)g * A.E * 5 : A.hdr_dw + (size_t)g * K * 5) +
                       cs_slot(A.E, (uint64_t)erased, t) * 5;
#pragma unroll
        for (int d = 0; d < 5; ++d)
            oh[d] = rec[d];
    }
    if (s == 0) {
        uint64_t rm = 0;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
            if ((uint32_t)s2 < X.n)
                rm |= 1ull << cs_tg(X, s2);
        A.recovered[2 * g] = rm;
        A.recovered[2 * g + 1] = 0;
        // the slots' tasks (and out_index: the e-th erased segment's index where it was recovered)
        uint32_t* task = kTasks ? reinterpret_cast<uint32_t*>(A.ws + (size_t)g * A.ws_stride + 16) : nullptr;
        uint64_t m = (uint64_t)erased;
        for (uint32_t q = 0; q < A.Q; ++q) {
            uint32_t ss = 8;
            if (A.E) {
                const uint32_t i = m ? (uint32_t)__ffsll((long long)m) - 1 : 0xFFu;
                m &= m - 1;
#pragma unroll
                for (int s2 = 0; s2 < 8; ++s2)
                    if ((uint32_t)s2 < X.n && cs_tg(X, s2) == i)
                        ss = s2;
                A.out_index[(size_t)g * A.E + q] = (uint8_t)(ss < 8 ? i : 0xFFu);
            } else if (q < X.n) {
                ss = q;
            }
            uint32_t w = 0;
            if (ss < 8) {
                const uint32_t tl = cs_line(X, ss), tt = cs_tg(X, ss);
                const bool casc = (LL.mask(tl) & (uint64_t)erased & ~(1ull << tt)) != 0;
                w = kTaskValid | (casc ? kTaskCascade : 0u) | tl | (tt << 8);
            }
            if (kTasks)
                task[q] = w;
        }
    }
    return cs_pack(X);
}

// The checker kernel: LPG = 4 lanes per group (16 groups per wave: the
// schedule's instruction stream is shared by a wave's groups, so fewer lanes
// per group means fewer waves; one round of loads covers up to 4 steps, i.e.
// up to 4 erasures recovered).  The group's 16-byte schedule record goes to
// the workspace for the payload kernel.
constexpr int kCheckLanes = 4;

template <typename MT>
__global__ __launch_bounds__(kBlock) void k_cascade_check(CascArgs A, rfec_kmask M)
{
    const uint32_t gt = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = gt / kCheckLanes, s = gt % kCheckLanes;
    const bool live = g < A.groups;
    const v4u r = cascade_check_lanes<MT, kCheckLanes, true>(A, M, KArgLines{M}, live ? g : 0u, live, s,
                                                       (threadIdx.x & (kWave - 1)) & ~(uint32_t)(kCheckLanes - 1));
    if (live && s == 0)
        *reinterpret_cast<v4u*>(A.ws + (size_t)g * A.ws_stride) = r;
}

// The payload kernel: lane (group, slot, chunk column) reads its slot's task
// word and, for a single-level step (the common case), loads the line's
// parity and other members, all in flight, and stores the recovered chunk --
// no mask work, one dependent load before the payload loads.  A cascade step
// replays the steps it reads from the group's schedule record.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_decode_cascade(CascArgs A, rfec_kmask M)
{
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    __shared__ uint64_t lmask[8];
    const rfec_kplan& P = M.plan;
    if (threadIdx.x < 8)
        lmask[threadIdx.x] = threadIdx.x < P.n_lines ? M.mask[threadIdx.x][0] : 0ull;
    stage_plan(lplan, P); // (ends in a barrier)
    // XCD-swizzled (the grid is a multiple of 8 blocks): a group's lanes share one L2
    const uint32_t t = xcd_block(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    if (t >= A.total)
        return;
    const uint32_t g = fdiv(t, A.divQC);
    const uint32_t rem = t - g * A.divQC.d;
    const uint32_t q = fdiv(rem, A.divC);
    const uint32_t j = rem - q * A.divC.d;
    const uint32_t K = P.k, NL = P.n_lines, C = A.C;
    const uint8_t* wg = A.ws + (size_t)g * A.ws_stride;
    const uint32_t task = reinterpret_cast<const uint32_t*>(wg + 16)[q];
    if (!(task & kTaskValid))
        return;
    const uint32_t l = task & 15u, tgt = (task >> 8) & 0xffu;
    const v4u* grp = A.shards + (size_t)g * K * C + j;
    const v4u* par = A.parity + (size_t)g * NL * C + j;
    v4u* slot0 = A.E ? A.out_sh + (size_t)g * A.E * C + j : A.shards + (size_t)g * K * C + j;
    v4u* dst = slot0 + (size_t)(A.E ? q : tgt) * C;
    if (!(task & kTaskCascade)) { // single level: every other member arrived
        const uint32_t ln = lplan[l];
        const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
        v4u acc = ld16(par + (size_t)l * C);
        v4u mv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = first + u * stride;
            mv[u] = v4u{0, 0, 0, 0};
            if ((uint32_t)u < count && i != tgt)
                mv[u] = ld16(grp + (size_t)i * C);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            acc ^= mv[u];
        st16(dst, acc);
        return;
    }
    // a cascade: the steps it reads, transitively (a step's erased members other than its target were
    // recovered by earlier steps), replayed from the schedule record
    const uint64_t kmask = K >= 64 ? ~0ull : (1ull << K) - 1ull;
    const uint64_t erased = ~A.present[2 * g] & kmask;
    const CSched S = cs_unpack(*reinterpret_cast<const v4u*>(wg));
    uint32_t ss = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s)
        if ((uint32_t)s < S.n && cs_tg(S, s) == tgt)
            ss = s;
    uint32_t need = 1u << ss;
#pragma unroll 1
    for (int s = (int)ss; s >= 0; --s) {
        if (!((need >> s) & 1u))
            continue;
        const uint64_t dm = lmask[cs_line(S, s)] & erased & ~(1ull << cs_tg(S, s));
        for (int s2 = 0; s2 < s; ++s2)
            if ((dm >> cs_tg(S, s2)) & 1ull)
                need |= 1u << s2;
    }
    st16(dst, cascade_replay(S, need, ss, erased, grp, par, slot0, A.E, C, LdsLines{lplan, lmask}));
}

// A dense payload lane whose target no line recovers at once (a cascade):
// the group's mask schedule (cascade_schedule without the header checks),
// the steps the target's step reads, transitively, replayed in registers.
// (SL: the schedule's masks -- kernel arguments or constants; LL: the replay's)
template <typename MT, class SLines, class Lines>
__device__ __forceinline__ void cascade_dense_tail(const CascArgs& A, const SLines& SL, uint32_t NL, uint64_t have,
                                                   uint64_t erased, uint64_t ppm, uint32_t tgt, const v4u* grp,
                                                   const v4u* par, v4u* slot0, v4u* dst, const Lines& LL)
{
    const CSched S = cascade_schedule<MT>(SL, NL, (MT)have, ppm, 0u, (MT)erased, A.E);
    uint32_t ss = 8;
#pragma unroll
    for (int s = 0; s < 8; ++s)
        if ((uint32_t)s < S.n && cs_tg(S, s) == tgt)
            ss = s;
    if (ss == 8)
        return; // not recoverable
    uint32_t need = 1u << ss;
#pragma unroll 1
    for (int s = (int)ss; s >= 0; --s) {
        if (!((need >> s) & 1u))
            continue;
        const uint64_t dm = LL.mask(cs_line(S, s)) & erased & ~(1ull << cs_tg(S, s));
        for (int s2 = 0; s2 < s; ++s2)
            if ((dm >> cs_tg(S, s2)) & 1ull)
                need |= 1u << s2;
    }
    st16(dst, cascade_replay(S, need, ss, erased, grp, par, slot0, A.E, A.C, LL));
}

// Dense output, one launch: rounds of 8 checker blocks spread over the grid
// (header_block_xcd; they write the headers, recovered masks and out_index, no
// task words) between the payload lanes' rounds, which need nothing from them: lane
// (group, slot q, chunk column) recovers the group's q-th erased segment
// through a line that fires at once for it (parity received, every other
// member present) or, when none does, replays the group's mask schedule
// (cascade_schedule without the header checks).  Any line that recovers a
// segment gives its bytes, so the data equal the exact peel's wherever it
// recovers; a segment it leaves unrecovered (a rejected line) may still be
// written, its out_index 0xFF.  The checker's latency-bound work overlaps the
// payload traffic instead of preceding it: c3 full 128.3-128.8 us vs 131.5-131.8
// us for check + k_decode_cascade (A/Bs on one box; the checker's blocks all at
// the head of the grid: 134.6 us; spread but not XCD-aligned with the payload:
// 129.4-130.3 us; the line search through LDS copies of the masks instead of
// the kernel arguments: 131 us; checker rounds 3 or 8 rounds further ahead: no
// change).  The payload lanes wait on the masks where k_decode_cascade waited
// on its task word (L2).

template <typename MT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_decode_cascade_dense(
    CascArgs A, rfec_kmask M, uint32_t n_hr, uint32_t every, uint32_t npay8)
{
    uint32_t hb = 0, pb = 0;
    if (header_block_xcd(n_hr, every, npay8, &hb, &pb)) { // (checker blocks XCD-aligned with the payload sweep)
        const uint32_t gt = hb * kBlock + threadIdx.x;
        const uint32_t g = gt / kCheckLanes, s = gt % kCheckLanes;
        const bool live = g < A.groups;
        cascade_check_lanes<MT, kCheckLanes, false>(A, M, KArgLines{M}, live ? g : 0u, live, s,
                                                    (threadIdx.x & (kWave - 1)) & ~(uint32_t)(kCheckLanes - 1));
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    __shared__ uint64_t lmask[8];
    const rfec_kplan& P = M.plan;
    if (threadIdx.x < 8)
        lmask[threadIdx.x] = threadIdx.x < P.n_lines ? M.mask[threadIdx.x][0] : 0ull;
    stage_plan(lplan, P); // (ends in a barrier)
    const uint32_t t = pb * kBlock + threadIdx.x; // (XCD-swizzled: a group's lanes share one L2)
    if (t >= A.total)
        return;
    const uint32_t g = fdiv(t, A.divQC);
    const uint32_t rem = t - g * A.divQC.d;
    const uint32_t q = fdiv(rem, A.divC);
    const uint32_t j = rem - q * A.divC.d;
    const uint32_t K = P.k, NL = P.n_lines, C = A.C;
    // (MT: 32-bit masks for k <= 32, the low words of present / parity_present)
    constexpr uint32_t MB = 8 * sizeof(MT);
    const MT kmaskM = K >= MB ? ~(MT)0 : (((MT)1 << K) - 1);
    const MT hv = (MT)A.present[2 * g] & kmaskM, er = ~hv & kmaskM;
    const uint64_t have = hv, erased = er, ppm = (uint32_t)A.parity_present[g]; // (NL <= 8 here)
    MT e = er; // slot q: the q-th erased segment
    for (uint32_t i = 0; i < q; ++i)
        e &= e - 1;
    if (!e)
        return;
    const uint32_t tgt = MB == 32 ? (uint32_t)__ffs((int)e) - 1 : (uint32_t)__ffsll((long long)e) - 1;
    // the first line that fires at once for it (masks and line records from the
    // kernel arguments: scalar loads, no LDS round trips before the payload loads)
    uint32_t l = 0xFFu, ln = 0;
    {
        const MT tb = (MT)1 << tgt;
        const uint32_t pp = (uint32_t)ppm;
#pragma unroll
        for (int x = 7; x >= 0; --x) {
            const MT lm = (MT)M.mask[x][0];
            if ((uint32_t)x < NL && ((pp >> x) & 1u) && (lm & er) == tb && (lm & hv)) {
                l = (uint32_t)x;
                ln = reinterpret_cast<const uint32_t*>(P.line)[x];
            }
        }
    }
    const v4u* grp = A.shards + (size_t)g * K * C + j;
    const v4u* par = A.parity + (size_t)g * NL * C + j;
    v4u* slot0 = A.out_sh + (size_t)g * A.E * C + j;
    v4u* dst = slot0 + (size_t)q * C;
    if (l != 0xFFu) { // single level
        const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
        v4u acc = ld16(par + (size_t)l * C);
        // members through a descriptor over the first active lane's group (wave_rsrc: no per-load
        // branch, all four loads in flight; with `if (used) load` hipcc waited on each load in turn)
        const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g); // lanes' groups ascend
        const __amdgpu_buffer_rsrc_t rs = wave_rsrc(A.shards + (size_t)gb * K * C);
        const uint32_t grp0 = ((g - gb) * K * C + j) * 16u;
        v4u mv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = first + u * stride;
            mv[u] = bld16(rs, (uint32_t)u < count && i != tgt ? grp0 + i * C * 16u : kNoLoad);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            acc ^= mv[u];
        st16(dst, acc);
        return;
    }
    cascade_dense_tail<MT>(A, KArgLines{M}, NL, have, erased, ppm, tgt, grp, par, slot0, dst, LdsLines{lplan, lmask});
}

// The sender's full matrix plans (rows of COL consecutive segments, then the
// columns, flex_fec_sender.c:166-233), K = 6..16 as
// flex_fec_sender_num_packets picks them (COL 3 for K <= 9, else 4): the dense
// cascade decode with the plan folded into the code.  A payload lane's target
// lies in exactly one row and one column, so the first line that fires at
// once for it (plan order: rows first) is its row, else its column -- two
// mask tests on masks that are shifts of constants, instead of the generic
// kernel's search over eight kernel-argument masks and line records; the
// q-th erased segment is found by clearing q low bits without a run-time
// loop for q < 4.  Cascades (no line fires at once) replay the mask schedule
// as the generic kernel does, with the line records computed from the index.
template <int K, int COL>
struct MatLines {
    using Sh = MatrixShape<K, COL>;
    static constexpr int NR = Sh::n_rows();
    static constexpr uint32_t KM = (1u << K) - 1u, ROW = (1u << COL) - 1u;
    static constexpr uint32_t col0()
    {
        uint32_t m = 0;
        for (int r = 0; r < Sh::R; ++r)
            m |= 1u << (r * COL);
        return m;
    }
    static constexpr uint32_t COL0 = col0();
    // line l: first | stride << 8 | count << 16 (rows l < NR, then column l - NR)
    __device__ uint32_t rec(uint32_t l) const
    {
        const bool row = l < (uint32_t)NR;
        const uint32_t c = l - NR;
        const uint32_t first = row ? l * COL : c, stride = row ? 1u : (uint32_t)COL;
        const uint32_t count = row ? min((uint32_t)COL, K - l * COL) : (K - c + COL - 1) / COL;
        return first | stride << 8 | count << 16;
    }
    __device__ uint64_t mask(uint32_t l) const
    {
        return l < (uint32_t)NR ? (ROW << (l * COL)) & KM : (COL0 << (l - NR)) & KM;
    }
    __device__ uint32_t nl(uint32_t) const { return NR + COL; }
};

template <int K, int COL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_decode_matrix_dense(
    CascArgs A, rfec_kmask M, uint32_t n_hr, uint32_t every, uint32_t npay8)
{
    using LL = MatLines<K, COL>;
    constexpr int NR = LL::NR, NL = NR + COL, R = MatrixShape<K, COL>::R, MX = COL > R ? COL : R;
    static_assert(K >= 2 * COL && K <= 16 && NL <= 8 && MX <= 4, "the cascade kernels' shapes");
    uint32_t hb = 0, pb = 0;
    if (header_block_xcd(n_hr, every, npay8, &hb, &pb)) { // the checker blocks, as the generic kernel's
        const uint32_t gt = hb * kBlock + threadIdx.x;
        const uint32_t g = gt / kCheckLanes, s = gt % kCheckLanes;
        const bool live = g < A.groups;
        cascade_check_lanes<uint32_t, kCheckLanes, false>(A, M, LL{}, live ? g : 0u, live, s,
                                                          (threadIdx.x & (kWave - 1)) & ~(uint32_t)(kCheckLanes - 1));
        return;
    }
    const uint32_t t = pb * kBlock + threadIdx.x; // (XCD-swizzled: a group's lanes share one L2)
    if (t >= A.total)
        return;
    const uint32_t g = fdiv(t, A.divQC);
    const uint32_t rem = t - g * A.divQC.d;
    const uint32_t q = fdiv(rem, A.divC);
    const uint32_t j = rem - q * A.divC.d;
    const uint32_t C = A.C;
    const uint32_t hv = (uint32_t)A.present[2 * g] & LL::KM, er = ~hv & LL::KM;
    const uint32_t pp = (uint32_t)A.parity_present[g];
    uint32_t e = er; // slot q: the q-th erased segment
#pragma unroll
    for (int i = 0; i < 3; ++i)
        e = (uint32_t)i < q ? e & (e - 1u) : e;
    for (uint32_t i = 3; i < q; ++i)
        e &= e - 1u;
    if (!e)
        return;
    const uint32_t tgt = (uint32_t)__ffs((int)e) - 1, tb = 1u << tgt;
    const uint32_t r = tgt / COL, c = tgt - r * COL;
    const uint32_t rm = (LL::ROW << (r * COL)) & LL::KM, cm = (LL::COL0 << c) & LL::KM;
    const bool row_fires = r < (uint32_t)NR && ((pp >> r) & 1u) && (rm & er) == tb && (rm & hv);
    const bool col_fires = ((pp >> (NR + c)) & 1u) && (cm & er) == tb && (cm & hv);
    const v4u* grp = A.shards + (size_t)g * K * C + j;
    const v4u* par = A.parity + (size_t)g * NL * C + j;
    v4u* slot0 = A.out_sh + (size_t)g * A.E * C + j;
    v4u* dst = slot0 + (size_t)q * C;
    if (row_fires || col_fires) { // single level
        const uint32_t l = row_fires ? r : NR + c;
        const uint32_t first = row_fires ? r * COL : c, stride = row_fires ? 1u : (uint32_t)COL;
        const uint32_t count = row_fires ? min((uint32_t)COL, K - r * COL) : (K - c + COL - 1) / COL;
        v4u acc = ld16(par + (size_t)l * C);
        // members through a descriptor over the first active lane's group (see k_decode_cascade_dense)
        const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g); // lanes' groups ascend
        const __amdgpu_buffer_rsrc_t rs = wave_rsrc(A.shards + (size_t)gb * K * C);
        const uint32_t grp0 = ((g - gb) * K * C + j) * 16u;
        v4u mv[MX];
#pragma unroll
        for (int u = 0; u < MX; ++u) {
            const uint32_t i = first + u * stride;
            mv[u] = bld16(rs, (uint32_t)u < count && i != tgt ? grp0 + i * C * 16u : kNoLoad);
        }
#pragma unroll
        for (int u = 0; u < MX; ++u)
            acc ^= mv[u];
        st16(dst, acc);
        return;
    }
    cascade_dense_tail<uint32_t>(A, LL{}, NL, hv, er, pp, tgt, grp, par, slot0, dst, LL{});
}

// ---------------------------------------------------------------------------
// Recover, fused form for plans whose lines are pairwise disjoint (the row
// layer alone, strip mode).  No recovery there can complete another line, so
// which lines fire follows from the received masks alone and no schedule has
// to travel between kernels.  Header blocks spread over the grid do the
// peel's header work (size checks, recovered headers, the recovered mask);
// the payload lanes XOR each line with exactly one missing member and its
// parity received into that member's slot (or its dense output slot).  A line
// the header checks reject is still written, into an erased slot whose
// recovered bit stays clear (rfec_recover_batch documents such slots as
// unspecified).
// ---------------------------------------------------------------------------

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

// Header lanes of the packed decode (rfec_recover_packed_out), one per (group,
// output slot e): 2^nlp_log2 >= E consecutive lanes per group.  Slot e's
// record holds the fec_meta, fec_data_size and the other members' records of
// the row of the group's e-th erased segment, so a lane's header bytes are one
// contiguous run after the group's two masks (line_headers reads them from
// three arrays: the meta and member runs in sectors shared with the lines that
// do not fire).  The checks and the recovered record are line_headers'.
template <int COL>
__device__ void packed_headers(const PeelArgs& A, uint32_t blk, uint32_t KK, uint32_t CC)
{
    const uint32_t ep = 1u << A.nlp_log2;
    const uint32_t hl = blk * kBlock + threadIdx.x;
    const uint32_t g = hl >> A.nlp_log2, e = hl & (ep - 1);
    uint64_t rec = 0;
    if (g < A.groups && e < A.out_per_group) {
        const uint8_t* pg = A.packed + (size_t)g * A.pk_stride;
        const uint64_t h = reinterpret_cast<const uint64_t*>(pg)[0], pp = reinterpret_cast<const uint64_t*>(pg)[1];
        uint64_t m = ~h & (KK == 64 ? ~0ull : (1ull << KK) - 1ull);
        for (uint32_t u = 0; u < e; ++u) // the e-th erased segment
            m &= m - 1ull;
        uint32_t v = 0xFF;
        if (m) {
            const uint32_t tgt = (uint32_t)__ffsll((long long)m) - 1, r = tgt / CC;
            const uint32_t R = (KK + CC - 1) / CC, cnt = r + 1 < R ? CC : KK - (R - 1) * CC;
            const uint64_t rm = ((1ull << cnt) - 1ull) << (r * CC);
            if (__popcll(rm & ~h) == 1 && (rm & h) && ((pp >> r) & 1ull)) {
                const uint32_t* sr = reinterpret_cast<const uint32_t*>(pg + 16 + (size_t)e * A.pk_slot);
                uint32_t r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3], r4 = sr[4];
                const uint32_t L = sr[5] & 0xFFFFu;
                uint32_t w[COL - 1][5];
#pragma unroll
                for (int q = 0; q < COL - 1; ++q) // one round of loads, as line_headers
#pragma unroll
                    for (int d = 0; d < 5; ++d)
                        w[q][d] = (uint32_t)q + 1 < cnt ? sr[6 + 5 * q + d] : 0u;
                bool ok = L <= A.capacity;
#pragma unroll
                for (int q = 0; q < COL - 1; ++q) {
                    r0 ^= w[q][0];
                    r1 ^= w[q][1];
                    r2 ^= w[q][2];
                    r3 ^= w[q][3];
                    r4 ^= w[q][4];
                    ok = ok && (w[q][4] >> 16) <= L;
                }
                if (ok && (r4 >> 16) <= L) {
                    uint32_t* ht = reinterpret_cast<uint32_t*>(A.out_hdr + (size_t)g * A.out_per_group + e);
                    ht[0] = r0, ht[1] = r1, ht[2] = r2, ht[3] = r3, ht[4] = r4;
                    v = tgt;
                    rec = 1ull << tgt;
                }
            }
        }
        A.out_index[(size_t)g * A.out_per_group + e] = (uint8_t)v;
    }
    for (uint32_t sh = 1; sh < ep; sh <<= 1)
        rec |= __shfl_xor(rec, sh);
    if (g < A.groups && e == 0) {
        A.recovered[2 * g] = rec;
        A.recovered[2 * g + 1] = 0;
    }
}

// Header blocks of the fused decodes: every (every + 1)-th block until they
// run out (every == 0: the first n_hdr of the grid), spread over the grid so
// their latency-bound chains overlap the payload stream (cold: k = 32 / 256 B
// 41.6 vs 46.9 us at the head; k = 10 / 1,200 B 139.4-141.1 vs 144.0-144.4
// us).  Returns true with *hb = header block index, else false with *pb =
// payload block index.
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


// Flat form, slots under 64 chunks (k = 32 / 256 B): one lane per (group,
// chunk column) XORs every fired line of its group, two lines' loads in
// flight together, in place or into the dense output.
template <int MAXC>
__global__ __launch_bounds__(kBlock) void k_decode_disjoint(v4u* shards, const v4u* __restrict__ parity,
                                                            uint32_t total, uint32_t C, FastDiv divC,
                                                            uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                            rfec_kmask M, DenseOut D)
{
    uint32_t hb, pb;
    if (header_block(n_hdr_blocks, hdr_every, &hb, &pb)) {
        line_headers(A, M, hb);
        return;
    }
    __shared__ uint32_t lplan[RFEC_MAX_LINES];
    const rfec_kplan& P = M.plan;
    stage_plan(lplan, P);
    const uint32_t t = pb * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divC);
    const uint32_t j = t - g * divC.d; // chunk column (divC.d = chunks of work per slot)
    const uint64_t h0 = A.present[2 * g], h1 = A.present[2 * g + 1];
    uint64_t fire = A.parity_present[g];
    v4u* grp = shards + (size_t)g * P.k * C + j;
    v4u* out = D.E ? D.sh + (size_t)g * D.E * C + j : nullptr;
    // descriptors over the wave's first group (its lanes span a few groups)
    const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
    const __amdgpu_buffer_rsrc_t rs = wave_rsrc(shards + (size_t)gb * P.k * C);
    const __amdgpu_buffer_rsrc_t rp = wave_rsrc(parity + (size_t)gb * P.n_lines * C);
    const uint32_t grp0 = ((g - gb) * P.k * C + j) * 16u, par0 = ((g - gb) * P.n_lines * C + j) * 16u;
    {   // lines with their parity received and exactly one member missing
        // (uniform loop: the line masks stay scalar kernel-argument loads)
        uint64_t f = 0;
        for (uint32_t l = 0; l < P.n_lines; ++l) {
            const uint64_t x0 = M.mask[l][0] & ~h0, x1 = M.mask[l][1] & ~h1;
            if (__popcll(x0) + __popcll(x1) == 1)
                f |= 1ull << l;
        }
        fire &= f;
    }
    while (fire) {
        // two fired lines per round, every load of both in flight together
        // (predicated loads through the wave's descriptors, see wave_rsrc)
        v4u acc[2], mv[2][MAXC];
        uint32_t tg[2];
        bool on[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            on[b] = fire != 0;
            const uint32_t l = on[b] ? (uint32_t)__ffsll((long long)fire) - 1 : 0;
            fire &= fire - 1;
            const uint32_t ln = lplan[l];
            const uint32_t first = ln & 0xff, stride = (ln >> 8) & 0xff, count = (ln >> 16) & 0xff;
            acc[b] = bld16(rp, on[b] ? par0 + l * C * 16u : kNoLoad);
            tg[b] = first;
#pragma unroll
            for (int q = 0; q < MAXC; ++q) {
                const uint32_t i = first + q * stride;
                const bool in = on[b] && (uint32_t)q < count, have = has_bit(h0, h1, i);
                tg[b] = in && !have ? i : tg[b];
                mv[b][q] = bld16(rs, in && have ? grp0 + i * C * 16u : kNoLoad);
            }
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int q = 0; q < MAXC; ++q)
                acc[b] ^= mv[b][q];
            if (on[b]) {
                if (!D.E) {
                    st16(grp + (size_t)tg[b] * C, acc[b]);
                } else {
                    const uint32_t e = missing_rank(h0, h1, tg[b]);
                    if (e < D.E)
                        st16(out + (size_t)e * C, acc[b]);
                }
            }
        }
    }
}

// Fused disjoint-plan decode, output-mapped (slots of >= 64 chunks): one lane
// per (group, line, chunk column).  A lane whose line does not fire (parity
// missing, or not exactly one member missing) exits; the others load the
// parity chunk and the line's present members' chunks, all in flight, and
// store one chunk of the missing member.  A wave's loads and its store each
// cover 1 KiB of one slot.  142.7 us vs 157.8 us flat at k = 10 / 1,200 B.
// SLOTS (dense output): one lane per (group, output slot e, chunk column)
// instead: slot e's target is the group's e-th erased segment and its line
// comes from a segment -> line table (disjoint plan), so no lane sits on a
// line that does not fire (divLC divides by E C then).
template <int MAXC, bool SLOTS>
__global__ __launch_bounds__(kBlock) void k_decode_out(v4u* shards, const v4u* __restrict__ parity, uint32_t total,
                                                       uint32_t C, FastDiv divC, FastDiv divLC,
                                                       uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                       rfec_kmask M, DenseOut D)
{
    uint32_t hb, pb;
    if (header_block(n_hdr_blocks, hdr_every, &hb, &pb)) {
        line_headers(A, M, hb);
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
    const v4u* pl = parity + ((size_t)g * P.n_lines + l) * C + j;
    v4u acc = ld16(pl);
    const ptrdiff_t to_par = pl - grp;
    v4u mv[MAXC];
    bool use[MAXC];
#pragma unroll
    for (int q = 0; q < MAXC; ++q) { // (unconditional loads, see k_decode_rows)
        const uint32_t i = first + q * stride;
        use[q] = (uint32_t)q < count && i != tgt; // every other member of a firing line is present
        mv[q] = ld16(grp + (use[q] ? (ptrdiff_t)i * C : to_par));
    }
#pragma unroll
    for (int q = 0; q < MAXC; ++q)
        acc ^= use[q] ? mv[q] : v4u{0, 0, 0, 0};
    st16(dst, acc);
}

// The same for the row layouts (rows of COL consecutive segments, K <= 64):
// the line masks and members are arithmetic in the row index, so no plan is
// staged through LDS (no barrier before the first load).  SLOTS (dense
// output): one lane per (group, output slot e, chunk) instead of (group, row,
// chunk): slot e's target is the group's e-th erased segment, recovered when
// its row fires, so no lane sits on a row that does not (divRC divides by E C
// then; c3: 125-127 vs 137-141 us).  XCD-swizzled blocks in rounds of 8
// (traffic 1.077 vs 1.107 x algorithmic at k = 10 / 1,200 B).
// K = 0: k and col at run time (k_rt <= 64, col_rt <= COL), the member loads
// unrolled to COL and predicated on the row's size (the strip-mode plans).
// PK (with SLOTS): the masks and header records from the packed erasure
// records (rfec_recover_packed_out), header lanes packed_headers.
template <int K, int COL, bool SLOTS, bool PK = false>
__global__ __launch_bounds__(kBlock) void k_decode_rows(v4u* shards, const v4u* __restrict__ parity, uint32_t total,
                                                        uint32_t C, FastDiv divC, FastDiv divRC,
                                                        uint32_t n_hdr_blocks, uint32_t hdr_every, PeelArgs A,
                                                        rfec_kmask M, DenseOut D, uint32_t npay8, uint32_t k_rt,
                                                        uint32_t col_rt, FastDiv divCol)
{
    static_assert(K <= 64, "row decode keeps the present mask in one word");
    static_assert(!PK || SLOTS, "packed records are per output slot");
    const uint32_t KK = K ? (uint32_t)K : k_rt, CC = K ? (uint32_t)COL : col_rt;
    uint32_t hb, pb;
    if (header_block_xcd((n_hdr_blocks + 7u) >> 3, hdr_every, npay8, &hb, &pb)) {
        if (hb < n_hdr_blocks) {
            if constexpr (PK)
                packed_headers<COL>(A, hb, KK, CC);
            else
                line_headers(A, M, hb);
        }
        return;
    }
    const uint32_t R = (KK + CC - 1) / CC, LAST = KK - (R - 1) * CC;
    const uint32_t t = pb * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t g = fdiv(t, divRC);
    const uint32_t rem = t - g * divRC.d;
    const uint32_t q0 = fdiv(rem, divC); // row, or output slot (SLOTS)
    const uint32_t j = rem - q0 * divC.d;
    uint64_t h, ppm = 0;
    if constexpr (PK) { // the record's two masks: one 16-B load
        const uint64_t* pg = reinterpret_cast<const uint64_t*>(A.packed + (size_t)g * A.pk_stride);
        h = pg[0];
        ppm = pg[1];
    } else {
        h = A.present[2 * g];
    }
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
    if (__popcll(miss) != 1 || !(((PK ? ppm : A.parity_present[g]) >> r) & 1ull))
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
    // members through a descriptor over the wave's first group (wave_rsrc)
    const uint32_t gb = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
    const __amdgpu_buffer_rsrc_t rs = wave_rsrc(shards + (size_t)gb * KK * C);
    const uint32_t row0 = (((g - gb) * KK + r * CC) * C + j) * 16u;
    v4u acc = ld16(parity + ((size_t)g * R + r) * C + j);
    v4u mv[COL];
#pragma unroll
    for (int q = 0; q < COL; ++q)
        mv[q] = bld16(rs, (uint32_t)q < cnt && r * CC + q != tgt ? row0 + (uint32_t)q * C * 16u : kNoLoad);
#pragma unroll
    for (int q = 0; q < COL; ++q)
        acc ^= mv[q];
    st16(dst, acc);
}

// The batch layout -> packed erasure records (rfec_pack_erasures): one lane
// per (group, output slot e), 2^lg >= E lanes per group.  Slot e: the fec_meta
// and fec_data_size of the row of the group's e-th erased segment and the
// row's other members' records in index order (zeros past the row's end);
// all zeros where the group has no e-th erased segment.  Lane 0 writes the
// masks and zeros the record's tail.
__global__ __launch_bounds__(kBlock) void k_pack_rows(uint8_t* __restrict__ packed, const uint32_t* __restrict__ hdr,
                                                      const uint64_t* __restrict__ present,
                                                      const uint32_t* __restrict__ meta,
                                                      const uint16_t* __restrict__ fsize,
                                                      const uint64_t* __restrict__ parity_present, uint32_t groups,
                                                      uint32_t KK, uint32_t CC, uint32_t NL, uint32_t E, uint32_t lg,
                                                      uint32_t pk_stride, uint32_t pk_slot)
{
    const uint32_t hl = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = hl >> lg, e = hl & ((1u << lg) - 1u);
    if (g >= groups || e >= E)
        return;
    uint8_t* pg = packed + (size_t)g * pk_stride;
    const uint64_t h = present[2 * g];
    if (e == 0) {
        reinterpret_cast<uint64_t*>(pg)[0] = h;
        reinterpret_cast<uint64_t*>(pg)[1] = parity_present[g];
        for (uint32_t o = 16 + E * pk_slot; o < pk_stride; o += 4)
            *reinterpret_cast<uint32_t*>(pg + o) = 0;
    }
    uint64_t m = ~h & (KK == 64 ? ~0ull : (1ull << KK) - 1ull);
    for (uint32_t u = 0; u < e; ++u)
        m &= m - 1ull;
    uint32_t* so = reinterpret_cast<uint32_t*>(pg + 16 + (size_t)e * pk_slot);
    const uint32_t nd = pk_slot / 4;
    if (!m) {
        for (uint32_t d = 0; d < nd; ++d)
            so[d] = 0;
        return;
    }
    const uint32_t tgt = (uint32_t)__ffsll((long long)m) - 1, r = tgt / CC;
    const uint32_t first = r * CC, cnt = KK - first < CC ? KK - first : CC;
    const uint32_t* mr = meta + ((size_t)g * NL + r) * 5;
    for (uint32_t d = 0; d < 5; ++d)
        so[d] = mr[d];
    so[5] = fsize[(size_t)g * NL + r];
    uint32_t o = 6;
    for (uint32_t i = first; i < first + cnt; ++i) {
        if (i == tgt)
            continue;
        const uint32_t* hr = hdr + ((size_t)g * KK + i) * 5;
        for (uint32_t d = 0; d < 5; ++d)
            so[o + d] = hr[d];
        o += 5;
    }
    for (; o < nd; ++o)
        so[o] = 0;
}

// dst row r <- src row map[r] (all `C` 16-B chunks), or zeros for map[r] < 0:
// the receiver's scatter of parsed payloads into group slots and its gather
// of recovered segments.  One lane per chunk, streaming.
// The receiver session's batch split (rfec_rx.c rx_phase0), one lane per
// parsed record: the host then reads 8 bytes per record instead of the 64-B
// records the parse just wrote (cache-cold on the host), and the replay
// threads take those cache misses in parallel.  Reads only the fields the
// split needs (status, mid, seq, ts, send_ts, fec_id; rfec_wire_rec layout).
__global__ __launch_bounds__(kBlock) void k_rx_split(const rfec_wire_rec* __restrict__ recs, uint32_t n, uint32_t T,
                                                    rfec_rx_split* __restrict__ out)
{
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n)
        return;
    static_assert(offsetof(rfec_wire_rec, mid) == 2 && offsetof(rfec_wire_rec, hdr) == 8 &&
                      offsetof(rfec_wire_rec, send_ts) == 32 && offsetof(rfec_wire_rec, fec_id) == 36 &&
                      sizeof(rfec_rx_split) == 8,
                  "record layout");
    const uint32_t* r = reinterpret_cast<const uint32_t*>(recs + p);
    const uint32_t w0 = r[0], seq = r[2], ts = r[4], send_ts = r[8], fec_id = r[9] & 0xFFFFu;
    const int8_t status = (int8_t)(w0 & 0xFFu);
    const uint32_t mid = (w0 >> 16) & 0xFFu;
    uint32_t shard = 0xFFu, kind = RX_SPLIT_NONE, value = 0;
    if (status == RFEC_WIRE_OK && mid == RFEC_WIRE_SEG) {
        shard = (fec_id ? fec_id : seq) % T;
        kind = fec_id && seq ? RX_SPLIT_SEG_TS : RX_SPLIT_SEG;
        value = ts;
    } else if (status == RFEC_WIRE_OK && mid == RFEC_WIRE_FEC) {
        shard = fec_id % T;
        kind = RX_SPLIT_FEC;
        value = send_ts + 3000u;
    }
    uint2 o;
    o.x = shard | kind << 8;
    o.y = value;
    *reinterpret_cast<uint2*>(out + p) = o;
}

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
    const v4u v = s >= 0 ? ld16(src + (size_t)s * C + j) : v4u{0, 0, 0, 0};
    st16(dst + (size_t)r * C + j, v);
}

// The receiver session's device stage of one ingestion call (rfec_rx.c
// rx_device): the delivering groups' member and parity rows gathered from the
// row arena by a map the host wrote into pinned memory (read over PCIe by the
// lanes themselves), and, by the lanes after them, the host's tables (header
// records, masks, sizes, the output map) copied from pinned into device
// memory -- one launch where an H2D copy and two gathers ran in sequence (each
// step a few us of dispatch latency for ~5 MB of rows per 4,096-datagram
// batch).  The rows are stored with the default policy: the decode reads them
// next.
__global__ __launch_bounds__(kBlock) void k_rx_stage(v4u* __restrict__ dst, const v4u* __restrict__ src,
                                                     const int32_t* __restrict__ map, uint32_t total, uint32_t C,
                                                     FastDiv divC, v4u* __restrict__ tdst,
                                                     const v4u* __restrict__ tsrc, uint32_t tchunks)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t < total) {
        const uint32_t r = fdiv(t, divC);
        const uint32_t j = t - r * C;
        const int32_t s = map[r];
        dst[(size_t)r * C + j] = s >= 0 ? ld16(src + (size_t)s * C + j) : v4u{0, 0, 0, 0};
        return;
    }
    const uint32_t u = t - total;
    if (u < tchunks)
        tdst[u] = tsrc[u];
}

// Receiver groups above RFEC_MAX_K segments (a foreign peer's flexes): one
// line job per recovered segment, recovered = parity ^ the line's present
// members (flex_fec_xor.c:73-95), the host's peel in dependency levels (one
// launch per level: a job reads only arrived rows and outputs of earlier
// levels).  One lane per (job, 16-byte column); member code m >= 0: row m of
// `rows`, m < 0: output row -1 - m.
__global__ __launch_bounds__(kBlock) void k_line_jobs(const rfec_line_job* __restrict__ jobs,
                                                      const int32_t* __restrict__ members,
                                                      const v4u* __restrict__ rows, v4u* outrows, uint32_t total,
                                                      uint32_t C, FastDiv divC)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total)
        return;
    const uint32_t q = fdiv(t, divC);
    const uint32_t j = t - q * C;
    const rfec_line_job J = jobs[q];
    v4u acc = ld16(rows + (size_t)J.parity * C + j);
    uint32_t i = 0;
    for (; i + 4 <= J.n_members; i += 4) { // four loads in flight
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t m = members[J.member0 + i + u];
            v[u] = m >= 0 ? rows[(size_t)m * C + j] : outrows[(size_t)(-1 - m) * C + j];
        }
        acc ^= (v[0] ^ v[1]) ^ (v[2] ^ v[3]);
    }
    for (; i < J.n_members; ++i) {
        const int32_t m = members[J.member0 + i];
        acc ^= m >= 0 ? rows[(size_t)m * C + j] : outrows[(size_t)(-1 - m) * C + j];
    }
    outrows[(size_t)J.out * C + j] = acc;
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

// meta blocks + padding to a multiple of 8 (the swizzled grids)
inline uint32_t enc_head(const EncLaunch& a) { return (a.E.n_meta_blocks + 7u) & ~7u; }
// payload blocks for `total` lanes, in whole rounds of 8 (enc_payload_block)
inline uint32_t enc_rounds(uint64_t total) { return (blocks_for(total) + 7u) & ~7u; }

template <int K, int COL>
hipError_t launch_rows_out(const EncLaunch& a)
{
    constexpr uint32_t R = (K + COL - 1) / COL;
    const uint64_t total = (uint64_t)a.groups * R * a.cd; // < 2^32: checked by the caller
    const uint32_t head = enc_head(a);
    RFEC_LAUNCH((k_encode_out<K, COL>), dim3(head + enc_rounds(total)), dim3(kBlock), 0, a.stream, a.s, a.p,
                (uint32_t)total, a.stride / 16, make_fastdiv(a.cd), make_fastdiv(R * a.cd), head, a.E, *a.P);
    return hipGetLastError();
}

template <int CMAX>
hipError_t launch_rows_out_rt(const EncLaunch& a, uint32_t col)
{
    const uint32_t K = a.P->k, R = (K + col - 1) / col;
    const uint64_t total = (uint64_t)a.groups * R * a.cd; // < 2^32: checked by the caller
    const uint32_t head = enc_head(a);
    RFEC_LAUNCH((k_encode_out_rt<CMAX>), dim3(head + enc_rounds(total)), dim3(kBlock), 0, a.stream, a.s, a.p,
                (uint32_t)total, a.stride / 16, make_fastdiv(a.cd), make_fastdiv(R * a.cd), K, col, head, a.E,
                *a.P);
    return hipGetLastError();
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

hipError_t launch_encode(const EncLaunch& a, unsigned flags)
{
    const rfec_kplan* P = a.P;
    const bool generic = (flags & RFEC_KFLAG_GENERIC) != 0;
    uint32_t col = 0;
    // k_encode_out / k_encode_matrix_out address a wave's groups (at most kWave + 1 of them) through one
    // buffer descriptor of range kNoLoad: per-lane offsets must stay below it, or a large stride would
    // read zeros past the range (the same bound as the fused decodes, launch_recover)
    const bool rsrc_ok = (uint64_t)(kWave + 1) * P->k * a.stride < kNoLoad;
    if (!generic && is_row_layout(P, &col) && (uint64_t)a.groups * ((P->k + col - 1) / col) * a.cd < (1ull << 32)) {
        if (P->k == 10 && col == 4 && rsrc_ok)
            return launch_rows_out<10, 4>(a);
        if (P->k == 32 && col == 4 && rsrc_ok)
            return launch_rows_out<32, 4>(a);
        // other row layouts: the same output-mapped lanes with k and col at run time
        // (an 8-wide instantiation compiled to 230 VGPRs, two waves per SIMD: 0.33 of 8 TB/s at k = 20,
        // col = 5, so rows of 5..16 take the 16-wide one, 74 VGPRs)
        if (col <= 4)
            return launch_rows_out_rt<4>(a, col);
        if (col <= 16)
            return launch_rows_out_rt<16>(a, col);
    }
    const uint32_t C = a.stride / 16;
    const uint32_t total = a.groups * a.cd;
    if (!generic && rsrc_ok && P->k >= 6 && P->k <= 16 && is_full_matrix(P, P->k <= 9 ? 3 : 4)) {
        const uint32_t head = enc_head(a);
        const uint32_t nl = P->n_lines, tot = a.groups * nl * a.cd;
        const dim3 grid_o(head + enc_rounds(tot));
#define RFEC_MX(KK, CC)                                                                                           \
    case KK:                                                                                                      \
        RFEC_LAUNCH((k_encode_matrix_out<KK, CC>), grid_o, dim3(kBlock), 0, a.stream, a.s, a.p, tot, C,          \
                    make_fastdiv(a.cd), make_fastdiv(nl * a.cd), head, a.E, *P);                                  \
        return hipGetLastError();
        switch (P->k) {
            RFEC_MX(6, 3) RFEC_MX(7, 3) RFEC_MX(8, 3) RFEC_MX(9, 3) RFEC_MX(10, 4) RFEC_MX(11, 4) RFEC_MX(12, 4)
            RFEC_MX(13, 4) RFEC_MX(14, 4) RFEC_MX(15, 4) RFEC_MX(16, 4)
        default: break;
        }
#undef RFEC_MX
    }
    RFEC_LAUNCH(k_encode, dim3(a.E.n_meta_blocks + blocks_for(total)), dim3(kBlock), 0, a.stream, a.s, a.p, total, C,
                make_fastdiv(a.cd), a.E, *P);
    return hipGetLastError();
}

struct FusedArgs {
    v4u* shards;
    const v4u* parity;
    uint32_t total, C;
    FastDiv f;
    uint32_t n_hdr;
    hipStream_t stream;
    DenseOut D; // recovered payloads in place (E == 0) or to the dense output
};

// header_block()'s period for npay payload blocks: n_hdr periods of
// (every + 1) blocks must fit the grid: every <= npay / n_hdr, so fewer
// payload than header blocks keeps them at the head.
inline uint32_t hdr_every(const FusedArgs& F, uint32_t npay) { return F.n_hdr ? npay / F.n_hdr : 0; }

// cascade decode, dense: one launch (k_decode_cascade_dense); in place: the checker (schedule records and
// task words into the workspace), then the payload lanes, Q slots per group (one per possible step)
bool is_full_matrix(const rfec_kplan* P, uint32_t col);

void launch_cascade(CascArgs A, const rfec_kmask& M, uint32_t groups, uint32_t cd, void* ws, uint32_t ws_stride,
                    hipStream_t st, bool generic)
{
    A.Q = A.E ? A.E : (M.plan.n_lines < M.plan.k ? M.plan.n_lines : M.plan.k);
    A.groups = groups;
    A.total = groups * A.Q * cd; // < 2^32: checked by the caller
    A.divC = make_fastdiv(cd);
    A.divQC = make_fastdiv(A.Q * cd);
    A.ws = reinterpret_cast<uint8_t*>(ws);
    A.ws_stride = ws_stride;
    if (A.E) { // dense: one launch, the checker's blocks spread over the payload's
        const uint32_t n_hr = (blocks_for((uint64_t)groups * kCheckLanes) + 7u) >> 3; // rounds of 8 check blocks
        const uint32_t npay8 = (blocks_for(A.total) + 7u) & ~7u;
        const uint32_t every = n_hr ? (npay8 >> 3) / n_hr : 0u;
        const dim3 grid(8u * n_hr + npay8);
        const uint32_t k = M.plan.k;
        if (!generic && k >= 6 && k <= 16 && is_full_matrix(&M.plan, k <= 9 ? 3 : 4)) {
#define RFEC_MD(KK, CC)                                                                                           \
    case KK:                                                                                                      \
        RFEC_LAUNCH((k_decode_matrix_dense<KK, CC>), grid, dim3(kBlock), 0, st, A, M, n_hr, every, npay8);        \
        return;
            switch (k) {
                RFEC_MD(6, 3) RFEC_MD(7, 3) RFEC_MD(8, 3) RFEC_MD(9, 3) RFEC_MD(10, 4) RFEC_MD(11, 4) RFEC_MD(12, 4)
                RFEC_MD(13, 4) RFEC_MD(14, 4) RFEC_MD(15, 4) RFEC_MD(16, 4)
            default: break;
            }
#undef RFEC_MD
        }
        if (M.plan.k <= 32)
            RFEC_LAUNCH(k_decode_cascade_dense<uint32_t>, grid, dim3(kBlock), 0, st, A, M, n_hr, every, npay8);
        else
            RFEC_LAUNCH(k_decode_cascade_dense<uint64_t>, grid, dim3(kBlock), 0, st, A, M, n_hr, every, npay8);
        return;
    }
    const dim3 gc(blocks_for((uint64_t)groups * kCheckLanes));
    if (M.plan.k <= 32)
        RFEC_LAUNCH(k_cascade_check<uint32_t>, gc, dim3(kBlock), 0, st, A, M);
    else
        RFEC_LAUNCH(k_cascade_check<uint64_t>, gc, dim3(kBlock), 0, st, A, M);
    const uint32_t nb = (blocks_for(A.total) + 7u) & ~7u; // whole rounds of 8 (XCD swizzle)
    RFEC_LAUNCH(k_decode_cascade, dim3(nb), dim3(kBlock), 0, st, A, M);
}

// output-mapped fused decode: one lane per (group, line or output slot, chunk column)
template <int MAXC>
void launch_fused_out(const FusedArgs& F, const PeelArgs& B, const rfec_kmask& M, uint32_t cd, bool slots)
{
    const uint32_t per = slots ? F.D.E : M.plan.n_lines;
    const uint32_t total = B.groups * per * cd; // < 2^32: checked by the caller
    const uint32_t npay = blocks_for(total);
    const dim3 grid(F.n_hdr + npay);
    const FastDiv dC = make_fastdiv(cd), dLC = make_fastdiv(per * cd);
    const uint32_t every = hdr_every(F, npay);
    if (slots)
        RFEC_LAUNCH((k_decode_out<MAXC, true>), grid, dim3(kBlock), 0, F.stream, F.shards, F.parity, total, F.C, dC,
                    dLC, F.n_hdr, every, B, M, F.D);
    else
        RFEC_LAUNCH((k_decode_out<MAXC, false>), grid, dim3(kBlock), 0, F.stream, F.shards, F.parity, total, F.C, dC,
                    dLC, F.n_hdr, every, B, M, F.D);
}

// row-layout fused decode: one lane per (group, row, chunk column), or per
// (group, dense output slot, chunk column) when `slots`
template <int K, int COL>
void launch_fused_rows(const FusedArgs& F, const PeelArgs& B, const rfec_kmask& M, uint32_t cd, bool slots,
                       uint32_t col_rt = 0)
{
    const uint32_t kk = K ? (uint32_t)K : M.plan.k, cc = K ? (uint32_t)COL : col_rt;
    const uint32_t R = (kk + cc - 1) / cc;
    const uint32_t per = slots ? F.D.E : R;
    const uint32_t total = B.groups * per * cd; // < 2^32: checked by the caller
    const uint32_t npay = blocks_for(total), npay8 = (npay + 7u) & ~7u, nhr = (F.n_hdr + 7u) >> 3;
    // rounds of 8 blocks, nhr header rounds spread over npay8 / 8 payload rounds
    const dim3 grid(8u * nhr + npay8);
    const uint32_t every = nhr ? (npay8 >> 3) / nhr : 0u;
    const FastDiv dC = make_fastdiv(cd), dRC = make_fastdiv(per * cd), dCol = make_fastdiv(cc);
    if (slots)
        RFEC_LAUNCH((k_decode_rows<K, COL, true>), grid, dim3(kBlock), 0, F.stream, F.shards, F.parity, total, F.C,
                    dC, dRC, F.n_hdr, every, B, M, F.D, npay8, kk, cc, dCol);
    else
        RFEC_LAUNCH((k_decode_rows<K, COL, false>), grid, dim3(kBlock), 0, F.stream, F.shards, F.parity, total, F.C,
                    dC, dRC, F.n_hdr, every, B, M, F.D, npay8, kk, cc, dCol);
}

// packed dense decode of row layouts: lanes per (group, output slot, chunk column), header lanes per
// (group, output slot)
template <int K, int COL>
void launch_packed_rows(const FusedArgs& F, const PeelArgs& B, const rfec_kmask& M, uint32_t cd, uint32_t col_rt)
{
    const uint32_t kk = K ? (uint32_t)K : M.plan.k, cc = K ? (uint32_t)COL : col_rt;
    const uint32_t total = B.groups * F.D.E * cd; // < 2^32: checked by the caller
    const uint32_t npay = blocks_for(total), npay8 = (npay + 7u) & ~7u, nhr = (F.n_hdr + 7u) >> 3;
    const dim3 grid(8u * nhr + npay8);
    const uint32_t every = nhr ? (npay8 >> 3) / nhr : 0u;
    const FastDiv dC = make_fastdiv(cd), dRC = make_fastdiv(F.D.E * cd), dCol = make_fastdiv(cc);
    RFEC_LAUNCH((k_decode_rows<K, COL, true, true>), grid, dim3(kBlock), 0, F.stream, F.shards, F.parity, total, F.C,
                dC, dRC, F.n_hdr, every, B, M, F.D, npay8, kk, cc, dCol);
}

template <int MAXC>
void launch_fused_flat(const FusedArgs& F, const PeelArgs& B, const rfec_kmask& M)
{
    const uint32_t npay = blocks_for(F.total);
    RFEC_LAUNCH((k_decode_disjoint<MAXC>), dim3(F.n_hdr + npay), dim3(kBlock), 0, F.stream, F.shards, F.parity,
                F.total, F.C, F.f, F.n_hdr, hdr_every(F, npay), B, M, F.D);
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
    E.n_meta_blocks = (groups + gpb - 1) / gpb;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    const EncLaunch a = {P, groups, stride, cd, reinterpret_cast<const v4u*>(shards), reinterpret_cast<v4u*>(parity),
                         E, reinterpret_cast<hipStream_t>(stream)};
    return (int)launch_encode(a, flags);
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
    const bool generic = (flags & RFEC_KFLAG_GENERIC) != 0;
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
    B.rec_bytes = rfec_sched_record_bytes(P.k, P.n_lines);
    B.out_hdr = dense ? out->hdr : nullptr;
    B.out_index = dense ? out->index : nullptr;
    B.out_per_group = dense ? out->per_group : 0u;
    B.packed = nullptr;
    B.pk_stride = B.pk_slot = 0;
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
    const uint32_t C = stride / 16;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    // disjoint plans (row layer alone, strip mode), lines of <= 8 members: one launch, header lanes
    // (the fused kernels address a wave's groups through one buffer descriptor: offsets < kNoLoad)
    const bool fused = B.disjoint && maxc <= 8 && !generic &&
                       (uint64_t)(kWave + 1) * (P.k > P.n_lines ? P.k : P.n_lines) * stride < kNoLoad;
    // plans with cascades within the register schedule (the sender's matrix plans): one launch
    const uint32_t Q = dense ? out->per_group : (P.n_lines < P.k ? P.n_lines : P.k);
    const bool cascade = !B.disjoint && maxc <= 4 && P.n_lines <= 8 && P.k <= 64 && !generic &&
                         (uint64_t)groups * Q * cd < (1ull << 32) && (uint64_t)(kWave + 1) * P.k * stride < kNoLoad;
    // everything else (and RFEC_TUNE_GENERIC): the LDS peel + schedule replay, in place or dense
    // LDS per group: K + NL header records (5 dwords) + NL u16 sizes; block
    // ranges start on 8-group boundaries so the staged slices are 16-B aligned
    const uint32_t per = 5u * P.k + 6u * P.n_lines;
    // (at most 64 groups per block: the peel is one serial chain per lane, so
    // more, smaller blocks give each SIMD more chains to interleave)
    uint32_t gpb = (kPeelDwords - 8) / per;
    gpb = gpb > 64u ? 64u : gpb;
    if (gpb >= 8)
        gpb &= ~7u;
    B.gpb = gpb < 1 ? 1 : gpb;
    uint32_t n_hdr = (groups + B.gpb - 1) / B.gpb;
    B.nlp_log2 = 0;
    if (fused) { // header lanes, one per (group, line)
        uint32_t lg = 1;
        while ((1u << lg) < P.n_lines)
            ++lg;
        B.nlp_log2 = lg;
        n_hdr = (uint32_t)((((uint64_t)groups << lg) + kBlock - 1) / kBlock); // host checks groups << lg < 2^32
    }
    const uint32_t total = groups * cd;
    const FastDiv f = make_fastdiv(cd);
    const v4u* pp = reinterpret_cast<const v4u*>(parity);
    v4u* sh = reinterpret_cast<v4u*>(shards);
    if (fused) {
        const FusedArgs F = {sh, pp, total, C, f, n_hdr, st, DO};
        // output-mapped (a lane per (group, line or slot, chunk)) where a line's slot spans at least a wave
        // of chunks; below that most of its lanes would sit on lines that do not fire (k = 32 / 256 B, 2
        // erasures: 6 of 8 rows idle, 60.0 vs 41.6 us flat), so the flat form -- except a dense output of
        // row layouts with slots of >= 16 chunks: lanes per output slot sit on no idle line (k = 32 /
        // 256 B: 33.2-33.9 vs 34.6-34.9 us flat, round 5)
        uint32_t col = 0;
        const bool slots = F.D.E && F.D.E <= P.n_lines; // dense output: lanes per output slot
        const bool rows = !generic && is_row_layout(&P, &col) && col <= 4 && P.k <= 64;
        if ((cd >= (uint32_t)kWave || (slots && rows && cd >= 16)) &&
            (uint64_t)groups * P.n_lines * cd < (1ull << 32)) {
            if (rows) {
                if (P.k == 10 && col == 4)
                    launch_fused_rows<10, 4>(F, B, *M, cd, slots);
                else if (P.k == 32 && col == 4)
                    launch_fused_rows<32, 4>(F, B, *M, cd, slots);
                else // other row layouts of k <= 64, rows of <= 4 members: k and col at run time
                    launch_fused_rows<0, 4>(F, B, *M, cd, slots, col);
                return (int)hipGetLastError();
            }
            if (maxc <= 4)
                launch_fused_out<4>(F, B, *M, cd, slots);
            else
                launch_fused_out<8>(F, B, *M, cd, slots);
            return (int)hipGetLastError();
        }
        if (maxc <= 4)
            launch_fused_flat<4>(F, B, *M);
        else
            launch_fused_flat<8>(F, B, *M);
        return (int)hipGetLastError();
    }
    if (cascade) {
        CascArgs A;
        A.shards = sh;
        A.parity = pp;
        A.hdr_dw = reinterpret_cast<uint32_t*>(hdr);
        A.meta_dw = reinterpret_cast<const uint32_t*>(meta);
        A.fsize = fsize;
        A.present = present;
        A.parity_present = parity_present;
        A.recovered = recovered;
        A.out_sh = DO.sh;
        A.out_hdr_dw = dense ? reinterpret_cast<uint32_t*>(out->hdr) : nullptr;
        A.out_index = dense ? out->index : nullptr;
        A.E = DO.E;
        A.C = C;
        A.capacity = capacity;
        launch_cascade(A, *M, groups, cd, ws, B.rec_bytes, st, (flags & RFEC_KFLAG_MATRIX_GENERIC) != 0);
        return (int)hipGetLastError();
    }
    RFEC_LAUNCH(k_peel_lds, dim3(n_hdr), dim3(kBlock), 0, st, B, *M);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return (int)e;
    const uint32_t fast = maxc <= 8 ? 1u : 0u;
    const dim3 grid(blocks_for(total));
    if (maxc <= 4)
        RFEC_LAUNCH((k_recover_flat<4, 2>), grid, dim3(kBlock), 0, st, sh, pp, B.sched, total, C, f, B.rec_bytes, fast,
                    P, DO, present);
    else
        RFEC_LAUNCH((k_recover_flat<8, 1>), grid, dim3(kBlock), 0, st, sh, pp, B.sched, total, C, f, B.rec_bytes, fast,
                    P, DO, present);
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

int rfec_launch_pack_rows(const rfec_kplan* P, uint32_t col, uint32_t groups, const rfec_hdr* hdr,
                          const uint64_t* present, const rfec_hdr* meta, const uint16_t* fsize,
                          const uint64_t* parity_present, uint32_t per_group, uint8_t* packed, uint32_t pk_stride,
                          uint32_t pk_slot, void* stream)
{
    uint32_t lg = 0;
    while ((1u << lg) < per_group)
        ++lg;
    const uint32_t lanes = groups << lg; // < 2^32: host-checked
    RFEC_LAUNCH(k_pack_rows, dim3(blocks_for(lanes)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), packed,
                reinterpret_cast<const uint32_t*>(hdr), present, reinterpret_cast<const uint32_t*>(meta), fsize,
                parity_present, groups, P->k, col, P->n_lines, per_group, lg, pk_stride, pk_slot);
    return (int)hipGetLastError();
}

int rfec_launch_recover_packed(const rfec_kmask* M, uint32_t col, uint32_t groups, uint32_t stride,
                               uint32_t capacity, const uint8_t* shards, const uint8_t* parity, const uint8_t* packed,
                               uint32_t pk_stride, uint32_t pk_slot, uint64_t* recovered,
                               const rfec_dense_out* out, void* stream)
{
    const rfec_kplan* P = &M->plan;
    PeelArgs B = {};
    B.recovered = recovered;
    B.groups = groups;
    B.capacity = capacity;
    B.out_hdr = out->hdr;
    B.out_index = out->index;
    B.out_per_group = out->per_group;
    B.packed = packed;
    B.pk_stride = pk_stride;
    B.pk_slot = pk_slot;
    uint32_t lg = 0;
    while ((1u << lg) < out->per_group)
        ++lg;
    B.nlp_log2 = lg;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    const uint32_t n_hdr = (uint32_t)((((uint64_t)groups << lg) + kBlock - 1) / kBlock);
    const DenseOut DO = {reinterpret_cast<v4u*>(out->shards), out->per_group};
    const FusedArgs F = {const_cast<v4u*>(reinterpret_cast<const v4u*>(shards)), reinterpret_cast<const v4u*>(parity),
                         groups * cd, stride / 16, make_fastdiv(cd), n_hdr, reinterpret_cast<hipStream_t>(stream), DO};
    if (P->k == 10 && col == 4)
        launch_packed_rows<10, 4>(F, B, *M, cd, col);
    else if (P->k == 32 && col == 4)
        launch_packed_rows<32, 4>(F, B, *M, cd, col);
    else
        launch_packed_rows<0, 4>(F, B, *M, cd, col);
    return (int)hipGetLastError();
}

int rfec_launch_line_jobs(const rfec_line_job* jobs, uint32_t n_jobs, const int32_t* members, const uint8_t* rows,
                          uint8_t* outrows, uint32_t stride, void* stream)
{
    if (n_jobs == 0)
        return 0;
    const uint32_t C = stride / 16, total = n_jobs * C; // n_jobs * C < 2^32: host-bounded
    RFEC_LAUNCH(k_line_jobs, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), jobs,
                members, reinterpret_cast<const v4u*>(rows), reinterpret_cast<v4u*>(outrows), total, C,
                make_fastdiv(C));
    return (int)hipGetLastError();
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

int rfec_launch_rx_stage(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                         void* tdst, const void* tsrc, size_t tbytes, void* stream)
{
    const uint32_t C = stride / 16;
    const uint64_t total = (uint64_t)rows * C, tchunks = (tbytes + 15) / 16;
    if (total + tchunks >= (1ull << 32) || stride % 16)
        return (int)hipErrorInvalidValue;
    if (!(total + tchunks))
        return 0;
    RFEC_LAUNCH(k_rx_stage, dim3(blocks_for(total + tchunks)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                reinterpret_cast<v4u*>(dst), reinterpret_cast<const v4u*>(src), map, (uint32_t)total, C,
                make_fastdiv(C ? C : 1), reinterpret_cast<v4u*>(tdst), reinterpret_cast<const v4u*>(tsrc),
                (uint32_t)tchunks);
    return (int)hipGetLastError();
}

int rfec_launch_rx_split(const rfec_wire_rec* recs, uint32_t n, uint32_t T, rfec_rx_split* out, void* stream)
{
    if (!n)
        return 0;
    RFEC_LAUNCH(k_rx_split, dim3(blocks_for(n)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), recs, n, T,
                out);
    return (int)hipGetLastError();
}

int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream)
{
    const uint32_t C = stride / 16;
    const uint32_t total = slots * C;
    RFEC_LAUNCH(k_zero_tails, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                reinterpret_cast<v4u*>(shards), hdr, total, C, make_fastdiv(C));
    return (int)hipGetLastError();
}

const char* rfec_hip_error_string(int code) { return hipGetErrorString((hipError_t)code); }

} // extern "C"
