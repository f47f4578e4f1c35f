// rfec_hostio.hip -- CDNA4 (gfx950) kernels that move razor's own structs
// between host memory and the HBM slot layout over PCIe, for the zero-copy
// form of the host-memory batch paths (rfec_hostmem.c): when the caller's
// sim_segment_t / sim_fec_t structs lie in pinned memory the device maps
// (rfec_pinned_alloc), the device reads and writes them itself, so the host
// threads' gather / scatter and the bulk H2D / D2H copies drop out.
//
// Layouts (include/razor_fec.h, the reference's sim_proto.h:80-174):
//   sim_segment_t  header fields at bytes 0-17, data_size at 32, data at 34
//   sim_fec_t      stamps at 0-19, fec_meta at 20-39, fec_data_size at 40,
//                  fec_data at 42
// The structs are 4-byte aligned (their sizes are multiples of 4), their data
// 2 bytes off a dword.  A lane moves one 16-byte chunk: it loads the aligned
// 16 bytes that start 2 bytes before its chunk and takes the last 2 bytes from
// the next lane (DPP wave_shl:1); lane 63 and the last chunk of a struct load
// that dword themselves.  Writes go the same way round: a lane stores the
// aligned 16 bytes from its chunk's third byte on, the next lane's first two
// bytes included, and each struct's first lane the dword holding the size and
// the data's first two bytes.
//
// Semantics follow the host paths they replace (rfec_hostmem.c): the gather
// stages min(size, SIM_VIDEO_SIZE) payload bytes and zeros to the slot's end
// (stage_payload), a NULL pointer is a lost struct (zero slot, zero header);
// the parity scatter stamps fec_id / base_id / row / col / index / count as
// flex_fec_sender_update does (flex_fec_sender.c:176-181, :220-225), leaves
// send_ts and transport_seq alone, and writes fec_data_size = 0xFFFF and
// nothing else of the line where flex_fec_generate fails; the recovered-segment
// scatter writes what flex_fec_recover writes (flex_fec_xor.c:64-101) plus the
// group's fec_id, the whole data array.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rfec_internal.h"
#include "rfec_launch.h"

namespace {

constexpr int kBlock = 256;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct FastDiv {
    uint32_t d, m, s;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f)
{
    return (uint32_t)(((uint64_t)__umulhi(n, f.m) + n) >> f.s);
}
FastDiv make_fastdiv(uint32_t d)
{
    uint32_t s = 0;
    while ((1ull << s) < d)
        ++s;
    const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
    return FastDiv{d, (uint32_t)m, s};
}

// lane i + 1's value (0 in lane 63): DPP wave_shl:1; every lane must take part
__device__ __forceinline__ uint32_t next_lane(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

__device__ __forceinline__ v4u ld_host16(const uint8_t* p) // 4-byte aligned
{
    v4u v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
    return v;
}
__device__ __forceinline__ uint32_t ld_host4(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void st_host16(uint8_t* p, v4u v) { __builtin_memcpy(__builtin_assume_aligned(p, 4), &v, 16); }
__device__ __forceinline__ void st_host4(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
__device__ __forceinline__ void st_host2(uint8_t* p, uint32_t v) { *reinterpret_cast<uint16_t*>(p) = (uint16_t)v; }

// The part of a 16-byte access that lies inside a struct: `avail` = the
// struct's bytes from the access on (a multiple of 4, the structs' sizes and
// the accesses' offsets being so).  With SIM_VIDEO_SIZE % 16 != 0 (1000: 63
// chunks = 1,008 bytes of data lanes) a struct's last chunk reaches past its
// end; those dwords are neither read nor written (the next struct's header,
// or past the pinned block for the last one).
__device__ __forceinline__ v4u ld_host_part(const uint8_t* p, int avail)
{
    if (avail >= 16)
        return ld_host16(p);
    v4u v = {0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < 3; ++d)
        if (4 * d < avail)
            v[d] = ld_host4(p + 4 * d);
    return v;
}
__device__ __forceinline__ void st_host_part(uint8_t* p, v4u v, int avail)
{
    if (avail >= 16) {
        st_host16(p, v);
        return;
    }
#pragma unroll
    for (int d = 0; d < 3; ++d)
        if (4 * d < avail)
            st_host4(p + 4 * d, v[d]);
}
// sizeof(sim_segment_t) / sizeof(sim_fec_t) for a SIM_VIDEO_SIZE: the data
// offset + video, up to the structs' 4-byte alignment (sim_proto.h:80-99,157-174)
__device__ __forceinline__ int struct_bytes(uint32_t doff, uint32_t video) { return (int)((doff + video + 3u) & ~3u); }

// bytes [2, 18) of the 20 bytes (x0..x3, nx)
__device__ __forceinline__ v4u shift2(const v4u& x, uint32_t nx)
{
    return v4u{__builtin_amdgcn_alignbyte(x[1], x[0], 2), __builtin_amdgcn_alignbyte(x[2], x[1], 2),
               __builtin_amdgcn_alignbyte(x[3], x[2], 2), __builtin_amdgcn_alignbyte(nx, x[3], 2)};
}

// bytes >= n of a 16-byte chunk zeroed (n may be <= 0 or >= 16)
__device__ __forceinline__ v4u keep16(v4u v, int n)
{
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t t8 = 8u * (uint32_t)min(max(n - 4 * i, 0), 4);
        v[i] &= (uint32_t)~(0xFFFFFFFFull << t8);
    }
    return v;
}

// Host structs -> slots [n][C] (16-B chunks) + 20-byte header records.
// KIND 0: sim_segment_t (header = bytes 0-17 + data_size); KIND 1: sim_fec_t
// (header = fec_meta, and its fec_data_size / fec_id into fsize / fecid).
// A pointer with bit 0 set is header only: the struct's header fields are
// read, its payload is not (the slot is zeroed) -- the receive side marks so
// the structs on no line that can fire, whose bytes the decode never reads.
struct GatherSide {
    const uint64_t* ptrs; // device addresses of the structs (0: lost, bit 0: header only)
    uint32_t total;       // lanes: structs x C
    v4u* dst;             // slots [n][C]
    uint32_t* hdr_dw;     // 20-byte header records
    uint16_t* fsize;      // KIND 1: fec_data_size, fec_id
    uint16_t* fecid;
};

template <int KIND>
__device__ __forceinline__ void gather_lane(const GatherSide& S, uint32_t t, uint32_t C, const FastDiv& divC,
                                            uint32_t video)
{
    constexpr uint32_t DOFF = KIND ? 42u : 34u; // data
    const bool live = t < S.total;
    const uint32_t slot = live ? fdiv(t, divC) : 0u, j = live ? t - slot * C : 0u;
    const uint64_t raw = live ? S.ptrs[slot] : 0u;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(raw & ~(uint64_t)3);
    const uint32_t nload = (video + 15u) / 16u; // chunks that hold struct bytes
    const bool ld = p && !(raw & 1u) && j < nload;
    const int avail = struct_bytes(DOFF, video) - (int)(DOFF - 2u + 16u * j); // struct bytes from the load on
    v4u x = {0, 0, 0, 0};
    uint32_t sz = 0;
    if (ld)
        x = ld_host_part(p + DOFF - 2u + 16u * j, avail);
    if (p && (ld || j == 0))
        sz = *reinterpret_cast<const uint16_t*>(p + DOFF - 2u); // (one address per struct: coalesced)
    uint32_t nx = next_lane(x[0]);
    if (ld && ((threadIdx.x & 63u) == 63u || j + 1u >= nload))
        nx = avail >= 20 ? ld_host4(p + DOFF + 14u + 16u * j) : 0u; // (only inside the struct)
    if (!live)
        return;
    const int n = (int)min(sz, video) - (int)(16u * j);
    __builtin_nontemporal_store(keep16(shift2(x, nx), n), S.dst + (size_t)slot * C + j);
    if (j != 0)
        return;
    uint32_t h[5] = {0, 0, 0, 0, 0};
    uint32_t fs = 0, id = 0;
    if (p) {
        if constexpr (KIND == 0) {
            const v4u a = ld_host16(p);
            h[0] = a[0], h[1] = a[1], h[2] = a[2], h[3] = a[3];
            h[4] = (ld_host4(p + 16) & 0xFFFFu) | sz << 16;
        } else {
            const v4u a = ld_host16(p + 20);
            h[0] = a[0], h[1] = a[1], h[2] = a[2], h[3] = a[3];
            h[4] = ld_host4(p + 36);
            fs = sz;
            id = ld_host4(p) & 0xFFFFu;
        }
    }
    uint32_t* o = S.hdr_dw + (size_t)slot * 5;
#pragma unroll
    for (int d = 0; d < 5; ++d)
        o[d] = h[d];
    if constexpr (KIND == 1) {
        S.fsize[slot] = (uint16_t)fs;
        S.fecid[slot] = (uint16_t)id;
    }
}

// One launch for both kinds: blocks [0, b1) gather the segments (side 0),
// the rest the parities (side 1), so the receive side's two gathers share one
// tail; the first aux_n lanes also copy aux_src -> aux_dst (the masks into HBM).
__global__ __launch_bounds__(kBlock) void k_host_gather(GatherSide s0, GatherSide s1, uint32_t b1, uint32_t C,
                                                        FastDiv divC, uint32_t video,
                                                        const uint64_t* __restrict__ aux_src,
                                                        uint64_t* __restrict__ aux_dst, uint32_t aux_n)
{
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    if (g < aux_n)
        aux_dst[g] = aux_src[g];
    if (blockIdx.x < b1)
        gather_lane<0>(s0, g, C, divC, video);
    else
        gather_lane<1>(s1, (blockIdx.x - b1) * kBlock + threadIdx.x, C, divC, video);
}

// Parity slots [G][n][C] + meta / fsize / status -> the callers' sim_fec_t.
__global__ __launch_bounds__(kBlock) void k_host_scatter_fec(const uint64_t* __restrict__ fptrs, uint32_t total,
                                                             uint32_t C, FastDiv divC, FastDiv divN,
                                                             const v4u* __restrict__ parity,
                                                             const uint32_t* __restrict__ meta_dw,
                                                             const uint16_t* __restrict__ fsize,
                                                             const int8_t* __restrict__ status,
                                                             const uint32_t* __restrict__ hdr_dw, uint32_t k,
                                                             uint32_t fec_base, uint32_t g0, rfec_kplan P,
                                                             uint32_t video)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const bool live = t < total;
    const uint32_t o = live ? fdiv(t, divC) : 0u, j = live ? t - o * C : 0u;
    const uint32_t nch = (video + 15u) / 16u;
    const bool ok = live && status[o] == 0;
    const bool dat = ok && j < nch;
    v4u c = {0, 0, 0, 0};
    if (dat)
        c = __builtin_nontemporal_load(parity + (size_t)o * C + j);
    uint32_t nx = next_lane(c[0]);
    if (dat && (threadIdx.x & 63u) == 63u)
        nx = j + 1u < nch ? parity[(size_t)o * C + j + 1u][0] : 0u;
    if (dat && j + 1u >= nch)
        nx = 0; // past fec_data: the struct's two padding bytes
    if (!live)
        return;
    uint8_t* p = reinterpret_cast<uint8_t*>(fptrs[o]);
    if (dat) // (the last chunk only up to the struct's end: 1,044 B at SIM_VIDEO_SIZE 1000)
        st_host_part(p + 44u + 16u * j, shift2(c, nx), struct_bytes(42u, video) - (int)(44u + 16u * j));
    if (j != 0)
        return;
    const uint32_t g = fdiv(o, divN), l = o - g * divN.d;
    uint32_t base = 0xFFFFFFFFu; // base_id: the group's smallest packet id
    for (uint32_t i = 0; i < k; ++i)
        base = min(base, hdr_dw[((size_t)g * k + i) * 5]);
    const uint32_t fec_id = (fec_base + g0 + g) % 65535u + 1u;
    st_host4(p, fec_id | (uint32_t)P.row << 16 | (uint32_t)P.col << 24);
    st_host4(p + 4, (uint32_t)P.line[l].index | (uint32_t)P.k << 16);
    st_host4(p + 8, base);
    if (ok) {
        const uint32_t* m = meta_dw + (size_t)o * 5;
        st_host16(p + 20, v4u{m[0], m[1], m[2], m[3]});
        st_host4(p + 36, m[4]);
        st_host4(p + 40, (uint32_t)fsize[o] | (c[0] & 0xFFFFu) << 16);
    } else {
        st_host2(p + 40, 0xFFFFu);
    }
}

// Recovered segments (dense output [G][E][C], headers, out_index) -> the
// callers' sim_segment_t (NULL or out_index 0xFF: left alone); out_index and
// the recovered masks also into host memory (oidx_host, rec_host).
__global__ __launch_bounds__(kBlock) void k_host_scatter_seg(const uint64_t* __restrict__ optrs, uint32_t total,
                                                             uint32_t C, FastDiv divC, FastDiv divE,
                                                             const v4u* __restrict__ out_sh,
                                                             const uint32_t* __restrict__ out_hdr_dw,
                                                             const uint8_t* __restrict__ out_index,
                                                             const uint16_t* __restrict__ fecid,
                                                             const uint64_t* __restrict__ ppm, uint32_t n,
                                                             uint32_t video, uint8_t* __restrict__ oidx_host,
                                                             const uint64_t* __restrict__ rec,
                                                             uint64_t* __restrict__ rec_host)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const bool live = t < total;
    const uint32_t o = live ? fdiv(t, divC) : 0u, j = live ? t - o * C : 0u;
    const uint32_t nch = (video + 15u) / 16u;
    uint8_t* p = live ? reinterpret_cast<uint8_t*>(optrs[o]) : nullptr;
    const uint32_t oi = live ? out_index[o] : 0xFFu;
    if (live && j == 0) {
        oidx_host[o] = (uint8_t)oi;
        const uint32_t g = fdiv(o, divE);
        if (o == g * divE.d) {
            rec_host[2 * g] = rec[2 * g];
            rec_host[2 * g + 1] = rec[2 * g + 1];
        }
    }
    const bool on = p && oi != 0xFFu;
    const bool dat = on && j < nch;
    v4u c = {0, 0, 0, 0};
    if (dat)
        c = __builtin_nontemporal_load(out_sh + (size_t)o * C + j);
    uint32_t nx = next_lane(c[0]);
    if (dat && (threadIdx.x & 63u) == 63u)
        nx = j + 1u < nch ? out_sh[(size_t)o * C + j + 1u][0] : 0u;
    if (dat && j + 1u >= nch)
        nx = 0; // past data: the struct's padding
    if (!dat)
        return;
    st_host_part(p + 36u + 16u * j, shift2(c, nx), struct_bytes(34u, video) - (int)(36u + 16u * j));
    if (j != 0)
        return;
    const uint32_t* h = out_hdr_dw + (size_t)o * 5;
    st_host16(p, v4u{h[0], h[1], h[2], h[3]}); // packet_id, fid, timestamp, index, total
    st_host2(p + 16, h[4]);                    // ftype, payload_type (remb kept)
    st_host4(p + 32, (h[4] >> 16) | (c[0] & 0xFFFFu) << 16);
    const uint32_t g = fdiv(o, divE);
    const uint64_t pm = ppm[g];
    st_host2(p + 20, pm ? fecid[(size_t)g * n + (uint32_t)__ffsll((long long)pm) - 1u] : 0u); // the group's fec_id
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

// Sender staging without a host copy (rfec_sender.c rfec_host_send_frames,
// frames in rfec_pinned_alloc memory): slot s <- the segment bytes [src[s],
// src[s] + size[s]) read over PCIe by the lanes themselves, zeros past size
// (src 0: a zero slot).  The bytes lie at any alignment (sim_split_frame's
// offsets): a lane loads the 4-byte-aligned 16 bytes at or before its chunk --
// only the dwords holding segment bytes, so no load leaves the segment's last
// dword -- and takes the bytes past them from the next lane (DPP wave_shl:1;
// the wave's last lane and a slot's last chunk load that dword themselves).
__global__ __launch_bounds__(kBlock) void k_send_gather(const uint64_t* __restrict__ src,
                                                        const uint16_t* __restrict__ size, uint32_t total, uint32_t C,
                                                        FastDiv divC, v4u* __restrict__ dst)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const bool live = t < total;
    const uint32_t slot = live ? fdiv(t, divC) : 0u, j = live ? t - slot * C : 0u;
    const uint64_t a = live ? src[slot] : 0u;
    const uint32_t n = a ? size[slot] : 0u, mis = (uint32_t)a & 3u;
    const uint8_t* base = reinterpret_cast<const uint8_t*>(a - mis) + 16u * j;
    const int need = (int)(mis + n) - (int)(16u * j); // window bytes from this lane's load on that are wanted
    v4u x = {0, 0, 0, 0};
    if (need > 0)
        x = ld_host_part(base, (need + 3) & ~3);
    uint32_t nx = next_lane(x[0]);
    if (mis && need > 16 && ((threadIdx.x & 63u) == 63u || j + 1u == C))
        nx = ld_host4(base + 16);
    if (!live)
        return;
    const v4u v = {__builtin_amdgcn_alignbyte(x[1], x[0], mis), __builtin_amdgcn_alignbyte(x[2], x[1], mis),
                   __builtin_amdgcn_alignbyte(x[3], x[2], mis), __builtin_amdgcn_alignbyte(nx, x[3], mis)};
    dst[(size_t)slot * C + j] = keep16(v, (int)n - (int)(16u * j));
}

} // namespace

extern "C" {

int rfec_launch_host_gather(const uint64_t* sptrs, uint32_t ns, uint8_t* shards, rfec_hdr* hdr,
                            const uint64_t* fptrs, uint32_t nf, uint8_t* parity, rfec_hdr* meta, uint16_t* fsize,
                            uint16_t* fecid, uint32_t stride, uint32_t video, const uint64_t* aux_src,
                            uint64_t* aux_dst, uint32_t aux_n, void* stream)
{
    const uint32_t C = stride / 16;
    const GatherSide s0{sptrs, ns * C, reinterpret_cast<v4u*>(shards), reinterpret_cast<uint32_t*>(hdr), nullptr,
                        nullptr};
    const GatherSide s1{fptrs, nf * C, reinterpret_cast<v4u*>(parity), reinterpret_cast<uint32_t*>(meta), fsize,
                        fecid};
    const uint32_t b1 = blocks_for(s0.total > aux_n ? s0.total : aux_n), nb = b1 + blocks_for(s1.total);
    if (!nb)
        return 0;
    RFEC_LAUNCH(k_host_gather, dim3(nb), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), s0, s1, b1, C,
                make_fastdiv(C), video, aux_src, aux_dst, aux_n);
    return (int)hipGetLastError();
}

int rfec_launch_send_gather(const uint64_t* src, const uint16_t* size, uint32_t slots, uint32_t stride, uint8_t* dst,
                            void* stream)
{
    const uint32_t C = stride / 16, total = slots * C; // slots * C < 2^32: host-bounded
    if (!total)
        return 0;
    RFEC_LAUNCH(k_send_gather, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), src,
                size, total, C, make_fastdiv(C), reinterpret_cast<v4u*>(dst));
    return (int)hipGetLastError();
}

int rfec_launch_host_scatter_fec(const uint64_t* fptrs, uint32_t groups, const rfec_kplan* P, uint32_t stride,
                                 const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                                 const int8_t* status, const rfec_hdr* hdr, uint16_t fec_id0, uint32_t g0,
                                 uint32_t video, void* stream)
{
    const uint32_t C = stride / 16, nl = P->n_lines, total = groups * nl * C;
    if (!total)
        return 0;
    const uint32_t fec_base = fec_id0 ? fec_id0 - 1u : 0u; // flex_fec_sender.c:241-243: +1 per group, 0 skipped
    RFEC_LAUNCH(k_host_scatter_fec, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                fptrs, total, C, make_fastdiv(C), make_fastdiv(nl), reinterpret_cast<const v4u*>(parity),
                reinterpret_cast<const uint32_t*>(meta), fsize, status, reinterpret_cast<const uint32_t*>(hdr),
                (uint32_t)P->k, fec_base, g0, *P, video);
    return (int)hipGetLastError();
}

int rfec_launch_host_scatter_seg(const uint64_t* optrs, uint32_t groups, uint32_t E, uint32_t stride,
                                 const uint8_t* out_shards, const rfec_hdr* out_hdr, const uint8_t* out_index,
                                 const uint16_t* fecid, const uint64_t* ppm, uint32_t n_lines, uint32_t video,
                                 uint8_t* oidx_host, const uint64_t* recovered, uint64_t* rec_host, void* stream)
{
    const uint32_t C = stride / 16, total = groups * E * C;
    if (!total)
        return 0;
    RFEC_LAUNCH(k_host_scatter_seg, dim3(blocks_for(total)), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                optrs, total, C, make_fastdiv(C), make_fastdiv(E), reinterpret_cast<const v4u*>(out_shards),
                reinterpret_cast<const uint32_t*>(out_hdr), out_index, fecid, ppm, n_lines, video, oidx_host,
                recovered, rec_host);
    return (int)hipGetLastError();
}

} // extern "C"
