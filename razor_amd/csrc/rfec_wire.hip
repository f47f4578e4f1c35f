// rfec_wire.hip -- CDNA4 (gfx950) kernels of the batched wire codec: SIM_FEC /
// SIM_SEG datagrams with their CRC32 trailer, and the receive-side parse.
//
// Restated from the reference (yuanrongxi/razor):
//   datagram = header (sim_proto.c:13-18) | body | crc32 BE (sim_proto.c:92-94)
//   SIM_FEC body  sim_proto.inl:244-254, 270-285;  SIM_SEG body :83-125
//   parse         sim_proto.c:21-37 (CRC check), sim_session.c:594 (mid range),
//                 sim_proto.inl:127-179, 256-307; reads past the datagram end
//                 yield 0 without advancing (cf_stream.c mach_*_read)
//   crc32         cf_crc32.c:56-68, seed 0x0e3dfc0a (sim_proto.c:11)
//
// Framing into, and parsing of, datagram slots of at most 1,280 bytes: the
// quarter-wave kernels at the end of this file (k_frame_seg_q, k_frame_fec_q,
// k_parse_q: 16 lanes per datagram, four datagrams per wave).  The parse of
// wider payload slots (and with RFEC_TUNE_WAVE_PARSE), and framing into wider
// slots: one wavefront per datagram; lane j owns bytes [B j, B j + B) of it,
// B = 20 when the slot holds at most 1,280 bytes (a 1,249-byte SIM_FEC or
// 1,236-byte SIM_SEG at 1,200-byte payloads then keeps 63 of 64 lanes busy),
// else B = 32 (slots up to 2 KiB).  Every lane load / store is a dword buffer access at a
// dword-aligned offset, range-checked per dword against its slot.  Payload
// bytes move through registers with a wave-uniform byte funnel (no LDS
// staging); the header is assembled with compile-time byte positions.  CRC32
// is computed wave-parallel: each lane takes the raw CRC of its B bytes with
// slice-by-16 / slice-by-4 tables in LDS and scales it to the end of the
// message by x^(8e) mod P, e = the bytes after its run.  With
// n = 64 B - B q - r, e = 8 B (63 - j - q) - 8r: the x^(8 B (63 - c)) part is
// a fixed per-column multiplier (eight nibble lookups in column c = j + q,
// zlib's multmodp tabulated), the x^(-8r) part is applied once to the wave's
// XOR-reduced sum (one lookup per bit lane).  The CRC's initial register is
// folded into the first four message bytes, so every lane runs from a zero
// register.  Cross-lane sums use DPP within rows plus readlane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rfec_internal.h"
#include "rfec_launch.h"

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 1024;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr uint32_t kPoly = 0xEDB88320u; // reflected CRC-32 polynomial (cf_crc32.c table)

// LDS tables (built at compile time, copied to LDS once per block), per lane
// width B:
//   t[s][b]         CRC register after byte b then s zero bytes, from 0 (slice-by-16)
//   nib[i][v][c]    (nibble v at nibble position i of a register) * x^(8 B (63-c)):
//                   a B-byte run in column c of a 64 B-byte window, carried to the
//                   window's end.  [i][v][c]: the lanes read distinct columns, so
//                   they never share an LDS bank.
//   inv[r][i]       x^(31-i) * x^(-8r), r < B: bit i of a register times x^(-8r)
// (bit p of a register is the coefficient of x^(31-p))
template <int B>
struct CrcTables {
    uint32_t t[16][256];
    uint32_t nib[8][16][kWave];
    uint32_t inv[B][32];
};

constexpr uint32_t mul_x(uint32_t v) { return (v & 1u) ? (v >> 1) ^ kPoly : v >> 1; }
// the inverse of mul_x (kPoly has bit 31 set, v >> 1 never does)
constexpr uint32_t div_x(uint32_t v) { return (v & 0x80000000u) ? (((v ^ kPoly) << 1) | 1u) : (v << 1); }

template <int B>
constexpr CrcTables<B> make_crc_tables()
{
    CrcTables<B> r{};
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int i = 0; i < 8; ++i)
            c = mul_x(c);
        r.t[0][b] = c;
    }
    for (int s = 1; s < 16; ++s)
        for (uint32_t b = 0; b < 256; ++b)
            r.t[s][b] = (r.t[s - 1][b] >> 8) ^ r.t[0][r.t[s - 1][b] & 0xffu];
    // V_c = x^(8 B (63 - c))
    uint32_t V = 0x80000000u; // x^0, for column 63
    for (int j = kWave - 1; j >= 0; --j) {
        uint32_t basis[32]{}; // basis[e] = x^e * V_j
        uint32_t v = V;
        for (int e = 0; e < 32; ++e) {
            basis[e] = v;
            v = mul_x(v);
        }
        for (int i = 0; i < 8; ++i)
            for (uint32_t nv = 0; nv < 16; ++nv) {
                uint32_t acc = 0;
                for (int k = 0; k < 4; ++k)
                    if (nv & (1u << k))
                        acc ^= basis[31 - (4 * i + k)];
                r.nib[i][nv][j] = acc;
            }
        for (int q = 0; q < 8 * B; ++q)
            V = mul_x(V);
    }
    for (int i = 0; i < 32; ++i) {
        uint32_t v = 1u << i; // x^(31-i)
        for (int q = 0; q < B; ++q) {
            r.inv[q][i] = v;
            for (int b = 0; b < 8; ++b)
                v = div_x(v);
        }
    }
    return r;
}

__device__ const CrcTables<20> kCrc20 = make_crc_tables<20>();
__device__ const CrcTables<32> kCrc32 = make_crc_tables<32>();

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int B>
constexpr int kTabDwords = (int)(sizeof(CrcTables<B>) / 4);
constexpr int kNibBase = 16 * 256;                 // dword offset of nib in the LDS copy
constexpr int kInvBase = kNibBase + 8 * 16 * kWave; // dword offset of inv
template <int B>
__device__ __forceinline__ void load_tables(uint32_t* T)
{
    const v4u* s;
    if constexpr (B == 20)
        s = reinterpret_cast<const v4u*>(&kCrc20);
    else
        s = reinterpret_cast<const v4u*>(&kCrc32);
    v4u* d = reinterpret_cast<v4u*>(T);
    for (int i = threadIdx.x; i < kTabDwords<B> / 4; i += kBlock)
        d[i] = s[i];
    __syncthreads();
}

__device__ __forceinline__ uint32_t tb(const uint32_t* T, int s, uint32_t byte) { return T[s * 256 + byte]; }

// raw CRC (zero register) of 16 bytes given as LE dwords
__device__ __forceinline__ uint32_t slice16(const uint32_t* T, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return tb(T, 15, a & 0xff) ^ tb(T, 14, (a >> 8) & 0xff) ^ tb(T, 13, (a >> 16) & 0xff) ^ tb(T, 12, a >> 24) ^
           tb(T, 11, b & 0xff) ^ tb(T, 10, (b >> 8) & 0xff) ^ tb(T, 9, (b >> 16) & 0xff) ^ tb(T, 8, b >> 24) ^
           tb(T, 7, c & 0xff) ^ tb(T, 6, (c >> 8) & 0xff) ^ tb(T, 5, (c >> 16) & 0xff) ^ tb(T, 4, c >> 24) ^
           tb(T, 3, d & 0xff) ^ tb(T, 2, (d >> 8) & 0xff) ^ tb(T, 1, (d >> 16) & 0xff) ^ tb(T, 0, d >> 24);
}

// raw CRC (zero register) of 4 bytes given as one LE dword
__device__ __forceinline__ uint32_t slice4(const uint32_t* T, uint32_t a)
{
    return tb(T, 3, a & 0xff) ^ tb(T, 2, (a >> 8) & 0xff) ^ tb(T, 1, (a >> 16) & 0xff) ^ tb(T, 0, a >> 24);
}

// raw CRC of a lane's B bytes (w: B / 4 LE dwords, w0 replacing w[0])
template <int B>
__device__ __forceinline__ uint32_t lane_crc(const uint32_t* T, uint32_t w0, const uint32_t* w)
{
    uint32_t c = slice16(T, w0, w[1], w[2], w[3]);
    if constexpr (B == 20)
        return slice4(T, w[4] ^ c);
    else
        return slice16(T, w[4] ^ c, w[5], w[6], w[7]);
}

// c * x^(8 B (63 - col)) mod P: eight nibble lookups in column `col`
__device__ __forceinline__ uint32_t carry_to_end(const uint32_t* T, uint32_t c, uint32_t col)
{
    const uint32_t* nb = T + kNibBase + col;
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        r ^= nb[(i * 16 + ((c >> (4 * i)) & 15u)) * kWave];
    return r;
}

// DPP controls (GFX9): quad_perm [1,0,3,2], [2,3,0,1]; row_ror 4, 8
constexpr int kDppQuadSwap1 = 0xB1, kDppQuadSwap2 = 0x4E, kDppRowRor4 = 0x124, kDppRowRor8 = 0x128,
              kDppRowRor15 = 0x12F; // row_ror:15: lane i of a 16-lane row reads lane (i + 1) mod 16
__device__ __forceinline__ uint32_t dpp(uint32_t v, int ctrl)
{
    switch (ctrl) { // the builtin needs a constant
    case kDppQuadSwap1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppQuadSwap1, 0xF, 0xF, false);
    case kDppQuadSwap2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppQuadSwap2, 0xF, 0xF, false);
    case kDppRowRor4: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppRowRor4, 0xF, 0xF, false);
    case kDppRowRor15: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppRowRor15, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppRowRor8, 0xF, 0xF, false);
    }
}

// XOR of v over the wave (wave-uniform result): a 16-lane row reduction with
// DPP (every lane of a row ends up with the row's XOR), then the four rows
// through readlane.  Every lane must be active.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
    v ^= dpp(v, kDppQuadSwap1);
    v ^= dpp(v, kDppQuadSwap2);
    v ^= dpp(v, kDppRowRor4);
    v ^= dpp(v, kDppRowRor8);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// crc32(seed, msg[0:n)) (cf_crc32.c:56-68) of a message held lane-wise:
// lane j has bytes [B j, B j + B) in w (LE dwords), bytes >= n zero; n <= 64 B.
template <int B>
__device__ __forceinline__ uint32_t wave_crc32(const uint32_t* T, const uint32_t* w, uint32_t n, uint32_t seed, uint32_t lane)
{
    if (n < 4) { // too short to fold the initial register into: bytewise
        uint32_t r = ~seed;
        for (uint32_t i = 0; i < n; ++i)
            r = tb(T, 0, (r ^ (w[0] >> (8 * i))) & 0xffu) ^ (r >> 8);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)~r);
    }
    const uint32_t D = (uint32_t)(kWave * B) - n, q = D / B, rr = D - q * B;
    // initial register folded into message bytes 0-3
    const uint32_t c = lane_crc<B>(T, w[0] ^ (lane == 0 ? ~seed : 0u), w);
    // lanes past the message hold zeros (c == 0): their column is clamped
    const uint32_t R = wave_xor(carry_to_end(T, c, min(lane + q, (uint32_t)kWave - 1u)));
    // R = crc register * x^(8 rr): bit i of R times x^(31-i-8rr), summed
    const uint32_t b = lane < 32 && ((R >> (lane & 31u)) & 1u) ? T[kInvBase + rr * 32 + (lane & 31u)] : 0u;
    return ~wave_xor(b);
}

__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

// Buffer descriptor over `bytes` bytes at p (wave-uniform inputs made
// provably uniform): loads outside [0, bytes) return 0 without a branch.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    void* q = reinterpret_cast<void*>((uint64_t)hi << 32 | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)__builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
// Wave priority (s_setprio 3, measured against the other placements in round
// 2): the frame kernels raise it over finish_frame (the CRC,
// the trailer, the store staging), the parse over its payload store and over
// the batch header pass; each raise is dropped again before the next phase.
constexpr int kAuxNT = 2; // gfx950 cache-policy bits: nt
constexpr int kAuxST = kAuxNT; // datagram / payload stores: non-temporal

// A lane window of NX dwords at byte offset `off` (a multiple of 4, may be
// negative) of a range of `bytes` at base; dwords outside the range read as
// 0.  16-byte loads plus a tail at dword-aligned offsets.  An access whose
// offset is negative wraps past the range and reads 0 as a whole, so the
// one lane of the frame kernels whose first 16-byte load would start less
// than 16 bytes before the slot (FIX_LANE, S dwords before it) loads from 0
// instead and win_dwords shifts its window back by S dwords.
template <int NX>
struct Win {
    uint32_t c[NX];
};

template <int NX>
__device__ __forceinline__ void load_window(const uint8_t* base, uint32_t bytes, int off, Win<NX>& w)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
#pragma unroll
    for (int k = 0; k + 4 <= NX; k += 4) {
        const v4u v = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(off + 4 * k), 0, kAuxNT));
        w.c[k] = v[0], w.c[k + 1] = v[1], w.c[k + 2] = v[2], w.c[k + 3] = v[3];
    }
    constexpr int k = NX & ~3;
    if constexpr (NX - k == 3) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (uint32_t)(off + 4 * k), 0, kAuxNT);
        w.c[k] = v[0], w.c[k + 1] = v[1], w.c[k + 2] = v[2];
    } else if constexpr (NX - k == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)(off + 4 * k), 0, kAuxNT);
        w.c[k] = v[0], w.c[k + 1] = v[1];
    } else if constexpr (NX - k == 1) {
        w.c[k] = __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)(off + 4 * k), 0, kAuxNT);
    }
}

// lane windows at B j - SRC: the lane whose offset lies in (-16, 0) and is
// not a multiple of 16 (-1 when none), and how many dwords before 0 it starts
template <int B, int SRC>
constexpr int fix_lane()
{
    for (int l = 0; l < 4; ++l) {
        const int o = B * l - SRC;
        if (o > -16 && o < 0 && o % 16 != 0)
            return l;
    }
    return -1;
}
template <int B, int SRC>
__device__ __forceinline__ int win_offset(uint32_t lane)
{
    constexpr int FL = fix_lane<B, SRC>();
    const int off = B * (int)lane - SRC;
    if constexpr (FL >= 0)
        return lane == (uint32_t)FL ? 0 : off;
    else
        return off;
}
template <int B, int SRC, int NX>
__device__ __forceinline__ void win_dwords(const Win<NX>& w, uint32_t lane, uint32_t (&x)[NX])
{
    constexpr int FL = fix_lane<B, SRC>();
    constexpr int S = FL >= 0 ? (SRC - B * FL) / 4 : 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        if constexpr (FL >= 0)
            x[i] = lane == (uint32_t)FL ? (i >= S ? w.c[i - S] : 0u) : w.c[i];
        else
            x[i] = w.c[i];
    }
}

// out[k] = dword k of the window x shifted down by SH bytes (k < ND)
template <int ND, int SH, int NX>
__device__ __forceinline__ void funnel(const uint32_t (&x)[NX], uint32_t* out)
{
    static_assert((SH >> 2) + ND + ((SH & 3) ? 1 : 0) <= NX, "window too short");
#pragma unroll
    for (int k = 0; k < ND; ++k)
        out[k] = (SH & 3) ? __builtin_amdgcn_alignbyte(x[(SH >> 2) + k + 1], x[(SH >> 2) + k], SH & 3)
                          : x[(SH >> 2) + k];
}

// Mask of dword k of lane `lane` for a message of nb bytes held lane-wise
// (lane j = bytes [B j, B j + B)): the byte position of nb is wave-uniform, so
// per lane this is two selects of uniform values.
template <int B>
__device__ __forceinline__ uint32_t len_mask(int k, uint32_t lane, uint32_t nb)
{
    constexpr uint32_t ND = B / 4;
    const uint32_t qd = nb >> 2, s = nb & 3u, lq = qd / ND, kq = qd - lq * ND;
    const uint32_t ck = (uint32_t)k < kq ? ~0u : ((uint32_t)k == kq ? (s ? (1u << (8 * s)) - 1u : 0u) : 0u);
    return lane < lq ? ~0u : (lane == lq ? ck : 0u);
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a lane's B bytes (B = 32) to [B lane, B lane + B) of a slot of slot_bytes:
// 16-byte stores range-checked by the buffer descriptor (nothing lands past
// the slot)
template <int B>
__device__ __forceinline__ void store_slot(uint8_t* __restrict__ slot, uint32_t slot_bytes, uint32_t lane,
                                           const uint32_t* w)
{
    static_assert(B % 16 == 0, "whole 16-byte stores");
    const __amdgpu_buffer_rsrc_t r = rsrc(slot, slot_bytes);
#pragma unroll
    for (int k = 0; k + 4 <= B / 4; k += 4)
        __builtin_amdgcn_raw_buffer_store_b128(v4u{w[k], w[k + 1], w[k + 2], w[k + 3]}, r, B * lane + 4 * k, 0, kAuxST);
}

// Header bytes at compile-time positions (big-endian fields, cf_stream.c:366-385)
struct Hdr {
    uint32_t h[12];
};
template <int POS, int NB>
__device__ __forceinline__ void put(Hdr& b, uint32_t v)
{
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int p = POS + i;
        b.h[p >> 2] |= ((v >> (8 * (NB - 1 - i))) & 0xffu) << (8 * (p & 3));
    }
}

// Datagram of header H (bytes [0, hsize), zero beyond) and payload `pay`
// (zero below hsize): mask at n = hsize + L, CRC32 BE at [n, n+4), store.
template <int B>
__device__ __forceinline__ void finish_frame(const uint32_t* T, const Hdr& H, uint32_t n, const uint32_t* pay,
                                             uint32_t lane, uint8_t* __restrict__ slot, uint32_t dstride,
                                             uint16_t* dlen_out)
{
    __builtin_amdgcn_s_setprio(3);
    constexpr int ND = B / 4;
    uint32_t w[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) {
        // header dword i (hsize <= 48: i < 12) lives in lane i / ND
        uint32_t hd = 0;
#pragma unroll
        for (int L = 0; L * ND < 12; ++L)
            if (L * ND + k < 12)
                hd = lane == (uint32_t)L ? H.h[L * ND + k] : hd;
        w[k] = (pay[k] | hd) & len_mask<B>(k, lane, n);
    }
    const uint32_t crc = wave_crc32<B>(T, w, n, RFEC_WIRE_CRC_SEED, lane);
    // big-endian trailer at byte n: its first 4 - s bytes end dword n / 4, the
    // rest start the next one (both positions wave-uniform)
    const uint32_t be = bswap(crc), s = n & 3u, q0 = n >> 2, q1 = q0 + 1;
    const uint32_t lo = be << (8 * s), hi = s ? be >> (32 - 8 * s) : 0u;
    const uint32_t l0 = q0 / ND, k0 = q0 - l0 * ND, l1 = q1 / ND, k1 = q1 - l1 * ND;
#pragma unroll
    for (int k = 0; k < ND; ++k) {
        if ((uint32_t)k == k0)
            w[k] |= lane == l0 ? lo : 0u;
        if ((uint32_t)k == k1)
            w[k] |= lane == l1 ? hi : 0u;
    }
    store_slot<B>(slot, dstride, lane, w);
    if (lane == 0)
        *dlen_out = (uint16_t)(n + 4);
    __builtin_amdgcn_s_setprio(0);
}

template <int B>
__device__ __forceinline__ void zero_slot(uint8_t* __restrict__ slot, uint32_t dstride, uint32_t lane,
                                          uint16_t* dlen_out)
{
    const uint32_t z[B / 4] = {};
    store_slot<B>(slot, dstride, lane, z);
    if (lane == 0)
        *dlen_out = 0;
}

__device__ __forceinline__ uint32_t wave_id()
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
}

// ---------------------------------------------------------------------------
// Framing.  Persistent waves walk datagrams d, d + nw, ...; everything the
// next datagram needs from memory (its payload window and, one dword per
// lane, its header fields) is loaded before the current one is processed, so
// no load inside an iteration waits behind the prefetch (vmcnt is in order).
// Lane j's window starts 48 (FEC) / 32 (SEG) bytes before its output bytes'
// source, so the window does not depend on the per-datagram header size.
// ---------------------------------------------------------------------------

// dword k of the prefetched per-datagram fields (wave-uniform)
__device__ __forceinline__ uint32_t fld(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }

// SIM_FEC fields, one dword per lane: 0-5 rfec_fec_stamp, 6-10 fec_meta,
// 11 fec_data_size, 12 status (sign-extended; 0 when status is NULL)
__device__ __forceinline__ uint32_t load_fec_fields(const rfec_fec_stamp* __restrict__ stamps,
                                                    const rfec_hdr* __restrict__ meta,
                                                    const uint16_t* __restrict__ fsize,
                                                    const int8_t* __restrict__ status, uint32_t d, uint32_t lane)
{
    // four loads, each in range for its own lanes only (the rest read 0)
    const uint32_t s = __builtin_amdgcn_raw_buffer_load_b32(rsrc(stamps + d, 24), 4u * lane, 0, kAuxNT);
    const uint32_t m = __builtin_amdgcn_raw_buffer_load_b32(rsrc(meta + d, 20), 4u * (lane - 6u), 0, kAuxNT);
    const uint32_t f = __builtin_amdgcn_raw_buffer_load_b16(rsrc(fsize + d, 2), 2u * (lane - 11u), 0, kAuxNT);
    const uint32_t t = __builtin_amdgcn_raw_buffer_load_b8(rsrc(status ? status + d : status, status ? 1u : 0u),
                                                           lane - 12u, 0, kAuxNT);
    return s | m | f | (uint32_t)(int32_t)(int8_t)t;
}

// SIM_SEG fields: 0-4 rfec_hdr, 5-7 rfec_seg_stamp
__device__ __forceinline__ uint32_t load_seg_fields(const rfec_hdr* __restrict__ hdr,
                                                    const rfec_seg_stamp* __restrict__ stamps, uint32_t d,
                                                    uint32_t lane)
{
    const uint32_t h = __builtin_amdgcn_raw_buffer_load_b32(rsrc(hdr + d, 20), 4u * lane, 0, kAuxNT);
    const uint32_t s = __builtin_amdgcn_raw_buffer_load_b32(rsrc(stamps + d, 12), 4u * (lane - 5u), 0, kAuxNT);
    return h | s;
}

// Ping-pong software pipeline over datagrams d0, d0 + nw, ...: the loads of
// datagram i+1 go into the other buffer before datagram i is processed, and
// no register copy ever waits on them (vmcnt is an in-order counter).
template <class Pre, class Load, class Proc>
__device__ __forceinline__ void ping_pong(uint32_t d, uint32_t count, uint32_t nw, Load load, Proc proc)
{
    Pre a, b;
    load(d, a);
    for (;;) {
        // past the end the last datagram is loaded again (branch-free prefetch)
        const uint32_t d1 = d + nw;
        load(min(d1, count - 1), b);
        proc(a, d);
        if (d1 >= count)
            break;
        const uint32_t d2 = d1 + nw;
        load(min(d2, count - 1), a);
        proc(b, d1);
        if (d2 >= count)
            break;
        d = d2;
    }
}

// Three-deep form: two datagrams' loads in flight while one is processed
// (the frame kernels' staged chunks are 8 dwords, so a third buffer fits the
// register budget of 8 waves per SIMD).
template <class W>
struct Pre {
    W w;        // payload: a lane window (Win) or aligned chunks (Chunks)
    uint32_t f; // per-datagram fields, one dword per lane
};

template <bool C, class A, class B_>
struct Sel {
    using T = A;
};
template <class A, class B_>
struct Sel<false, A, B_> {
    using T = B_;
};

// 20-byte lanes (the parse), staged: the slot's first 1,280 bytes as aligned
// 16-byte chunks (chunk j in lane j, chunk 64 + j in lane j < 16), coalesced
// 1 KiB loads, then through the wave's LDS buffer.
struct Chunks {
    v4u c0, c1;
};

__device__ __forceinline__ void load_chunks(const uint8_t* base, uint32_t bytes, uint32_t lane, Chunks& ch)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    ch.c0 = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, 16u * lane, 0, kAuxNT));
    ch.c1 = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, 1024u + 16u * (lane & 15u), 0, kAuxNT));
}

constexpr int kWaveBuf = 336; // dwords per wave: 48 + 1,280 bytes staged, or 1,280 stored


// Lane j's window starts 48 (FEC) / 32 (SEG) bytes before the source of its
// output bytes [B j, B j + B), so it does not depend on the header size.

// SIM_FEC: 45-byte header (sim_proto.c:13-18, sim_proto.inl:244-254, 270-283)
template <int B>
__global__ __launch_bounds__(kBlock) void k_frame_fec(const uint8_t* __restrict__ parity,
                                                      const rfec_hdr* __restrict__ meta,
                                                      const uint16_t* __restrict__ fsize,
                                                      const int8_t* __restrict__ status,
                                                      const rfec_fec_stamp* __restrict__ stamps,
                                                      const uint32_t* __restrict__ order,
                                                      uint8_t* __restrict__ dgram, uint16_t* __restrict__ dlen,
                                                      uint32_t count, uint32_t stride, uint32_t capacity,
                                                      uint32_t dstride)
{
    constexpr int ND = B / 4;
    static_assert(B == 32, "slots up to 1,280 bytes take k_frame_fec_q");
    __shared__ __attribute__((aligned(16))) uint32_t T[kTabDwords<B>];
    load_tables<B>(T);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t range = (capacity + 15u) & ~15u;
    const int off = win_offset<B, 48>(lane);
    uint32_t d = wave_id();
    if (d >= count)
        return;
    using PW = Pre<Win<ND + 1>>;
    ping_pong<PW>(d, count, nw,
                              [&](uint32_t dd, PW& P) {
                                  P.f = load_fec_fields(stamps, meta, fsize, status, dd, lane);
                                  load_window<ND + 1>(parity + (size_t)dd * stride, range, off, P.w);
                              },
                              [&](const PW& P, uint32_t d) {
            const uint32_t o = order ? order[d] : d; // output slot
            uint8_t* slot = dgram + (size_t)o * dstride;
            const uint32_t L = fld(P.f, 11);
            const int st = (int)fld(P.f, 12);
            if (st < 0 || L > capacity) {
                zero_slot<B>(slot, dstride, lane, dlen + o);
            } else {
                const uint32_t s3 = fld(P.f, 3), s4 = fld(P.f, 4), s5 = fld(P.f, 5);
                const uint32_t m3 = fld(P.f, 9), m4 = fld(P.f, 10);
                Hdr H = {};
                put<0, 1>(H, RFEC_WIRE_VER);
                put<1, 1>(H, RFEC_WIRE_FEC);
                put<2, 4>(H, fld(P.f, 0));     // uid
                put<6, 2>(H, s3 & 0xffffu);     // fec_id
                put<8, 1>(H, (s4 >> 16) & 0xffu); // row
                put<9, 1>(H, s4 >> 24);         // col
                put<10, 1>(H, s5 & 0xffu);      // index
                put<11, 2>(H, s3 >> 16);        // count
                put<13, 4>(H, fld(P.f, 1));    // base_id
                put<17, 2>(H, s4 & 0xffffu);    // transport_seq
                put<19, 4>(H, fld(P.f, 2));    // send_ts
                put<23, 4>(H, fld(P.f, 6));    // fec_meta: seq, fid, ts, index, total, ftype, payload_type, size
                put<27, 4>(H, fld(P.f, 7));
                put<31, 4>(H, fld(P.f, 8));
                put<35, 2>(H, m3 & 0xffffu);
                put<37, 2>(H, m3 >> 16);
                put<39, 1>(H, m4 & 0xffu);
                put<40, 1>(H, (m4 >> 8) & 0xffu);
                put<41, 2>(H, m4 >> 16);
                put<43, 2>(H, L); // mach_data_write length (cf_stream.c:328-337)
                uint32_t pay[ND], x[ND + 1];
                win_dwords<B, 48>(P.w, lane, x);
                funnel<ND, 3>(x, pay); // window [B j - 48, ...) -> bytes [B j - 45, ...)
                finish_frame<B>(T, H, 45 + L, pay, lane, slot, dstride, dlen + o);
            }
                              });
}

// SIM_SEG header, one of 8 layouts (sim_proto.inl:83-125): PW / FW = 4-byte
// packet_id / fid, TW = 2-byte index and total.  Returns the header size.
template <bool PW, bool FW, bool TW>
__device__ __forceinline__ uint32_t seg_header(Hdr& H, const rfec_hdr& h, const rfec_seg_stamp& s)
{
    constexpr int P1 = 8 + (PW ? 4 : 2);  // after packet_id
    constexpr int P2 = P1 + (FW ? 4 : 2); // after fid
    constexpr int P3 = P2 + 4;            // after timestamp
    constexpr int P4 = P3 + (TW ? 4 : 2); // after index, total
    const uint32_t mask = (h.ftype & 1u) | (PW ? 0x80u : 0u) | (FW ? 0x40u : 0u) | (TW ? 0x20u : 0u) |
                          (s.remb == 0 ? 0x10u : 0u);
    put<0, 1>(H, RFEC_WIRE_VER);
    put<1, 1>(H, RFEC_WIRE_SEG);
    put<2, 4>(H, s.uid);
    put<6, 1>(H, mask);
    put<7, 1>(H, h.payload_type);
    put<8, PW ? 4 : 2>(H, h.seq);
    put<P1, FW ? 4 : 2>(H, h.fid);
    put<P2, 4>(H, h.ts);
    if constexpr (TW) {
        put<P3, 2>(H, h.index);
        put<P3 + 2, 2>(H, h.total);
    } else {
        put<P3, 1>(H, h.index);
        put<P3 + 1, 1>(H, h.total);
    }
    put<P4, 2>(H, s.fec_id);
    put<P4 + 2, 2>(H, s.send_ts);
    put<P4 + 4, 2>(H, s.transport_seq);
    put<P4 + 6, 2>(H, h.size);
    return P4 + 8;
}

template <int B>
__global__ __launch_bounds__(kBlock) void k_frame_seg(const uint8_t* __restrict__ shards,
                                                      const rfec_hdr* __restrict__ hdr,
                                                      const rfec_seg_stamp* __restrict__ stamps,
                                                      const uint32_t* __restrict__ order,
                                                      uint8_t* __restrict__ dgram, uint16_t* __restrict__ dlen,
                                                      uint32_t count, uint32_t stride, uint32_t capacity,
                                                      uint32_t dstride, uint32_t rows_out)
{
    constexpr int ND = B / 4;
    static_assert(B == 32, "slots up to 1,280 bytes take k_frame_seg_q");
    __shared__ __attribute__((aligned(16))) uint32_t T[kTabDwords<B>];
    load_tables<B>(T);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t range = (capacity + 15u) & ~15u;
    const int off = win_offset<B, 32>(lane); // header sizes 26..32
    uint32_t d = wave_id();
    if (d >= count)
        return;
    using PW = Pre<Win<ND + 2>>;
    ping_pong<PW>(d, count, nw,
                              [&](uint32_t dd, PW& P) {
                                  P.f = load_seg_fields(hdr, stamps, dd, lane);
                                  load_window<ND + 2>(shards + (size_t)dd * stride, range, off, P.w);
                              },
                              [&](const PW& P, uint32_t d) {
            const uint32_t o = order ? order[d] : d; // output slot
            if (o >= rows_out) // (a row the caller's output does not hold: not framed)
                return;
            uint8_t* slot = dgram + (size_t)o * dstride;
            rfec_hdr h;
            {
                const uint32_t h3 = fld(P.f, 3), h4 = fld(P.f, 4);
                h.seq = fld(P.f, 0);
                h.fid = fld(P.f, 1);
                h.ts = fld(P.f, 2);
                h.index = (uint16_t)h3;
                h.total = (uint16_t)(h3 >> 16);
                h.ftype = (uint8_t)h4;
                h.payload_type = (uint8_t)(h4 >> 8);
                h.size = (uint16_t)(h4 >> 16);
            }
            const uint32_t L = h.size;
            if (L > capacity) {
                zero_slot<B>(slot, dstride, lane, dlen + o);
            } else {
                rfec_seg_stamp s;
                {
                    const uint32_t s1 = fld(P.f, 6), s2 = fld(P.f, 7);
                    s.uid = fld(P.f, 5);
                    s.fec_id = (uint16_t)s1;
                    s.send_ts = (uint16_t)(s1 >> 16);
                    s.transport_seq = (uint16_t)s2;
                    s.remb = (uint8_t)(s2 >> 16);
                    s.reserved = 0;
                }
                Hdr H = {};
                const uint32_t layout = (h.seq > 65535u ? 4u : 0u) | (h.fid > 65535u ? 2u : 0u) |
                                        (h.total > 255u ? 1u : 0u);
                uint32_t hs, pay[ND], x[ND + 2];
                win_dwords<B, 32>(P.w, lane, x);
                // window [B j - 32, ...) shifted by 32 - hs bytes
                switch (layout) {
                case 0: hs = seg_header<false, false, false>(H, h, s); funnel<ND, 6>(x, pay); break;
                case 1: hs = seg_header<false, false, true>(H, h, s); funnel<ND, 4>(x, pay); break;
                case 2: hs = seg_header<false, true, false>(H, h, s); funnel<ND, 4>(x, pay); break;
                case 3: hs = seg_header<false, true, true>(H, h, s); funnel<ND, 2>(x, pay); break;
                case 4: hs = seg_header<true, false, false>(H, h, s); funnel<ND, 4>(x, pay); break;
                case 5: hs = seg_header<true, false, true>(H, h, s); funnel<ND, 2>(x, pay); break;
                case 6: hs = seg_header<true, true, false>(H, h, s); funnel<ND, 2>(x, pay); break;
                default: hs = seg_header<true, true, true>(H, h, s); funnel<ND, 0>(x, pay); break;
                }
                finish_frame<B>(T, H, hs + L, pay, lane, slot, dstride, dlen + o);
            }
                              });
}

// ---------------------------------------------------------------------------
// Parse (receive side)
//
// Two passes per batch of up to 64 of a wave's datagrams d_i = base + i nw:
//   1. headers, one datagram per LANE: lane i reads the first 48 bytes of d_i
//      and its length, decodes the header (sim_proto.inl:127-179 / 287-307)
//      as if the CRC were good, writes recs[d_i] and keeps one packed dword
//      (length, data position, data size) for pass 2.  The per-datagram
//      scalar work of a wave-per-datagram header decode is done once per 64.
//   2. one datagram per WAVE, as the frame kernels: CRC over the lane-wise
//      datagram against its trailer; a mismatch rewrites the record as
//      EBADCRC; the payload slot gets the data bytes (zero when the CRC failed
//      or there are none) and zeros to the slot's end.
// ---------------------------------------------------------------------------

// big-endian field at a compile-time byte position of header dwords H
template <int POS, int NB>
__device__ __forceinline__ uint32_t get(const uint32_t* H)
{
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i)
        v = (v << 8) | ((H[(POS + i) >> 2] >> (8 * ((POS + i) & 3))) & 0xffu);
    return v;
}

// field at a per-lane position pos in {P, P + 2, ..., HI}
template <int P, int HI, int NB>
__device__ __forceinline__ uint32_t get_at(const uint32_t* H, uint32_t pos)
{
    if constexpr (P >= HI)
        return get<P, NB>(H);
    else
        return pos == (uint32_t)P ? get<P, NB>(H) : get_at<P + 2, HI, NB>(H, pos);
}

constexpr int kHdrDwords = 12; // 48 bytes: the longest header read, SIM_FEC's, ends at byte 47

// byte p (< 48, per lane) of the header dwords
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&H)[kHdrDwords], uint32_t p)
{
    // the dwords pass an empty asm first: a select chain over plain loads of H
    // is folded into one indexed load, which puts the header array in scratch
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kHdrDwords; ++k) {
        uint32_t h = H[k];
        __asm__("" : "+v"(h));
        v = (p >> 2) == (uint32_t)k ? h : v;
    }
    return (v >> (8 * (p & 3u))) & 0xffu;
}

// bin_stream reader of one lane's datagram (cf_stream.c mach_*_read): a read
// past `used` yields 0 and does not advance.  Only for datagrams too short
// for their header; the rest take fixed offsets.
struct LaneCursor {
    const uint32_t (&H)[kHdrDwords];
    uint32_t used, pos;
    __device__ uint32_t rd(uint32_t nb)
    {
        if (used < pos + nb)
            return 0;
        uint32_t v = 0;
        for (uint32_t i = 0; i < nb; ++i)
            v = (v << 8) | byte_at(H, pos + i);
        pos += nb;
        return v;
    }
};

// pass-2 facts of a datagram, one dword: bit 31 length in range (the CRC is
// checked), bits 0-11 length, 12-17 data position + 1 (0: no data), 18-29
// data size
constexpr uint32_t kPkValid = 1u << 31;

// Header decode of one lane's datagram (length len, first bytes H) as if its
// CRC matched: sim_decode_header (sim_proto.c:21-37) past the CRC,
// sim_session.c:594 (mid range), sim_segment_decode (sim_proto.inl:127-179),
// sim_fec_decode (:287-307), mach_data_read (cf_stream.c:339-355).
__device__ __forceinline__ uint32_t decode_lane(const uint32_t (&H)[kHdrDwords], uint32_t len, uint32_t capacity,
                                                rfec_wire_rec& rec)
{
    rec = rfec_wire_rec{};
    rec.status = RFEC_WIRE_EBADCRC;
    if (!(len >= 4)) // shorter than the trailer
        return 0;
    rec.ver = (uint8_t)get<0, 1>(H);
    rec.mid = (uint8_t)get<1, 1>(H);
    const uint32_t mid = rec.mid;
    const uint32_t smask = get<6, 1>(H);
    const uint32_t seg_hl = 26u + ((smask & 0x80u) ? 2u : 0u) + ((smask & 0x40u) ? 2u : 0u) +
                            ((smask & 0x20u) ? 2u : 0u); // through the data length field
    const bool fast = len >= 6 && ((mid == RFEC_WIRE_FEC && len >= 45) || (mid == RFEC_WIRE_SEG && len >= seg_hl) ||
                                   (mid != RFEC_WIRE_FEC && mid != RFEC_WIRE_SEG));
    uint32_t npos = 0, nval = 0;
    if (fast) {
        rec.uid = get<2, 4>(H);
        if (mid < RFEC_WIRE_MIN_MID || mid > RFEC_WIRE_MAX_MID) {
            rec.status = RFEC_WIRE_EMID;
        } else if (mid == RFEC_WIRE_SEG) {
            const bool pw = smask & 0x80u, fw = smask & 0x40u, tw = smask & 0x20u;
            const uint32_t p1 = pw ? 12u : 10u, p2 = p1 + (fw ? 4u : 2u), p3 = p2 + 4u, p4 = p3 + (tw ? 4u : 2u);
            rec.hdr.payload_type = (uint8_t)get<7, 1>(H);
            rec.hdr.ftype = (uint8_t)(smask & 1u);
            rec.remb = (smask & 0x10u) ? 0 : 0xff;
            rec.hdr.seq = pw ? get<8, 4>(H) : get<8, 2>(H);
            rec.hdr.fid = fw ? get_at<10, 12, 4>(H, p1) : get_at<10, 12, 2>(H, p1);
            rec.hdr.ts = get_at<12, 16, 4>(H, p2);
            rec.hdr.index = (uint16_t)(tw ? get_at<16, 20, 2>(H, p3) : get_at<16, 20, 1>(H, p3));
            rec.hdr.total = (uint16_t)(tw ? get_at<18, 22, 2>(H, p3 + 2) : get_at<17, 21, 1>(H, p3 + 1));
            rec.fec_id = (uint16_t)get_at<18, 24, 2>(H, p4);
            rec.send_ts = get_at<20, 26, 2>(H, p4 + 2);
            rec.transport_seq = (uint16_t)get_at<22, 28, 2>(H, p4 + 4);
            nval = get_at<24, 30, 2>(H, p4 + 6);
            npos = p4 + 8;
            rec.status = RFEC_WIRE_OK;
        } else if (mid == RFEC_WIRE_FEC) {
            rec.fec_id = (uint16_t)get<6, 2>(H);
            rec.row = (uint8_t)get<8, 1>(H);
            rec.col = (uint8_t)get<9, 1>(H);
            rec.index = (uint8_t)get<10, 1>(H);
            rec.count = (uint16_t)get<11, 2>(H);
            rec.base_id = get<13, 4>(H);
            rec.transport_seq = (uint16_t)get<17, 2>(H);
            rec.send_ts = get<19, 4>(H);
            rec.hdr.seq = get<23, 4>(H);
            rec.hdr.fid = get<27, 4>(H);
            rec.hdr.ts = get<31, 4>(H);
            rec.hdr.index = (uint16_t)get<35, 2>(H);
            rec.hdr.total = (uint16_t)get<37, 2>(H);
            rec.hdr.ftype = (uint8_t)get<39, 1>(H);
            rec.hdr.payload_type = (uint8_t)get<40, 1>(H);
            rec.hdr.size = (uint16_t)get<41, 2>(H);
            nval = get<43, 2>(H);
            npos = 45;
            rec.status = RFEC_WIRE_OK;
        } else {
            rec.status = RFEC_WIRE_OTHER;
        }
    } else { // truncated header
        LaneCursor c{H, len, 2};
        rec.uid = c.rd(4);
        if (mid < RFEC_WIRE_MIN_MID || mid > RFEC_WIRE_MAX_MID) {
            rec.status = RFEC_WIRE_EMID;
        } else if (mid == RFEC_WIRE_SEG) {
            const uint32_t mk = c.rd(1);
            rec.hdr.payload_type = (uint8_t)c.rd(1);
            rec.hdr.ftype = (uint8_t)(mk & 1u);
            rec.hdr.seq = c.rd((mk & 0x80u) ? 4 : 2);
            rec.hdr.fid = c.rd((mk & 0x40u) ? 4 : 2);
            rec.hdr.ts = c.rd(4);
            rec.hdr.index = (uint16_t)c.rd((mk & 0x20u) ? 2 : 1);
            rec.hdr.total = (uint16_t)c.rd((mk & 0x20u) ? 2 : 1);
            rec.remb = (mk & 0x10u) ? 0 : 0xff;
            rec.fec_id = (uint16_t)c.rd(2);
            rec.send_ts = c.rd(2);
            rec.transport_seq = (uint16_t)c.rd(2);
            nval = c.rd(2);
            npos = c.pos;
            rec.status = RFEC_WIRE_OK;
        } else if (mid == RFEC_WIRE_FEC) {
            rec.fec_id = (uint16_t)c.rd(2);
            rec.row = (uint8_t)c.rd(1);
            rec.col = (uint8_t)c.rd(1);
            rec.index = (uint8_t)c.rd(1);
            rec.count = (uint16_t)c.rd(2);
            rec.base_id = c.rd(4);
            rec.transport_seq = (uint16_t)c.rd(2);
            rec.send_ts = c.rd(4);
            rec.hdr.seq = c.rd(4);
            rec.hdr.fid = c.rd(4);
            rec.hdr.ts = c.rd(4);
            rec.hdr.index = (uint16_t)c.rd(2);
            rec.hdr.total = (uint16_t)c.rd(2);
            rec.hdr.ftype = (uint8_t)c.rd(1);
            rec.hdr.payload_type = (uint8_t)c.rd(1);
            rec.hdr.size = (uint16_t)c.rd(2);
            nval = c.rd(2);
            npos = c.pos;
            rec.status = RFEC_WIRE_OK;
        } else {
            rec.status = RFEC_WIRE_OTHER;
        }
    }
    // mach_data_read, cf_stream.c:339-355
    const bool data_ok = nval <= capacity && npos + nval <= len;
    uint32_t dsize = 0, at1 = 0;
    if (mid == RFEC_WIRE_SEG && rec.status == RFEC_WIRE_OK) {
        dsize = data_ok ? nval : 0u; // a bad length decodes as size 0 (sim_proto.inl:174-176)
        at1 = data_ok ? npos + 1u : 0u;
        rec.hdr.size = (uint16_t)dsize;
    } else if (mid == RFEC_WIRE_FEC && rec.status == RFEC_WIRE_OK) {
        if (data_ok) {
            dsize = nval;
            at1 = npos + 1u;
        } else {
            rec.status = RFEC_WIRE_EBODY; // sim_proto.inl:301-305
        }
    }
    rec.data_size = (uint16_t)dsize;
    return kPkValid | len | at1 << 12 | dsize << 18;
}

// pass 1, split so its loads can be issued ahead of the next datagram's:
// lane `lane` of the batch reads datagram d's length and first 48 bytes
// (when active), then decodes them and writes recs[d]
struct HdrIn {
    uint32_t H[kHdrDwords];
    uint32_t len;
};

__device__ __forceinline__ void load_header(const uint8_t* __restrict__ dgram, const uint16_t* __restrict__ dlen,
                                            uint32_t d, bool active, uint32_t dstride, HdrIn& in)
{
    in.len = 0;
    for (int k = 0; k < kHdrDwords; ++k)
        in.H[k] = 0;
    if (!active)
        return;
    in.len = dlen[d];
    // dstride >= 64: the 48 bytes lie in the slot
    const v4u* src = reinterpret_cast<const v4u*>(dgram + (size_t)d * dstride);
#pragma unroll
    for (int t = 0; t < kHdrDwords / 4; ++t) {
        const v4u v = src[t];
        in.H[4 * t] = v[0], in.H[4 * t + 1] = v[1], in.H[4 * t + 2] = v[2], in.H[4 * t + 3] = v[3];
    }
}

// the receiver session's split entry of a record (rfec_rx.c; k_rx_split's rules, rfec_kernels.hip)
__device__ __forceinline__ void split_entry(const rfec_wire_rec& rec, uint32_t T, rfec_rx_split* __restrict__ out)
{
    uint32_t shard = 0xFFu, kind = RX_SPLIT_NONE, value = 0;
    if (rec.status == RFEC_WIRE_OK && rec.mid == RFEC_WIRE_SEG) {
        shard = (rec.fec_id ? rec.fec_id : rec.hdr.seq) % T;
        kind = rec.fec_id && rec.hdr.seq ? RX_SPLIT_SEG_TS : RX_SPLIT_SEG;
        value = rec.hdr.ts;
    } else if (rec.status == RFEC_WIRE_OK && rec.mid == RFEC_WIRE_FEC) {
        shard = rec.fec_id % T;
        kind = RX_SPLIT_FEC;
        value = rec.send_ts + 3000u;
    }
    *reinterpret_cast<uint2*>(out) = uint2{shard | kind << 8, value};
}

template <int B>
__device__ __forceinline__ uint32_t decode_header(const HdrIn& in, rfec_wire_rec* __restrict__ recs, uint32_t d,
                                                  bool active, uint32_t dstride, uint32_t capacity,
                                                  rfec_rx_split* __restrict__ split = nullptr, uint32_t T = 1)
{
    if (!active)
        return 0;
    rfec_wire_rec rec;
    uint32_t pk = 0;
    if (in.len <= dstride && in.len <= (uint32_t)(kWave * B)) {
        pk = decode_lane(in.H, in.len, capacity, rec);
    } else {
        rec = rfec_wire_rec{};
        rec.status = RFEC_WIRE_EBADCRC;
    }
    const v4u* s = reinterpret_cast<const v4u*>(&rec);
    v4u* o = reinterpret_cast<v4u*>(recs + d);
#pragma unroll
    for (int t = 0; t < 4; ++t)
        o[t] = s[t]; // plain stores: the four 16-byte pieces merge in L2 (nontemporal ones measured slower)
    if (split) // (a CRC mismatch found later rewrites the entry)
        split_entry(rec, T, split + d);
    return pk;
}

// v of lane + 1 (0 in lane 63): DPP wave_shl:1, no LDS traffic
__device__ __forceinline__ uint32_t next_lane(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

// out lane j = datagram bytes [pos + B j, pos + B j + B) from the lane-wise
// datagram w (pos wave-uniform, <= 45: the data field of a SIM_FEC starts at
// byte 45, of a SIM_SEG at <= 34): lanes j + q and j + q + 1, q = pos / B,
// brought over with DPP, then a funnel by the uniform remainder
template <int B>
__device__ __forceinline__ void shift_down_bytes(const uint32_t* w, uint32_t pos, uint32_t* out)
{
    constexpr int ND = B / 4;
    constexpr int QMAX = 45 / B;
    const uint32_t q = pos / B, r = pos - q * B;
    uint32_t x[2 * ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) {
        uint32_t v = w[k];
#pragma unroll
        for (int t = 1; t <= QMAX; ++t) {
            const uint32_t nv = next_lane(v); // every lane active: computed, then selected
            v = q >= (uint32_t)t ? nv : v;
        }
        x[k] = v;
        x[ND + k] = next_lane(v);
    }
    const uint32_t rb = r & 3u;
#define RFEC_SHIFT(S)                                                                                              \
    _Pragma("unroll") for (int k = 0; k < ND; ++k) out[k] = __builtin_amdgcn_alignbyte(x[(S) + k + 1], x[(S) + k], rb);
    switch (r >> 2) {
    case 0: RFEC_SHIFT(0) break;
    case 1: RFEC_SHIFT(1) break;
    case 2: RFEC_SHIFT(2) break;
    case 3: RFEC_SHIFT(3) break;
    case 4: RFEC_SHIFT(4) break;
    case 5: if constexpr (ND > 5) { RFEC_SHIFT(5) } break;
    case 6: if constexpr (ND > 6) { RFEC_SHIFT(6) } break;
    default: if constexpr (ND > 7) { RFEC_SHIFT(7) } break;
    }
#undef RFEC_SHIFT
}

// dword k of w, k wave-uniform
template <int ND>
__device__ __forceinline__ uint32_t pick(const uint32_t* w, uint32_t k)
{
    uint32_t v = w[0];
#pragma unroll
    for (int i = 1; i < ND; ++i)
        v = k == (uint32_t)i ? w[i] : v;
    return v;
}

// bytes of a 16-byte output chunk past dsize zeroed: nb = valid bytes of the chunk (per lane)
__device__ __forceinline__ uint32_t keep_bytes(uint32_t v, int k, uint32_t nb)
{
    const uint32_t c = min(nb - min(nb, 4u * (uint32_t)k), 4u);
    return c == 4u ? v : v & ((1u << (8 * c)) - 1u);
}

// payload slot of `stride` bytes from the datagram staged in this wave's LDS
// buffer (dwords [0, 320)): bytes [at, at + dsize), zeros after.  Lane j
// writes 16-byte chunk j (then 64 + j): two aligned LDS reads of the source
// chunks it straddles, a funnel by the uniform remainder.
__device__ __forceinline__ void store_payload20(const uint32_t* wb, uint8_t* __restrict__ slot, uint32_t stride,
                                                uint32_t at, uint32_t dsize, uint32_t lane)
{
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = rsrc(slot, stride);
    const v4u* w4 = reinterpret_cast<const v4u*>(wb);
    const uint32_t a = at >> 4, rb = at & 3u;
    for (uint32_t o = 0; o < stride; o += 16 * kWave) {
        const uint32_t q = o / 16 + lane;
        const uint32_t nb = dsize > 16 * q ? dsize - 16 * q : 0u;
        uint32_t y[4] = {0, 0, 0, 0};
        if (dsize > o) { // wave-uniform: some lane has data bytes
            const v4u x0 = w4[min(a + q, (uint32_t)kWaveBuf / 4 - 2)];
            const v4u x1 = w4[min(a + q, (uint32_t)kWaveBuf / 4 - 2) + 1];
            const uint32_t x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#define RFEC_FUNNEL(S)                                                                                             \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) y[k] = __builtin_amdgcn_alignbyte(x[(S) + k + 1], x[(S) + k], rb);
            switch ((at >> 2) & 3u) {
            case 0: RFEC_FUNNEL(0) break;
            case 1: RFEC_FUNNEL(1) break;
            case 2: RFEC_FUNNEL(2) break;
            default: RFEC_FUNNEL(3) break;
            }
#undef RFEC_FUNNEL
            if (dsize < o + 16 * kWave) { // wave-uniform: the data ends in this round
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    y[k] = keep_bytes(y[k], k, nb);
            }
        }
        __builtin_amdgcn_raw_buffer_store_b128(u4{y[0], y[1], y[2], y[3]}, r, 16 * q, 0, kAuxST);
    }
}

// parse: 4 waves per SIMD (one 16-wave block per CU), registers for a
// three-deep datagram pipeline without spills (107 VGPRs).  At the 64-register
// cap of 8 waves the two-deep kernel spilled 39 VGPRs to scratch; 5 waves
// (96 registers, no spill) ran as fast as it, 6-7 waves (19-22 spills) slower;
// three deep at 4 waves: parse_seg 395-400 vs 404-410 us, parse_fec 120-124 vs
// 125-126 us; four or five deep: no further gain
// (profiles/r05/ab/parse_occupancy/).
constexpr int kParseWaves = 4;

template <int B>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kParseWaves))) void k_parse(const uint8_t* __restrict__ dgram,
                                                  const uint16_t* __restrict__ dlen,
                                                  rfec_wire_rec* __restrict__ recs, uint8_t* __restrict__ payload,
                                                  uint32_t n, uint32_t dstride, uint32_t stride, uint32_t capacity)
{
    constexpr int ND = B / 4;
    __shared__ __attribute__((aligned(16))) uint32_t T[kTabDwords<B>];
    // 20-byte lanes: the datagram comes in as aligned 16-byte chunks, staged
    // in this wave's LDS buffer; the lanes' windows, the trailer and the
    // payload's output chunks are read from there
    __shared__ __attribute__((aligned(16))) uint32_t WB[kWavesPerBlock][B == 20 ? kWaveBuf : 4];
    uint32_t* wb = WB[threadIdx.x >> 6];
    load_tables<B>(T);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t d0 = wave_id();
    if (d0 >= n)
        return;
    using PW = typename Sel<B == 20, Chunks, Win<ND>>::T;
    auto load = [&](uint32_t dd, PW& P) {
        if constexpr (B == 20)
            load_chunks(dgram + (size_t)dd * dstride, dstride, lane, P);
        else
            load_window<ND>(dgram + (size_t)dd * dstride, dstride, B * (int)lane, P);
    };
    uint32_t pk = 0, i = kWave; // i: the datagram's index in its batch (kWave: a batch starts)
    auto proc = [&](const PW& P, uint32_t d) {
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)pk, (int)i++);
        const uint32_t len = f & 0xfffu, at1 = (f >> 12) & 63u, dsize = (f >> 18) & 0xfffu;
        bool ok = false;
        if constexpr (B == 20) { // stage the datagram: LDS dwords [0, 320)
            v4u* w4 = reinterpret_cast<v4u*>(wb);
            w4[lane] = P.c0;
            if (lane < 16)
                w4[64 + lane] = P.c1;
            wave_lds_sync();
        }
        uint32_t w[ND];
        if constexpr (B == 20) {
#pragma unroll
            for (int k = 0; k < ND; ++k)
                w[k] = wb[ND * lane + k];
        } else {
            win_dwords<B, 0>(P, lane, w);
        }
        if (f & kPkValid) {
            // CRC over [0, len-4) against the big-endian trailer (sim_proto.c:21-37)
            uint32_t m[ND];
#pragma unroll
            for (int k = 0; k < ND; ++k)
                m[k] = w[k] & len_mask<B>(k, lane, len - 4);
            const uint32_t crc = wave_crc32<B>(T, m, len - 4, RFEC_WIRE_CRC_SEED, lane);
            const uint32_t tp = len - 4, q0 = tp >> 2;
            uint32_t trailer;
            if constexpr (B == 20) {
                trailer = (uint32_t)__builtin_amdgcn_readfirstlane(
                    (int)bswap(__builtin_amdgcn_alignbyte(wb[q0 + 1], wb[q0], tp & 3u)));
            } else {
                const uint32_t q1 = q0 + 1;
                const uint32_t l0 = q0 / ND, k0 = q0 - l0 * ND, l1 = q1 / ND, k1 = q1 - l1 * ND;
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)pick<ND>(w, k0), (int)l0);
                const uint32_t hi = l1 < (uint32_t)kWave
                                        ? (uint32_t)__builtin_amdgcn_readlane((int)pick<ND>(w, k1), (int)l1)
                                        : 0u;
                trailer = bswap((uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (tp & 3u))));
            }
            ok = crc == trailer;
            if (!ok) { // the record pass 1 wrote assumed a good CRC
                __builtin_amdgcn_s_waitcnt(0);
                rfec_wire_rec bad = {};
                bad.status = RFEC_WIRE_EBADCRC;
                if (lane == 0) {
                    const v4u* s = reinterpret_cast<const v4u*>(&bad);
                    v4u* o = reinterpret_cast<v4u*>(recs + d);
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        o[t] = s[t];
                }
            }
        }
        const uint32_t dsz = ok && at1 ? dsize : 0u, at = at1 ? at1 - 1u : 0u;
        uint8_t* slot = payload + (size_t)d * stride;
        if constexpr (B == 20) {
            __builtin_amdgcn_s_setprio(3);
            store_payload20(wb, slot, stride, at, dsz, lane);
            wave_lds_sync(); // the buffer is refilled by the next datagram
            __builtin_amdgcn_s_setprio(0);
        } else {
            uint32_t pay[ND];
            shift_down_bytes<B>(w, at, pay);
#pragma unroll
            for (int k = 0; k < ND; ++k)
                pay[k] &= len_mask<B>(k, lane, dsz);
            store_slot<B>(slot, stride, lane, pay);
        }
    };
    // Datagrams d0, d0 + nw, ... one per step, the loads of the datagram two
    // steps ahead issued before the current one is processed (three buffers in
    // rotation).  A batch's header pass runs first in its first step (it waits
    // on its own loads and the current datagram's, already in flight).
    auto step = [&](const PW& cur, PW& nxt, uint32_t d) {
        const uint32_t d1 = d + nw, d2 = d + 2 * nw;
        if (i == (uint32_t)kWave) { // (a batch short of kWave is the wave's last)
            const uint32_t cnt = min((uint32_t)kWave, (n - 1 - d) / nw + 1);
            HdrIn in;
            const uint32_t dl = d + lane * nw;
            __builtin_amdgcn_s_setprio(3);
            load_header(dgram, dlen, dl, lane < cnt, dstride, in);
            pk = decode_header<B>(in, recs, dl, lane < cnt, dstride, capacity);
            __builtin_amdgcn_s_setprio(0);
            i = 0;
        }
        load(min(d2, n - 1), nxt); // two ahead; past the end: the last datagram again (branch-free)
        proc(cur, d);
        return d1 < n;
    };
    PW a, b, c; // datagrams d, d + nw in flight while d is processed, d + 2 nw issued
    load(d0, a);
    load(min(d0 + nw, n - 1), b);
    for (uint32_t d = d0;; d += 3 * nw) {
        if (!step(a, c, d) || !step(b, a, d + nw) || !step(c, b, d + 2 * nw))
            break;
    }
}

// ---------------------------------------------------------------------------
// Quarter-wave SIM_SEG framing (slots of at most 1,280 bytes).  A wave frames
// four consecutive datagrams, 16 lanes each: lane s of group g owns 16-byte
// chunks c = 16 k + s (k = 0..4) of datagram 4 q + g, so every per-datagram
// quantity (header layout and size, length, CRC alignment, trailer position)
// is a per-lane value computed once for four datagrams, the payload moves
// from its slot to the datagram with one byte funnel per chunk and no LDS
// staging, and a load or store instruction covers 256 contiguous bytes of
// each of the four slots.  (The wave-per-datagram kernels above spend most
// of their ~400 instructions per datagram on wave-uniform scalar work, LDS
// transposes and cross-lane reductions: DESIGN.md §5.1.)
//
// Headers: a per-lane pass builds the 32 header bytes of 64 datagrams at once
// (the wave's next 16 quads, lane 4 t + g = quad t's datagram g), from which
// each quad takes its own with ds_bpermute.
//
// CRC32 over the datagram's n bytes: lane s's five chunks are folded by
// Horner's rule over the rows (acc = acc * x^(8 * 256) + raw CRC of the next
// chunk; slice-by-16 for a chunk, four byte lookups for the multiply), then
// carried from the end of its row-4 chunk (byte 1,040 + 16 s) to the end of
// the message: x^(8 (240 - 16 s - D)) with D = 1280 - n = 16 Dq + Dr, as
// column s + Dq of the nibble tables (columns past 15 hold the negative
// powers a lane needs when its row-4 chunk lies past the message) and one
// x^(-8 Dr) correction of the group's XOR-reduced sum (bit tables, two bits
// per lane).  Row-level DPP reduces the 16 lanes.
// ---------------------------------------------------------------------------
constexpr int kQLanes = 16, kQRows = 5, kQChunks = kQLanes * kQRows; // 80 chunks = 1,280 bytes
constexpr uint32_t kQWindow = 16u * kQChunks;
constexpr int kQCols = kQLanes + kQChunks; // carry columns s + Dq, Dq <= 80

struct CrcQTables {
    uint32_t t[16][256];         // slice-by-16, as CrcTables
    uint32_t m[4][256];          // (byte v at byte position b of a register) * x^(8 * 256)
    uint32_t nib[8][16][kQCols]; // (nibble v at nibble position i) * x^(8 (240 - 16 j))
    uint32_t inv[16][32];        // x^(31-i) * x^(-8 r)
};

constexpr CrcQTables make_crcq_tables()
{
    CrcQTables r{};
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int i = 0; i < 8; ++i)
            c = mul_x(c);
        r.t[0][b] = c;
    }
    for (int s = 1; s < 16; ++s)
        for (uint32_t b = 0; b < 256; ++b)
            r.t[s][b] = (r.t[s - 1][b] >> 8) ^ r.t[0][r.t[s - 1][b] & 0xffu];
    {
        uint32_t Y = 0x80000000u; // x^0
        for (int q = 0; q < 8 * 256; ++q)
            Y = mul_x(Y);
        uint32_t bas[32]{}; // x^e * x^2048
        for (int e = 0; e < 32; ++e) {
            bas[e] = Y;
            Y = mul_x(Y);
        }
        for (int b = 0; b < 4; ++b)
            for (uint32_t v = 0; v < 256; ++v) {
                uint32_t acc = 0;
                for (int i = 0; i < 8; ++i)
                    if (v & (1u << i))
                        acc ^= bas[31 - (8 * b + i)];
                r.m[b][v] = acc;
            }
    }
    uint32_t Vj = 0x80000000u; // x^(8 (240 - 16 j)), from x^1920 at j = 0 down by x^128 per column
    for (int q = 0; q < 8 * 240; ++q)
        Vj = mul_x(Vj);
    for (int j = 0; j < kQCols; ++j) {
        uint32_t V = Vj;
        for (int q = 0; q < 128; ++q)
            Vj = div_x(Vj);
        uint32_t basis[32]{};
        for (int e = 0; e < 32; ++e) {
            basis[e] = V;
            V = mul_x(V);
        }
        for (int i = 0; i < 8; ++i)
            for (uint32_t nv = 0; nv < 16; ++nv) {
                uint32_t acc = 0;
                for (int k = 0; k < 4; ++k)
                    if (nv & (1u << k))
                        acc ^= basis[31 - (4 * i + k)];
                r.nib[i][nv][j] = acc;
            }
    }
    for (int i = 0; i < 32; ++i) {
        uint32_t v = 1u << i;
        for (int q = 0; q < 16; ++q) {
            r.inv[q][i] = v;
            for (int b = 0; b < 8; ++b)
                v = div_x(v);
        }
    }
    return r;
}

__device__ const CrcQTables kCrcQ = make_crcq_tables();
constexpr int kQTabDwords = (int)(sizeof(CrcQTables) / 4);
constexpr int kQM = 16 * 256, kQNib = kQM + 4 * 256, kQInv = kQNib + 8 * 16 * kQCols;

// The tables into the block's LDS (no barrier: the caller's): every thread's
// loads in flight before its first LDS write -- the rolled copy waited for each
// 16-byte load in turn, five round trips at the kernels' start.
__device__ __forceinline__ void fill_tables(uint32_t* T)
{
    constexpr int N = kQTabDwords / 4, U = (N + kBlock - 1) / kBlock;
    const v4u* src = reinterpret_cast<const v4u*>(&kCrcQ);
    v4u* dst = reinterpret_cast<v4u*>(T);
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = (int)threadIdx.x + u * kBlock;
        v[u] = src[i < N ? i : N - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = (int)threadIdx.x + u * kBlock;
        if (i < N)
            dst[i] = v[u];
    }
}

// v * x^(8 * 256): four byte lookups
__device__ __forceinline__ uint32_t mul_row(const uint32_t* T, uint32_t v)
{
    return T[kQM + (v & 0xffu)] ^ T[kQM + 256 + ((v >> 8) & 0xffu)] ^ T[kQM + 512 + ((v >> 16) & 0xffu)] ^
           T[kQM + 768 + (v >> 24)];
}

// XOR of v over each 16-lane row (every lane of the row gets its row's XOR)
__device__ __forceinline__ uint32_t row_xor(uint32_t v)
{
    v ^= dpp(v, kDppQuadSwap1);
    v ^= dpp(v, kDppQuadSwap2);
    v ^= dpp(v, kDppRowRor4);
    v ^= dpp(v, kDppRowRor8);
    return v;
}

// chunk c's raw CRC r carried by column col of the nibble tables
__device__ __forceinline__ uint32_t carry_q(const uint32_t* T, uint32_t r, uint32_t col)
{
    const uint32_t* nb = T + kQNib + col;
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x ^= nb[(i * 16 + ((r >> (4 * i)) & 15u)) * kQCols];
    return x;
}

// SIM_SEG header of one datagram (sim_proto.inl:83-125), per lane: the
// header's bytes as 8 LE dwords (zero past hs) and m = valid << 31 | hs << 16
// | data_size.  The maximal layout (4-byte packet_id and fid, 2-byte index /
// total) in 16-bit big-endian units, then the narrow fields' units removed
// from the back (each removal is one select per later unit).
struct SegHdrQ {
    uint32_t h[8];
    uint32_t m;
};

__device__ __forceinline__ SegHdrQ seg_header_q(const rfec_hdr* __restrict__ hdr,
                                                const rfec_seg_stamp* __restrict__ stamps, uint32_t d, bool act,
                                                uint32_t capacity)
{
    const uint32_t* hp = reinterpret_cast<const uint32_t*>(hdr + d);
    const uint32_t* sp = reinterpret_cast<const uint32_t*>(stamps + d);
    const uint32_t seq = hp[0], fid = hp[1], ts = hp[2], h3 = hp[3], h4 = hp[4];
    const uint32_t uid = sp[0], s1 = sp[1], s2 = sp[2];
    const uint32_t idx = h3 & 0xffffu, tot = h3 >> 16, L = h4 >> 16;
    const bool PW = seq > 65535u, FW = fid > 65535u, TW = tot > 255u;
    const uint32_t mask = (h4 & 1u) | (PW ? 0x80u : 0u) | (FW ? 0x40u : 0u) | (TW ? 0x20u : 0u) |
                          (((s2 >> 16) & 0xffu) == 0 ? 0x10u : 0u);
    uint32_t u[17];
    u[0] = (RFEC_WIRE_VER << 8) | RFEC_WIRE_SEG;
    u[1] = uid >> 16;
    u[2] = uid & 0xffffu;
    u[3] = (mask << 8) | ((h4 >> 8) & 0xffu);
    // maximal tail: seq 2, fid 2, ts 2, index, total, fec_id, send_ts, transport_seq, size
    u[4] = seq >> 16, u[5] = seq & 0xffffu, u[6] = fid >> 16, u[7] = fid & 0xffffu;
    u[8] = ts >> 16, u[9] = ts & 0xffffu, u[10] = idx, u[11] = tot;
    u[12] = s1 & 0xffffu, u[13] = s1 >> 16, u[14] = s2 & 0xffffu, u[15] = L, u[16] = 0;
    // 1-byte index and total: one unit (index low byte, total low byte)
    u[10] = TW ? u[10] : ((idx & 0xffu) << 8) | (tot & 0xffu);
#pragma unroll
    for (int r = 11; r < 16; ++r)
        u[r] = TW ? u[r] : u[r + 1];
    // 2-byte fid: drop its high unit
#pragma unroll
    for (int r = 6; r < 16; ++r)
        u[r] = FW ? u[r] : u[r + 1];
    // 2-byte packet_id
#pragma unroll
    for (int r = 4; r < 16; ++r)
        u[r] = PW ? u[r] : u[r + 1];
    SegHdrQ H;
#pragma unroll
    for (int k = 0; k < 8; ++k) // bytes of unit 2k, then of unit 2k + 1 (big-endian each)
        H.h[k] = __builtin_amdgcn_perm(u[2 * k + 1], u[2 * k], 0x04050001u);
    const uint32_t hs = 26u + 2u * ((uint32_t)PW + (uint32_t)FW + (uint32_t)TW);
    // units past hs / 2 were shifted in from u[16] = 0: the bytes past hs are zero
    H.m = (act && L <= capacity ? 0x80000000u : 0u) | hs << 16 | L;
    return H;
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4u), (int)v);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc64(const void* p, uint64_t bytes)
{
    return rsrc(p, bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes);
}

// bytes >= m of a quarter-wave's chunks to zero (rows that some lane's range ends in or before)
__device__ __forceinline__ void mask_q(uint32_t (&x)[kQRows][4], uint32_t m, uint32_t s)
{
#pragma unroll
    for (int k = 0; k < kQRows; ++k) {
        const int e = (int)m - (int)(16u * (16u * k + s));
        if (__builtin_amdgcn_ballot_w64(e < 16) != 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) { // keep min(max(e - 4 j, 0), 4) bytes of dword j
                const uint32_t t8 = 8u * (uint32_t)min(max(e - 4 * j, 0), 4);
                x[k][j] &= ~(uint32_t)(0xFFFFFFFFull << t8);
            }
        }
    }
}

// payload windows of a quad's datagram for its five chunk rows: chunk c
// needs payload bytes [16 c - hs, 16 c - hs + 16), read from the dword below
// (for c < 2, from payload byte 0: see the row-0 fix-up)
__device__ __forceinline__ void load_rows_q(__amdgpu_buffer_rsrc_t rin, uint32_t pbase, uint32_t m, uint32_t s,
                                            v4u (&W)[kQRows])
{
    const uint32_t hs = (m >> 16) & 63u, sh = hs & 2u;
#pragma unroll
    for (int k = 0; k < kQRows; ++k) {
        const uint32_t c = 16u * k + s;
        const uint32_t off = pbase + (c >= 2 ? 16u * c - hs - sh : 0u);
        W[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kAuxNT));
    }
}

// (registers capped for 8 waves per SIMD, two blocks per CU: the LDS tables
// allow two; 4 waves per SIMD with a software-pipelined next quad took 452 vs
// 381 us, the same pipeline capped at 64 registers spilled: 680 us)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_frame_seg_q(
    const uint8_t* __restrict__ shards, const rfec_hdr* __restrict__ hdr, const rfec_seg_stamp* __restrict__ stamps,
    const uint32_t* __restrict__ order, uint8_t* __restrict__ dgram, uint16_t* __restrict__ dlen, uint32_t count,
    uint32_t stride, uint32_t capacity, uint32_t dstride, uint32_t rows_out)
{
    __shared__ __attribute__((aligned(16))) uint32_t T[kQTabDwords];
    fill_tables(T);
    __syncthreads();
    const uint32_t lane = threadIdx.x & (kWave - 1), g = lane >> 4, s = lane & 15u;
    const uint32_t nquads = (count + 3u) / 4u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t q = wave_id();
    if (q >= nquads)
        return;
    const __amdgpu_buffer_rsrc_t rin = rsrc64(shards, (uint64_t)count * stride);
    const __amdgpu_buffer_rsrc_t rout = rsrc64(dgram, (uint64_t)rows_out * dstride); // (rows >= rows_out: dropped)
    // the batch: lane 4 t + g holds quad q + t nw's datagram g
    SegHdrQ B;
    auto pass = [&](uint32_t q0) {
        const uint32_t dd = 4u * (q0 + (lane >> 2) * nw) + (lane & 3u);
        const bool a = dd < count;
        B = seg_header_q(hdr, stamps, a ? dd : 0u, a, capacity);
    };
    uint32_t bt = 16;
    for (;;) {
        if (bt == 16) { // the next 16 quads' headers
            pass(q);
            bt = 0;
        }
        const uint32_t src = 4u * bt + g;
        const uint32_t mc = bperm(B.m, src);
        v4u W[kQRows];
        load_rows_q(rin, (4u * q + g) * stride, mc, s, W);
        const uint32_t oc = order ? order[min(4u * q + g, count - 1u)] : 4u * q + g;
        uint32_t Hd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            Hd[j] = bperm(B.h[j], src);
        ++bt;
        const uint32_t d = 4u * q + g;
        const bool act = d < count;
        const uint32_t hs = (mc >> 16) & 63u, L = mc & 0xffffu;
        const bool valid = (mc >> 31) != 0;
        const uint32_t n = valid ? hs + L : 0u; // invalid: every byte masked, length 0
        const uint32_t sh = hs & 2u;             // (16 c - hs) mod 4 for an even hs
        const uint32_t o = oc;
        // datagram chunks from the payload windows; a window's fifth dword is
        // the next chunk's first (lane s + 1's, for s = 15 lane 0's in the next
        // row; chunk 79's lies past any message)
        uint32_t out[kQRows][4];
        {
            uint32_t nx[kQRows];
#pragma unroll
            for (int k = 0; k < kQRows; ++k)
                nx[k] = dpp(W[k][0], kDppRowRor15);
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                uint32_t w[5] = {W[k][0], W[k][1], W[k][2], W[k][3], s == 15 ? (k + 1 < kQRows ? nx[k + 1 < kQRows ? k + 1 : k] : 0u) : nx[k]};
                if (k == 0) {
                    // lane 0: header bytes 0-15; lane 1: header bytes 16-31 over
                    // the payload's first 32 - hs bytes (loaded from payload byte 0,
                    // they start 3 or 4 dwords into the window)
                    const bool z3 = hs + sh == 28u;
                    const uint32_t p0 = w[0], p1 = w[1];
                    w[0] = s > 1 ? w[0] : 0u;
                    w[1] = s > 1 ? w[1] : 0u;
                    w[2] = s > 1 ? w[2] : 0u;
                    w[3] = s > 1 ? w[3] : (s == 1 && z3 ? p0 : 0u);
                    w[4] = s > 1 ? w[4] : (s == 1 ? (z3 ? p1 : p0) : 0u);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    out[k][j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            out[0][j] |= s == 0 ? Hd[j] : (s == 1 ? Hd[4 + j] : 0u);
        mask_q(out, n, s);
        // CRC32 (Horner over the rows, seed folded into the first dword)
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kQRows; ++k) {
            const uint32_t x0 = out[k][0] ^ (k == 0 && s == 0 ? ~RFEC_WIRE_CRC_SEED : 0u);
            acc = (k ? mul_row(T, acc) : 0u) ^ slice16(T, x0, out[k][1], out[k][2], out[k][3]);
        }
        const uint32_t D = kQWindow - n, Dq = D >> 4, Dr = D & 15u;
        const uint32_t R = row_xor(carry_q(T, acc, s + Dq));
        const uint32_t* iv = T + kQInv + Dr * 32u;
        const uint32_t b = (((R >> s) & 1u) ? iv[s] : 0u) ^ (((R >> (s + 16u)) & 1u) ? iv[s + 16u] : 0u);
        const uint32_t crc = ~row_xor(b);
        // big-endian trailer at byte n: dwords n / 4 and n / 4 + 1.  (Storing
        // the rows as they are hashed and holding back the trailer's chunks
        // took registers the CRC needs: spills, 495 vs 381 us.)
        if (valid) {
            const uint32_t be = bswap(crc), s4 = n & 3u, q0 = n >> 2;
            const uint32_t lo = be << (8 * s4), hi = s4 ? be >> (32 - 8 * s4) : 0u;
            const int x0 = (int)q0 - (int)(4u * s); // relative to the lane's row-0 chunk
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                const int x = x0 - 64 * k;
                if (__builtin_amdgcn_ballot_w64(x >= -1 && x < 4) == 0)
                    continue; // (wave-uniform: no lane's trailer in this row)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    out[k][j] |= x == j ? lo : (x == j - 1 ? hi : 0u);
            }
        }
        if (act) {
            const uint32_t obase = o * dstride;
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                const uint32_t c = 16u * k + s;
                if (16u * c < dstride)
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{out[k][0], out[k][1], out[k][2], out[k][3]}, rout,
                                                           obase + 16u * c, 0, kAuxST);
            }
            if (s == 0 && o < rows_out)
                dlen[o] = (uint16_t)(valid ? n + 4u : 0u);
        }
        q += nw;
        if (q >= nquads)
            break;
    }
}

// Quarter-wave SIM_FEC framing, as k_frame_seg_q: the 45-byte header
// (sim_proto.c:13-18, sim_proto.inl:244-254, 270-283) has one layout, so no
// header pass: lane i < 13 of a group loads field dword i of its datagram
// (0-5 rfec_fec_stamp, 6-10 fec_meta, 11 fec_data_size, 12 status), every
// lane takes the 13 with ds_bpermute, and lanes 0-2 byte-permute them into
// header dwords 0-11.  The payload starts at byte 45: chunk c >= 3 takes
// payload bytes [16 (c - 3), 16 (c - 2)) plus the next chunk's first dword
// shifted by 3 bytes; chunk 2 holds the header's last 13 bytes and payload
// bytes 0-2.
__device__ __forceinline__ uint32_t fec_hdr_dword(const uint32_t (&F)[13], int m)
{
    // header bytes 4 m .. 4 m + 3 from big-endian fields (v_perm: selector
    // bytes 0-3 pick from the second operand, 4-7 from the first, 12 = zero)
    switch (m) {
    case 0: return __builtin_amdgcn_perm(0u, F[0], 0x02030C0Cu) | (RFEC_WIRE_FEC << 8) | RFEC_WIRE_VER;
    case 1: return __builtin_amdgcn_perm(F[3], F[0], 0x04050001u);
    case 2: return (__builtin_amdgcn_perm(F[5], F[4], 0x07040302u) & 0x00FFFFFFu) | (F[3] >> 24) << 24;
    case 3: return __builtin_amdgcn_perm(F[1], F[3], 0x05060702u);
    case 4: return (__builtin_amdgcn_perm(F[4], F[1], 0x07040500u) & 0x00FFFFFFu) | (F[2] >> 24) << 24;
    case 5: return __builtin_amdgcn_perm(F[6], F[2], 0x07000102u);
    case 6: return __builtin_amdgcn_perm(F[7], F[6], 0x07000102u);
    case 7: return __builtin_amdgcn_perm(F[8], F[7], 0x07000102u);
    case 8: return __builtin_amdgcn_perm(F[9], F[8], 0x05000102u);
    case 9: return __builtin_amdgcn_perm(F[10], F[9], 0x04020300u);
    case 10: return __builtin_amdgcn_perm(F[11], F[10], 0x05020301u);
    default: return F[11] & 0xffu;
    }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_frame_fec_q(
    const uint8_t* __restrict__ parity, const rfec_hdr* __restrict__ meta, const uint16_t* __restrict__ fsize,
    const int8_t* __restrict__ status, const rfec_fec_stamp* __restrict__ stamps, const uint32_t* __restrict__ order,
    uint8_t* __restrict__ dgram, uint16_t* __restrict__ dlen, uint32_t count, uint32_t stride, uint32_t capacity,
    uint32_t dstride)
{
    __shared__ __attribute__((aligned(16))) uint32_t T[kQTabDwords];
    const uint32_t lane = threadIdx.x & (kWave - 1), g = lane >> 4, s = lane & 15u;
    const uint32_t nquads = (count + 3u) / 4u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t q = wave_id();
    const __amdgpu_buffer_rsrc_t rin = rsrc64(parity, (uint64_t)count * stride);
    const __amdgpu_buffer_rsrc_t rout = rsrc64(dgram, (uint64_t)count * dstride);
    // field descriptors over the whole arrays: a lane's offset past the end reads 0
    const __amdgpu_buffer_rsrc_t rst = rsrc64(stamps, (uint64_t)count * sizeof(rfec_fec_stamp));
    const __amdgpu_buffer_rsrc_t rme = rsrc64(meta, (uint64_t)count * sizeof(rfec_hdr));
    const __amdgpu_buffer_rsrc_t rfs = rsrc64(fsize, (uint64_t)count * 2u);
    const __amdgpu_buffer_rsrc_t rsu = rsrc64(status, status ? count : 0u);
    constexpr uint32_t kOut = 0xFFFFFFF0u;
    // payload windows (chunk c >= 3: payload bytes from 16 (c - 3); chunk 2: from 0)
    // and the field dwords of quad q, issued at the bottom of the loop (117.6-118.4
    // vs 119.9-120.5 us at the top; before the copy of the tables 120.3-120.8 us)
    v4u W[kQRows];
    uint32_t fv;
    auto load = [&](uint32_t qq) {
        const uint32_t dd = 4u * qq + g, pbase = dd * stride;
#pragma unroll
        for (int k = 0; k < kQRows; ++k) {
            const uint32_t c = 16u * k + s;
            W[k] = __builtin_bit_cast(
                v4u, __builtin_amdgcn_raw_buffer_load_b128(rin, pbase + (c >= 3 ? 16u * (c - 3) : 0u), 0, kAuxNT));
        }
        fv = __builtin_amdgcn_raw_buffer_load_b32(rst, s < 6 ? 24u * dd + 4u * s : kOut, 0, kAuxNT);
        fv |= __builtin_amdgcn_raw_buffer_load_b32(rme, s - 6u < 5u ? 20u * dd + 4u * (s - 6u) : kOut, 0, kAuxNT);
        fv |= __builtin_amdgcn_raw_buffer_load_b16(rfs, s == 11 ? 2u * dd : kOut, 0, kAuxNT);
        fv |= (uint32_t)(int32_t)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(rsu, s == 12 ? dd : kOut, 0, kAuxNT);
    };
    fill_tables(T);
    __syncthreads();
    if (q >= nquads)
        return;
    load(q);
    for (;;) {
        const uint32_t d = 4u * q + g;
        const bool act = d < count;
        const uint32_t o = order ? order[act ? d : 0u] : d;
        uint32_t F[13];
#pragma unroll
        for (int i = 0; i < 13; ++i)
            F[i] = bperm(fv, 16u * g + i);
        const uint32_t L = F[11];
        const bool valid = (int32_t)F[12] >= 0 && L <= capacity;
        const uint32_t n = valid ? 45u + L : 0u;
        // header dwords 4 s .. 4 s + 3 for lanes 0-2
        uint32_t Hd[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t h0 = fec_hdr_dword(F, j), h1 = fec_hdr_dword(F, 4 + j), h2 = fec_hdr_dword(F, 8 + j);
            Hd[j] = s == 0 ? h0 : (s == 1 ? h1 : (s == 2 ? h2 : 0u));
        }
        uint32_t out[kQRows][4];
        {
            uint32_t nx[kQRows];
#pragma unroll
            for (int k = 0; k < kQRows; ++k)
                nx[k] = dpp(W[k][0], kDppRowRor15);
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                uint32_t w[5] = {W[k][0], W[k][1], W[k][2], W[k][3],
                                 s == 15 ? (k + 1 < kQRows ? nx[k + 1 < kQRows ? k + 1 : k] : 0u) : nx[k]};
                if (k == 0) { // lanes 0-1: header only; lane 2: payload bytes 0-2 at its end
                    const uint32_t p0 = w[0];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        w[j] = s > 2 ? w[j] : 0u;
                    w[4] = s > 2 ? w[4] : (s == 2 ? p0 : 0u);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    out[k][j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], 3);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            out[0][j] |= Hd[j];
        mask_q(out, n, s);
        // CRC32 (Horner over the rows, seed folded into the first dword)
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kQRows; ++k) {
            const uint32_t x0 = out[k][0] ^ (k == 0 && s == 0 ? ~RFEC_WIRE_CRC_SEED : 0u);
            acc = (k ? mul_row(T, acc) : 0u) ^ slice16(T, x0, out[k][1], out[k][2], out[k][3]);
        }
        const uint32_t D = kQWindow - n, Dq = D >> 4, Dr = D & 15u;
        const uint32_t R = row_xor(carry_q(T, acc, s + Dq));
        const uint32_t* iv = T + kQInv + Dr * 32u;
        const uint32_t b = (((R >> s) & 1u) ? iv[s] : 0u) ^ (((R >> (s + 16u)) & 1u) ? iv[s + 16u] : 0u);
        const uint32_t crc = ~row_xor(b);
        if (valid) { // big-endian trailer at byte n
            const uint32_t be = bswap(crc), s4 = n & 3u, q0 = n >> 2;
            const uint32_t lo = be << (8 * s4), hi = s4 ? be >> (32 - 8 * s4) : 0u;
            const int x0 = (int)q0 - (int)(4u * s);
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                const int x = x0 - 64 * k;
                if (__builtin_amdgcn_ballot_w64(x >= -1 && x < 4) == 0)
                    continue;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    out[k][j] |= x == j ? lo : (x == j - 1 ? hi : 0u);
            }
        }
        if (act) {
            const uint32_t obase = o * dstride;
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                const uint32_t c = 16u * k + s;
                if (16u * c < dstride)
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{out[k][0], out[k][1], out[k][2], out[k][3]}, rout,
                                                           obase + 16u * c, 0, kAuxST);
            }
            if (s == 0)
                dlen[o] = (uint16_t)(valid ? n + 4u : 0u);
        }
        q += nw;
        if (q >= nquads)
            break;
        load(q);
    }
}

// ---------------------------------------------------------------------------
// Quarter-wave parse (slots of at most 1,280 bytes, or datagrams that fit
// 1,280 bytes; payload slots of at most 1,280 bytes): the framing's layout
// run backwards.  A wave parses four consecutive datagrams, 16 lanes each;
// lane s of group g holds 16-byte chunks c = 16 k + s (k = 0..4) of datagram
// 4 q + g, aligned b128 loads, no LDS staging.
//
// Headers: a per-lane pass over the wave's next 64 datagrams (lane 4 t + g =
// quad t's datagram g) decodes each header as if its CRC matched (decode_lane,
// as k_parse), writes the record and keeps the packed facts (length, data
// position, data size) and the big-endian trailer (one b64 load at the
// trailer's dword); each quad takes its datagram's two dwords by ds_bpermute.
//
// CRC32 over [0, len - 4): the framing's (Horner over the five rows, one carry
// by column s + Dq, one x^(-8 Dr) correction, row-level DPP XORs) on the
// chunks with the bytes from len - 4 on masked, against the trailer.
//
// Payload: the data starts at byte `at` = 16 A + r of the datagram (26-32 for
// a SIM_SEG, 45 for a SIM_FEC).  The lane that holds datagram chunk C produces
// payload chunk j = (C - A) mod 80: its own chunk and the next one (lane s + 1
// of the row, a row_ror:15 DPP move; lane 15 takes lane 0's of the next row)
// shifted down by r bytes in registers, masked at the data size, one aligned
// b128 store -- every payload chunk of the slot is produced by exactly one
// lane, so the zeros to the slot's end come out of the same stores (the A
// chunks that wrap round are past any data).  The payload is stored as if the
// CRC matched; a group whose CRC fails (rare) zeroes its slot afterwards and
// rewrites its record as EBADCRC.
// ---------------------------------------------------------------------------
// (rin: a descriptor over the whole batch, per-lane offsets < 2^32; the second
// dword may lie in the next slot, or past the batch: 0)
// bytes >= m of one 16-byte chunk (byte offset c0 in its message) zeroed
__device__ __forceinline__ uint32_t keep_below(uint32_t v, int j, int e)
{
    const uint32_t t8 = 8u * (uint32_t)min(max(e - 4 * j, 0), 4);
    return v & ~(uint32_t)(0xFFFFFFFFull << t8);
}

// 4 waves per SIMD: the next quad's rows in flight beside this quad's (125
// VGPRs, no spill).  Capped at 64 VGPRs for 8 waves it spilled 53 and ran
// 8-13 % slower than the wave-per-datagram parse; at 4 waves: parse_seg
// 361 vs 386-389 us, parse_fec 111-113 vs 122-123 us against that kernel's
// three-deep 4-wave form (profiles/r05/ab/parse_occupancy/).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_parse_q(
    const uint8_t* __restrict__ dgram, const uint16_t* __restrict__ dlen, rfec_wire_rec* __restrict__ recs,
    uint8_t* __restrict__ payload, uint32_t n, uint32_t dstride, uint32_t stride, uint32_t capacity,
    rfec_rx_split* __restrict__ split, uint32_t shards)
{
    __shared__ __attribute__((aligned(16))) uint32_t T[kQTabDwords];
    const uint32_t lane = threadIdx.x & (kWave - 1), g = lane >> 4, s = lane & 15u;
    const uint32_t nquads = (n + 3u) / 4u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t q = wave_id();
    const bool live = q < nquads; // (the others still fill the tables)
    const __amdgpu_buffer_rsrc_t rin = rsrc64(dgram, (uint64_t)n * dstride);
    const __amdgpu_buffer_rsrc_t rout = rsrc64(payload, (uint64_t)n * stride);
    constexpr uint32_t kOut = 0xFFFFFFF0u;
    const uint32_t rows_in = min(dstride, kQWindow); // the slot's bytes a lane may load
    uint32_t F = 0, bt = 0;
    // the headers of quads q0, q0 + nw, ... (16 of them), one datagram per lane:
    // loads, then the decode and the records (a batch's loads are issued before
    // the previous quad's payload stores)
    HdrIn hin;
    auto header_load = [&](uint32_t q0) {
        const uint32_t dd = 4u * (q0 + (lane >> 2) * nw) + (lane & 3u);
        load_header(dgram, dlen, dd, dd < n, dstride, hin);
    };
    auto header_decode = [&](uint32_t q0) {
        const uint32_t dd = 4u * (q0 + (lane >> 2) * nw) + (lane & 3u);
        __builtin_amdgcn_s_setprio(3);
        F = decode_header<20>(hin, recs, dd, dd < n, dstride, capacity, split, shards);
        __builtin_amdgcn_s_setprio(0);
    };
    // row k of quad qq's datagram (a lane past the batch or the slot reads 0 without a memory access)
    auto load_row = [&](uint32_t qq, int k) {
        const uint32_t dd = 4u * qq + g, o = 16u * (16u * k + s);
        return __builtin_bit_cast(
            v4u, __builtin_amdgcn_raw_buffer_load_b128(rin, qq < nquads && dd < n && o < rows_in ? dd * dstride + o
                                                                                             : kOut,
                                                       0, kAuxNT));
    };
    // The next quad's rows are loaded as soon as this quad's are consumed, and
    // before this quad's payload stores: vmcnt counts loads and stores in issue
    // order, so a load issued after a store can only be waited for together
    // with that store (loads issued after the previous quad's stores wait for
    // their write acknowledgements).  At a batch's end the next batch's header
    // loads take the rows' place before the stores (fewer registers live across
    // them); its first quad's rows are loaded after the stores, in flight while
    // the headers decode.
    // the first batch: the tables first (row loads issued ahead of them held
    // the block's barrier back: SIM_FEC parse +2 %), then its header loads and
    // the first quad's rows, in flight together while the headers decode
    v4u X[kQRows];
    fill_tables(T);
    __syncthreads();
    if (!live)
        return;
    header_load(q);
#pragma unroll
    for (int k = 0; k < kQRows; ++k)
        X[k] = load_row(q, k);
    header_decode(q);
    for (;;) {
        const uint32_t d = 4u * q + g;
        const bool act = d < n;
        const uint32_t src = 4u * bt + g;
        const uint32_t f = bperm(F, src);
        ++bt;
        const bool valid = (f & kPkValid) != 0;
        const uint32_t len = f & 0xfffu, at1 = (f >> 12) & 63u, dsize = (f >> 18) & 0xfffu;
        const uint32_t nb = valid ? len - 4u : 0u;
        const uint32_t at = at1 ? at1 - 1u : 0u, A = at >> 4, r = at & 15u;
        const uint32_t dsz = at1 ? dsize : 0u;
        // One pass over the rows: row k's CRC (Horner, the bytes from nb on
        // masked, the seed folded into the first dword) and its payload chunk
        // (j = (C - A) mod 80 from chunks C, C + 1 shifted down by r; stored
        // as if the CRC matched).
        __builtin_amdgcn_s_setprio(3);
        uint32_t acc = 0, trl = 0; // trl: the trailer (the datagram's CRC32), from the lane whose chunk holds it
        v4u Y[kQRows]; // the payload chunks
        uint32_t PO[kQRows];
#pragma unroll
        for (int k = 0; k < kQRows; ++k) {
            {
                const int e = (int)nb - (int)(16u * (16u * k + s));
                uint32_t x[4] = {X[k][0], X[k][1], X[k][2], X[k][3]};
                if (__builtin_amdgcn_ballot_w64(e < 16) != 0) { // (wave-uniform: a message ends in this row)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        x[j] = keep_below(x[j], j, e);
                }
                x[0] ^= k == 0 && s == 0 ? ~RFEC_WIRE_CRC_SEED : 0u;
                acc = (k ? mul_row(T, acc) : 0u) ^ slice16(T, x[0], x[1], x[2], x[3]);
            }
            // window: own chunk w[0..3], the next one w[4..7] (lane s + 1 of the row; lane 15: lane 0 of
            // the next row, which row_ror:15 of that row's register brings to lane 15)
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[i] = X[k][i];
                const uint32_t a = dpp(X[k][i], kDppRowRor15);
                const uint32_t b = k + 1 < kQRows ? dpp(X[k + 1 < kQRows ? k + 1 : k][i], kDppRowRor15) : 0u;
                w[4 + i] = s == 15 ? b : a;
            }
            // the trailer, bytes [nb, nb + 4), from the rows already in registers (a separate load of the
            // datagram's last line was a second HBM fetch of it: the parse fetched 1.17 x its reads)
            if (16u * k + s == (nb >> 4)) {
                const uint32_t i0 = (nb >> 2) & 3u;
                const uint32_t lo = i0 == 0 ? w[0] : i0 == 1 ? w[1] : i0 == 2 ? w[2] : w[3];
                const uint32_t hi = i0 == 0 ? w[1] : i0 == 1 ? w[2] : i0 == 2 ? w[3] : w[4];
                trl = bswap(__builtin_amdgcn_alignbyte(hi, lo, nb & 3u));
            }
            // shift down by r: 8 bytes, 4 bytes, then the byte funnel.  The selects are byte permutes with a
            // per-lane selector (all bytes of one operand or the other): selects over array elements are
            // otherwise folded into an indexed access, i.e. the window in scratch
            const uint32_t s8 = (r & 8u) ? 0x07060504u : 0x03020100u, s4 = (r & 4u) ? 0x07060504u : 0x03020100u;
#pragma unroll
            for (int i = 0; i < 6; ++i)
                w[i] = __builtin_amdgcn_perm(w[i + 2], w[i], s8);
#pragma unroll
            for (int i = 0; i < 5; ++i)
                w[i] = __builtin_amdgcn_perm(w[i + 1], w[i], s4);
            const uint32_t C = 16u * k + s;
            const uint32_t jj = C >= A ? C - A : C + kQChunks - A; // payload chunk
            const int e = (int)dsz - (int)(16u * jj);               // its data bytes
            uint32_t y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                y[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], r & 3u);
            if (__builtin_amdgcn_ballot_w64(e < 16) != 0) { // (wave-uniform: some lane's data ends here)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    y[i] = keep_below(y[i], i, e);
            }
            const uint32_t po = 16u * jj;
            Y[k] = v4u{y[0], y[1], y[2], y[3]};
            PO[k] = act && po < stride ? d * stride + po : kOut;
        }
        const uint32_t D = kQWindow - nb, Dq = D >> 4, Dr = D & 15u;
        const uint32_t R = row_xor(carry_q(T, acc, s + Dq));
        const uint32_t* iv = T + kQInv + Dr * 32u;
        const uint32_t b = (((R >> s) & 1u) ? iv[s] : 0u) ^ (((R >> (s + 16u)) & 1u) ? iv[s + 16u] : 0u);
        const bool ok = valid && ~row_xor(b) == row_xor(trl);
        __builtin_amdgcn_s_setprio(0);
        const uint32_t qn = q + nw;
        const bool batch_end = bt == 16; // (wave-uniform) the next quad starts a header batch
        if (!batch_end) {
#pragma unroll
            for (int k = 0; k < kQRows; ++k)
                X[k] = load_row(qn, k);
        } else if (qn < nquads) {
            header_load(qn);
        }
#pragma unroll
        for (int k = 0; k < kQRows; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(Y[k], rout, PO[k], 0, kAuxST);
        if (valid && !ok && act) { // rare: a CRC mismatch -- zero the slot, the record reads EBADCRC
            __builtin_amdgcn_s_waitcnt(0); // after this wave's header-pass record and payload stores
#pragma unroll
            for (int k = 0; k < kQRows; ++k) {
                const uint32_t po = 16u * (16u * k + s);
                __builtin_amdgcn_raw_buffer_store_b128(v4u{0, 0, 0, 0}, rout, po < stride ? d * stride + po : kOut,
                                                       0, kAuxST);
            }
            if (s < 4) { // the record's four 16-byte pieces: status EBADCRC (byte 0), every other field 0
                static_assert(RFEC_WIRE_EBADCRC == -1 && offsetof(rfec_wire_rec, status) == 0, "record layout");
                reinterpret_cast<v4u*>(recs + d)[s] = v4u{s == 0 ? 0xFFu : 0u, 0u, 0u, 0u};
            }
            if (split && s == 0) // no control-plane effect
                *reinterpret_cast<uint2*>(split + d) = uint2{0xFFu | RX_SPLIT_NONE << 8, 0u};
        }
        q = qn;
        if (q >= nquads)
            break;
        if (batch_end) {
#pragma unroll
            for (int k = 0; k < kQRows; ++k)
                X[k] = load_row(q, k);
            header_decode(q);
            bt = 0;
        }
    }
}

// Persistent grid: exactly the blocks that are resident at once (occupancy
// from the kernel's registers / LDS x CUs), so no block waits for a second
// round; fewer when the batch is small.  TAG: one cache per kernel instance.
template <int TAG>
uint32_t grid_for(const void* kernel, uint32_t count)
{
    static int resident = 0; // blocks per device, per kernel
    if (!resident) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || cus <= 0 ||
            per_cu <= 0)
            cus = 256, per_cu = 2;
        resident = cus * per_cu;
    }
    const uint32_t blocks = (count + kWavesPerBlock - 1) / kWavesPerBlock;
    return blocks < (uint32_t)resident ? (blocks ? blocks : 1u) : (uint32_t)resident;
}

// lane width: 20 bytes while a wave of them covers the slot, else 32
inline bool narrow(uint32_t dstride) { return dstride <= (uint32_t)(kWave * 20); }

// quarter-wave framing: datagram slots of 16-byte multiples up to 1,280 bytes,
// dword-aligned payload slots, both arrays addressable by 32-bit buffer offsets
inline bool quarter_ok(uint32_t count, uint32_t stride, uint32_t dstride)
{
    return dstride <= kQWindow && dstride % 16 == 0 && stride % 4 == 0 &&
           ((uint64_t)count + 4) * stride + kQWindow < 0xFFFFFFF0ull && (uint64_t)count * dstride < 0xFFFFFFF0ull;
}


} // namespace

extern "C" {

int rfec_launch_wire_frame_fec(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                               const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                               const rfec_fec_stamp* stamps, const uint32_t* order, uint32_t dstride,
                               uint8_t* dgram, uint16_t* dlen, void* stream)
{
    hipStream_t sm = reinterpret_cast<hipStream_t>(stream);
    if (quarter_ok(count, stride, dstride)) {
        const uint32_t quads = (count + 3u) / 4u;
        RFEC_LAUNCH(k_frame_fec_q, dim3(grid_for<7>((const void*)k_frame_fec_q, quads)), dim3(kBlock), 0, sm, parity,
                    meta, fec_size, status, stamps, order, dgram, dlen, count, stride, capacity, dstride);
    } else // slots above 1,280 bytes (or a batch past 32-bit buffer offsets): 32-byte lanes
        RFEC_LAUNCH(k_frame_fec<32>, dim3(grid_for<1>((const void*)k_frame_fec<32>, count)), dim3(kBlock), 0, sm,
                           parity, meta, fec_size, status, stamps, order, dgram, dlen, count, stride, capacity, dstride);
    return (int)hipGetLastError();
}

int rfec_launch_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                               const rfec_hdr* hdr, const rfec_seg_stamp* stamps, const uint32_t* order,
                               uint32_t dstride, uint8_t* dgram, uint16_t* dlen, uint32_t rows_out, void* stream)
{
    hipStream_t sm = reinterpret_cast<hipStream_t>(stream);
    if (quarter_ok(count, stride, dstride)) {
        const uint32_t quads = (count + 3u) / 4u;
        RFEC_LAUNCH(k_frame_seg_q, dim3(grid_for<6>((const void*)k_frame_seg_q, quads)), dim3(kBlock), 0, sm, shards,
                    hdr, stamps, order, dgram, dlen, count, stride, capacity, dstride, rows_out);
    } else // slots above 1,280 bytes (or a batch past 32-bit buffer offsets): 32-byte lanes
        RFEC_LAUNCH(k_frame_seg<32>, dim3(grid_for<3>((const void*)k_frame_seg<32>, count)), dim3(kBlock), 0, sm,
                           shards, hdr, stamps, order, dgram, dlen, count, stride, capacity, dstride, rows_out);
    return (int)hipGetLastError();
}

int rfec_launch_wire_parse(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                           uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                           uint32_t max_len, void* stream)
{
    return rfec_launch_wire_parse_split(n, dstride, dgram, dlen, stride, capacity, recs, payload, max_len, nullptr, 1,
                                        stream);
}

int rfec_launch_wire_parse_split(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                                 uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                                 uint32_t max_len, rfec_rx_split* split, uint32_t shards, void* stream)
{
    hipStream_t sm = reinterpret_cast<hipStream_t>(stream);
    // quarter-wave: the first 1,280 bytes of a slot, enough when the slot or every datagram fits;
    // payload slots of at most 1,280 bytes; both arrays within 32-bit buffer offsets
    const bool fits = dstride <= kQWindow || (max_len && max_len <= kQWindow);
    if (fits && stride <= kQWindow && !(rfec_get_tuning() & RFEC_TUNE_WAVE_PARSE) &&
        (uint64_t)n * dstride + kQWindow < 0xFFFFFFF0ull && (uint64_t)n * stride < 0xFFFFFFF0ull) {
        const uint32_t quads = (n + 3u) / 4u;
        RFEC_LAUNCH(k_parse_q, dim3(grid_for<8>((const void*)k_parse_q, quads)), dim3(kBlock), 0, sm, dgram, dlen,
                    recs, payload, n, dstride, stride, capacity, split, shards ? shards : 1u);
        return (int)hipGetLastError();
    }
    // 20-byte lanes cover 1,280 bytes of a slot: enough when the slot or every datagram fits
    if (narrow(dstride) || (max_len && max_len <= (uint32_t)(kWave * 20)))
        RFEC_LAUNCH(k_parse<20>, dim3(grid_for<4>((const void*)k_parse<20>, n)), dim3(kBlock), 0, sm, dgram,
                           dlen, recs, payload, n, dstride, stride, capacity);
    else
        RFEC_LAUNCH(k_parse<32>, dim3(grid_for<5>((const void*)k_parse<32>, n)), dim3(kBlock), 0, sm, dgram,
                           dlen, recs, payload, n, dstride, stride, capacity);
    const int e = (int)hipGetLastError();
    // the wave parses write no split entries: the split kernel after them
    return e || !split ? e : rfec_launch_rx_split(recs, n, shards ? shards : 1u, split, stream);
}

} // extern "C"
