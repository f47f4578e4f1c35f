// rfec_service.hip -- the drop-in's resident service: ONE workgroup that stays
// on the device between calls and takes flex_fec_generate / group-level
// flex_fec_sender_update / flex_fec_recover jobs from a doorbell in pinned,
// host-coherent memory, so that a call costs PCIe round trips instead of a
// kernel launch plus a stream synchronisation (rfec_host.c, "resident
// service").
//
// Arithmetic restated from the reference (yuanrongxi/razor), as the batch
// kernels of rfec_kernels.hip:
//   parity payload  = XOR of zero-padded member payloads  flex_fec_xor.c:30-32, 46-49
//   parity meta     = XOR of member headers, max data_size flex_fec_xor.c:13-26, 37-44
//   recovery        = parity ^ XOR of present members, refused when a member is
//                     longer than fec_data_size (:88-89) or the recovered size
//                     is (:98-99)                          flex_fec_xor.c:55-104
//
// Protocol (rfec_svc_ctl, razor_amd/csrc/rfec_internal.h): the host writes a
// job (payload slots into the staging area, the job description into the
// request-side control block -- host-mapped device memory, or pinned host
// memory where the host cannot map it), then the doorbell word (sequence
// number, slot count, op); lane 0 of the workgroup polls it (relaxed
// system-scope loads + s_sleep), the workgroup loads the job description and
// its payload slots into LDS in ONE burst (one device-memory or PCIe round
// trip), XORs one wave per line, stores the results to the output slots in
// pinned host memory with system-coherent stores, waits for their
// acknowledgements and writes `done`; the job's timestamps follow `done`.  The
// workgroup returns when `stop` is set, after `idle_ticks` without a job, or
// after `life_ticks` in total (every wave leaves through the same uniform
// test); the host relaunches it when a job finds it gone.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rfec_internal.h"
#include "rfec_launch.h"

namespace {

constexpr int kSvcBlock = 256;
constexpr int kSvcLdsChunks = 3840; // 60 KiB of staged 16-byte chunks
constexpr int kSvcU = (kSvcLdsChunks + kSvcBlock - 1) / kSvcBlock; // chunk loads per thread for a full tile
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct SvcArgs {
    rfec_svc_ctl* ctl;   // control block, results side: done / alive / out (device view of host memory)
    rfec_svc_ctl* in;    // control block, request side: bell / stop / quit / job (host-written device
                         // memory when the host can map it, else == ctl)
    const v4u* shards;   // staging slots (device view), C chunks each
    v4u* out;            // output slots
    uint32_t C;          // chunks per slot
    uint64_t idle_ticks; // s_memrealtime ticks without a job before leaving
    uint64_t life_ticks; // ticks in total before leaving
};

__device__ __forceinline__ uint32_t poll_u32(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The results are written with system-coherent buffer stores (sc0 sc1: past
// this CU's L1 and the XCD's L2, to the host memory itself) and drained
// before `done`, so no L2 write-back release is needed (0.4 vs 1.0 us).
constexpr int kSys = 1 | 16; // gfx950 cache-policy bits: sc0 | sc1
// The job's bytes are read with plain loads behind a system-scope acquire
// (tools/svc_ab.sh, a k = 10 group encode: 3.0-3.3 us from the doorbell to the
// job in LDS; the same with the invalidate issued at the end of the previous
// job instead, or with an agent-scope acquire; sc1 loads without an acquire
// 6.0 us; sc0 loads read stale lines from L1).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ v4u ld_job(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, uint32_t off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys32(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint16_t v)
{
    __builtin_amdgcn_raw_buffer_store_b16(v, r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t v)
{
    __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, kSys);
}
#define CTL_OFF(field) ((uint32_t)offsetof(rfec_svc_ctl, field))

// Chunk columns [j0, j0 + tj) of slots [0, ns) into lds (slot s at s tj), all
// loads issued before the first LDS store; stale chunks (past a slot's bytes)
// come along and are masked by the readers.  With `J` (the job description
// copy, first tile), its loads go out in the same burst: one PCIe round trip.
__device__ __forceinline__ void stage_tile(const SvcArgs& A, uint32_t ns, uint32_t j0, uint32_t tj, v4u* lds,
                                           bool jsrc, rfec_svc_job* jdst)
{
    constexpr uint32_t njmax = sizeof(rfec_svc_job) / 16, UJ = (njmax + kSvcBlock - 1) / kSvcBlock;
    static_assert(sizeof(rfec_svc_job) % 16 == 0 && offsetof(rfec_svc_ctl, job) % 16 == 0 &&
                      offsetof(rfec_svc_job, hdr) % 16 == 0, "job layout");
    // the job description up to its ns header records only
    const uint32_t nj = offsetof(rfec_svc_job, hdr) / 16 + (5 * ns + 3) / 4;
    const uint32_t items = max(ns * tj, 1u);
    v4u v[kSvcU], t[UJ];
    // (unconditional loads at clamped indices: under per-load branches hipcc
    // waits on each load before issuing the next)
    const __amdgpu_buffer_rsrc_t rc = sys_rsrc(A.in, sizeof(rfec_svc_ctl));
    const __amdgpu_buffer_rsrc_t rs = sys_rsrc(A.shards, RFEC_SVC_SLOTS * A.C * 16u);
    const uint32_t njr = nj;
#pragma unroll
    for (uint32_t u = 0; u < UJ; ++u)
        t[u] = ld_job(rc, CTL_OFF(job) + 16u * min(u * kSvcBlock + threadIdx.x, njr - 1));
#pragma unroll
    for (int u = 0; u < kSvcU; ++u) {
        const uint32_t it = min(u * kSvcBlock + threadIdx.x, items - 1);
        const uint32_t s = it / max(tj, 1u);
        v[u] = ld_job(rs, 16u * (s * A.C + j0 + (it - s * tj)));
    }
    if (jsrc) {
#pragma unroll
        for (uint32_t u = 0; u < UJ; ++u)
            if (u * kSvcBlock + threadIdx.x < njr)
                reinterpret_cast<v4u*>(jdst)[u * kSvcBlock + threadIdx.x] = t[u];
    }
#pragma unroll
    for (int u = 0; u < kSvcU; ++u) {
        const uint32_t it = u * kSvcBlock + threadIdx.x;
        if (it < ns * tj)
            lds[it] = v[u];
    }
}

constexpr int kSvcWaves = kSvcBlock / 64;
constexpr int kSvcMemU = 4; // members per pass: their loads in flight together

// One XOR line of a tile, on one wave: slots s_q = first + q * stride (q <
// count), lane t on tile columns jb + t and jb + 64 + t.  The host stages
// every slot zero-filled to its end (the zero padding of flex_fec_xor.c:30-32,
// 46-49, 84-86), so whole slots are XORed.  With `hdr_lanes`, lanes 0-4 also
// XOR header word `lane` of the records at hrec + q * hstride and keep the
// largest upper half (the size on lane 4).  nck: the longest member's chunks.
// Every load of a pass goes out before the first is used (members past the
// count read the last one again and are dropped): one LDS round trip per
// kSvcMemU members (a lone wave's job is latency-bound: 1.78 -> 1.51 us for a
// k = 10 group against a wait per member; 8 per pass: 2.12 us).
struct LineAcc {
    v4u a[2];
    uint32_t h, L, nck;
};
__device__ __forceinline__ void line_pass(const rfec_svc_job& J, const v4u* lds, uint32_t tj, uint32_t jb,
                                          uint32_t first, uint32_t stride, uint32_t count, uint32_t hrec,
                                          uint32_t hstride, bool hdr_lanes, LineAcc& R)
{
    const uint32_t lane = threadIdx.x & 63u, hl = min(lane, 4u);
    const uint32_t c0 = min(jb + lane, tj - 1u), c1 = min(jb + 64u + lane, tj - 1u);
    for (uint32_t q0 = 0; q0 < count; q0 += kSvcMemU) {
        uint32_t n[kSvcMemU], h[kSvcMemU];
        v4u x0[kSvcMemU], x1[kSvcMemU];
#pragma unroll
        for (int u = 0; u < kSvcMemU; ++u) {
            const uint32_t q = min(q0 + u, count - 1u);
            const uint32_t sl = first + q * stride;
            n[u] = J.slot_nck[sl];
            x0[u] = lds[sl * tj + c0];
            x1[u] = lds[sl * tj + c1];
            h[u] = J.hdr[5u * (hrec + q * hstride) + hl];
        }
#pragma unroll
        for (int u = 0; u < kSvcMemU; ++u) {
            const bool in = q0 + u < count; // (uniform)
            const bool hin = in && hdr_lanes;
            R.nck = max(R.nck, in ? n[u] : 0u);
            R.a[0] ^= in ? x0[u] : v4u{0, 0, 0, 0};
            R.a[1] ^= in ? x1[u] : v4u{0, 0, 0, 0};
            R.h ^= hin ? h[u] : 0u;
            R.L = max(R.L, hin ? h[u] >> 16 : 0u);
        }
    }
}

// One job, this workgroup's chunk columns [c0, c1) of every slot: staged
// tile by tile (the first tile together with the job description), then one
// wave per line (encode) or per recover job, from LDS.  The header results
// (workgroup 0, first tile) ride along on lanes 0-4 of the same passes:
//   encode line l: meta = XOR of the member records, fec_data_size = the
//     largest member size, status -1 for a single member or a size over
//     capacity (flex_fec_xor.c:9-28)
//   recover job g: recovered record = the parity's meta ^ the members'
//     (records slot0[g], then its members'), status -1 when fec_data_size is
//     over capacity or a member or the recovered size exceeds it
//     (flex_fec_xor.c:64-71, 75-99)
__device__ void svc_job(const SvcArgs& A, uint32_t ns, uint32_t c0, uint32_t c1, bool leader, v4u* lds,
                        rfec_svc_job& J, uint64_t* t1)
{
    const uint32_t C = A.C;
    const uint32_t tmax = ns ? max(1u, min(c1 - c0, (uint32_t)kSvcLdsChunks / ns)) : c1 - c0;
    const __amdgpu_buffer_rsrc_t ro = sys_rsrc(A.out, RFEC_MAX_LINES * C * 16u);
    const __amdgpu_buffer_rsrc_t rc = sys_rsrc(A.ctl, sizeof(rfec_svc_ctl));
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t j0 = c0, first = 1; first || j0 < c1; j0 += tmax, first = 0) {
        const uint32_t tj = j0 < c1 ? min(tmax, c1 - j0) : 0u;
        if (!first)
            __syncthreads(); // the previous tile's readers are done
        stage_tile(A, ns, j0, tj, lds, first, &J);
        __syncthreads();
        if (first && leader && threadIdx.x == 0)
            *t1 = __builtin_amdgcn_s_memrealtime();
        const bool hdr = first && leader;
        const bool enc = J.op == RFEC_SVC_ENCODE;
        const uint32_t nitems = enc ? (uint32_t)J.plan.n_lines : J.groups;
        for (uint32_t x = wv; x < nitems; x += kSvcWaves) {
            uint32_t sf, sstr, cnt, hrec, hstr, bound;
            LineAcc R{{v4u{0, 0, 0, 0}, v4u{0, 0, 0, 0}}, 0u, 0u, 0u};
            if (enc) {
                const rfec_line ln = J.plan.line[x];
                sf = ln.first, sstr = ln.stride, cnt = ln.count, hrec = ln.first, hstr = ln.stride;
            } else { // the members, then the parity slot; records: the parity's, then the members'
                sf = J.slot0[x], sstr = 1u, cnt = J.count[x] + 1u, hrec = J.slot0[x], hstr = 1u;
            }
            for (uint32_t jb = 0; jb < max(tj, 1u); jb += 128u) {
                R.a[0] = R.a[1] = v4u{0, 0, 0, 0};
                if (tj || hdr) // (no columns in this workgroup: the records alone)
                    line_pass(J, lds, max(tj, 1u), jb, sf, sstr, cnt, hrec, hstr, hdr && jb == 0, R);
                bound = enc ? R.nck : (J.fsize[x] + 15u) / 16u; // past fec_data_size: never read back
                if (!tj)
                    break;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t jj = jb + 64u * h + lane;
                    if (jj < tj && j0 + jj < bound)
                        st_sys(ro, 16u * (x * C + j0 + jj), R.a[h]);
                }
            }
            if (hdr && lane < 5u) {
                st_sys32(rc, CTL_OFF(out.meta) + 20u * x + 4u * lane, R.h);
                if (lane == 4u) {
                    if (enc) {
                        st_sys16(rc, CTL_OFF(out.fsize) + 2u * x, (uint16_t)R.L);
                        st_sys8(rc, CTL_OFF(out.status) + x, (cnt <= 1u || R.L > J.capacity) ? 0xFFu : 0u);
                    } else {
                        // R.L: the largest of the parity's and the members' sizes; R.h: the recovered
                        // record's size word.  The parity's own size field is fec_meta's XOR, not a
                        // length: check the members and the recovered size against fec_data_size.
                        const uint32_t L = J.fsize[x];
                        bool ok = L <= J.capacity && (R.h >> 16) <= L;
                        for (uint32_t q = 1; q < cnt; ++q)
                            ok = ok && (J.hdr[5u * (hrec + q) + 4u] >> 16) <= L;
                        st_sys8(rc, CTL_OFF(out.status) + x, ok ? 0u : 0xFFu);
                    }
                }
            }
        }
        if (tj == 0)
            break;
    }
}

// gridDim.x workgroups (<= RFEC_SVC_MAX_GROUPS), workgroup w on chunk columns
// [C w / n, C (w + 1) / n) of every job: the PCIe round trips of a job's
// staging spread over several CUs.  Workgroup 0 leads: it writes the header
// results and the timing, and it alone decides to leave (idle / lifetime):
// `quit`, then `alive` = 0; the others leave on `quit` or `stop` (and, as a
// backstop only, after ten lifetimes: a non-leader that started late must not
// leave while `alive` is 1).  Every workgroup answers in done[w].
__global__ __launch_bounds__(kSvcBlock) void k_service(SvcArgs A)
{
    __shared__ __attribute__((aligned(16))) v4u lds[kSvcLdsChunks];
    __shared__ uint32_t s_ns, s_exit, s_seq;
    __shared__ uint64_t s_t1;
    __shared__ __attribute__((aligned(16))) rfec_svc_job J; // the job description, copied per job
    const uint32_t w = blockIdx.x, nw = gridDim.x;
    const bool leader = w == 0;
    const uint32_t c0 = A.C * w / nw, c1 = A.C * (w + 1) / nw;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t life = leader ? A.life_ticks : 10 * A.life_ticks;
    uint64_t t_last = t_start;
    uint32_t done = poll_u32(&A.ctl->done[w]);
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t ex = 0;
            uint64_t bell = 0;
            for (;;) {
                bell = __hip_atomic_load(&A.in->bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (poll_u32(&A.in->stop) || (!leader && poll_u32(&A.in->quit))) {
                    ex = 1;
                    break;
                }
                if ((uint32_t)bell != done)
                    break;
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if ((leader && now - t_last > A.idle_ticks) || now - t_start > life) {
                    ex = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (ex && leader) { // a job posted after the poll above finds alive == 0 and relaunches
                __hip_atomic_store(&A.in->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&A.ctl->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            s_seq = (uint32_t)bell;
            s_ns = (uint32_t)(bell >> 32) & 0xffffu;
            s_exit = ex;
        }
        __syncthreads();
        if (s_exit) // uniform: every wave leaves here
            return;
        const uint32_t seq = s_seq;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // the job's bytes, written before the doorbell
        svc_job(A, min(s_ns, (uint32_t)RFEC_SVC_SLOTS), c0, c1, leader, lds, J, &s_t1);
        const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
        // every wave's system-coherent stores acknowledged before `done`
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_store(&A.ctl->done[w], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (leader) { // this job's timing (rfec_service_get_info) after `done`: off the call's path
                const __amdgpu_buffer_rsrc_t rc = sys_rsrc(A.ctl, sizeof(rfec_svc_ctl));
                const uint32_t o = CTL_OFF(out.t) + 32u * (seq & 1u);
                st_sys(rc, o, v4u{(uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)s_t1, (uint32_t)(s_t1 >> 32)});
                st_sys(rc, o + 16u, v4u{(uint32_t)t2, (uint32_t)(t2 >> 32), (uint32_t)t3, (uint32_t)(t3 >> 32)});
            }
        }
        done = seq;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

} // namespace

extern "C" int rfec_launch_service(rfec_svc_ctl* ctl, rfec_svc_ctl* in, const uint8_t* shards, uint8_t* out,
                                   uint32_t stride, uint64_t idle_ticks, uint64_t life_ticks, uint32_t groups,
                                   void* stream)
{
    if (stride % 16 || stride / 16 > 255 || groups < 1 || groups > RFEC_SVC_MAX_GROUPS)
        return (int)hipErrorInvalidValue;
    SvcArgs A{ctl, in, reinterpret_cast<const v4u*>(shards), reinterpret_cast<v4u*>(out), stride / 16, idle_ticks,
              life_ticks};
    hipLaunchKernelGGL(k_service, dim3(groups), dim3(kSvcBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}
