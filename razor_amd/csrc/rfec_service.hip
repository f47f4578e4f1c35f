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
// control block), then bumps `req`; lane 0 of the workgroup polls `req`
// (relaxed system-scope loads + s_sleep), the workgroup stages every member
// slot it needs into LDS in one burst of loads, XORs, stores the results to
// the staging area, releases at system scope and writes `done` = req.  The
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
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct SvcArgs {
    rfec_svc_ctl* ctl;   // control block (device view of host memory)
    const v4u* shards;   // staging slots (device view), C chunks each
    v4u* parity;         // encode: parity slots; recover: the parity inputs
    uint32_t C;          // chunks per slot
    uint64_t idle_ticks; // s_memrealtime ticks without a job before leaving
    uint64_t life_ticks; // ticks in total before leaving
};

__device__ __forceinline__ uint32_t poll_u32(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ const v4u* slot_src(const SvcArgs& A, uint32_t code)
{
    return (code & RFEC_SVC_PARITY_SLOT) ? A.parity + (size_t)(code & ~RFEC_SVC_PARITY_SLOT) * A.C
                                         : A.shards + (size_t)code * A.C;
}

// Chunk columns [j0, j0 + tj) of the job's ns slots into lds (slot s at s * tj),
// chunks at or past a slot's valid count as zero; every load of the tile is
// issued before the first LDS store waits on one.
__device__ __forceinline__ void stage_tile(const SvcArgs& A, const rfec_svc_job& J, uint32_t ns, uint32_t j0,
                                           uint32_t tj, v4u* lds)
{
    constexpr int U = 8;
    const uint32_t items = ns * tj;
    for (uint32_t base = 0; base < items; base += U * kSvcBlock) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t it = base + u * kSvcBlock + threadIdx.x;
            v[u] = v4u{0, 0, 0, 0};
            if (it < items) {
                const uint32_t s = it / tj, j = j0 + (it - s * tj);
                if (j < J.slot_nck[s])
                    v[u] = slot_src(A, J.slot_src[s])[j];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t it = base + u * kSvcBlock + threadIdx.x;
            if (it < items)
                lds[it] = v[u];
        }
    }
}

// encode: line l's meta / fec_data_size / status from the member headers (the
// job's hdr words, member i at 5 i), flex_fec_xor.c:9-28
__device__ void svc_encode_meta(const SvcArgs& A, const rfec_svc_job& J, uint16_t* fsz)
{
    const rfec_kplan& P = J.plan;
    for (uint32_t l = threadIdx.x; l < P.n_lines; l += kSvcBlock) {
        const rfec_line ln = P.line[l];
        uint32_t m[5] = {0, 0, 0, 0, 0}, L = 0;
        for (uint32_t q = 0; q < ln.count; ++q) {
            const uint32_t* r = J.hdr + 5u * (ln.first + q * ln.stride);
#pragma unroll
            for (int d = 0; d < 5; ++d)
                m[d] ^= r[d];
            L = max(L, r[4] >> 16);
        }
#pragma unroll
        for (int d = 0; d < 5; ++d)
            A.ctl->out.meta[l][d] = m[d];
        A.ctl->out.fsize[l] = (uint16_t)L;
        A.ctl->out.status[l] = (ln.count <= 1 || L > J.capacity) ? (int8_t)-1 : (int8_t)0;
        fsz[l] = (uint16_t)L;
    }
}

// recover: job g's recovered header (meta ^ members) and verdict,
// flex_fec_xor.c:64-71, 75-99; the job's hdr words: meta at 5 hdr0[g], then
// its members
__device__ void svc_recover_meta(const SvcArgs& A, const rfec_svc_job& J)
{
    for (uint32_t g = threadIdx.x; g < J.groups; g += kSvcBlock) {
        const uint32_t* r = J.hdr + 5u * J.hdr0[g];
        const uint32_t L = J.fsize[g];
        uint32_t m[5];
#pragma unroll
        for (int d = 0; d < 5; ++d)
            m[d] = r[d];
        bool ok = L <= J.capacity;
        for (uint32_t q = 1; q <= J.count[g]; ++q) {
#pragma unroll
            for (int d = 0; d < 5; ++d)
                m[d] ^= r[5 * q + d];
            ok = ok && (r[5 * q + 4] >> 16) <= L;
        }
        ok = ok && (m[4] >> 16) <= L;
#pragma unroll
        for (int d = 0; d < 5; ++d)
            A.ctl->out.meta[g][d] = m[d];
        A.ctl->out.status[g] = ok ? (int8_t)0 : (int8_t)-1;
    }
}

__device__ void svc_job(const SvcArgs& A, const rfec_svc_job& J, v4u* lds, uint16_t* fsz)
{
    const uint32_t ns = J.n_slots;
    if (J.op == RFEC_SVC_ENCODE)
        svc_encode_meta(A, J, fsz);
    else
        svc_recover_meta(A, J);
    const uint32_t C = A.C;
    const uint32_t tmax = ns ? min(C, (uint32_t)kSvcLdsChunks / ns) : C;
    for (uint32_t j0 = 0; j0 < C; j0 += tmax) {
        const uint32_t tj = min(tmax, C - j0);
        __syncthreads(); // the previous tile's readers are done (and fsz is written)
        stage_tile(A, J, ns, j0, tj, lds);
        __syncthreads();
        if (J.op == RFEC_SVC_ENCODE) {
            const rfec_kplan& P = J.plan;
            for (uint32_t it = threadIdx.x; it < P.n_lines * tj; it += kSvcBlock) {
                const uint32_t l = it / tj, jj = it - l * tj;
                const rfec_line ln = P.line[l];
                if (j0 + jj >= (fsz[l] + 15u) / 16u) // past fec_data_size: never read back
                    continue;
                v4u acc = lds[ln.first * tj + jj];
                for (uint32_t q = 1; q < ln.count; ++q)
                    acc ^= lds[(ln.first + q * ln.stride) * tj + jj];
                A.parity[(size_t)l * C + j0 + jj] = acc;
            }
        } else {
            for (uint32_t it = threadIdx.x; it < J.groups * tj; it += kSvcBlock) {
                const uint32_t g = it / tj, jj = it - g * tj;
                if (j0 + jj >= (J.fsize[g] + 15u) / 16u)
                    continue;
                const uint32_t s0 = J.slot0[g], n = J.count[g];
                v4u acc = lds[(s0 + n) * tj + jj]; // the parity slot follows the members
                for (uint32_t q = 0; q < n; ++q)
                    acc ^= lds[(s0 + q) * tj + jj];
                const_cast<v4u*>(A.shards)[(size_t)J.out_slot[g] * C + j0 + jj] = acc;
            }
        }
    }
}

__global__ __launch_bounds__(kSvcBlock) void k_service(SvcArgs A)
{
    __shared__ __attribute__((aligned(16))) v4u lds[kSvcLdsChunks];
    __shared__ uint32_t s_cmd, s_exit;
    __shared__ uint16_t fsz[RFEC_MAX_LINES];
    // the job description, copied once per job from host memory
    __shared__ __attribute__((aligned(16))) rfec_svc_job J;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = t_start;
    uint32_t done = poll_u32(&A.ctl->done);
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t cmd = done, ex = 0;
            for (;;) {
                const uint32_t r = poll_u32(&A.ctl->req);
                if (poll_u32(&A.ctl->stop)) {
                    __hip_atomic_store(&A.ctl->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    ex = 1;
                    break;
                }
                if (r != done) {
                    cmd = r;
                    break;
                }
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if (now - t_last > A.idle_ticks || now - t_start > A.life_ticks) {
                    // a job posted after the poll above finds alive == 0 and relaunches
                    __hip_atomic_store(&A.ctl->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    ex = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_cmd = cmd;
            s_exit = ex;
        }
        __syncthreads();
        if (s_exit) // uniform: every wave leaves here
            return;
        const uint32_t cmd = s_cmd;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // the job's bytes, written before req
        { // one burst of 16-byte loads
            static_assert(sizeof(rfec_svc_job) % 16 == 0 && offsetof(rfec_svc_ctl, job) % 16 == 0, "job layout");
            constexpr uint32_t nv = sizeof(rfec_svc_job) / 16, U = (nv + kSvcBlock - 1) / kSvcBlock;
            const v4u* src = reinterpret_cast<const v4u*>(&A.ctl->job);
            v4u* dst = reinterpret_cast<v4u*>(&J);
            v4u t[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (u * kSvcBlock + threadIdx.x < nv)
                    t[u] = src[u * kSvcBlock + threadIdx.x];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (u * kSvcBlock + threadIdx.x < nv)
                    dst[u * kSvcBlock + threadIdx.x] = t[u];
        }
        __syncthreads();
        svc_job(A, J, lds, fsz);
        // every wave's stores complete and visible to the host before `done`
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(&A.ctl->done, cmd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        done = cmd;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

} // namespace

extern "C" int rfec_launch_service(rfec_svc_ctl* ctl, const uint8_t* shards, uint8_t* parity, uint32_t stride,
                                   uint64_t idle_ticks, uint64_t life_ticks, void* stream)
{
    if (stride % 16 || stride / 16 > 255)
        return (int)hipErrorInvalidValue;
    SvcArgs A{ctl, reinterpret_cast<const v4u*>(shards), reinterpret_cast<v4u*>(parity), stride / 16, idle_ticks,
              life_ticks};
    hipLaunchKernelGGL(k_service, dim3(1), dim3(kSvcBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}
