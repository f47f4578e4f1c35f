/*
 * stub_hip.c -- TEST INFRASTRUCTURE ONLY, never linked into librazor_fec.so.
 *
 * A host-memory stand-in for the handful of HIP runtime calls and kernel
 * launches rfec_host.c makes, so the host control plane (receiver ingestion,
 * sender staging, argument checks) can run on a machine without a GPU under
 * AddressSanitizer / UBSan.  "Device" pointers are host pointers; copies are
 * memcpy; streams and events are no-ops.
 *
 * The launches do no FEC arithmetic: payload-producing kernels leave their
 * outputs untouched.  Only data movement the host code depends on for its
 * own bookkeeping is mimicked:
 *   - rfec_launch_gather_rows copies rows by the map (so an out-of-range map
 *     index is an ASan report, not silent garbage);
 *   - rfec_launch_recover marks every erased member of every line-covered
 *     group as recovered (the host then reports what it would deliver).
 * Results produced through this stub are never compared as FEC outputs; the
 * tests using it check headers / bookkeeping against the oracle and that the
 * sanitizers stay quiet.
 */
#define _POSIX_C_SOURCE 200809L
#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__ 1
#endif
#include <hip/hip_runtime_api.h>

#include <stdlib.h>
#include <string.h>

#include "rfec_internal.h"

hipError_t hipGetDeviceCount(int* count)
{
    *count = 1;
    return hipSuccess;
}
hipError_t hipGetDevice(int* d)
{
    *d = 0;
    return hipSuccess;
}
/* no wall clock: the drop-in's resident service stays unavailable here and
 * the drop-in takes its per-call launch path */
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t a, int d)
{
    (void)a;
    (void)d;
    *v = 0;
    return hipErrorNotSupported;
}
int rfec_launch_service(rfec_svc_ctl* ctl, rfec_svc_ctl* in, const uint8_t* shards, uint8_t* out, uint32_t stride,
                        uint64_t idle_ticks, uint64_t life_ticks, uint32_t groups, void* stream)
{
    (void)ctl, (void)in, (void)shards, (void)out, (void)stride, (void)idle_ticks, (void)life_ticks, (void)groups,
        (void)stream;
    return (int)hipErrorNotSupported;
}
/* the large-group line jobs: copied through, as the gathers (no FEC arithmetic) */
int rfec_launch_line_jobs(const rfec_line_job* jobs, uint32_t n_jobs, const int32_t* members, const uint8_t* rows,
                          uint8_t* outrows, uint32_t stride, void* stream)
{
    (void)stream;
    for (uint32_t q = 0; q < n_jobs; ++q) {
        const rfec_line_job* J = &jobs[q];
        memcpy(outrows + (size_t)J->out * stride, rows + (size_t)J->parity * stride, stride);
        for (uint32_t i = 0; i < J->n_members; ++i) { /* every member code must address a valid row */
            const int32_t m = members[J->member0 + i];
            const uint8_t* src = m >= 0 ? rows + (size_t)m * stride : outrows + (size_t)(-1 - m) * stride;
            outrows[(size_t)J->out * stride] ^= src[0];
        }
    }
    return 0;
}
hipError_t hipMalloc(void** p, size_t n)
{
    *p = malloc(n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p)
{
    free(p);
    return hipSuccess;
}
/* device memory the host could map: none here (the service keeps its request side in host memory) */
hipError_t hipExtMallocWithFlags(void** p, size_t n, unsigned int flags)
{
    (void)n, (void)flags;
    *p = NULL;
    return hipErrorOutOfMemory;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int flags)
{
    (void)flags;
    return hipMalloc(p, n);
}
hipError_t hipHostFree(void* p) { return hipFree(p); }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int flags)
{
    (void)flags;
    *d = h;
    return hipSuccess;
}
/* no memory is "pinned" here: the callers' copy paths run */
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p)
{
    (void)p;
    memset(a, 0, sizeof(*a));
    return hipErrorInvalidValue;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s)
{
    (void)kind, (void)s;
    if (n)
        memmove(dst, src, n);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int flags)
{
    (void)flags;
    *s = (hipStream_t)malloc(1);
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s)
{
    free(s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s)
{
    (void)s;
    return hipSuccess;
}
hipError_t hipStreamQuery(hipStream_t s)
{
    (void)s;
    return hipSuccess;
}
hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi)
{
    *lo = 0;
    *hi = -1;
    return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned int flags, int prio)
{
    (void)flags;
    (void)prio;
    *s = (hipStream_t)malloc(1);
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e)
{
    *e = (hipEvent_t)malloc(1);
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned flags)
{
    (void)flags;
    return hipEventCreate(e);
}
hipError_t hipEventDestroy(hipEvent_t e)
{
    free(e);
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s)
{
    (void)e, (void)s;
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int flags)
{
    (void)s, (void)e, (void)flags;
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e)
{
    (void)e;
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b)
{
    (void)a, (void)b;
    *ms = 0.f;
    return hipSuccess;
}

int rfec_launch_encode(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                       const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                       uint16_t* fsize, int8_t* status, void* stream, unsigned flags)
{
    return 0;
}

int rfec_launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                        uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fsize, const uint64_t* parity_present,
                        uint64_t* recovered, void* ws, void* stream, unsigned flags)
{
    uint64_t all0 = 0, all1 = 0;
    for (uint32_t l = 0; l < M->plan.n_lines; ++l) {
        all0 |= M->mask[l][0];
        all1 |= M->mask[l][1];
    }
    for (uint32_t g = 0; g < groups; ++g) {
        recovered[2 * g] = all0 & ~present[2 * g];
        recovered[2 * g + 1] = all1 & ~present[2 * g + 1];
    }
    return 0;
}

/* dense output form (the receiver session's device peel): as rfec_launch_recover, for the erased members
 * of rank < per_group; out_index names them */
int rfec_launch_recover_out(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                            const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                            const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                            const uint64_t* parity_present, uint64_t* recovered, void* ws, void* stream,
                            unsigned flags, const rfec_dense_out* out)
{
    (void)stride, (void)capacity, (void)shards, (void)hdr, (void)parity, (void)meta, (void)fsize;
    (void)parity_present, (void)ws, (void)stream, (void)flags;
    uint64_t all[2] = {0, 0};
    for (uint32_t l = 0; l < M->plan.n_lines; ++l) {
        all[0] |= M->mask[l][0];
        all[1] |= M->mask[l][1];
    }
    for (uint32_t g = 0; g < groups; ++g) {
        uint32_t e = 0;
        recovered[2 * g] = recovered[2 * g + 1] = 0;
        for (uint32_t i = 0; i < M->plan.k && e < out->per_group; ++i) {
            if ((present[2 * g + (i >> 6)] >> (i & 63)) & 1ull)
                continue;
            const int ok = (int)((all[i >> 6] >> (i & 63)) & 1ull);
            if (ok)
                recovered[2 * g + (i >> 6)] |= 1ull << (i & 63);
            out->index[(size_t)g * out->per_group + e++] = ok ? (uint8_t)i : 0xFF;
        }
    }
    return 0;
}

/* packed erasure records: not used by the host control plane; refused */
int rfec_launch_pack_rows(const rfec_kplan* P, uint32_t col, uint32_t groups, const rfec_hdr* hdr,
                          const uint64_t* present, const rfec_hdr* meta, const uint16_t* fsize,
                          const uint64_t* parity_present, uint32_t per_group, uint8_t* packed, uint32_t pk_stride,
                          uint32_t pk_slot, void* stream)
{
    (void)P, (void)col, (void)groups, (void)hdr, (void)present, (void)meta, (void)fsize, (void)parity_present;
    (void)per_group, (void)packed, (void)pk_stride, (void)pk_slot, (void)stream;
    return (int)hipErrorInvalidValue;
}

int rfec_launch_recover_packed(const rfec_kmask* M, uint32_t col, uint32_t groups, uint32_t stride,
                               uint32_t capacity, const uint8_t* shards, const uint8_t* parity, const uint8_t* packed,
                               uint32_t pk_stride, uint32_t pk_slot, uint64_t* recovered,
                               const rfec_dense_out* out, void* stream)
{
    (void)M, (void)col, (void)groups, (void)stride, (void)capacity, (void)shards, (void)parity, (void)packed;
    (void)pk_stride, (void)pk_slot, (void)recovered, (void)out, (void)stream;
    return (int)hipErrorInvalidValue;
}

int rfec_launch_wire_frame_fec(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                               const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                               const rfec_fec_stamp* stamps, const uint32_t* order, uint32_t dstride,
                               uint8_t* dgram, uint16_t* dlen, void* stream)
{
    return 0;
}

int rfec_launch_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                               const rfec_hdr* hdr, const rfec_seg_stamp* stamps, const uint32_t* order,
                               uint32_t dstride, uint8_t* dgram, uint16_t* dlen, uint32_t rows_out, void* stream)
{
    return 0;
}

int rfec_launch_wire_parse(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                           uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                           uint32_t max_len, void* stream)
{
    return 0;
}

int rfec_launch_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                            void* stream)
{
    for (uint32_t r = 0; r < rows; ++r) {
        if (map[r] >= 0)
            memcpy(dst + (size_t)r * stride, src + (size_t)map[r] * stride, stride);
        else
            memset(dst + (size_t)r * stride, 0, stride);
    }
    return 0;
}

int rfec_launch_wire_parse_split(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                                 uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                                 uint32_t max_len, rfec_rx_split* split, uint32_t shards, void* stream)
{
    rfec_launch_wire_parse(n, dstride, dgram, dlen, stride, capacity, recs, payload, max_len, stream);
    return split ? rfec_launch_rx_split(recs, n, shards, split, stream) : 0;
}

/* the receiver session's device stage: the gather and the table copy */
int rfec_launch_rx_stage(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                         void* tdst, const void* tsrc, size_t tbytes, void* stream)
{
    rfec_launch_gather_rows(dst, src, map, rows, stride, stream);
    if (tbytes)
        memcpy(tdst, tsrc, tbytes);
    return 0;
}

/* the receiver session's batch split (k_rx_split): the same summary on the host */
int rfec_launch_rx_split(const rfec_wire_rec* recs, uint32_t n, uint32_t T, rfec_rx_split* out, void* stream)
{
    (void)stream;
    for (uint32_t p = 0; p < n; ++p) {
        const rfec_wire_rec* r = &recs[p];
        rfec_rx_split e = {0xFF, RX_SPLIT_NONE, 0, 0};
        if (r->status == RFEC_WIRE_OK && r->mid == RFEC_WIRE_SEG) {
            e.shard = (uint8_t)((r->fec_id ? r->fec_id : r->hdr.seq) % T);
            e.kind = r->fec_id && r->hdr.seq ? RX_SPLIT_SEG_TS : RX_SPLIT_SEG;
            e.value = r->hdr.ts;
        } else if (r->status == RFEC_WIRE_OK && r->mid == RFEC_WIRE_FEC) {
            e.shard = (uint8_t)(r->fec_id % T);
            e.kind = RX_SPLIT_FEC;
            e.value = r->send_ts + 3000u;
        }
        out[p] = e;
    }
    return 0;
}

int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream)
{
    return 0;
}

/* the zero-copy host-memory paths: not exercised here (no pinned blocks are
 * registered through the stub), refused if reached */
int rfec_launch_host_gather(const uint64_t* sptrs, uint32_t ns, uint8_t* shards, rfec_hdr* hdr,
                            const uint64_t* fptrs, uint32_t nf, uint8_t* parity, rfec_hdr* meta, uint16_t* fsize,
                            uint16_t* fecid, uint32_t stride, uint32_t video, const uint64_t* aux_src,
                            uint64_t* aux_dst, uint32_t aux_n, void* stream)
{
    (void)sptrs, (void)ns, (void)shards, (void)hdr, (void)fptrs, (void)nf, (void)parity, (void)meta, (void)fsize,
        (void)fecid, (void)stride, (void)video, (void)aux_src, (void)aux_dst, (void)aux_n, (void)stream;
    return (int)hipErrorNotSupported;
}
int rfec_launch_send_gather(const uint64_t* src, const uint16_t* size, uint32_t slots, uint32_t stride, uint8_t* dst,
                            void* stream)
{
    (void)stream;
    for (uint32_t s = 0; s < slots; ++s) {
        memset(dst + (size_t)s * stride, 0, stride);
        if (src[s])
            memcpy(dst + (size_t)s * stride, (const void*)(uintptr_t)src[s], size[s]);
    }
    return 0;
}
int rfec_launch_host_scatter_fec(const uint64_t* fptrs, uint32_t groups, const rfec_kplan* P, uint32_t stride,
                                 const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                                 const int8_t* status, const rfec_hdr* hdr, uint16_t fec_id0, uint32_t g0,
                                 uint32_t video, void* stream)
{
    (void)fptrs, (void)groups, (void)P, (void)stride, (void)parity, (void)meta, (void)fsize, (void)status,
        (void)hdr, (void)fec_id0, (void)g0, (void)video, (void)stream;
    return (int)hipErrorNotSupported;
}
int rfec_launch_host_scatter_seg(const uint64_t* optrs, uint32_t groups, uint32_t E, uint32_t stride,
                                 const uint8_t* out_shards, const rfec_hdr* out_hdr, const uint8_t* out_index,
                                 const uint16_t* fecid, const uint64_t* ppm, uint32_t n_lines, uint32_t video,
                                 uint8_t* oidx_host, const uint64_t* recovered, uint64_t* rec_host, void* stream)
{
    (void)optrs, (void)groups, (void)E, (void)stride, (void)out_shards, (void)out_hdr, (void)out_index,
        (void)fecid, (void)ppm, (void)n_lines, (void)video, (void)oidx_host, (void)recovered, (void)rec_host,
        (void)stream;
    return (int)hipErrorNotSupported;
}
const char* rfec_hip_error_string(int code) { return code ? "stub error" : "no error"; }

/* HBM probes: not available without a device */
int rfec_probe_read(const void* src, size_t bytes, void* sink, unsigned flags, void* stream) { return 1; }
int rfec_probe_copy(const void* src, void* dst, size_t bytes, unsigned flags, void* stream) { return 1; }
int rfec_probe_write(void* dst, size_t bytes, unsigned flags, void* stream) { return 1; }
