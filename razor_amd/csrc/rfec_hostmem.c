/*
 * rfec_hostmem.c -- the host-memory batch paths: rfec_host_encode_groups
 * (sim_segment_t in, sim_fec_t out) and rfec_host_recover_groups (received
 * sim_segment_t / sim_fec_t in, recovered segments out), chunked and
 * double-buffered over two streams (gather -> H2D -> kernels -> D2H -> scatter).
 */
#define _POSIX_C_SOURCE 200809L
#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__ 1
#endif
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "razor_fec.h"
#include "rfec_internal.h"
#include "rfec_host_internal.h"

/* ------------------------------------------------------------------------ */
/* 4. host-resident batch (gather -> H2D -> encode -> D2H -> scatter)        */
/* ------------------------------------------------------------------------ */
typedef struct {
    size_t shards, hdr, parity, meta, fsize, status, in_bytes, total;
} hb_layout;

static hb_layout hb_offsets(uint32_t G, uint32_t k, uint32_t n)
{
    hb_layout L;
    size_t o = 0;
#define HB_TAKE(field, bytes)                       \
    do {                                             \
        L.field = o;                                 \
        o = (o + (size_t)(bytes) + 255) & ~(size_t)255; \
    } while (0)
    HB_TAKE(shards, (size_t)G * k * DI_STRIDE);
    HB_TAKE(hdr, (size_t)G * k * sizeof(rfec_hdr));
    L.in_bytes = o; /* [shards, hdr] go host -> device in one copy */
    HB_TAKE(parity, (size_t)G * n * DI_STRIDE);
    HB_TAKE(meta, (size_t)G * n * sizeof(rfec_hdr));
    HB_TAKE(fsize, (size_t)G * n * sizeof(uint16_t));
    HB_TAKE(status, (size_t)G * n);
#undef HB_TAKE
    L.total = o;
    return L;
}

/* two staging slots: host_slot bytes of pinned memory and dev_slot bytes of
 * device memory each (the recover path keeps device-only regions past the
 * host-mirrored ones, so dev_slot >= host_slot there) */
static int hb_reserve(di_ctx* c, size_t host_slot, size_t dev_slot, uint32_t nslot)
{
    hipError_t e;
    if (!c->have_ev) {
        /* stream 0 at the lowest priority: the zero-copy paths run their PCIe-bound
         * gathers on it, and the encode / decode and scatters queued on stream 1
         * then get CUs at once instead of waiting behind the gathers' waves (the
         * highest priority is the resident service's queue) */
        int prio_lo = 0, prio_hi = 0;
        if ((e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "stream priorities", e);
        for (int s = 0; s < 2; ++s)
            if ((e = s == 0 ? hipStreamCreateWithPriority(&c->bstream[s], hipStreamNonBlocking, prio_lo)
                            : hipStreamCreateWithFlags(&c->bstream[s], hipStreamNonBlocking)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "stream create", e);
        for (int s = 0; s < RFEC_HB_SLOTS; ++s)
            for (int i = 0; i < 4; ++i)
                if ((e = hipEventCreate(&c->ev[s][i])) != hipSuccess)
                    return set_err(RFEC_EDEVICE, "event create", e);
        c->have_ev = 1;
    }
    host_slot *= nslot;
    dev_slot *= nslot;
    if (c->bh_bytes < host_slot) {
        if (c->bh)
            (void)hipHostFree(c->bh);
        c->bh = c->bh_dev = NULL;
        c->bh_bytes = 0;
        if ((e = hipHostMalloc((void**)&c->bh, host_slot, hipHostMallocDefault)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "pinned staging", e);
        void* d = NULL;
        if ((e = hipHostGetDevicePointer(&d, c->bh, 0)) != hipSuccess || !d) {
            (void)hipHostFree(c->bh);
            c->bh = NULL;
            return set_err(RFEC_EDEVICE, "pinned staging: no device address", e);
        }
        c->bh_dev = (uint8_t*)d;
        c->bh_bytes = host_slot;
    }
    if (c->bd_bytes < dev_slot) {
        if (c->bd)
            (void)hipFree(c->bd);
        c->bd = NULL;
        c->bd_bytes = 0;
        if ((e = hipMalloc((void**)&c->bd, dev_slot)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "device staging", e);
        c->bd_bytes = dev_slot;
    }
    return RFEC_OK;
}

#define RFEC_HR_SLOT_BYTES ((size_t)640 << 20)

/* ---- pinned blocks the device maps ---------------------------------------
 * rfec_pinned_alloc registers each block (host range and the device address
 * of its first byte), so that the host-memory batch paths can tell that every
 * struct of a call lies in memory the device reads and writes itself: then
 * the zero-copy form runs (rfec_hostio.hip kernels read the callers' structs
 * over PCIe and write the results into theirs; no host gather / scatter, no
 * bulk copies).  Any struct outside a registered block keeps the staged form. */
typedef struct {
    uintptr_t lo, hi;
    intptr_t delta; /* device address - host address */
} pin_block;
static pin_block* g_pin;
static size_t g_npin, g_pincap;
static pthread_mutex_t g_pin_mu = PTHREAD_MUTEX_INITIALIZER;

void* rfec_pinned_alloc(size_t bytes)
{
    void* p = NULL;
    void* d = NULL;
    hipError_t e;
    if (bytes == 0)
        return NULL;
    if ((e = hipHostMalloc(&p, bytes, hipHostMallocDefault)) != hipSuccess) {
        set_err(RFEC_ENOMEM, "pinned alloc", e);
        return NULL;
    }
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return p; /* pinned, but not registered for the zero-copy paths */
    }
    pthread_mutex_lock(&g_pin_mu);
    if (g_npin == g_pincap) {
        const size_t cap = g_pincap ? 2 * g_pincap : 16;
        pin_block* nb = (pin_block*)realloc(g_pin, cap * sizeof(pin_block));
        if (nb) {
            g_pin = nb;
            g_pincap = cap;
        }
    }
    if (g_npin < g_pincap)
        g_pin[g_npin++] = (pin_block){(uintptr_t)p, (uintptr_t)p + bytes, (intptr_t)((uintptr_t)d - (uintptr_t)p)};
    pthread_mutex_unlock(&g_pin_mu);
    return p;
}

void rfec_pinned_free(void* p)
{
    if (!p)
        return;
    pthread_mutex_lock(&g_pin_mu);
    for (size_t i = 0; i < g_npin; ++i)
        if (g_pin[i].lo == (uintptr_t)p) {
            g_pin[i] = g_pin[--g_npin];
            break;
        }
    pthread_mutex_unlock(&g_pin_mu);
    (void)hipHostFree(p);
}

/* 1 when every non-NULL pointer of ptrs[0, n) addresses `obj` bytes inside one
 * registered block (its device offset in *delta); 1 with delta 0 when all are
 * NULL.  0 when a pointer is not 4-byte aligned: the zero-copy kernels move
 * the structs in dwords and use the pointers' low 2 bits as flags
 * (rfec_hostio.hip), so such a batch takes the staged form. */
static int pinned_span(const void* const* ptrs, size_t n, size_t obj, intptr_t* delta)
{
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    *delta = 0;
    for (size_t i = 0; i < n; ++i) {
        const uintptr_t a = (uintptr_t)ptrs[i];
        if (!a)
            continue;
        if (a & 3u)
            return 0;
        lo = a < lo ? a : lo;
        hi = a > hi ? a : hi;
    }
    if (lo == UINTPTR_MAX)
        return 1;
    hi += obj;
    int ok = 0;
    pthread_mutex_lock(&g_pin_mu);
    for (size_t i = 0; i < g_npin && !ok; ++i)
        if (lo >= g_pin[i].lo && hi <= g_pin[i].hi) {
            ok = 1;
            *delta = g_pin[i].delta;
        }
    pthread_mutex_unlock(&g_pin_mu);
    return ok;
}

static int zerocopy_enabled(void)
{
    const char* v = getenv("RFEC_HOST_ZEROCOPY");
    return !(v && v[0] == '0');
}

int zerocopy_on(void) { return zerocopy_enabled(); }

/* 1 when [lo, hi) lies inside one registered block (its device offset in *delta) */
int pinned_range(uintptr_t lo, uintptr_t hi, intptr_t* delta)
{
    int ok = 0;
    *delta = 0;
    pthread_mutex_lock(&g_pin_mu);
    for (size_t i = 0; i < g_npin && !ok; ++i)
        if (lo >= g_pin[i].lo && hi <= g_pin[i].hi) {
            ok = 1;
            *delta = g_pin[i].delta;
        }
    pthread_mutex_unlock(&g_pin_mu);
    return ok;
}

/* groups per zero-copy chunk: RFEC_ZC_CHUNK (measurement knob) or G / 8, at least 2,048 */
static uint32_t zc_chunk(uint32_t groups)
{
    const char* v = getenv("RFEC_ZC_CHUNK");
    uint32_t chunk = v && atoi(v) > 0 ? (uint32_t)atoi(v) : (groups + 7) / 8;
    if (!(v && atoi(v) > 0) && chunk < 2048)
        chunk = 2048;
    return chunk;
}

/* device addresses of structs (0 for NULL) into a pinned table */
static void dev_ptrs(uint64_t* out, const void* const* ptrs, size_t n, intptr_t delta)
{
    for (size_t i = 0; i < n; ++i)
        out[i] = ptrs[i] ? (uint64_t)((uintptr_t)ptrs[i] + (uintptr_t)delta) : 0u;
}

/* the sender's fec_id sequence: +1 per group, 0 skipped (flex_fec_sender.c:241-243) */
static uint16_t fec_id_at(uint16_t id0, uint32_t g)
{
    const uint32_t base = id0 ? (uint32_t)id0 - 1u : 0u;
    return (uint16_t)((base + g) % 65535u + 1u);
}

typedef struct {
    const rfec_plan* plan;
    sim_segment_t* const* segs; /* first segment of the chunk */
    sim_fec_t* const* fecs;     /* first parity of the chunk */
    uint8_t* slot;              /* host staging slot */
    hb_layout L;
    uint32_t g0;                /* global index of the chunk's first group */
    uint16_t fec_id0;
} hb_chunk;

/* gather: AoS segments (payload at offset 34, not 16-B aligned) -> SoA slots */
static void hb_gather(void* arg, size_t lo, size_t hi)
{
    const hb_chunk* h = (const hb_chunk*)arg;
    rfec_hdr* hh = (rfec_hdr*)(h->slot + h->L.hdr);
    for (size_t s = lo; s < hi; ++s) {
        const sim_segment_t* seg = h->segs[s];
        stage_payload(h->slot + h->L.shards + s * DI_STRIDE, seg->data, seg->data_size);
        seg_to_hdr(seg, &hh[s]);
    }
}

/* scatter into the caller's sim_fec_t, stamped as flex_fec_sender_update does */
static void hb_scatter(void* arg, size_t lo, size_t hi)
{
    const hb_chunk* h = (const hb_chunk*)arg;
    const rfec_plan* plan = h->plan;
    const uint32_t k = plan->k, n = plan->n_lines;
    const rfec_hdr* hh = (const rfec_hdr*)(h->slot + h->L.hdr);
    const rfec_hdr* mh = (const rfec_hdr*)(h->slot + h->L.meta);
    const uint16_t* fs = (const uint16_t*)(h->slot + h->L.fsize);
    const int8_t* st = (const int8_t*)(h->slot + h->L.status);
    for (size_t g = lo; g < hi; ++g) {
        uint32_t base = hh[g * k].seq;
        for (uint32_t i = 1; i < k; ++i)
            base = hh[g * k + i].seq < base ? hh[g * k + i].seq : base;
        for (uint32_t l = 0; l < n; ++l) {
            const size_t o = g * n + l;
            sim_fec_t* f = h->fecs[o];
            f->fec_id = fec_id_at(h->fec_id0, h->g0 + (uint32_t)g);
            f->base_id = base;
            f->row = plan->row;
            f->col = plan->col;
            f->index = plan->line[l].index;
            f->count = plan->k;
            if (st[o] != 0) {
                f->fec_data_size = 0xFFFF;
                continue;
            }
            memcpy(&f->fec_meta, &mh[o], sizeof(rfec_hdr));
            f->fec_data_size = fs[o];
            memcpy(f->fec_data, h->slot + h->L.parity + o * DI_STRIDE, fs[o]);
        }
    }
}

/* The zero-copy encode: per chunk, the host writes the structs' device
 * addresses into pinned slot s; on the device the gather stream reads the
 * segments from the callers' structs into HBM slot s, and the second stream
 * (after that gather's event) encodes and scatters the parities into the
 * callers' sim_fec_t.  Gathers follow each other on their own stream, so
 * chunk c's PCIe writes run beside chunk c+1's PCIe reads (with one stream
 * per slot, both slots' gathers ran together and then both scatters: the
 * link saw reads, then writes, 20.3 vs ~18 ms for c3). */
typedef struct {
    size_t sp, fp, shards, hdr, parity, meta, fsize, status, total, host_total;
} hz_layout;

static hz_layout hz_offsets(uint32_t G, uint32_t k, uint32_t n)
{
    hz_layout L;
    size_t o = 0;
#define HZ_TAKE(field, bytes)                           \
    do {                                                \
        L.field = o;                                    \
        o = (o + (size_t)(bytes) + 255) & ~(size_t)255; \
    } while (0)
    HZ_TAKE(sp, (size_t)G * k * 8);
    HZ_TAKE(fp, (size_t)G * n * 8);
    L.host_total = o; /* the pointer tables: pinned, copied H2D */
    HZ_TAKE(shards, (size_t)G * k * DI_STRIDE);
    HZ_TAKE(hdr, (size_t)G * k * sizeof(rfec_hdr));
    HZ_TAKE(parity, (size_t)G * n * DI_STRIDE);
    HZ_TAKE(meta, (size_t)G * n * sizeof(rfec_hdr));
    HZ_TAKE(fsize, (size_t)G * n * sizeof(uint16_t));
    HZ_TAKE(status, (size_t)G * n);
#undef HZ_TAKE
    L.total = o;
    return L;
}

static int zc_encode_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                            sim_fec_t* const* fecs, uint16_t fec_id0, rfec_host_timing* timing, intptr_t ds,
                            intptr_t df)
{
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const uint32_t k = plan->k, n = plan->n_lines;
    uint32_t chunk = zc_chunk(groups);
    chunk = chunk > groups ? groups : chunk;
    const uint32_t nch = (groups + chunk - 1) / chunk;
    const hz_layout L = hz_offsets(chunk, k, n);
    int rc = hb_reserve(c, L.host_total, L.total, RFEC_HB_SLOTS);
    if (rc)
        return rc;
    double tab_us = 0, h2d_us = 0, kernel_us = 0, d2h_us = 0;
    const double t0 = now_us();
    for (uint32_t it = 0; it < nch + RFEC_HB_SLOTS && rc == RFEC_OK; ++it) {
        if (it >= RFEC_HB_SLOTS) { /* retire chunk it - RFEC_HB_SLOTS: its slot may be refilled */
            const uint32_t s = (it - RFEC_HB_SLOTS) % RFEC_HB_SLOTS;
            const hipError_t e = hipEventSynchronize(c->ev[s][3]);
            if (e != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "zero-copy encode wait", e);
                break;
            }
            float a = 0, b = 0, d = 0;
            (void)hipEventElapsedTime(&a, c->ev[s][0], c->ev[s][1]);
            (void)hipEventElapsedTime(&b, c->ev[s][1], c->ev[s][2]);
            (void)hipEventElapsedTime(&d, c->ev[s][2], c->ev[s][3]);
            h2d_us += a * 1e3;
            kernel_us += b * 1e3;
            d2h_us += d * 1e3;
        }
        if (it >= nch)
            continue;
        const uint32_t s = it % RFEC_HB_SLOTS, g0 = it * chunk, ng = it == nch - 1 ? groups - g0 : chunk;
        uint8_t* h = c->bh + (size_t)s * L.host_total;
        uint8_t* dv = c->bd + (size_t)s * L.total;
        hipStream_t ga = c->bstream[0], gb = c->bstream[1]; /* gathers; encode + scatter */
        const double tt = now_us();
        dev_ptrs((uint64_t*)(h + L.sp), (const void* const*)(segs + (size_t)g0 * k), (size_t)ng * k, ds);
        dev_ptrs((uint64_t*)(h + L.fp), (const void* const*)(fecs + (size_t)g0 * n), (size_t)ng * n, df);
        tab_us += now_us() - tt;
        /* the kernels read the pointer tables where the host wrote them (a DMA
         * copy queued beside the PCIe-bound kernels started ~1.4 ms late) */
        const uint8_t* hd = c->bh_dev + (size_t)s * L.host_total;
        hipError_t e;
        int ke = 0;
        if ((e = hipEventRecord(c->ev[s][0], ga)) != hipSuccess) {
            rc = set_err(RFEC_EDEVICE, "zero-copy encode event", e);
            break;
        }
        ke = rfec_launch_host_gather((const uint64_t*)(hd + L.sp), ng * k, dv + L.shards, (rfec_hdr*)(dv + L.hdr),
                                     NULL, 0, NULL, NULL, NULL, NULL, DI_STRIDE, SIM_VIDEO_SIZE, NULL, NULL, 0, ga);
        if (!ke && ((e = hipEventRecord(c->ev[s][1], ga)) != hipSuccess ||
                    (e = hipStreamWaitEvent(gb, c->ev[s][1], 0)) != hipSuccess))
            ke = (int)e;
        if (!ke)
            ke = rfec_launch_encode(plan, ng, DI_STRIDE, SIM_VIDEO_SIZE, dv + L.shards, (const rfec_hdr*)(dv + L.hdr),
                                    dv + L.parity, (rfec_hdr*)(dv + L.meta), (uint16_t*)(dv + L.fsize),
                                    (int8_t*)(dv + L.status), gb, g_tuning);
        if (!ke && (e = hipEventRecord(c->ev[s][2], gb)) != hipSuccess)
            ke = (int)e;
        if (!ke)
            ke = rfec_launch_host_scatter_fec((const uint64_t*)(hd + L.fp), ng, plan, DI_STRIDE, dv + L.parity,
                                              (const rfec_hdr*)(dv + L.meta), (const uint16_t*)(dv + L.fsize),
                                              (const int8_t*)(dv + L.status), (const rfec_hdr*)(dv + L.hdr), fec_id0,
                                              g0, SIM_VIDEO_SIZE, gb);
        if (ke || (e = hipEventRecord(c->ev[s][3], gb)) != hipSuccess) {
            rc = set_err(RFEC_EDEVICE, "zero-copy encode launch", ke ? ke : (int)e);
            break;
        }
    }
    if (rc != RFEC_OK) {
        (void)hipStreamSynchronize(c->bstream[0]);
        (void)hipStreamSynchronize(c->bstream[1]);
        return rc;
    }
    if (timing) { /* gather: the host's pointer tables; h2d: the device's gather; d2h: its scatter */
        timing->gather_us = tab_us;
        timing->h2d_us = h2d_us;
        timing->kernel_us = kernel_us;
        timing->d2h_us = d2h_us;
        timing->scatter_us = 0;
        timing->total_us = now_us() - t0;
        timing->zero_copy = 1;
        timing->reserved = 0;
    }
    return RFEC_OK;
}

/*
 * Chunked and double-buffered: while the GPU copies / encodes / copies back
 * chunk c on slot c%2's stream, the CPU threads scatter chunk c-1's parities
 * and gather chunk c+1 into the other slot, so the wall time approaches the
 * slowest stage (the PCIe copies) instead of the sum of all five.
 */
int rfec_host_encode_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                            sim_fec_t* const* fecs, uint16_t fec_id0, rfec_host_timing* timing)
{
    int rc = check_plan(plan, RFEC_MAX_K_ENCODE);
    if (rc)
        return rc;
    if (groups == 0 || plan->n_lines == 0)
        return RFEC_OK;
    if (!segs || !fecs)
        return set_err(RFEC_EINVAL, "NULL segs / fecs", 0);
    if ((rc = check_geometry(groups, DI_STRIDE, SIM_VIDEO_SIZE, plan->k)))
        return rc;
    intptr_t ds = 0, df = 0;
    if (zerocopy_enabled() && pinned_span((const void* const*)segs, (size_t)groups * plan->k, sizeof(sim_segment_t), &ds) &&
        pinned_span((const void* const*)fecs, (size_t)groups * plan->n_lines, sizeof(sim_fec_t), &df)) {
        for (size_t i = 0; i < (size_t)groups * plan->k; ++i)
            if (!segs[i])
                return set_err(RFEC_EINVAL, "NULL segment", 0);
        for (size_t i = 0; i < (size_t)groups * plan->n_lines; ++i)
            if (!fecs[i])
                return set_err(RFEC_EINVAL, "NULL parity", 0);
        return zc_encode_groups(plan, groups, segs, fecs, fec_id0, timing, ds, df);
    }
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const uint32_t k = plan->k, n = plan->n_lines;
    uint32_t chunk = (groups + 7) / 8;
    chunk = chunk < 2048 ? 2048 : chunk;
    chunk = chunk > groups ? groups : chunk;
    const uint32_t nch = (groups + chunk - 1) / chunk;
    const hb_layout L = hb_offsets(chunk, k, n);
    if ((rc = hb_reserve(c, L.total, L.total, 2)))
        return rc;
    const int threads = host_threads();
    double gather_us = 0, scatter_us = 0, h2d_us = 0, kernel_us = 0, d2h_us = 0;
    hb_chunk job[2];
    const double t0 = now_us();
    for (uint32_t it = 0; it < nch + 2; ++it) {
        if (it >= 2) { /* retire chunk it-2 */
            const uint32_t s = (it - 2) & 1;
            hipError_t e = hipEventSynchronize(c->ev[s][3]);
            if (e != hipSuccess)
                return set_err(RFEC_EDEVICE, "D2H wait", e);
            float a = 0, b = 0, d = 0;
            (void)hipEventElapsedTime(&a, c->ev[s][0], c->ev[s][1]);
            (void)hipEventElapsedTime(&b, c->ev[s][1], c->ev[s][2]);
            (void)hipEventElapsedTime(&d, c->ev[s][2], c->ev[s][3]);
            h2d_us += a * 1e3;
            kernel_us += b * 1e3;
            d2h_us += d * 1e3;
            const double ts = now_us();
            const uint32_t ng = (it - 2 == nch - 1) ? groups - (it - 2) * chunk : chunk;
            parallel_for(ng, threads, hb_scatter, &job[s]);
            scatter_us += now_us() - ts;
        }
        if (it < nch) { /* stage chunk it */
            const uint32_t s = it & 1;
            const uint32_t g0 = it * chunk;
            const uint32_t ng = (it == nch - 1) ? groups - g0 : chunk;
            hb_chunk* h = &job[s];
            h->plan = plan;
            h->segs = segs + (size_t)g0 * k;
            h->fecs = fecs + (size_t)g0 * n;
            h->slot = c->bh + (size_t)s * L.total;
            h->L = L;
            h->g0 = g0;
            h->fec_id0 = fec_id0;
            const double tg = now_us();
            parallel_for((size_t)ng * k, threads, hb_gather, h);
            gather_us += now_us() - tg;
            uint8_t* dv = c->bd + (size_t)s * L.total;
            hipStream_t st = c->bstream[s];
            hipError_t e;
            /* the slot holds `chunk` groups; a short last chunk copies its own extent */
            const hb_layout Ln = hb_offsets(ng, k, n);
            if ((e = hipEventRecord(c->ev[s][0], st)) != hipSuccess ||
                (e = hipMemcpyAsync(dv + L.shards, h->slot + L.shards, Ln.hdr, hipMemcpyHostToDevice, st)) !=
                    hipSuccess ||
                (e = hipMemcpyAsync(dv + L.hdr, h->slot + L.hdr, (size_t)ng * k * sizeof(rfec_hdr),
                                    hipMemcpyHostToDevice, st)) != hipSuccess ||
                (e = hipEventRecord(c->ev[s][1], st)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "H2D", e);
            const int ke = rfec_launch_encode(plan, ng, DI_STRIDE, SIM_VIDEO_SIZE, dv + L.shards,
                                              (const rfec_hdr*)(dv + L.hdr), dv + L.parity, (rfec_hdr*)(dv + L.meta),
                                              (uint16_t*)(dv + L.fsize), (int8_t*)(dv + L.status), st, g_tuning);
            if (ke)
                return set_err(RFEC_EDEVICE, "encode launch", ke);
            if ((e = hipEventRecord(c->ev[s][2], st)) != hipSuccess ||
                (e = hipMemcpyAsync(h->slot + L.parity, dv + L.parity, (size_t)ng * n * DI_STRIDE,
                                    hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipMemcpyAsync(h->slot + L.meta, dv + L.meta, (size_t)ng * n * sizeof(rfec_hdr),
                                    hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipMemcpyAsync(h->slot + L.fsize, dv + L.fsize, (size_t)ng * n * sizeof(uint16_t),
                                    hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipMemcpyAsync(h->slot + L.status, dv + L.status, (size_t)ng * n, hipMemcpyDeviceToHost,
                                    st)) != hipSuccess ||
                (e = hipEventRecord(c->ev[s][3], st)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "D2H", e);
        }
    }
    if (timing) {
        timing->gather_us = gather_us;
        timing->h2d_us = h2d_us;
        timing->kernel_us = kernel_us;
        timing->d2h_us = d2h_us;
        timing->scatter_us = scatter_us;
        timing->total_us = now_us() - t0;
        timing->zero_copy = 0;
        timing->reserved = 0;
    }
    return RFEC_OK;
}

/* ---- the receive direction: rfec_host_recover_groups --------------------- */
/* Host -> device in one copy: the headers, masks and maps, then only the
 * RECEIVED payloads, packed (`packed`, last, so the copy ends at the last
 * used slot; lost segments and parities are not shipped).  On the device two
 * row gathers expand them into the dense slot arrays the recover kernels read
 * (`shards`, `parity`, device-only; a lost slot zero), then the recover
 * kernel, then the recovered rows back.  The pinned slot mirrors the regions
 * that cross PCIe only ([0, host_total)); the device-only regions follow them
 * in the device slot. */
typedef struct {
    size_t hdr, present, meta, fsize, ppm, smap, pmap, packed; /* host -> device: [0, packed + used slots) */
    size_t out_shards, out_hdr, out_index, recovered, out_bytes; /* device -> host */
    size_t host_total;                                           /* the pinned slot */
    size_t shards, parity, ws, total;                            /* device only: dense slots, workspace */
} hr_layout;


static hr_layout hr_offsets(const rfec_plan* plan, uint32_t G, uint32_t E)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    hr_layout L;
    size_t o = 0;
#define HR_TAKE(field, bytes)                           \
    do {                                                \
        L.field = o;                                    \
        o = (o + (size_t)(bytes) + 255) & ~(size_t)255; \
    } while (0)
    HR_TAKE(hdr, (size_t)G * k * sizeof(rfec_hdr));
    HR_TAKE(present, (size_t)G * 16);
    HR_TAKE(meta, (size_t)G * n * sizeof(rfec_hdr));
    HR_TAKE(fsize, (size_t)G * n * sizeof(uint16_t));
    HR_TAKE(ppm, (size_t)G * 8);
    HR_TAKE(smap, (size_t)G * k * sizeof(int32_t));
    HR_TAKE(pmap, (size_t)G * n * sizeof(int32_t));
    HR_TAKE(packed, (size_t)G * (k + n) * DI_STRIDE);
    HR_TAKE(out_shards, (size_t)G * E * DI_STRIDE);
    HR_TAKE(out_hdr, (size_t)G * E * sizeof(rfec_hdr));
    HR_TAKE(out_index, (size_t)G * E);
    HR_TAKE(recovered, (size_t)G * 16);
    L.out_bytes = o - L.out_shards;
    L.host_total = o;
    HR_TAKE(shards, (size_t)G * k * DI_STRIDE);
    HR_TAKE(parity, (size_t)G * n * DI_STRIDE);
    HR_TAKE(ws, rfec_recover_workspace_size(plan, G));
#undef HR_TAKE
    L.total = o;
    return L;
}

typedef struct {
    const rfec_plan* plan;
    sim_segment_t* const* segs; /* the chunk's first group */
    sim_fec_t* const* fecs;
    sim_segment_t* const* out;
    uint8_t* out_index;
    uint64_t* recovered;
    uint8_t* slot;
    uint32_t* base; /* group g's first packed slot (prefix sums of the received counts) */
    hr_layout L;
    uint32_t E;
} hr_chunk;

/* received segments + parities of each group (the first pass: packed offsets) */
static void hr_count(void* arg, size_t lo, size_t hi)
{
    const hr_chunk* h = (const hr_chunk*)arg;
    const uint32_t k = h->plan->k, n = h->plan->n_lines;
    for (size_t g = lo; g < hi; ++g) {
        uint32_t c = 0;
        for (uint32_t i = 0; i < k; ++i)
            c += h->segs[g * k + i] != NULL;
        for (uint32_t l = 0; l < n; ++l)
            c += h->fecs[g * n + l] != NULL;
        h->base[g] = c;
    }
}

/* gather one group per index: received payloads into the packed slots from
 * base[g] on (members, then parities) with their rows in the maps (-1: lost,
 * a zero row on the device), headers (a lost member's zero), masks */
static void hr_gather(void* arg, size_t lo, size_t hi)
{
    const hr_chunk* h = (const hr_chunk*)arg;
    const uint32_t k = h->plan->k, n = h->plan->n_lines;
    rfec_hdr* hh = (rfec_hdr*)(h->slot + h->L.hdr);
    uint64_t* pres = (uint64_t*)(h->slot + h->L.present);
    rfec_hdr* mh = (rfec_hdr*)(h->slot + h->L.meta);
    uint16_t* fs = (uint16_t*)(h->slot + h->L.fsize);
    uint64_t* ppm = (uint64_t*)(h->slot + h->L.ppm);
    int32_t* smap = (int32_t*)(h->slot + h->L.smap);
    int32_t* pmap = (int32_t*)(h->slot + h->L.pmap);
    uint8_t* packed = h->slot + h->L.packed;
    for (size_t g = lo; g < hi; ++g) {
        uint64_t m0 = 0, m1 = 0, pm = 0;
        uint32_t r = h->base[g];
        for (uint32_t i = 0; i < k; ++i) {
            const size_t s = g * k + i;
            const sim_segment_t* seg = h->segs[s];
            if (!seg) {
                smap[s] = -1;
                memset(&hh[s], 0, sizeof(rfec_hdr));
                continue;
            }
            smap[s] = (int32_t)r;
            stage_payload(packed + (size_t)r++ * DI_STRIDE, seg->data, seg->data_size);
            seg_to_hdr(seg, &hh[s]);
            if (i < 64)
                m0 |= 1ull << i;
            else
                m1 |= 1ull << (i - 64);
        }
        for (uint32_t l = 0; l < n; ++l) {
            const size_t o = g * n + l;
            const sim_fec_t* f = h->fecs[o];
            if (!f) {
                pmap[o] = -1;
                fs[o] = 0;
                continue;
            }
            pm |= 1ull << l;
            memcpy(&mh[o], &f->fec_meta, sizeof(rfec_hdr));
            fs[o] = f->fec_data_size;
            pmap[o] = (int32_t)r;
            stage_payload(packed + (size_t)r++ * DI_STRIDE, f->fec_data,
                          f->fec_data_size < SIM_VIDEO_SIZE ? f->fec_data_size : SIM_VIDEO_SIZE);
        }
        pres[2 * g] = m0;
        pres[2 * g + 1] = m1;
        ppm[g] = pm;
    }
}

/* the recovered segments into the callers' sim_segment_t (flex_fec_recover's out_seg) */
static void hr_scatter(void* arg, size_t lo, size_t hi)
{
    const hr_chunk* h = (const hr_chunk*)arg;
    const uint32_t n = h->plan->n_lines, E = h->E;
    const rfec_hdr* oh = (const rfec_hdr*)(h->slot + h->L.out_hdr);
    const uint8_t* oi = h->slot + h->L.out_index;
    const uint64_t* rec = (const uint64_t*)(h->slot + h->L.recovered);
    for (size_t g = lo; g < hi; ++g) {
        uint16_t fec_id = 0;
        for (uint32_t l = 0; l < n; ++l)
            if (h->fecs[g * n + l]) {
                fec_id = h->fecs[g * n + l]->fec_id;
                break;
            }
        for (uint32_t e = 0; e < E; ++e) {
            const size_t o = g * E + e;
            if (h->out_index)
                h->out_index[o] = oi[o];
            if (oi[o] == 0xFF || !h->out[o])
                continue;
            sim_segment_t* s = h->out[o];
            const rfec_hdr* r = &oh[o];
            s->packet_id = r->seq;
            s->fid = r->fid;
            s->timestamp = r->ts;
            s->index = r->index;
            s->total = r->total;
            s->ftype = r->ftype;
            s->payload_type = r->payload_type;
            s->data_size = r->size;
            memcpy(s->data, h->slot + h->L.out_shards + o * DI_STRIDE, SIM_VIDEO_SIZE);
            s->fec_id = fec_id;
        }
        if (h->recovered) {
            h->recovered[2 * g] = rec[2 * g];
            h->recovered[2 * g + 1] = rec[2 * g + 1];
        }
    }
}

/* The zero-copy recover: per chunk, the host writes the pointer tables and
 * the received masks (from which pointers are NULL) into pinned slot s; on
 * the gather stream the received
 * segments and parities gathered from the callers' structs into the dense
 * slots (a lost one zero), the dense decode, the recovered segments scattered
 * into the callers' out_seg structs, out_index and the recovered masks into
 * the pinned slot -- the decode and the scatter on the second stream, so one
 * chunk's PCIe writes run beside the next chunk's reads (as the encode). */
typedef struct {
    size_t sp, fp, op, present, ppm, in_bytes;       /* host -> device */
    size_t oidx, rec, host_total;                    /* device -> host (pinned) */
    size_t shards, hdr, parity, meta, fsize, fecid;  /* device only */
    size_t out_shards, out_hdr, out_index, recovered, ws, total;
} hy_layout;

static hy_layout hy_offsets(const rfec_plan* plan, uint32_t G, uint32_t E)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    hy_layout L;
    size_t o = 0;
#define HY_TAKE(field, bytes)                           \
    do {                                                \
        L.field = o;                                    \
        o = (o + (size_t)(bytes) + 255) & ~(size_t)255; \
    } while (0)
    HY_TAKE(sp, (size_t)G * k * 8);
    HY_TAKE(fp, (size_t)G * n * 8);
    HY_TAKE(op, (size_t)G * E * 8);
    HY_TAKE(present, (size_t)G * 16);
    HY_TAKE(ppm, (size_t)G * 8);
    L.in_bytes = o;
    HY_TAKE(oidx, (size_t)G * E);
    HY_TAKE(rec, (size_t)G * 16);
    L.host_total = o;
    HY_TAKE(shards, (size_t)G * k * DI_STRIDE);
    HY_TAKE(hdr, (size_t)G * k * sizeof(rfec_hdr));
    HY_TAKE(parity, (size_t)G * n * DI_STRIDE);
    HY_TAKE(meta, (size_t)G * n * sizeof(rfec_hdr));
    HY_TAKE(fsize, (size_t)G * n * sizeof(uint16_t));
    HY_TAKE(fecid, (size_t)G * n * sizeof(uint16_t));
    HY_TAKE(out_shards, (size_t)G * E * DI_STRIDE);
    HY_TAKE(out_hdr, (size_t)G * E * sizeof(rfec_hdr));
    HY_TAKE(out_index, (size_t)G * E);
    HY_TAKE(recovered, (size_t)G * 16);
    HY_TAKE(ws, rfec_recover_workspace_size(plan, G));
#undef HY_TAKE
    L.total = o;
    return L;
}

/* The plans whose dense recovery takes the cascade decodes (rfec_kernels.hip
 * launch_recover: lines cross, <= 4 members a line, <= 8 lines, k <= 64, not
 * forced generic), whose payload lanes read only the lines zc_lines_read
 * names. */
static int zc_cascade_plan(const rfec_plan* p, const rfec_kmask* M)
{
    if (p->k > 64 || p->n_lines > 8 || (g_tuning & RFEC_KFLAG_GENERIC))
        return 0;
    uint64_t seen = 0;
    int cross = 0;
    for (uint32_t l = 0; l < p->n_lines; ++l) {
        if (p->line[l].count > 4)
            return 0;
        cross |= (seen & M->mask[l][0]) != 0;
        seen |= M->mask[l][0];
    }
    return cross;
}

/* The lines a dense cascade decode reads for one group (k <= 64): for each
 * erased member of rank < E, the first line in plan order that fires at once
 * for it (parity received, it the line's only missing member, one member
 * present); if some target has none, every step of the canonical mask
 * schedule (lines in plan order to a fixpoint, targets of rank < E) --
 * cascade_schedule's rules. */
static uint64_t zc_lines_read(const rfec_kmask* M, uint32_t n, uint64_t have, uint64_t ppm, uint32_t E)
{
    const uint32_t k = M->plan.k;
    const uint64_t km = k >= 64 ? ~0ull : (1ull << k) - 1ull;
    const uint64_t er = ~have & km;
    uint64_t lines = 0, e = er;
    int casc = 0;
    for (uint32_t q = 0; q < E && e; ++q, e &= e - 1) {
        const uint64_t tb = e & (~e + 1);
        uint32_t l = 0;
        while (l < n && !((ppm >> l & 1) && (M->mask[l][0] & er) == tb && (M->mask[l][0] & have)))
            ++l;
        if (l < n)
            lines |= 1ull << l;
        else
            casc = 1;
    }
    if (casc) {
        uint64_t h = have;
        for (int progress = 1; progress;) {
            progress = 0;
            for (uint32_t l = 0; l < n; ++l) {
                const uint64_t m = M->mask[l][0], x = m & ~h;
                if (!(ppm >> l & 1) || __builtin_popcountll(x) != 1 || !(m & h))
                    continue;
                if ((uint32_t)__builtin_popcountll(er & (x - 1)) >= E)
                    continue;
                lines |= 1ull << l;
                h |= x;
                progress = 1;
            }
        }
    }
    return lines;
}

static int zc_recover_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                             sim_fec_t* const* fecs, uint32_t E, sim_segment_t* const* out, uint8_t* out_index,
                             uint64_t* recovered, rfec_host_timing* timing, intptr_t ds, intptr_t df, intptr_t dout)
{
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const uint32_t k = plan->k, n = plan->n_lines;
    const size_t group_bytes = hy_offsets(plan, 1024, E).total / 1024 + 1;
    const size_t by_bytes = RFEC_HR_SLOT_BYTES / group_bytes;
    uint32_t chunk = zc_chunk(groups);
    chunk = chunk > 16384 ? 16384 : chunk;
    chunk = (size_t)chunk > by_bytes ? (uint32_t)(by_bytes ? by_bytes : 1) : chunk;
    chunk = chunk > groups ? groups : chunk;
    const uint32_t nch = (groups + chunk - 1) / chunk;
    const hy_layout L = hy_offsets(plan, chunk, E);
    int rc = hb_reserve(c, L.host_total, L.total, RFEC_HB_SLOTS);
    if (rc)
        return rc;
    rfec_kmask M;
    make_masks(plan, &M);
    const int trim = zc_cascade_plan(plan, &M);
    double tab_us = 0, h2d_us = 0, kernel_us = 0, d2h_us = 0, out_us = 0;
    const double t0 = now_us();
    for (uint32_t it = 0; it < nch + RFEC_HB_SLOTS && rc == RFEC_OK; ++it) {
        if (it >= RFEC_HB_SLOTS) { /* retire chunk it - RFEC_HB_SLOTS: its out_index / recovered masks to the caller */
            const uint32_t s = (it - RFEC_HB_SLOTS) % RFEC_HB_SLOTS, g0 = (it - RFEC_HB_SLOTS) * chunk;
            const uint32_t ng = it - RFEC_HB_SLOTS == nch - 1 ? groups - g0 : chunk;
            const hipError_t e = hipEventSynchronize(c->ev[s][3]);
            if (e != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "zero-copy recover wait", e);
                break;
            }
            float a = 0, b = 0, d = 0;
            (void)hipEventElapsedTime(&a, c->ev[s][0], c->ev[s][1]);
            (void)hipEventElapsedTime(&b, c->ev[s][1], c->ev[s][2]);
            (void)hipEventElapsedTime(&d, c->ev[s][2], c->ev[s][3]);
            h2d_us += a * 1e3;
            kernel_us += b * 1e3;
            d2h_us += d * 1e3;
            const double to = now_us();
            const uint8_t* h = c->bh + (size_t)s * L.host_total;
            if (out_index)
                memcpy(out_index + (size_t)g0 * E, h + L.oidx, (size_t)ng * E);
            if (recovered)
                memcpy(recovered + (size_t)g0 * 2, h + L.rec, (size_t)ng * 16);
            out_us += now_us() - to;
        }
        if (it >= nch)
            continue;
        const uint32_t s = it % RFEC_HB_SLOTS, g0 = it * chunk, ng = it == nch - 1 ? groups - g0 : chunk;
        uint8_t* h = c->bh + (size_t)s * L.host_total;
        uint8_t* dv = c->bd + (size_t)s * L.total;
        hipStream_t ga = c->bstream[0], gb = c->bstream[1]; /* gathers; decode + scatter */
        const double tt = now_us();
        sim_segment_t* const* sg = segs + (size_t)g0 * k;
        sim_fec_t* const* fg = fecs + (size_t)g0 * n;
        dev_ptrs((uint64_t*)(h + L.sp), (const void* const*)sg, (size_t)ng * k, ds);
        dev_ptrs((uint64_t*)(h + L.fp), (const void* const*)fg, (size_t)ng * n, df);
        dev_ptrs((uint64_t*)(h + L.op), (const void* const*)(out + (size_t)g0 * E), (size_t)ng * E, dout);
        uint64_t* pres = (uint64_t*)(h + L.present);
        uint64_t* ppm = (uint64_t*)(h + L.ppm);
        uint64_t* spt = (uint64_t*)(h + L.sp);
        uint64_t* fpt = (uint64_t*)(h + L.fp);
        for (uint32_t g = 0; g < ng; ++g) {
            uint64_t m0 = 0, m1 = 0, pm = 0;
            for (uint32_t i = 0; i < k; ++i)
                if (sg[(size_t)g * k + i]) {
                    if (i < 64)
                        m0 |= 1ull << i;
                    else
                        m1 |= 1ull << (i - 64);
                }
            for (uint32_t l = 0; l < n; ++l)
                if (fg[(size_t)g * n + l])
                    pm |= 1ull << l;
            pres[2 * g] = m0;
            pres[2 * g + 1] = m1;
            ppm[g] = pm;
            /* A line fires only to rebuild a member it lacks, so the decode
             * reads the payloads of received lines that hold an erased member
             * and nothing else: the rest cross PCIe as headers only.  Plans
             * with cascades on the dense cascade decodes read fewer: a payload
             * lane takes the first line that fires at once for its target, else
             * the steps of the canonical mask schedule (k_decode_cascade_dense,
             * k_decode_matrix_dense; the header checks pick only out_index and
             * the recovered masks) -- those lines' members and parities cross
             * whole, every other struct as its header. */
            const uint64_t e0 = ~m0, e1 = ~m1; /* (line masks hold members only) */
            uint64_t n0 = 0, n1 = 0, pn = 0;
            if (trim) {
                pn = zc_lines_read(&M, n, m0, pm, E);
                for (uint32_t l = 0; l < n; ++l)
                    if (pn >> l & 1)
                        n0 |= M.mask[l][0];
            } else {
                for (uint32_t l = 0; l < n; ++l)
                    if ((pm >> l & 1) && ((M.mask[l][0] & e0) | (M.mask[l][1] & e1))) {
                        n0 |= M.mask[l][0];
                        n1 |= M.mask[l][1];
                        pn |= 1ull << l;
                    }
            }
            /* a struct on no received line that holds an erased member is read by no peel, not even the
               exact one after a rejected line: it does not cross at all (pointer 0; the masks above still
               say it arrived) -- except the group's first parity, whose fec_id the scatter stamps */
            uint64_t a0 = 0, a1 = 0, pa = 0;
            if (trim)
                for (uint32_t l = 0; l < n; ++l)
                    if ((pm >> l & 1) && ((M.mask[l][0] & e0) | (M.mask[l][1] & e1))) {
                        a0 |= M.mask[l][0];
                        a1 |= M.mask[l][1];
                        pa |= 1ull << l;
                    }
            pa |= pm & (~pm + 1);
            for (uint32_t i = 0; i < k; ++i) {
                uint64_t* sp = &spt[(size_t)g * k + i];
                if (!*sp || ((i < 64 ? n0 >> i : n1 >> (i - 64)) & 1))
                    continue;
                *sp = trim && !((i < 64 ? a0 >> i : a1 >> (i - 64)) & 1) ? 0 : *sp | 1;
            }
            for (uint32_t l = 0; l < n; ++l) {
                uint64_t* fp = &fpt[(size_t)g * n + l];
                if (*fp && !(pn >> l & 1))
                    *fp = trim && !(pa >> l & 1) ? 0 : *fp | 1;
            }
        }
        tab_us += now_us() - tt;
        /* no DMA: the kernels read the tables from the pinned slot, the first
         * gather copies the masks into HBM for the decode, the scatter writes
         * out_index and the recovered masks back */
        const uint8_t* hd = c->bh_dev + (size_t)s * L.host_total;
        hipError_t e;
        if ((e = hipEventRecord(c->ev[s][0], ga)) != hipSuccess) {
            rc = set_err(RFEC_EDEVICE, "zero-copy recover event", e);
            break;
        }
        int ke = rfec_launch_host_gather((const uint64_t*)(hd + L.sp), ng * k, dv + L.shards, (rfec_hdr*)(dv + L.hdr),
                                         (const uint64_t*)(hd + L.fp), ng * n, dv + L.parity, (rfec_hdr*)(dv + L.meta),
                                         (uint16_t*)(dv + L.fsize), (uint16_t*)(dv + L.fecid), DI_STRIDE,
                                         SIM_VIDEO_SIZE, (const uint64_t*)(hd + L.present),
                                         (uint64_t*)(dv + L.present), (uint32_t)((L.in_bytes - L.present) / 8), ga);
        if (!ke && ((e = hipEventRecord(c->ev[s][1], ga)) != hipSuccess ||
                    (e = hipStreamWaitEvent(gb, c->ev[s][1], 0)) != hipSuccess))
            ke = (int)e;
        const rfec_dense_out D = {dv + L.out_shards, (rfec_hdr*)(dv + L.out_hdr), dv + L.out_index, E};
        if (!ke)
            ke = rfec_launch_recover_out(&M, ng, DI_STRIDE, SIM_VIDEO_SIZE, dv + L.shards,
                                         (const rfec_hdr*)(dv + L.hdr), (const uint64_t*)(dv + L.present),
                                         dv + L.parity, (const rfec_hdr*)(dv + L.meta), (const uint16_t*)(dv + L.fsize),
                                         (const uint64_t*)(dv + L.ppm), (uint64_t*)(dv + L.recovered), dv + L.ws, gb,
                                         g_tuning, &D);
        if (!ke && (e = hipEventRecord(c->ev[s][2], gb)) != hipSuccess)
            ke = (int)e;
        if (!ke)
            ke = rfec_launch_host_scatter_seg((const uint64_t*)(hd + L.op), ng, E, DI_STRIDE, dv + L.out_shards,
                                              (const rfec_hdr*)(dv + L.out_hdr), dv + L.out_index,
                                              (const uint16_t*)(dv + L.fecid), (const uint64_t*)(dv + L.ppm), n,
                                              SIM_VIDEO_SIZE, c->bh_dev + (size_t)s * L.host_total + L.oidx,
                                              (const uint64_t*)(dv + L.recovered),
                                              (uint64_t*)(c->bh_dev + (size_t)s * L.host_total + L.rec), gb);
        if (ke || (e = hipEventRecord(c->ev[s][3], gb)) != hipSuccess) {
            rc = set_err(RFEC_EDEVICE, "zero-copy recover launch", ke ? ke : (int)e);
            break;
        }
    }
    if (rc != RFEC_OK) {
        (void)hipStreamSynchronize(c->bstream[0]);
        (void)hipStreamSynchronize(c->bstream[1]);
        return rc;
    }
    if (timing) { /* gather: tables + masks; h2d: the device gathers; kernel: decode; d2h: the scatter */
        timing->gather_us = tab_us;
        timing->h2d_us = h2d_us;
        timing->kernel_us = kernel_us;
        timing->d2h_us = d2h_us;
        timing->scatter_us = out_us;
        timing->total_us = now_us() - t0;
        timing->zero_copy = 1;
        timing->reserved = 0;
    }
    return RFEC_OK;
}

int rfec_host_recover_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                             sim_fec_t* const* fecs, uint32_t per_group, sim_segment_t* const* out,
                             uint8_t* out_index, uint64_t* recovered, rfec_host_timing* timing)
{
    int rc = check_plan(plan, RFEC_MAX_K);
    if (rc)
        return rc;
    if (groups == 0 || plan->n_lines == 0 || per_group == 0)
        return RFEC_OK;
    if (!segs || !fecs || !out)
        return set_err(RFEC_EINVAL, "NULL segs / fecs / out", 0);
    if (per_group > plan->k)
        return set_err(RFEC_EINVAL, "per_group above k", 0);
    if ((rc = check_geometry(groups, DI_STRIDE, SIM_VIDEO_SIZE, plan->k)))
        return rc;
    intptr_t ds = 0, df = 0, dout = 0;
    if (zerocopy_enabled() &&
        pinned_span((const void* const*)segs, (size_t)groups * plan->k, sizeof(sim_segment_t), &ds) &&
        pinned_span((const void* const*)fecs, (size_t)groups * plan->n_lines, sizeof(sim_fec_t), &df) &&
        pinned_span((const void* const*)out, (size_t)groups * per_group, sizeof(sim_segment_t), &dout))
        return zc_recover_groups(plan, groups, segs, fecs, per_group, out, out_index, recovered, timing, ds, df, dout);
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const uint32_t k = plan->k, E = per_group;
    /* 2,048-16,384 groups a step, and at most RFEC_HR_SLOT_BYTES of device
     * staging per slot (its pinned mirror is smaller): at k = 10 / 3 lines a
     * 16,384-group slot takes ~570 MB, at k = 128 / 64 lines ~470 KB a group */
    const size_t group_bytes = hr_offsets(plan, 1024, E).total / 1024 + 1;
    const size_t by_bytes = RFEC_HR_SLOT_BYTES / group_bytes;
    uint32_t chunk = (groups + 7) / 8;
    chunk = chunk < 2048 ? 2048 : chunk > 16384 ? 16384 : chunk;
    chunk = (size_t)chunk > by_bytes ? (uint32_t)(by_bytes ? by_bytes : 1) : chunk;
    chunk = chunk > groups ? groups : chunk;
    const uint32_t nch = (groups + chunk - 1) / chunk;
    const hr_layout L = hr_offsets(plan, chunk, E);
    if ((rc = hb_reserve(c, L.host_total, L.total, 2)))
        return rc;
    rfec_kmask M;
    make_masks(plan, &M);
    const int threads = host_threads();
    double gather_us = 0, scatter_us = 0, h2d_us = 0, kernel_us = 0, d2h_us = 0;
    hr_chunk job[2];
    uint32_t* base = (uint32_t*)malloc(2 * (size_t)chunk * sizeof(uint32_t));
    if (!base)
        return set_err(RFEC_ENOMEM, "recover offsets", 0);
    rc = RFEC_OK;
    const double t0 = now_us();
    for (uint32_t it = 0; it < nch + 2; ++it) {
        if (it >= 2) { /* retire chunk it-2 */
            const uint32_t s = (it - 2) & 1;
            hipError_t e = hipEventSynchronize(c->ev[s][3]);
            if (e != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "D2H wait", e);
                break;
            }
            float a = 0, b = 0, d = 0;
            (void)hipEventElapsedTime(&a, c->ev[s][0], c->ev[s][1]);
            (void)hipEventElapsedTime(&b, c->ev[s][1], c->ev[s][2]);
            (void)hipEventElapsedTime(&d, c->ev[s][2], c->ev[s][3]);
            h2d_us += a * 1e3;
            kernel_us += b * 1e3;
            d2h_us += d * 1e3;
            const double ts = now_us();
            const uint32_t ng = (it - 2 == nch - 1) ? groups - (it - 2) * chunk : chunk;
            parallel_for(ng, threads, hr_scatter, &job[s]);
            scatter_us += now_us() - ts;
        }
        if (it < nch) { /* stage chunk it */
            const uint32_t s = it & 1;
            const uint32_t g0 = it * chunk;
            const uint32_t ng = (it == nch - 1) ? groups - g0 : chunk;
            hr_chunk* h = &job[s];
            h->plan = plan;
            h->segs = segs + (size_t)g0 * k;
            h->fecs = fecs + (size_t)g0 * plan->n_lines;
            h->out = out + (size_t)g0 * E;
            h->out_index = out_index ? out_index + (size_t)g0 * E : NULL;
            h->recovered = recovered ? recovered + (size_t)g0 * 2 : NULL;
            h->slot = c->bh + (size_t)s * L.host_total;
            h->base = base + (size_t)s * chunk;
            h->L = L;
            h->E = E;
            const double tg = now_us();
            parallel_for(ng, threads, hr_count, h);
            uint32_t used = 0;
            for (uint32_t g = 0; g < ng; ++g) { /* counts -> first packed slots */
                const uint32_t cg = h->base[g];
                h->base[g] = used;
                used += cg;
            }
            parallel_for(ng, threads, hr_gather, h);
            gather_us += now_us() - tg;
            uint8_t* dv = c->bd + (size_t)s * L.total;
            hipStream_t st = c->bstream[s];
            hipError_t e;
            if ((e = hipEventRecord(c->ev[s][0], st)) != hipSuccess ||
                (e = hipMemcpyAsync(dv, h->slot, L.packed + (size_t)used * DI_STRIDE, hipMemcpyHostToDevice, st)) !=
                    hipSuccess ||
                (e = hipEventRecord(c->ev[s][1], st)) != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "H2D", e);
                break;
            }
            int ke = rfec_launch_gather_rows(dv + L.shards, dv + L.packed, (const int32_t*)(dv + L.smap), ng * k,
                                             DI_STRIDE, st);
            if (!ke)
                ke = rfec_launch_gather_rows(dv + L.parity, dv + L.packed, (const int32_t*)(dv + L.pmap),
                                             ng * plan->n_lines, DI_STRIDE, st);
            const rfec_dense_out D = {dv + L.out_shards, (rfec_hdr*)(dv + L.out_hdr), dv + L.out_index, E};
            if (!ke)
                ke = rfec_launch_recover_out(
                &M, ng, DI_STRIDE, SIM_VIDEO_SIZE, dv + L.shards, (const rfec_hdr*)(dv + L.hdr),
                (const uint64_t*)(dv + L.present), dv + L.parity, (const rfec_hdr*)(dv + L.meta),
                (const uint16_t*)(dv + L.fsize), (const uint64_t*)(dv + L.ppm), (uint64_t*)(dv + L.recovered),
                dv + L.ws, st, g_tuning, &D);
            if (ke) {
                rc = set_err(RFEC_EDEVICE, "recover launch", ke);
                break;
            }
            if ((e = hipEventRecord(c->ev[s][2], st)) != hipSuccess ||
                (e = hipMemcpyAsync(h->slot + L.out_shards, dv + L.out_shards, L.out_bytes, hipMemcpyDeviceToHost,
                                    st)) != hipSuccess ||
                (e = hipEventRecord(c->ev[s][3], st)) != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "D2H", e);
                break;
            }
        }
    }
    free(base);
    if (rc != RFEC_OK) {
        /* a failed step: the other buffer's work drains before its staging is reused */
        (void)hipStreamSynchronize(c->bstream[0]);
        (void)hipStreamSynchronize(c->bstream[1]);
        return rc;
    }
    if (timing) {
        timing->gather_us = gather_us;
        timing->h2d_us = h2d_us;
        timing->kernel_us = kernel_us;
        timing->d2h_us = d2h_us;
        timing->scatter_us = scatter_us;
        timing->total_us = now_us() - t0;
        timing->zero_copy = 0;
        timing->reserved = 0;
    }
    return RFEC_OK;
}
