/*
 * rfec_dropin.c -- the drop-in flex_fec_generate / flex_fec_recover
 * (sim_transport/fec/flex_fec_xor.h:7-8) and the group-level calls behind
 * rfec_flex.c: per-thread pinned staging, and the resident service
 * (rfec_service.hip) that takes a call's job from a doorbell.  No CPU compute
 * path: without a usable HIP device the calls print an error once and return -1.
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
/* 3. drop-in single-call path                                               */
/* ------------------------------------------------------------------------ */
/* DI_STRIDE, DI_MAXK, di_ctx: rfec_host_internal.h */

typedef struct { /* offsets inside the staging area */
    size_t shards, parity, hdr, meta, fsize, status, present, ppresent, recovered, ws, total;
} di_layout;

static di_layout di_offsets(void)
{
    di_layout L;
    size_t o = 0;
#define DI_TAKE(field, n)                  \
    do {                                    \
        L.field = o;                        \
        o = (o + (size_t)(n) + 255) & ~(size_t)255; \
    } while (0)
    /* a whole group (k <= RFEC_MAX_K segments, every line of its plan) for
     * the group-level sender, or up to RFEC_DI_GROUPS one-line groups */
    DI_TAKE(shards, (size_t)DI_MAXK * DI_STRIDE);
    DI_TAKE(parity, (size_t)RFEC_MAX_LINES * DI_STRIDE);
    DI_TAKE(hdr, DI_MAXK * sizeof(rfec_hdr));
    DI_TAKE(meta, RFEC_MAX_LINES * sizeof(rfec_hdr));
    DI_TAKE(fsize, RFEC_MAX_LINES * sizeof(uint16_t));
    DI_TAKE(status, RFEC_MAX_LINES);
    DI_TAKE(present, RFEC_DI_GROUPS * 2 * sizeof(uint64_t));
    DI_TAKE(ppresent, RFEC_DI_GROUPS * sizeof(uint64_t));
    DI_TAKE(recovered, RFEC_DI_GROUPS * 2 * sizeof(uint64_t));
    DI_TAKE(ws, rfec_ws_bytes(RFEC_MAX_K, RFEC_MAX_LINES, RFEC_DI_GROUPS));
#undef DI_TAKE
    L.total = o;
    return L;
}

static pthread_key_t di_key;
static pthread_once_t di_once = PTHREAD_ONCE_INIT;
static int di_reported = 0;

static void di_free(void* p)
{
    di_ctx* c = (di_ctx*)p;
    if (!c)
        return;
    if (c->host)
        (void)hipHostFree(c->host);
    if (c->bh)
        (void)hipHostFree(c->bh);
    if (c->bd)
        (void)hipFree(c->bd);
    for (int s = 0; c->have_ev && s < RFEC_HB_SLOTS; ++s)
        for (int i = 0; i < 4; ++i)
            (void)hipEventDestroy(c->ev[s][i]);
    for (int s = 0; c->have_ev && s < 2; ++s)
        (void)hipStreamDestroy(c->bstream[s]);
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    free(c);
}

static void di_make_key(void) { (void)pthread_key_create(&di_key, di_free); }

static void di_loud(const char* msg)
{
    if (!di_reported) {
        di_reported = 1;
        fprintf(stderr, "razor_fec: %s -- flex_fec_generate/flex_fec_recover need a HIP device (no CPU path)\n",
                msg);
    }
}

di_ctx* di_get(void)
{
    pthread_once(&di_once, di_make_key);
    di_ctx* c = (di_ctx*)pthread_getspecific(di_key);
    if (c)
        return c;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        set_err(RFEC_EDEVICE, "no HIP device", e);
        di_loud(rfec_last_error());
        return NULL;
    }
    c = (di_ctx*)calloc(1, sizeof(*c));
    if (!c)
        return NULL;
    const di_layout L = di_offsets();
    c->bytes = L.total;
    if ((e = hipGetDevice(&c->device)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipHostMalloc((void**)&c->host, c->bytes, hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->dev, c->host, 0)) != hipSuccess) {
        set_err(RFEC_EDEVICE, "staging setup", e);
        di_loud(rfec_last_error());
        di_free(c);
        return NULL;
    }
    pthread_setspecific(di_key, c);
    return c;
}

void seg_to_hdr(const sim_segment_t* s, rfec_hdr* h)
{
    h->seq = s->packet_id;
    h->fid = s->fid;
    h->ts = s->timestamp;
    h->index = s->index;
    h->total = s->total;
    h->ftype = s->ftype;
    h->payload_type = s->payload_type;
    h->size = s->data_size;
}

void stage_payload(uint8_t* slot, const uint8_t* data, uint32_t size)
{
    const uint32_t n = size < SIM_VIDEO_SIZE ? size : SIM_VIDEO_SIZE;
    memcpy(slot, data, n);
    memset(slot + n, 0, DI_STRIDE - n);
}

static int di_sync(di_ctx* c, int launch_err, const char* what)
{
    if (launch_err)
        return set_err(RFEC_EDEVICE, what, launch_err);
    const hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? RFEC_OK : set_err(RFEC_EDEVICE, what, e);
}


/* ---- resident service (rfec_service.hip) --------------------------------
 * The drop-in symbols are called once per group under razor's session mutex
 * (sim_session.c:241, sim_sender.c:286-304), so their cost is latency: a
 * launch plus hipStreamSynchronize is ~15-20 us before any work.  Instead ONE
 * workgroup stays on the device and polls a doorbell; a call stages its job
 * and segments next to the doorbell (host-mapped device memory when the host
 * maps it, else pinned host memory: svc_map_request_side), rings it and spins
 * on `done` in pinned host memory (a PCIe write each way).  The workgroup leaves after
 * RFEC_SERVICE_IDLE_US (default 2 ms) without a job, after
 * RFEC_SERVICE_LIFE_US (default 4 ms) in total, on `stop` (rfec_service_stop,
 * atexit); a call that finds `alive` == 0 launches it again (~10-20 us for
 * that call).  The lifetime bounds what the resident kernel can hold up: a
 * device-wide synchronize (hipDeviceSynchronize, torch.cuda.synchronize)
 * waits for it, and so would any kernel queued behind it on a shared
 * hardware queue -- which is why its stream is a non-blocking stream of the
 * highest priority: a queue of its own, so no other stream's kernels sit
 * behind the service (tests/test_service.py times torch kernels on 9 streams
 * while it is resident).  One service per process, calls serialised by its
 * mutex. */
typedef struct {
    pthread_mutex_t mu;
    int state;     /* 0 not set up, 1 ready, -1 unavailable (per-call launches), -2 timed out: a launch may
                      still be live (stop set); retried after 1 s once its stream is idle */
    double t_fail; /* when it timed out */
    hipStream_t stream;
    rfec_svc_ctl* ctl;   /* results side (done / alive / out), pinned host memory; the output slots follow it */
    uint8_t* dev;        /* device view of the same allocation */
    rfec_svc_ctl* in;    /* request side (bell / stop / quit / job), the staging slots follow it: device memory
                            the host writes through its mapping when it can (in_vram), else == ctl */
    uint8_t* in_dev;     /* device view of `in` */
    void* vram;          /* the device allocation behind `in`, or NULL */
    rfec_svc_ctl* req;   /* where a call composes its job and staged slots: `in` itself, or with `vram` a
                            host shadow of it copied over in whole lines before the doorbell */
    size_t o_shards, o_parity;
    uint32_t seq, groups;
    uint32_t last_ok; /* the seq of the last job answered through the service (its timing record is valid) */
    uint64_t idle_ticks, life_ticks;
    uint64_t jobs, launches, dev_jobs;
    double tick_us;                                  /* s_memrealtime period */
    double t_stage, t_wait, t_dstage, t_dwork, t_drel; /* sums over the jobs, us */
} svc_state;
static svc_state g_svc = {.mu = PTHREAD_MUTEX_INITIALIZER};

/* host stores into device memory go through a write-combining mapping: drain
 * them (the staged job before its doorbell, the doorbell itself) */
static void svc_flush(void)
{
    if (!g_svc.vram)
        return;
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_sfence();
#else
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
#endif
}

/* 1 when [p, p + n) lies in one readable and writable mapping of this
 * process (/proc/self/maps) */
static int host_mapped_rw(const void* p, size_t n)
{
    FILE* f = fopen("/proc/self/maps", "r");
    if (!f)
        return 0;
    char line[512];
    int ok = 0;
    const uintptr_t a = (uintptr_t)p;
    while (!ok && fgets(line, sizeof(line), f)) {
        unsigned long lo = 0, hi = 0;
        char perm[5] = {0};
        if (sscanf(line, "%lx-%lx %4s", &lo, &hi, perm) == 3 && a >= lo && a + n <= hi)
            ok = perm[0] == 'r' && perm[1] == 'w';
    }
    fclose(f);
    return ok;
}

/* The request side (doorbell, stop / quit, the job and its staging slots) in
 * device memory the host writes through its BAR mapping: a call's staging is
 * posted writes, and the workgroup polls and reads device memory, instead of
 * reading the job over PCIe after the doorbell (one PCIe read round trip per
 * call).  Fine-grained device memory, used when the runtime
 * has mapped it into this process at the same address (a large-BAR host;
 * /proc/self/maps says so); otherwise (or RFEC_SERVICE_STAGE=host) the request
 * side stays in the pinned host block.  `bytes`: control block + staging
 * slots. */
static void svc_map_request_side(size_t bytes)
{
    const char* env = getenv("RFEC_SERVICE_STAGE");
    if (env && strcmp(env, "host") == 0)
        return;
    void* d = NULL;
    if (hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained) != hipSuccess || !d) {
        (void)hipGetLastError();
        return;
    }
    if (!host_mapped_rw(d, bytes)) {
        (void)hipFree(d);
        return;
    }
    void* sh = NULL;
    if (posix_memalign(&sh, 64, bytes) != 0) {
        (void)hipFree(d);
        return;
    }
    memset(sh, 0, bytes);
    g_svc.vram = d;
    g_svc.in = (rfec_svc_ctl*)d;
    g_svc.in_dev = (uint8_t*)d;
    g_svc.req = (rfec_svc_ctl*)sh;
    memset(g_svc.in, 0, bytes);
    svc_flush();
}

static void svc_pause(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

/* mutex held; leaves the workgroup off the device.  The workgroup polls
 * `stop` and leaves within microseconds (its lifetime is 4 ms anyway), so the
 * wait is bounded: a launch still live after RFEC_SVC_STOP_US is wedged, and
 * this reports it instead of blocking in hipStreamSynchronize for good (the
 * service then stays unavailable). */
#define RFEC_SVC_STOP_US 2e6
static int svc_stop_locked(void)
{
    if (g_svc.state != 1 && g_svc.state != -2)
        return RFEC_OK;
    __atomic_store_n(&g_svc.in->stop, 1u, __ATOMIC_RELEASE);
    svc_flush();
    const double t0 = now_us();
    hipError_t e;
    while ((e = hipStreamQuery(g_svc.stream)) == hipErrorNotReady) {
        if (now_us() - t0 > RFEC_SVC_STOP_US) {
            g_svc.state = -1;
            fprintf(stderr, "razor_fec: the resident FEC service did not leave within %.0f s of stop\n",
                    RFEC_SVC_STOP_US / 1e6);
            return set_err(RFEC_EDEVICE, "service stop: the resident workgroup did not leave", 0);
        }
        svc_pause();
    }
    __atomic_store_n(&g_svc.in->stop, 0u, __ATOMIC_RELEASE);
    g_svc.in->quit = 0;
    svc_flush();
    g_svc.ctl->alive = 0;
    return e == hipSuccess ? RFEC_OK : set_err(RFEC_EDEVICE, "service stop", e);
}

int rfec_service_stop(void)
{
    pthread_mutex_lock(&g_svc.mu);
    const int rc = svc_stop_locked();
    pthread_mutex_unlock(&g_svc.mu);
    return rc;
}

int rfec_service_get_info(rfec_service_info* info)
{
    if (!info)
        return set_err(RFEC_EINVAL, "service info: NULL", 0);
    pthread_mutex_lock(&g_svc.mu);
    memset(info, 0, sizeof(*info));
    info->jobs = g_svc.jobs;
    info->launches = g_svc.launches;
    info->request_in_device = g_svc.vram != NULL;
    if (g_svc.jobs) {
        const double n = (double)g_svc.jobs;
        info->stage_host_us = g_svc.t_stage / n;
        info->wait_us = g_svc.t_wait / n;
    }
    if (g_svc.dev_jobs) {
        const double n = (double)g_svc.dev_jobs;
        info->dev_stage_us = g_svc.t_dstage / n;
        info->dev_work_us = g_svc.t_dwork / n;
        info->dev_release_us = g_svc.t_drel / n;
    }
    pthread_mutex_unlock(&g_svc.mu);
    return RFEC_OK;
}

/* at exit: a wedged workgroup would hold the process in the runtime's
 * teardown; leave with a failure status instead */
static void svc_atexit(void)
{
    if (rfec_service_stop() != RFEC_OK && g_svc.state == -1 && hipStreamQuery(g_svc.stream) == hipErrorNotReady) {
        fflush(stdout);
        fflush(stderr);
        _exit(70);
    }
}

static size_t svc_align(size_t x) { return (x + 255) & ~(size_t)255; }

/* Locks the service and returns 1 when calls should go through it (set up on
 * first use), else 0 with the mutex released. */
static int svc_acquire(void)
{
    if (g_tuning & RFEC_TUNE_NO_SERVICE)
        return 0;
    pthread_mutex_lock(&g_svc.mu);
    if (g_svc.state == 0) {
        g_svc.state = -1;
        const char* env = getenv("RFEC_SERVICE");
        int dev = 0, khz = 0, n = 0;
        hipError_t e;
        if (env && env[0] == '0') {
            pthread_mutex_unlock(&g_svc.mu);
            return 0;
        }
        const size_t o_shards = svc_align(sizeof(rfec_svc_ctl));
        const size_t o_parity = o_shards + svc_align((size_t)RFEC_SVC_SLOTS * DI_STRIDE);
        const size_t bytes = o_parity + svc_align((size_t)RFEC_MAX_LINES * DI_STRIDE);
        void* h = NULL;
        if ((e = hipGetDeviceCount(&n)) != hipSuccess || n == 0 || (e = hipGetDevice(&dev)) != hipSuccess ||
            (e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev)) != hipSuccess || khz <= 0) {
            set_err(RFEC_EDEVICE, "service setup", e);
            pthread_mutex_unlock(&g_svc.mu);
            return 0;
        }
        /* a hardware queue of its own: a non-blocking stream of the highest
         * priority (the runtime keeps a queue pool per priority, and the
         * application's streams are normal priority; measured on the MI355X
         * with 8 torch streams + the default one held up for the service's
         * whole lifetime: a normal-priority stream shared a queue with one of
         * them, a CU-masked stream -- blocking -- held the legacy default
         * stream, the high-priority one held none) */
        int prio_lo = 0, prio_hi = 0;
        if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
            hipStreamCreateWithPriority(&g_svc.stream, hipStreamNonBlocking, prio_hi) != hipSuccess) {
            (void)hipGetLastError();
            g_svc.stream = NULL;
        }
        if ((!g_svc.stream && (e = hipStreamCreateWithFlags(&g_svc.stream, hipStreamNonBlocking)) != hipSuccess) ||
            (e = hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&g_svc.dev, h, 0)) != hipSuccess) {
            set_err(RFEC_EDEVICE, "service setup", e);
            if (h)
                (void)hipHostFree(h);
            pthread_mutex_unlock(&g_svc.mu);
            return 0;
        }
        memset(h, 0, bytes);
        g_svc.ctl = (rfec_svc_ctl*)h;
        g_svc.o_shards = o_shards;
        g_svc.o_parity = o_parity;
        g_svc.in = g_svc.ctl;
        g_svc.in_dev = g_svc.dev;
        g_svc.req = g_svc.ctl;
        svc_map_request_side(o_parity);
        const char* idle = getenv("RFEC_SERVICE_IDLE_US");
        const char* life = getenv("RFEC_SERVICE_LIFE_US");
        const double idle_us = idle && atof(idle) > 0 ? atof(idle) : 2000.0;
        const double life_us = life && atof(life) > 0 ? atof(life) : 4000.0;
        g_svc.idle_ticks = (uint64_t)(idle_us * khz / 1000.0);
        g_svc.life_ticks = (uint64_t)(life_us * khz / 1000.0);
        g_svc.tick_us = 1000.0 / khz;
        /* workgroups: 1 (tools/svc_groups.sh: 1 / 2 / 4 / 8 took 12.8 / 15.9 / 12.8 / 14.4 us per group
         * encode on one box; more CUs shorten the XOR + stores, 2.0 -> 1.35 us, but not the PCIe round
         * trip of the staging, 3.0-3.4 us, and the host then waits on more answers) */
        const char* grp = getenv("RFEC_SERVICE_GROUPS");
        const int ng = grp ? atoi(grp) : 1;
        g_svc.groups = ng >= 1 && ng <= RFEC_SVC_MAX_GROUPS ? (uint32_t)ng : 1u;
        g_svc.state = 1;
        atexit(svc_atexit);
    }
    if (g_svc.state == -2 && now_us() - g_svc.t_fail > 1e6 && hipStreamQuery(g_svc.stream) == hipSuccess) {
        /* the timed-out launch has left: take the service up again */
        g_svc.in->stop = 0;
        g_svc.in->quit = 0;
        svc_flush();
        g_svc.ctl->alive = 0;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        g_svc.state = 1;
    }
    if (g_svc.state != 1) {
        pthread_mutex_unlock(&g_svc.mu);
        return 0;
    }
    return 1;
}

static uint8_t* svc_shard(uint32_t i) { return (uint8_t*)g_svc.req + g_svc.o_shards + (size_t)i * DI_STRIDE; }
static uint8_t* svc_out(uint32_t i) { return (uint8_t*)g_svc.ctl + g_svc.o_parity + (size_t)i * DI_STRIDE; }

/* a payload into a service slot: the bytes, zeros to the end of the slot (the
 * zero padding of flex_fec_xor.c:30-32, 84-86: the device XORs whole slots);
 * returns the 16-byte chunks that hold the bytes */
static uint8_t svc_stage(uint8_t* slot, const uint8_t* data, uint32_t size)
{
    const uint32_t n = size < SIM_VIDEO_SIZE ? size : SIM_VIDEO_SIZE, nck = (n + 15) / 16;
    memcpy(slot, data, n);
    memset(slot + n, 0, (size_t)DI_STRIDE - n);
    return (uint8_t)nck;
}

/* mutex held, the job written: ring the doorbell, (re)launch the workgroup
 * when it is gone, wait for `done` */
static int svc_run(uint32_t n_slots, uint32_t op, double t_begin)
{
    rfec_svc_ctl* q = g_svc.ctl;
    const uint32_t seq = ++g_svc.seq;
    if (g_svc.vram) {
        /* the job description up to its n_slots header records, and the slots, from the shadow in whole
         * lines (scattered partial writes through the write-combining mapping cost ~3 us a call) */
        const size_t oj = offsetof(rfec_svc_ctl, job);
        const size_t nj = (offsetof(rfec_svc_job, hdr) + 20u * (size_t)n_slots + 63u) & ~(size_t)63u;
        memcpy((uint8_t*)g_svc.in + oj, (const uint8_t*)g_svc.req + oj, nj);
        memcpy((uint8_t*)g_svc.in + g_svc.o_shards, (const uint8_t*)g_svc.req + g_svc.o_shards,
               (size_t)n_slots * DI_STRIDE);
    }
    svc_flush(); /* the staged job lands before its doorbell */
    const double t0 = now_us();
    __atomic_store_n(&g_svc.in->bell, RFEC_SVC_BELL(seq, n_slots, op), __ATOMIC_RELEASE);
    svc_flush();
    for (uint64_t spin = 0;; ++spin) {
        uint32_t w = 0;
        while (w < g_svc.groups && __atomic_load_n(&q->done[w], __ATOMIC_ACQUIRE) == seq)
            ++w;
        if (w == g_svc.groups)
            break;
        if (__atomic_load_n(&q->alive, __ATOMIC_ACQUIRE) == 0) {
            /* gone (or leaving): wait until every workgroup of the old launch
             * has left (they leave on `quit`; a part of this job one of them
             * answered stays answered in its done[w]), then launch again: the
             * new workgroups take the parts still missing */
            hipError_t se = hipStreamSynchronize(g_svc.stream);
            if (se != hipSuccess) {
                g_svc.state = -1;
                return set_err(RFEC_EDEVICE, "service relaunch", se);
            }
            g_svc.in->quit = 0;
            svc_flush();
            q->alive = 1;
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            const int ke = rfec_launch_service((rfec_svc_ctl*)g_svc.dev, (rfec_svc_ctl*)g_svc.in_dev,
                                               g_svc.in_dev + g_svc.o_shards, g_svc.dev + g_svc.o_parity, DI_STRIDE,
                                               g_svc.idle_ticks, g_svc.life_ticks, g_svc.groups, g_svc.stream);
            if (ke) {
                q->alive = 0;
                g_svc.state = -1;
                return set_err(RFEC_EDEVICE, "service launch", ke);
            }
            ++g_svc.launches;
        }
        if ((spin & 4095) == 4095 && now_us() - t0 > 5e6) {
            /* no answer in 5 s: tell any live launch to leave (it may still
             * take the job; rfec_service_stop / atexit synchronise its
             * stream), fall back to per-call launches, retry in 1 s */
            __atomic_store_n(&g_svc.in->stop, 1u, __ATOMIC_RELEASE);
            svc_flush();
            g_svc.state = -2;
            g_svc.t_fail = now_us();
            return set_err(RFEC_EDEVICE, "service timeout", 0);
        }
        svc_pause();
    }
    const double t1 = now_us();
    ++g_svc.jobs;
    g_svc.t_stage += t0 - t_begin;
    g_svc.t_wait += t1 - t0;
    /* the previous job's device timing: written after its `done`, landed
     * before this one's -- when that job was answered here (a timed-out job
     * leaves its slot holding seq - 3's record) */
    const int prev_ok = seq > 1 && g_svc.last_ok == seq - 1;
    g_svc.last_ok = seq;
    if (prev_ok) {
        const uint64_t* t = q->out.t[(seq - 1) & 1u];
        if (t[0] && t[3] >= t[0]) {
            ++g_svc.dev_jobs;
            g_svc.t_dstage += (double)(t[1] - t[0]) * g_svc.tick_us;
            g_svc.t_dwork += (double)(t[2] - t[1]) * g_svc.tick_us;
            g_svc.t_drel += (double)(t[3] - t[2]) * g_svc.tick_us;
        }
    }
    return RFEC_OK;
}

/* the group encode of rfec_di_generate_group through the service (mutex held) */
static int svc_generate_group(sim_segment_t* const* segs, int k, const rfec_plan* plan)
{
    const double t_begin = now_us();
    rfec_svc_job* J = &g_svc.req->job;
    J->op = RFEC_SVC_ENCODE;
    J->n_slots = (uint32_t)k;
    J->groups = 1;
    J->capacity = SIM_VIDEO_SIZE;
    J->plan = *plan;
    for (int i = 0; i < k; ++i) {
        J->slot_nck[i] = svc_stage(svc_shard((uint32_t)i), segs[i]->data, segs[i]->data_size);
        seg_to_hdr(segs[i], (rfec_hdr*)&J->hdr[5 * i]);
    }
    return svc_run((uint32_t)k, RFEC_SVC_ENCODE, t_begin);
}

/* a group encode's results (line l: meta m[l], fec_data_size fds[l], status
 * st[l], payload at parity + l * DI_STRIDE) into the callers' sim_fec_t */
static void di_take_group(sim_segment_t* const* segs, const rfec_plan* plan, sim_fec_t* const* outs, int* rets,
                          const rfec_hdr* m, const uint16_t* fds, const int8_t* st, const uint8_t* parity)
{
    for (int l = 0; l < plan->n_lines; ++l) {
        const rfec_line* ln = &plan->line[l];
        sim_fec_t* f = outs[l];
        if (ln->count <= 1) /* :9-10 */
            continue;
        f->fec_data_size = fds[l];
        if (st[l] != 0) {
            /* over capacity (:27-28): the reference has written the first
             * member's header and the size by then, nothing else */
            seg_to_hdr(segs[ln->first], (rfec_hdr*)&f->fec_meta);
            continue;
        }
        memcpy(&f->fec_meta, &m[l], sizeof(rfec_hdr));
        memcpy(f->fec_data, parity + (size_t)l * DI_STRIDE, fds[l]);
        /* in-place zero padding of the line's members 1.. to fec_data_size (:47) */
        for (int q = 1; q < ln->count; ++q) {
            sim_segment_t* s = segs[ln->first + q * ln->stride];
            if (s->data_size < fds[l])
                memset(s->data + s->data_size, 0, (size_t)(fds[l] - s->data_size));
        }
        rets[l] = 0;
    }
}

/* Every line of `plan` over segs[0..k) in one launch (flex_fec_xor.c:4-53 per
 * line): line l's meta, fec_data_size and fec_data go to outs[l], the return
 * value flex_fec_generate would give to rets[l].  The group-level sender
 * (rfec_flex.c) and flex_fec_generate (a one-line plan) share it. */
int rfec_di_generate_group(sim_segment_t* const* segs, int k, const rfec_plan* plan, sim_fec_t* const* outs,
                           int* rets)
{
    if (k < 1 || k > DI_MAXK || plan->k != k || plan->n_lines > RFEC_MAX_LINES)
        return set_err(RFEC_EINVAL, "group above RFEC_MAX_K segments / RFEC_MAX_LINES lines", 0);
    for (int l = 0; l < plan->n_lines; ++l)
        rets[l] = -1;
    if (check_plan(plan, RFEC_MAX_K_ENCODE) != RFEC_OK)
        return RFEC_EINVAL;
    if (plan->n_lines == 0)
        return RFEC_OK;
    if (svc_acquire()) {
        const int rc = svc_generate_group(segs, k, plan);
        if (rc == RFEC_OK) {
            const rfec_svc_ctl* q = g_svc.ctl;
            di_take_group(segs, plan, outs, rets, (const rfec_hdr*)q->out.meta, q->out.fsize, q->out.status,
                          svc_out(0));
        }
        pthread_mutex_unlock(&g_svc.mu);
        if (rc == RFEC_OK)
            return RFEC_OK; /* else: the per-call launch below */
    }
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const di_layout L = di_offsets();
    rfec_hdr* hh = (rfec_hdr*)(c->host + L.hdr);
    for (int i = 0; i < k; ++i) {
        stage_payload(c->host + L.shards + (size_t)i * DI_STRIDE, segs[i]->data, segs[i]->data_size);
        seg_to_hdr(segs[i], &hh[i]);
    }
    const int e = rfec_launch_encode(plan, 1, DI_STRIDE, SIM_VIDEO_SIZE, c->dev + L.shards,
                                     (const rfec_hdr*)(c->dev + L.hdr), c->dev + L.parity,
                                     (rfec_hdr*)(c->dev + L.meta), (uint16_t*)(c->dev + L.fsize),
                                     (int8_t*)(c->dev + L.status), c->stream, g_tuning);
    if (di_sync(c, e, "group encode") != RFEC_OK) {
        di_loud(rfec_last_error());
        return RFEC_EDEVICE;
    }
    di_take_group(segs, plan, outs, rets, (const rfec_hdr*)(c->host + L.meta), (const uint16_t*)(c->host + L.fsize),
                  (const int8_t*)(c->host + L.status), c->host + L.parity);
    return RFEC_OK;
}

/* flex_fec_xor.c:4-53 on the GPU: a one-line group. */
int flex_fec_generate(sim_segment_t* segs[], int segs_count, sim_fec_t* fec)
{
    if (segs_count <= 1) /* :9-10 */
        return -1;
    if (segs_count > DI_MAXK) {
        set_err(RFEC_EINVAL, "segs_count above RFEC_MAX_K_ENCODE", 0);
        return -1;
    }
    rfec_plan p;
    memset(&p, 0, sizeof(p));
    p.k = (uint16_t)segs_count;
    p.n_lines = 1;
    p.line[0].first = 0;
    p.line[0].stride = 1;
    p.line[0].count = (uint8_t)segs_count;
    int ret = -1;
    sim_fec_t* const outs[1] = {fec};
    if (rfec_di_generate_group(segs, segs_count, &p, outs, &ret) != RFEC_OK)
        return -1;
    return ret;
}

/* n independent flex_fec_recover calls (flex_fec_xor.c:55-104) in as few
 * launches as the staging area allows: job j is a one-line group of K slots,
 * its count present members first, then zero-filled present slots (neutral
 * for the XOR of payloads and header records, and for the size checks), the
 * erased member last; K = 1 + the largest count of the launch.  rets[j] is
 * what flex_fec_recover returns for the job. */
/* a recover job's in-place zero padding of its present segments (:91), up to
 * the first one the reference rejects (:88-89) */
static void di_pad_members(const rfec_di_recover_job* J)
{
    const uint32_t Lfec = J->fec->fec_data_size;
    for (int i = 0; i < J->count; ++i) {
        if (J->segs[i]->data_size > Lfec)
            break;
        memset(J->segs[i]->data + J->segs[i]->data_size, 0, (size_t)(Lfec - J->segs[i]->data_size));
    }
}

/* a recovered segment (header r, payload data) into the job's out_seg (:64-73, :101) */
static void di_take_recovered(const rfec_di_recover_job* J, const rfec_hdr* r, const uint8_t* data)
{
    sim_segment_t* o = J->out;
    o->packet_id = r->seq;
    o->fid = r->fid;
    o->timestamp = r->ts;
    o->index = r->index;
    o->total = r->total;
    o->ftype = r->ftype;
    o->payload_type = r->payload_type;
    o->data_size = r->size;
    memcpy(o->data, data, J->fec->fec_data_size);
    o->fec_id = J->fec->fec_id;
}

/* a recover job the drop-in refuses alone: flex_fec_recover's own refusal
 * (:60-61) or this library's limits */
static int di_refused(const rfec_di_recover_job* J)
{
    if (J->count <= 0)
        return 1;
    if (J->count + 1 > RFEC_MAX_K) {
        set_err(RFEC_EINVAL, "segs_count above RFEC_MAX_K-1", 0);
        return 1;
    }
    if (J->fec->fec_data_size > SIM_VIDEO_SIZE) {
        set_err(RFEC_EINVAL, "fec_data_size above SIM_VIDEO_SIZE", 0);
        return 1;
    }
    return 0;
}

/* rfec_di_recover_lines through the service (mutex held): up to
 * RFEC_DI_GROUPS jobs per post, each its members then its parity in
 * consecutive slots, its recovered payload to output slot g */
static int svc_recover_lines(const rfec_di_recover_job* jobs, int n, int* rets)
{
    const rfec_svc_ctl* q = g_svc.ctl;
    rfec_svc_job* S = &g_svc.req->job;
    int j = 0;
    while (j < n) {
        int idx[RFEC_DI_GROUPS];
        uint32_t G = 0, ns = 0;
        const double t_begin = now_us();
        for (; j < n && G < RFEC_DI_GROUPS; ++j) {
            const rfec_di_recover_job* J = &jobs[j];
            if (di_refused(J))
                continue;
            const uint32_t c = (uint32_t)J->count;
            if (ns + c + 1 > RFEC_SVC_SLOTS || ns + c + 1 > DI_MAXK)
                break;
            S->slot0[G] = (uint16_t)ns;
            S->count[G] = (uint16_t)c;
            S->fsize[G] = J->fec->fec_data_size;
            memcpy(&S->hdr[5 * ns], &J->fec->fec_meta, sizeof(rfec_hdr));
            for (uint32_t i = 0; i < c; ++i) {
                S->slot_nck[ns + i] = svc_stage(svc_shard(ns + i), J->segs[i]->data, J->segs[i]->data_size);
                seg_to_hdr(J->segs[i], (rfec_hdr*)&S->hdr[5 * (ns + 1 + i)]);
            }
            S->slot_nck[ns + c] = svc_stage(svc_shard(ns + c), J->fec->fec_data, J->fec->fec_data_size);
            idx[G++] = j;
            ns += c + 1;
        }
        if (G == 0)
            continue;
        S->op = RFEC_SVC_RECOVER;
        S->n_slots = ns;
        S->groups = G;
        S->capacity = SIM_VIDEO_SIZE;
        const int rc = svc_run(ns, RFEC_SVC_RECOVER, t_begin);
        if (rc != RFEC_OK)
            return rc;
        for (uint32_t g = 0; g < G; ++g) {
            const rfec_di_recover_job* J = &jobs[idx[g]];
            di_pad_members(J);
            if (q->out.status[g] != 0)
                continue;
            di_take_recovered(J, (const rfec_hdr*)q->out.meta[g], svc_out(g));
            rets[idx[g]] = 0;
        }
    }
    return RFEC_OK;
}

int rfec_di_recover_lines(const rfec_di_recover_job* jobs, int n, int* rets)
{
    for (int j = 0; j < n; ++j)
        rets[j] = -1;
    if (n > 0 && svc_acquire()) {
        const int rc = svc_recover_lines(jobs, n, rets);
        pthread_mutex_unlock(&g_svc.mu);
        if (rc == RFEC_OK)
            return RFEC_OK;
        for (int j = 0; j < n; ++j) /* the per-call launches below redo them all */
            rets[j] = -1;
    }
    di_ctx* c = NULL;
    const di_layout L = di_offsets();
    int j0 = 0;
    while (j0 < n) {
        /* jobs [j0, j1) in one launch */
        int j1 = j0, K = 0;
        while (j1 < n && j1 - j0 < RFEC_DI_GROUPS) {
            const rfec_di_recover_job* J = &jobs[j1];
            if (J->count <= 0 || J->count + 1 > RFEC_MAX_K || J->fec->fec_data_size > SIM_VIDEO_SIZE) {
                if (j1 == j0) { /* refused alone: :60-61, or beyond this library's limits */
                    (void)di_refused(J);
                    ++j0;
                    ++j1;
                    continue;
                }
                break;
            }
            const int k1 = J->count + 1 > K ? J->count + 1 : K;
            if (k1 * (j1 - j0 + 1) > RFEC_MAX_K)
                break;
            K = k1;
            ++j1;
        }
        if (j1 == j0)
            continue;
        if (!c && !(c = di_get()))
            return RFEC_EDEVICE;
        const int G = j1 - j0;
        rfec_hdr* hh = (rfec_hdr*)(c->host + L.hdr);
        uint64_t* pres = (uint64_t*)(c->host + L.present);
        uint64_t* pp = (uint64_t*)(c->host + L.ppresent);
        rfec_hdr* mh = (rfec_hdr*)(c->host + L.meta);
        uint16_t* fs = (uint16_t*)(c->host + L.fsize);
        memset(pres, 0, (size_t)G * 2 * sizeof(uint64_t));
        for (int g = 0; g < G; ++g) {
            const rfec_di_recover_job* J = &jobs[j0 + g];
            uint8_t* base = c->host + L.shards + (size_t)g * K * DI_STRIDE;
            for (int i = 0; i < K - 1; ++i) {
                if (i < J->count) {
                    stage_payload(base + (size_t)i * DI_STRIDE, J->segs[i]->data, J->segs[i]->data_size);
                    seg_to_hdr(J->segs[i], &hh[g * K + i]);
                } else {
                    memset(base + (size_t)i * DI_STRIDE, 0, DI_STRIDE);
                    memset(&hh[g * K + i], 0, sizeof(rfec_hdr));
                }
                pres[2 * g + (i >> 6)] |= 1ull << (i & 63);
            }
            memset(&hh[g * K + K - 1], 0, sizeof(rfec_hdr));
            stage_payload(c->host + L.parity + (size_t)g * DI_STRIDE, J->fec->fec_data, J->fec->fec_data_size);
            memcpy(&mh[g], &J->fec->fec_meta, sizeof(rfec_hdr));
            fs[g] = J->fec->fec_data_size;
            pp[g] = 1;
        }
        static __thread rfec_kmask M; /* 1.3 KB: keep it off the stack */
        memset(&M, 0, sizeof(M));
        M.plan.k = (uint16_t)K;
        M.plan.n_lines = 1;
        M.plan.line[0].first = 0;
        M.plan.line[0].stride = 1;
        M.plan.line[0].count = (uint8_t)K;
        for (int i = 0; i < K; ++i)
            M.mask[0][i >> 6] |= 1ull << (i & 63);
        const int e = rfec_launch_recover(&M, (uint32_t)G, DI_STRIDE, SIM_VIDEO_SIZE, c->dev + L.shards,
                                          (rfec_hdr*)(c->dev + L.hdr), (const uint64_t*)(c->dev + L.present),
                                          c->dev + L.parity, (const rfec_hdr*)(c->dev + L.meta),
                                          (const uint16_t*)(c->dev + L.fsize), (const uint64_t*)(c->dev + L.ppresent),
                                          (uint64_t*)(c->dev + L.recovered), c->dev + L.ws, c->stream, g_tuning);
        if (di_sync(c, e, "flex_fec_recover") != RFEC_OK) {
            di_loud(rfec_last_error());
            return RFEC_EDEVICE;
        }
        const uint64_t* rec = (const uint64_t*)(c->host + L.recovered);
        for (int g = 0; g < G; ++g) {
            const rfec_di_recover_job* J = &jobs[j0 + g];
            di_pad_members(J);
            if (!((rec[2 * g + ((K - 1) >> 6)] >> ((K - 1) & 63)) & 1ull))
                continue;
            di_take_recovered(J, &hh[g * K + K - 1], c->host + L.shards + ((size_t)g * K + K - 1) * DI_STRIDE);
            rets[j0 + g] = 0;
        }
        j0 = j1;
    }
    return RFEC_OK;
}

/* flex_fec_xor.c:55-104 on the GPU: the n present segments plus one erased
 * slot form a one-line group that the peel + recovery kernels repair. */
int flex_fec_recover(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, sim_segment_t* out_seg)
{
    if (segs_count <= 0) /* :60-61 */
        return -1;
    const rfec_di_recover_job J = {segs, segs_count, fec, out_seg};
    int ret = -1;
    if (rfec_di_recover_lines(&J, 1, &ret) != RFEC_OK)
        return -1;
    return ret;
}
