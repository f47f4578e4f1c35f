/*
 * rfec_host.c -- C host layer of the MI355X flex-FEC engine (C99 + the HIP
 * runtime C API).  Three parts:
 *
 *  1. The planner: restates flex_fec_sender_num_packets and the row / column
 *     line layout of flex_fec_sender_update
 *     (sim_transport/fec/flex_fec_sender.c:81-135, :158-233).
 *  2. The batched device API (rfec_encode_batch / rfec_recover_batch):
 *     argument checks, then one launch through the shim in rfec_kernels.hip.
 *  3. The drop-in flex_fec_generate / flex_fec_recover
 *     (sim_transport/fec/flex_fec_xor.h:7-8): each call stages its segments
 *     into a per-thread pinned, device-mapped area and runs the same kernels
 *     on the GPU as a one-group batch.  There is no CPU compute path: without
 *     a usable HIP device the calls print an error once and return -1.
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

#include "razor_fec.h"
#include "rfec_internal.h"

/* ------------------------------------------------------------------------ */
/* errors                                                                    */
/* ------------------------------------------------------------------------ */
static __thread char t_err[256];

static int set_err(int code, const char* what, int hip_code)
{
    if (hip_code)
        snprintf(t_err, sizeof(t_err), "%s: %s (hip %d)", what, rfec_hip_error_string(hip_code), hip_code);
    else
        snprintf(t_err, sizeof(t_err), "%s", what);
    return code;
}

const char* rfec_last_error(void) { return t_err; }

int rfec_sim_video_size(void) { return SIM_VIDEO_SIZE; }

static unsigned g_tuning = 0;
void rfec_set_tuning(unsigned flags) { g_tuning = flags; }
unsigned rfec_get_tuning(void) { return g_tuning; }

/* ------------------------------------------------------------------------ */
/* 1. planner                                                                */
/* ------------------------------------------------------------------------ */
int rfec_num_packets(uint16_t k, uint8_t protect_fraction, uint8_t* row, uint8_t* col)
{
    const int n = k, pf = protect_fraction;
    uint8_t r = 0, c = 0;
    int rc = 0;
    if (n == 0) {
        /* (0, 0) */
    } else if (pf >= 10 && n >= 6) {
        /* matrix mode: near-square, column count clamped to [3, 20] */
        const double f = sqrt((double)n);
        int cols = (int)f;
        if ((float)cols + 0.1f < f)
            cols = 1 + (int)f;
        cols = cols < 3 ? 3 : (cols > 20 ? 20 : cols);
        r = (uint8_t)(n / cols + (n % cols != 0));
        c = (uint8_t)(n / r + (n % r != 0));
        rc = 1;
    } else if (pf > 0) {
        /* strip mode: about n*pf/256 row parities */
        const int lines = (n * pf + 128) >> 8;
        if (lines == 0) {
            r = 1;
            c = (uint8_t)n;
        } else {
            c = (uint8_t)(n / lines + (n % lines > 0));
            r = (uint8_t)(n / c + (n % c != 0));
        }
    }
    if (row)
        *row = r;
    if (col)
        *col = c;
    return rc;
}

static void add_line(rfec_plan* p, int first, int stride, int count, int index)
{
    if (count < 2) /* flex_fec_generate refuses <2 members: no parity on the wire */
        return;
    rfec_line* l = &p->line[p->n_lines++];
    l->first = (uint8_t)first;
    l->stride = (uint8_t)stride;
    l->count = (uint8_t)count;
    l->index = (uint8_t)index;
}

static int build_plan(uint16_t k, uint8_t row, uint8_t col, int rc, unsigned layers, rfec_plan* p)
{
    if (!p)
        return set_err(RFEC_EINVAL, "plan is NULL", 0);
    memset(p, 0, sizeof(*p));
    if (k < 1 || k > RFEC_MAX_K)
        return set_err(RFEC_EINVAL, "k out of range [1, RFEC_MAX_K]", 0);
    p->k = k;
    p->row = row;
    p->col = col;
    p->rc = (uint8_t)rc;
    if (col <= 1)
        return RFEC_OK; /* no parity at all (flex_fec_sender.c:158) */
    if (layers & RFEC_LAYER_ROWS) {
        for (int r = 0; r < row; ++r) {
            const int first = r * col;
            const int left = (int)k - first;
            add_line(p, first, 1, left < col ? left : col, r);
        }
    }
    p->n_row_lines = p->n_lines;
    if ((layers & RFEC_LAYER_COLS) && row > 1 && rc == 1) {
        for (int c = 0; c < col; ++c) {
            int count = 0;
            while (count < row && count * col + c < (int)k)
                ++count;
            add_line(p, c, col, count, 0x80 | c);
        }
    }
    return RFEC_OK;
}

int rfec_plan_from_fraction(uint16_t k, uint8_t protect_fraction, unsigned layers, rfec_plan* plan)
{
    uint8_t row, col;
    const int rc = rfec_num_packets(k, protect_fraction, &row, &col);
    return build_plan(k, row, col, rc, layers, plan);
}

int rfec_plan_matrix(uint16_t k, uint8_t row, uint8_t col, unsigned layers, rfec_plan* plan)
{
    if (row == 0 || col == 0 || (uint32_t)row * col < k)
        return set_err(RFEC_EINVAL, "row*col must cover k", 0);
    return build_plan(k, row, col, 1, layers, plan);
}

/* ------------------------------------------------------------------------ */
/* 2. batched device API                                                     */
/* ------------------------------------------------------------------------ */
static int check_plan(const rfec_plan* p)
{
    if (!p)
        return set_err(RFEC_EINVAL, "plan is NULL", 0);
    if (p->k < 1 || p->k > RFEC_MAX_K || p->n_lines > RFEC_MAX_LINES)
        return set_err(RFEC_EINVAL, "plan k / n_lines out of range", 0);
    for (int l = 0; l < p->n_lines; ++l) {
        const rfec_line* ln = &p->line[l];
        if (ln->count < 1 || ln->stride < 1)
            return set_err(RFEC_EINVAL, "plan line with zero count or stride", 0);
        if ((uint32_t)ln->first + (uint32_t)(ln->count - 1) * ln->stride >= p->k)
            return set_err(RFEC_EINVAL, "plan line member beyond k", 0);
    }
    return RFEC_OK;
}

static int check_geometry(uint32_t groups, uint32_t stride, uint32_t capacity, uint32_t rows_per_group)
{
    if (stride == 0 || stride % 16 != 0)
        return set_err(RFEC_EINVAL, "stride must be a positive multiple of 16", 0);
    if (capacity > stride || capacity > 65535)
        return set_err(RFEC_EINVAL, "capacity must be <= stride and <= 65535", 0);
    if ((uint64_t)groups * (stride / 16) >= (1ull << 31) ||
        (uint64_t)groups * rows_per_group * (stride / 16) >= (1ull << 40))
        return set_err(RFEC_EINVAL, "batch too large for one launch", 0);
    return RFEC_OK;
}

int rfec_encode_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                      const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                      uint16_t* fec_size, int8_t* status, void* stream)
{
    int rc = check_plan(plan);
    if (rc)
        return rc;
    if ((rc = check_geometry(groups, stride, capacity, plan->k)))
        return rc;
    if (groups == 0 || plan->n_lines == 0)
        return RFEC_OK;
    if (!shards || !hdr || !parity || !meta || !fec_size)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_encode(plan, groups, stride, capacity, shards, hdr, parity, meta, fec_size, status,
                                     stream, g_tuning);
    return e ? set_err(RFEC_EDEVICE, "encode launch", e) : RFEC_OK;
}

size_t rfec_recover_workspace_size(const rfec_plan* plan, uint32_t groups)
{
    if (!plan)
        return 0;
    return (size_t)groups * rfec_sched_record_bytes(plan->n_lines);
}

static void make_masks(const rfec_plan* p, rfec_kmask* M)
{
    memset(M, 0, sizeof(*M));
    M->plan = *p;
    for (int l = 0; l < p->n_lines; ++l) {
        const rfec_line* ln = &p->line[l];
        for (int q = 0; q < ln->count; ++q) {
            const int i = ln->first + q * ln->stride;
            M->mask[l][i >> 6] |= 1ull << (i & 63);
        }
    }
}

int rfec_recover_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                       uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                       const rfec_hdr* meta, const uint16_t* fec_size, const uint64_t* parity_present,
                       uint64_t* recovered, void* workspace, void* stream)
{
    int rc = check_plan(plan);
    if (rc)
        return rc;
    if ((rc = check_geometry(groups, stride, capacity, plan->k)))
        return rc;
    if (groups == 0)
        return RFEC_OK;
    if (!shards || !hdr || !present || !parity_present || !recovered || !workspace ||
        (plan->n_lines && (!parity || !meta || !fec_size)))
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    static __thread rfec_kmask M; /* 1.3 KB: keep it off the stack */
    make_masks(plan, &M);
    const int e = rfec_launch_recover(&M, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                                      parity_present, recovered, workspace, stream, g_tuning);
    return e ? set_err(RFEC_EDEVICE, "recover launch", e) : RFEC_OK;
}

int rfec_zero_tails(uint32_t groups, uint32_t k, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr,
                    void* stream)
{
    int rc = check_geometry(groups * k, stride, 0, 1);
    if (rc)
        return rc;
    if (!shards || !hdr)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    if (groups == 0 || k == 0)
        return RFEC_OK;
    const int e = rfec_launch_zero_tails(groups * k, stride, shards, hdr, stream);
    return e ? set_err(RFEC_EDEVICE, "zero_tails launch", e) : RFEC_OK;
}

/* ------------------------------------------------------------------------ */
/* 2b. wire codec (sim_proto.c / sim_proto.inl), batched                     */
/* ------------------------------------------------------------------------ */
static int check_wire(uint32_t count, uint32_t stride, uint32_t capacity, uint32_t dstride, uint32_t overhead)
{
    if (stride == 0 || stride % 16 || stride > RFEC_WIRE_MAX_DSTRIDE)
        return set_err(RFEC_EINVAL, "stride must be a positive multiple of 16, at most 2048", 0);
    if (capacity > stride || capacity > 0xFFFE)
        return set_err(RFEC_EINVAL, "capacity must be <= stride", 0);
    if (dstride % 16 || dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE)
        return set_err(RFEC_EINVAL, "dstride must be a multiple of 16 in [64, 2048]", 0);
    if (overhead && capacity + overhead > dstride)
        return set_err(RFEC_EINVAL, "dstride too small for capacity", 0);
    if ((uint64_t)count * dstride > ((uint64_t)1 << 40))
        return set_err(RFEC_EINVAL, "batch too large", 0);
    return RFEC_OK;
}

int rfec_wire_frame_fec(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                        const rfec_fec_stamp* stamps, uint32_t dstride, uint8_t* dgram, uint16_t* dlen,
                        void* stream)
{
    int rc = check_wire(count, stride, capacity, dstride, RFEC_WIRE_FEC_OVERHEAD);
    if (rc)
        return rc;
    if (count == 0)
        return RFEC_OK;
    if (!parity || !meta || !fec_size || !stamps || !dgram || !dlen)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_wire_frame_fec(count, stride, capacity, parity, meta, fec_size, status, stamps,
                                             dstride, dgram, dlen, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_frame_fec launch", e) : RFEC_OK;
}

int rfec_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                        const rfec_hdr* hdr, const rfec_seg_stamp* stamps, uint32_t dstride, uint8_t* dgram,
                        uint16_t* dlen, void* stream)
{
    int rc = check_wire(count, stride, capacity, dstride, 36);
    if (rc)
        return rc;
    if (count == 0)
        return RFEC_OK;
    if (!shards || !hdr || !stamps || !dgram || !dlen)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_wire_frame_seg(count, stride, capacity, shards, hdr, stamps, dstride, dgram, dlen,
                                             stream);
    return e ? set_err(RFEC_EDEVICE, "wire_frame_seg launch", e) : RFEC_OK;
}

int rfec_wire_parse(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen, uint32_t stride,
                    uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload, void* stream)
{
    int rc = check_wire(n, stride, capacity, dstride, 0);
    if (rc)
        return rc;
    if (n == 0)
        return RFEC_OK;
    if (!dgram || !dlen || !recs || !payload)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_wire_parse(n, dstride, dgram, dlen, stride, capacity, recs, payload, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_parse launch", e) : RFEC_OK;
}

/* ------------------------------------------------------------------------ */
/* 3. drop-in single-call path                                               */
/* ------------------------------------------------------------------------ */
#define DI_STRIDE ((SIM_VIDEO_SIZE + 15) & ~15)
#define DI_MAXK RFEC_MAX_K

/* one pinned, device-mapped staging area per calling thread */
typedef struct {
    int device;
    hipStream_t stream;
    uint8_t* host;   /* host view */
    uint8_t* dev;    /* device view of the same bytes */
    size_t bytes;
    /* rfec_host_encode_groups: two pinned host staging slots + their HBM
     * mirrors, one stream and four events per slot */
    uint8_t* bh;
    uint8_t* bd;
    size_t b_bytes;
    hipStream_t bstream[2];
    hipEvent_t ev[2][4];
    int have_ev;
} di_ctx;

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
    DI_TAKE(shards, (size_t)DI_MAXK * DI_STRIDE);
    DI_TAKE(parity, DI_STRIDE);
    DI_TAKE(hdr, DI_MAXK * sizeof(rfec_hdr));
    DI_TAKE(meta, sizeof(rfec_hdr));
    DI_TAKE(fsize, sizeof(uint16_t));
    DI_TAKE(status, 1);
    DI_TAKE(present, 2 * sizeof(uint64_t));
    DI_TAKE(ppresent, sizeof(uint64_t));
    DI_TAKE(recovered, 2 * sizeof(uint64_t));
    DI_TAKE(ws, 16);
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
    for (int s = 0; c->have_ev && s < 2; ++s) {
        for (int i = 0; i < 4; ++i)
            (void)hipEventDestroy(c->ev[s][i]);
        (void)hipStreamDestroy(c->bstream[s]);
    }
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

static di_ctx* di_get(void)
{
    pthread_once(&di_once, di_make_key);
    di_ctx* c = (di_ctx*)pthread_getspecific(di_key);
    if (c)
        return c;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        set_err(RFEC_EDEVICE, "no HIP device", e);
        di_loud(t_err);
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
        di_loud(t_err);
        di_free(c);
        return NULL;
    }
    pthread_setspecific(di_key, c);
    return c;
}

static void seg_to_hdr(const sim_segment_t* s, rfec_hdr* h)
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

static void stage_payload(uint8_t* slot, const uint8_t* data, uint32_t size)
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

/* flex_fec_xor.c:4-53 on the GPU. */
int flex_fec_generate(sim_segment_t* segs[], int segs_count, sim_fec_t* fec)
{
    if (segs_count <= 1) /* :9-10 */
        return -1;
    if (segs_count > DI_MAXK) {
        set_err(RFEC_EINVAL, "segs_count above RFEC_MAX_K", 0);
        return -1;
    }
    di_ctx* c = di_get();
    if (!c)
        return -1;
    const di_layout L = di_offsets();
    rfec_hdr* hh = (rfec_hdr*)(c->host + L.hdr);
    for (int i = 0; i < segs_count; ++i) {
        stage_payload(c->host + L.shards + (size_t)i * DI_STRIDE, segs[i]->data, segs[i]->data_size);
        seg_to_hdr(segs[i], &hh[i]);
    }
    rfec_plan p;
    memset(&p, 0, sizeof(p));
    p.k = (uint16_t)segs_count;
    p.n_lines = 1;
    p.line[0].first = 0;
    p.line[0].stride = 1;
    p.line[0].count = (uint8_t)segs_count;
    const int e = rfec_launch_encode(&p, 1, DI_STRIDE, SIM_VIDEO_SIZE, c->dev + L.shards,
                                     (const rfec_hdr*)(c->dev + L.hdr), c->dev + L.parity,
                                     (rfec_hdr*)(c->dev + L.meta), (uint16_t*)(c->dev + L.fsize),
                                     (int8_t*)(c->dev + L.status), c->stream, g_tuning);
    if (di_sync(c, e, "flex_fec_generate") != RFEC_OK) {
        di_loud(t_err);
        return -1;
    }
    const rfec_hdr* m = (const rfec_hdr*)(c->host + L.meta);
    const uint16_t fds = *(const uint16_t*)(c->host + L.fsize);
    const int8_t st = *(const int8_t*)(c->host + L.status);
    fec->fec_data_size = fds;
    if (st != 0) {
        /* over capacity (:27-28): the reference has written seg0's header and
         * the size by then, nothing else */
        seg_to_hdr(segs[0], (rfec_hdr*)&fec->fec_meta);
        return -1;
    }
    memcpy(&fec->fec_meta, m, sizeof(rfec_hdr));
    memcpy(fec->fec_data, c->host + L.parity, fds);
    /* in-place zero padding of segs[1..] to fec_data_size (:47) */
    for (int i = 1; i < segs_count; ++i)
        if (segs[i]->data_size < fds)
            memset(segs[i]->data + segs[i]->data_size, 0, (size_t)(fds - segs[i]->data_size));
    return 0;
}

/* flex_fec_xor.c:55-104 on the GPU: the n present segments plus one erased
 * slot form a one-line group that the peel + recovery kernels repair. */
int flex_fec_recover(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, sim_segment_t* out_seg)
{
    if (segs_count <= 0) /* :60-61 */
        return -1;
    if (segs_count + 1 > DI_MAXK) {
        set_err(RFEC_EINVAL, "segs_count above RFEC_MAX_K-1", 0);
        return -1;
    }
    const uint32_t Lfec = fec->fec_data_size;
    if (Lfec > SIM_VIDEO_SIZE) {
        set_err(RFEC_EINVAL, "fec_data_size above SIM_VIDEO_SIZE", 0);
        return -1;
    }
    di_ctx* c = di_get();
    if (!c)
        return -1;
    const di_layout L = di_offsets();
    const int k = segs_count + 1;
    rfec_hdr* hh = (rfec_hdr*)(c->host + L.hdr);
    for (int i = 0; i < segs_count; ++i) {
        stage_payload(c->host + L.shards + (size_t)i * DI_STRIDE, segs[i]->data, segs[i]->data_size);
        seg_to_hdr(segs[i], &hh[i]);
    }
    memset(&hh[segs_count], 0, sizeof(rfec_hdr));
    stage_payload(c->host + L.parity, fec->fec_data, Lfec);
    memcpy(c->host + L.meta, &fec->fec_meta, sizeof(rfec_hdr));
    *(uint16_t*)(c->host + L.fsize) = (uint16_t)Lfec;
    uint64_t* pres = (uint64_t*)(c->host + L.present);
    pres[0] = pres[1] = 0;
    for (int i = 0; i < segs_count; ++i)
        pres[i >> 6] |= 1ull << (i & 63);
    *(uint64_t*)(c->host + L.ppresent) = 1;
    rfec_kmask* M = (rfec_kmask*)calloc(1, sizeof(rfec_kmask));
    if (!M)
        return -1;
    M->plan.k = (uint16_t)k;
    M->plan.n_lines = 1;
    M->plan.line[0].first = 0;
    M->plan.line[0].stride = 1;
    M->plan.line[0].count = (uint8_t)k;
    for (int i = 0; i < k; ++i)
        M->mask[0][i >> 6] |= 1ull << (i & 63);
    const int e = rfec_launch_recover(M, 1, DI_STRIDE, SIM_VIDEO_SIZE, c->dev + L.shards,
                                      (rfec_hdr*)(c->dev + L.hdr), (const uint64_t*)(c->dev + L.present),
                                      c->dev + L.parity, (const rfec_hdr*)(c->dev + L.meta),
                                      (const uint16_t*)(c->dev + L.fsize), (const uint64_t*)(c->dev + L.ppresent),
                                      (uint64_t*)(c->dev + L.recovered), c->dev + L.ws, c->stream, g_tuning);
    free(M);
    if (di_sync(c, e, "flex_fec_recover") != RFEC_OK) {
        di_loud(t_err);
        return -1;
    }
    /* in-place zero padding of the present segments (:91), up to the first
     * one the reference rejects (:88-89) */
    for (int i = 0; i < segs_count; ++i) {
        if (segs[i]->data_size > Lfec)
            break;
        memset(segs[i]->data + segs[i]->data_size, 0, (size_t)(Lfec - segs[i]->data_size));
    }
    const uint64_t* rec = (const uint64_t*)(c->host + L.recovered);
    if (!((rec[segs_count >> 6] >> (segs_count & 63)) & 1ull))
        return -1;
    const rfec_hdr* r = &hh[segs_count];
    out_seg->packet_id = r->seq;
    out_seg->fid = r->fid;
    out_seg->timestamp = r->ts;
    out_seg->index = r->index;
    out_seg->total = r->total;
    out_seg->ftype = r->ftype;
    out_seg->payload_type = r->payload_type;
    out_seg->data_size = r->size;
    memcpy(out_seg->data, c->host + L.shards + (size_t)segs_count * DI_STRIDE, Lfec);
    out_seg->fec_id = fec->fec_id; /* :101 */
    return 0;
}

/* ------------------------------------------------------------------------ */
/* 4. host-resident batch (gather -> H2D -> encode -> D2H -> scatter)        */
/* ------------------------------------------------------------------------ */
#include <time.h>

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

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

static int hb_reserve(di_ctx* c, size_t slot_bytes)
{
    hipError_t e;
    if (!c->have_ev) {
        for (int s = 0; s < 2; ++s) {
            if ((e = hipStreamCreateWithFlags(&c->bstream[s], hipStreamNonBlocking)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "stream create", e);
            for (int i = 0; i < 4; ++i)
                if ((e = hipEventCreate(&c->ev[s][i])) != hipSuccess)
                    return set_err(RFEC_EDEVICE, "event create", e);
        }
        c->have_ev = 1;
    }
    if (c->b_bytes >= 2 * slot_bytes)
        return RFEC_OK;
    if (c->bh)
        (void)hipHostFree(c->bh);
    if (c->bd)
        (void)hipFree(c->bd);
    c->bh = NULL;
    c->bd = NULL;
    c->b_bytes = 0;
    if ((e = hipHostMalloc((void**)&c->bh, 2 * slot_bytes, hipHostMallocDefault)) != hipSuccess)
        return set_err(RFEC_ENOMEM, "pinned staging", e);
    if ((e = hipMalloc((void**)&c->bd, 2 * slot_bytes)) != hipSuccess)
        return set_err(RFEC_ENOMEM, "device staging", e);
    c->b_bytes = 2 * slot_bytes;
    return RFEC_OK;
}

/* the sender's fec_id sequence: +1 per group, 0 skipped (flex_fec_sender.c:241-243) */
static uint16_t fec_id_at(uint16_t id0, uint32_t g)
{
    const uint32_t base = id0 ? (uint32_t)id0 - 1u : 0u;
    return (uint16_t)((base + g) % 65535u + 1u);
}

/* ---- a tiny fork/join helper for the host-side gather / scatter ---------- */
typedef void (*pf_fn)(void* arg, size_t lo, size_t hi);
typedef struct {
    pf_fn fn;
    void* arg;
    size_t lo, hi;
} pf_job;

static void* pf_run(void* p)
{
    pf_job* j = (pf_job*)p;
    j->fn(j->arg, j->lo, j->hi);
    return NULL;
}

static int host_threads(void)
{
    const char* v = getenv("RFEC_HOST_THREADS");
    int t = v ? atoi(v) : 8;
    return t < 1 ? 1 : (t > 64 ? 64 : t);
}

static void parallel_for(size_t n, int threads, pf_fn fn, void* arg)
{
    if (threads <= 1 || n < 256) {
        fn(arg, 0, n);
        return;
    }
    pthread_t tid[64];
    pf_job job[64];
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        job[t].fn = fn;
        job[t].arg = arg;
        job[t].lo = n * t / threads;
        job[t].hi = n * (t + 1) / threads;
        if (t == threads - 1 || pthread_create(&tid[t], NULL, pf_run, &job[t]) != 0)
            break; /* the last share (or any share a thread could not take) runs here */
        started++;
    }
    for (int t = started; t < threads; ++t)
        fn(arg, job[t].lo, job[t].hi);
    for (int t = 0; t < started; ++t)
        pthread_join(tid[t], NULL);
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

/*
 * Chunked and double-buffered: while the GPU copies / encodes / copies back
 * chunk c on slot c%2's stream, the CPU threads scatter chunk c-1's parities
 * and gather chunk c+1 into the other slot, so the wall time approaches the
 * slowest stage (the PCIe copies) instead of the sum of all five.
 */
int rfec_host_encode_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                            sim_fec_t* const* fecs, uint16_t fec_id0, rfec_host_timing* timing)
{
    int rc = check_plan(plan);
    if (rc)
        return rc;
    if (groups == 0 || plan->n_lines == 0)
        return RFEC_OK;
    if (!segs || !fecs)
        return set_err(RFEC_EINVAL, "NULL segs / fecs", 0);
    if ((rc = check_geometry(groups, DI_STRIDE, SIM_VIDEO_SIZE, plan->k)))
        return rc;
    di_ctx* c = di_get();
    if (!c)
        return RFEC_EDEVICE;
    const uint32_t k = plan->k, n = plan->n_lines;
    uint32_t chunk = (groups + 7) / 8;
    chunk = chunk < 2048 ? 2048 : chunk;
    chunk = chunk > groups ? groups : chunk;
    const uint32_t nch = (groups + chunk - 1) / chunk;
    const hb_layout L = hb_offsets(chunk, k, n);
    if ((rc = hb_reserve(c, L.total)))
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
    }
    return RFEC_OK;
}
