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
#include <unistd.h>

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

int rfec_set_error(int code, const char* what) { return set_err(code, what, 0); }

/* for the other host translation units (rfec_net.c): an OS error */
int rfec_set_error_sys(int code, const char* what, int err)
{
    if (err)
        snprintf(t_err, sizeof(t_err), "%s: %s (errno %d)", what, strerror(err), err);
    else
        snprintf(t_err, sizeof(t_err), "%s", what);
    return code;
}

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
            /* the reference stores col in a uint8_t before dividing by it: a group of
             * >= 256 segments can truncate it to 0 and divide by zero there
             * (flex_fec_sender.c:122-126); here such a group gets no parity */
            c = (uint8_t)(n / lines + (n % lines > 0));
            r = c ? (uint8_t)(n / c + (n % c != 0)) : 0;
        }
    }
    if (row)
        *row = r;
    if (col)
        *col = c;
    return rc;
}

/* returns -1 when the plan would exceed RFEC_MAX_LINES lines */
static int add_line(rfec_plan* p, int first, int stride, int count, int index)
{
    if (count < 2) /* flex_fec_generate refuses <2 members: no parity on the wire */
        return 0;
    if (p->n_lines >= RFEC_MAX_LINES)
        return -1;
    rfec_line* l = &p->line[p->n_lines++];
    l->first = (uint8_t)first;
    l->stride = (uint8_t)stride;
    l->count = (uint8_t)count;
    l->index = (uint8_t)index;
    return 0;
}

static int build_plan(uint16_t k, uint8_t row, uint8_t col, int rc, unsigned layers, rfec_plan* p)
{
    if (!p)
        return set_err(RFEC_EINVAL, "plan is NULL", 0);
    memset(p, 0, sizeof(*p));
    if (k < 1 || k > RFEC_MAX_K_ENCODE)
        return set_err(RFEC_EINVAL, "k out of range [1, RFEC_MAX_K_ENCODE]", 0);
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
            if (add_line(p, first, 1, left < col ? left : col, r))
                return set_err(RFEC_EINVAL, "plan above RFEC_MAX_LINES lines", 0);
        }
    }
    p->n_row_lines = p->n_lines;
    if ((layers & RFEC_LAYER_COLS) && row > 1 && rc == 1) {
        for (int c = 0; c < col; ++c) {
            int count = 0;
            while (count < row && count * col + c < (int)k)
                ++count;
            if (add_line(p, c, col, count, 0x80 | c))
                return set_err(RFEC_EINVAL, "plan above RFEC_MAX_LINES lines", 0);
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
/* max_k: RFEC_MAX_K_ENCODE for encode plans, RFEC_MAX_K for recovery (128-bit masks) */
static int check_plan(const rfec_plan* p, uint32_t max_k)
{
    if (!p)
        return set_err(RFEC_EINVAL, "plan is NULL", 0);
    if (p->k < 1 || p->k > max_k || p->n_lines > RFEC_MAX_LINES)
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
    int rc = check_plan(plan, RFEC_MAX_K_ENCODE);
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
    return rfec_ws_bytes(plan->k, plan->n_lines, groups);
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
    int rc = check_plan(plan, RFEC_MAX_K);
    if (rc)
        return rc;
    if ((rc = check_geometry(groups, stride, capacity, plan->k)))
        return rc;
    if (groups == 0)
        return RFEC_OK;
    if (!shards || !hdr || !present || !parity_present || !recovered || !workspace ||
        (plan->n_lines && (!parity || !meta || !fec_size)))
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    if ((uintptr_t)workspace % 16) /* schedule records are read as 16-B vectors */
        return set_err(RFEC_EINVAL, "workspace must be 16-byte aligned", 0);
    {   /* the fused decode's header lanes: one per (group, line slot), 32-bit lane index */
        unsigned lg = 1;
        while ((1u << lg) < plan->n_lines)
            ++lg;
        if (((uint64_t)groups << lg) >= (1ull << 32))
            return set_err(RFEC_EINVAL, "batch too large for one launch (groups x lines)", 0);
    }
    static __thread rfec_kmask M; /* 1.3 KB: keep it off the stack */
    make_masks(plan, &M);
    const int e = rfec_launch_recover(&M, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                                      parity_present, recovered, workspace, stream, g_tuning);
    return e ? set_err(RFEC_EDEVICE, "recover launch", e) : RFEC_OK;
}

int rfec_recover_batch_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                           const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                           const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                           const uint64_t* parity_present, uint64_t* recovered, uint32_t per_group,
                           uint8_t* out_shards, rfec_hdr* out_hdr, uint8_t* out_index, void* workspace,
                           void* stream)
{
    int rc = check_plan(plan, RFEC_MAX_K);
    if (rc)
        return rc;
    if ((rc = check_geometry(groups, stride, capacity, plan->k)))
        return rc;
    if (per_group == 0 || per_group > plan->k)
        return set_err(RFEC_EINVAL, "per_group must be in [1, k]", 0);
    if ((uint64_t)groups * per_group * (stride / 16) >= (1ull << 40))
        return set_err(RFEC_EINVAL, "dense output too large", 0);
    if (groups == 0)
        return RFEC_OK;
    if (!shards || !hdr || !present || !parity_present || !recovered || !workspace || !out_shards || !out_hdr ||
        !out_index || (plan->n_lines && (!parity || !meta || !fec_size)))
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    if ((uintptr_t)workspace % 16)
        return set_err(RFEC_EINVAL, "workspace must be 16-byte aligned", 0);
    static __thread rfec_kmask M;
    make_masks(plan, &M);
    {   /* header lanes: one per (group, line slot), 32-bit lane index */
        unsigned lg = 1;
        while ((1u << lg) < plan->n_lines)
            ++lg;
        if (((uint64_t)groups << lg) >= (1ull << 32))
            return set_err(RFEC_EINVAL, "batch too large for one launch (groups x lines)", 0);
    }
    const rfec_dense_out D = {out_shards, out_hdr, out_index, per_group};
    const int e = rfec_launch_recover_out(&M, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                                          parity_present, recovered, workspace, stream, g_tuning, &D);
    return e ? set_err(RFEC_EDEVICE, "recover launch", e) : RFEC_OK;
}

int rfec_zero_tails(uint32_t groups, uint32_t k, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr,
                    void* stream)
{
    if ((uint64_t)groups * k > 0xFFFFFFFFull)
        return set_err(RFEC_EINVAL, "groups * k overflows", 0);
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
                        const rfec_fec_stamp* stamps, const uint32_t* order, uint32_t dstride, uint8_t* dgram,
                        uint16_t* dlen, void* stream)
{
    int rc = check_wire(count, stride, capacity, dstride, RFEC_WIRE_FEC_OVERHEAD);
    if (rc)
        return rc;
    if (count == 0)
        return RFEC_OK;
    if (!parity || !meta || !fec_size || !stamps || !dgram || !dlen)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_wire_frame_fec(count, stride, capacity, parity, meta, fec_size, status, stamps,
                                             order, dstride, dgram, dlen, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_frame_fec launch", e) : RFEC_OK;
}

int rfec_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                        const rfec_hdr* hdr, const rfec_seg_stamp* stamps, const uint32_t* order, uint32_t dstride,
                        uint8_t* dgram, uint16_t* dlen, void* stream)
{
    int rc = check_wire(count, stride, capacity, dstride, 36);
    if (rc)
        return rc;
    if (count == 0)
        return RFEC_OK;
    if (!shards || !hdr || !stamps || !dgram || !dlen)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_wire_frame_seg(count, stride, capacity, shards, hdr, stamps, order, dstride, dgram,
                                             dlen, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_frame_seg launch", e) : RFEC_OK;
}

/* the longest of n host-side datagram lengths (0 for none) */
static uint32_t max_dlen(const uint16_t* dlen, uint32_t n)
{
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
        m = dlen[i] > m ? dlen[i] : m;
    return m;
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
    const int e = rfec_launch_wire_parse(n, dstride, dgram, dlen, stride, capacity, recs, payload, 0, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_parse launch", e) : RFEC_OK;
}

/* ------------------------------------------------------------------------ */
/* 3. drop-in single-call path                                               */
/* ------------------------------------------------------------------------ */
#define DI_STRIDE ((SIM_VIDEO_SIZE + 15) & ~15)
#define DI_MAXK RFEC_MAX_K_ENCODE /* staging slots: a whole encode group, or the recover jobs' slots */

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
    size_t bh_bytes, bd_bytes; /* the two pinned / device staging slots, together */
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

static double now_us(void);

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
        di_loud(t_err);
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
            di_loud(t_err);
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

/* two staging slots: host_slot bytes of pinned memory and dev_slot bytes of
 * device memory each (the recover path keeps device-only regions past the
 * host-mirrored ones, so dev_slot >= host_slot there) */
static int hb_reserve(di_ctx* c, size_t host_slot, size_t dev_slot)
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
    if (c->bh_bytes < 2 * host_slot) {
        if (c->bh)
            (void)hipHostFree(c->bh);
        c->bh = NULL;
        c->bh_bytes = 0;
        if ((e = hipHostMalloc((void**)&c->bh, 2 * host_slot, hipHostMallocDefault)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "pinned staging", e);
        c->bh_bytes = 2 * host_slot;
    }
    if (c->bd_bytes < 2 * dev_slot) {
        if (c->bd)
            (void)hipFree(c->bd);
        c->bd = NULL;
        c->bd_bytes = 0;
        if ((e = hipMalloc((void**)&c->bd, 2 * dev_slot)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "device staging", e);
        c->bd_bytes = 2 * dev_slot;
    }
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
    int rc = check_plan(plan, RFEC_MAX_K_ENCODE);
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
    if ((rc = hb_reserve(c, L.total, L.total)))
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

#define RFEC_HR_SLOT_BYTES ((size_t)640 << 20)

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
    if ((rc = hb_reserve(c, L.host_total, L.total)))
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
    }
    return RFEC_OK;
}

/* ------------------------------------------------------------------------ */
/* 5. sender staging: sim_sender_put (sim_sender.c:254-377) + the flex sender */
/*    grouping (flex_fec_sender.c:49-245), frames -> datagrams                */
/* ------------------------------------------------------------------------ */
void rfec_sender_init(rfec_sender_state* st)
{
    memset(st, 0, sizeof(*st));
    st->first_ts = -1; /* no frame yet (sim_sender.c:333) */
    st->fec_id = 1;    /* flex_fec_sender_create (flex_fec_sender.c:40) */
    st->first = 1;
}

/* sizes of sim_split_frame (sim_sender.c:254-284): near-equal, the first
 * size % total segments one byte longer */
static uint32_t split_size(uint32_t size, uint32_t seg_size, uint32_t total, uint32_t i)
{
    if (size <= seg_size)
        return size;
    return size / total + (i < size % total ? 1u : 0u);
}

/* the open group closes (flex_fec_sender_update, flex_fec_sender.c:146-245)
 * if flex_fec_sender_over (:137-143); returns -1 when `groups` is full */
static int sender_close(rfec_sender_state* s, int64_t now, uint8_t pf, rfec_seg_plan* segs, uint32_t ns,
                        rfec_group_plan* groups, uint32_t max_groups, uint32_t* ng)
{
    if (!(s->fec_ts + 500 < now || s->segs_count >= 6)) /* FEC_REPAIR_WINDOW 500 ms, or >= 6 segments */
        return 0;
    rfec_plan plan;
    uint32_t n_lines = 0;
    if (s->segs_count > 0 &&
        rfec_plan_from_fraction(s->segs_count, pf, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, &plan) == RFEC_OK)
        n_lines = plan.n_lines;
    int32_t gid = -1;
    if (n_lines > 0) {
        if (*ng >= max_groups)
            return -1;
        gid = (int32_t)*ng;
        rfec_group_plan* g = &groups[(*ng)++];
        memset(g, 0, sizeof(*g));
        g->first_seg = s->open_seg;
        g->count = s->segs_count;
        g->fec_id = s->fec_id;
        g->base_id = s->base_id;
        g->protect_fraction = pf;
        g->n_lines = (uint8_t)n_lines;
        g->fec_send_id0 = s->send_id_seed + 1; /* sim_sender_fec: a send id per parity (sim_sender.c:295-296) */
        g->fec_ts = (uint32_t)(now - s->first_ts);
        s->send_id_seed += n_lines;
    }
    if (s->segs_count > 0)
        for (int32_t q = s->open_seg < 0 ? 0 : s->open_seg; q < (int32_t)ns; ++q)
            segs[q].group = gid;
    s->fec_ts = 0; /* reset, next fec_id, 0 skipped (flex_fec_sender.c:236-243) */
    s->segs_count = 0;
    s->base_id = 0;
    s->first = 1;
    if (++s->fec_id == 0)
        s->fec_id = 1;
    return 0;
}

int rfec_sender_plan(rfec_sender_state* st, const rfec_frame* frames, uint32_t n, uint32_t seg_size,
                     rfec_seg_plan* segs, uint32_t max_segs, uint32_t* n_segs, rfec_group_plan* groups,
                     uint32_t max_groups, uint32_t* n_groups)
{
    if (!st || (!frames && n) || !segs || !groups || !n_segs || !n_groups || seg_size == 0)
        return set_err(RFEC_EINVAL, "sender plan: bad argument", 0);
    rfec_sender_state s = *st;
    uint32_t ns = 0, ng = 0;
    for (uint32_t f = 0; f < n; ++f) {
        const rfec_frame* fr = &frames[f];
        const uint32_t total = fr->size <= seg_size ? 1u : (fr->size + seg_size - 1) / seg_size;
        uint32_t timestamp = 0;
        if (s.first_ts == -1)
            s.first_ts = fr->now_ms;
        else
            timestamp = (uint32_t)(fr->now_ms - s.first_ts);
        ++s.frame_id_seed;
        uint32_t off = 0;
        for (uint32_t i = 0; i < total; ++i) {
            if (ns >= max_segs)
                return set_err(RFEC_EINVAL, "sender plan: segment array too small", 0);
            rfec_seg_plan* g = &segs[ns];
            memset(g, 0, sizeof(*g));
            g->frame = f;
            g->offset = off;
            g->packet_id = ++s.packet_id_seed;
            g->send_id = ++s.send_id_seed;
            g->fid = s.frame_id_seed;
            g->timestamp = timestamp;
            g->index = (uint16_t)i;
            g->total = (uint16_t)total;
            g->ftype = fr->ftype;
            g->payload_type = fr->payload_type;
            g->data_size = (uint16_t)split_size(fr->size, seg_size, total, i);
            g->fec_id = s.fec_id;
            g->group = -2;
            off += g->data_size;
            /* flex_fec_sender_add_segment (flex_fec_sender.c:49-78) */
            if (s.fec_ts == 0) {
                s.fec_ts = fr->now_ms;
            } else if (s.fec_ts + 2000 < fr->now_ms) { /* stale open group: its segments stay unprotected */
                for (int32_t q = s.open_seg < 0 ? 0 : s.open_seg; q < (int32_t)ns; ++q)
                    segs[q].group = -1;
                s.segs_count = 0;
                s.base_id = 0;
                s.first = 1;
                s.fec_ts = fr->now_ms;
            }
            if (s.segs_count == 0)
                s.open_seg = (int32_t)ns;
            s.base_id = (s.first || g->packet_id < s.base_id) ? g->packet_id : s.base_id;
            s.first = 0;
            s.segs_count++;
            ns++;
            if (s.segs_count >= 100 && sender_close(&s, fr->now_ms, fr->protect_fraction, segs, ns, groups,
                                                    max_groups, &ng))
                return set_err(RFEC_EINVAL, "sender plan: group array too small", 0);
        }
        if (sender_close(&s, fr->now_ms, fr->protect_fraction, segs, ns, groups, max_groups, &ng))
            return set_err(RFEC_EINVAL, "sender plan: group array too small", 0);
    }
    s.open_seg = s.segs_count > 0 ? s.open_seg - (int32_t)ns : 0;
    *st = s;
    *n_segs = ns;
    *n_groups = ng;
    return RFEC_OK;
}

/* ---- frames -> datagrams ------------------------------------------------- */
typedef struct {
    uint8_t* h;     /* pinned host */
    uint8_t* d;     /* device */
    size_t bytes;
    uint8_t* carry; /* the open group's segments (slots then headers), host */
    uint32_t n_carry;
} sd_ctx;

static __thread sd_ctx t_sd;

static int sd_reserve(size_t bytes)
{
    if (t_sd.bytes >= bytes)
        return RFEC_OK;
    hipError_t e;
    if (t_sd.h)
        (void)hipHostFree(t_sd.h);
    if (t_sd.d)
        (void)hipFree(t_sd.d);
    t_sd.h = NULL;
    t_sd.d = NULL;
    t_sd.bytes = 0;
    bytes += bytes / 4;
    if ((e = hipHostMalloc((void**)&t_sd.h, bytes, hipHostMallocDefault)) != hipSuccess)
        return set_err(RFEC_ENOMEM, "send staging (host)", e);
    if ((e = hipMalloc((void**)&t_sd.d, bytes)) != hipSuccess)
        return set_err(RFEC_ENOMEM, "send staging (device)", e);
    t_sd.bytes = bytes;
    return RFEC_OK;
}

typedef struct { /* byte offsets in the staging block (host and device alike) */
    size_t slots, hdr, sstamp, sorder, fstamp, forder, in_end;
    size_t parity, meta, fsize, status, sdg, sdl, fdg, fdl, total;
} sd_layout;

static sd_layout sd_offsets(uint32_t n_slots, uint32_t n_par, uint32_t dstride)
{
    sd_layout L;
    size_t o = 0;
#define SD_TAKE(field, bytes)                           \
    do {                                                 \
        L.field = o;                                     \
        o = (o + (size_t)(bytes) + 255) & ~(size_t)255;  \
    } while (0)
    SD_TAKE(slots, (size_t)n_slots * DI_STRIDE);
    SD_TAKE(hdr, (size_t)n_slots * sizeof(rfec_hdr));
    SD_TAKE(sstamp, (size_t)n_slots * sizeof(rfec_seg_stamp));
    SD_TAKE(sorder, (size_t)n_slots * sizeof(uint32_t));
    SD_TAKE(fstamp, (size_t)n_par * sizeof(rfec_fec_stamp));
    SD_TAKE(forder, (size_t)n_par * sizeof(uint32_t));
    L.in_end = o; /* everything above goes host -> device in one copy */
    SD_TAKE(parity, (size_t)n_par * DI_STRIDE);
    SD_TAKE(meta, (size_t)n_par * sizeof(rfec_hdr));
    SD_TAKE(fsize, (size_t)n_par * sizeof(uint16_t));
    SD_TAKE(status, (size_t)n_par);
    SD_TAKE(sdg, (size_t)n_slots * dstride);
    SD_TAKE(sdl, (size_t)n_slots * sizeof(uint16_t));
    SD_TAKE(fdg, (size_t)n_par * dstride);
    SD_TAKE(fdl, (size_t)n_par * sizeof(uint16_t));
#undef SD_TAKE
    L.total = o;
    return L;
}

typedef struct {
    const rfec_frame* frames;
    const rfec_seg_plan* segs;
    const uint32_t* seg_of_slot; /* segment index, or UINT32_MAX - j for carried segment j */
    uint8_t* h;
    sd_layout L;
    uint32_t uid, n_segs;
    const uint16_t* tseq;       /* transport_seq per segment */
} sd_stage_job;

static void sd_stage(void* arg, size_t lo, size_t hi)
{
    const sd_stage_job* J = (const sd_stage_job*)arg;
    rfec_hdr* hh = (rfec_hdr*)(J->h + J->L.hdr);
    rfec_seg_stamp* ss = (rfec_seg_stamp*)(J->h + J->L.sstamp);
    uint32_t* so = (uint32_t*)(J->h + J->L.sorder);
    for (size_t s = lo; s < hi; ++s) {
        uint8_t* slot = J->h + J->L.slots + s * DI_STRIDE;
        const uint32_t i = J->seg_of_slot[s];
        if (i >= J->n_segs) { /* carried from the previous call: bytes and header already in place */
            so[s] = J->n_segs + (UINT32_MAX - i); /* framed into scratch rows past the real ones */
            memset(&ss[s], 0, sizeof(ss[s]));
            continue;
        }
        const rfec_seg_plan* g = &J->segs[i];
        memcpy(slot, J->frames[g->frame].data + g->offset, g->data_size);
        memset(slot + g->data_size, 0, DI_STRIDE - g->data_size);
        rfec_hdr* h = &hh[s];
        h->seq = g->packet_id;
        h->fid = g->fid;
        h->ts = g->timestamp;
        h->index = g->index;
        h->total = g->total;
        h->ftype = g->ftype;
        h->payload_type = g->payload_type;
        h->size = g->data_size;
        ss[s].uid = J->uid;
        ss[s].fec_id = g->fec_id;
        ss[s].send_ts = 0; /* immediate send: now - first_ts - timestamp (sim_sender.c:91) */
        ss[s].transport_seq = J->tseq[i];
        ss[s].remb = 1;    /* sim_sender.c:355 */
        ss[s].reserved = 0;
        so[s] = i;
    }
}

static int cmp_shape(const void* a, const void* b)
{
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

int rfec_host_send_frames(rfec_sender_state* st, const rfec_frame* frames, uint32_t n_frames, uint32_t uid,
                          rfec_seg_plan* segs, uint32_t max_segs, rfec_group_plan* groups, uint32_t max_groups,
                          uint32_t dstride, uint8_t* seg_dgram, uint16_t* seg_dlen, uint8_t* fec_dgram,
                          uint16_t* fec_dlen, uint32_t max_parities, rfec_send_report* rep)
{
    const double t0 = now_us();
    if (!seg_dgram || !seg_dlen || (!fec_dgram && max_parities) || !rep)
        return set_err(RFEC_EINVAL, "send frames: NULL output", 0);
    if (dstride % 16 || dstride > RFEC_WIRE_MAX_DSTRIDE || SIM_VIDEO_SIZE + RFEC_WIRE_FEC_OVERHEAD > dstride)
        return set_err(RFEC_EINVAL, "send frames: dstride must be a multiple of 16 >= SIM_VIDEO_SIZE + 49", 0);
    memset(rep, 0, sizeof(*rep));
    const rfec_sender_state st0 = *st;
    uint32_t ns = 0, ng = 0;
    int rc = rfec_sender_plan(st, frames, n_frames, SIM_VIDEO_SIZE, segs, max_segs, &ns, groups, max_groups, &ng);
    if (rc)
        return rc;
    const int32_t carried = st0.segs_count > 0 ? -st0.open_seg : 0; /* segments the carry holds */
    if (carried != (int32_t)t_sd.n_carry && carried > 0) {
        *st = st0;
        return set_err(RFEC_EINVAL, "send frames: open group carried by another thread or a plan-only call", 0);
    }
    /* parities and their creation-order indices; shapes (k, protect_fraction) */
    uint32_t n_par = 0;
    uint32_t* par0 = (uint32_t*)malloc((ng + 1) * sizeof(uint32_t));
    uint32_t* shape = (uint32_t*)malloc((ng + 1) * sizeof(uint32_t) * 2);
    uint16_t* tseq = (uint16_t*)malloc((ns + 1) * sizeof(uint16_t));
    uint32_t* seg_of_slot = (uint32_t*)malloc(((size_t)ns + RFEC_MAX_K + 1) * sizeof(uint32_t));
    uint16_t* ptseq = NULL;
    if (!par0 || !shape || !tseq || !seg_of_slot) {
        rc = set_err(RFEC_ENOMEM, "send frames: host arrays", 0);
        goto out;
    }
    for (uint32_t g = 0; g < ng; ++g) {
        par0[g] = n_par;
        n_par += groups[g].n_lines;
        shape[2 * g] = (uint32_t)groups[g].count << 8 | groups[g].protect_fraction;
        shape[2 * g + 1] = g;
    }
    if (n_par > max_parities) {
        rc = set_err(RFEC_EINVAL, "send frames: parity output too small", 0);
        goto out;
    }
    ptseq = (uint16_t*)malloc((n_par + 1) * sizeof(uint16_t));
    if (!ptseq) {
        rc = set_err(RFEC_ENOMEM, "send frames: host arrays", 0);
        goto out;
    }
    {
        /* transport_seq in creation order: each group's parities follow its last segment */
        uint32_t ts = st0.transport_seq_seed, g = 0;
        for (uint32_t i = 0; i < ns; ++i) {
            tseq[i] = (uint16_t)ts++;
            while (g < ng && groups[g].first_seg + (int32_t)groups[g].count - 1 == (int32_t)i) {
                for (uint32_t l = 0; l < groups[g].n_lines; ++l)
                    ptseq[par0[g] + l] = (uint16_t)ts++;
                ++g;
            }
        }
        st->transport_seq_seed = ts;
    }
    qsort(shape, ng, 2 * sizeof(uint32_t), cmp_shape); /* stable enough: ties keep creation order via index */
    /* slots: groups shape by shape (each group's segments contiguous), then the rest */
    uint32_t n_slots = 0;
    uint8_t* mark = (uint8_t*)calloc(ns + 1, 1);
    if (!mark) {
        rc = set_err(RFEC_ENOMEM, "send frames: host arrays", 0);
        goto out;
    }
    for (uint32_t q = 0; q < ng; ++q) {
        const rfec_group_plan* gp = &groups[shape[2 * q + 1]];
        for (int32_t j = 0; j < (int32_t)gp->count; ++j) {
            const int32_t i = gp->first_seg + j;
            seg_of_slot[n_slots++] = i >= 0 ? (uint32_t)i : UINT32_MAX - (uint32_t)(i + carried);
            if (i >= 0)
                mark[i] = 1;
        }
    }
    for (uint32_t i = 0; i < ns; ++i)
        if (!mark[i])
            seg_of_slot[n_slots++] = i;
    free(mark);
    const sd_layout L = sd_offsets(n_slots, n_par, dstride);
    if ((rc = sd_reserve(L.total)))
        goto out;
    di_ctx* c = di_get();
    if (!c) {
        rc = RFEC_EDEVICE;
        goto out;
    }
    const double t1 = now_us();
    rep->plan_us = t1 - t0;
    /* carried segments: their bytes / headers from the carry buffer */
    for (uint32_t s = 0; s < n_slots; ++s) {
        const uint32_t i = seg_of_slot[s];
        if (i < ns)
            continue;
        const uint32_t j = UINT32_MAX - i;
        memcpy(t_sd.h + L.slots + (size_t)s * DI_STRIDE, t_sd.carry + (size_t)j * DI_STRIDE, DI_STRIDE);
        memcpy(t_sd.h + L.hdr + (size_t)s * sizeof(rfec_hdr),
               t_sd.carry + (size_t)RFEC_MAX_K * DI_STRIDE + (size_t)j * sizeof(rfec_hdr), sizeof(rfec_hdr));
    }
    sd_stage_job J = {frames, segs, seg_of_slot, t_sd.h, L, uid, ns, tseq};
    parallel_for(n_slots, host_threads(), sd_stage, &J);
    /* parity stamps / order, shape by shape */
    {
        rfec_fec_stamp* fs = (rfec_fec_stamp*)(t_sd.h + L.fstamp);
        uint32_t* fo = (uint32_t*)(t_sd.h + L.forder);
        uint32_t p = 0;
        for (uint32_t q = 0; q < ng; ++q) {
            const uint32_t g = shape[2 * q + 1];
            const rfec_group_plan* gp = &groups[g];
            rfec_plan plan;
            (void)rfec_plan_from_fraction(gp->count, gp->protect_fraction, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, &plan);
            for (uint32_t l = 0; l < gp->n_lines; ++l, ++p) {
                rfec_fec_stamp* f = &fs[p];
                memset(f, 0, sizeof(*f));
                f->uid = uid;
                f->base_id = gp->base_id;
                f->send_ts = gp->fec_ts; /* sim_sender.c:113, immediate send */
                f->fec_id = gp->fec_id;
                f->count = gp->count;
                f->transport_seq = ptseq[par0[g] + l];
                f->row = plan.row;
                f->col = plan.col;
                f->index = plan.line[l].index;
                fo[p] = par0[g] + l;
            }
        }
    }
    /* remember the open group's segments for the call that closes it */
    if (st->segs_count > 0) {
        if (!t_sd.carry && !(t_sd.carry = (uint8_t*)malloc((size_t)RFEC_MAX_K * (DI_STRIDE + sizeof(rfec_hdr))))) {
            rc = set_err(RFEC_ENOMEM, "send frames: carry", 0);
            goto out;
        }
        const int32_t first = st->open_seg + (int32_t)ns; /* first open segment in this batch (may be < 0) */
        uint8_t* tmp = (uint8_t*)malloc((size_t)RFEC_MAX_K * (DI_STRIDE + sizeof(rfec_hdr)));
        if (!tmp) {
            rc = set_err(RFEC_ENOMEM, "send frames: carry", 0);
            goto out;
        }
        if (first < 0) /* still the group carried in: its earlier segments stay first */
            memcpy(tmp, t_sd.carry, (size_t)RFEC_MAX_K * (DI_STRIDE + sizeof(rfec_hdr)));
        for (uint32_t s = 0; s < n_slots; ++s) {
            const uint32_t i = seg_of_slot[s];
            const int32_t pos = i < ns ? (int32_t)i : (int32_t)(UINT32_MAX - i) - carried;
            if (pos < first)
                continue;
            const int32_t j = pos - first;
            memcpy(tmp + (size_t)j * DI_STRIDE, t_sd.h + L.slots + (size_t)s * DI_STRIDE, DI_STRIDE);
            memcpy(tmp + (size_t)RFEC_MAX_K * DI_STRIDE + (size_t)j * sizeof(rfec_hdr),
                   t_sd.h + L.hdr + (size_t)s * sizeof(rfec_hdr), sizeof(rfec_hdr));
        }
        memcpy(t_sd.carry, tmp, (size_t)RFEC_MAX_K * (DI_STRIDE + sizeof(rfec_hdr)));
        free(tmp);
        t_sd.n_carry = st->segs_count;
    } else {
        t_sd.n_carry = 0;
    }
    const double t2 = now_us();
    rep->stage_us = t2 - t1;
    {
        hipStream_t sm = c->stream;
        hipError_t e;
        hipEvent_t ev[4];
        for (int i = 0; i < 4; ++i)
            if ((e = hipEventCreate(&ev[i])) != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "event", e);
                goto out;
            }
        uint8_t* D = t_sd.d;
        (void)hipEventRecord(ev[0], sm);
        e = hipMemcpyAsync(D, t_sd.h, L.in_end, hipMemcpyHostToDevice, sm);
        (void)hipEventRecord(ev[1], sm);
        uint32_t slot0 = 0, p0 = 0;
        for (uint32_t q = 0; q < ng && e == hipSuccess && !rc;) {
            const uint32_t key = shape[2 * q];
            uint32_t q1 = q;
            while (q1 < ng && shape[2 * q1] == key)
                ++q1;
            const rfec_group_plan* gp = &groups[shape[2 * q + 1]];
            rfec_plan plan;
            (void)rfec_plan_from_fraction(gp->count, gp->protect_fraction, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, &plan);
            const uint32_t G = q1 - q;
            const int ke = rfec_launch_encode(&plan, G, DI_STRIDE, SIM_VIDEO_SIZE, D + L.slots + (size_t)slot0 * DI_STRIDE,
                                              (const rfec_hdr*)(D + L.hdr) + slot0, D + L.parity + (size_t)p0 * DI_STRIDE,
                                              (rfec_hdr*)(D + L.meta) + p0, (uint16_t*)(D + L.fsize) + p0,
                                              (int8_t*)(D + L.status) + p0, sm, g_tuning);
            if (ke)
                rc = set_err(RFEC_EDEVICE, "encode launch", ke);
            slot0 += G * gp->count;
            p0 += G * plan.n_lines;
            rep->n_shapes++;
            q = q1;
        }
        int ke = 0;
        if (!rc && e == hipSuccess && n_slots)
            ke = rfec_launch_wire_frame_seg(n_slots, DI_STRIDE, SIM_VIDEO_SIZE, D + L.slots,
                                            (const rfec_hdr*)(D + L.hdr), (const rfec_seg_stamp*)(D + L.sstamp),
                                            (const uint32_t*)(D + L.sorder), dstride, D + L.sdg,
                                            (uint16_t*)(D + L.sdl), sm);
        if (!rc && !ke && e == hipSuccess && n_par)
            ke = rfec_launch_wire_frame_fec(n_par, DI_STRIDE, SIM_VIDEO_SIZE, D + L.parity,
                                            (const rfec_hdr*)(D + L.meta), (const uint16_t*)(D + L.fsize),
                                            (const int8_t*)(D + L.status), (const rfec_fec_stamp*)(D + L.fstamp),
                                            (const uint32_t*)(D + L.forder), dstride, D + L.fdg,
                                            (uint16_t*)(D + L.fdl), sm);
        if (ke && !rc)
            rc = set_err(RFEC_EDEVICE, "frame launch", ke);
        (void)hipEventRecord(ev[2], sm);
        if (!rc && e == hipSuccess) {
            e = hipMemcpyAsync(seg_dgram, D + L.sdg, (size_t)ns * dstride, hipMemcpyDeviceToHost, sm);
            if (e == hipSuccess)
                e = hipMemcpyAsync(seg_dlen, D + L.sdl, (size_t)ns * sizeof(uint16_t), hipMemcpyDeviceToHost, sm);
            if (e == hipSuccess && n_par)
                e = hipMemcpyAsync(fec_dgram, D + L.fdg, (size_t)n_par * dstride, hipMemcpyDeviceToHost, sm);
            if (e == hipSuccess && n_par)
                e = hipMemcpyAsync(fec_dlen, D + L.fdl, (size_t)n_par * sizeof(uint16_t), hipMemcpyDeviceToHost,
                                   sm);
        }
        (void)hipEventRecord(ev[3], sm);
        hipError_t e2 = hipStreamSynchronize(sm);
        if (!rc && (e != hipSuccess || e2 != hipSuccess))
            rc = set_err(RFEC_EDEVICE, "send frames: copy / sync", e != hipSuccess ? e : e2);
        float a = 0, b = 0, d = 0;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        (void)hipEventElapsedTime(&d, ev[2], ev[3]);
        rep->h2d_us = a * 1e3;
        rep->kernel_us = b * 1e3;
        rep->d2h_us = d * 1e3;
        for (int i = 0; i < 4; ++i)
            (void)hipEventDestroy(ev[i]);
    }
    rep->n_segs = ns;
    rep->n_groups = ng;
    rep->n_parities = n_par;
out:
    if (rc && rc != RFEC_EDEVICE)
        *st = st0;
    free(par0);
    free(shape);
    free(tseq);
    free(seg_of_slot);
    free(ptseq);
    rep->total_us = now_us() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* 6. receiver ingestion (semantics: include/razor_fec.h, rfec_rx_recover)  */
/*    The control plane runs in arrival order on the host over headers only: */
/*    admission, flex lifetime, which line recovers which packet and when    */
/*    (so max_ts and first-arrival dedupe come out as the reference's).  The */
/*    bytes never leave the device: the groups are peeled there by           */
/*    rfec_recover_batch from their arrived members and registered parities. */
/* ------------------------------------------------------------------------ */
typedef struct { /* open addressing u32 -> u32, value 0 = empty */
    uint32_t* k;
    uint32_t* v;
    uint32_t mask, n;
} hmap;

static uint32_t hm_home(const hmap* m, uint32_t k) { return (k * 0x9E3779B1u) & m->mask; }

static int hm_init(hmap* m, uint32_t n)
{
    uint32_t cap = 64;
    while (cap < 2 * n + 64)
        cap <<= 1;
    m->k = (uint32_t*)malloc(cap * sizeof(uint32_t));
    m->v = (uint32_t*)calloc(cap, sizeof(uint32_t));
    m->mask = cap - 1;
    m->n = 0;
    return m->k && m->v ? 0 : -1;
}
static void hm_free(hmap* m)
{
    free(m->k);
    free(m->v);
    m->k = m->v = NULL;
}
static uint32_t hm_slot(const hmap* m, uint32_t k)
{
    uint32_t h = hm_home(m, k);
    while (m->v[h] && m->k[h] != k)
        h = (h + 1) & m->mask;
    return h;
}
static uint32_t hm_get(const hmap* m, uint32_t k) { return m->v[hm_slot(m, k)]; }
static int hm_put(hmap* m, uint32_t k, uint32_t v)
{
    if (2 * (m->n + 1) > m->mask + 1) {
        hmap g;
        if (hm_init(&g, 2 * (m->mask + 1)))
            return -1;
        for (uint32_t i = 0; i <= m->mask; ++i)
            if (m->v[i]) {
                const uint32_t s = hm_slot(&g, m->k[i]);
                g.k[s] = m->k[i];
                g.v[s] = m->v[i];
                g.n++;
            }
        hm_free(m);
        *m = g;
    }
    const uint32_t s = hm_slot(m, k);
    m->n += m->v[s] == 0;
    m->k[s] = k;
    m->v[s] = v;
    return 0;
}
static void hm_del(hmap* m, uint32_t k) /* backward-shift deletion */
{
    uint32_t h = hm_slot(m, k);
    if (!m->v[h])
        return;
    m->v[h] = 0;
    m->n--;
    for (uint32_t j = (h + 1) & m->mask; m->v[j]; j = (j + 1) & m->mask)
        if (((j - hm_home(m, m->k[j])) & m->mask) >= ((j - h) & m->mask)) {
            m->k[h] = m->k[j];
            m->v[h] = m->v[j];
            m->v[j] = 0;
            h = j;
        }
}

typedef struct {
    uint32_t count, row, col, n_groups, n_lines, row0, prow0, group0;
    uint32_t huge;        /* count > RX_MAX_COUNT or more than RFEC_MAX_LINES lines: no plan; line l = FEC
                             index l (members by rx_line_members), n_lines 256, peeled by the host into
                             line jobs (rx_big_peel) */
    uint64_t xcol[2];     /* columns c >= col a peer's parities named (bit c) */
    int16_t line_of[256]; /* FEC index -> plan line, -1: none */
    rfec_plan plan;
} rx_shape;

/* one flex receiver (flex_fec_receiver_t) from its creation to its removal */
typedef struct {
    uint32_t fec_id, base, count, row, col;
    uint32_t shape;        /* UINT32_MAX: geometry the reference ignores (col < 2, row 0, count 0) */
    uint32_t gslot, slot0, line0;
    uint32_t nsegs;        /* flex->segs.n */
    uint64_t have[4];      /* members in the flex (arrived or recovered); huge shapes: rx_has */
    uint64_t arrived[4];   /* members that arrived: the device peel starts from these (huge: slot_src) */
    uint64_t ppm;          /* registered parities, by plan line (huge: line_par >= 0) */
    uint32_t fec_ts;       /* flex->fec_ts = send_ts of the parity that created it (sim_fec.c:157) */
    int ref_ok;            /* col >= 2 && row >= 1 && count >= 1 (flex_fec_receiver.c:214, 250) */
    uint32_t gstamp;       /* == rx_sim.epoch: gslot is this device call's group slot */
} rx_inst;

typedef struct {
    rfec_hdr hdr;
    uint32_t inst;
} rx_event; /* a recovered segment: pending, then delivered */

typedef struct {
    const rfec_wire_rec* R;
    uint32_t capacity, max_ts, dropped, unmodelled;
    hmap seen, cache, flex_of, shape_of;
    rx_inst* G;
    uint32_t ng, gcap;
    rx_shape* S;
    uint32_t ns, scap;
    int32_t* slot_src; /* record of an arrived member, -1 otherwise */
    rfec_hdr* slot_hdr;
    uint32_t nslot, slotcap, slothcap; /* one count, two capacities (each array grows on its own) */
    int32_t* line_par; /* record of the registered parity, -1 otherwise */
    uint32_t nline, linecap;
    rx_event* pend;
    uint32_t npend, pendcap;
    rx_event* out;         /* delivered by this call */
    uint32_t nout, outcap;
    rfec_hdr* rh;          /* headers of delivered (recovered) segments the cache refers to */
    uint32_t nrh, rhcap;
    uint32_t* dl;          /* instances that deliver in this device call */
    uint32_t ndl, dlcap;
    rfec_line_job* jobs;   /* groups above RFEC_MAX_K: this call's line jobs (rx_big_peel) */
    uint32_t njobs, jobcap;
    uint16_t* jlevel;      /* a job's dependency level (1 = arrived members only) */
    uint32_t jlevelcap;
    int32_t* jmem;         /* member codes: record >= 0, job j as -1 - j */
    uint32_t njmem, jmemcap;
    uint32_t epoch;        /* device call counter (rx_inst.gstamp) */
    int oom;
} rx_sim;

#define RX_GROW(ptr, n, cap, need, T)                                                   \
    do {                                                                                \
        if ((n) + (need) > (cap)) {                                                     \
            uint32_t c_ = (cap) ? 2 * (cap) : 1024;                                     \
            while (c_ < (n) + (need))                                                   \
                c_ *= 2;                                                                \
            T* p_ = (T*)realloc((ptr), (size_t)c_ * sizeof(T));                         \
            if (!p_) {                                                                  \
                X->oom = 1;                                                             \
                break;                                                                  \
            }                                                                           \
            (ptr) = p_;                                                                 \
            (cap) = c_;                                                                 \
        }                                                                               \
    } while (0)

static rfec_hdr rec_hdr(const rfec_wire_rec* r)
{
    rfec_hdr h = r->hdr;
    h.size = r->data_size; /* seg.data_size = the datagram's (sim_receiver.c) */
    return h;
}

/* members of the reference's line `index` of a (count, row, col) flex:
 * flex_recover_row walks i < col, flex_recover_col i < row, both stopping at
 * the first position >= count (flex_fec_receiver.c:118-126, 175-183) */
static uint32_t rx_line_members(uint32_t count, uint32_t row, uint32_t col, uint32_t index, uint32_t* first,
                                uint32_t* stride)
{
    const uint32_t x = index & 0x7Fu;
    uint32_t n = 0;
    if (index & 0x80u) {
        while (n < row && n * col + x < count)
            ++n;
        *first = x;
        *stride = col;
    } else {
        while (n < col && x * col + n < count)
            ++n;
        *first = x * col;
        *stride = 1;
    }
    return n;
}

/* line l of flex g: its members and whether its parity is registered */
static uint32_t rx_line(const rx_sim* X, const rx_inst* g, uint32_t l, uint32_t* first, uint32_t* stride, int* reg)
{
    const rx_shape* sh = &X->S[g->shape];
    if (sh->huge) {
        *reg = X->line_par[g->line0 + l] >= 0;
        return rx_line_members(g->count, g->row, g->col, l, first, stride);
    }
    const rfec_line* ln = &sh->plan.line[l];
    *reg = (int)((g->ppm >> l) & 1ull);
    *first = ln->first;
    *stride = ln->stride;
    return ln->count;
}

/* member t of flex g is in it (arrived or recovered); a huge flex's slot
 * header holds the member's seq once it is in, ~(base + t) before */
static int rx_has(const rx_sim* X, const rx_inst* g, uint32_t t)
{
    if (X->S[g->shape].huge)
        return X->slot_hdr[g->slot0 + t].seq == g->base + t;
    return (int)((g->have[t >> 6] >> (t & 63)) & 1ull);
}

static void rx_pend(rx_sim* X, const rfec_hdr* h, uint32_t inst) /* sim_fec_packet_add_recover (sim_fec.c:104-119) */
{
    for (uint32_t i = 0; i < X->npend; ++i)
        if (X->pend[i].hdr.seq == h->seq)
            return;
    RX_GROW(X->pend, X->npend, X->pendcap, 1, rx_event);
    if (X->oom)
        return;
    X->pend[X->npend].hdr = *h;
    X->pend[X->npend++].inst = inst;
}

/* flex_recover_row / flex_recover_col (flex_fec_receiver.c:105-206) over headers */
static void rx_check_line(rx_sim* X, uint32_t ii, int l)
{
    const rx_inst* g = &X->G[ii];
    if (l < 0 || g->nsegs >= g->count)
        return;
    uint32_t first, stride;
    int reg;
    const uint32_t n = rx_line(X, g, (uint32_t)l, &first, &stride, &reg);
    if (!reg)
        return;
    uint32_t loss = 0, cnt = 0;
    for (uint32_t q = 0; q < n; ++q) {
        if (rx_has(X, g, first + q * stride))
            cnt++;
        else
            loss++;
    }
    if (loss != 1 || cnt == 0)
        return;
    const rfec_wire_rec* f = &X->R[X->line_par[g->line0 + l]];
    const uint32_t L = f->data_size;
    if (L > X->capacity)
        return;
    rfec_hdr h = f->hdr; /* flex_fec_xor.c:64-99 */
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t i = first + q * stride;
        if (!rx_has(X, g, i))
            continue;
        const rfec_hdr* m = &X->slot_hdr[g->slot0 + i];
        if (L < m->size)
            return;
        h.seq ^= m->seq;
        h.fid ^= m->fid;
        h.ts ^= m->ts;
        h.index ^= m->index;
        h.total ^= m->total;
        h.ftype ^= m->ftype;
        h.payload_type ^= m->payload_type;
        h.size ^= m->size;
    }
    if (h.size > L)
        return;
    rx_pend(X, &h, ii);
}

/* flex_fec_receiver_on_segment (flex_fec_receiver.c:243-280); src = record or -1 */
static void rx_on_segment(rx_sim* X, uint32_t ii, const rfec_hdr* h, int32_t src, int check)
{
    rx_inst* g = &X->G[ii];
    if (!g->ref_ok || h->seq < g->base)
        return;
    if (g->shape == UINT32_MAX) {
        X->unmodelled++;
        return;
    }
    const uint32_t t = h->seq - g->base;
    if (t < g->count) {
        if (rx_has(X, g, t))
            return;
        if (!X->S[g->shape].huge)
            g->have[t >> 6] |= 1ull << (t & 63);
        X->slot_hdr[g->slot0 + t] = *h;
        if (src >= 0) {
            if (!X->S[g->shape].huge)
                g->arrived[t >> 6] |= 1ull << (t & 63);
            X->slot_src[g->slot0 + t] = src;
        }
    } else if (src < 0) {
        X->unmodelled++; /* a recovered header outside its group: inconsistent parities */
    }
    g->nsegs++;
    if (check) {
        const rx_shape* sh = &X->S[g->shape];
        const uint32_t r = t / g->col, c = t % g->col;
        rx_check_line(X, ii, r < 128 ? sh->line_of[r] : -1);
        rx_check_line(X, ii, c < 128 ? sh->line_of[0x80 | c] : -1);
    }
}

static void rx_remove(rx_sim* X, uint32_t ii) /* sim_fec_evict_segment + flex removal (sim_fec.c:93-102, 199-205) */
{
    const rx_inst* g = &X->G[ii];
    for (uint32_t i = 0; i < g->count; ++i)
        hm_del(&X->cache, g->base + i);
    hm_del(&X->flex_of, g->fec_id);
}

/* sim_fec_put_segment (sim_fec.c:171-207); cache values: record + 1, or 0x80000000 | index into X->rh */
static void rx_put_segment(rx_sim* X, const rfec_hdr* h, uint16_t fec_id, uint32_t cval, int32_t src)
{
    if (h->seq == 0 || hm_get(&X->cache, h->seq))
        return;
    X->max_ts = h->ts > X->max_ts ? h->ts : X->max_ts;
    if (hm_put(&X->cache, h->seq, cval)) {
        X->oom = 1;
        return;
    }
    const uint32_t fi = hm_get(&X->flex_of, fec_id);
    if (!fi)
        return;
    rx_on_segment(X, fi - 1, h, src, 1);
    if (X->G[fi - 1].nsegs >= X->G[fi - 1].count) /* flex_fec_receiver_full */
        rx_remove(X, fi - 1);
}

/* The device plan of a flex geometry: every row with 2+ members (also rows
 * at and beyond `row` when row * col < count: the reference bounds rows by
 * count only), every column c < col with 2+ members, and the extra columns
 * c >= col of xcol.  Lines of fewer than 2 members can never recover (one
 * missing member leaves none present).  Standard geometry (row * col >=
 * count, no extra columns) is exactly rfec_plan_matrix's plan. */
static int rx_build_plan(uint32_t count, uint32_t row, uint32_t col, const uint64_t* xcol, rfec_plan* p)
{
    if (row * col >= count && !xcol[0] && !xcol[1])
        return rfec_plan_matrix((uint16_t)count, (uint8_t)row, (uint8_t)col, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, p);
    memset(p, 0, sizeof(*p));
    p->k = (uint16_t)count;
    p->row = (uint8_t)row;
    p->col = (uint8_t)col;
    p->rc = 1;
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t x = 0; x < 128; ++x) {
            if (pass == 1 && x >= col && !((xcol[x >> 6] >> (x & 63)) & 1ull))
                continue;
            uint32_t first, stride;
            const uint32_t n = rx_line_members(count, row, col, pass ? (0x80u | x) : x, &first, &stride);
            if (n < 2)
                continue;
            if (p->n_lines >= RFEC_MAX_LINES)
                return RFEC_EINVAL;
            rfec_line* l = &p->line[p->n_lines++];
            l->first = (uint8_t)first;
            l->stride = (uint8_t)stride;
            l->count = (uint8_t)n;
            l->index = (uint8_t)(pass ? (0x80u | x) : x);
        }
        if (pass == 0)
            p->n_row_lines = p->n_lines;
    }
    return RFEC_OK;
}

/* flexes of up to 255 segments and 64 lines have a device plan (8-bit
 * members); above RFEC_MAX_K the device recovery takes line jobs (rx_big_peel)
 * instead of the batched peel, whose masks hold 128 members.  Larger flexes
 * (a foreign peer's: the reference receiver takes any uint16_t count,
 * flex_fec_receiver.c:69-88, and up to 128 rows and 128 columns of FEC
 * indices) are huge shapes: line = FEC index, line jobs too. */
#define RX_MAX_COUNT 255u

static uint32_t rx_shape_of(rx_sim* X, uint32_t count, uint32_t row, uint32_t col, const uint64_t* xcol)
{
    if (row > 255 || col > 255)
        return UINT32_MAX;
    const int extended = xcol[0] || xcol[1];
    const uint32_t key = count << 16 | row << 8 | col;
    if (!extended) {
        const uint32_t s = hm_get(&X->shape_of, key);
        if (s)
            return s - 1;
    } else { /* rare (a peer's extra columns): a scan */
        for (uint32_t s = 0; s < X->ns; ++s)
            if (X->S[s].count == count && X->S[s].row == row && X->S[s].col == col && X->S[s].xcol[0] == xcol[0] &&
                X->S[s].xcol[1] == xcol[1])
                return s;
    }
    RX_GROW(X->S, X->ns, X->scap, 1, rx_shape);
    if (X->oom)
        return UINT32_MAX;
    rx_shape* sh = &X->S[X->ns];
    memset(sh, 0, sizeof(*sh));
    sh->count = count;
    sh->row = row;
    sh->col = col;
    sh->xcol[0] = xcol[0];
    sh->xcol[1] = xcol[1];
    sh->huge = count > RX_MAX_COUNT || rx_build_plan(count, row, col, xcol, &sh->plan) != RFEC_OK;
    if (sh->huge) { /* every FEC index is a line */
        sh->n_lines = 256;
        for (int i = 0; i < 256; ++i)
            sh->line_of[i] = (int16_t)i;
    } else {
        sh->n_lines = sh->plan.n_lines;
        for (int i = 0; i < 256; ++i)
            sh->line_of[i] = -1;
        for (uint32_t l = 0; l < sh->n_lines; ++l)
            sh->line_of[sh->plan.line[l].index] = (int16_t)l;
    }
    if (!extended && hm_put(&X->shape_of, key, X->ns + 1)) {
        X->oom = 1;
        return UINT32_MAX;
    }
    return X->ns++;
}

/* A parity for a column c >= col of flex ii (a peer's plan, not razor's
 * sender): the flex moves to the shape with that column added, its
 * registered parities carried over by index.  Returns the column's line in
 * the new shape, or -1 (no room: the parity stays unmodelled). */
static int rx_extend(rx_sim* X, uint32_t ii, uint32_t c)
{
    rx_inst* g = &X->G[ii];
    uint64_t xcol[2] = {X->S[g->shape].xcol[0], X->S[g->shape].xcol[1]};
    xcol[c >> 6] |= 1ull << (c & 63);
    const uint32_t ns = rx_shape_of(X, g->count, g->row, g->col, xcol);
    if (ns == UINT32_MAX)
        return -1;
    const rx_shape* nsh = &X->S[ns]; /* (X->S may have moved) */
    const rx_shape* osh = &X->S[g->shape];
    RX_GROW(X->line_par, X->nline, X->linecap, nsh->n_lines, int32_t);
    if (X->oom)
        return -1;
    uint64_t ppm = 0;
    for (uint32_t l = 0; l < nsh->n_lines; ++l) {
        const int ol = osh->line_of[nsh->huge ? l : nsh->plan.line[l].index];
        X->line_par[X->nline + l] = ol >= 0 && ((g->ppm >> ol) & 1ull) ? X->line_par[g->line0 + ol] : -1;
        if (ol >= 0 && ((g->ppm >> ol) & 1ull) && !nsh->huge)
            ppm |= 1ull << l;
    }
    if (nsh->huge) /* more than RFEC_MAX_LINES lines now: membership moves to the slot headers (rx_has) */
        for (uint32_t t = 0; t < g->count; ++t)
            if (!((g->have[t >> 6] >> (t & 63)) & 1ull))
                X->slot_hdr[g->slot0 + t].seq = ~(g->base + t);
    g->line0 = X->nline;
    X->nline += nsh->n_lines;
    g->ppm = ppm;
    g->shape = ns;
    return nsh->line_of[0x80u | c];
}

/* sim_fec_put_fec_packet (sim_fec.c:141-169) -> flex_fec_receiver_on_fec (flex_fec_receiver.c:208-241) */
static void rx_put_fec(rx_sim* X, uint32_t a)
{
    const rfec_wire_rec* f = &X->R[a];
    if (f->base_id + f->count == 0u || f->send_ts + 3000u < X->max_ts) {
        X->dropped++;
        return;
    }
    uint32_t fi = hm_get(&X->flex_of, f->fec_id);
    if (!fi) { /* flex_fec_receiver_active (flex_fec_receiver.c:69-88) */
        RX_GROW(X->G, X->ng, X->gcap, 1, rx_inst);
        if (X->oom)
            return;
        rx_inst* g = &X->G[X->ng];
        memset(g, 0, sizeof(*g));
        g->fec_id = f->fec_id;
        g->base = f->base_id;
        g->count = f->count;
        g->row = f->row;
        g->col = f->col;
        g->fec_ts = f->send_ts;
        g->ref_ok = g->col >= 2 && g->row >= 1 && g->count >= 1;
        static const uint64_t no_xcol[2] = {0, 0};
        g->shape = g->ref_ok ? rx_shape_of(X, g->count, g->row, g->col, no_xcol) : UINT32_MAX;
        if (g->shape != UINT32_MAX) {
            rx_shape* sh = &X->S[g->shape];
            g->gslot = sh->n_groups++;
            RX_GROW(X->slot_src, X->nslot, X->slotcap, g->count, int32_t);
            RX_GROW(X->slot_hdr, X->nslot, X->slothcap, g->count, rfec_hdr);
            RX_GROW(X->line_par, X->nline, X->linecap, sh->n_lines, int32_t);
            if (X->oom)
                return;
            g->slot0 = X->nslot;
            g->line0 = X->nline;
            for (uint32_t i = 0; i < g->count; ++i) {
                X->slot_src[X->nslot + i] = -1;
                X->slot_hdr[X->nslot + i].seq = ~(g->base + i); /* rx_has: not in the flex */
            }
            for (uint32_t l = 0; l < sh->n_lines; ++l)
                X->line_par[X->nline + l] = -1;
            X->nslot += g->count;
            X->nline += sh->n_lines;
        } else if (g->ref_ok) {
            X->unmodelled++;
        }
        fi = ++X->ng;
        if (hm_put(&X->flex_of, f->fec_id, fi)) {
            X->oom = 1;
            return;
        }
        for (uint32_t i = 0; i < g->count && g->shape != UINT32_MAX; ++i) { /* sim_fec_add_segment_to_flex */
            const uint32_t c = hm_get(&X->cache, g->base + i);
            if (!c)
                continue;
            if (c & 0x80000000u) {
                rx_on_segment(X, fi - 1, &X->rh[c & 0x7FFFFFFFu], -1, 0);
            } else {
                const rfec_hdr h = rec_hdr(&X->R[c - 1]);
                rx_on_segment(X, fi - 1, &h, (int32_t)(c - 1), 0);
            }
        }
    }
    rx_inst* g = &X->G[fi - 1];
    if (!g->ref_ok || g->shape == UINT32_MAX)
        return;
    int l = X->S[g->shape].line_of[f->index];
    if (X->S[g->shape].huge) { /* line = index; the parity registered once */
        uint32_t first, stride;
        if (rx_line_members(g->count, g->row, g->col, f->index, &first, &stride) < 2 ||
            X->line_par[g->line0 + l] >= 0)
            return;
        X->line_par[g->line0 + l] = (int32_t)a;
        rx_check_line(X, fi - 1, l);
        return;
    }
    if (l < 0) {
        uint32_t first, stride;
        if (rx_line_members(g->count, g->row, g->col, f->index, &first, &stride) < 2)
            return; /* a line that can never recover (flex_fec_receiver.c:133-134, 189-190) */
        /* a column c >= col (razor's sender never emits one; a peer may) */
        if ((l = rx_extend(X, fi - 1, f->index & 0x7Fu)) < 0) {
            X->unmodelled++;
            return;
        }
        g = &X->G[fi - 1];
    }
    if (X->S[g->shape].huge) { /* (the extension took it past RFEC_MAX_LINES lines) */
        if (X->line_par[g->line0 + l] >= 0)
            return;
    } else {
        if ((g->ppm >> l) & 1ull)
            return;
        g->ppm |= 1ull << l;
    }
    X->line_par[g->line0 + l] = (int32_t)a;
    rx_check_line(X, fi - 1, l);
}

/* sim_receiver_recover (sim_receiver.c:780-804): lowest packet_id first, cascading */
static void rx_drain(rx_sim* X)
{
    while (X->npend && !X->oom) {
        uint32_t b = 0;
        for (uint32_t i = 1; i < X->npend; ++i)
            if (X->pend[i].hdr.seq < X->pend[b].hdr.seq)
                b = i;
        const rx_event e = X->pend[b];
        X->pend[b] = X->pend[--X->npend];
        if (hm_get(&X->seen, e.hdr.seq))
            continue;
        RX_GROW(X->out, X->nout, X->outcap, 1, rx_event);
        RX_GROW(X->rh, X->nrh, X->rhcap, 1, rfec_hdr);
        if (X->oom || hm_put(&X->seen, e.hdr.seq, 1)) {
            X->oom = 1;
            return;
        }
        X->out[X->nout++] = e;
        X->rh[X->nrh] = e.hdr;
        const uint32_t idx = X->nrh++;
        rx_put_segment(X, &e.hdr, (uint16_t)X->G[e.inst].fec_id, 0x80000000u | idx, -1);
    }
}

static void rx_sim_free(rx_sim* X)
{
    hm_free(&X->seen);
    hm_free(&X->cache);
    hm_free(&X->flex_of);
    hm_free(&X->shape_of);
    free(X->G);
    free(X->S);
    free(X->slot_src);
    free(X->slot_hdr);
    free(X->line_par);
    free(X->pend);
    free(X->out);
    free(X->rh);
    free(X->dl);
    free(X->jobs);
    free(X->jlevel);
    free(X->jmem);
}

static int cmp_u32(const void* a, const void* b)
{
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* keys of a map, ascending (the skiplists' iteration order); NULL on OOM */
static uint32_t* hm_sorted_keys(const hmap* m, uint32_t* n)
{
    uint32_t* k = (uint32_t*)malloc(((size_t)m->n + 1) * sizeof(uint32_t));
    *n = 0;
    if (!k)
        return NULL;
    for (uint32_t i = 0; i <= m->mask; ++i)
        if (m->v[i])
            k[(*n)++] = m->k[i];
    qsort(k, *n, sizeof(uint32_t), cmp_u32);
    return k;
}

/* sim_fec_evict (sim_fec.c:209-241) past its 300 ms wall-clock gate: flexes in
 * fec_id order while stale (fec_ts + 3000 <= max_ts) or full, removed with
 * their members' cache entries; then cached segments in packet_id order while
 * older than 6 s (timestamp + 6000 < max_ts).  Both walks stop at the first
 * entry that stays, as the skiplist walks do. */
static void rx_evict(rx_sim* X)
{
    uint32_t n = 0;
    uint32_t* k = hm_sorted_keys(&X->flex_of, &n);
    if (!k) {
        X->oom = 1;
        return;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t fi = hm_get(&X->flex_of, k[i]) - 1;
        const rx_inst* g = &X->G[fi];
        if (!(g->fec_ts + 3000u <= X->max_ts || g->nsegs >= g->count))
            break;
        rx_remove(X, fi);
    }
    free(k);
    k = hm_sorted_keys(&X->cache, &n);
    if (!k) {
        X->oom = 1;
        return;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t c = hm_get(&X->cache, k[i]);
        const uint32_t ts = (c & 0x80000000u) ? X->rh[c & 0x7FFFFFFFu].ts : X->R[c - 1].hdr.ts;
        if (!(ts + 6000u < X->max_ts))
            break;
        hm_del(&X->cache, k[i]);
    }
    free(k);
}

static int cmp_event(const void* a, const void* b)
{
    const uint32_t x = ((const rx_event*)a)->hdr.seq, y = ((const rx_event*)b)->hdr.seq;
    return x < y ? -1 : x > y;
}

typedef struct {
    uint8_t* h;  /* pinned, device-mapped */
    uint8_t* hd; /* h as the device addresses it */
    size_t hb;
    uint8_t* d;
    size_t db;
} rx_ctx;
static __thread rx_ctx t_rx;

/* The device address of host memory the device can read directly (pinned:
 * rfec_pinned_alloc, hipHostMalloc, registered), else NULL (pageable: the
 * caller copies).  A failed query leaves no pending HIP error behind. */
static const uint8_t* host_mapped(const void* p)
{
    hipPointerAttribute_t a;
    void* d = NULL;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost ||
        hipHostGetDevicePointer(&d, (void*)p, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return NULL;
    }
    return (const uint8_t*)d;
}

/* Grows the per-thread pinned / device areas.  The first `keep` bytes of the
 * pinned area survive a grow (copied into the new block before the old one is
 * freed: the allocator may hand back the same address, so callers cannot tell
 * a grow from the pointer). */
static int rx_reserve(size_t host_bytes, size_t dev_bytes, size_t keep)
{
    hipError_t e;
    if (t_rx.hb < host_bytes) {
        uint8_t* nh = NULL;
        host_bytes += host_bytes / 4;
        void* nd = NULL;
        if ((e = hipHostMalloc((void**)&nh, host_bytes, hipHostMallocMapped)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx staging (host)", e);
        if ((e = hipHostGetDevicePointer(&nd, nh, 0)) != hipSuccess) {
            (void)hipHostFree(nh);
            return set_err(RFEC_EDEVICE, "rx staging (host): device view", e);
        }
        if (t_rx.h) {
            if (keep)
                memcpy(nh, t_rx.h, keep < t_rx.hb ? keep : t_rx.hb);
            (void)hipHostFree(t_rx.h);
        }
        t_rx.h = nh;
        t_rx.hd = (uint8_t*)nd;
        t_rx.hb = host_bytes;
    }
    if (t_rx.db < dev_bytes) {
        if (t_rx.d)
            (void)hipFree(t_rx.d);
        t_rx.d = NULL;
        t_rx.db = 0;
        dev_bytes += dev_bytes / 4;
        if ((e = hipMalloc((void**)&t_rx.d, dev_bytes)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx workspace (device)", e);
        t_rx.db = dev_bytes;
    }
    return RFEC_OK;
}

#define RX_ALIGN(x) (((x) + 255) & ~(size_t)255)

static int rx_tables_init(rx_sim* X, uint32_t n)
{
    return hm_init(&X->seen, n) || hm_init(&X->cache, n) || hm_init(&X->flex_of, 1024) || hm_init(&X->shape_of, 64);
}

/* The control plane, in arrival order, over records [a0, a0 + n) of X->R:
 * sim_receiver_put / sim_receiver_put_fec and the recovery cascade. */
static void rx_run(rx_sim* X, uint32_t a0, uint32_t n)
{
    for (uint32_t a = a0; a < a0 + n && !X->oom; ++a) {
        const rfec_wire_rec* r = &X->R[a];
        if (r->status != RFEC_WIRE_OK)
            continue;
        if (r->mid == RFEC_WIRE_SEG) { /* sim_receiver_put (sim_receiver.c:811-827) */
            if (hm_get(&X->seen, r->hdr.seq))
                continue;
            if (hm_put(&X->seen, r->hdr.seq, 1)) {
                X->oom = 1;
                break;
            }
            if (r->fec_id == 0)
                continue;
            const rfec_hdr h = rec_hdr(r);
            rx_put_segment(X, &h, r->fec_id, a + 1, (int32_t)a);
        } else if (r->mid == RFEC_WIRE_FEC) {
            rx_put_fec(X, a);
        }
        rx_drain(X);
    }
}

/* A group recovered by line jobs (rx_line_jobs: above RFEC_MAX_K segments or a
 * huge shape -- a foreign peer's flex): the canonical
 * peel (lines in plan order -- rows, then columns -- to a fixpoint, with
 * flex_fec_recover's header checks, flex_fec_xor.c:60-99) from its arrived
 * members and registered parities, over headers on the host; each firing
 * becomes a line job the device runs (rfec_launch_line_jobs).  job_of[t]: the
 * job recovering member t, or -1.  Returns -1 when out of memory. */
static int rx_big_peel(rx_sim* X, uint32_t gi, int32_t* job_of)
{
    const rx_inst* g = &X->G[gi];
    const rx_shape* sh = &X->S[g->shape];
    const uint32_t k = g->count, NL = sh->n_lines;
    rfec_hdr* hd = (rfec_hdr*)malloc((size_t)k * sizeof(rfec_hdr));
    int32_t* src = (int32_t*)malloc((size_t)k * sizeof(int32_t));
    uint16_t* lvl = (uint16_t*)malloc((size_t)k * sizeof(uint16_t));
    uint8_t* have = (uint8_t*)malloc(k);
    if (!hd || !src || !lvl || !have) {
        free(hd);
        free(src);
        free(lvl);
        free(have);
        return -1;
    }
    for (uint32_t i = 0; i < k; ++i) {
        job_of[i] = -1;
        lvl[i] = 0;
        src[i] = X->slot_src[g->slot0 + i];
        have[i] = src[i] >= 0; /* the peel starts from the arrived members */
        if (have[i])
            hd[i] = X->slot_hdr[g->slot0 + i];
    }
    for (int progress = 1; progress && !X->oom;) {
        progress = 0;
        for (uint32_t l = 0; l < NL && !X->oom; ++l) {
            uint32_t first, stride;
            int reg;
            const uint32_t n = rx_line(X, g, l, &first, &stride, &reg);
            if (!reg)
                continue;
            uint32_t miss = 0, present = 0, t = 0;
            for (uint32_t q = 0; q < n; ++q) {
                const uint32_t i = first + q * stride;
                if (have[i]) {
                    present++;
                } else {
                    miss++;
                    t = i;
                }
            }
            if (miss != 1 || present == 0)
                continue;
            const rfec_wire_rec* f = &X->R[X->line_par[g->line0 + l]];
            const uint32_t L = f->data_size;
            if (L > X->capacity)
                continue;
            rfec_hdr h = f->hdr;
            int ok = 1;
            uint16_t level = 0;
            for (uint32_t q = 0; q < n && ok; ++q) {
                const uint32_t i = first + q * stride;
                if (i == t)
                    continue;
                const rfec_hdr* m = &hd[i];
                ok = m->size <= L;
                h.seq ^= m->seq;
                h.fid ^= m->fid;
                h.ts ^= m->ts;
                h.index ^= m->index;
                h.total ^= m->total;
                h.ftype ^= m->ftype;
                h.payload_type ^= m->payload_type;
                h.size ^= m->size;
                level = lvl[i] > level ? lvl[i] : level;
            }
            if (!ok || h.size > L)
                continue;
            RX_GROW(X->jobs, X->njobs, X->jobcap, 1, rfec_line_job);
            RX_GROW(X->jlevel, X->njobs, X->jlevelcap, 1, uint16_t);
            RX_GROW(X->jmem, X->njmem, X->jmemcap, present, int32_t);
            if (X->oom)
                break;
            rfec_line_job* J = &X->jobs[X->njobs];
            J->out = (int32_t)X->njobs;
            J->parity = X->line_par[g->line0 + l];
            J->member0 = X->njmem;
            J->n_members = present;
            for (uint32_t q = 0; q < n; ++q) {
                const uint32_t i = first + q * stride;
                if (i != t)
                    X->jmem[X->njmem++] = src[i];
            }
            X->jlevel[X->njobs] = (uint16_t)(level + 1);
            job_of[t] = (int32_t)X->njobs;
            src[t] = -1 - (int32_t)X->njobs;
            lvl[t] = (uint16_t)(level + 1);
            hd[t] = h;
            have[t] = 1;
            X->njobs++;
            progress = 1;
        }
    }
    free(hd);
    free(src);
    free(lvl);
    free(have);
    return X->oom ? -1 : 0;
}

#define RX_MAX_LEVEL 256u

/* A group whose device recovery runs as the host peel's line jobs: above
 * RFEC_MAX_K segments (the batched peel's masks hold 128 members), or a huge
 * shape of any count (no device plan: more than RFEC_MAX_LINES lines, e.g. a
 * peer's 128-segment flex of 64 rows x 2 columns, or one rx_extend took past
 * 64 lines; its parity rows sit at a 256-line stride). */
static int rx_line_jobs(const rx_shape* sh) { return sh->count > RFEC_MAX_K || sh->huge; }

/* The device side of one call: the groups that delivered something in this
 * call, rebuilt from their arrived members and registered parities (rows of
 * `rows`, DEVICE, indexed by record), peeled by rfec_recover_batch, and the
 * delivered rows copied out.  The pinned tables go after the first `hoff`
 * bytes of t_rx.h, which survive a grow (X->R may live there). */
static int rx_device(rx_sim* X, const uint8_t* rows, uint32_t stride, uint32_t capacity, size_t hoff,
                     rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep,
                     hipStream_t sm)
{
    hipError_t e = hipSuccess;
    int rc = RFEC_OK, ke = 0;
    const double th = now_us();
    *n_out = 0;
    if (X->nout)
        qsort(X->out, X->nout, sizeof(rx_event), cmp_event);
    if (X->nout == 0) { /* nothing recovered: no device work */
        rep->host_us += now_us() - th;
        return RFEC_OK;
    }
    /* group tables, shape-major, for the groups that deliver something (work
     * proportional to the deliveries, not to the open flexes) */
    for (uint32_t s = 0; s < X->ns; ++s)
        X->S[s].n_groups = 0;
    if (++X->epoch == 0) { /* wrapped: no instance may carry a stale stamp */
        for (uint32_t gi = 0; gi < X->ng; ++gi)
            X->G[gi].gstamp = 0;
        X->epoch = 1;
    }
    X->ndl = 0;
    for (uint32_t q = 0; q < X->nout; ++q) {
        const uint32_t gi = X->out[q].inst;
        rx_inst* g = &X->G[gi];
        if (g->gstamp != X->epoch) {
            RX_GROW(X->dl, X->ndl, X->dlcap, 1, uint32_t);
            if (X->oom)
                return set_err(RFEC_ENOMEM, "rx: delivery list", 0);
            g->gstamp = X->epoch;
            g->gslot = X->S[g->shape].n_groups++;
            X->dl[X->ndl++] = gi;
        }
    }
    uint32_t nrows = 0, prows = 0, ngs = 0;
    for (uint32_t s = 0; s < X->ns; ++s) {
        rx_shape* sh = &X->S[s];
        sh->row0 = nrows;
        sh->prow0 = prows;
        sh->group0 = ngs;
        if (rx_line_jobs(sh)) /* line jobs instead (below) */
            continue;
        nrows += sh->n_groups * sh->count;
        prows += sh->n_groups * sh->n_lines;
        ngs += sh->n_groups;
    }
    /* groups above RFEC_MAX_K: the host peel's line jobs, output rows after
     * the batched peel's rows, launched level by level (jobs sorted by level) */
    X->njobs = X->njmem = 0;
    uint32_t nbig = 0, maxlvl = 0;
    for (uint32_t d = 0; d < X->ndl; ++d)
        if (rx_line_jobs(&X->S[X->G[X->dl[d]].shape]))
            nbig += X->G[X->dl[d]].count;
    int32_t* job_of = nbig ? (int32_t*)malloc((size_t)nbig * sizeof(int32_t)) : NULL;
    uint32_t* jperm = NULL;
    if (nbig && !job_of)
        return set_err(RFEC_ENOMEM, "rx: large groups", 0);
    for (uint32_t d = 0, off = 0; d < X->ndl; ++d) {
        rx_inst* g = &X->G[X->dl[d]];
        if (!rx_line_jobs(&X->S[g->shape]))
            continue;
        g->gslot = off; /* (a large group's slot: its job_of range) */
        if (rx_big_peel(X, X->dl[d], job_of + off))
            X->oom = 1;
        off += g->count;
    }
    if (X->oom) {
        free(job_of);
        return set_err(RFEC_ENOMEM, "rx: line jobs", 0);
    }
    /* a line fires at most once, so a chain is at most as deep as a group has lines (256 FEC indices) */
    uint32_t lvl_n[RX_MAX_LEVEL + 1] = {0};
    if (X->njobs) { /* stable sort by level; codes and job_of follow */
        for (uint32_t j = 0; j < X->njobs; ++j) {
            if (X->jlevel[j] > RX_MAX_LEVEL) {
                free(job_of);
                return set_err(RFEC_EINVAL, "rx: line job chain too deep", 0);
            }
            maxlvl = X->jlevel[j] > maxlvl ? X->jlevel[j] : maxlvl;
            lvl_n[X->jlevel[j]]++;
        }
        uint32_t start[RX_MAX_LEVEL + 2] = {0};
        for (uint32_t v = 1; v <= maxlvl; ++v)
            start[v + 1] = start[v] + lvl_n[v];
        jperm = (uint32_t*)malloc((size_t)X->njobs * sizeof(uint32_t));
        rfec_line_job* sorted = (rfec_line_job*)malloc((size_t)X->njobs * sizeof(rfec_line_job));
        if (!jperm || !sorted) {
            free(jperm);
            free(sorted);
            free(job_of);
            return set_err(RFEC_ENOMEM, "rx: line jobs", 0);
        }
        for (uint32_t j = 0; j < X->njobs; ++j)
            jperm[j] = start[X->jlevel[j]]++;
        for (uint32_t j = 0; j < X->njobs; ++j) {
            sorted[jperm[j]] = X->jobs[j];
            sorted[jperm[j]].out = (int32_t)jperm[j];
        }
        memcpy(X->jobs, sorted, (size_t)X->njobs * sizeof(rfec_line_job));
        free(sorted);
        for (uint32_t m = 0; m < X->njmem; ++m)
            if (X->jmem[m] < 0)
                X->jmem[m] = -1 - (int32_t)jperm[-1 - X->jmem[m]];
        for (uint32_t i = 0; i < nbig; ++i)
            if (job_of[i] >= 0)
                job_of[i] = (int32_t)jperm[job_of[i]];
    }
    const size_t o_smap = 0, o_pmap = RX_ALIGN((size_t)nrows * 4), o_hdr = RX_ALIGN(o_pmap + (size_t)prows * 4);
    const size_t o_meta = RX_ALIGN(o_hdr + (size_t)nrows * sizeof(rfec_hdr));
    const size_t o_fs = RX_ALIGN(o_meta + (size_t)prows * sizeof(rfec_hdr));
    const size_t o_pres = RX_ALIGN(o_fs + (size_t)prows * 2), o_pp = RX_ALIGN(o_pres + (size_t)ngs * 16);
    const size_t o_omap = RX_ALIGN(o_pp + (size_t)ngs * 8), o_jobs = RX_ALIGN(o_omap + (size_t)X->nout * 4);
    const size_t o_jmem = RX_ALIGN(o_jobs + (size_t)X->njobs * sizeof(rfec_line_job));
    const size_t o_in_end = RX_ALIGN(o_jmem + (size_t)X->njmem * 4);
    const size_t o_rec = o_in_end, host_bytes = RX_ALIGN(o_rec + (size_t)ngs * 16);
    size_t ws_bytes = 0;
    for (uint32_t s = 0; s < X->ns; ++s)
        if (!rx_line_jobs(&X->S[s]))
            ws_bytes += RX_ALIGN(rfec_recover_workspace_size(&X->S[s].plan, X->S[s].n_groups));
    const size_t d_shards = o_in_end, d_par = RX_ALIGN(d_shards + ((size_t)nrows + X->njobs) * stride);
    const size_t d_ws = RX_ALIGN(d_par + (size_t)prows * stride), d_rec = RX_ALIGN(d_ws + ws_bytes);
    const size_t d_out = RX_ALIGN(d_rec + (size_t)ngs * 16), dev_bytes = RX_ALIGN(d_out + (size_t)X->nout * stride);
    const int r_in_stage = (const uint8_t*)X->R == t_rx.h;
    if ((rc = rx_reserve(hoff + host_bytes, dev_bytes, hoff))) {
        free(job_of);
        free(jperm);
        return rc;
    }
    if (r_in_stage)
        X->R = (const rfec_wire_rec*)t_rx.h;
    uint8_t* H = t_rx.h + hoff;
    memset(H, 0, o_in_end);
    int32_t* smap = (int32_t*)(H + o_smap);
    int32_t* pmap = (int32_t*)(H + o_pmap);
    rfec_hdr* hh = (rfec_hdr*)(H + o_hdr);
    rfec_hdr* mh = (rfec_hdr*)(H + o_meta);
    uint16_t* fsz = (uint16_t*)(H + o_fs);
    uint64_t* pres = (uint64_t*)(H + o_pres);
    uint64_t* ppm = (uint64_t*)(H + o_pp);
    int32_t* omap = (int32_t*)(H + o_omap);
    if (X->njobs) {
        memcpy(H + o_jobs, X->jobs, (size_t)X->njobs * sizeof(rfec_line_job));
        memcpy(H + o_jmem, X->jmem, (size_t)X->njmem * 4);
    }
    for (uint32_t d = 0; d < X->ndl; ++d) {
        const rx_inst* g = &X->G[X->dl[d]];
        const rx_shape* sh = &X->S[g->shape];
        if (rx_line_jobs(sh))
            continue;
        const uint32_t gg = sh->group0 + g->gslot, r0 = sh->row0 + g->gslot * sh->count;
        const uint32_t p0 = sh->prow0 + g->gslot * sh->n_lines;
        pres[2 * gg] = g->arrived[0];
        pres[2 * gg + 1] = g->arrived[1];
        ppm[gg] = g->ppm;
        for (uint32_t i = 0; i < sh->count; ++i) {
            const int32_t src = X->slot_src[g->slot0 + i];
            smap[r0 + i] = src;
            if (src >= 0)
                hh[r0 + i] = X->slot_hdr[g->slot0 + i];
        }
        for (uint32_t l = 0; l < sh->n_lines; ++l) {
            const int32_t src = X->line_par[g->line0 + l];
            pmap[p0 + l] = src;
            if (src >= 0) {
                mh[p0 + l] = X->R[src].hdr;
                fsz[p0 + l] = X->R[src].data_size;
            }
        }
    }
    /* output rows: the recovering group's slot */
    uint32_t nok = 0;
    for (uint32_t q = 0; q < X->nout; ++q) {
        const rx_event* ev = &X->out[q];
        const rx_inst* g = &X->G[ev->inst];
        const rx_shape* sh = &X->S[g->shape];
        const uint32_t t = ev->hdr.seq - g->base;
        if (rx_line_jobs(sh)) /* the job that recovers t */
            omap[q] = t < g->count && job_of[g->gslot + t] >= 0 ? (int32_t)(nrows + (uint32_t)job_of[g->gslot + t]) : -1;
        else
            omap[q] = t < g->count ? (int32_t)(sh->row0 + g->gslot * sh->count + t) : -1;
    }
    free(job_of);
    free(jperm);
    rep->host_us += now_us() - th;
    rep->n_groups = ngs;
    for (uint32_t s = 0; s < X->ns; ++s)
        rep->n_shapes += X->S[s].n_groups != 0;
    /* the device: rows in place, one peel per shape, the delivered rows compacted */
    uint8_t* D = t_rx.d;
    double tt = now_us();
    if ((e = hipMemcpyAsync(D, H, o_in_end, hipMemcpyHostToDevice, sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: H2D", e);
    ke = rfec_launch_gather_rows(D + d_shards, rows, (const int32_t*)(D + o_smap), nrows, stride, sm);
    if (!ke)
        ke = rfec_launch_gather_rows(D + d_par, rows, (const int32_t*)(D + o_pmap), prows, stride, sm);
    for (uint32_t v = 1, lo = 0; v <= maxlvl && !ke; lo += lvl_n[v], ++v) /* the large groups' line jobs */
        ke = rfec_launch_line_jobs((const rfec_line_job*)(D + o_jobs) + lo, lvl_n[v], (const int32_t*)(D + o_jmem),
                                   rows, D + d_shards + (size_t)nrows * stride, stride, sm);
    size_t wso = 0;
    for (uint32_t s = 0; s < X->ns && !ke; ++s) {
        const rx_shape* sh = &X->S[s];
        if (!sh->n_groups || rx_line_jobs(sh))
            continue;
        rfec_kmask M;
        make_masks(&sh->plan, &M);
        ke = rfec_launch_recover(&M, sh->n_groups, stride, capacity, D + d_shards + (size_t)sh->row0 * stride,
                                 (rfec_hdr*)(D + o_hdr) + sh->row0, (const uint64_t*)(D + o_pres) + 2 * sh->group0,
                                 D + d_par + (size_t)sh->prow0 * stride, (const rfec_hdr*)(D + o_meta) + sh->prow0,
                                 (const uint16_t*)(D + o_fs) + sh->prow0, (const uint64_t*)(D + o_pp) + sh->group0,
                                 (uint64_t*)(D + d_rec) + 2 * sh->group0, D + d_ws + wso, sm, g_tuning);
        wso += RX_ALIGN(rfec_recover_workspace_size(&sh->plan, sh->n_groups));
    }
    /* delivered rows: straight into the caller's output when it is pinned and
       large enough (no second round trip; rows the peel did not cover are
       squeezed out on the host below), else into the device staging */
    uint8_t* outd = X->nout && X->nout <= max_out ? (uint8_t*)host_mapped(out_payload) : NULL;
    if (!ke && X->nout)
        ke = rfec_launch_gather_rows(outd ? outd : D + d_out, D + d_shards, (const int32_t*)(D + o_omap), X->nout,
                                     stride, sm);
    uint64_t* rec = (uint64_t*)(H + o_rec);
    if (ke || (e = hipMemcpyAsync(rec, D + d_rec, (size_t)ngs * 16, hipMemcpyDeviceToHost, sm)) != hipSuccess ||
        (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: recover", ke ? ke : (int)e);
    rep->kernel_us += now_us() - tt;
    /* the device peel covers every packet the arrival-order pass delivered (same lines, a superset of
       the members at each firing); anything else is reported, not delivered */
    for (uint32_t q = 0; q < X->nout; ++q) {
        const rx_event* ev = &X->out[q];
        const rx_inst* g = &X->G[ev->inst];
        const uint32_t t = ev->hdr.seq - g->base, gg = X->S[g->shape].group0 + g->gslot;
        const int big = rx_line_jobs(&X->S[g->shape]);
        if (big ? omap[q] < 0 : t >= g->count || !((rec[2 * gg + (t >> 6)] >> (t & 63)) & 1ull)) {
            X->unmodelled++;
            omap[q] = -1;
            continue;
        }
        nok++;
    }
    if (nok > max_out) {
        *n_out = nok;
        return set_err(RFEC_EINVAL, "rx: output too small", 0);
    }
    tt = now_us();
    uint32_t o = 0;
    if (outd) { /* the rows are in out_payload already (the sync above) */
        for (uint32_t q = 0; q < X->nout; ++q) {
            if (omap[q] < 0)
                continue;
            if (o != q)
                memmove(out_payload + (size_t)o * stride, out_payload + (size_t)q * stride, stride);
            X->out[o++] = X->out[q];
        }
    } else if (nok == X->nout) { /* the usual case: one copy */
        if (nok)
            e = hipMemcpyAsync(out_payload, D + d_out, (size_t)nok * stride, hipMemcpyDeviceToHost, sm);
        o = nok;
    }
    for (uint32_t q = 0; q < X->nout && !outd && nok != X->nout && e == hipSuccess; ++q) {
        if (omap[q] < 0)
            continue;
        e = hipMemcpyAsync(out_payload + (size_t)o * stride, D + d_out + (size_t)q * stride, stride,
                           hipMemcpyDeviceToHost, sm);
        X->out[o++] = X->out[q];
    }
    for (uint32_t q = 0; q < o; ++q) {
        out[q].hdr = X->out[q].hdr;
        out[q].fec_id = (uint16_t)X->G[X->out[q].inst].fec_id;
        out[q].reserved = 0;
    }
    if (e == hipSuccess && !outd)
        e = hipStreamSynchronize(sm);
    if (e != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: output D2H", e);
    rep->d2h_us += now_us() - tt;
    *n_out = o;
    rep->n_recovered = o;
    return RFEC_OK;
}

int rfec_rx_recover(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                    uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out,
                    uint32_t* n_out, rfec_rx_report* rep, void* stream)
{
    const double t0 = now_us();
    if (!max_ts || !n_out || !rep || (n && (!recs || !payload)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx: bad argument", 0);
    if (stride == 0 || stride % 16 || capacity > stride)
        return set_err(RFEC_EINVAL, "rx: stride must be a multiple of 16 and >= capacity", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    hipStream_t sm = (hipStream_t)stream;
    hipError_t e;
    int rc = RFEC_OK;
    /* 1. the records to the host (headers only: 64 B each) */
    const size_t rec_bytes = RX_ALIGN((size_t)n * sizeof(rfec_wire_rec));
    if ((rc = rx_reserve(rec_bytes, 0, 0)))
        return rc;
    double tt = now_us();
    if ((e = hipMemcpyAsync(t_rx.h, recs, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost, sm)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: records D2H", e);
    rep->d2h_us += now_us() - tt;
    /* 2. the control plane, in arrival order */
    const double th = now_us();
    rx_sim X;
    memset(&X, 0, sizeof(X));
    X.R = (const rfec_wire_rec*)t_rx.h;
    X.capacity = capacity;
    X.max_ts = *max_ts;
    if (rx_tables_init(&X, n)) {
        rx_sim_free(&X);
        return set_err(RFEC_ENOMEM, "rx: host tables", 0);
    }
    rx_run(&X, 0, n);
    if (X.oom) {
        rx_sim_free(&X);
        return set_err(RFEC_ENOMEM, "rx: host tables", 0);
    }
    *max_ts = X.max_ts;
    rep->n_fec_dropped = X.dropped;
    rep->host_us += now_us() - th;
    /* 3. the device: the records stay at the start of the pinned block */
    rc = rx_device(&X, payload, stride, capacity, rec_bytes, out, out_payload, max_out, n_out, rep, sm);
    rep->n_unmodelled = X.unmodelled;
    rx_sim_free(&X);
    rep->total_us = now_us() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Received datagrams (host) -> recovered segments (host)                    */
/* ------------------------------------------------------------------------ */
void* rfec_pinned_alloc(size_t bytes)
{
    void* p = NULL;
    hipError_t e;
    if (bytes == 0)
        return NULL;
    if ((e = hipHostMalloc(&p, bytes, hipHostMallocDefault)) != hipSuccess) {
        set_err(RFEC_ENOMEM, "pinned alloc", e);
        return NULL;
    }
    return p;
}

void rfec_pinned_free(void* p)
{
    if (p)
        (void)hipHostFree(p);
}

typedef struct {
    uint8_t* d;
    size_t db;
    hipStream_t sm;
} rv_ctx;
static __thread rv_ctx t_rv;

int rfec_host_recv_datagrams(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                             uint32_t stride, uint32_t capacity, uint32_t* max_ts, rfec_wire_rec* recs_out,
                             rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                             rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!max_ts || !n_out || !rep || (n && (!dgram || !dlen)))
        return set_err(RFEC_EINVAL, "recv: bad argument", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    if (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16 || stride == 0 || stride % 16 ||
        capacity > stride)
        return set_err(RFEC_EINVAL, "recv: dstride must be a multiple of 16 in [64, 2048], stride >= capacity", 0);
    hipError_t e;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    const size_t o_dl = RX_ALIGN((size_t)n * dstride), o_rec = RX_ALIGN(o_dl + (size_t)n * 2);
    const size_t o_pay = RX_ALIGN(o_rec + (size_t)n * sizeof(rfec_wire_rec));
    const size_t need = RX_ALIGN(o_pay + (size_t)n * stride);
    if (t_rv.db < need) {
        if (t_rv.d)
            (void)hipFree(t_rv.d);
        t_rv.d = NULL;
        t_rv.db = 0;
        const size_t b = need + need / 4;
        if ((e = hipMalloc((void**)&t_rv.d, b)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "recv: device staging", e);
        t_rv.db = b;
    }
    uint8_t* D = t_rv.d;
    double tt = now_us();
    if ((e = hipMemcpyAsync(D, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
        (e = hipMemcpyAsync(D + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
        (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: datagrams H2D", e);
    const double h2d = now_us() - tt;
    tt = now_us();
    int ke = rfec_launch_wire_parse(n, dstride, D, (const uint16_t*)(D + o_dl), stride, capacity,
                                    (rfec_wire_rec*)(D + o_rec), D + o_pay, max_dlen(dlen, n), t_rv.sm);
    if (ke || (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: parse", ke ? ke : (int)e);
    const double parse = now_us() - tt;
    if (recs_out) {
        tt = now_us();
        if ((e = hipMemcpyAsync(recs_out, D + o_rec, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost,
                                t_rv.sm)) != hipSuccess ||
            (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "recv: records D2H", e);
        rep->d2h_us += now_us() - tt;
    }
    const double d2h_recs = rep->d2h_us;
    const int rc = rfec_rx_recover(n, (const rfec_wire_rec*)(D + o_rec), D + o_pay, stride, capacity, max_ts, out,
                                   out_payload, max_out, n_out, rep, t_rv.sm);
    rep->h2d_us += h2d;
    rep->kernel_us += parse;
    rep->d2h_us += d2h_recs;
    rep->total_us = now_us() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Receiver session: rx_sim kept across calls, records by id in a host store, */
/* their payload rows by id in an HBM arena                                   */
/* ------------------------------------------------------------------------ */
/* a batch of the pipelined push: its parse in flight on the session's stream */
typedef struct {
    rfec_wire_rec* rec;  /* pinned, device-mapped records */
    rfec_wire_rec* recd; /* rec as the device addresses it */
    uint32_t reccap;
    uint8_t* dg; /* device copy of pageable datagram slots + lengths */
    size_t dgb;
    hipEvent_t done;
} rx_stage;

struct rfec_rx_session {
    rx_sim X;
    rfec_wire_rec* store; /* X.R */
    uint32_t nstore, storecap;
    uint8_t* arena; /* [arows][stride]: rows [0, nstore) ingested, then the pending batch's */
    uint32_t arows;
    uint32_t stride, capacity;
    /* pipelined push (rfec_rx_session_push_datagrams_async) */
    hipStream_t sa;
    rx_stage st[2];
    uint32_t pend_n; /* rows of the pending batch (arena rows [nstore, nstore + pend_n)) */
    int pend;        /* its stage, -1: none */
};

rfec_rx_session* rfec_rx_session_create(uint32_t stride, uint32_t capacity)
{
    if (stride == 0 || stride % 16 || capacity > stride) {
        set_err(RFEC_EINVAL, "rx session: stride must be a multiple of 16 and >= capacity", 0);
        return NULL;
    }
    rfec_rx_session* s = (rfec_rx_session*)calloc(1, sizeof(*s));
    if (!s || rx_tables_init(&s->X, 1024)) {
        if (s)
            rx_sim_free(&s->X);
        free(s);
        set_err(RFEC_ENOMEM, "rx session: host tables", 0);
        return NULL;
    }
    s->X.capacity = capacity;
    s->stride = stride;
    s->capacity = capacity;
    s->pend = -1;
    return s;
}

void rfec_rx_session_destroy(rfec_rx_session* s)
{
    if (!s)
        return;
    if (s->sa) /* a pending parse still writes into the arena */
        (void)hipStreamSynchronize(s->sa);
    for (int i = 0; i < 2; ++i) {
        if (s->st[i].rec)
            (void)hipHostFree(s->st[i].rec);
        if (s->st[i].dg)
            (void)hipFree(s->st[i].dg);
        if (s->st[i].done)
            (void)hipEventDestroy(s->st[i].done);
    }
    if (s->sa)
        (void)hipStreamDestroy(s->sa);
    rx_sim_free(&s->X);
    free(s->store);
    if (s->arena)
        (void)hipFree(s->arena);
    free(s);
}

/* Keeps only what the open state refers to: the flexes still registered (with
 * their slot / line tables), the records of cached segments and of those
 * flexes' members and parities (their rows gathered into a fresh arena with
 * room for `extra` more), the headers of cached recovered segments.  The rows
 * of a pending pipelined batch (parsed, not ingested) move along behind the
 * kept ones. */
static int rx_compact(rfec_rx_session* S, uint32_t extra, hipStream_t sm)
{
    const uint32_t tail = S->pend >= 0 ? S->pend_n : 0;
    hipError_t e;
    if (tail && (e = hipEventSynchronize(S->st[S->pend].done)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: pending parse", e);
    rx_sim* X = &S->X;
    int rc = RFEC_OK;
    const uint32_t ng_live = X->flex_of.n;
    rx_inst* NG = (rx_inst*)malloc(((size_t)ng_live + 1) * sizeof(rx_inst));
    uint32_t nslot = 0, nline = 0;
    for (uint32_t i = 0; i <= X->flex_of.mask; ++i)
        if (X->flex_of.v[i]) {
            const rx_inst* g = &X->G[X->flex_of.v[i] - 1];
            if (g->shape != UINT32_MAX) {
                nslot += g->count;
                nline += X->S[g->shape].n_lines;
            }
        }
    int32_t* nsrc = (int32_t*)malloc(((size_t)nslot + 1) * sizeof(int32_t));
    rfec_hdr* nhdr = (rfec_hdr*)malloc(((size_t)nslot + 1) * sizeof(rfec_hdr));
    int32_t* npar = (int32_t*)malloc(((size_t)nline + 1) * sizeof(int32_t));
    uint32_t* rmap = (uint32_t*)calloc((size_t)S->nstore + 1, sizeof(uint32_t)); /* old record -> new + 1 */
    uint32_t* hmap_ = (uint32_t*)calloc((size_t)X->nrh + 1, sizeof(uint32_t));  /* old rh -> new + 1 */
    if (!NG || !nsrc || !nhdr || !npar || !rmap || !hmap_) {
        rc = set_err(RFEC_ENOMEM, "rx session: compaction", 0);
        goto done;
    }
    /* 1. live flexes, their tables; the records they refer to */
    uint32_t ng = 0, ns = 0, nl = 0;
    for (uint32_t i = 0; i <= X->flex_of.mask; ++i) {
        if (!X->flex_of.v[i])
            continue;
        rx_inst g = X->G[X->flex_of.v[i] - 1];
        if (g.shape != UINT32_MAX) {
            const uint32_t nlines = X->S[g.shape].n_lines;
            memcpy(nsrc + ns, X->slot_src + g.slot0, g.count * sizeof(int32_t));
            memcpy(nhdr + ns, X->slot_hdr + g.slot0, g.count * sizeof(rfec_hdr));
            memcpy(npar + nl, X->line_par + g.line0, nlines * sizeof(int32_t));
            for (uint32_t q = 0; q < g.count; ++q)
                if (nsrc[ns + q] >= 0)
                    rmap[nsrc[ns + q]] = 1;
            for (uint32_t q = 0; q < nlines; ++q)
                if (npar[nl + q] >= 0)
                    rmap[npar[nl + q]] = 1;
            g.slot0 = ns;
            g.line0 = nl;
            ns += g.count;
            nl += nlines;
        }
        NG[ng] = g;
        X->flex_of.v[i] = ++ng;
    }
    /* 2. cached segments: arrived ones keep their record, recovered ones their header */
    for (uint32_t i = 0; i <= X->cache.mask; ++i) {
        const uint32_t c = X->cache.v[i];
        if (!c)
            continue;
        if (c & 0x80000000u)
            hmap_[c & 0x7FFFFFFFu] = 1;
        else
            rmap[c - 1] = 1;
    }
    /* 3. new ids, in arrival order */
    uint32_t nr = 0, nh = 0;
    for (uint32_t r = 0; r < S->nstore; ++r)
        if (rmap[r])
            rmap[r] = ++nr;
    for (uint32_t h = 0; h < X->nrh; ++h)
        if (hmap_[h])
            hmap_[h] = ++nh;
    for (uint32_t q = 0; q < ns; ++q)
        if (nsrc[q] >= 0)
            nsrc[q] = (int32_t)rmap[nsrc[q]] - 1;
    for (uint32_t q = 0; q < nl; ++q)
        if (npar[q] >= 0)
            npar[q] = (int32_t)rmap[npar[q]] - 1;
    for (uint32_t i = 0; i <= X->cache.mask; ++i) {
        const uint32_t c = X->cache.v[i];
        if (c)
            X->cache.v[i] = (c & 0x80000000u) ? (0x80000000u | (hmap_[c & 0x7FFFFFFFu] - 1)) : rmap[c - 1];
    }
    /* 4. records (host) and rows (device) */
    uint32_t* gmap = (uint32_t*)malloc(((size_t)nr + tail + 1) * sizeof(uint32_t)); /* new -> old */
    const uint32_t arows = 2 * (nr + tail + extra) > 4096 ? 2 * (nr + tail + extra) : 4096;
    uint8_t* arena = NULL;
    if (!gmap) {
        rc = set_err(RFEC_ENOMEM, "rx session: compaction", 0);
        goto done;
    }
    for (uint32_t r = 0; r < S->nstore; ++r)
        if (rmap[r]) {
            gmap[rmap[r] - 1] = r;
            S->store[rmap[r] - 1] = S->store[r]; /* rmap[r] - 1 <= r: in place, ascending */
        }
    for (uint32_t t = 0; t < tail; ++t)
        gmap[nr + t] = S->nstore + t;
    S->nstore = nr;
    X->R = S->store;
    for (uint32_t h = 0; h < X->nrh; ++h)
        if (hmap_[h])
            X->rh[hmap_[h] - 1] = X->rh[h];
    X->nrh = nh;
    if ((e = hipMalloc((void**)&arena, (size_t)arows * S->stride)) != hipSuccess) {
        free(gmap);
        rc = set_err(RFEC_ENOMEM, "rx session: arena", e);
        goto done;
    }
    if (nr + tail) {
        int32_t* dmap = NULL;
        int ke = 0;
        const uint32_t nm = nr + tail;
        if ((e = hipMalloc((void**)&dmap, (size_t)nm * sizeof(int32_t))) != hipSuccess ||
            (e = hipMemcpyAsync(dmap, gmap, (size_t)nm * sizeof(int32_t), hipMemcpyHostToDevice, sm)) != hipSuccess ||
            (ke = rfec_launch_gather_rows(arena, S->arena, dmap, nm, S->stride, sm)) != 0 ||
            (e = hipStreamSynchronize(sm)) != hipSuccess) {
            if (dmap)
                (void)hipFree(dmap);
            (void)hipFree(arena);
            free(gmap);
            rc = set_err(RFEC_EDEVICE, "rx session: row compaction", ke ? ke : (int)e);
            goto done;
        }
        (void)hipFree(dmap);
    }
    free(gmap);
    if (S->arena)
        (void)hipFree(S->arena);
    S->arena = arena;
    S->arows = arows;
    /* 5. the group tables */
    free(X->G);
    free(X->slot_src);
    free(X->slot_hdr);
    free(X->line_par);
    X->G = NG;
    X->ng = X->gcap = ng;
    X->slot_src = nsrc;
    X->slot_hdr = nhdr;
    X->nslot = X->slotcap = X->slothcap = ns;
    X->line_par = npar;
    X->nline = X->linecap = nl;
    NG = NULL;
    nsrc = npar = NULL;
    nhdr = NULL;
done:
    free(NG);
    free(nsrc);
    free(nhdr);
    free(npar);
    free(rmap);
    free(hmap_);
    return rc;
}

/* room for n more arena rows and records: drop what the open state no longer
 * refers to (and grow) */
static int rx_session_room(rfec_rx_session* S, uint32_t n, hipStream_t sm)
{
    int rc;
    const uint32_t tail = S->pend >= 0 ? S->pend_n : 0; /* a pending pipelined batch's rows */
    if (S->nstore + tail + n > S->arows && (rc = rx_compact(S, n, sm)))
        return rc;
    if (S->nstore + tail + n > S->storecap) {
        uint32_t c = S->storecap ? S->storecap : 4096;
        while (c < S->nstore + tail + n)
            c *= 2;
        rfec_wire_rec* p = (rfec_wire_rec*)realloc(S->store, (size_t)c * sizeof(rfec_wire_rec));
        if (!p)
            return set_err(RFEC_ENOMEM, "rx session: record store", 0);
        S->store = p;
        S->storecap = c;
    }
    return RFEC_OK;
}

/* records already on the host (rh[0, n)), payload rows on the device at
 * `payload`, or already in the arena's next n rows (payload NULL; the caller
 * made the room) */
static int rx_session_push_staged(rfec_rx_session* S, uint32_t n, const rfec_wire_rec* rh, const uint8_t* payload,
                                  rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                                  rfec_rx_report* rep, hipStream_t sm)
{
    rx_sim* X = &S->X;
    hipError_t e;
    int rc;
    if (payload && (rc = rx_session_room(S, n, sm)))
        return rc;
    X->R = S->store;
    memcpy(S->store + S->nstore, rh, (size_t)n * sizeof(rfec_wire_rec));
    if (payload) {
        double tt = now_us();
        if ((e = hipMemcpyAsync(S->arena + (size_t)S->nstore * S->stride, payload, (size_t)n * S->stride,
                                hipMemcpyDeviceToDevice, sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: rows", e);
        rep->kernel_us += now_us() - tt;
    }
    const uint32_t a0 = S->nstore;
    S->nstore += n;
    const double th = now_us();
    X->nout = 0;
    X->dropped = 0;
    X->unmodelled = 0;
    rx_run(X, a0, n);
    if (X->oom)
        return set_err(RFEC_ENOMEM, "rx session: host tables", 0);
    rep->n_fec_dropped = X->dropped;
    rep->host_us += now_us() - th;
    rc = rx_device(X, S->arena, S->stride, S->capacity, 0, out, out_payload, max_out, n_out, rep, sm);
    rep->n_unmodelled = X->unmodelled;
    return rc;
}

int rfec_rx_session_push(rfec_rx_session* S, uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload,
                         rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                         rfec_rx_report* rep, void* stream)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!recs || !payload)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    if (S->pend >= 0)
        return set_err(RFEC_EINVAL, "rx session: a pipelined batch is pending (flush it: async push with n = 0)", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    hipStream_t sm = (hipStream_t)stream;
    hipError_t e;
    int rc;
    if ((rc = rx_reserve(RX_ALIGN((size_t)n * sizeof(rfec_wire_rec)), 0, 0)))
        return rc;
    double tt = now_us();
    if ((e = hipMemcpyAsync(t_rx.h, recs, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost, sm)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: records D2H", e);
    rep->d2h_us += now_us() - tt;
    rc = rx_session_push_staged(S, n, (const rfec_wire_rec*)t_rx.h, payload, out, out_payload, max_out, n_out, rep,
                                sm);
    rep->total_us = now_us() - t0;
    return rc;
}

int rfec_rx_session_push_datagrams(rfec_rx_session* S, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                   const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                   uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!dgram || !dlen)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    if (S->pend >= 0)
        return set_err(RFEC_EINVAL, "rx session: a pipelined batch is pending (flush it: async push with n = 0)", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    if (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16)
        return set_err(RFEC_EINVAL, "rx session: dstride must be a multiple of 16 in [64, 2048]", 0);
    hipError_t e;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    const uint32_t stride = S->stride;
    const size_t o_dl = RX_ALIGN((size_t)n * dstride), need = RX_ALIGN(o_dl + (size_t)n * 2);
    if (t_rv.db < need) {
        if (t_rv.d)
            (void)hipFree(t_rv.d);
        t_rv.d = NULL;
        t_rv.db = 0;
        const size_t b = need + need / 4;
        if ((e = hipMalloc((void**)&t_rv.d, b)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "recv: device staging", e);
        t_rv.db = b;
    }
    uint8_t* D = t_rv.d;
    int rc;
    if ((rc = rx_reserve(RX_ALIGN((size_t)n * sizeof(rfec_wire_rec)), 0, 0)))
        return rc;
    /* the payload rows are parsed straight into the arena's next n rows */
    if ((rc = rx_session_room(S, n, t_rv.sm)))
        return rc;
    double tt = now_us();
    /* datagrams in pinned memory (the UDP batch slots) are read by the parse
     * itself; pageable ones are copied first.  The records go straight to the
     * pinned staging area. */
    const uint8_t* dg = host_mapped(dgram);
    const uint8_t* dl = host_mapped(dlen);
    if (!dg || !dl) {
        if ((e = hipMemcpyAsync(D, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
            (e = hipMemcpyAsync(D + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "recv: datagrams H2D", e);
        dg = D;
        dl = D + o_dl;
    }
    const double h2d_issue = now_us() - tt;
    int ke = rfec_launch_wire_parse(n, dstride, dg, (const uint16_t*)dl, stride, S->capacity,
                                    (rfec_wire_rec*)t_rx.hd, S->arena + (size_t)S->nstore * stride,
                                    max_dlen(dlen, n), t_rv.sm);
    if (ke || (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: parse", ke ? ke : (int)e);
    const double staged = now_us() - tt;
    if (recs_out)
        memcpy(recs_out, t_rx.h, (size_t)n * sizeof(rfec_wire_rec));
    rc = rx_session_push_staged(S, n, (const rfec_wire_rec*)t_rx.h, NULL, out, out_payload, max_out, n_out, rep,
                                t_rv.sm);
    rep->h2d_us += h2d_issue;
    rep->kernel_us += staged - h2d_issue; /* the H2D completes inside this interval too */
    rep->total_us = now_us() - t0;
    return rc;
}

/* The pipelined push: this call starts batch i (H2D if pageable, parse into
 * the arena's rows after the pending batch's, records into its stage's mapped
 * area, on the session's own stream) and then ingests batch i-1 (control
 * plane, peel on the thread's stream) while the device parses batch i. */
static int rx_stage_reserve(rx_stage* st, uint32_t n, size_t dg_bytes)
{
    hipError_t e;
    if (!st->done && (e = hipEventCreateWithFlags(&st->done, hipEventDisableTiming)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: event", e);
    if (st->reccap < n) {
        const uint32_t c = n + n / 4 + 64;
        void* h = NULL;
        void* d = NULL;
        if ((e = hipHostMalloc(&h, (size_t)c * sizeof(rfec_wire_rec), hipHostMallocMapped)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx session: record stage", e);
        if ((e = hipHostGetDevicePointer(&d, h, 0)) != hipSuccess) {
            (void)hipHostFree(h);
            return set_err(RFEC_EDEVICE, "rx session: record stage device view", e);
        }
        if (st->rec)
            (void)hipHostFree(st->rec);
        st->rec = (rfec_wire_rec*)h;
        st->recd = (rfec_wire_rec*)d;
        st->reccap = c;
    }
    if (dg_bytes > st->dgb) {
        if (st->dg)
            (void)hipFree(st->dg);
        st->dg = NULL;
        st->dgb = 0;
        const size_t b = dg_bytes + dg_bytes / 4;
        if ((e = hipMalloc((void**)&st->dg, b)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx session: datagram stage", e);
        st->dgb = b;
    }
    return RFEC_OK;
}

int rfec_rx_session_push_datagrams_async(rfec_rx_session* S, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                         const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                         uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!dgram || !dlen)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n && (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16))
        return set_err(RFEC_EINVAL, "rx session: dstride must be a multiple of 16 in [64, 2048]", 0);
    hipError_t e;
    int rc;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    if (!S->sa && (e = hipStreamCreateWithFlags(&S->sa, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: stream", e);
    const int prev = S->pend;
    const uint32_t p = prev >= 0 ? S->pend_n : 0;
    int cur = -1;
    if (n) {
        /* 1. start batch i behind the pending one's rows */
        cur = prev == 0 ? 1 : 0;
        rx_stage* st = &S->st[cur];
        const size_t o_dl = RX_ALIGN((size_t)n * dstride);
        if ((rc = rx_session_room(S, n, t_rv.sm)) || (rc = rx_stage_reserve(st, n, o_dl + (size_t)n * 2)))
            return rc;
        double tt = now_us();
        const uint8_t* dg = host_mapped(dgram);
        const uint8_t* dl = host_mapped(dlen);
        if (!dg || !dl) {
            if ((e = hipMemcpyAsync(st->dg, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, S->sa)) != hipSuccess ||
                (e = hipMemcpyAsync(st->dg + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, S->sa)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "rx session: datagrams H2D", e);
            dg = st->dg;
            dl = st->dg + o_dl;
        }
        rep->h2d_us += now_us() - tt;
        const int ke = rfec_launch_wire_parse(n, dstride, dg, (const uint16_t*)dl, S->stride, S->capacity, st->recd,
                                              S->arena + (size_t)(S->nstore + p) * S->stride, max_dlen(dlen, n),
                                              S->sa);
        if (ke || (e = hipEventRecord(st->done, S->sa)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: parse", ke ? ke : (int)e);
    }
    /* 2. ingest batch i-1 while the device parses batch i */
    if (prev >= 0) {
        rx_stage* ps = &S->st[prev];
        double tt = now_us();
        if ((e = hipEventSynchronize(ps->done)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: parse", e);
        rep->kernel_us += now_us() - tt;
        if (recs_out)
            memcpy(recs_out, ps->rec, (size_t)p * sizeof(rfec_wire_rec));
        S->pend = -1; /* its rows are the arena's next p rows now */
        rc = rx_session_push_staged(S, p, ps->rec, NULL, out, out_payload, max_out, n_out, rep, t_rv.sm);
        if (rc) {
            S->pend = cur; /* batch i stays pending behind whatever was ingested */
            S->pend_n = n;
            return rc;
        }
    }
    S->pend = cur;
    S->pend_n = n;
    rep->total_us = now_us() - t0;
    return RFEC_OK;
}

int rfec_rx_session_evict(rfec_rx_session* S, void* stream)
{
    if (!S)
        return set_err(RFEC_EINVAL, "rx session: NULL", 0);
    rx_evict(&S->X);
    if (S->X.oom)
        return set_err(RFEC_ENOMEM, "rx session: evict", 0);
    return rx_compact(S, 0, (hipStream_t)stream);
}

int rfec_rx_session_get_info(const rfec_rx_session* S, rfec_rx_session_info* info)
{
    if (!S || !info)
        return set_err(RFEC_EINVAL, "rx session: NULL", 0);
    memset(info, 0, sizeof(*info));
    info->max_ts = S->X.max_ts;
    info->open_flexes = S->X.flex_of.n;
    info->cached_segments = S->X.cache.n;
    info->records_held = S->nstore;
    info->rows_held = S->arows;
    info->pending = S->pend >= 0 ? S->pend_n : 0;
    return RFEC_OK;
}
