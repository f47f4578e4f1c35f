/*
 * rfec_host.c -- C host layer of the MI355X flex-FEC engine (C99 + the HIP
 * runtime C API): errors and tuning, the planner, the batched device and wire
 * API, and the utilities the other host translation units share
 * (rfec_host_internal.h).
 *
 *  1. The planner: restates flex_fec_sender_num_packets and the row / column
 *     line layout of flex_fec_sender_update
 *     (sim_transport/fec/flex_fec_sender.c:81-135, :158-233).
 *  2. The batched device API (rfec_encode_batch / rfec_recover_batch, the
 *     wire codec): argument checks, then the launches through the shims in
 *     rfec_kernels.hip / rfec_wire.hip.
 *
 * The rest of the host layer, by concern: rfec_dropin.c (the drop-in
 * flex_fec_generate / flex_fec_recover and the resident service),
 * rfec_hostmem.c (host-memory batches), rfec_sender.c (sender staging),
 * rfec_rx.c (receiver ingestion and sessions).
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
/* errors                                                                    */
/* ------------------------------------------------------------------------ */
static __thread char t_err[256];

int set_err(int code, const char* what, int hip_code)
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

uint32_t rfec_abi_version(void) { return RFEC_ABI_VERSION; }
_Static_assert(sizeof(rfec_host_timing) == 56, "rfec_host_timing: ABI 5 layout (bump RFEC_ABI_VERSION)");
_Static_assert(sizeof(rfec_send_report) == 72, "rfec_send_report: ABI 7 layout (bump RFEC_ABI_VERSION)");

unsigned g_tuning = 0;
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
int check_plan(const rfec_plan* p, uint32_t max_k)
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

int check_geometry(uint32_t groups, uint32_t stride, uint32_t capacity, uint32_t rows_per_group)
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

void make_masks(const rfec_plan* p, rfec_kmask* M)
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

/* the row width of a plan the packed records cover (rows of col <= 4 consecutive segments, no columns,
 * k <= 64), else 0 */
static uint32_t packed_col(const rfec_plan* p)
{
    if (!p || p->k == 0 || p->k > 64 || p->n_lines == 0)
        return 0;
    const uint32_t col = p->line[0].count;
    if (col < 2 || col > 4 || p->n_lines != (p->k + col - 1) / col)
        return 0;
    for (uint32_t l = 0; l < p->n_lines; ++l) {
        const uint32_t first = l * col, count = p->k - first < col ? p->k - first : col;
        if (p->line[l].first != first || p->line[l].stride != 1 || p->line[l].count != count)
            return 0;
    }
    return col;
}

size_t rfec_packed_stride(const rfec_plan* plan, uint32_t per_group)
{
    const uint32_t col = packed_col(plan);
    if (!col || per_group == 0 || per_group > plan->k)
        return 0;
    return ((16u + per_group * (24u + 20u * (col - 1u))) + 63u) & ~(size_t)63u;
}

/* the checks both packed entry points share; sets *col and *pk_stride */
static int packed_check(const rfec_plan* plan, uint32_t groups, uint32_t per_group, const void* packed,
                        uint32_t* col, size_t* pk_stride)
{
    int rc = check_plan(plan, RFEC_MAX_K);
    if (rc)
        return rc;
    *col = packed_col(plan);
    if (!*col)
        return set_err(RFEC_EINVAL, "packed records need a row layout (rows of <= 4 segments, k <= 64)", 0);
    if (per_group == 0 || per_group > plan->k)
        return set_err(RFEC_EINVAL, "per_group must be in [1, k]", 0);
    *pk_stride = rfec_packed_stride(plan, per_group);
    unsigned lg = 0;
    while ((1u << lg) < per_group)
        ++lg;
    if (((uint64_t)groups << lg) >= (1ull << 32) || (uint64_t)groups * *pk_stride >= (1ull << 40))
        return set_err(RFEC_EINVAL, "batch too large for one launch (groups x slots)", 0);
    if (groups && (!packed || (uintptr_t)packed % 16))
        return set_err(RFEC_EINVAL, "packed records: NULL or not 16-byte aligned", 0);
    return RFEC_OK;
}

int rfec_pack_erasures(const rfec_plan* plan, uint32_t groups, const rfec_hdr* hdr, const uint64_t* present,
                       const rfec_hdr* meta, const uint16_t* fec_size, const uint64_t* parity_present,
                       uint32_t per_group, uint8_t* packed, void* stream)
{
    uint32_t col;
    size_t pks;
    int rc = packed_check(plan, groups, per_group, packed, &col, &pks);
    if (rc)
        return rc;
    if (groups == 0)
        return RFEC_OK;
    if (!hdr || !present || !meta || !fec_size || !parity_present)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    const int e = rfec_launch_pack_rows(plan, col, groups, hdr, present, meta, fec_size, parity_present, per_group,
                                        packed, (uint32_t)pks, 24u + 20u * (col - 1u), stream);
    return e ? set_err(RFEC_EDEVICE, "pack launch", e) : RFEC_OK;
}

int rfec_recover_packed_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                            const uint8_t* shards, const uint8_t* parity, const uint8_t* packed,
                            uint64_t* recovered, uint32_t per_group, uint8_t* out_shards, rfec_hdr* out_hdr,
                            uint8_t* out_index, void* stream)
{
    uint32_t col;
    size_t pks;
    int rc = packed_check(plan, groups, per_group, packed, &col, &pks);
    if (rc)
        return rc;
    if ((rc = check_geometry(groups, stride, capacity, plan->k)))
        return rc;
    const uint32_t cd = capacity ? (capacity + 15) / 16 : 1;
    if ((uint64_t)groups * per_group * cd >= (1ull << 32) || (uint64_t)65 * plan->k * stride >= 0x7FFFFFF0ull)
        return set_err(RFEC_EINVAL, "batch too large for one launch (groups x slots x chunks)", 0);
    if (groups == 0)
        return RFEC_OK;
    if (!shards || !parity || !recovered || !out_shards || !out_hdr || !out_index)
        return set_err(RFEC_EINVAL, "NULL buffer", 0);
    static __thread rfec_kmask M;
    make_masks(plan, &M);
    const rfec_dense_out D = {out_shards, out_hdr, out_index, per_group};
    const int e = rfec_launch_recover_packed(&M, col, groups, stride, capacity, shards, parity, packed, (uint32_t)pks,
                                             24u + 20u * (col - 1u), recovered, &D, stream);
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
                                             dlen, count, stream);
    return e ? set_err(RFEC_EDEVICE, "wire_frame_seg launch", e) : RFEC_OK;
}

/* the longest of n host-side datagram lengths (0 for none) */
uint32_t max_dlen(const uint16_t* dlen, uint32_t n)
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
/* shared host utilities                                                     */
/* ------------------------------------------------------------------------ */
double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

/* ---- a tiny fork/join helper for the host-side gather / scatter ---------- */
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

int host_threads(void)
{
    const char* v = getenv("RFEC_HOST_THREADS");
    int t = v ? atoi(v) : 8;
    return t < 1 ? 1 : (t > 64 ? 64 : t);
}

void parallel_for(size_t n, int threads, pf_fn fn, void* arg)
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
