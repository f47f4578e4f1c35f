/*
 * rfec_sender.c -- sender staging: sim_sender_put (sim_sender.c:254-377) and
 * the flex sender's grouping (flex_fec_sender.c:49-245) over frames in host
 * memory, then encode and framing on the device (frames -> datagrams).
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
#define SD_CHUNKS 16 /* slot chunks of one call at most */
typedef struct {
    uint8_t* h;     /* pinned host */
    uint8_t* hd;    /* h as the device addresses it (NULL: not mapped) */
    uint8_t* d;     /* device */
    size_t bytes;
    uint8_t* carry; /* the open group's segments (slots then headers), host */
    uint32_t n_carry;
    hipStream_t sg;                  /* the slots' arrival (chunks), beside the framing's stream */
    hipEvent_t evc[SD_CHUNKS + 1];   /* chunk c arrived; [SD_CHUNKS]: the tables copied */
    int have_ev;
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
    void* hd = NULL;
    t_sd.hd = hipHostGetDevicePointer(&hd, t_sd.h, 0) == hipSuccess ? (uint8_t*)hd : NULL;
    (void)hipGetLastError();
    if ((e = hipMalloc((void**)&t_sd.d, bytes)) != hipSuccess)
        return set_err(RFEC_ENOMEM, "send staging (device)", e);
    t_sd.bytes = bytes;
    return RFEC_OK;
}

typedef struct { /* byte offsets in the staging block (host and device alike) */
    size_t slots, hdr, sstamp, sorder, fstamp, forder, src, ssz, in_end;
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
    SD_TAKE(src, (size_t)n_slots * sizeof(uint64_t)); /* zero copy: each slot's bytes (device address), size */
    SD_TAKE(ssz, (size_t)n_slots * sizeof(uint16_t));
    L.in_end = o; /* everything above goes host -> device in one copy (zero copy: from hdr on) */
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
    int zc;                     /* zero copy: the device reads the frames (din: their device offset) */
    intptr_t din;
    const uint8_t* hd;          /* the staging block as the device addresses it */
} sd_stage_job;

static void sd_stage(void* arg, size_t lo, size_t hi)
{
    const sd_stage_job* J = (const sd_stage_job*)arg;
    rfec_hdr* hh = (rfec_hdr*)(J->h + J->L.hdr);
    rfec_seg_stamp* ss = (rfec_seg_stamp*)(J->h + J->L.sstamp);
    uint32_t* so = (uint32_t*)(J->h + J->L.sorder);
    uint64_t* src = (uint64_t*)(J->h + J->L.src);
    uint16_t* ssz = (uint16_t*)(J->h + J->L.ssz);
    for (size_t s = lo; s < hi; ++s) {
        uint8_t* slot = J->h + J->L.slots + s * DI_STRIDE;
        const uint32_t i = J->seg_of_slot[s];
        if (i >= J->n_segs) { /* carried from the previous call: bytes and header already in place */
            so[s] = J->n_segs + (UINT32_MAX - i); /* framed into scratch rows past the real ones */
            memset(&ss[s], 0, sizeof(ss[s]));
            src[s] = J->zc ? (uint64_t)(uintptr_t)(J->hd + J->L.slots + s * DI_STRIDE) : 0u;
            ssz[s] = DI_STRIDE;
            continue;
        }
        const rfec_seg_plan* g = &J->segs[i];
        if (J->zc) { /* the device gathers the bytes from the frame itself */
            src[s] = (uint64_t)((uintptr_t)(J->frames[g->frame].data + g->offset) + J->din);
            ssz[s] = g->data_size;
        } else {
            memcpy(slot, J->frames[g->frame].data + g->offset, g->data_size);
            memset(slot + g->data_size, 0, DI_STRIDE - g->data_size);
        }
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
    /* Zero copy: frames inside one rfec_pinned_alloc block -> the device reads their bytes itself (no host
       copy into the staging slots, no bulk H2D); datagram outputs inside such blocks -> the framing writes
       them there (no D2H).  Either side independently; RFEC_HOST_ZEROCOPY=0 turns both off. */
    intptr_t din = 0, dsg = 0, dsl = 0, dfg = 0, dfl = 0;
    int zc_in = 0, zc_out = 0;
    if (zerocopy_on()) {
        uintptr_t lo = UINTPTR_MAX, hi = 0;
        for (uint32_t f = 0; f < n_frames; ++f)
            if (frames[f].size) {
                const uintptr_t a = (uintptr_t)frames[f].data;
                lo = a < lo ? a : lo;
                hi = a + frames[f].size > hi ? a + frames[f].size : hi;
            }
        zc_in = t_sd.hd && lo < hi && pinned_range(lo, hi, &din);
        zc_out = pinned_range((uintptr_t)seg_dgram, (uintptr_t)seg_dgram + (size_t)ns * dstride, &dsg) &&
                 pinned_range((uintptr_t)seg_dlen, (uintptr_t)(seg_dlen + ns), &dsl) &&
                 (!n_par || (pinned_range((uintptr_t)fec_dgram, (uintptr_t)fec_dgram + (size_t)n_par * dstride, &dfg) &&
                             pinned_range((uintptr_t)fec_dlen, (uintptr_t)(fec_dlen + n_par), &dfl)));
    }
    rep->zero_copy = (uint32_t)(zc_in | zc_out << 1);
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
    sd_stage_job J = {frames, segs, seg_of_slot, t_sd.h, L, uid, ns, tseq, zc_in, din, t_sd.hd};
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
            if (zc_in && i < ns) { /* (the staging slot holds no bytes: from the frame) */
                const rfec_seg_plan* g = &segs[i];
                memcpy(tmp + (size_t)j * DI_STRIDE, frames[g->frame].data + g->offset, g->data_size);
                memset(tmp + (size_t)j * DI_STRIDE + g->data_size, 0, DI_STRIDE - g->data_size);
            } else {
                memcpy(tmp + (size_t)j * DI_STRIDE, t_sd.h + L.slots + (size_t)s * DI_STRIDE, DI_STRIDE);
            }
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
        /* The slots arrive in chunks on a second stream (the device's reads of the frames, or the slots'
           H2D) while the SIM_SEG framing of the chunks before writes on this one: the link carries reads
           and writes together.  The encode and the SIM_FEC framing follow the last chunk. */
        uint32_t K = zc_in && n_slots >= 8192 ? n_slots / 2048 : 1; /* (staged: one H2D measured faster) */
        {
            const char* v = getenv("RFEC_SEND_CHUNKS");
            K = v ? (uint32_t)atoi(v) : K;
            K = K < 1 ? 1 : K > SD_CHUNKS ? SD_CHUNKS : K;
        }
        if (!t_sd.sg && (e = hipStreamCreateWithFlags(&t_sd.sg, hipStreamNonBlocking)) != hipSuccess) {
            rc = set_err(RFEC_EDEVICE, "send stream", e);
            goto out;
        }
        for (uint32_t c = 0; c <= SD_CHUNKS && !t_sd.have_ev; ++c)
            if ((e = hipEventCreate(&t_sd.evc[c])) != hipSuccess) {
                rc = set_err(RFEC_EDEVICE, "send event", e);
                goto out;
            }
        t_sd.have_ev = 1;
        (void)hipEventRecord(ev[0], sm);
        e = hipMemcpyAsync(D + L.hdr, t_sd.h + L.hdr, L.in_end - L.hdr, hipMemcpyHostToDevice, sm); /* tables */
        (void)hipEventRecord(t_sd.evc[SD_CHUNKS], sm);
        (void)hipEventRecord(ev[1], sm);
        if (e == hipSuccess)
            e = hipStreamWaitEvent(t_sd.sg, t_sd.evc[SD_CHUNKS], 0);
        for (uint32_t c = 0; c < K && e == hipSuccess && !rc; ++c) {
            const uint32_t s0 = (uint32_t)((uint64_t)n_slots * c / K), s1 = (uint32_t)((uint64_t)n_slots * (c + 1) / K);
            if (zc_in) {
                const int ke = rfec_launch_send_gather((const uint64_t*)(D + L.src) + s0, (const uint16_t*)(D + L.ssz) + s0,
                                                       s1 - s0, DI_STRIDE, D + L.slots + (size_t)s0 * DI_STRIDE, t_sd.sg);
                if (ke)
                    rc = set_err(RFEC_EDEVICE, "send gather launch", ke);
            } else {
                e = hipMemcpyAsync(D + L.slots + (size_t)s0 * DI_STRIDE, t_sd.h + L.slots + (size_t)s0 * DI_STRIDE,
                                   (size_t)(s1 - s0) * DI_STRIDE, hipMemcpyHostToDevice, t_sd.sg);
            }
            if (e == hipSuccess)
                e = hipEventRecord(t_sd.evc[c], t_sd.sg);
            if (e == hipSuccess)
                e = hipStreamWaitEvent(sm, t_sd.evc[c], 0);
            int ke = 0;
            if (e == hipSuccess && !rc && s1 > s0) /* (zero copy: the carried rows, past ns, dropped) */
                ke = rfec_launch_wire_frame_seg(s1 - s0, DI_STRIDE, SIM_VIDEO_SIZE, D + L.slots + (size_t)s0 * DI_STRIDE,
                                                (const rfec_hdr*)(D + L.hdr) + s0,
                                                (const rfec_seg_stamp*)(D + L.sstamp) + s0,
                                                (const uint32_t*)(D + L.sorder) + s0, dstride,
                                                zc_out ? (uint8_t*)((uintptr_t)seg_dgram + dsg) : D + L.sdg,
                                                zc_out ? (uint16_t*)((uintptr_t)seg_dlen + dsl) : (uint16_t*)(D + L.sdl),
                                                zc_out ? ns : n_slots, sm);
            if (ke)
                rc = set_err(RFEC_EDEVICE, "frame launch", ke);
        }
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
        if (!rc && e == hipSuccess && n_par)
            ke = rfec_launch_wire_frame_fec(n_par, DI_STRIDE, SIM_VIDEO_SIZE, D + L.parity,
                                            (const rfec_hdr*)(D + L.meta), (const uint16_t*)(D + L.fsize),
                                            (const int8_t*)(D + L.status), (const rfec_fec_stamp*)(D + L.fstamp),
                                            (const uint32_t*)(D + L.forder), dstride,
                                            zc_out ? (uint8_t*)((uintptr_t)fec_dgram + dfg) : D + L.fdg,
                                            zc_out ? (uint16_t*)((uintptr_t)fec_dlen + dfl) : (uint16_t*)(D + L.fdl),
                                            sm);
        if (ke && !rc)
            rc = set_err(RFEC_EDEVICE, "frame launch", ke);
        (void)hipEventRecord(ev[2], sm);
        if (!rc && e == hipSuccess && !zc_out) {
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
        float a = 0, b = 0, d = 0; /* h2d: the tables and the slots' arrival (overlapped with the SIM_SEG
                                       framing, in kernel_us too) */
        (void)hipEventElapsedTime(&a, ev[0], t_sd.evc[K - 1]);
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
