/*
 * rfec_oracle.c -- CPU restatement of razor's flex-FEC path (TEST
 * INFRASTRUCTURE ONLY: the checker and CPU baseline, never the product).
 *
 * Every function cites the reference file:line it restates.  Reference paths
 * are relative to the razor tree (yuanrongxi/razor @ 2025-12-05).
 * Pinned against the compiled reference by tests/golden (oracle/gen_golden.c).
 */
#include "rfec_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_SEED 0x52415A4F52464543ull /* "RAZORFEC" */
#define ORACLE_RAGGED_SALT 0x0000524147474544ull

int oracle_sim_video_size(void) { return SIM_VIDEO_SIZE; }
size_t oracle_segment_size(void) { return sizeof(sim_segment_t); }
size_t oracle_fec_size(void) { return sizeof(sim_fec_t); }

/* ---- PRNG: test/common_test.c:10-26 ------------------------------------ */
uint64_t oracle_xs_next(uint64_t* s)
{
    uint64_t x = *s;
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    *s = x;
    return x * 2685821657736338717ull;
}

uint32_t oracle_xs_rand(uint64_t* s, uint32_t t)
{
    uint32_t x = (uint32_t)oracle_xs_next(s); /* truncation as in cf_rand */
    return (uint32_t)(((uint64_t)x * ((uint64_t)t + 1)) >> 32);
}

void oracle_fill_groups(uint64_t config_id, uint32_t groups, uint32_t k, uint32_t S, uint32_t stride,
                        int ragged, uint8_t* shards, rfec_hdr* hdr)
{
    uint64_t state[2] = {0, 0};
    oracle_fill_stream(config_id, state, 0, groups, k, S, stride, ragged, shards, hdr);
}

void oracle_fill_stream(uint64_t config_id, uint64_t state[2], uint32_t g0, uint32_t groups, uint32_t k,
                        uint32_t S, uint32_t stride, int ragged, uint8_t* shards, rfec_hdr* hdr)
{
    if (state[0] == 0 && state[1] == 0) {
        state[0] = ORACLE_SEED ^ config_id;
        state[1] = ORACLE_SEED ^ config_id ^ ORACLE_RAGGED_SALT;
    }
    uint64_t st = state[0], st2 = state[1];
    for (uint32_t gl = 0; gl < groups; ++gl) {
        const uint32_t g = g0 + gl;
        for (uint32_t i = 0; i < k; ++i) {
            uint8_t* d = shards + ((size_t)gl * k + i) * stride;
            uint32_t b = 0;
            for (; b + 8 <= S; b += 8) { /* little-endian bytes of each output */
                uint64_t v = oracle_xs_next(&st);
                for (uint32_t q = 0; q < 8; ++q)
                    d[b + q] = (uint8_t)(v >> (8 * q));
            }
            if (b < S) {
                uint64_t v = oracle_xs_next(&st);
                for (uint32_t q = 0; b + q < S; ++q)
                    d[b + q] = (uint8_t)(v >> (8 * q));
            }
            memset(d + S, 0, stride - S);
            rfec_hdr* h = &hdr[(size_t)gl * k + i];
            h->seq = 1u + g * k + i; /* contiguous ids, sim_sender.c:338 */
            h->fid = 1u + g;
            h->ts = 33u * g;
            h->index = (uint16_t)i;
            h->total = (uint16_t)k;
            h->ftype = (uint8_t)(g % 60 == 0);
            h->payload_type = 0;
            h->size = (uint16_t)S;
            if (ragged) {
                uint32_t sz = 1u + oracle_xs_rand(&st2, S - 1);
                h->size = (uint16_t)sz;
                memset(d + sz, 0, stride - sz);
            }
        }
    }
    state[0] = st;
    state[1] = st2;
}

/* ---- single-line XOR core: flex_fec_xor.c:4-53 ---------------------------- */
int oracle_generate(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, int capacity)
{
    if (segs_count <= 1) /* :9-10 */
        return -1;
    sim_segment_t* s0 = segs[0];
    fec->fec_meta.seq = s0->packet_id; /* :13-20 */
    fec->fec_meta.fid = s0->fid;
    fec->fec_meta.ts = s0->timestamp;
    fec->fec_meta.payload_type = s0->payload_type;
    fec->fec_meta.ftype = s0->ftype;
    fec->fec_meta.index = s0->index;
    fec->fec_meta.total = s0->total;
    fec->fec_meta.size = s0->data_size;

    int L = 0; /* :22-26 */
    for (int i = 0; i < segs_count; ++i)
        if (L < segs[i]->data_size)
            L = segs[i]->data_size;
    fec->fec_data_size = (uint16_t)L;
    if (L > capacity) /* :27-28 */
        return -1;

    memcpy(fec->fec_data, s0->data, s0->data_size); /* :30-32 */
    memset(fec->fec_data + s0->data_size, 0, (size_t)(L - s0->data_size));
    for (int i = 1; i < segs_count; ++i) { /* :34-50 */
        sim_segment_t* s = segs[i];
        fec->fec_meta.seq ^= s->packet_id;
        fec->fec_meta.fid ^= s->fid;
        fec->fec_meta.ts ^= s->timestamp;
        fec->fec_meta.payload_type ^= s->payload_type;
        fec->fec_meta.ftype ^= s->ftype;
        fec->fec_meta.index ^= s->index;
        fec->fec_meta.total ^= s->total;
        fec->fec_meta.size ^= s->data_size;
        memset(s->data + s->data_size, 0, (size_t)(L - s->data_size)); /* in-place pad, :47 */
        for (int j = 0; j < L; ++j)
            fec->fec_data[j] ^= s->data[j];
    }
    return 0;
}

/* ---- flex_fec_xor.c:55-104 ------------------------------------------------ */
int oracle_recover(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, sim_segment_t* out)
{
    if (segs_count <= 0) /* :60-61 */
        return -1;
    out->packet_id = fec->fec_meta.seq; /* :64-71 */
    out->fid = fec->fec_meta.fid;
    out->timestamp = fec->fec_meta.ts;
    out->payload_type = fec->fec_meta.payload_type;
    out->ftype = fec->fec_meta.ftype;
    out->index = fec->fec_meta.index;
    out->total = fec->fec_meta.total;
    out->data_size = fec->fec_meta.size;
    int L = fec->fec_data_size;
    memcpy(out->data, fec->fec_data, (size_t)L); /* :73 */
    for (int i = 0; i < segs_count; ++i) { /* :75-95 */
        sim_segment_t* s = segs[i];
        out->packet_id ^= s->packet_id;
        out->fid ^= s->fid;
        out->timestamp ^= s->timestamp;
        out->payload_type ^= s->payload_type;
        out->ftype ^= s->ftype;
        out->index ^= s->index;
        out->total ^= s->total;
        out->data_size ^= s->data_size;
        if (L < s->data_size) /* :88-89 */
            return -1;
        memset(s->data + s->data_size, 0, (size_t)(L - s->data_size));
        for (int j = 0; j < L; ++j)
            out->data[j] ^= s->data[j];
    }
    if (out->data_size > L) /* :98-99 */
        return -1;
    out->fec_id = fec->fec_id; /* :101 */
    return 0;
}

/* ---- planner: flex_fec_sender.c:81-135 ------------------------------------ */
int oracle_num_packets(int n, int pf, int* row, int* col)
{
    int ret = 0;
    if (n == 0) { /* :88-92 */
        *row = *col = 0;
        return 0;
    }
    if (pf >= 10 && n >= 6) { /* :94-111 matrix mode */
        double f = sqrt((double)n);
        int colum = (int)f;
        if (colum + 0.1f < f) /* float/double mix kept as written */
            colum = 1 + (int)f;
        if (colum < 3) colum = 3;
        if (colum > 20) colum = 20;
        int r = n / colum + ((n % colum) != 0);
        int c = n / r + ((n % r) != 0);
        *row = (uint8_t)r; /* stored into uint8_t fields */
        *col = (uint8_t)c;
        ret = 1;
    } else { /* :112-132 strip mode */
        int colum = (n * pf + (1 << 7)) >> 8;
        int r = 1, c;
        if (pf > 0) {
            if (colum == 0) {
                c = n;
            } else {
                c = n / colum + ((n % colum) > 0);
                r = n / c + ((n % c) != 0);
            }
        } else {
            r = 0;
            c = 0;
        }
        *row = (uint8_t)r;
        *col = (uint8_t)c;
    }
    return ret;
}

/* ---- line layout: flex_fec_sender.c:158-233 -------------------------------- */
static void plan_push(rfec_plan* p, int first, int stride, int count, int index)
{
    if (count < 2) /* flex_fec_generate fails for <2 members (xor.c:9-10): no parity */
        return;
    rfec_line* l = &p->line[p->n_lines++];
    l->first = (uint8_t)first;
    l->stride = (uint8_t)stride;
    l->count = (uint8_t)count;
    l->index = (uint8_t)index;
}

static int plan_lines(rfec_plan* p, int k, int row, int col, int rc, unsigned layers)
{
    memset(p, 0, sizeof(*p));
    p->k = (uint16_t)k;
    p->row = (uint8_t)row;
    p->col = (uint8_t)col;
    p->rc = (uint8_t)rc;
    if (k < 1 || k > RFEC_MAX_K)
        return -1;
    if (col <= 1) /* :158 */
        return 0;
    if (layers & RFEC_LAYER_ROWS) {
        for (int r = 0; r < row; ++r) { /* :166-188 */
            int first = r * col;
            int count = col;
            if (count > k - first)
                count = k - first;
            if (count >= 1)
                plan_push(p, first, 1, count, r);
        }
    }
    p->n_row_lines = p->n_lines;
    if ((layers & RFEC_LAYER_COLS) && row > 1 && rc == 1) { /* :199-233 */
        for (int c = 0; c < col; ++c) {
            int count = 0;
            for (int r = 0; r < row; ++r) {
                if (r * col + c < k)
                    count++;
                else
                    break;
            }
            if (count >= 1)
                plan_push(p, c, col, count, 0x80 | c);
        }
    }
    return 0;
}

int oracle_plan_from_fraction(int k, int pf, unsigned layers, rfec_plan* plan)
{
    int row, col;
    int rc = oracle_num_packets(k, pf, &row, &col);
    return plan_lines(plan, k, row, col, rc, layers);
}

int oracle_plan_matrix(int k, int row, int col, unsigned layers, rfec_plan* plan)
{
    return plan_lines(plan, k, row, col, 1, layers);
}

/* ---- batched restatement over the device layout ---------------------------- */
static void hdr_xor(rfec_hdr* a, const rfec_hdr* b)
{
    a->seq ^= b->seq;
    a->fid ^= b->fid;
    a->ts ^= b->ts;
    a->index ^= b->index;
    a->total ^= b->total;
    a->ftype ^= b->ftype;
    a->payload_type ^= b->payload_type;
    a->size ^= b->size;
}

void oracle_encode_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                         const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                         uint16_t* fec_size, int8_t* status)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    for (uint32_t g = 0; g < groups; ++g) {
        for (uint32_t l = 0; l < n; ++l) {
            const rfec_line* ln = &plan->line[l];
            size_t o = (size_t)g * n + l;
            uint8_t* out = parity + o * stride;
            rfec_hdr m;
            memset(&m, 0, sizeof(m));
            uint32_t L = 0;
            memset(out, 0, stride);
            for (uint32_t q = 0; q < ln->count; ++q) {
                uint32_t i = ln->first + q * ln->stride;
                const rfec_hdr* h = &hdr[(size_t)g * k + i];
                hdr_xor(&m, h);
                if (h->size > L)
                    L = h->size;
                const uint8_t* s = shards + ((size_t)g * k + i) * stride;
                for (uint32_t j = 0; j < stride; ++j)
                    out[j] ^= s[j];
            }
            meta[o] = m;
            fec_size[o] = (uint16_t)L;
            status[o] = (int8_t)((ln->count <= 1 || L > capacity) ? -1 : 0);
        }
    }
}

#define BIT_GET(m, i) (((m)[(i) >> 6] >> ((i)&63)) & 1ull)
#define BIT_CLR(m, i) ((m)[(i) >> 6] &= ~(1ull << ((i)&63)))
#define BIT_SET(m, i) ((m)[(i) >> 6] |= (1ull << ((i)&63)))

/*
 * Peeling decoder: the fixpoint reached by flex_recover_row / flex_recover_col
 * (flex_fec_receiver.c:105-206) as segments, parities and recovered segments
 * (sim_receiver.c:780-804) keep arriving.  Canonical order: lines in plan
 * order (rows, then columns), repeated until nothing changes.  A line fires
 * when its parity is present, exactly one member is missing and at least one
 * is present (:133-140, :189-196), and flex_fec_recover would succeed
 * (member sizes <= fec_data_size, recovered size <= fec_data_size;
 * flex_fec_xor.c:88-89, 98-99).
 */
void oracle_recover_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                          uint8_t* shards, rfec_hdr* hdr, const uint64_t* present,
                          const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                          const uint64_t* parity_present, uint64_t* recovered)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    for (uint32_t g = 0; g < groups; ++g) {
        uint64_t have[2] = {present[2 * g], present[2 * g + 1]};
        uint64_t rec[2] = {0, 0};
        uint64_t pp = parity_present[g];
        int progress = 1;
        while (progress) {
            progress = 0;
            for (uint32_t l = 0; l < n; ++l) {
                if (!((pp >> l) & 1))
                    continue;
                const rfec_line* ln = &plan->line[l];
                int miss = 0, got = 0;
                uint32_t t = 0;
                for (uint32_t q = 0; q < ln->count; ++q) {
                    uint32_t i = ln->first + q * ln->stride;
                    if (BIT_GET(have, i))
                        got++;
                    else {
                        miss++;
                        t = i;
                    }
                }
                if (miss != 1 || got == 0)
                    continue;
                size_t o = (size_t)g * n + l;
                uint32_t L = fec_size[o];
                if (L > capacity)
                    continue;
                rfec_hdr r = meta[o];
                int ok = 1;
                for (uint32_t q = 0; q < ln->count; ++q) {
                    uint32_t i = ln->first + q * ln->stride;
                    if (i == t)
                        continue;
                    const rfec_hdr* h = &hdr[(size_t)g * k + i];
                    hdr_xor(&r, h);
                    if (h->size > L)
                        ok = 0;
                }
                if (!ok || r.size > L)
                    continue;
                uint8_t* dst = shards + ((size_t)g * k + t) * stride;
                memcpy(dst, parity + o * stride, stride);
                for (uint32_t q = 0; q < ln->count; ++q) {
                    uint32_t i = ln->first + q * ln->stride;
                    if (i == t)
                        continue;
                    const uint8_t* s = shards + ((size_t)g * k + i) * stride;
                    for (uint32_t j = 0; j < stride; ++j)
                        dst[j] ^= s[j];
                }
                hdr[(size_t)g * k + t] = r;
                BIT_SET(have, t);
                BIT_SET(rec, t);
                progress = 1;
            }
        }
        recovered[2 * g] = rec[0];
        recovered[2 * g + 1] = rec[1];
    }
}

/* ---- reference-shaped AoS path (CPU baseline) ------------------------------ */
static void encode_aos_range(const rfec_plan* plan, uint32_t g0, uint32_t g1, sim_segment_t* segs,
                             sim_fec_t* fecs, long* produced)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    sim_segment_t* ptrs[RFEC_MAX_K];
    long cnt = 0;
    for (uint32_t g = g0; g < g1; ++g) {
        sim_segment_t* base = segs + (size_t)g * k;
        for (uint32_t l = 0; l < n; ++l) {
            const rfec_line* ln = &plan->line[l];
            for (uint32_t q = 0; q < ln->count; ++q)
                ptrs[q] = &base[ln->first + q * ln->stride];
            sim_fec_t* out = &fecs[(size_t)g * n + l];
            if (oracle_generate(ptrs, ln->count, out, SIM_VIDEO_SIZE) == 0) {
                /* stamps of flex_fec_sender.c:176-181 / 220-225 */
                out->fec_id = (uint16_t)(g + 1);
                out->base_id = base[0].packet_id;
                out->col = plan->col;
                out->row = plan->row;
                out->index = ln->index;
                out->count = plan->k;
                cnt++;
            }
        }
    }
    *produced = cnt;
}

long oracle_encode_aos(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs)
{
    long c = 0;
    encode_aos_range(plan, 0, groups, segs, fecs, &c);
    return c;
}

typedef struct {
    const rfec_plan* plan;
    uint32_t g0, g1;
    sim_segment_t* segs;
    sim_fec_t* fecs;
    long produced;
} enc_job;

static void* enc_worker(void* p)
{
    enc_job* j = (enc_job*)p;
    encode_aos_range(j->plan, j->g0, j->g1, j->segs, j->fecs, &j->produced);
    return NULL;
}

long oracle_encode_aos_mt(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                          int threads)
{
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    pthread_t tid[256];
    enc_job jobs[256];
    for (int t = 0; t < threads; ++t) {
        jobs[t].plan = plan;
        jobs[t].g0 = (uint32_t)((uint64_t)groups * t / threads);
        jobs[t].g1 = (uint32_t)((uint64_t)groups * (t + 1) / threads);
        jobs[t].segs = segs;
        jobs[t].fecs = fecs;
        jobs[t].produced = 0;
        pthread_create(&tid[t], NULL, enc_worker, &jobs[t]);
    }
    long total = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(tid[t], NULL);
        total += jobs[t].produced;
    }
    return total;
}

long oracle_recover_aos(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                        const uint64_t* present, sim_segment_t* out)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    sim_segment_t* ptrs[RFEC_MAX_K];
    long total = 0;
    for (uint32_t g = 0; g < groups; ++g) {
        sim_segment_t* base = segs + (size_t)g * k;
        sim_segment_t* obase = out + (size_t)g * k;
        uint64_t have[2] = {present[2 * g], present[2 * g + 1]};
        int progress = 1;
        while (progress) {
            progress = 0;
            for (uint32_t l = 0; l < n; ++l) {
                const rfec_line* ln = &plan->line[l];
                int miss = 0, cnt = 0;
                uint32_t t = 0;
                for (uint32_t q = 0; q < ln->count; ++q) {
                    uint32_t i = ln->first + q * ln->stride;
                    if (BIT_GET(have, i))
                        ptrs[cnt++] = BIT_GET(present + 2 * g, i) ? &base[i] : &obase[i];
                    else {
                        miss++;
                        t = i;
                    }
                }
                if (miss != 1 || cnt == 0)
                    continue;
                if (oracle_recover(ptrs, cnt, &fecs[(size_t)g * n + l], &obase[t]) == 0) {
                    BIT_SET(have, t);
                    total++;
                    progress = 1;
                }
            }
        }
    }
    return total;
}
