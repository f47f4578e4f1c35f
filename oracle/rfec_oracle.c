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
    if (k < 1 || k > RFEC_MAX_K_ENCODE)
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
/* rank of erased segment t among the group's erased segments (index order) */
static uint32_t erased_rank(const uint64_t pres[2], uint32_t t)
{
    uint32_t r = 0;
    for (uint32_t i = 0; i < t; ++i)
        r += !BIT_GET(pres, i);
    return r;
}

/* The canonical peel (flex_fec_receiver.c:105-206 to a fixpoint, lines in plan
 * order; flex_fec_xor.c:55-104 per line) in place.  max_rank > 0: only erased
 * segments of rank < max_rank may be recovered (the dense output's slots). */
static void recover_batch_ranked(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                                 uint8_t* shards, rfec_hdr* hdr, const uint64_t* present,
                                 const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                                 const uint64_t* parity_present, uint64_t* recovered, uint32_t max_rank)
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
                if (max_rank && erased_rank(&present[2 * g], t) >= max_rank)
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

void oracle_recover_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                          uint8_t* shards, rfec_hdr* hdr, const uint64_t* present,
                          const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                          const uint64_t* parity_present, uint64_t* recovered)
{
    recover_batch_ranked(plan, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                         parity_present, recovered, 0);
}

void oracle_recover_batch_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                              const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                              const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                              const uint64_t* parity_present, uint64_t* recovered, uint32_t per_group,
                              uint8_t* out_shards, rfec_hdr* out_hdr, uint8_t* out_index)
{
    const uint32_t k = plan->k;
    uint8_t* sh = malloc((size_t)k * stride);
    rfec_hdr* hd = malloc(sizeof(rfec_hdr) * k);
    for (uint32_t g = 0; g < groups; ++g) {
        memcpy(sh, shards + (size_t)g * k * stride, (size_t)k * stride);
        memcpy(hd, hdr + (size_t)g * k, sizeof(rfec_hdr) * k);
        /* one group at a time over copies: the plan's per-group arrays offset by g */
        recover_batch_ranked(plan, 1, stride, capacity, sh, hd, present + 2 * g, parity + (size_t)g * plan->n_lines * stride,
                             meta + (size_t)g * plan->n_lines, fec_size + (size_t)g * plan->n_lines,
                             parity_present + g, recovered + 2 * g, per_group);
        uint32_t e = 0;
        for (uint32_t i = 0; i < k && e < per_group; ++i) {
            if (BIT_GET(&present[2 * g], i))
                continue;
            const size_t o = (size_t)g * per_group + e;
            if (BIT_GET(&recovered[2 * g], i)) {
                memcpy(out_shards + o * stride, sh + (size_t)i * stride, stride);
                out_hdr[o] = hd[i];
                out_index[o] = (uint8_t)i;
            } else {
                out_index[o] = 0xFF;
            }
            ++e;
        }
        for (; e < per_group; ++e)
            out_index[(size_t)g * per_group + e] = 0xFF;
    }
    free(sh);
    free(hd);
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

static long recover_aos_range(const rfec_plan* plan, uint32_t g0, uint32_t g1, sim_segment_t* segs,
                              sim_fec_t* fecs, const uint64_t* present, sim_segment_t* out)
{
    const uint32_t k = plan->k, n = plan->n_lines;
    sim_segment_t* ptrs[RFEC_MAX_K];
    long total = 0;
    for (uint32_t g = g0; g < g1; ++g) {
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

long oracle_recover_aos(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                        const uint64_t* present, sim_segment_t* out)
{
    return recover_aos_range(plan, 0, groups, segs, fecs, present, out);
}

typedef struct {
    const rfec_plan* plan;
    uint32_t g0, g1;
    sim_segment_t *segs, *out;
    sim_fec_t* fecs;
    const uint64_t* present;
    long recovered;
} rec_job;

static void* rec_worker(void* p)
{
    rec_job* j = (rec_job*)p;
    j->recovered = recover_aos_range(j->plan, j->g0, j->g1, j->segs, j->fecs, j->present, j->out);
    return NULL;
}

/* the CPU baseline's all-cores leg: a pthread group split */
long oracle_recover_aos_mt(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                           const uint64_t* present, sim_segment_t* out, int threads)
{
    if (threads < 1)
        threads = 1;
    if (threads > 256)
        threads = 256;
    pthread_t tid[256];
    rec_job jobs[256];
    for (int t = 0; t < threads; ++t) {
        jobs[t].plan = plan;
        jobs[t].g0 = (uint32_t)((uint64_t)groups * t / threads);
        jobs[t].g1 = (uint32_t)((uint64_t)groups * (t + 1) / threads);
        jobs[t].segs = segs;
        jobs[t].out = out;
        jobs[t].fecs = fecs;
        jobs[t].present = present;
        jobs[t].recovered = 0;
        pthread_create(&tid[t], NULL, rec_worker, &jobs[t]);
    }
    long total = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(tid[t], NULL);
        total += jobs[t].recovered;
    }
    return total;
}

/* ---- wire codec: sim_proto.c / sim_proto.inl / cf_stream.c / cf_crc32.c ---- */

/* cf_crc32.c:56-68: reflected CRC-32 (poly 0xEDB88320), pre/post inverted;
 * the table (cf_crc32.c:10-54) is the standard one, rebuilt here bitwise. */
uint32_t oracle_crc32(uint32_t crc, const void* buf, size_t size)
{
    static uint32_t tab[256];
    static int init;
    if (!init) {
        for (uint32_t b = 0; b < 256; ++b) {
            uint32_t c = b;
            for (int i = 0; i < 8; ++i)
                c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
            tab[b] = c;
        }
        init = 1;
    }
    const uint8_t* p = (const uint8_t*)buf;
    crc = crc ^ ~0u;
    while (size--)
        crc = tab[(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return crc ^ ~0u;
}

/* bin_stream writers: big-endian (cf_stream.c:366-385 mach_put_2/4 on a
 * little-endian host), mach_data_write = u16 length + bytes (:328-337) */
typedef struct {
    uint8_t* p;
    size_t n;
} wbuf;
static void w8(wbuf* w, uint8_t v) { w->p[w->n++] = v; }
static void w16(wbuf* w, uint16_t v)
{
    w8(w, (uint8_t)(v >> 8));
    w8(w, (uint8_t)v);
}
static void w32(wbuf* w, uint32_t v)
{
    w16(w, (uint16_t)(v >> 16));
    w16(w, (uint16_t)v);
}
static void wdata(wbuf* w, const uint8_t* d, size_t n)
{
    w16(w, (uint16_t)n);
    memcpy(w->p + w->n, d, n);
    w->n += n;
}
/* sim_proto.c:13-18 header, :92-94 CRC trailer */
static void w_header(wbuf* w, uint8_t mid, uint32_t uid)
{
    w8(w, RFEC_WIRE_VER);
    w8(w, mid);
    w32(w, uid);
}
static size_t w_crc(wbuf* w)
{
    w32(w, oracle_crc32(RFEC_WIRE_CRC_SEED, w->p, w->n));
    return w->n;
}

/* sim_fec_encode, sim_proto.inl:270-285 (+ sim_fec_meta_encode :244-254) */
size_t oracle_wire_frame_fec(const sim_fec_t* f, uint32_t uid, uint8_t* out)
{
    wbuf w = {out, 0};
    w_header(&w, RFEC_WIRE_FEC, uid);
    w16(&w, f->fec_id);
    w8(&w, f->row);
    w8(&w, f->col);
    w8(&w, f->index);
    w16(&w, f->count);
    w32(&w, f->base_id);
    w16(&w, f->transport_seq);
    w32(&w, f->send_ts);
    w32(&w, f->fec_meta.seq);
    w32(&w, f->fec_meta.fid);
    w32(&w, f->fec_meta.ts);
    w16(&w, f->fec_meta.index);
    w16(&w, f->fec_meta.total);
    w8(&w, f->fec_meta.ftype);
    w8(&w, f->fec_meta.payload_type);
    w16(&w, f->fec_meta.size);
    wdata(&w, f->fec_data, f->fec_data_size);
    return w_crc(&w);
}

/* sim_segment_encode, sim_proto.inl:83-125: field widths follow the values */
size_t oracle_wire_frame_seg(const sim_segment_t* s, uint32_t uid, uint8_t* out)
{
    wbuf w = {out, 0};
    w_header(&w, RFEC_WIRE_SEG, uid);
    uint8_t mask = s->ftype & 0x01;
    if (s->packet_id > 65535)
        mask |= 1 << 7;
    if (s->fid > 65535)
        mask |= 1 << 6;
    if (s->total > 255)
        mask |= 1 << 5;
    if (s->remb == 0)
        mask |= 1 << 4;
    w8(&w, mask);
    w8(&w, s->payload_type);
    if (s->packet_id > 65535)
        w32(&w, s->packet_id);
    else
        w16(&w, (uint16_t)s->packet_id);
    if (s->fid > 65535)
        w32(&w, s->fid);
    else
        w16(&w, (uint16_t)s->fid);
    w32(&w, s->timestamp);
    if (s->total > 255) {
        w16(&w, s->index);
        w16(&w, s->total);
    } else {
        w8(&w, (uint8_t)s->index);
        w8(&w, (uint8_t)s->total);
    }
    w16(&w, s->fec_id);
    w16(&w, s->send_ts);
    w16(&w, s->transport_seq);
    wdata(&w, s->data, s->data_size);
    return w_crc(&w);
}

/* bin_stream readers: a read past `used` yields 0 and does not advance
 * (cf_stream.c mach_uint8/16/32_read); `used` covers the CRC trailer too. */
typedef struct {
    const uint8_t* p;
    size_t used, r;
} rbuf;
static uint8_t r8(rbuf* b)
{
    if (b->used < b->r + 1)
        return 0;
    return b->p[b->r++];
}
static uint16_t r16(rbuf* b)
{
    if (b->used < b->r + 2)
        return 0;
    uint16_t v = (uint16_t)(b->p[b->r] << 8 | b->p[b->r + 1]);
    b->r += 2;
    return v;
}
static uint32_t r32(rbuf* b)
{
    if (b->used < b->r + 4)
        return 0;
    uint32_t v = (uint32_t)b->p[b->r] << 24 | (uint32_t)b->p[b->r + 1] << 16 | (uint32_t)b->p[b->r + 2] << 8 |
                 b->p[b->r + 3];
    b->r += 4;
    return v;
}
/* mach_data_read, cf_stream.c:339-355: 0xFFFF on a bad length */
static uint16_t rdata(rbuf* b, uint8_t* dst, size_t cap)
{
    uint16_t len = r16(b);
    if (len > cap || b->r + len > b->used)
        return 0xFFFF;
    memcpy(dst, b->p + b->r, len);
    b->r += len;
    return len;
}

/* sim_session_process (sim_session.c:587-596) -> sim_decode_header
 * (sim_proto.c:21-37) -> sim_decode_msg (:99-146) for SIM_SEG / SIM_FEC.
 * Fills rec and payload[0:data_size) (payload zeroed to `capacity`). */
int oracle_wire_parse(const uint8_t* d, size_t len, uint32_t capacity, rfec_wire_rec* rec, uint8_t* payload)
{
    memset(rec, 0, sizeof(*rec));
    memset(payload, 0, capacity);
    if (len < 4) { /* the reference would read before the buffer; rejected here */
        rec->status = RFEC_WIRE_EBADCRC;
        return rec->status;
    }
    const uint32_t src = (uint32_t)d[len - 4] << 24 | (uint32_t)d[len - 3] << 16 | (uint32_t)d[len - 2] << 8 |
                         d[len - 1];
    if (oracle_crc32(RFEC_WIRE_CRC_SEED, d, len - 4) != src) {
        rec->status = RFEC_WIRE_EBADCRC;
        return rec->status;
    }
    rbuf b = {d, len, 0};
    rec->ver = r8(&b);
    rec->mid = r8(&b);
    rec->uid = r32(&b);
    if (rec->mid < RFEC_WIRE_MIN_MID || rec->mid > RFEC_WIRE_MAX_MID) {
        rec->status = RFEC_WIRE_EMID;
        return rec->status;
    }
    if (rec->mid == RFEC_WIRE_SEG) { /* sim_segment_decode, sim_proto.inl:127-179 */
        const uint8_t mask = r8(&b);
        rec->hdr.payload_type = r8(&b);
        rec->hdr.ftype = mask & 0x01;
        rec->hdr.seq = (mask & (1 << 7)) ? r32(&b) : r16(&b);
        rec->hdr.fid = (mask & (1 << 6)) ? r32(&b) : r16(&b);
        rec->hdr.ts = r32(&b);
        if (mask & (1 << 5)) {
            rec->hdr.index = r16(&b);
            rec->hdr.total = r16(&b);
        } else {
            rec->hdr.index = r8(&b);
            rec->hdr.total = r8(&b);
        }
        rec->remb = (mask & (1 << 4)) ? 0 : 0xff;
        rec->fec_id = r16(&b);
        rec->send_ts = r16(&b);
        rec->transport_seq = r16(&b);
        uint16_t n = rdata(&b, payload, capacity);
        if (n == 0xFFFF)
            n = 0;
        rec->data_size = n;
        rec->hdr.size = n;
        rec->status = RFEC_WIRE_OK;
        return rec->status;
    }
    if (rec->mid == RFEC_WIRE_FEC) { /* sim_fec_decode, sim_proto.inl:287-307 */
        rec->fec_id = r16(&b);
        rec->row = r8(&b);
        rec->col = r8(&b);
        rec->index = r8(&b);
        rec->count = r16(&b);
        rec->base_id = r32(&b);
        rec->transport_seq = r16(&b);
        rec->send_ts = r32(&b);
        rec->hdr.seq = r32(&b); /* sim_fec_meta_decode, :256-268 */
        rec->hdr.fid = r32(&b);
        rec->hdr.ts = r32(&b);
        rec->hdr.index = r16(&b);
        rec->hdr.total = r16(&b);
        rec->hdr.ftype = r8(&b);
        rec->hdr.payload_type = r8(&b);
        rec->hdr.size = r16(&b);
        uint16_t n = rdata(&b, payload, capacity);
        if (n > capacity) {
            rec->data_size = 0;
            rec->status = RFEC_WIRE_EBODY;
            return rec->status;
        }
        rec->data_size = n;
        rec->status = RFEC_WIRE_OK;
        return rec->status;
    }
    rec->status = RFEC_WIRE_OTHER;
    return rec->status;
}

/* Batched forms over the product's device layout (include/razor_fec.h). */
void oracle_wire_frame_fec_batch(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                                 const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                                 const rfec_fec_stamp* stamps, uint32_t dstride, uint8_t* dgram, uint16_t* dlen)
{
    sim_fec_t* f = (sim_fec_t*)calloc(1, sizeof(sim_fec_t) + 65536);
    for (size_t d = 0; d < count; ++d) {
        uint8_t* out = dgram + d * dstride;
        memset(out, 0, dstride);
        if ((status && status[d] < 0) || fec_size[d] > capacity) {
            dlen[d] = 0;
            continue;
        }
        const rfec_fec_stamp* s = &stamps[d];
        f->fec_id = s->fec_id;
        f->row = s->row;
        f->col = s->col;
        f->index = s->index;
        f->count = s->count;
        f->base_id = s->base_id;
        f->transport_seq = s->transport_seq;
        f->send_ts = s->send_ts;
        memcpy(&f->fec_meta, &meta[d], sizeof(rfec_hdr));
        f->fec_data_size = fec_size[d];
        memcpy(f->fec_data, parity + d * stride, fec_size[d]);
        dlen[d] = (uint16_t)oracle_wire_frame_fec(f, s->uid, out);
    }
    free(f);
}

void oracle_wire_frame_seg_batch(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                                 const rfec_hdr* hdr, const rfec_seg_stamp* stamps, uint32_t dstride, uint8_t* dgram,
                                 uint16_t* dlen)
{
    sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t) + 65536);
    for (size_t i = 0; i < count; ++i) {
        uint8_t* out = dgram + i * dstride;
        memset(out, 0, dstride);
        const rfec_hdr* h = &hdr[i];
        if (h->size > capacity) {
            dlen[i] = 0;
            continue;
        }
        s->packet_id = h->seq;
        s->fid = h->fid;
        s->timestamp = h->ts;
        s->index = h->index;
        s->total = h->total;
        s->ftype = h->ftype;
        s->payload_type = h->payload_type;
        s->data_size = h->size;
        s->fec_id = stamps[i].fec_id;
        s->send_ts = stamps[i].send_ts;
        s->transport_seq = stamps[i].transport_seq;
        s->remb = stamps[i].remb;
        memcpy(s->data, shards + i * stride, h->size);
        dlen[i] = (uint16_t)oracle_wire_frame_seg(s, stamps[i].uid, out);
    }
    free(s);
}

void oracle_wire_parse_batch(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                             uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload)
{
    uint8_t* tmp = (uint8_t*)malloc(capacity + 1);
    for (size_t i = 0; i < n; ++i) {
        oracle_wire_parse(dgram + i * dstride, dlen[i], capacity, &recs[i], tmp);
        memset(payload + i * stride, 0, stride);
        memcpy(payload + i * stride, tmp, recs[i].data_size);
    }
    free(tmp);
}

/* ---- sender staging: sim_sender.c:254-284, 286-377; flex_fec_sender.c ------ */
void oracle_sender_init(rfec_sender_state* st)
{
    memset(st, 0, sizeof(*st));
    st->first_ts = -1;  /* sim_sender.c:215-ish: first_ts = -1 until the first frame */
    st->fec_id = 1;     /* flex_fec_sender_create / reset: fec_id = 1 (flex_fec_sender.c:40) */
    st->first = 1;
}

/* sim_split_frame, sim_sender.c:254-284 */
static uint32_t oracle_split(uint32_t size, uint32_t seg, uint32_t i, uint32_t total)
{
    if (size <= seg)
        return size;
    const uint32_t packet_size = size / total, remain = size % total;
    return i < remain ? packet_size + 1 : packet_size;
}

/* flex_fec_sender_update (flex_fec_sender.c:146-245) called by sim_sender_fec
 * (sim_sender.c:286-304) at time now: on flex_fec_sender_over (:137-143) it
 * emits the group's parities (if any line has >= 2 members), resets and
 * advances fec_id, skipping 0 (:236-243).  Returns 0, or -1 when `groups` is full. */
static int oracle_sender_update(rfec_sender_state* s, int64_t now, uint8_t pf, rfec_seg_plan* segs, uint32_t ns,
                                rfec_group_plan* groups, uint32_t max_groups, uint32_t* ng)
{
    if (!(s->fec_ts + 500 < now || s->segs_count >= 6)) /* FEC_REPAIR_WINDOW = 500 */
        return 0;
    rfec_plan plan;
    int n_lines = 0;
    if (s->segs_count > 0 &&
        oracle_plan_from_fraction((int)s->segs_count, pf, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, &plan) == 0)
        n_lines = plan.n_lines;
    const int32_t gid = n_lines > 0 ? (int32_t)*ng : -1;
    if (n_lines > 0) {
        if (*ng >= max_groups)
            return -1;
        rfec_group_plan* gp = &groups[(*ng)++];
        memset(gp, 0, sizeof(*gp));
        gp->first_seg = s->open_seg;
        gp->count = s->segs_count;
        gp->fec_id = s->fec_id;
        gp->base_id = s->base_id;
        gp->protect_fraction = pf;
        gp->n_lines = (uint8_t)n_lines;
        gp->fec_send_id0 = s->send_id_seed + 1; /* one send id per parity, sim_sender.c:295-296 */
        gp->fec_ts = (uint32_t)(now - s->first_ts); /* :299 */
        s->send_id_seed += (uint32_t)n_lines;
    }
    if (s->segs_count > 0)
        for (int32_t q = s->open_seg; q < (int32_t)ns; ++q)
            if (q >= 0)
                segs[q].group = gid;
    s->fec_ts = 0;
    s->segs_count = 0;
    s->base_id = 0;
    s->first = 1;
    s->fec_id++;
    if (s->fec_id == 0)
        s->fec_id = 1;
    return 0;
}

int oracle_sender_plan(rfec_sender_state* st, const rfec_frame* frames, uint32_t n, uint32_t seg_size,
                       rfec_seg_plan* segs, uint32_t max_segs, uint32_t* n_segs, rfec_group_plan* groups,
                       uint32_t max_groups, uint32_t* n_groups)
{
    uint32_t ns = 0, ng = 0;
    rfec_sender_state s = *st;
    for (uint32_t f = 0; f < n; ++f) {
        const rfec_frame* fr = &frames[f];
        const uint32_t total = fr->size <= seg_size ? 1u : (fr->size + seg_size - 1) / seg_size; /* :258-265 */
        uint32_t timestamp;
        if (s.first_ts == -1) { /* :333-338 */
            timestamp = 0;
            s.first_ts = fr->now_ms;
        } else {
            timestamp = (uint32_t)(fr->now_ms - s.first_ts);
        }
        ++s.frame_id_seed; /* :341 */
        uint32_t off = 0;
        for (uint32_t i = 0; i < total; ++i) {
            if (ns >= max_segs)
                return -1;
            rfec_seg_plan* g = &segs[ns];
            memset(g, 0, sizeof(*g));
            g->frame = f;
            g->offset = off;
            g->packet_id = ++s.packet_id_seed; /* :344-352 */
            g->send_id = ++s.send_id_seed;
            g->fid = s.frame_id_seed;
            g->timestamp = timestamp;
            g->ftype = fr->ftype;
            g->payload_type = fr->payload_type;
            g->index = (uint16_t)i;
            g->total = (uint16_t)total;
            g->data_size = (uint16_t)oracle_split(fr->size, seg_size, i, total);
            off += g->data_size;
            g->fec_id = s.fec_id; /* :360-362 */
            g->group = -2;
            /* flex_fec_sender_add_segment, flex_fec_sender.c:49-78 */
            if (s.fec_ts == 0) {
                s.fec_ts = fr->now_ms;
            } else if (s.fec_ts + 500 * 4 < fr->now_ms) { /* stale: the open segments are dropped */
                for (int32_t q = s.open_seg; q < (int32_t)ns; ++q)
                    if (q >= 0)
                        segs[q].group = -1;
                s.segs_count = 0;
                s.base_id = 0;
                s.first = 1;
                s.fec_ts = fr->now_ms;
            }
            if (s.segs_count == 0)
                s.open_seg = (int32_t)ns;
            s.base_id = s.first ? g->packet_id : (g->packet_id < s.base_id ? g->packet_id : s.base_id);
            s.first = 0;
            s.segs_count++;
            ns++;
            if (s.segs_count >= 100 && /* sim_sender.c:370-371 */
                oracle_sender_update(&s, fr->now_ms, fr->protect_fraction, segs, ns, groups, max_groups, &ng))
                return -1;
        }
        /* sim_sender.c:373-374: after every frame */
        if (oracle_sender_update(&s, fr->now_ms, fr->protect_fraction, segs, ns, groups, max_groups, &ng))
            return -1;
    }
    if (s.segs_count > 0)
        s.open_seg -= (int32_t)ns;
    else
        s.open_seg = 0;
    *st = s;
    *n_segs = ns;
    *n_groups = ng;
    return 0;
}

/* ---- receiver ingestion: sim_fec.c:104-207 + flex_fec_receiver.c:69-280, ----
 * event by event (the reference's own order), with the recovery cascade of
 * sim_receiver_recover (sim_receiver.c:780-804). */
typedef struct { /* open-addressing u32 -> int32 map */
    uint32_t* key;
    int32_t* val;
    uint32_t cap, n;
} omap;

static void om_init(omap* m, uint32_t cap)
{
    m->cap = 16;
    while (m->cap < 2 * cap)
        m->cap <<= 1;
    m->key = (uint32_t*)calloc(m->cap, sizeof(uint32_t));
    m->val = (int32_t*)malloc(m->cap * sizeof(int32_t));
    for (uint32_t i = 0; i < m->cap; ++i)
        m->val[i] = -1;
    m->n = 0;
}
static void om_free(omap* m)
{
    free(m->key);
    free(m->val);
}
static uint32_t om_slot(const omap* m, uint32_t k)
{
    uint32_t h = (k * 2654435761u) & (m->cap - 1);
    while (m->val[h] != -1 && m->key[h] != k)
        h = (h + 1) & (m->cap - 1);
    return h;
}
static int32_t om_get(const omap* m, uint32_t k)
{
    return m->val[om_slot(m, k)];
}
static void om_put(omap* m, uint32_t k, int32_t v)
{
    if (2 * (m->n + 1) > m->cap) { /* keep the load <= 1/2: a full table never terminates a probe */
        omap g;
        om_init(&g, m->cap);
        for (uint32_t i = 0; i < m->cap; ++i)
            if (m->val[i] != -1) {
                const uint32_t s = om_slot(&g, m->key[i]);
                g.key[s] = m->key[i];
                g.val[s] = m->val[i];
                g.n++;
            }
        om_free(m);
        *m = g;
    }
    const uint32_t h = om_slot(m, k);
    if (m->val[h] == -1)
        m->n++;
    m->key[h] = k;
    m->val[h] = v;
}
static void om_del(omap* m, uint32_t k) /* backward-shift deletion */
{
    uint32_t h = om_slot(m, k);
    if (m->val[h] == -1)
        return;
    m->val[h] = -1;
    m->n--;
    uint32_t j = h;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (m->val[j] == -1)
            return;
        const uint32_t want = (m->key[j] * 2654435761u) & (m->cap - 1);
        if ((j > h && (want <= h || want > j)) || (j < h && (want <= h && want > j))) {
            m->key[h] = m->key[j];
            m->val[h] = m->val[j];
            m->val[j] = -1;
            h = j;
        }
    }
}

typedef struct {
    uint16_t fec_id;
    uint8_t row, col;
    uint32_t base_id, count;
    uint32_t fec_ts;  /* flex->fec_ts: send_ts of the parity that created it (sim_fec.c:157) */
    omap segs; /* packet_id -> segment pool index */
    omap fecs; /* index -> parity record index */
    int live;
} oflex;

typedef struct {
    const rfec_wire_rec* recs;
    const uint8_t* payload;
    uint32_t stride, capacity;
    sim_segment_t* pool; /* cached + recovered segments */
    uint32_t pool_n, pool_cap;
    omap seen, cache, recov;
    omap flex_of;        /* fec_id -> flex index */
    oflex* flex;
    uint32_t n_flex, flex_cap;
    uint32_t max_ts;
    uint32_t dropped;
} orx;

static int32_t rx_pool_add(orx* R, const sim_segment_t* s)
{
    if (R->pool_n == R->pool_cap) {
        R->pool_cap = R->pool_cap ? 2 * R->pool_cap : 1024;
        R->pool = (sim_segment_t*)realloc(R->pool, (size_t)R->pool_cap * sizeof(sim_segment_t));
    }
    R->pool[R->pool_n] = *s;
    return (int32_t)R->pool_n++;
}

static void rx_fec_struct(const orx* R, int32_t rec, sim_fec_t* f)
{
    const rfec_wire_rec* r = &R->recs[rec];
    memset(f, 0, sizeof(*f));
    f->fec_id = r->fec_id;
    f->row = r->row;
    f->col = r->col;
    f->index = r->index;
    f->count = r->count;
    f->base_id = r->base_id;
    f->send_ts = r->send_ts;
    f->transport_seq = r->transport_seq;
    memcpy(&f->fec_meta, &r->hdr, sizeof(rfec_hdr));
    f->fec_data_size = r->data_size;
    memcpy(f->fec_data, R->payload + (size_t)rec * R->stride, r->data_size < SIM_VIDEO_SIZE ? r->data_size : SIM_VIDEO_SIZE);
}

/* flex_recover_row / flex_recover_col (flex_fec_receiver.c:105-206) */
static int rx_recover_line(orx* R, oflex* x, int is_col, uint32_t line, sim_segment_t* out)
{
    if (x->segs.n >= x->count)
        return 0;
    sim_segment_t* cache[256];
    int cnt = 0, loss = 0;
    const uint32_t lim = is_col ? x->row : x->col;
    for (uint32_t i = 0; i < lim; ++i) {
        const uint32_t key = is_col ? i * x->col + line + x->base_id : line * x->col + i + x->base_id;
        if (key >= x->base_id + x->count)
            break;
        const int32_t p = om_get(&x->segs, key);
        if (p >= 0)
            cache[cnt++] = &R->pool[p];
        else
            loss++;
    }
    if (loss != 1 || cnt == 0)
        return 0;
    const int32_t fr = om_get(&x->fecs, is_col ? (line | 0x80u) : line);
    if (fr < 0)
        return 0;
    static sim_fec_t fec;
    rx_fec_struct(R, fr, &fec);
    memset(out, 0, sizeof(*out));
    return oracle_recover(cache, cnt, &fec, out) == 0;
}

/* sim_fec_packet_add_recover (sim_fec.c:104-119): first copy per packet_id */
static void rx_add_recover(orx* R, const sim_segment_t* s)
{
    if (om_get(&R->recov, s->packet_id) >= 0)
        return;
    om_put(&R->recov, s->packet_id, rx_pool_add(R, s));
}

/* flex_fec_receiver_on_segment (flex_fec_receiver.c:243-280) */
static void rx_on_segment(orx* R, oflex* x, int32_t pi, int add)
{
    const sim_segment_t* s = &R->pool[pi];
    if (x->col < 2 || x->row == 0 || x->count == 0 || s->packet_id < x->base_id)
        return;
    if (om_get(&x->segs, s->packet_id) >= 0)
        return;
    om_put(&x->segs, s->packet_id, pi);
    const uint32_t c = (s->packet_id - x->base_id) % x->col, r = (s->packet_id - x->base_id) / x->col;
    sim_segment_t out;
    if (rx_recover_line(R, x, 0, r, &out) && add)
        rx_add_recover(R, &out);
    if (rx_recover_line(R, x, 1, c, &out) && add)
        rx_add_recover(R, &out);
}

static void rx_remove_flex(orx* R, uint32_t fi)
{
    oflex* x = &R->flex[fi];
    for (uint32_t i = 0; i < x->count; ++i) /* sim_fec_evict_segment (sim_fec.c:93-102) */
        om_del(&R->cache, x->base_id + i);
    om_del(&R->flex_of, x->fec_id);
    om_free(&x->segs);
    om_free(&x->fecs);
    x->live = 0;
}

/* sim_fec_put_segment (sim_fec.c:171-207) */
static void rx_put_segment(orx* R, const sim_segment_t* s)
{
    if (s->packet_id <= 0) /* f->base_id == 0 */
        return;
    if (om_get(&R->cache, s->packet_id) >= 0)
        return;
    R->max_ts = s->timestamp > R->max_ts ? s->timestamp : R->max_ts;
    const int32_t pi = rx_pool_add(R, s);
    om_put(&R->cache, s->packet_id, pi);
    const int32_t fi = om_get(&R->flex_of, s->fec_id);
    if (fi < 0)
        return;
    rx_on_segment(R, &R->flex[fi], pi, 1);
    if (R->flex[fi].segs.n >= R->flex[fi].count) /* flex_fec_receiver_full */
        rx_remove_flex(R, (uint32_t)fi);
}

/* sim_fec_put_fec_packet (sim_fec.c:141-169) */
static void rx_put_fec(orx* R, int32_t rec)
{
    const rfec_wire_rec* f = &R->recs[rec];
    if (f->base_id + f->count < 0u + 1u || f->send_ts + 3000u < R->max_ts) { /* EVICT_FEC_DELAY */
        R->dropped++;
        return;
    }
    int32_t fi = om_get(&R->flex_of, f->fec_id);
    if (fi < 0) {
        if (R->n_flex == R->flex_cap) {
            R->flex_cap = R->flex_cap ? 2 * R->flex_cap : 64;
            R->flex = (oflex*)realloc(R->flex, R->flex_cap * sizeof(oflex));
        }
        fi = (int32_t)R->n_flex++;
        oflex* x = &R->flex[fi];
        memset(x, 0, sizeof(*x));
        x->fec_id = f->fec_id; /* flex_fec_receiver_active (flex_fec_receiver.c:69-88) */
        x->base_id = f->base_id;
        x->row = f->row;
        x->col = f->col;
        x->count = f->count;
        x->fec_ts = f->send_ts;
        x->live = 1;
        om_init(&x->segs, x->count + 8);
        om_init(&x->fecs, 64);
        om_put(&R->flex_of, f->fec_id, fi);
        for (uint32_t i = 0; i < f->count; ++i) { /* sim_fec_add_segment_to_flex (sim_fec.c:121-138) */
            const int32_t pi = om_get(&R->cache, f->base_id + i);
            if (pi >= 0)
                rx_on_segment(R, x, pi, 0);
        }
    }
    oflex* x = &R->flex[fi];
    /* flex_fec_receiver_on_fec (flex_fec_receiver.c:208-241) */
    if (x->col < 2 || x->row == 0 || x->count == 0 || om_get(&x->fecs, f->index) >= 0)
        return;
    om_put(&x->fecs, f->index, rec);
    sim_segment_t out;
    if (rx_recover_line(R, x, (f->index & 0x80) != 0, f->index & 0x7Fu, &out))
        rx_add_recover(R, &out);
}

static int cmp_u32(const void* a, const void* b)
{
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* sim_fec_evict (sim_fec.c:209-241) past its 300 ms wall-clock gate: flexes in
 * fec_id order (the u16 skiplist) while stale (fec_ts + 3000 <= max_ts) or
 * full, then cached segments in packet_id order while older than 6 s */
static void rx_evict(orx* R)
{
    uint32_t* keys = (uint32_t*)malloc(((size_t)R->flex_of.n + R->cache.n + 1) * sizeof(uint32_t));
    uint32_t nk = 0;
    for (uint32_t h = 0; h < R->flex_of.cap; ++h)
        if (R->flex_of.val[h] != -1)
            keys[nk++] = R->flex_of.key[h];
    qsort(keys, nk, sizeof(uint32_t), cmp_u32);
    for (uint32_t i = 0; i < nk; ++i) {
        const int32_t fi = om_get(&R->flex_of, keys[i]);
        const oflex* x = &R->flex[fi];
        if (!(x->fec_ts + 3000u <= R->max_ts || x->segs.n >= x->count))
            break;
        rx_remove_flex(R, (uint32_t)fi);
    }
    nk = 0;
    for (uint32_t h = 0; h < R->cache.cap; ++h)
        if (R->cache.val[h] != -1)
            keys[nk++] = R->cache.key[h];
    qsort(keys, nk, sizeof(uint32_t), cmp_u32);
    for (uint32_t i = 0; i < nk; ++i) {
        const int32_t pi = om_get(&R->cache, keys[i]);
        if (!(R->pool[pi].timestamp + 6000u < R->max_ts))
            break;
        om_del(&R->cache, keys[i]);
    }
    free(keys);
}

int oracle_rx_recover(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                      uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out,
                      uint32_t* n_out, uint32_t* dropped)
{
    return oracle_rx_recover_ev(n, recs, payload, stride, capacity, max_ts, out, out_payload, max_out, n_out, dropped, 0);
}

/* As oracle_rx_recover, with sim_fec_evict after every evict_every arrivals
 * (0: never), as the session heartbeat runs it between datagrams. */
int oracle_rx_recover_ev(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                         uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload,
                         uint32_t max_out, uint32_t* n_out, uint32_t* dropped, uint32_t evict_every)
{
    orx R;
    memset(&R, 0, sizeof(R));
    R.recs = recs;
    R.payload = payload;
    R.stride = stride;
    R.capacity = capacity;
    R.max_ts = *max_ts;
    om_init(&R.seen, n + 16);
    om_init(&R.cache, n + 16);
    om_init(&R.recov, 64);
    om_init(&R.flex_of, 1024);
    uint32_t no = 0;
    sim_segment_t seg;
    for (uint32_t a = 0; a < n; ++a) {
        const rfec_wire_rec* r = &recs[a];
        if (r->status != RFEC_WIRE_OK)
            continue;
        if (r->mid == RFEC_WIRE_SEG) { /* sim_receiver_put (sim_receiver.c:811-827) */
            if (om_get(&R.seen, r->hdr.seq) >= 0)
                continue;
            om_put(&R.seen, r->hdr.seq, 1);
            if (r->fec_id == 0)
                continue;
            memset(&seg, 0, sizeof(seg));
            seg.packet_id = r->hdr.seq;
            seg.fid = r->hdr.fid;
            seg.timestamp = r->hdr.ts;
            seg.index = r->hdr.index;
            seg.total = r->hdr.total;
            seg.ftype = r->hdr.ftype;
            seg.payload_type = r->hdr.payload_type;
            seg.fec_id = r->fec_id;
            seg.data_size = r->data_size;
            memcpy(seg.data, payload + (size_t)a * stride, r->data_size < SIM_VIDEO_SIZE ? r->data_size : SIM_VIDEO_SIZE);
            rx_put_segment(&R, &seg);
        } else if (r->mid == RFEC_WIRE_FEC) {
            rx_put_fec(&R, (int32_t)a);
        }
        /* sim_receiver_recover (sim_receiver.c:780-804): lowest packet_id first */
        while (R.recov.n > 0) {
            uint32_t best = 0xFFFFFFFFu;
            for (uint32_t h = 0; h < R.recov.cap; ++h)
                if (R.recov.val[h] != -1 && R.recov.key[h] < best)
                    best = R.recov.key[h];
            const int32_t pi = om_get(&R.recov, best);
            om_del(&R.recov, best);
            const sim_segment_t rs = R.pool[pi];
            if (om_get(&R.seen, rs.packet_id) >= 0)
                continue;
            om_put(&R.seen, rs.packet_id, 1);
            if (no < max_out) {
                rfec_rx_seg* o = &out[no];
                memset(o, 0, sizeof(*o));
                o->hdr.seq = rs.packet_id;
                o->hdr.fid = rs.fid;
                o->hdr.ts = rs.timestamp;
                o->hdr.index = rs.index;
                o->hdr.total = rs.total;
                o->hdr.ftype = rs.ftype;
                o->hdr.payload_type = rs.payload_type;
                o->hdr.size = rs.data_size;
                o->fec_id = rs.fec_id;
                memset(out_payload + (size_t)no * stride, 0, stride);
                memcpy(out_payload + (size_t)no * stride, rs.data, rs.data_size);
            }
            no++;
            rx_put_segment(&R, &rs);
        }
        if (evict_every && a % evict_every == evict_every - 1)
            rx_evict(&R);
    }
    *max_ts = R.max_ts;
    *n_out = no;
    if (dropped)
        *dropped = R.dropped;
    for (uint32_t i = 0; i < R.n_flex; ++i)
        if (R.flex[i].live) {
            om_free(&R.flex[i].segs);
            om_free(&R.flex[i].fecs);
        }
    free(R.flex);
    free(R.pool);
    om_free(&R.seen);
    om_free(&R.cache);
    om_free(&R.recov);
    om_free(&R.flex_of);
    (void)capacity;
    return no > max_out ? -1 : 0;
}
