/*
 * gen_golden.c -- golden-vector generator (own code).  Links the reference's
 * FEC sources compiled out-of-tree from /root/reference (oracle/Makefile) and
 * writes expected outputs to tests/golden/.  Inputs are not stored: they are
 * regenerated from the PRNG spec (oracle_fill_groups).
 *
 * Reference entry points exercised:
 *   flex_fec_sender_add_segment / _update   flex_fec_sender.c:49-78, 146-245
 *   flex_fec_sender_num_packets              flex_fec_sender.c:81-135
 *   flex_fec_generate / flex_fec_recover     flex_fec_xor.c:4-53, 55-104
 *   flex_fec_receiver_active/_on_segment/_on_fec (peeling) flex_fec_receiver.c:69-280
 *
 * Usage: gen_golden <outdir>
 */
#include "flex_fec_receiver.h"
#include "flex_fec_sender.h"

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* oracle PRNG + fill (rfec_oracle.c); declared here to keep the reference's
 * type definitions the only ones in this translation unit. */
typedef struct {
    uint32_t seq, fid, ts;
    uint16_t index, total;
    uint8_t ftype, payload_type;
    uint16_t size;
} g_hdr; /* layout of rfec_hdr */
uint64_t oracle_xs_next(uint64_t* state);
uint32_t oracle_xs_rand(uint64_t* state, uint32_t t);
void oracle_fill_groups(uint64_t config_id, uint32_t groups, uint32_t k, uint32_t S, uint32_t stride,
                        int ragged, uint8_t* shards, void* hdr);

static const char* g_outdir;
static FILE* g_manifest;
static int g_first_case = 1;

/* ---- fixture records ------------------------------------------------------ */
#pragma pack(push, 1)
typedef struct {
    uint16_t fec_id;
    uint8_t row, col, index;
    int8_t status;
    uint16_t count;
    uint32_t base_id;
    uint8_t meta[20];
    uint16_t fec_data_size;
    uint16_t group;
    uint8_t line;
    uint8_t pad[11];
} parity_rec; /* 48 bytes, followed by S payload bytes */

#define MAX_HASH 16
typedef struct {
    uint64_t present[2];
    uint64_t parity_present;
    uint64_t recovered[2];
    uint32_t group;
    uint32_t n_recovered;
    uint64_t hash[MAX_HASH]; /* by ascending segment position */
} erasure_rec;
#pragma pack(pop)

static uint64_t fnv1a(uint64_t h, const void* p, size_t n)
{
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

static void seg_record(const sim_segment_t* s, uint8_t rec[20])
{
    g_hdr h;
    h.seq = s->packet_id;
    h.fid = s->fid;
    h.ts = s->timestamp;
    h.index = s->index;
    h.total = s->total;
    h.ftype = s->ftype;
    h.payload_type = s->payload_type;
    h.size = s->data_size;
    memcpy(rec, &h, 20);
}

static uint64_t seg_hash(const sim_segment_t* s)
{
    uint8_t rec[20];
    seg_record(s, rec);
    uint64_t h = fnv1a(0xcbf29ce484222325ull, rec, 20);
    return fnv1a(h, s->data, s->data_size);
}

static void meta_bytes(const sim_fec_meta_t* m, uint8_t out[20])
{
    g_hdr h;
    h.seq = m->seq;
    h.fid = m->fid;
    h.ts = m->ts;
    h.index = m->index;
    h.total = m->total;
    h.ftype = m->ftype;
    h.payload_type = m->payload_type;
    h.size = m->size;
    memcpy(out, &h, 20);
}

static FILE* open_out(const char* name)
{
    char path[1024];
    snprintf(path, sizeof(path), "%s/%s", g_outdir, name);
    FILE* f = fopen(path, "wb");
    if (!f) {
        perror(path);
        exit(1);
    }
    return f;
}

static void manifest_case(const char* json)
{
    fprintf(g_manifest, "%s  %s", g_first_case ? "" : ",\n", json);
    g_first_case = 0;
}

/* ---- group construction ---------------------------------------------------- */
typedef struct {
    uint32_t k, S, stride;
    sim_segment_t** segs;
} group_t;

static uint8_t* g_shards;
static g_hdr* g_hdrs;

static void make_groups(uint64_t cfg, uint32_t G, uint32_t k, uint32_t S, int ragged)
{
    uint32_t stride = (S + 15) & ~15u;
    free(g_shards);
    free(g_hdrs);
    g_shards = (uint8_t*)calloc((size_t)G * k, stride);
    g_hdrs = (g_hdr*)calloc((size_t)G * k, sizeof(g_hdr));
    oracle_fill_groups(cfg, G, k, S, stride, ragged, g_shards, g_hdrs);
}

/* Reference segments of group g (calloc'd like test_func.c:18, :159, :304). */
static sim_segment_t** ref_segments(uint32_t g, uint32_t k, uint32_t S, uint32_t off, uint32_t span)
{
    uint32_t stride = (S + 15) & ~15u;
    sim_segment_t** v = (sim_segment_t**)calloc(k, sizeof(*v));
    for (uint32_t i = 0; i < k; ++i) {
        const g_hdr* h = &g_hdrs[(size_t)g * k + i];
        sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t));
        s->packet_id = h->seq;
        s->fid = h->fid;
        s->timestamp = h->ts;
        s->index = h->index;
        s->total = h->total;
        s->ftype = h->ftype;
        s->payload_type = h->payload_type;
        /* window [off, off+span) of the payload (used to pin >SIM_VIDEO_SIZE
         * payloads by halves); span == S gives the whole payload */
        int ds = (int)h->size - (int)off;
        if (ds < 0)
            ds = 0;
        if (ds > (int)span)
            ds = (int)span;
        s->data_size = (uint16_t)ds;
        memcpy(s->data, g_shards + ((size_t)g * k + i) * stride + off, (size_t)ds);
        v[i] = s;
    }
    return v;
}

static void free_segments(sim_segment_t** v, uint32_t k)
{
    for (uint32_t i = 0; i < k; ++i)
        free(v[i]);
    free(v);
}

/* Run the reference sender over one group; returns the parity list. */
static base_list_t* ref_sender_group(flex_fec_sender_t* snd, sim_segment_t** segs, uint32_t k, uint8_t pf)
{
    for (uint32_t i = 0; i < k; ++i)
        flex_fec_sender_add_segment(snd, segs[i]);
    snd->fec_ts = 1; /* make flex_fec_sender_over (:137-143) fire for groups < 6 too */
    base_list_t* out = create_list();
    flex_fec_sender_update(snd, pf, out);
    return out;
}

static void write_parity(FILE* f, const sim_fec_t* p, uint32_t g, uint32_t line, int8_t status, uint32_t S)
{
    parity_rec r;
    memset(&r, 0, sizeof(r));
    r.fec_id = p->fec_id;
    r.row = p->row;
    r.col = p->col;
    r.index = p->index;
    r.status = status;
    r.count = p->count;
    r.base_id = p->base_id;
    meta_bytes(&p->fec_meta, r.meta);
    r.fec_data_size = p->fec_data_size;
    r.group = (uint16_t)g;
    r.line = (uint8_t)line;
    fwrite(&r, sizeof(r), 1, f);
    uint8_t* buf = (uint8_t*)calloc(1, S);
    uint32_t L = p->fec_data_size < S ? p->fec_data_size : S;
    memcpy(buf, p->fec_data, L);
    fwrite(buf, 1, S, f);
    free(buf);
}

/* ---- encode cases driven by the reference sender --------------------------- */
static void case_sender_kind(const char* name, const char* kind, uint64_t cfg, uint32_t G, uint32_t k, uint32_t S,
                             int ragged, uint8_t pf)
{
    char fn[256];
    snprintf(fn, sizeof(fn), "enc_%s.bin", name);
    FILE* f = open_out(fn);
    make_groups(cfg, G, k, S, ragged);
    flex_fec_sender_t* snd = flex_fec_sender_create();
    long total = 0;
    for (uint32_t g = 0; g < G; ++g) {
        sim_segment_t** segs = ref_segments(g, k, S, 0, S);
        base_list_t* out = ref_sender_group(snd, segs, k, pf);
        base_list_unit_t* it;
        uint32_t line = 0;
        LIST_FOREACH(out, it) {
            write_parity(f, (sim_fec_t*)it->pdata, g, line++, 0, S);
            total++;
        }
        flex_fec_sender_release(snd, out);
        destroy_list(out);
        free_segments(segs, k);
    }
    flex_fec_sender_destroy(snd);
    fclose(f);
    char js[512];
    snprintf(js, sizeof(js),
             "{\"name\": \"%s\", \"kind\": \"%s\", \"file\": \"%s\", \"config_id\": %llu, \"groups\": %u, "
             "\"k\": %u, \"S\": %u, \"ragged\": %d, \"protect_fraction\": %u, \"parities\": %ld}",
             name, kind, fn, (unsigned long long)cfg, G, k, S, ragged, pf, total);
    manifest_case(js);
}

static void case_sender(const char* name, uint64_t cfg, uint32_t G, uint32_t k, uint32_t S, int ragged, uint8_t pf)
{
    case_sender_kind(name, "sender", cfg, G, k, S, ragged, pf);
}

/* Random k / random protect fraction per group, one sender across groups. */
static void case_sender_random(const char* name, uint64_t cfg, uint32_t G, uint32_t S)
{
    char fn[256];
    snprintf(fn, sizeof(fn), "enc_%s.bin", name);
    FILE* f = open_out(fn);
    FILE* fk = NULL;
    char fnk[256];
    snprintf(fnk, sizeof(fnk), "enc_%s_groups.bin", name);
    fk = open_out(fnk);
    uint64_t st = 0x9E3779B97F4A7C15ull ^ cfg;
    flex_fec_sender_t* snd = flex_fec_sender_create();
    long total = 0;
    for (uint32_t g = 0; g < G; ++g) {
        uint32_t k = 2 + oracle_xs_rand(&st, 98);   /* 2..100 */
        uint8_t pf = (uint8_t)oracle_xs_rand(&st, 255);
        uint32_t gid[3] = {k, pf, 0};
        make_groups(cfg * 1000 + g, 1, k, S, 1);
        sim_segment_t** segs = ref_segments(0, k, S, 0, S);
        base_list_t* out = ref_sender_group(snd, segs, k, pf);
        base_list_unit_t* it;
        uint32_t line = 0;
        LIST_FOREACH(out, it) {
            write_parity(f, (sim_fec_t*)it->pdata, g, line++, 0, S);
            total++;
        }
        gid[2] = line;
        fwrite(gid, sizeof(gid), 1, fk);
        flex_fec_sender_release(snd, out);
        destroy_list(out);
        free_segments(segs, k);
    }
    flex_fec_sender_destroy(snd);
    fclose(f);
    fclose(fk);
    char js[512];
    snprintf(js, sizeof(js),
             "{\"name\": \"%s\", \"kind\": \"sender_random\", \"file\": \"%s\", \"groups_file\": \"%s\", "
             "\"config_id\": %llu, \"groups\": %u, \"S\": %u, \"ragged\": 1, \"parities\": %ld, "
             "\"group_config_id\": \"config_id*1000+g\"}",
             name, fn, fnk, (unsigned long long)cfg, G, S, total);
    manifest_case(js);
}

/* Explicit row layout (rows of `col` consecutive segments) through
 * flex_fec_generate directly, payload pinned in windows of `span` bytes so
 * payloads wider than SIM_VIDEO_SIZE are still computed by the reference. */
static void case_rows(const char* name, uint64_t cfg, uint32_t G, uint32_t k, uint32_t S, int ragged,
                      uint32_t col, uint32_t span)
{
    char fn[256];
    snprintf(fn, sizeof(fn), "enc_%s.bin", name);
    FILE* f = open_out(fn);
    make_groups(cfg, G, k, S, ragged);
    uint32_t rows = (k + col - 1) / col;
    long total = 0;
    for (uint32_t g = 0; g < G; ++g) {
        for (uint32_t r = 0; r < rows; ++r) {
            uint32_t first = r * col, cnt = k - first < col ? k - first : col;
            if (cnt < 2)
                continue;
            sim_fec_t full;
            memset(&full, 0, sizeof(full));
            uint8_t* data = (uint8_t*)calloc(1, S);
            uint32_t L = 0;
            int ok = 1;
            for (uint32_t off = 0; off < S; off += span) {
                sim_segment_t** segs = ref_segments(g, k, S, off, span);
                sim_fec_t part;
                memset(&part, 0, sizeof(part));
                int rc = flex_fec_generate(&segs[first], (int)cnt, &part);
                if (rc != 0)
                    ok = 0;
                if (off == 0) {
                    full = part; /* meta from the first window: size field below */
                }
                memcpy(data + off, part.fec_data, part.fec_data_size);
                L += part.fec_data_size;
                free_segments(segs, k);
            }
            assert(ok);
            full.fec_data_size = (uint16_t)L;
            if (span < S) {
                /* meta.size: the reference only saw window sizes; the true XOR
                 * of data_size is not pinned by it -> mark 0xFFFF (test skips) */
                full.fec_meta.size = 0xFFFF;
            }
            full.fec_id = (uint16_t)(g + 1);
            full.base_id = g_hdrs[(size_t)g * k].seq;
            full.row = (uint8_t)rows;
            full.col = (uint8_t)col;
            full.index = (uint8_t)r;
            full.count = (uint16_t)k;
            /* write with the assembled payload */
            parity_rec rec;
            memset(&rec, 0, sizeof(rec));
            rec.fec_id = full.fec_id;
            rec.row = full.row;
            rec.col = full.col;
            rec.index = full.index;
            rec.count = full.count;
            rec.base_id = full.base_id;
            meta_bytes(&full.fec_meta, rec.meta);
            rec.fec_data_size = full.fec_data_size;
            rec.group = (uint16_t)g;
            rec.line = (uint8_t)r;
            fwrite(&rec, sizeof(rec), 1, f);
            fwrite(data, 1, S, f);
            free(data);
            total++;
        }
    }
    fclose(f);
    char js[512];
    snprintf(js, sizeof(js),
             "{\"name\": \"%s\", \"kind\": \"rows\", \"file\": \"%s\", \"config_id\": %llu, \"groups\": %u, "
             "\"k\": %u, \"S\": %u, \"ragged\": %d, \"col\": %u, \"span\": %u, \"parities\": %ld}",
             name, fn, (unsigned long long)cfg, G, k, S, ragged, col, span, total);
    manifest_case(js);
}

/* ---- erasure cases: the reference receiver, driven like test_func.c:225-288 - */
typedef struct {
    sim_segment_t* seg[256];
    int n;
} seg_bag;

static void recover_map_add(seg_bag* map, sim_segment_t* s)
{
    if (!s)
        return;
    for (int i = 0; i < map->n; ++i)
        if (map->seg[i]->packet_id == s->packet_id) {
            free(s); /* duplicate, as sim_fec_packet_add_recover (sim_fec.c:104-119) */
            return;
        }
    map->seg[map->n++] = s;
}

static sim_segment_t* recover_map_pop_first(seg_bag* map)
{
    int best = -1;
    for (int i = 0; i < map->n; ++i)
        if (best < 0 || map->seg[i]->packet_id < map->seg[best]->packet_id)
            best = i;
    if (best < 0)
        return NULL;
    sim_segment_t* s = map->seg[best];
    map->seg[best] = map->seg[--map->n];
    return s;
}

static void run_receiver(sim_segment_t** segs, uint32_t k, sim_fec_t** fecs, int nf, const uint64_t present[2],
                         uint64_t parity_present, erasure_rec* out, uint32_t base_id)
{
    memset(out, 0, sizeof(*out));
    out->present[0] = present[0];
    out->present[1] = present[1];
    out->parity_present = parity_present;
    flex_fec_receiver_t* r = flex_fec_receiver_create(NULL, NULL, NULL);
    flex_fec_receiver_active(r, fecs[0]->fec_id, fecs[0]->col, fecs[0]->row, fecs[0]->base_id, fecs[0]->count);
    base_list_t* lst = create_list();
    seg_bag map;
    map.n = 0;
    for (uint32_t i = 0; i < k; ++i)
        if ((present[i >> 6] >> (i & 63)) & 1) {
            flex_fec_receiver_on_segment(r, segs[i], lst);
            while (list_size(lst) > 0)
                recover_map_add(&map, (sim_segment_t*)list_pop(lst));
        }
    for (int l = 0; l < nf; ++l)
        if ((parity_present >> l) & 1) {
            sim_fec_t* c = (sim_fec_t*)malloc(sizeof(sim_fec_t)); /* receiver owns it */
            *c = *fecs[l];
            recover_map_add(&map, flex_fec_receiver_on_fec(r, c));
        }
    sim_segment_t* keep[256];
    int nkeep = 0;
    sim_segment_t* s;
    while ((s = recover_map_pop_first(&map)) != NULL) {
        uint32_t pos = s->packet_id - base_id;
        assert(pos < k);
        out->recovered[pos >> 6] |= 1ull << (pos & 63);
        keep[nkeep++] = s;
        flex_fec_receiver_on_segment(r, s, lst); /* cascade, sim_receiver.c:780-804 */
        while (list_size(lst) > 0)
            recover_map_add(&map, (sim_segment_t*)list_pop(lst));
    }
    /* hashes by ascending position */
    int nh = 0;
    for (uint32_t i = 0; i < k && nh < MAX_HASH; ++i)
        for (int q = 0; q < nkeep; ++q)
            if (keep[q]->packet_id - base_id == i)
                out->hash[nh++] = seg_hash(keep[q]);
    out->n_recovered = (uint32_t)nkeep;
    destroy_list(lst);
    flex_fec_receiver_desotry(r);
    for (int q = 0; q < nkeep; ++q)
        free(keep[q]);
}

static int popcount64(uint64_t x)
{
    return __builtin_popcountll(x);
}

typedef enum { PAT_EXHAUSTIVE = 0, PAT_RANDOM = 1 } pat_kind;

static void case_erasures(const char* name, uint64_t cfg, uint32_t k, uint32_t S, int ragged, uint8_t pf,
                          int rows_only, pat_kind kind, int max_erase, int n_random, double parity_loss)
{
    char fn[256];
    snprintf(fn, sizeof(fn), "era_%s.bin", name);
    FILE* f = open_out(fn);
    make_groups(cfg, 1, k, S, ragged);
    sim_segment_t** segs = ref_segments(0, k, S, 0, S);
    flex_fec_sender_t* snd = flex_fec_sender_create();
    /* the sender zero-pads the segments in place; regenerate pristine copies */
    sim_segment_t** work = ref_segments(0, k, S, 0, S);
    base_list_t* out = ref_sender_group(snd, work, k, pf);
    sim_fec_t* fecs[64];
    int nf = 0;
    base_list_unit_t* it;
    LIST_FOREACH(out, it) fecs[nf++] = (sim_fec_t*)it->pdata;
    uint64_t all_par = (nf >= 64) ? ~0ull : ((1ull << nf) - 1);
    uint64_t row_par = 0;
    for (int l = 0; l < nf; ++l)
        if ((fecs[l]->index & 0x80) == 0)
            row_par |= 1ull << l;
    uint32_t base_id = segs[0]->packet_id;
    long npat = 0;
    uint64_t st = 0xD1B54A32D192ED03ull ^ cfg;
    if (kind == PAT_EXHAUSTIVE) {
        /* all patterns of 1..max_erase erasures (k <= 64 here) */
        uint64_t lim = 1ull << k;
        for (uint64_t m = 1; m < lim; ++m) {
            int e = popcount64(m);
            if (e > max_erase)
                continue;
            uint64_t present[2] = {(~m) & (lim - 1), 0};
            erasure_rec rec;
            run_receiver(segs, k, fecs, nf, present, rows_only ? row_par : all_par, &rec, base_id);
            fwrite(&rec, sizeof(rec), 1, f);
            npat++;
        }
    } else {
        for (int p = 0; p < n_random; ++p) {
            int e = 1 + (int)oracle_xs_rand(&st, (uint32_t)max_erase - 1);
            uint64_t present[2] = {0, 0};
            for (uint32_t i = 0; i < k; ++i)
                present[i >> 6] |= 1ull << (i & 63);
            for (int q = 0; q < e; ++q) {
                uint32_t i = oracle_xs_rand(&st, k - 1);
                present[i >> 6] &= ~(1ull << (i & 63));
            }
            uint64_t pp = rows_only ? row_par : all_par;
            for (int l = 0; l < nf; ++l)
                if (oracle_xs_rand(&st, 999) < (uint32_t)(parity_loss * 1000))
                    pp &= ~(1ull << l);
            erasure_rec rec;
            run_receiver(segs, k, fecs, nf, present, pp, &rec, base_id);
            fwrite(&rec, sizeof(rec), 1, f);
            npat++;
        }
    }
    flex_fec_sender_release(snd, out);
    destroy_list(out);
    flex_fec_sender_destroy(snd);
    free_segments(segs, k);
    free_segments(work, k);
    fclose(f);
    char js[600];
    snprintf(js, sizeof(js),
             "{\"name\": \"%s\", \"kind\": \"erasures\", \"file\": \"%s\", \"config_id\": %llu, \"k\": %u, "
             "\"S\": %u, \"ragged\": %d, \"protect_fraction\": %u, \"rows_only\": %d, \"patterns\": %ld, "
             "\"parities\": %d}",
             name, fn, (unsigned long long)cfg, k, S, ragged, pf, rows_only, npat, nf);
    manifest_case(js);
}

/* ---- planner table: flex_fec_sender_num_packets for n<256, pf<256 ---------- */
static void planner_table(void)
{
    FILE* f = open_out("plan_table.bin");
    flex_fec_sender_t snd;
    for (int n = 0; n < 256; ++n)
        for (int pf = 0; pf < 256; ++pf) {
            memset(&snd, 0, sizeof(snd));
            snd.segs_count = (uint16_t)n;
            int rc = flex_fec_sender_num_packets(&snd, (uint8_t)pf);
            uint8_t rec[3] = {(uint8_t)rc, snd.row, snd.col};
            fwrite(rec, 1, 3, f);
        }
    fclose(f);
    manifest_case("{\"name\": \"plan_table\", \"kind\": \"plan_table\", \"file\": \"plan_table.bin\", "
                  "\"shape\": [256, 256, 3], \"fields\": [\"rc\", \"row\", \"col\"]}");
}

/* ---- single-call cases for the drop-in symbols ----------------------------- */
static void dump_seg(FILE* f, const char* key, const sim_segment_t* s, int with_data, int data_len)
{
    fprintf(f, "\"%s\": {\"packet_id\": %u, \"fid\": %u, \"timestamp\": %u, \"index\": %u, \"total\": %u, "
               "\"ftype\": %u, \"payload_type\": %u, \"data_size\": %u, \"fec_id\": %u",
            key, s->packet_id, s->fid, s->timestamp, s->index, s->total, s->ftype, s->payload_type,
            s->data_size, s->fec_id);
    if (with_data) {
        fprintf(f, ", \"data\": \"");
        for (int i = 0; i < data_len; ++i)
            fprintf(f, "%02x", s->data[i]);
        fprintf(f, "\"");
    }
    fprintf(f, "}");
}

static void dump_fec(FILE* f, const char* key, const sim_fec_t* p, int with_data)
{
    fprintf(f, "\"%s\": {\"seq\": %u, \"fid\": %u, \"ts\": %u, \"index\": %u, \"total\": %u, \"ftype\": %u, "
               "\"payload_type\": %u, \"size\": %u, \"fec_data_size\": %u",
            key, p->fec_meta.seq, p->fec_meta.fid, p->fec_meta.ts, p->fec_meta.index, p->fec_meta.total,
            p->fec_meta.ftype, p->fec_meta.payload_type, p->fec_meta.size, p->fec_data_size);
    if (with_data) {
        fprintf(f, ", \"data\": \"");
        for (int i = 0; i < p->fec_data_size && i < SIM_VIDEO_SIZE; ++i)
            fprintf(f, "%02x", p->fec_data[i]);
        fprintf(f, "\"");
    }
    fprintf(f, "}");
}

/* segment i of a small crafted set: sizes given, payload from a PRNG,
 * tails beyond data_size filled with 0xEE to expose the in-place padding */
static sim_segment_t* craft_seg(uint64_t* st, uint32_t id, uint16_t ds)
{
    sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t));
    s->packet_id = id;
    s->fid = id / 3;
    s->timestamp = id * 100;
    s->index = (uint16_t)(id % 7);
    s->total = 7;
    s->ftype = (uint8_t)(id & 1);
    s->payload_type = (uint8_t)(id % 3);
    s->fec_id = 0x5555;
    s->data_size = ds;
    for (int i = 0; i < SIM_VIDEO_SIZE; ++i)
        s->data[i] = (i < ds) ? (uint8_t)oracle_xs_next(st) : 0xEE;
    return s;
}

static void single_cases(void)
{
    FILE* f = open_out("single_cases.json");
    uint64_t st = 0x5EED5EED5EEDull;
    fprintf(f, "[\n");
    /* each case: sizes of the segments; generate over all, then recover
     * segment `drop` from the rest (when generate succeeded) */
    struct {
        const char* name;
        int n;
        uint16_t sizes[8];
        int drop;
        int corrupt; /* 0 none, 1 member bigger than fec_data_size, 2 meta.size > L */
    } cs[] = {
        {"gen_n0", 0, {0}, -1, 0},
        {"gen_n1", 1, {100}, -1, 0},
        {"ragged4", 4, {100, 37, 250, 1}, 1, 0},
        {"ragged6_drop0", 6, {1000, 999, 1, 500, 16, 17}, 0, 0},
        {"ragged3_droplast", 3, {5, 900, 33}, 2, 0},
        {"zero_sizes", 3, {0, 0, 0}, 1, 0},
        {"over_capacity", 3, {10, SIM_VIDEO_SIZE + 1, 20}, -1, 0},
        {"member_too_big", 4, {100, 200, 300, 50}, 0, 1},
        {"recovered_size_too_big", 4, {100, 200, 300, 50}, 2, 2},
        {"full_10", 4, {1000, 1000, 1000, 1000}, 3, 0},
    };
    int ncs = (int)(sizeof(cs) / sizeof(cs[0]));
    for (int c = 0; c < ncs; ++c) {
        sim_segment_t* segs[8];
        for (int i = 0; i < cs[c].n; ++i)
            segs[i] = craft_seg(&st, 1000 + 10 * c + i, cs[c].sizes[i]);
        /* inputs as given (before the call mutates tails) */
        fprintf(f, "%s{\"name\": \"%s\", \"n\": %d, \"inputs\": [", c ? ",\n" : "", cs[c].name, cs[c].n);
        for (int i = 0; i < cs[c].n; ++i) {
            if (i)
                fprintf(f, ", ");
            fprintf(f, "{");
            dump_seg(f, "seg", segs[i], 1, SIM_VIDEO_SIZE);
            fprintf(f, "}");
        }
        fprintf(f, "], ");
        sim_fec_t* fec = (sim_fec_t*)malloc(sizeof(sim_fec_t));
        memset(fec, 0xCD, sizeof(*fec));
        fec->fec_id = 77;
        int rc = flex_fec_generate(segs, cs[c].n, fec);
        fprintf(f, "\"generate_rc\": %d, ", rc);
        if (rc == 0 || cs[c].n > 1) {
            dump_fec(f, "fec", fec, rc == 0);
            fprintf(f, ", ");
        }
        /* inputs after generate (in-place zero padding of segs[1..]) */
        fprintf(f, "\"after_generate\": [");
        for (int i = 0; i < cs[c].n; ++i)
            fprintf(f, "%s\"%016llx\"", i ? ", " : "",
                    (unsigned long long)fnv1a(0xcbf29ce484222325ull, segs[i]->data, SIM_VIDEO_SIZE));
        fprintf(f, "]");
        if (rc == 0 && cs[c].drop >= 0) {
            if (cs[c].corrupt == 1) {
                segs[1]->data_size = (uint16_t)(fec->fec_data_size + 1);
            } else if (cs[c].corrupt == 2) {
                fec->fec_meta.size ^= 0x7000;
            }
            sim_segment_t* rest[8];
            int nr = 0;
            for (int i = 0; i < cs[c].n; ++i)
                if (i != cs[c].drop)
                    rest[nr++] = segs[i];
            sim_segment_t* out = (sim_segment_t*)malloc(sizeof(sim_segment_t));
            memset(out, 0xAB, sizeof(*out));
            int rr = flex_fec_recover(rest, nr, fec, out);
            fprintf(f, ", \"drop\": %d, \"corrupt\": %d, \"recover_rc\": %d", cs[c].drop, cs[c].corrupt, rr);
            if (cs[c].corrupt == 2)
                fprintf(f, ", \"meta_size_xor\": %d", 0x7000);
            if (rr == 0) {
                fprintf(f, ", ");
                dump_seg(f, "recovered", out, 1, fec->fec_data_size);
            }
            fprintf(f, ", \"after_recover\": [");
            for (int i = 0; i < nr; ++i)
                fprintf(f, "%s\"%016llx\"", i ? ", " : "",
                        (unsigned long long)fnv1a(0xcbf29ce484222325ull, rest[i]->data, SIM_VIDEO_SIZE));
            fprintf(f, "]");
            free(out);
        }
        /* recover with zero present segments */
        if (c == 2) {
            sim_segment_t out;
            int r0 = flex_fec_recover(segs, 0, fec, &out);
            fprintf(f, ", \"recover_n0_rc\": %d", r0);
        }
        fprintf(f, "}");
        free(fec);
        for (int i = 0; i < cs[c].n; ++i)
            free(segs[i]);
    }
    fprintf(f, "\n]\n");
    fclose(f);
    manifest_case("{\"name\": \"single_cases\", \"kind\": \"single\", \"file\": \"single_cases.json\"}");
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s <outdir>\n", argv[0]);
        return 2;
    }
    g_outdir = argv[1];
    g_manifest = open_out("manifest.json");
    fprintf(g_manifest, "{\"generator\": \"oracle/gen_golden.c\", \"sim_video_size\": %d, "
                        "\"seed\": \"0x52415A4F52464543 ^ config_id\", \"record_bytes\": {\"parity\": %zu, "
                        "\"erasure\": %zu}, \"cases\": [\n",
            SIM_VIDEO_SIZE, sizeof(parity_rec), sizeof(erasure_rec));

    planner_table();
    single_cases();
    /* encode: reference sender (flex_fec_sender_update) */
    case_sender("k10_pf80_S1000", 2, 16, 10, 1000, 0, 80);
    case_sender("k10_pf80_S1000_ragged", 3, 16, 10, 1000, 1, 80);
    case_sender("k10_pf5_S1000", 4, 8, 10, 1000, 0, 5);   /* strip mode, 1 parity */
    case_sender("k21_pf80_S104", 5, 8, 21, 104, 1, 80);   /* test_flex_sender shape: 9 parities */
    case_sender("k25_pf80_S256", 6, 8, 25, 256, 1, 80);   /* test_flex_receiver shape: 10 parities */
    case_sender("k100_pf200_S512", 7, 4, 100, 512, 1, 200);
    /* groups above the batched recovery's 128 segments, through the reference sender; the group-level
     * drop-in's large-group paths (one launch up to 255 segments, line by line above) */
    case_sender_kind("k200_pf10_S104", "sender_large", 71, 2, 200, 104, 1, 10);   /* 14 x 15 matrix, 29 lines */
    case_sender_kind("k200_pf5_S104", "sender_large", 72, 2, 200, 104, 1, 5);     /* strip: 4 rows of 50 */
    case_sender_kind("k300_pf10_S64", "sender_large", 73, 1, 300, 64, 1, 10);     /* 17 x 18 matrix */
    case_sender_kind("k1100_pf255_S64", "sender_large", 74, 1, 1100, 64, 1, 255); /* 55 x 20 matrix, 75 lines */
    /* strip mode with col truncated by the uint8_t field: 275 -> 19, 58 rows of 19 */
    case_sender_kind("k1100_pf1_S64", "sender_large", 75, 1, 1100, 64, 1, 1);
    case_sender_random("random_k", 8, 64, 328);
    /* encode: explicit rows (config 5 shape, and 1200-B payloads in 600-B windows) */
    case_rows("k32_rows4_S256", 9, 16, 32, 256, 0, 4, 256);
    case_rows("k10_rows4_S1200", 10, 8, 10, 1200, 0, 4, 600);
    case_rows("k10_rows4_S1200_ragged", 11, 8, 10, 1200, 1, 4, 600);
    /* erasures: reference receiver */
    case_erasures("k10_full_le3", 12, 10, 1000, 0, 80, 0, PAT_EXHAUSTIVE, 3, 0, 0.0);
    case_erasures("k10_rows_le3", 12, 10, 1000, 0, 80, 1, PAT_EXHAUSTIVE, 3, 0, 0.0);
    case_erasures("k10_full_ragged_le4", 13, 10, 1000, 1, 80, 0, PAT_EXHAUSTIVE, 4, 0, 0.0);
    case_erasures("k25_random", 14, 25, 256, 1, 80, 0, PAT_RANDOM, 8, 400, 0.2);
    case_erasures("k64_random", 15, 64, 128, 1, 120, 0, PAT_RANDOM, 12, 300, 0.15);
    case_erasures("k100_random", 16, 100, 64, 1, 255, 0, PAT_RANDOM, 16, 200, 0.1);
    /* plans whose lines are pairwise disjoint: strip mode (k < 6 or pf < 10)
     * and row parities only, the latter also replayed against a rows-only plan */
    case_erasures("k5_strip_le3", 17, 5, 1000, 1, 80, 0, PAT_EXHAUSTIVE, 3, 0, 0.0);
    case_erasures("k5_strip_pf200_le3", 18, 5, 1000, 1, 200, 0, PAT_EXHAUSTIVE, 3, 0, 0.0);
    case_erasures("k40_strip_random", 19, 40, 256, 1, 8, 0, PAT_RANDOM, 4, 200, 0.1);
    case_erasures("k10_rows_ragged_le4", 13, 10, 1000, 1, 80, 1, PAT_EXHAUSTIVE, 4, 0, 0.0);
    case_erasures("k16_rows_random", 20, 16, 512, 1, 80, 1, PAT_RANDOM, 8, 300, 0.2);
    case_erasures("k24_rows_random", 21, 24, 512, 1, 80, 1, PAT_RANDOM, 8, 300, 0.2);

    fprintf(g_manifest, "\n]}\n");
    fclose(g_manifest);
    free(g_shards);
    free(g_hdrs);
    return 0;
}
