/*
 * gen_full.c -- full-size golden digests (own code, TEST INFRASTRUCTURE ONLY).
 * Links the reference's flex_fec_generate (flex_fec_xor.c:4-53) compiled out
 * of tree (oracle/Makefile) and digests its outputs over the BASELINE.json
 * batch sizes, so the GPU tests can check every group of a full-size batch,
 * not a sample.  Inputs are regenerated from the PRNG spec (oracle_fill_stream,
 * SURVEY.md §8d); nothing but the digests is stored.
 *
 * Digest = SHA-256 over the groups in order, each group contributing
 *   parity [n][stride] | meta [n] (20-B rfec_hdr) | fec_data_size [n] (u16 LE)
 * i.e. the bytes of rfec_encode_batch's outputs for that group.
 *
 * Payloads wider than the reference's SIM_VIDEO_SIZE (1000) are computed in
 * windows of `span` bytes (XOR is bytewise: window w of the parity is the
 * reference's parity of window w of the members).  For those configs the
 * meta.size field (XOR of the members' data_size) is restated here, since the
 * reference only saw window sizes; it is pinned at S <= 1000 by every other
 * fixture.  The same digests are recomputed through the oracle's batched
 * restatement and must agree.
 *
 * Usage: gen_full <out.json>
 */
#include "flex_fec_xor.h"
#include "razor_fec.h" /* rfec_plan / rfec_hdr (its sim types yield to the reference's) */
#include "sha256.h"

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_fill_stream(uint64_t config_id, uint64_t state[2], uint32_t g0, uint32_t groups, uint32_t k,
                        uint32_t S, uint32_t stride, int ragged, uint8_t* shards, rfec_hdr* hdr);
int oracle_plan_from_fraction(int k, int protect_fraction, unsigned layers, rfec_plan* plan);
int oracle_plan_matrix(int k, int row, int col, unsigned layers, rfec_plan* plan);
void oracle_encode_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                         const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                         uint16_t* fec_size, int8_t* status);

typedef struct {
    const char* name;
    uint64_t cfg;
    uint32_t G, k, S;
    int ragged;
    int matrix; /* 0: plan_from_fraction(k, pf, layers); 1: plan_matrix(k, row, col, layers) */
    int pf, row, col;
    unsigned layers;
    uint32_t chunk; /* > 0: also a digest of every `chunk` groups (the weak-scaling ranks' slices) */
} full_case;

enum { CHUNK = 4096 };

static void meta_out(const sim_fec_meta_t* m, rfec_hdr* h)
{
    h->seq = m->seq;
    h->fid = m->fid;
    h->ts = m->ts;
    h->index = m->index;
    h->total = m->total;
    h->ftype = m->ftype;
    h->payload_type = m->payload_type;
    h->size = m->size;
}

static void digest_group(sha256_ctx* c, const uint8_t* par, const rfec_hdr* meta, const uint16_t* fs, uint32_t n,
                         uint32_t stride)
{
    sha256_update(c, par, (size_t)n * stride);
    sha256_update(c, meta, (size_t)n * sizeof(rfec_hdr));
    sha256_update(c, fs, (size_t)n * sizeof(uint16_t));
}

static void run_case(FILE* js, const full_case* fc, int first)
{
    const uint32_t k = fc->k, S = fc->S, stride = (S + 15) & ~15u;
    const uint32_t span = S <= SIM_VIDEO_SIZE ? S : 600;
    rfec_plan plan;
    int rc = fc->matrix ? oracle_plan_matrix((int)k, fc->row, fc->col, fc->layers, &plan)
                        : oracle_plan_from_fraction((int)k, fc->pf, fc->layers, &plan);
    assert(rc == 0 && plan.n_lines > 0);
    const uint32_t n = plan.n_lines;
    uint8_t* shards = (uint8_t*)malloc((size_t)CHUNK * k * stride);
    rfec_hdr* hdr = (rfec_hdr*)malloc((size_t)CHUNK * k * sizeof(rfec_hdr));
    uint8_t* par = (uint8_t*)malloc((size_t)n * stride);
    uint8_t* opar = (uint8_t*)malloc((size_t)CHUNK * n * stride);
    rfec_hdr* ometa = (rfec_hdr*)malloc((size_t)CHUNK * n * sizeof(rfec_hdr));
    uint16_t* ofs = (uint16_t*)malloc((size_t)CHUNK * n * sizeof(uint16_t));
    int8_t* ost = (int8_t*)malloc((size_t)CHUNK * n);
    sim_segment_t* seg = (sim_segment_t*)calloc(k, sizeof(sim_segment_t));
    sim_fec_t* fec = (sim_fec_t*)calloc(1, sizeof(sim_fec_t));
    sim_segment_t* mem[RFEC_MAX_K];
    rfec_hdr meta[RFEC_MAX_LINES];
    uint16_t fs[RFEC_MAX_LINES];
    sha256_ctx cref, cora;
    sha256_init(&cref);
    sha256_init(&cora);
    /* per-rank slice digests for the multi-GPU split (razor_amd/dist.py
     * shard_groups: rank r of N owns [G*r/N, G*(r+1)/N)), config 4 only */
    static const uint32_t NS[3] = {2, 4, 8};
    const int slices = fc->cfg == 4;
    sha256_ctx cs[3][8];
    uint32_t cur[3] = {0, 0, 0};
    if (slices)
        for (int a = 0; a < 3; ++a)
            sha256_init(&cs[a][0]);
    /* weak scaling (bench.py at N > 1): rank r runs groups [r * chunk, (r + 1) * chunk) */
    const uint32_t nchunks = fc->chunk ? fc->G / fc->chunk : 0;
    sha256_ctx* cc = nchunks ? (sha256_ctx*)malloc(sizeof(sha256_ctx) * nchunks) : NULL;
    for (uint32_t c = 0; c < nchunks; ++c)
        sha256_init(&cc[c]);
    uint64_t state[2] = {0, 0};
    for (uint32_t g0 = 0; g0 < fc->G; g0 += CHUNK) {
        const uint32_t ng = fc->G - g0 < CHUNK ? fc->G - g0 : CHUNK;
        oracle_fill_stream(fc->cfg, state, g0, ng, k, S, stride, fc->ragged, shards, hdr);
        for (uint32_t gl = 0; gl < ng; ++gl) {
            memset(par, 0, (size_t)n * stride);
            for (uint32_t l = 0; l < n; ++l) {
                const rfec_line ln = plan.line[l];
                uint32_t L = 0;
                for (uint32_t off = 0; off < S; off += span) {
                    for (uint32_t q = 0; q < ln.count; ++q) {
                        const uint32_t i = ln.first + q * ln.stride;
                        const rfec_hdr* h = &hdr[(size_t)gl * k + i];
                        sim_segment_t* s = &seg[q];
                        s->packet_id = h->seq;
                        s->fid = h->fid;
                        s->timestamp = h->ts;
                        s->index = h->index;
                        s->total = h->total;
                        s->ftype = h->ftype;
                        s->payload_type = h->payload_type;
                        int ds = (int)h->size - (int)off;
                        ds = ds < 0 ? 0 : (ds > (int)span ? (int)span : ds);
                        s->data_size = (uint16_t)ds;
                        memcpy(s->data, shards + ((size_t)gl * k + i) * stride + off, (size_t)ds);
                        mem[q] = s;
                    }
                    memset(fec, 0, sizeof(*fec));
                    rc = flex_fec_generate(mem, (int)ln.count, fec);
                    assert(rc == 0);
                    memcpy(par + (size_t)l * stride + off, fec->fec_data, fec->fec_data_size);
                    L += fec->fec_data_size;
                    if (off == 0)
                        meta_out(&fec->fec_meta, &meta[l]);
                }
                if (span < S) { /* restated: XOR of data_size (flex_fec_xor.c:20, :44) */
                    uint16_t x = 0;
                    for (uint32_t q = 0; q < ln.count; ++q)
                        x ^= hdr[(size_t)gl * k + ln.first + q * ln.stride].size;
                    meta[l].size = x;
                }
                fs[l] = (uint16_t)L;
            }
            digest_group(&cref, par, meta, fs, n, stride);
            if (nchunks)
                digest_group(&cc[(g0 + gl) / fc->chunk], par, meta, fs, n, stride);
            for (int a = 0; slices && a < 3; ++a) {
                const uint64_t g = (uint64_t)g0 + gl;
                while (g >= (uint64_t)fc->G * (cur[a] + 1) / NS[a])
                    sha256_init(&cs[a][++cur[a]]);
                digest_group(&cs[a][cur[a]], par, meta, fs, n, stride);
            }
        }
        oracle_encode_batch(&plan, ng, stride, S, shards, hdr, opar, ometa, ofs, ost);
        for (uint32_t gl = 0; gl < ng; ++gl) {
            for (uint32_t l = 0; l < n; ++l)
                assert(ost[(size_t)gl * n + l] == 0);
            digest_group(&cora, opar + (size_t)gl * n * stride, ometa + (size_t)gl * n, ofs + (size_t)gl * n, n,
                         stride);
        }
    }
    uint8_t d1[32], d2[32];
    char h1[65], h2[65];
    sha256_final(&cref, d1);
    sha256_final(&cora, d2);
    sha256_hex(d1, h1);
    sha256_hex(d2, h2);
    fprintf(stderr, "%-32s ref %s oracle %s\n", fc->name, h1, h2);
    if (strcmp(h1, h2) != 0) {
        fprintf(stderr, "oracle disagrees with the reference on %s\n", fc->name);
        exit(1);
    }
    fprintf(js,
            "%s  {\"name\": \"%s\", \"config_id\": %llu, \"groups\": %u, \"k\": %u, \"S\": %u, \"stride\": %u, "
            "\"ragged\": %d, \"plan\": \"%s\", \"pf\": %d, \"row\": %d, \"col\": %d, \"layers\": %u, "
            "\"n_lines\": %u, \"window\": %u, \"sha256\": \"%s\"",
            first ? "" : ",\n", fc->name, (unsigned long long)fc->cfg, fc->G, k, S, stride, fc->ragged,
            fc->matrix ? "matrix" : "fraction", fc->pf, fc->row, fc->col, fc->layers, n, span, h1);
    if (nchunks) {
        fprintf(js, ", \"chunk\": %u, \"chunks\": [", fc->chunk);
        for (uint32_t c = 0; c < nchunks; ++c) {
            uint8_t d[32];
            char hx[65];
            sha256_final(&cc[c], d);
            sha256_hex(d, hx);
            fprintf(js, "%s\"%s\"", c ? ", " : "", hx);
        }
        fprintf(js, "]");
        free(cc);
    }
    if (slices) {
        fprintf(js, ", \"slices\": {");
        for (int a = 0; a < 3; ++a) {
            fprintf(js, "%s\"%u\": [", a ? ", " : "", NS[a]);
            for (uint32_t r = 0; r < NS[a]; ++r) {
                uint8_t d[32];
                char hx[65];
                sha256_final(&cs[a][r], d);
                sha256_hex(d, hx);
                fprintf(js, "%s\"%s\"", r ? ", " : "", hx);
            }
            fprintf(js, "]");
        }
        fprintf(js, "}");
    }
    fprintf(js, "}");
    free(shards);
    free(hdr);
    free(par);
    free(opar);
    free(ometa);
    free(ofs);
    free(ost);
    free(seg);
    free(fec);
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: gen_full <out.json>\n");
        return 2;
    }
    /* BASELINE.json configs 2-5 plus a ragged full-plan batch */
    static const full_case cases[] = {
        {"c2_k10_rows_S1200_G65536", 2, 65536, 10, 1200, 0, 0, 80, 0, 0, RFEC_LAYER_ROWS},
        {"c3_k10_full_S1200_G65536", 3, 65536, 10, 1200, 0, 0, 80, 0, 0, RFEC_LAYER_ROWS | RFEC_LAYER_COLS},
        {"c4_k10_rows_S1200_G1048576", 4, 1048576, 10, 1200, 0, 0, 80, 0, 0, RFEC_LAYER_ROWS},
        {"c5_k32_rows4_S256_G65536", 5, 65536, 32, 256, 0, 1, 0, 8, 4, RFEC_LAYER_ROWS},
        {"k10_full_ragged_S1000_G65536", 6, 65536, 10, 1000, 1, 0, 80, 0, 0, RFEC_LAYER_ROWS | RFEC_LAYER_COLS},
        /* the c3 stream continued: the weak-scaling ranks' slices of 65,536 groups, N <= 8 */
        {"c3_weak_k10_rows_S1200_G524288", 2, 524288, 10, 1200, 0, 0, 80, 0, 0, RFEC_LAYER_ROWS, 65536},
    };
    FILE* js = fopen(argv[1], "w");
    if (!js) {
        perror(argv[1]);
        return 1;
    }
    fprintf(js, "{\"digest\": \"sha256 over groups of parity[n][stride] | meta[n] (20 B) | fec_data_size[n] (u16)\",\n"
                " \"generator\": \"oracle/gen_full.c (reference flex_fec_generate, out-of-tree build)\",\n"
                " \"cases\": [\n");
    for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i)
        run_case(js, &cases[i], i == 0);
    fprintf(js, "\n]}\n");
    fclose(js);
    return 0;
}
