/*
 * gen_stage.c -- sender-staging golden vectors (own code, TEST INFRASTRUCTURE
 * ONLY).  Links the reference's flex_fec_sender.c / flex_fec_xor.c compiled
 * out of tree (oracle/Makefile) and replays sim_sender_put's segment
 * construction (sim_sender.c:306-377; its static sim_split_frame :254-284 is
 * restated here) over scripted frame sequences, letting the reference flex
 * sender decide the grouping and emit the parities.  Writes
 * tests/golden/stage.json: per scenario the frames, every segment's stamps and
 * group, every group's fec_id / base_id / count / shape and each parity's
 * index, meta, fec_data_size and FNV-1a hash of fec_data[0:size).
 *
 * Frame bytes: per frame, the xorshift64* stream (oracle_xs_next, seed
 * 0x5354414745 ^ scenario, continuing across frames), 8 little-endian bytes
 * per step, the last step of a frame truncated.
 * The reference reads the wall clock; every scenario runs in well under the
 * 500 ms FEC window, so only the segment-count rules fire (the restatements
 * are driven with one constant now_ms > 500 to match).
 *
 * Usage: gen_stage <out.json>
 */
#include "flex_fec_sender.h"

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t oracle_xs_next(uint64_t* state);
uint32_t oracle_xs_rand(uint64_t* state, uint32_t t);

typedef struct {
    uint32_t size;
    uint8_t ftype, payload_type, pf;
} frame_t;

static uint64_t fnv1a(const uint8_t* p, size_t n, uint64_t h)
{
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

static FILE* js;
static int first_case = 1;

static void scenario(const char* name, uint64_t id, const frame_t* frames, int nf)
{
    uint64_t st = 0x5354414745ull ^ id;
    flex_fec_sender_t* flex = flex_fec_sender_create();
    uint32_t pid = 0, sid = 0, fid = 0;
    enum { MAXS = 8192 };
    static sim_segment_t* segs[MAXS];
    static int seg_group[MAXS];
    int ns = 0, ngroups = 0;
    char* gbuf = (char*)malloc(1 << 22);
    size_t gl = 0;
    base_list_t* out = create_list();
    fprintf(js, "%s  {\"name\": \"%s\", \"id\": %llu, \"seg_size\": %d, \"frames\": [", first_case ? "" : ",\n", name,
            (unsigned long long)id, SIM_VIDEO_SIZE);
    first_case = 0;
    for (int f = 0; f < nf; ++f)
        fprintf(js, "%s[%u, %u, %u, %u]", f ? ", " : "", frames[f].size, frames[f].ftype, frames[f].payload_type,
                frames[f].pf);
    fprintf(js, "],\n   \"groups\": [");
    for (int f = 0; f < nf; ++f) {
        const frame_t* fr = &frames[f];
        static uint8_t fbuf[200 * SIM_VIDEO_SIZE];
        assert(fr->size <= sizeof(fbuf));
        for (uint32_t b = 0; b < fr->size; b += 8) {
            uint64_t v = oracle_xs_next(&st);
            for (uint32_t q = 0; q < 8 && b + q < fr->size; ++q)
                fbuf[b + q] = (uint8_t)(v >> (8 * q));
        }
        uint32_t off = 0;
        /* sim_split_frame, sim_sender.c:254-284 */
        uint32_t total = fr->size <= SIM_VIDEO_SIZE ? 1 : (fr->size + SIM_VIDEO_SIZE - 1) / SIM_VIDEO_SIZE;
        ++fid;
        for (uint32_t i = 0; i < total; ++i) {
            assert(ns < MAXS);
            sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t));
            s->packet_id = ++pid; /* sim_sender.c:344-362 */
            s->send_id = ++sid;
            s->fid = fid;
            s->timestamp = 0;
            s->ftype = fr->ftype;
            s->payload_type = fr->payload_type;
            s->index = (uint16_t)i;
            s->total = (uint16_t)total;
            s->remb = 1;
            s->data_size = (uint16_t)(fr->size <= SIM_VIDEO_SIZE
                                          ? fr->size
                                          : fr->size / total + (i < fr->size % total ? 1 : 0));
            memcpy(s->data, fbuf + off, s->data_size);
            off += s->data_size;
            s->fec_id = flex->fec_id;
            flex_fec_sender_add_segment(flex, s);
            seg_group[ns] = -2;
            segs[ns++] = s;
            for (int pass = 0; pass < 2; ++pass) {
                /* sim_sender.c:370-371 (>= 100 segments) and :373-374 (frame end) */
                if (pass == 0 ? flex->segs_count < 100 : i + 1 < total)
                    continue;
                const int k = flex->segs_count;
                const uint16_t fec_id = flex->fec_id;
                const uint32_t base_id = flex->base_id;
                list_clear(out);
                flex_fec_sender_update(flex, fr->pf, out);
                const int emitted = list_size(out);
                if (k > 0 && flex->segs_count == 0) { /* it fired: the last k segments were the group */
                    for (int q = ns - k; q < ns; ++q)
                        seg_group[q] = emitted ? ngroups : -1;
                }
                if (emitted) {
                    gl += (size_t)sprintf(gbuf + gl,
                                          "%s\n    {\"fec_id\": %u, \"base_id\": %u, \"count\": %d, \"first_seg\": %d, "
                                          "\"send_id0\": %u, \"parities\": [",
                                          ngroups ? "," : "", fec_id, base_id, k, ns - k, sid + 1);
                    base_list_unit_t* it;
                    int pi = 0;
                    LIST_FOREACH(out, it)
                    {
                        sim_fec_t* p = (sim_fec_t*)it->pdata;
                        const sim_fec_meta_t* m = &p->fec_meta;
                        gl += (size_t)sprintf(
                            gbuf + gl,
                            "%s[%u, %u, %u, %u, %u, %u, %u, %u, %u, %u, %u, %u, %u, \"%016llx\"]", pi ? ", " : "",
                            p->index, p->row, p->col, p->count, m->seq, m->fid, m->ts, m->index, m->total, m->ftype,
                            m->payload_type, m->size, p->fec_data_size,
                            (unsigned long long)fnv1a(p->fec_data, p->fec_data_size, 0xCBF29CE484222325ull));
                        pi++;
                    }
                    sid += (uint32_t)emitted; /* sim_sender_fec: one send id per parity (sim_sender.c:295-296) */
                    gl += (size_t)sprintf(gbuf + gl, "]}");
                    ngroups++;
                    flex_fec_sender_release(flex, out);
                }
            }
        }
    }
    fwrite(gbuf, 1, gl, js);
    fprintf(js, "],\n   \"open_fec_id\": %u, \"open_count\": %u,\n   \"segments\": [", flex->fec_id,
            flex->segs_count);
    for (int q = 0; q < ns; ++q) {
        const sim_segment_t* s = segs[q];
        fprintf(js, "%s[%u, %u, %u, %u, %u, %u, %u, %d]", q ? ", " : "", s->packet_id, s->send_id, s->fid, s->index,
                s->total, s->data_size, s->fec_id, seg_group[q]);
    }
    fprintf(js, "]}");
    for (int q = 0; q < ns; ++q)
        free(segs[q]);
    destroy_list(out);
    flex_fec_sender_destroy(flex);
    free(gbuf);
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: gen_stage <out.json>\n");
        return 2;
    }
    js = fopen(argv[1], "w");
    if (!js) {
        perror(argv[1]);
        return 1;
    }
    fprintf(js, "{\"generator\": \"oracle/gen_stage.c (reference flex_fec_sender + flex_fec_xor)\",\n"
                " \"frame_bytes\": \"xorshift64* from 0x5354414745 ^ id across frames, 8 LE bytes per step, last step of a frame truncated\",\n"
                " \"segment\": [\"packet_id\", \"send_id\", \"fid\", \"index\", \"total\", \"data_size\", \"fec_id\", \"group\"],\n"
                " \"parity\": [\"index\", \"row\", \"col\", \"count\", \"seq\", \"fid\", \"ts\", \"m_index\", \"m_total\", "
                "\"ftype\", \"payload_type\", \"m_size\", \"fec_data_size\", \"fnv1a\"],\n"
                " \"scenarios\": [\n");
    enum { N = 200 };
    static frame_t fr[N];
    /* 1: steady 10-segment frames (the bench shape), pf 80 */
    for (int i = 0; i < 40; ++i)
        fr[i] = (frame_t){10u * SIM_VIDEO_SIZE, (uint8_t)(i % 30 == 0), 96, 80};
    scenario("steady_k10_pf80", 1, fr, 40);
    /* 2: mixed sizes: small frames accumulate across frames, > 100 segments
     * flush mid-frame, exactly 100 then an empty frame-end update */
    uint64_t r = 0xC0FFEEull;
    int n = 0;
    const uint32_t sizes[] = {1, 999, 1000, 1001, 2500, 5 * SIM_VIDEO_SIZE, 6 * SIM_VIDEO_SIZE - 7,
                              100 * SIM_VIDEO_SIZE, 150 * SIM_VIDEO_SIZE + 3, 37 * SIM_VIDEO_SIZE + 11};
    for (int i = 0; i < 10; ++i)
        fr[n++] = (frame_t){sizes[i], (uint8_t)(i == 0), 100, 80};
    for (int i = 0; i < 60; ++i) {
        uint32_t segs = 1 + oracle_xs_rand(&r, i % 7 == 0 ? 130 : 12);
        fr[n++] = (frame_t){segs * SIM_VIDEO_SIZE - oracle_xs_rand(&r, SIM_VIDEO_SIZE - 1), (uint8_t)(i % 25 == 0),
                            (uint8_t)oracle_xs_rand(&r, 255), (uint8_t)oracle_xs_rand(&r, 255)};
    }
    scenario("mixed", 2, fr, n);
    /* 3: protect fractions that give no parity (pf 0), strip mode, tiny groups */
    n = 0;
    const uint8_t pfs[] = {0, 1, 5, 9, 10, 40, 128, 255};
    for (int i = 0; i < 48; ++i)
        fr[n++] = (frame_t){(1 + (uint32_t)(i % 9)) * SIM_VIDEO_SIZE / 2 + 17, 0, 7, pfs[i % 8]};
    scenario("fractions", 3, fr, n);
    fprintf(js, "\n]}\n");
    fclose(js);
    return 0;
}
