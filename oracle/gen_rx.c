/*
 * gen_rx.c -- receiver-ingestion golden vectors (own code, TEST
 * INFRASTRUCTURE ONLY).  Links the reference's sim_fec.c, flex_fec_receiver.c,
 * flex_fec_sender.c and flex_fec_xor.c compiled out of tree (oracle/Makefile)
 * and runs the reference receiver-side FEC on scripted, lossy, reordered
 * packet streams:
 *
 *   sender   sim_sender_put's segments (sim_sender.c:306-377, split restated)
 *            grouped by the reference flex sender (flex_fec_sender.c)
 *   network  drops, reordering within a window, duplicates, late parities
 *   receiver sim_fec_put_segment / sim_fec_put_fec_packet (sim_fec.c:141-207)
 *            with the recovery cascade of sim_receiver_recover
 *            (sim_receiver.c:780-804): recovered packets drained lowest
 *            packet_id first, re-fed unless already in the receiver; with
 *            evict_every > 0, sim_fec_evict (sim_fec.c:209-241) after every
 *            evict_every arrivals, as the session heartbeat's
 *            sim_receiver_timer calls it (sim_receiver.c:880), its 300 ms
 *            wall-clock gate always open
 *
 * Writes tests/golden/rx.json: per scenario the frames, the sender's groups,
 * the arrival sequence and the packets the receiver recovered, in delivery
 * order (header fields + FNV-1a of the data).  Frame bytes follow
 * gen_stage.c's stream (seed 0x5354414745 ^ id); segment timestamps are
 * 33 ms per frame, a parity's send_ts the timestamp of the frame that closed
 * its group.
 *
 * Usage: gen_rx <out.json>
 */
#include "sim_internal.h"

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t oracle_xs_next(uint64_t* state);
uint32_t oracle_xs_rand(uint64_t* state, uint32_t t);

static uint64_t fnv1a(const uint8_t* p, size_t n, uint64_t h)
{
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

typedef struct {
    uint32_t size;
    uint8_t ftype, payload_type, pf;
} frame_t;

typedef struct {
    int kind;      /* 0 segment, 1 parity */
    int idx;       /* segment index, or parity index */
    uint64_t key;  /* arrival order key */
    int dup;
} arrival_t;

static int cmp_arrival(const void* a, const void* b)
{
    const arrival_t *x = (const arrival_t*)a, *y = (const arrival_t*)b;
    return x->key < y->key ? -1 : x->key > y->key;
}

enum { MAXS = 16384, MAXP = 8192 };
static sim_segment_t* segs[MAXS];
static sim_fec_t* fecs[MAXP];
static int fec_group[MAXP];
static uint8_t seen[1 << 20]; /* packet ids already in the receiver (received or recovered) */

static FILE* js;
static int first_case = 1;
/* the sender closes a group at this many segments (sim_sender.c:370: 100);
 * a foreign peer's sender may close them later */
static int g_flush_at = 100;

static void scenario_x(const char* name, uint64_t id, const frame_t* frames, int nf, uint32_t seg_loss_pm,
                       uint32_t fec_loss_pm, uint32_t window, uint32_t dup_pm, uint32_t late_pm, int protect_tail,
                       uint32_t late_seg_pm, int evict_every)
{
    uint64_t st = 0x5354414745ull ^ id, rs = 0x52585258ull ^ id;
    flex_fec_sender_t* flex = flex_fec_sender_create();
    uint32_t pid = 0, fid = 0;
    int ns = 0, np = 0, ng = 0;
    base_list_t* out = create_list();
    /* sender order: segments, each group's parities right after its closing segment */
    static arrival_t order[MAXS + MAXP];
    int no = 0;
    fprintf(js, "%s  {\"name\": \"%s\", \"id\": %llu, ", first_case ? "" : ",\n", name, (unsigned long long)id);
    if (g_flush_at != 100)
        fprintf(js, "\"flush_at\": %d, ", g_flush_at);
    fprintf(js, "\"frames\": [");
    first_case = 0;
    for (int f = 0; f < nf; ++f)
        fprintf(js, "%s[%u, %u, %u, %u]", f ? ", " : "", frames[f].size, frames[f].ftype, frames[f].payload_type,
                frames[f].pf);
    fprintf(js, "],\n   \"groups\": [");
    for (int f = 0; f < nf; ++f) {
        const frame_t* fr = &frames[f];
        static uint8_t fbuf[1100 * SIM_VIDEO_SIZE];
        for (uint32_t b = 0; b < fr->size; b += 8) {
            uint64_t v = oracle_xs_next(&st);
            for (uint32_t q = 0; q < 8 && b + q < fr->size; ++q)
                fbuf[b + q] = (uint8_t)(v >> (8 * q));
        }
        uint32_t total = fr->size <= SIM_VIDEO_SIZE ? 1 : (fr->size + SIM_VIDEO_SIZE - 1) / SIM_VIDEO_SIZE;
        uint32_t off = 0;
        ++fid;
        for (uint32_t i = 0; i < total; ++i) {
            assert(ns < MAXS);
            sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t));
            s->packet_id = ++pid;
            s->fid = fid;
            s->timestamp = 33u * (uint32_t)f;
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
            segs[ns] = s;
            order[no++] = (arrival_t){0, ns, 0, 0};
            ns++;
            for (int pass = 0; pass < 2; ++pass) {
                if (pass == 0 ? flex->segs_count < g_flush_at : i + 1 < total)
                    continue;
                const uint16_t gid = flex->fec_id;
                const uint32_t base = flex->base_id;
                const int k = flex->segs_count;
                list_clear(out);
                flex_fec_sender_update(flex, fr->pf, out);
                if (list_size(out) == 0)
                    continue;
                fprintf(js, "%s[%u, %u, %d, %u]", ng ? ", " : "", gid, base, k, fr->pf);
                base_list_unit_t* it;
                LIST_FOREACH(out, it)
                {
                    assert(np < MAXP);
                    sim_fec_t* p = (sim_fec_t*)it->pdata;
                    p->send_ts = 33u * (uint32_t)f; /* sim_sender_fec stamps send_ts (sim_sender.c:299) */
                    fecs[np] = p;
                    fec_group[np] = ng;
                    order[no++] = (arrival_t){1, np, 0, 0};
                    np++;
                }
                list_clear(out); /* the parities are owned by fecs[] now */
                ng++;
            }
        }
    }
    /* network: loss, jitter within `window`, duplicates, late parities */
    static arrival_t arr[2 * (MAXS + MAXP)];
    int na = 0;
    for (int q = 0; q < no; ++q) {
        const arrival_t* a = &order[q];
        const int tail = a->kind == 0 && segs[a->idx]->timestamp + 33u * 12 > 33u * (uint32_t)(nf - 1);
        const uint32_t loss = a->kind ? fec_loss_pm : seg_loss_pm;
        if (oracle_xs_rand(&rs, 999) < loss && !(protect_tail && tail))
            continue;
        uint64_t key = (uint64_t)q * 1024 + oracle_xs_rand(&rs, window * 1024);
        if (a->kind == 1 && oracle_xs_rand(&rs, 999) < late_pm)
            key += (uint64_t)(150 + oracle_xs_rand(&rs, 200)) * 1024 * 12; /* seconds late */
        if (late_seg_pm && a->kind == 0 && oracle_xs_rand(&rs, 999) < late_seg_pm)
            key += (uint64_t)(100 + oracle_xs_rand(&rs, 150)) * 1024 * 12; /* segments seconds late */
        arr[na++] = (arrival_t){a->kind, a->idx, key, 0};
        if (oracle_xs_rand(&rs, 999) < dup_pm)
            arr[na++] = (arrival_t){a->kind, a->idx, key + 1 + oracle_xs_rand(&rs, window * 2048), 1};
    }
    qsort(arr, (size_t)na, sizeof(arr[0]), cmp_arrival);
    fprintf(js, "],\n   \"parities\": [");
    for (int p = 0; p < np; ++p)
        fprintf(js, "%s[%d, %u]", p ? ", " : "", fec_group[p], fecs[p]->index);
    fprintf(js, "],\n   \"arrivals\": [");
    for (int a = 0; a < na; ++a)
        fprintf(js, "%s[%d, %d]", a ? ", " : "", arr[a].kind, arr[a].idx);
    fprintf(js, "],\n   \"recovered\": [");
    /* receiver: sim_receiver_put (sim_receiver.c:811-827) / _put_fec (:829-838) */
    memset(seen, 0, sizeof(seen));
    sim_receiver_fec_t* rx = sim_fec_create(NULL);
    int64_t clock = rx->evict_ts;
    int nrec = 0;
    for (int a = 0; a < na; ++a) {
        if (arr[a].kind == 0) {
            const sim_segment_t* s = segs[arr[a].idx];
            if (seen[s->packet_id]) /* sim_receiver_internal_put refuses a packet it has */
                continue;
            seen[s->packet_id] = 1;
            sim_segment_t tmp = *s;
            if (tmp.fec_id > 0)
                sim_fec_put_segment(NULL, rx, &tmp);
        } else {
            sim_fec_t* p = (sim_fec_t*)malloc(sizeof(sim_fec_t));
            *p = *fecs[arr[a].idx];
            sim_fec_put_fec_packet(NULL, rx, p);
        }
        /* sim_receiver_recover, sim_receiver.c:780-804 */
        while (skiplist_size(rx->recover_packets) > 0) {
            skiplist_iter_t* iter = skiplist_first(rx->recover_packets);
            sim_segment_t* seg = (sim_segment_t*)iter->val.ptr;
            sim_segment_t in = *seg;
            skiplist_remove(rx->recover_packets, iter->key);
            if (seen[in.packet_id])
                continue;
            seen[in.packet_id] = 1;
            fprintf(js, "%s[%u, %u, %u, %u, %u, %u, %u, %u, %u, \"%016llx\"]", nrec ? ", " : "", in.packet_id, in.fid,
                    in.timestamp, in.index, in.total, in.ftype, in.payload_type, in.data_size, in.fec_id,
                    (unsigned long long)fnv1a(in.data, in.data_size, 0xCBF29CE484222325ull));
            nrec++;
            sim_fec_put_segment(NULL, rx, &in);
        }
        if (evict_every > 0 && a % evict_every == evict_every - 1) {
            clock += 1000; /* past EVICT_FEC_TIMER (sim_fec.c:209) */
            sim_fec_evict(NULL, rx, clock);
        }
    }
    fprintf(js, "],\n   \"max_ts\": %u, \"segments\": %d, \"n_parities\": %d, \"evict_every\": %d, "
                "\"flexes_left\": %u, \"cache_left\": %u}",
            rx->max_ts, ns, np, evict_every, (unsigned)skiplist_size(rx->flexes), (unsigned)skiplist_size(rx->segs_cache));
    fprintf(stderr, "%-22s segments %d parities %d arrivals %d recovered %d\n", name, ns, np, na, nrec);
    sim_fec_destroy(NULL, rx);
    for (int q = 0; q < ns; ++q)
        free(segs[q]);
    for (int p = 0; p < np; ++p)
        free(fecs[p]);
    destroy_list(out);
    flex_fec_sender_destroy(flex);
}

static void scenario(const char* name, uint64_t id, const frame_t* frames, int nf, uint32_t seg_loss_pm,
                     uint32_t fec_loss_pm, uint32_t window, uint32_t dup_pm, uint32_t late_pm, int protect_tail)
{
    scenario_x(name, id, frames, nf, seg_loss_pm, fec_loss_pm, window, dup_pm, late_pm, protect_tail, 0, 0);
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: gen_rx <out.json>\n");
        return 2;
    }
    js = fopen(argv[1], "w");
    if (!js) {
        perror(argv[1]);
        return 1;
    }
    fprintf(js, "{\"generator\": \"oracle/gen_rx.c (reference sim_fec.c + flex receiver / sender)\",\n"
                " \"group\": [\"fec_id\", \"base_id\", \"count\", \"protect_fraction\"],\n"
                " \"parity\": [\"group\", \"index\"],\n"
                " \"arrival\": [\"kind (0 segment, 1 parity)\", \"segment or parity index\"],\n"
                " \"recovered\": [\"packet_id\", \"fid\", \"timestamp\", \"index\", \"total\", \"ftype\", "
                "\"payload_type\", \"data_size\", \"fec_id\", \"fnv1a\"],\n"
                " \"scenarios\": [\n");
    enum { N = 400 };
    static frame_t fr[N];
    for (int i = 0; i < 60; ++i)
        fr[i] = (frame_t){10u * SIM_VIDEO_SIZE, (uint8_t)(i % 30 == 0), 96, 80};
    scenario("k10_loss10", 1, fr, 60, 100, 100, 6, 30, 0, 0);
    scenario("k10_loss25_dup", 2, fr, 60, 250, 150, 20, 80, 0, 0);
    uint64_t r = 0xBADC0DEull;
    for (int i = 0; i < 120; ++i) {
        uint32_t segs_n = 1 + oracle_xs_rand(&r, i % 9 == 0 ? 110 : 14);
        fr[i] = (frame_t){segs_n * SIM_VIDEO_SIZE - oracle_xs_rand(&r, SIM_VIDEO_SIZE - 1), (uint8_t)(i % 25 == 0),
                          (uint8_t)oracle_xs_rand(&r, 255), (uint8_t)(10 + oracle_xs_rand(&r, 245))};
    }
    scenario("mixed_loss15", 3, fr, 120, 150, 100, 40, 20, 0, 0);
    /* parities arriving > 3 s late (sim_fec.c:148: dropped when send_ts + 3000 < max_ts);
     * the newest frames are never lost, so recovered timestamps stay below max_ts */
    for (int i = 0; i < 400; ++i)
        fr[i] = (frame_t){(4u + (uint32_t)(i % 9)) * SIM_VIDEO_SIZE - 13u * (uint32_t)i % 97u, 0, 100, 60};
    scenario("late_parities", 4, fr, 400, 120, 50, 10, 10, 300, 1);
    /* streams with the heartbeat's eviction between arrivals (a receiver
     * session): segments arriving seconds late find their flex evicted
     * (fec_ts + 3000 <= max_ts) or still open; parities lost wholesale leave
     * cached segments to the 6 s cache rule */
    for (int i = 0; i < 400; ++i)
        fr[i] = (frame_t){(3u + (uint32_t)(i % 11)) * SIM_VIDEO_SIZE - 7u * (uint32_t)i % 89u,
                          (uint8_t)(i % 40 == 0), 98, (uint8_t)(i % 7 == 0 ? 5 : 80)};
    scenario_x("evict_late_segments", 5, fr, 400, 100, 60, 12, 10, 20, 1, 60, 40);
    scenario_x("evict_lost_parities", 6, fr, 400, 80, 550, 8, 10, 0, 1, 20, 97);
    scenario_x("no_evict_late_segments", 5, fr, 400, 100, 60, 12, 10, 20, 1, 60, 0);
    /* a foreign peer's groups above 128 segments (one group per frame of 130-200
     * segments): razor's own sender closes groups at 100, the flex receiver
     * takes any count (flex_fec_receiver.c:69-88) */
    g_flush_at = 256;
    for (int i = 0; i < 40; ++i)
        fr[i] = (frame_t){(130u + (uint32_t)(i * 37 % 71)) * SIM_VIDEO_SIZE - 11u * (uint32_t)i, (uint8_t)(i % 20 == 0),
                          97, (uint8_t)(i % 5 == 0 ? 30 : 80)};
    scenario("peer_large_groups", 7, fr, 40, 60, 80, 24, 10, 0, 1);
    /* a foreign peer's groups above 255 segments (one group per frame of
     * 300-1,000 segments): planes of up to 50 rows x 20 columns, 70 lines at
     * 1,000 (flex_fec_sender.c:81-135 clamps the column count to 20), deep
     * row / column cascades */
    g_flush_at = 1100;
    for (int i = 0; i < 10; ++i)
        fr[i] = (frame_t){(300u + (uint32_t)(i * 131 % 701)) * SIM_VIDEO_SIZE - 17u * (uint32_t)i, (uint8_t)(i == 0),
                          97, 80};
    scenario("peer_huge_groups", 8, fr, 10, 50, 60, 30, 10, 0, 0);
    g_flush_at = 100;
    fprintf(js, "\n]}\n");
    fclose(js);
    return 0;
}
