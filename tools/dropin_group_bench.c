/*
 * dropin_group_bench.c -- cost per FEC group of the drop-in paths razor's own
 * sender / receiver would take (GPU box; built by razor_amd/build.py next to
 * librazor_fec_v1200.so):
 *
 *   sender, group level   10 x flex_fec_sender_add_segment + one
 *                         flex_fec_sender_update (protect fraction 80: the 3 x 4
 *                         plan, 7 parity lines, ONE launch) + release
 *   sender, line level    the same 7 lines as 7 flex_fec_generate calls (what
 *                         the reference flex_fec_sender.c:175,219 does when only
 *                         flex_fec_xor.c is replaced)
 *   receiver              an on_segment whose arrival makes its row AND its
 *                         column recoverable (two recoveries, ONE launch) vs two
 *                         flex_fec_recover calls
 *
 * 1,200-byte segments.  Outputs of the group and line paths are compared.
 * Prints one JSON object.  Usage: fec_dropin_group_bench [groups]
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "razor_fec.h"
#include "razor_flex.h"

#define K 10

static int cmp_d(const void* a, const void* b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

/* the q-quantile of n samples (sorts them) */
static double quantile(double* v, int n, double q)
{
    if (n <= 0)
        return 0;
    qsort(v, (size_t)n, sizeof(double), cmp_d);
    return v[(int)(q * (n - 1) + 0.5)];
}

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static uint64_t rng = 0x52415A4F52464543ull;
static uint64_t next(void)
{
    rng ^= rng >> 12;
    rng ^= rng << 25;
    rng ^= rng >> 27;
    return rng * 2685821657736338717ull;
}

static void fill(sim_segment_t** segs, uint32_t id0)
{
    for (int i = 0; i < K; ++i) {
        sim_segment_t* s = segs[i];
        memset(s, 0, sizeof(*s));
        s->packet_id = id0 + i;
        s->fid = id0 / K;
        s->timestamp = 33 * (id0 / K);
        s->index = (uint16_t)i;
        s->total = K;
        s->data_size = SIM_VIDEO_SIZE;
        for (int b = 0; b < SIM_VIDEO_SIZE; b += 8) {
            const uint64_t v = next();
            memcpy(s->data + b, &v, SIM_VIDEO_SIZE - b < 8 ? SIM_VIDEO_SIZE - b : 8);
        }
    }
}

static void drain(base_list_t* l)
{
    while (l->head) {
        base_list_unit_t* u = l->head;
        l->head = u->next;
        free(u->pdata);
        free(u);
    }
    l->tailer = NULL;
    l->size = 0;
}

int main(int argc, char** argv)
{
    const int groups = argc > 1 ? atoi(argv[1]) : 2000;
    sim_segment_t* segs[K];
    for (int i = 0; i < K; ++i)
        segs[i] = (sim_segment_t*)malloc(sizeof(sim_segment_t));
    base_list_t out = {NULL, NULL, 0};
    flex_fec_sender_t* fs = flex_fec_sender_create();
    int ok = 1;

    /* sender, group level (first group: staging set-up, untimed) */
    double t_group = 0;
    double* tg = (double*)malloc((size_t)groups * sizeof(double));
    for (int g = -1; g < groups; ++g) {
        fill(segs, 1 + (uint32_t)(g + 1) * K);
        const double t0 = now_us();
        for (int i = 0; i < K; ++i)
            flex_fec_sender_add_segment(fs, segs[i]);
        flex_fec_sender_update(fs, 80, &out);
        const double t1 = now_us();
        if (g >= 0) {
            t_group += t1 - t0;
            tg[g] = t1 - t0;
        }
        if (out.size != 7)
            ok = 0;
        flex_fec_sender_release(fs, &out);
    }

    rfec_service_info si; /* the resident service's breakdown of the group-level sender calls */
    memset(&si, 0, sizeof(si));
    rfec_service_get_info(&si);

    /* sender, line level: the same 7 lines (3 x 4 plan) as 7 calls */
    static const int first[7] = {0, 4, 8, 0, 1, 2, 3}, stride[7] = {1, 1, 1, 4, 4, 4, 4}, count[7] = {4, 4, 2, 3, 3, 2, 2};
    sim_fec_t* fl = (sim_fec_t*)malloc(7 * sizeof(sim_fec_t));
    double t_line = 0;
    for (int g = -1; g < groups; ++g) {
        fill(segs, 1 + (uint32_t)(g + 1) * K);
        const double t0 = now_us();
        for (int l = 0; l < 7; ++l) {
            sim_segment_t* mem[4];
            for (int q = 0; q < count[l]; ++q)
                mem[q] = segs[first[l] + q * stride[l]];
            if (flex_fec_generate(mem, count[l], &fl[l]) != 0)
                ok = 0;
        }
        const double t1 = now_us();
        if (g >= 0)
            t_line += t1 - t0;
    }
    /* equality: the last group both ways */
    for (int i = 0; i < K; ++i)
        flex_fec_sender_add_segment(fs, segs[i]);
    flex_fec_sender_update(fs, 80, &out);
    int l = 0;
    for (base_list_unit_t* u = out.head; u; u = u->next, ++l) {
        const sim_fec_t* f = (const sim_fec_t*)u->pdata;
        if (l >= 7 || f->fec_data_size != fl[l].fec_data_size ||
            memcmp(&f->fec_meta, &fl[l].fec_meta, sizeof(f->fec_meta)) != 0 ||
            memcmp(f->fec_data, fl[l].fec_data, f->fec_data_size) != 0)
            ok = 0;
    }
    if (l != 7)
        ok = 0;

    /* receiver: with only the row-1 and column-1 parities, segments 4 (row 1)
     * and 9 (column 1) lost, segment 5 (row 1, column 1 of the 3 x 4 matrix)
     * arrives last: its arrival recovers both */
    double t_rx = 0, t_rx2 = 0;
    double* tr = (double*)malloc(500 * sizeof(double));
    const int rx_groups = groups < 500 ? groups : 500;
    for (int g = -1; g < rx_groups; ++g) {
        flex_fec_receiver_t* r = flex_fec_receiver_create(NULL, NULL, NULL);
        const sim_fec_t* f0 = (const sim_fec_t*)out.head->pdata;
        flex_fec_receiver_active(r, f0->fec_id, f0->col, f0->row, f0->base_id, f0->count);
        for (base_list_unit_t* u = out.head; u; u = u->next) { /* row 1 and column 1 parities only */
            if (((const sim_fec_t*)u->pdata)->index != 1 && ((const sim_fec_t*)u->pdata)->index != (0x80 | 1))
                continue;
            sim_fec_t* c = (sim_fec_t*)malloc(sizeof(sim_fec_t));
            memcpy(c, u->pdata, sizeof(sim_fec_t));
            sim_segment_t* rec = flex_fec_receiver_on_fec(r, c);
            if (rec)
                ok = 0, free(rec);
        }
        base_list_t got = {NULL, NULL, 0};
        for (int i = 0; i < K; ++i)
            if (i != 4 && i != 9 && i != 5)
                flex_fec_receiver_on_segment(r, segs[i], &got);
        if (got.size != 0)
            ok = 0;
        const double t0 = now_us();
        flex_fec_receiver_on_segment(r, segs[5], &got);
        const double t1 = now_us();
        if (g >= 0) {
            t_rx += t1 - t0;
            tr[g] = t1 - t0;
        }
        if (got.size != 2 || ((sim_segment_t*)got.head->pdata)->packet_id != segs[4]->packet_id ||
            ((sim_segment_t*)got.tailer->pdata)->packet_id != segs[9]->packet_id ||
            memcmp(((sim_segment_t*)got.head->pdata)->data, segs[4]->data, SIM_VIDEO_SIZE) != 0 ||
            memcmp(((sim_segment_t*)got.tailer->pdata)->data, segs[9]->data, SIM_VIDEO_SIZE) != 0)
            ok = 0;
        drain(&got);
        flex_fec_receiver_desotry(r);
        /* the same two recoveries as two flex_fec_recover calls */
        sim_segment_t* row1[3] = {segs[5], segs[6], segs[7]};
        sim_segment_t* col1[2] = {segs[1], segs[5]};
        sim_segment_t o1, o2;
        const sim_fec_t* pr = NULL;
        const sim_fec_t* pc = NULL;
        for (base_list_unit_t* u = out.head; u; u = u->next) {
            const sim_fec_t* f = (const sim_fec_t*)u->pdata;
            if (f->index == 1)
                pr = f;
            if (f->index == (0x80 | 1))
                pc = f;
        }
        const double t2 = now_us();
        const int a = flex_fec_recover(row1, 3, (sim_fec_t*)pr, &o1);
        const int b = flex_fec_recover(col1, 2, (sim_fec_t*)pc, &o2);
        const double t3 = now_us();
        if (g >= 0)
            t_rx2 += t3 - t2;
        if (a || b || o1.packet_id != segs[4]->packet_id || o2.packet_id != segs[9]->packet_id)
            ok = 0;
    }
    printf("{\"groups\": %d, \"k\": %d, \"payload_bytes\": %d, \"lines_per_group\": 7,\n"
           " \"sender_group_level_us_per_group\": %.2f,\n"
           " \"sender_line_level_us_per_group\": %.2f,\n"
           " \"receiver_on_segment_row_and_col_us\": %.2f,\n"
           " \"sender_group_level_us_median\": %.2f, \"sender_group_level_us_p10\": %.2f,"
           " \"receiver_on_segment_us_median\": %.2f,\n"
           " \"receiver_two_flex_fec_recover_us\": %.2f,\n"
           " \"outputs_equal\": %s,\n"
           " \"service_sender\": {\"jobs\": %llu, \"launches\": %llu, \"stage_host_us\": %.2f, \"wait_us\": %.2f,"
           " \"dev_stage_us\": %.2f, \"dev_work_us\": %.2f, \"dev_release_us\": %.2f, \"request_in_device\": %u}}\n",
           groups, K, SIM_VIDEO_SIZE, t_group / groups, t_line / groups, t_rx / rx_groups,
           quantile(tg, groups, 0.5), quantile(tg, groups, 0.1), quantile(tr, rx_groups, 0.5), t_rx2 / rx_groups,
           ok ? "true" : "false", (unsigned long long)si.jobs, (unsigned long long)si.launches, si.stage_host_us,
           si.wait_us, si.dev_stage_us, si.dev_work_us, si.dev_release_us, si.request_in_device);
    drain(&out);
    flex_fec_sender_destroy(fs);
    free(fl);
    for (int i = 0; i < K; ++i)
        free(segs[i]);
    return ok ? 0 : 1;
}
