/*
 * fec_test_harness.c -- the reference's FEC known-answer tests
 * (sim_test/fec_test/test_func.c:8-334, all six as oracle/ref_tests_main.c
 * runs them) replayed through librazor_fec.so's drop-in symbols alone:
 * flex_fec_generate / flex_fec_recover (razor_fec.h) and the group-level flex
 * sender / receiver (razor_flex.h).  Own code, no reference source or binary:
 * it makes the same calls in the same order with the same inputs and prints
 * the same lines, so its stdout must equal tests/golden/ref_fec_test_stdout.txt
 * (what the reference build printed).  Every check the reference asserts
 * (segment_assert) prints a MISMATCH line and fails the exit status instead.
 *
 * The lists are this file's own; they are not exported, so the library takes
 * its own push onto base_list_t (razor_flex.h) here -- the reference-linked
 * build (oracle/Makefile `dropin_flex`, container-side) covers the other way.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "razor_fec.h"
#include "razor_flex.h"

#define DATA_INFO "1234567890123456789012345678901234567890123456789012345678901234567890123456789012345678901234567890"

static int g_fail = 0;

/* ---- lists (the base_list_t layout of razor_flex.h) ---------------------- */
static base_list_t* lst_new(void) { return (base_list_t*)calloc(1, sizeof(base_list_t)); }

static void* lst_pop(base_list_t* l)
{
    base_list_unit_t* u = l->head;
    if (!u)
        return NULL;
    void* d = u->pdata;
    l->head = u->next;
    if (!l->head)
        l->tailer = NULL;
    --l->size;
    free(u);
    return d;
}

static void lst_free(base_list_t* l)
{
    while (l->head)
        lst_pop(l);
    free(l);
}

/* ---- segments --------------------------------------------------------------*/
static sim_segment_t* make_seg(int i, int n)
{
    sim_segment_t* s = (sim_segment_t*)calloc(1, sizeof(sim_segment_t));
    s->packet_id = s->fid = (uint32_t)i;
    s->payload_type = (uint8_t)(i % 2);
    s->ftype = 1;
    s->index = 0;
    s->total = 1;
    s->timestamp = (uint32_t)i * 100;
    s->data_size = (uint16_t)(strlen(DATA_INFO) - n + i + 1);
    memcpy(s->data, DATA_INFO, s->data_size);
    return s;
}

static void same_seg(const sim_segment_t* a, const sim_segment_t* b, const char* where)
{
    if (a->packet_id != b->packet_id || a->payload_type != b->payload_type || a->fid != b->fid ||
        a->timestamp != b->timestamp || a->ftype != b->ftype || a->index != b->index || a->total != b->total ||
        a->data_size != b->data_size || memcmp(a->data, b->data, b->data_size) != 0) {
        printf("MISMATCH %s: packet %u\n", where, b->packet_id);
        g_fail = 1;
    }
}

/* test_func.c:8-71 */
static void xor_roundtrip(void)
{
    enum { N = 12, LOST = 9 };
    sim_segment_t* segs[N];
    sim_segment_t* rest[N];
    sim_fec_t fec;
    sim_segment_t rec;
    for (int i = 0; i < N; ++i)
        segs[i] = make_seg(i, N);
    if (flex_fec_generate(segs, N, &fec) != 0) {
        printf("fec generate failed!\n");
        goto done;
    }
    if (fec.fec_data_size > strlen(DATA_INFO)) {
        printf("fec data size is error, fec data size = %d, max data size = %ld\n", fec.fec_data_size,
               (long)strlen(DATA_INFO));
        goto done;
    }
    int n = 0;
    for (int i = 0; i < N; ++i)
        if (i != LOST)
            rest[n++] = segs[i];
    if (flex_fec_recover(rest, n, &fec, &rec) != 0) {
        printf("fec recover failed!\n");
        goto done;
    }
    rec.data[segs[N - 1]->data_size] = 0;
    printf("seg[%d]:\n", LOST);
    printf("\tpacket id = %d\n", rec.packet_id);
    printf("\tfid = %d\n", rec.fid);
    printf("\ttimestamp = %d\n", rec.timestamp);
    printf("\tpayload_type = %d\n", rec.payload_type);
    printf("\tftype = %d\n", rec.ftype);
    printf("\ttotal = %d\n", rec.total);
    printf("\tindex = %d\n", rec.index);
    printf("\tdata size = %d\n", rec.data_size);
    printf("\tdata info = %s\n", (char*)rec.data);
done:
    for (int i = 0; i < N; ++i)
        free(segs[i]);
}

/* test_func.c:73-87 */
static void plan_sizes(void)
{
    static const int counts[10] = {1, 5, 7, 15, 20, 36, 41, 50, 72, 122};
    flex_fec_sender_t f;
    memset(&f, 0, sizeof(f));
    for (int i = 0; i < 10; ++i) {
        f.segs_count = (uint16_t)counts[i];
        flex_fec_sender_num_packets(&f, 80);
        printf("num = %d, col = %d, row = %d\n", f.segs_count, f.col, f.row);
    }
}

/* test_func.c:104-145: every parity recovers its line's first member from the others */
static void check_sender_output(sim_segment_t** segs, int n, base_list_t* l)
{
    for (base_list_unit_t* u = l->head; u; u = u->next) {
        sim_fec_t* f = (sim_fec_t*)u->pdata;
        const int idx = f->index & 0x7f;
        const int is_col = (f->index & 0x80) != 0;
        sim_segment_t* mem[256];
        int cnt = 0;
        const int len = is_col ? f->row : f->col;
        for (int i = 1; i < len; ++i) {
            const int pos = is_col ? i * f->col + idx : idx * f->col + i;
            if (pos < n)
                mem[cnt++] = segs[pos];
        }
        sim_segment_t rec;
        if (flex_fec_recover(mem, cnt, f, &rec) == 0)
            same_seg(segs[is_col ? idx : idx * f->col], &rec, "sender line");
        else
            printf("recover failed, %s fec index = %d\n", is_col ? "colum" : "row", idx);
    }
}

/* test_func.c:147-189 */
static void sender_case(uint8_t pf)
{
    enum { N = 21 };
    sim_segment_t* segs[N];
    flex_fec_sender_t* fs = flex_fec_sender_create();
    for (int i = 0; i < N; ++i) {
        segs[i] = make_seg(i, N);
        flex_fec_sender_add_segment(fs, segs[i]);
    }
    base_list_t* out = lst_new();
    flex_fec_sender_update(fs, pf, out);
    printf("%s, segment count = %d, protect = %u, fec num = %ld\n", pf > 52 ? "multiFEC" : "singleFEC", N, 80,
           (long)out->size);
    if (out->size > 0) {
        const sim_fec_t* f = (const sim_fec_t*)out->head->pdata;
        printf("fec col = %d, row = %d\n", f->col, f->row);
        check_sender_output(segs, N, out);
    }
    flex_fec_sender_release(fs, out);
    lst_free(out);
    flex_fec_sender_destroy(fs);
    for (int i = 0; i < N; ++i)
        free(segs[i]);
}

/* the recovered-segment map of test_func.c:191-212 (ascending packet id, no duplicates) */
typedef struct {
    sim_segment_t* v[256];
    int n;
} rec_map;

static void map_add(rec_map* m, sim_segment_t* s)
{
    if (!s)
        return;
    int at = 0;
    while (at < m->n && m->v[at]->packet_id < s->packet_id)
        ++at;
    if ((at < m->n && m->v[at]->packet_id == s->packet_id) || m->n == 256) {
        free(s);
        return;
    }
    memmove(&m->v[at + 1], &m->v[at], (size_t)(m->n - at) * sizeof(m->v[0]));
    m->v[at] = s;
    ++m->n;
}

/* test_func.c:214-275 */
static void receive_in_order(sim_segment_t** segs, int n, base_list_t* fecs, const uint8_t* lost, int n_lost)
{
    flex_fec_receiver_t* r = flex_fec_receiver_create(NULL, NULL, NULL);
    const sim_fec_t* f0 = (const sim_fec_t*)fecs->head->pdata;
    flex_fec_receiver_active(r, f0->fec_id, f0->col, f0->row, f0->base_id, f0->count);
    printf("fec row = %d, colum = %d\n", f0->row, f0->col);
    rec_map m;
    m.n = 0;
    base_list_t* out = lst_new();
    for (int i = 0; i < n; ++i) {
        int gone = 0;
        for (int j = 0; j < n_lost; ++j)
            gone |= lost[j] == i;
        if (gone)
            continue;
        flex_fec_receiver_on_segment(r, segs[i], out);
        if (out->size != 0) {
            printf("MISMATCH: recovery before any parity arrived\n");
            g_fail = 1;
        }
    }
    for (base_list_unit_t* u = fecs->head; u; u = u->next) /* the receiver takes the parities */
        map_add(&m, flex_fec_receiver_on_fec(r, (sim_fec_t*)u->pdata));
    while (m.n > 0) {
        sim_segment_t* s = m.v[0];
        printf("recover seg packet id = %u\n", s->packet_id);
        same_seg(segs[s->packet_id], s, "receiver");
        flex_fec_receiver_on_segment(r, segs[s->packet_id], out); /* cascade */
        memmove(&m.v[0], &m.v[1], (size_t)(m.n - 1) * sizeof(m.v[0]));
        --m.n;
        free(s);
        do
            map_add(&m, (sim_segment_t*)lst_pop(out));
        while (out->size > 0);
    }
    lst_free(out);
    flex_fec_receiver_desotry(r);
}

/* test_func.c:277-334 */
static void receiver_case(uint8_t pf, uint8_t n_lost)
{
    enum { N = 25 };
    static const uint8_t lost[] = {5, 6, 7, 9};
    sim_segment_t* segs[N];
    flex_fec_sender_t* fs = flex_fec_sender_create();
    base_list_t* fecs = lst_new();
    for (int i = 0; i < N; ++i) {
        segs[i] = make_seg(i, N);
        flex_fec_sender_add_segment(fs, segs[i]);
    }
    flex_fec_sender_update(fs, pf, fecs);
    printf("%s, segment count = %d, protect = %u, fec num = %ld\n", pf > 52 ? "multiFEC" : "singleFEC", 21, 80,
           (long)fecs->size);
    if (fecs->size > 0)
        receive_in_order(segs, N, fecs, lost, n_lost < N ? n_lost : N);
    for (int i = 0; i < N; ++i)
        free(segs[i]);
    while (fecs->head) /* the units only: the receiver owns and freed the parities */
        lst_pop(fecs);
    free(fecs);
    flex_fec_sender_destroy(fs);
}

int main(void)
{
    setvbuf(stdout, NULL, _IONBF, 0);
    xor_roundtrip();
    plan_sizes();
    sender_case(20);
    sender_case(80);
    receiver_case(20, 2);
    receiver_case(80, 4);
    return g_fail;
}
