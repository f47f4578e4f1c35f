/*
 * rfec_flex.c -- group-level drop-in of razor's flex FEC sender and receiver
 * (include/razor_flex.h).  The control logic restates
 * sim_transport/fec/flex_fec_sender.c and flex_fec_receiver.c call for call
 * (file:line at each function); the XOR work of a whole call goes to the GPU
 * in one launch through the drop-in staging area of rfec_host.c:
 *
 *   sender update:        every parity line of the group     (rfec_di_generate_group)
 *   receiver on_segment:  its row and its column recovery     (rfec_di_recover_lines)
 *   receiver on_fec:      the one recovery it can trigger     (rfec_di_recover_lines)
 *
 * The receiver replaces the reference's two skiplists (members keyed by
 * packet_id, parities keyed by index) with a position-indexed member table for
 * the group [base_id, base_id + count), a small list of the members above it
 * (the reference accepts any id >= base_id, :259-263, and counts it in
 * skiplist_size), and a 256-entry parity table (index is a u8).
 */
#define _POSIX_C_SOURCE 200809L
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "razor_fec.h"
#include "razor_flex.h"
#include "rfec_internal.h"

/* ------------------------------------------------------------------------ */
/* the caller's cf_list                                                      */
/* ------------------------------------------------------------------------ */
/* razor links common/cf_list.c: use its functions; a process without them
 * (ctypes, tests) gets a push onto the same layout with the same allocator. */
extern void list_push(base_list_t* l, void* data) __attribute__((weak));
extern void list_clear(base_list_t* l) __attribute__((weak));

static void out_push(base_list_t* l, void* data)
{
    if (list_push) {
        list_push(l, data);
        return;
    }
    base_list_unit_t* u = (base_list_unit_t*)malloc(sizeof(*u));
    if (!u)
        return;
    u->next = NULL;
    u->pdata = data;
    if (l->tailer)
        l->tailer->next = u;
    else
        l->head = u;
    l->tailer = u;
    ++l->size;
}

static void out_clear(base_list_t* l)
{
    if (list_clear) {
        list_clear(l);
        return;
    }
    while (l->head) {
        base_list_unit_t* u = l->head;
        l->head = u->next;
        free(u);
    }
    l->tailer = NULL;
    l->size = 0;
}

/* GET_SYS_MS (common/cf_platform.h:101, posix.c:127-132) */
static int64_t sys_ms(void)
{
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return ((int64_t)tv.tv_sec * 1000 * 1000 + tv.tv_usec) / 1000;
}

/* ------------------------------------------------------------------------ */
/* sender (flex_fec_sender.c)                                                */
/* ------------------------------------------------------------------------ */
#define SENDER_CHUNK 32        /* DEFAULT_SIZE, :3 */
#define REPAIR_WINDOW_MS 500   /* FEC_REPAIR_WINDOW, :4 */

flex_fec_sender_t* flex_fec_sender_create(void) /* :8-19 */
{
    flex_fec_sender_t* f = (flex_fec_sender_t*)calloc(1, sizeof(*f));
    if (!f)
        return NULL;
    f->seg_size = SENDER_CHUNK;
    f->segs = (sim_segment_t**)calloc(SENDER_CHUNK, sizeof(sim_segment_t*));
    f->cache_size = SENDER_CHUNK;
    f->cache = (sim_segment_t**)calloc(SENDER_CHUNK, sizeof(sim_segment_t*));
    f->fec_id = 1;
    f->first = 1;
    return f;
}

void flex_fec_sender_destroy(flex_fec_sender_t* f) /* :21-36 */
{
    if (!f)
        return;
    free(f->segs);
    free(f->cache);
    free(f);
}

void flex_fec_sender_reset(flex_fec_sender_t* f) /* :38-46 */
{
    f->fec_id = 1;
    f->first = 1;
    f->col = f->row = 0;
    f->base_id = 0;
    f->fec_ts = 0;
    f->segs_count = 0;
}

void flex_fec_sender_add_segment(flex_fec_sender_t* f, sim_segment_t* seg) /* :49-78 */
{
    const int64_t now = sys_ms();
    if (f->fec_ts == 0) {
        f->fec_ts = now;
    } else if (f->fec_ts + REPAIR_WINDOW_MS * 4 < now) { /* a stale group starts over */
        f->segs_count = 0;
        f->base_id = 0;
        f->first = 1;
        f->fec_ts = now;
    }
    if (f->first == 1 || seg->packet_id < f->base_id)
        f->base_id = seg->packet_id;
    f->first = 0;
    if (f->segs_count >= f->seg_size) {
        uint32_t sz = f->seg_size;
        while (f->segs_count >= sz)
            sz += SENDER_CHUNK;
        sim_segment_t** p = (sim_segment_t**)realloc(f->segs, sz * sizeof(sim_segment_t*));
        if (!p)
            return;
        f->segs = p;
        f->seg_size = (uint16_t)sz;
    }
    f->segs[f->segs_count++] = seg;
}

int flex_fec_sender_num_packets(flex_fec_sender_t* f, uint8_t protect_fraction) /* :81-135 */
{
    uint8_t row = 0, col = 0;
    const int rc = rfec_num_packets(f->segs_count, protect_fraction, &row, &col);
    f->row = row;
    f->col = col;
    return rc;
}

/* the lines of :158-233 over segs[0..n): rows of `col`, then (matrix mode)
 * columns; a line of one member is skipped as flex_fec_generate refuses it */
typedef struct {
    int n_lines;
    int first[2 * 256], stride[2 * 256], count[2 * 256], index[2 * 256];
} line_list;

/* row and col are uint8_t in flex_fec_sender_t (the reference truncates the
 * planner's values the same way), so at most 255 + 255 lines fit line_list */
static void sender_lines(const flex_fec_sender_t* f, int rc, line_list* L)
{
    const int n = f->segs_count, row = f->row, col = f->col;
    _Static_assert(sizeof(f->row) == 1 && sizeof(f->col) == 1, "line_list holds 2 x 256 lines");
    L->n_lines = 0;
    for (int r = 0; r < row; ++r) {
        const int left = n - r * col;
        const int cnt = left < col ? left : col;
        if (cnt >= 2) {
            L->first[L->n_lines] = r * col;
            L->stride[L->n_lines] = 1;
            L->count[L->n_lines] = cnt;
            L->index[L->n_lines++] = r;
        }
    }
    if (row > 1 && rc == 1) {
        for (int c = 0; c < col; ++c) {
            int cnt = 0;
            while (cnt < row && cnt * col + c < n)
                ++cnt;
            if (cnt >= 2) {
                L->first[L->n_lines] = c;
                L->stride[L->n_lines] = col;
                L->count[L->n_lines] = cnt;
                L->index[L->n_lines++] = 0x80 | c;
            }
        }
    }
}

static void stamp(sim_fec_t* o, const flex_fec_sender_t* f, int index) /* :176-181, 220-225 */
{
    o->fec_id = f->fec_id;
    o->base_id = f->base_id;
    o->col = f->col;
    o->row = f->row;
    o->index = (uint8_t)index;
    o->count = f->segs_count;
}

void flex_fec_sender_update(flex_fec_sender_t* f, uint8_t protect_fraction, base_list_t* out_fecs) /* :146-245 */
{
    const int64_t now = sys_ms();
    if (!(f->fec_ts + REPAIR_WINDOW_MS < now || f->segs_count >= 6)) /* flex_fec_sender_over, :137-143 */
        return;
    const int rc = flex_fec_sender_num_packets(f, protect_fraction);
    if (f->col > 1) {
        if (f->row > 1 && rc == 1 && f->cache_size < f->row) { /* the reference's column cache, :200-204 */
            uint32_t sz = f->cache_size;
            while (sz < f->row)
                sz += SENDER_CHUNK;
            sim_segment_t** p = (sim_segment_t**)realloc(f->cache, sz * sizeof(sim_segment_t*));
            if (p) {
                f->cache = p;
                f->cache_size = (uint16_t)sz;
            }
        }
        static __thread line_list L;
        sender_lines(f, rc, &L);
        sim_fec_t* outs[2 * 256];
        int rets[2 * 256];
        int n_out = 0;
        for (int l = 0; l < L.n_lines; ++l, ++n_out)
            if (!(outs[l] = (sim_fec_t*)malloc(sizeof(sim_fec_t))))
                break;
        if (n_out == L.n_lines) {
            const int n = f->segs_count;
            if (n <= RFEC_MAX_K_ENCODE && L.n_lines <= RFEC_MAX_LINES) {
                /* the whole group in one launch */
                rfec_plan p;
                memset(&p, 0, sizeof(p));
                p.k = (uint16_t)n;
                p.row = f->row;
                p.col = f->col;
                p.rc = (uint8_t)rc;
                p.n_lines = (uint8_t)L.n_lines;
                for (int l = 0; l < L.n_lines; ++l) {
                    p.line[l].first = (uint8_t)L.first[l];
                    p.line[l].stride = (uint8_t)L.stride[l];
                    p.line[l].count = (uint8_t)L.count[l];
                    p.line[l].index = (uint8_t)L.index[l];
                    if (L.index[l] < 0x80)
                        p.n_row_lines = (uint8_t)(l + 1);
                }
                if (rfec_di_generate_group(f->segs, n, &p, outs, rets) != RFEC_OK)
                    for (int l = 0; l < L.n_lines; ++l)
                        rets[l] = -1;
            } else {
                /* a group above the staging area: line by line */
                sim_segment_t* mem[RFEC_MAX_K_ENCODE]; /* a line has at most 255 members (uint8 row / col) */
                for (int l = 0; l < L.n_lines; ++l) {
                    rets[l] = -1;
                    for (int q = 0; q < L.count[l]; ++q)
                        mem[q] = f->segs[L.first[l] + q * L.stride[l]];
                    rets[l] = flex_fec_generate(mem, L.count[l], outs[l]);
                }
            }
            for (int l = 0; l < L.n_lines; ++l) {
                if (rets[l] == 0) {
                    stamp(outs[l], f, L.index[l]);
                    out_push(out_fecs, outs[l]);
                } else {
                    free(outs[l]);
                }
            }
        } else {
            for (int l = 0; l < n_out; ++l)
                free(outs[l]);
        }
    }
    f->fec_ts = 0; /* :236-243 */
    f->segs_count = 0;
    f->base_id = 0;
    f->first = 1;
    f->fec_id++;
    if (f->fec_id == 0)
        f->fec_id = 1;
}

void flex_fec_sender_release(flex_fec_sender_t* f, base_list_t* out_fecs) /* :247-260 */
{
    (void)f;
    for (base_list_unit_t* u = out_fecs->head; u; u = u->next)
        free(u->pdata);
    out_clear(out_fecs);
}

/* ------------------------------------------------------------------------ */
/* receiver (flex_fec_receiver.c)                                            */
/* ------------------------------------------------------------------------ */
#define RX_CACHE 20 /* k_default_cache_size, :3 */

typedef struct {
    flex_fec_receiver_t pub; /* first: callers hold &pub */
    sim_segment_t** slot;    /* member at position p = id - base_id, p < pub.count */
    uint32_t slot_cap;
    uint32_t* above;         /* ids >= base_id + count the reference also keeps */
    uint32_t n_above, above_cap;
    uint32_t n_segs;         /* skiplist_size(r->segs) */
    sim_fec_t* par[256];     /* r->fecs keyed by index */
} flex_rx;

static flex_rx* rx_of(flex_fec_receiver_t* r) { return (flex_rx*)r; }

static void rx_clear(flex_rx* x) /* skiplist_clear of both lists: parities are freed (:10-13) */
{
    if (x->slot)
        memset(x->slot, 0, x->slot_cap * sizeof(sim_segment_t*));
    x->n_above = 0;
    x->n_segs = 0;
    for (int i = 0; i < 256; ++i) {
        free(x->par[i]);
        x->par[i] = NULL;
    }
}

flex_fec_receiver_t* flex_fec_receiver_create(flex_segment_free_f seg_free, flex_fec_free_f fec_free,
                                              void* args) /* :15-30 */
{
    flex_rx* x = (flex_rx*)calloc(1, sizeof(*x));
    if (!x)
        return NULL;
    x->pub.cache_size = RX_CACHE;
    x->pub.cache = (sim_segment_t**)calloc(RX_CACHE, sizeof(sim_segment_t*));
    x->pub.args = args;
    x->pub.flex_fec_free_cb = fec_free;
    x->pub.flex_seg_free_cb = seg_free;
    return &x->pub;
}

void flex_fec_receiver_desotry(flex_fec_receiver_t* r) /* :32-51 */
{
    if (!r)
        return;
    flex_rx* x = rx_of(r);
    rx_clear(x);
    free(x->slot);
    free(x->above);
    free(r->cache);
    free(x);
}

void flex_fec_receiver_reset(flex_fec_receiver_t* r) /* :53-67 */
{
    if (!r)
        return;
    r->base_id = 0;
    r->row = 0;
    r->col = 0;
    r->fec_id = 0;
    r->inited = 0;
    r->fec_ts = 0;
    rx_clear(rx_of(r));
}

void flex_fec_receiver_active(flex_fec_receiver_t* r, uint16_t fec_id, uint8_t col, uint8_t row, uint32_t base_id,
                              uint16_t count) /* :69-88 */
{
    flex_rx* x = rx_of(r);
    r->fec_id = fec_id;
    r->base_id = base_id;
    r->row = row;
    r->col = col;
    r->count = count;
    r->inited = 1;
    rx_clear(x);
    if (x->slot_cap < count) {
        sim_segment_t** p = (sim_segment_t**)realloc(x->slot, (size_t)count * sizeof(sim_segment_t*));
        if (p) {
            x->slot = p;
            x->slot_cap = count;
        }
    }
    if (x->slot)
        memset(x->slot, 0, x->slot_cap * sizeof(sim_segment_t*));
    const int need = col > row ? col : row;
    if (r->cache_size < need) {
        const int sz = (need / RX_CACHE + 1) * RX_CACHE;
        sim_segment_t** p = (sim_segment_t**)realloc(r->cache, (size_t)sz * sizeof(sim_segment_t*));
        if (p) {
            r->cache = p;
            r->cache_size = (uint16_t)sz;
        }
    }
}

int flex_fec_receiver_full(flex_fec_receiver_t* r) /* :90-96 */
{
    return rx_of(r)->n_segs >= r->count ? 0 : -1;
}

/* skiplist_search(r->segs, id) */
static sim_segment_t* rx_find(flex_rx* x, uint32_t id)
{
    const flex_fec_receiver_t* r = &x->pub;
    if (id < r->base_id)
        return NULL; /* never inserted (:259) */
    const uint32_t p = id - r->base_id;
    if (p < r->count)
        return p < x->slot_cap ? x->slot[p] : NULL;
    for (uint32_t i = 0; i < x->n_above; ++i)
        if (x->above[i] == id)
            return (sim_segment_t*)x; /* any non-NULL: present */
    return NULL;
}

/* A recovery the line (row `line`, or column `line` with is_col) can make:
 * flex_recover_row :105-150 / flex_recover_col :162-206 up to the
 * flex_fec_recover call.  Fills the job (members in line order) and returns
 * 1, or 0 when the line cannot recover. */
static int rx_line_job(flex_rx* x, uint8_t line, int is_col, sim_segment_t** mem, rfec_di_recover_job* J)
{
    flex_fec_receiver_t* r = &x->pub;
    if (x->n_segs >= r->count)
        return 0;
    int count = 0, loss = 0;
    const int n = is_col ? r->row : r->col;
    const uint32_t end = r->base_id + r->count;
    for (int i = 0; i < n; ++i) {
        const uint32_t key = (uint32_t)(is_col ? i * r->col + line : line * r->col + i) + r->base_id;
        if (key >= end)
            break;
        sim_segment_t* s = rx_find(x, key);
        if (s)
            mem[count++] = s;
        else
            loss++;
    }
    if (loss != 1 || count == 0)
        return 0;
    sim_fec_t* fec = x->par[is_col ? (line | 0x80) : line];
    if (!fec)
        return 0;
    J->segs = mem;
    J->count = count;
    J->fec = fec;
    J->out = NULL;
    return 1;
}

/* the jobs' flex_fec_recover calls in one launch; out[j] = the malloc'd
 * recovered segment, or NULL (:142-147, 198-203) */
static void rx_run(rfec_di_recover_job* J, int n, sim_segment_t** out)
{
    int rets[2];
    for (int j = 0; j < n; ++j)
        out[j] = J[j].out = (sim_segment_t*)malloc(sizeof(sim_segment_t));
    for (int j = 0; j < n; ++j)
        if (!out[j]) {
            for (int i = 0; i < n; ++i)
                free(out[i]);
            memset(out, 0, (size_t)n * sizeof(*out));
            return;
        }
    if (rfec_di_recover_lines(J, n, rets) != RFEC_OK)
        rets[0] = rets[1] = -1;
    for (int j = 0; j < n; ++j)
        if (rets[j] != 0) {
            free(out[j]);
            out[j] = NULL;
        }
}

sim_segment_t* flex_fec_receiver_on_fec(flex_fec_receiver_t* r, sim_fec_t* fec) /* :208-241 */
{
    if (!r || r->inited == 0 || fec == NULL || r->col < 2 || r->row == 0 || r->count == 0) {
        free(fec);
        return NULL;
    }
    flex_rx* x = rx_of(r);
    if (x->par[fec->index]) { /* a parity of this index is held already */
        free(fec);
        return NULL;
    }
    x->par[fec->index] = fec;
    sim_segment_t* mem[256];
    rfec_di_recover_job J;
    if (!rx_line_job(x, fec->index & 0x7F, (fec->index & 0x80) == 0x80, mem, &J))
        return NULL;
    sim_segment_t* out = NULL;
    rx_run(&J, 1, &out);
    return out;
}

int flex_fec_receiver_on_segment(flex_fec_receiver_t* r, sim_segment_t* seg, base_list_t* out) /* :243-280 */
{
    if (!r || r->inited == 0 || seg == NULL)
        return -1;
    if (r->col < 2 || r->row == 0 || r->count == 0 || seg->packet_id < r->base_id)
        return -1;
    flex_rx* x = rx_of(r);
    if (rx_find(x, seg->packet_id))
        return -1;
    const uint32_t p = seg->packet_id - r->base_id;
    if (p < r->count) {
        if (p >= x->slot_cap)
            return -1; /* the table could not be allocated */
        x->slot[p] = seg;
    } else {
        if (x->n_above == x->above_cap) {
            const uint32_t cap = x->above_cap ? 2 * x->above_cap : 16;
            uint32_t* a = (uint32_t*)realloc(x->above, cap * sizeof(uint32_t));
            if (!a)
                return -1;
            x->above = a;
            x->above_cap = cap;
        }
        x->above[x->n_above++] = seg->packet_id;
    }
    x->n_segs++;
    const uint8_t col = (uint8_t)(p % r->col), row = (uint8_t)(p / r->col);
    /* the row and the column recovery see the same member set (the reference
     * pushes recovered segments to `out`, it does not insert them): one launch */
    sim_segment_t* mem[2][256];
    rfec_di_recover_job J[2];
    int n = 0;
    n += rx_line_job(x, row, 0, mem[n], &J[n]);
    n += rx_line_job(x, col, 1, mem[n], &J[n]);
    if (n == 0)
        return 0;
    sim_segment_t* rec[2] = {NULL, NULL};
    rx_run(J, n, rec);
    for (int j = 0; j < n; ++j) /* row first, then column (:271-277) */
        if (rec[j])
            out_push(out, rec[j]);
    return 0;
}
