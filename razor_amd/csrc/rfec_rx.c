/*
 * rfec_rx.c -- receiver ingestion: rfec_rx_recover, the receiver sessions
 * (rfec_rx_session_*) and rfec_host_recv_datagrams.  The arrival-order control
 * plane of sim_fec.c:104-241 / flex_fec_receiver.c:69-280 runs on the host
 * over headers; the bytes are peeled on the device.
 */
#define _GNU_SOURCE /* sched_getcpu, CPU_SET, pthread_attr_setaffinity_np: the replay threads' placement */
#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__ 1
#endif
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "razor_fec.h"
#include "rfec_internal.h"
#include "rfec_host_internal.h"

/* ------------------------------------------------------------------------ */
/* 6. receiver ingestion (semantics: include/razor_fec.h, rfec_rx_recover)  */
/*    The control plane runs in arrival order on the host over headers only: */
/*    admission, flex lifetime, which line recovers which packet and when    */
/*    (so max_ts and first-arrival dedupe come out as the reference's).  The */
/*    bytes never leave the device: the groups are peeled there by           */
/*    rfec_recover_batch from their arrived members and registered parities. */
/* ------------------------------------------------------------------------ */
typedef struct { /* open addressing u32 -> u32, value 0 = empty */
    uint32_t* k;
    uint32_t* v;
    uint32_t mask, n;
} hmap;

/* Home slot: keys in blocks of 16 (consecutive keys, consecutive slots: one
 * cache line serves several lookups, as packet ids and fec_ids arrive nearly
 * in sequence), the blocks spread by Fibonacci hashing on the table's bit
 * width.  (A multiplicative hash of each key sent every lookup of the c3
 * stream to a new line; the key's low bits alone alias a shard's keys, which
 * take every T-th group, onto a quarter of the table.) */
static uint32_t key_home(uint32_t mask, uint32_t k)
{
    const uint32_t bits = 32u - (uint32_t)__builtin_clz(mask); /* log2(capacity), >= 6 */
    return ((((k >> 4) * 0x9E3779B1u) >> (36u - bits)) << 4 | (k & 15u)) & mask;
}
static uint32_t hm_home(const hmap* m, uint32_t k) { return key_home(m->mask, k); }

static int hm_init(hmap* m, uint32_t n)
{
    uint32_t cap = 64;
    while (cap < 2 * n + 64)
        cap <<= 1;
    m->k = (uint32_t*)malloc(cap * sizeof(uint32_t));
    m->v = (uint32_t*)calloc(cap, sizeof(uint32_t));
    m->mask = cap - 1;
    m->n = 0;
    return m->k && m->v ? 0 : -1;
}
static void hm_free(hmap* m)
{
    free(m->k);
    free(m->v);
    m->k = m->v = NULL;
}
static uint32_t hm_slot(const hmap* m, uint32_t k)
{
    uint32_t h = hm_home(m, k);
    while (m->v[h] && m->k[h] != k)
        h = (h + 1) & m->mask;
    return h;
}
static uint32_t hm_get(const hmap* m, uint32_t k) { return m->v[hm_slot(m, k)]; }
static int hm_put(hmap* m, uint32_t k, uint32_t v)
{
    if (2 * (m->n + 1) > m->mask + 1) {
        hmap g;
        if (hm_init(&g, 2 * (m->mask + 1)))
            return -1;
        for (uint32_t i = 0; i <= m->mask; ++i)
            if (m->v[i]) {
                const uint32_t s = hm_slot(&g, m->k[i]);
                g.k[s] = m->k[i];
                g.v[s] = m->v[i];
                g.n++;
            }
        hm_free(m);
        *m = g;
    }
    const uint32_t s = hm_slot(m, k);
    m->n += m->v[s] == 0;
    m->k[s] = k;
    m->v[s] = v;
    return 0;
}
static void hm_del(hmap* m, uint32_t k) /* backward-shift deletion */
{
    uint32_t h = hm_slot(m, k);
    if (!m->v[h])
        return;
    m->v[h] = 0;
    m->n--;
    for (uint32_t j = (h + 1) & m->mask; m->v[j]; j = (j + 1) & m->mask)
        if (((j - hm_home(m, m->k[j])) & m->mask) >= ((j - h) & m->mask)) {
            m->k[h] = m->k[j];
            m->v[h] = m->v[j];
            m->v[j] = 0;
            h = j;
        }
}

/* Packet-id maps (first-arrival dedupe, the segment cache, fec_id -> flex,
 * packet-id ownership): u32 key -> u32 value (0 = absent) in a radix table,
 * 14 + 10 + 8 key bits: a directory of mids, a mid of leaves, a leaf of 256
 * values, allocated on first use and freed when empty.  Ids arrive nearly in
 * sequence, so consecutive lookups hit one leaf (the last one is cached): no
 * hashing, no probing, no rehash, and the key order is the walk order (the
 * evictions' sorted walks).  (An open-addressing hash spent 35-70 % of the
 * control plane in probes that missed the cache, and its growth in page
 * faults.)  Each level keeps a bitmap of what is occupied below it, so a walk
 * (pm_next) skips empty directory slots, leaves and values by bit scans: the
 * evictions and compaction walk the open state, not the key space (the
 * directory scan from key 0 was ~30 % of the control plane with an eviction
 * per batch). */
#define PM_LEAF_BITS 8
#define PM_MID_BITS 10
#define PM_DIR_BITS (32 - PM_LEAF_BITS - PM_MID_BITS)
#define PM_LEAF (1u << PM_LEAF_BITS)
#define PM_MID (1u << PM_MID_BITS)
#define PM_DIR (1u << PM_DIR_BITS)
typedef struct {
    uint32_t n;
    uint64_t bits[PM_LEAF / 64]; /* values != 0 */
    uint32_t v[PM_LEAF];
} pm_leaf;
typedef struct {
    pm_leaf* leaf[PM_MID];
    uint64_t bits[PM_MID / 64]; /* leaves present */
    uint32_t nleaf;
} pm_mid;
typedef struct {
    pm_mid** dir; /* [PM_DIR] */
    uint64_t* dbits; /* [PM_DIR / 64]: mids present */
    uint32_t n;   /* entries */
    uint32_t last_pg;
    pm_leaf* last; /* the leaf of page last_pg (key >> PM_LEAF_BITS), or NULL */
} pmap;

static int pm_init(pmap* m)
{
    memset(m, 0, sizeof(*m));
    m->dir = (pm_mid**)calloc(PM_DIR, sizeof(pm_mid*));
    m->dbits = (uint64_t*)calloc(PM_DIR / 64, sizeof(uint64_t));
    return m->dir && m->dbits ? 0 : -1;
}

static void pm_free(pmap* m)
{
    if (m->dir)
        for (uint32_t d = 0; d < PM_DIR; ++d)
            if (m->dir[d]) {
                for (uint32_t l = 0; l < PM_MID; ++l)
                    free(m->dir[d]->leaf[l]);
                free(m->dir[d]);
            }
    free(m->dir);
    free(m->dbits);
    memset(m, 0, sizeof(*m));
}

static pm_leaf* pm_find(pmap* m, uint32_t k)
{
    const uint32_t pg = k >> PM_LEAF_BITS;
    if (m->last && m->last_pg == pg)
        return m->last;
    const pm_mid* d = m->dir[pg >> PM_MID_BITS];
    pm_leaf* f = d ? d->leaf[pg & (PM_MID - 1)] : NULL;
    if (f) {
        m->last = f;
        m->last_pg = pg;
    }
    return f;
}

static uint32_t pm_get(pmap* m, uint32_t k)
{
    const pm_leaf* f = pm_find(m, k);
    return f ? f->v[k & (PM_LEAF - 1)] : 0u;
}

static int pm_put(pmap* m, uint32_t k, uint32_t v) /* v != 0 */
{
    pm_leaf* f = pm_find(m, k);
    if (!f) {
        const uint32_t pg = k >> PM_LEAF_BITS, di = pg >> PM_MID_BITS, li = pg & (PM_MID - 1);
        pm_mid** d = &m->dir[di];
        if (!*d) {
            if (!(*d = (pm_mid*)calloc(1, sizeof(pm_mid))))
                return -1;
            m->dbits[di >> 6] |= 1ull << (di & 63);
        }
        if (!(f = (pm_leaf*)calloc(1, sizeof(pm_leaf))))
            return -1;
        (*d)->leaf[li] = f;
        (*d)->bits[li >> 6] |= 1ull << (li & 63);
        (*d)->nleaf++;
        m->last = f;
        m->last_pg = pg;
    }
    const uint32_t i = k & (PM_LEAF - 1);
    uint32_t* s = &f->v[i];
    if (*s == 0) {
        f->n++;
        m->n++;
        f->bits[i >> 6] |= 1ull << (i & 63);
    }
    *s = v;
    return 0;
}

static void pm_del(pmap* m, uint32_t k)
{
    pm_leaf* f = pm_find(m, k);
    const uint32_t i = k & (PM_LEAF - 1);
    uint32_t* s = f ? &f->v[i] : NULL;
    if (!s || !*s)
        return;
    *s = 0;
    f->bits[i >> 6] &= ~(1ull << (i & 63));
    m->n--;
    if (--f->n == 0) { /* the leaf (and an empty mid) go */
        const uint32_t pg = k >> PM_LEAF_BITS, di = pg >> PM_MID_BITS, li = pg & (PM_MID - 1);
        pm_mid** d = &m->dir[di];
        (*d)->leaf[li] = NULL;
        (*d)->bits[li >> 6] &= ~(1ull << (li & 63));
        free(f);
        if (--(*d)->nleaf == 0) {
            free(*d);
            *d = NULL;
            m->dbits[di >> 6] &= ~(1ull << (di & 63));
        }
        m->last = NULL;
    }
}

/* the first set bit of bits[0, nbits) at or after `from`, or nbits */
static uint32_t pm_scan(const uint64_t* bits, uint32_t nbits, uint32_t from)
{
    if (from >= nbits)
        return nbits;
    uint32_t w = from >> 6;
    uint64_t x = bits[w] & (~0ull << (from & 63));
    while (!x) {
        if (++w >= nbits / 64)
            return nbits;
        x = bits[w];
    }
    return w * 64 + (uint32_t)__builtin_ctzll(x);
}

/* In key order: the next entry at or after *key (its value's address, the key
 * in *key), NULL past the last.  Start with *key = 0; continue from key + 1. */
static uint32_t* pm_next(const pmap* m, uint32_t* key, uint32_t* done)
{
    uint32_t pg = *key >> PM_LEAF_BITS, i = *key & (PM_LEAF - 1);
    uint32_t di = pg >> PM_MID_BITS, li = pg & (PM_MID - 1);
    if (!m->dir) {
        *done = 1;
        return NULL;
    }
    for (;;) {
        const pm_mid* d = m->dir[di];
        if (!d) { /* the next mid */
            if ((di = pm_scan(m->dbits, PM_DIR, di + 1)) >= PM_DIR)
                break;
            li = i = 0;
            continue;
        }
        pm_leaf* f = d->leaf[li];
        if (f && (i = pm_scan(f->bits, PM_LEAF, i)) < PM_LEAF) {
            *key = (di << (PM_MID_BITS + PM_LEAF_BITS)) | (li << PM_LEAF_BITS) | i;
            return &f->v[i];
        }
        i = 0;
        if ((li = pm_scan(d->bits, PM_MID, li + 1)) < PM_MID)
            continue;
        if ((di = pm_scan(m->dbits, PM_DIR, di + 1)) >= PM_DIR)
            break;
        li = 0;
    }
    *done = 1;
    return NULL;
}
/* for (PM_EACH(m, key, val)) { ... *val ... } -- entries in key order; the body
 * may change *val (not to 0) but not insert or delete */
#define PM_EACH(m, key, val)                                                                        \
    uint32_t key = 0, *val = NULL, pm_d_ = 0;                                                       \
    !pm_d_ && (val = pm_next((m), &key, &pm_d_)) != NULL;                                           \
    key = key == UINT32_MAX ? (pm_d_ = 1, key) : key + 1

typedef struct {
    uint32_t count, row, col, n_groups, n_lines, row0, prow0, group0;
    uint32_t huge;        /* count > RX_MAX_COUNT or more than RFEC_MAX_LINES lines: no plan; line l = FEC
                             index l (members by rx_line_members), n_lines 256, peeled by the host into
                             line jobs (rx_big_peel) */
    uint64_t xcol[2];     /* columns c >= col a peer's parities named (bit c) */
    int16_t line_of[256]; /* FEC index -> plan line, -1: none */
    rfec_plan plan;
} rx_shape;

/* one flex receiver (flex_fec_receiver_t) from its creation to its removal */
typedef struct {
    uint32_t fec_id, base, count, row, col;
    uint32_t shape;        /* UINT32_MAX: geometry the reference ignores (col < 2, row 0, count 0) */
    uint32_t gslot, slot0, line0;
    uint32_t nsegs;        /* flex->segs.n */
    uint64_t have[4];      /* members in the flex (arrived or recovered); huge shapes: rx_has */
    uint64_t arrived[4];   /* members that arrived: the device peel starts from these (huge: slot_src) */
    uint64_t ppm;          /* registered parities, by plan line (huge: line_par >= 0) */
    uint32_t fec_ts;       /* flex->fec_ts = send_ts of the parity that created it (sim_fec.c:157) */
    int ref_ok;            /* col >= 2 && row >= 1 && count >= 1 (flex_fec_receiver.c:214, 250) */
    uint32_t gstamp;       /* == rx_sim.epoch: gslot is this device call's group slot */
    uint32_t jstamp;       /* == rx_sim.jepoch: saved in this batch's journal (rx_touch) */
} rx_inst;

typedef struct {
    rfec_hdr hdr;
    uint32_t inst;
    uint32_t shard; /* rx_device's merged list: the shard holding inst */
} rx_event; /* a recovered segment: pending, then delivered */

/* ------------------------------------------------------------------------ */
/* Sharded sessions (rfec_rx_session_*): the control plane partitioned by     */
/* fec_id over T shards, each a full rx_sim replayed by its own thread in     */
/* arrival order.  Groups are independent in the reference (the receiver     */
/* keys a flex by fec_id, sim_fec.c:141-207), and every other piece of       */
/* state is keyed by packet id: first-arrival dedupe, the segment cache a    */
/* new flex replays (sim_fec.c:121-138), the recovered-id map (:104-119).    */
/* Those stay inside one shard as long as every packet id belongs to one     */
/* fec_id -- its segments carry it, the parity ranges [base_id, base_id +    */
/* count) claim it, and recovery stays inside its flex's range -- which is  */
/* checked after each batch (each shard logs its claims; T threads insert    */
/* them into the owner tables, partitioned by packet-id block, so no two     */
/* threads write one table; recovery ranges as they happen).  The one global */
/* quantity is max_ts, which gates the 3 s parity drop (sim_fec.c:148): a    */
/* batch runs in parallel only when no parity can be dropped by it (its      */
/* send_ts + 3000 >= every earlier segment timestamp of the batch, checked   */
/* before the replay, and >= every segment recovered before it, checked as   */
/* recoveries happen).  A batch that breaks either rule is rolled back       */
/* (journal below) and replayed in arrival order: over the shards with one   */
/* max_ts, or, when a packet id crossed fec_ids, after merging the shards    */
/* into one (the session then stays serial).                                */
/* ------------------------------------------------------------------------ */
#define RX_MAX_THREADS 64 /* shards (= replay threads) of a session */
/* records a shard's replay prefetches ahead (RFEC_RX_PREFETCH, default 16) */
static uint32_t rx_prefetch(void)
{
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("RFEC_RX_PREFETCH");
        v = e ? atoi(e) : 16;
        v = v < 0 ? 0 : v > 64 ? 64 : v;
    }
    return (uint32_t)v;
}


#define RX_CONFLICT_OWNER 1
#define RX_CONFLICT_TS 2
#define RX_CONFLICT_RISKY 4 /* a parity of the batch could meet the 3 s drop (found by the replay threads) */

typedef struct { /* one batch's parallel replay, shared by the shards */
    uint32_t T;           /* shards */
    const uint32_t* smin; /* [n]: min over the batch's later parities of send_ts + 3000 (by batch position);
                             NULL: each shard computes its own from `sum` */
    const rfec_rx_split* sum; /* the batch's split summary (k_rx_split), or NULL (host lists) */
    uint32_t n, max0;     /* the batch's records; max_ts at its start */
    uint32_t a0;          /* the batch's first record */
    int ts_check;         /* recoveries checked against smin (the parallel replay) */
    int conflict;         /* RX_CONFLICT_* (atomic) */
    double t0;            /* the replay's start (now_us), for the per-shard timings */
} rx_par;

typedef struct {
    uint8_t map; /* 0 seen, 1 cache, 2 flex_of, 3 shape_of */
    uint32_t key, old; /* old value, 0 = absent */
} rx_jop;

typedef struct {
    const rfec_wire_rec* R;
    uint32_t capacity, max_ts, dropped, unmodelled;
    pmap seen, cache, flex_of; /* packet id -> 1; packet id -> record + 1 | 0x80000000 + rh index; fec_id -> instance + 1 */
    hmap shape_of;
    rx_inst* G;
    uint32_t ng, gcap;
    rx_shape* S;
    uint32_t ns, scap;
    int32_t* slot_src; /* record of an arrived member, -1 otherwise */
    rfec_hdr* slot_hdr;
    uint32_t nslot, slotcap, slothcap; /* one count, two capacities (each array grows on its own) */
    int32_t* line_par; /* record of the registered parity, -1 otherwise */
    uint32_t nline, linecap;
    rx_event* pend;
    uint32_t npend, pendcap;
    rx_event* out;         /* delivered by this call */
    uint32_t nout, outcap;
    rfec_hdr* rh;          /* headers of delivered (recovered) segments the cache refers to */
    uint32_t nrh, rhcap;
    uint32_t epoch;        /* device call counter (rx_inst.gstamp) */
    int oom;
    /* sharded sessions: the batch's shared context, and the journal that rolls
       this shard back to the batch's start (map operations, the instances the
       batch touched -- saved on first touch with their slot / line tables --,
       and the tables' lengths) */
    rx_par* P;
    uint32_t smin_cur;  /* smin of the record being replayed (parallel replay) */
    uint32_t* mine;     /* this shard's records of the batch (the device's split), and their smin */
    uint32_t* mine_sm;
    uint32_t minecap;
    /* the batch split of chunk t of the summary (rx_split_job, on this shard's thread): the chunk's
       positions grouped by shard in arrival order (cof: per-shard offsets), each with the chunk-local
       min over later parities of send_ts + 3000; the chunk's largest segment timestamp, smallest parity
       limit, and whether a parity meets a segment timestamp before it inside the chunk */
    uint32_t *cpos, *csm;
    uint32_t ccap;
    uint32_t cof[RX_MAX_THREADS + 1];
    uint32_t c_maxseg, c_minfec;
    int c_flag;
    uint64_t* claims;   /* this batch's packet-id claims: seq << 32 | fec_id + 1 */
    uint32_t nclaims, claimcap;
    uint64_t* cpart;    /* the claims by owner-table partition (rx_bucket_claims), offsets in coff */
    uint32_t cpartcap;
    uint32_t coff[RX_MAX_THREADS + 1];
    uint32_t* claimed;  /* [65536 / T + 1][2]: the range last claimed per fec_id / T (base, count + 1) */
    int jon;
    uint32_t jepoch, j_ng, j_nslot, j_nline, j_ns, j_nrh, j_max_ts, j_dropped, j_unmod;
    rx_jop* jops;
    uint32_t njops, jopcap;
    uint8_t* jsave;
    size_t njsave, jsavecap;
    double tw_wake, tw_run, tw_pre; /* parallel replays: this shard's start after the replay's, its run and the
                                       part of it before the first arrival (us, summed) */
    double tw_start;
    uint32_t tw_n, tw_recs;
} rx_sim;

#define RX_GROW_F(flag, ptr, n, cap, need, T)                                          \
    do {                                                                                \
        if ((n) + (need) > (cap)) {                                                     \
            uint32_t c_ = (cap) ? 2 * (cap) : 1024;                                     \
            while (c_ < (n) + (need))                                                   \
                c_ *= 2;                                                                \
            T* p_ = (T*)realloc((ptr), (size_t)c_ * sizeof(T));                         \
            if (!p_) {                                                                  \
                (flag) = 1;                                                             \
                break;                                                                  \
            }                                                                           \
            (ptr) = p_;                                                                 \
            (cap) = c_;                                                                 \
        }                                                                               \
    } while (0)
#define RX_GROW(ptr, n, cap, need, T) RX_GROW_F(X->oom, ptr, n, cap, need, T)

/* -- the journal (sharded sessions) ------------------------------------------ */
static pmap* rx_map(rx_sim* X, int m) /* 0 seen, 1 cache, 2 flex_of (3: shape_of, a hash map) */
{
    return m == 0 ? &X->seen : m == 1 ? &X->cache : &X->flex_of;
}
static uint32_t rx_get(rx_sim* X, int m, uint32_t k)
{
    return m == 3 ? hm_get(&X->shape_of, k) : pm_get(rx_map(X, m), k);
}

static void rx_jlog(rx_sim* X, int m, uint32_t k, uint32_t old)
{
    RX_GROW(X->jops, X->njops, X->jopcap, 1, rx_jop);
    if (X->oom)
        return;
    X->jops[X->njops++] = (rx_jop){(uint8_t)m, k, old};
}

/* put / delete on one of X's maps, journaled while a batch may roll back */
static int rx_put(rx_sim* X, int m, uint32_t k, uint32_t v)
{
    if (X->jon)
        rx_jlog(X, m, k, rx_get(X, m, k));
    return m == 3 ? hm_put(&X->shape_of, k, v) : pm_put(rx_map(X, m), k, v);
}
/* as rx_put on map m < 3 for a key the caller just found absent (no second lookup for the journal) */
static int rx_put_new(rx_sim* X, int m, uint32_t k, uint32_t v)
{
    if (X->jon)
        rx_jlog(X, m, k, 0);
    return pm_put(rx_map(X, m), k, v);
}
static void rx_del(rx_sim* X, int m, uint32_t k)
{
    if (X->jon) {
        const uint32_t o = rx_get(X, m, k);
        if (!o)
            return;
        rx_jlog(X, m, k, o);
    }
    if (m == 3)
        hm_del(&X->shape_of, k);
    else
        pm_del(rx_map(X, m), k);
}

/* Saves instance ii (and its slot / line tables) the first time this batch
 * changes it; instances the batch created are dropped whole on rollback. */
static void rx_touch(rx_sim* X, uint32_t ii)
{
    if (!X->jon || ii >= X->j_ng || X->G[ii].jstamp == X->jepoch)
        return;
    rx_inst* g = &X->G[ii];
    const int sh = g->shape != UINT32_MAX;
    const uint32_t nc = sh ? g->count : 0, nl = sh ? X->S[g->shape].n_lines : 0;
    const size_t need = 4 + sizeof(rx_inst) + (size_t)nc * (4 + sizeof(rfec_hdr)) + (size_t)nl * 4;
    if (X->njsave + need > X->jsavecap) {
        size_t c = X->jsavecap ? 2 * X->jsavecap : 1 << 16;
        while (c < X->njsave + need)
            c *= 2;
        uint8_t* p = (uint8_t*)realloc(X->jsave, c);
        if (!p) {
            X->oom = 1;
            return;
        }
        X->jsave = p;
        X->jsavecap = c;
    }
    uint8_t* w = X->jsave + X->njsave;
    memcpy(w, &ii, 4);
    memcpy(w + 4, g, sizeof(rx_inst));
    w += 4 + sizeof(rx_inst);
    memcpy(w, X->slot_src + g->slot0, (size_t)nc * 4);
    memcpy(w + (size_t)nc * 4, X->slot_hdr + g->slot0, (size_t)nc * sizeof(rfec_hdr));
    memcpy(w + (size_t)nc * (4 + sizeof(rfec_hdr)), X->line_par + g->line0, (size_t)nl * 4);
    X->njsave += need;
    g->jstamp = X->jepoch;
}

static void rx_journal_begin(rx_sim* X)
{
    X->jon = 1;
    if (++X->jepoch == 0) { /* wrapped: no instance may carry a stale stamp */
        for (uint32_t i = 0; i < X->ng; ++i)
            X->G[i].jstamp = 0;
        X->jepoch = 1;
    }
    X->njops = 0;
    X->njsave = 0;
    X->j_ng = X->ng;
    X->j_nslot = X->nslot;
    X->j_nline = X->nline;
    X->j_ns = X->ns;
    X->j_nrh = X->nrh;
    X->j_max_ts = X->max_ts;
    X->j_dropped = X->dropped;
    X->j_unmod = X->unmodelled;
}

static void rx_journal_end(rx_sim* X)
{
    X->jon = 0;
    X->njops = 0;
    X->njsave = 0;
}

/* Back to the state rx_journal_begin saw. */
static void rx_rollback(rx_sim* X)
{
    X->jon = 0;
    for (uint32_t q = X->njops; q-- > 0;) {
        const rx_jop* o = &X->jops[q];
        if (o->old) {
            if (o->map == 3 ? hm_put(&X->shape_of, o->key, o->old) : pm_put(rx_map(X, o->map), o->key, o->old))
                X->oom = 1;
        } else if (o->map == 3) {
            hm_del(&X->shape_of, o->key);
        } else {
            pm_del(rx_map(X, o->map), o->key);
        }
    }
    for (size_t off = 0; off < X->njsave;) {
        uint32_t ii;
        memcpy(&ii, X->jsave + off, 4);
        rx_inst* g = &X->G[ii];
        memcpy(g, X->jsave + off + 4, sizeof(rx_inst));
        const int sh = g->shape != UINT32_MAX;
        const uint32_t nc = sh ? g->count : 0, nl = sh ? X->S[g->shape].n_lines : 0;
        const uint8_t* r = X->jsave + off + 4 + sizeof(rx_inst);
        memcpy(X->slot_src + g->slot0, r, (size_t)nc * 4);
        memcpy(X->slot_hdr + g->slot0, r + (size_t)nc * 4, (size_t)nc * sizeof(rfec_hdr));
        memcpy(X->line_par + g->line0, r + (size_t)nc * (4 + sizeof(rfec_hdr)), (size_t)nl * 4);
        off += 4 + sizeof(rx_inst) + (size_t)nc * (4 + sizeof(rfec_hdr)) + (size_t)nl * 4;
    }
    X->ng = X->j_ng;
    X->nslot = X->j_nslot;
    X->nline = X->j_nline;
    X->ns = X->j_ns;
    X->nrh = X->j_nrh;
    X->max_ts = X->j_max_ts;
    X->dropped = X->j_dropped;
    X->unmodelled = X->j_unmod;
    X->npend = X->nout = 0;
    X->njops = 0;
    X->njsave = 0;
}

/* -- packet-id ownership (sharded sessions) ---------------------------------- */
static void rx_conflict(rx_sim* X, int what) { __atomic_fetch_or(&X->P->conflict, what, __ATOMIC_RELAXED); }

/* owner-table partition of a packet id: blocks of 256 ids, round robin */
static uint32_t rx_part(uint32_t seq, uint32_t T) { return (seq >> 8) % T; }

/* the claims grouped by partition (counting sort), for the T verifiers */
static void rx_bucket_claims(rx_sim* X, uint32_t T)
{
    uint32_t cnt[RX_MAX_THREADS + 1] = {0};
    RX_GROW(X->cpart, 0, X->cpartcap, X->nclaims + 1, uint64_t);
    if (X->oom)
        return;
    for (uint32_t q = 0; q < X->nclaims; ++q)
        cnt[rx_part((uint32_t)(X->claims[q] >> 32), T)]++;
    X->coff[0] = 0;
    for (uint32_t j = 0; j < T; ++j)
        X->coff[j + 1] = X->coff[j] + cnt[j];
    uint32_t pos[RX_MAX_THREADS];
    memcpy(pos, X->coff, T * sizeof(uint32_t));
    for (uint32_t q = 0; q < X->nclaims; ++q)
        X->cpart[pos[rx_part((uint32_t)(X->claims[q] >> 32), T)]++] = X->claims[q];
}

static void rx_claim(rx_sim* X, uint32_t seq, uint32_t code)
{
    RX_GROW(X->claims, X->nclaims, X->claimcap, 1, uint64_t);
    if (!X->oom)
        X->claims[X->nclaims++] = (uint64_t)seq << 32 | code;
}

/* a parity's range [base_id, base_id + count) for its fec_id (logged once per range) */
static void rx_claim_range(rx_sim* X, const rfec_wire_rec* r)
{
    uint32_t* c = X->claimed + 2u * (r->fec_id / X->P->T);
    if (c[0] == r->base_id && c[1] == (uint32_t)r->count + 1u)
        return;
    for (uint32_t i = 0; i < r->count; ++i)
        rx_claim(X, r->base_id + i, (uint32_t)r->fec_id + 1u);
    c[0] = r->base_id;
    c[1] = (uint32_t)r->count + 1u;
}

static rfec_hdr rec_hdr(const rfec_wire_rec* r)
{
    rfec_hdr h = r->hdr;
    h.size = r->data_size; /* seg.data_size = the datagram's (sim_receiver.c) */
    return h;
}

/* members of the reference's line `index` of a (count, row, col) flex:
 * flex_recover_row walks i < col, flex_recover_col i < row, both stopping at
 * the first position >= count (flex_fec_receiver.c:118-126, 175-183) */
static uint32_t rx_line_members(uint32_t count, uint32_t row, uint32_t col, uint32_t index, uint32_t* first,
                                uint32_t* stride)
{
    const uint32_t x = index & 0x7Fu;
    uint32_t n = 0;
    if (index & 0x80u) {
        while (n < row && n * col + x < count)
            ++n;
        *first = x;
        *stride = col;
    } else {
        while (n < col && x * col + n < count)
            ++n;
        *first = x * col;
        *stride = 1;
    }
    return n;
}

/* line l of flex g: its members and whether its parity is registered */
static uint32_t rx_line(const rx_sim* X, const rx_inst* g, uint32_t l, uint32_t* first, uint32_t* stride, int* reg)
{
    const rx_shape* sh = &X->S[g->shape];
    if (sh->huge) {
        *reg = X->line_par[g->line0 + l] >= 0;
        return rx_line_members(g->count, g->row, g->col, l, first, stride);
    }
    const rfec_line* ln = &sh->plan.line[l];
    *reg = (int)((g->ppm >> l) & 1ull);
    *first = ln->first;
    *stride = ln->stride;
    return ln->count;
}

/* member t of flex g is in it (arrived or recovered); a huge flex's slot
 * header holds the member's seq once it is in, ~(base + t) before */
static int rx_has(const rx_sim* X, const rx_inst* g, uint32_t t)
{
    if (X->S[g->shape].huge)
        return X->slot_hdr[g->slot0 + t].seq == g->base + t;
    return (int)((g->have[t >> 6] >> (t & 63)) & 1ull);
}

static void rx_pend(rx_sim* X, const rfec_hdr* h, uint32_t inst) /* sim_fec_packet_add_recover (sim_fec.c:104-119) */
{
    for (uint32_t i = 0; i < X->npend; ++i)
        if (X->pend[i].hdr.seq == h->seq)
            return;
    RX_GROW(X->pend, X->npend, X->pendcap, 1, rx_event);
    if (X->oom)
        return;
    X->pend[X->npend].hdr = *h;
    X->pend[X->npend++].inst = inst;
}

/* flex_recover_row / flex_recover_col (flex_fec_receiver.c:105-206) over headers */
static void rx_check_line(rx_sim* X, uint32_t ii, int l)
{
    const rx_inst* g = &X->G[ii];
    if (l < 0 || g->nsegs >= g->count)
        return;
    uint32_t first, stride;
    int reg;
    const uint32_t n = rx_line(X, g, (uint32_t)l, &first, &stride, &reg);
    if (!reg)
        return;
    uint32_t loss = 0, cnt = 0;
    for (uint32_t q = 0; q < n; ++q) {
        if (rx_has(X, g, first + q * stride))
            cnt++;
        else
            loss++;
    }
    if (loss != 1 || cnt == 0)
        return;
    const rfec_wire_rec* f = &X->R[X->line_par[g->line0 + l]];
    const uint32_t L = f->data_size;
    if (L > X->capacity)
        return;
    rfec_hdr h = f->hdr; /* flex_fec_xor.c:64-99 */
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t i = first + q * stride;
        if (!rx_has(X, g, i))
            continue;
        const rfec_hdr* m = &X->slot_hdr[g->slot0 + i];
        if (L < m->size)
            return;
        h.seq ^= m->seq;
        h.fid ^= m->fid;
        h.ts ^= m->ts;
        h.index ^= m->index;
        h.total ^= m->total;
        h.ftype ^= m->ftype;
        h.payload_type ^= m->payload_type;
        h.size ^= m->size;
    }
    if (h.size > L)
        return;
    rx_pend(X, &h, ii);
}

/* flex_fec_receiver_on_segment (flex_fec_receiver.c:243-280); src = record or -1 */
static void rx_on_segment(rx_sim* X, uint32_t ii, const rfec_hdr* h, int32_t src, int check)
{
    rx_inst* g = &X->G[ii];
    if (!g->ref_ok || h->seq < g->base)
        return;
    if (g->shape == UINT32_MAX) {
        X->unmodelled++;
        return;
    }
    rx_touch(X, ii);
    const uint32_t t = h->seq - g->base;
    if (t < g->count) {
        if (rx_has(X, g, t))
            return;
        if (!X->S[g->shape].huge)
            g->have[t >> 6] |= 1ull << (t & 63);
        X->slot_hdr[g->slot0 + t] = *h;
        if (src >= 0) {
            if (!X->S[g->shape].huge)
                g->arrived[t >> 6] |= 1ull << (t & 63);
            X->slot_src[g->slot0 + t] = src;
        }
    } else if (src < 0) {
        X->unmodelled++; /* a recovered header outside its group: inconsistent parities */
    }
    g->nsegs++;
    if (check) {
        const rx_shape* sh = &X->S[g->shape];
        const uint32_t r = t / g->col, c = t % g->col;
        rx_check_line(X, ii, r < 128 ? sh->line_of[r] : -1);
        rx_check_line(X, ii, c < 128 ? sh->line_of[0x80 | c] : -1);
    }
}

static void rx_remove(rx_sim* X, uint32_t ii) /* sim_fec_evict_segment + flex removal (sim_fec.c:93-102, 199-205) */
{
    const rx_inst* g = &X->G[ii];
    for (uint32_t i = 0; i < g->count; ++i)
        rx_del(X, 1, g->base + i);
    rx_del(X, 2, g->fec_id);
}

/* sim_fec_put_segment (sim_fec.c:171-207); cache values: record + 1, or 0x80000000 | index into X->rh */
static void rx_put_segment(rx_sim* X, const rfec_hdr* h, uint16_t fec_id, uint32_t cval, int32_t src)
{
    if (h->seq == 0 || pm_get(&X->cache, h->seq))
        return;
    X->max_ts = h->ts > X->max_ts ? h->ts : X->max_ts;
    if (rx_put_new(X, 1, h->seq, cval)) {
        X->oom = 1;
        return;
    }
    const uint32_t fi = pm_get(&X->flex_of, fec_id);
    if (!fi)
        return;
    rx_on_segment(X, fi - 1, h, src, 1);
    if (X->G[fi - 1].nsegs >= X->G[fi - 1].count) /* flex_fec_receiver_full */
        rx_remove(X, fi - 1);
}

/* The device plan of a flex geometry: every row with 2+ members (also rows
 * at and beyond `row` when row * col < count: the reference bounds rows by
 * count only), every column c < col with 2+ members, and the extra columns
 * c >= col of xcol.  Lines of fewer than 2 members can never recover (one
 * missing member leaves none present).  Standard geometry (row * col >=
 * count, no extra columns) is exactly rfec_plan_matrix's plan. */
static int rx_build_plan(uint32_t count, uint32_t row, uint32_t col, const uint64_t* xcol, rfec_plan* p)
{
    if (row * col >= count && !xcol[0] && !xcol[1])
        return rfec_plan_matrix((uint16_t)count, (uint8_t)row, (uint8_t)col, RFEC_LAYER_ROWS | RFEC_LAYER_COLS, p);
    memset(p, 0, sizeof(*p));
    p->k = (uint16_t)count;
    p->row = (uint8_t)row;
    p->col = (uint8_t)col;
    p->rc = 1;
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t x = 0; x < 128; ++x) {
            if (pass == 1 && x >= col && !((xcol[x >> 6] >> (x & 63)) & 1ull))
                continue;
            uint32_t first, stride;
            const uint32_t n = rx_line_members(count, row, col, pass ? (0x80u | x) : x, &first, &stride);
            if (n < 2)
                continue;
            if (p->n_lines >= RFEC_MAX_LINES)
                return RFEC_EINVAL;
            rfec_line* l = &p->line[p->n_lines++];
            l->first = (uint8_t)first;
            l->stride = (uint8_t)stride;
            l->count = (uint8_t)n;
            l->index = (uint8_t)(pass ? (0x80u | x) : x);
        }
        if (pass == 0)
            p->n_row_lines = p->n_lines;
    }
    return RFEC_OK;
}

/* flexes of up to 255 segments and 64 lines have a device plan (8-bit
 * members); above RFEC_MAX_K the device recovery takes line jobs (rx_big_peel)
 * instead of the batched peel, whose masks hold 128 members.  Larger flexes
 * (a foreign peer's: the reference receiver takes any uint16_t count,
 * flex_fec_receiver.c:69-88, and up to 128 rows and 128 columns of FEC
 * indices) are huge shapes: line = FEC index, line jobs too. */
#define RX_MAX_COUNT 255u

static uint32_t rx_shape_of(rx_sim* X, uint32_t count, uint32_t row, uint32_t col, const uint64_t* xcol)
{
    if (row > 255 || col > 255)
        return UINT32_MAX;
    const int extended = xcol[0] || xcol[1];
    const uint32_t key = count << 16 | row << 8 | col;
    if (!extended) {
        const uint32_t s = hm_get(&X->shape_of, key);
        if (s)
            return s - 1;
    } else { /* rare (a peer's extra columns): a scan */
        for (uint32_t s = 0; s < X->ns; ++s)
            if (X->S[s].count == count && X->S[s].row == row && X->S[s].col == col && X->S[s].xcol[0] == xcol[0] &&
                X->S[s].xcol[1] == xcol[1])
                return s;
    }
    RX_GROW(X->S, X->ns, X->scap, 1, rx_shape);
    if (X->oom)
        return UINT32_MAX;
    rx_shape* sh = &X->S[X->ns];
    memset(sh, 0, sizeof(*sh));
    sh->count = count;
    sh->row = row;
    sh->col = col;
    sh->xcol[0] = xcol[0];
    sh->xcol[1] = xcol[1];
    sh->huge = count > RX_MAX_COUNT || rx_build_plan(count, row, col, xcol, &sh->plan) != RFEC_OK;
    if (sh->huge) { /* every FEC index is a line */
        sh->n_lines = 256;
        for (int i = 0; i < 256; ++i)
            sh->line_of[i] = (int16_t)i;
    } else {
        sh->n_lines = sh->plan.n_lines;
        for (int i = 0; i < 256; ++i)
            sh->line_of[i] = -1;
        for (uint32_t l = 0; l < sh->n_lines; ++l)
            sh->line_of[sh->plan.line[l].index] = (int16_t)l;
    }
    if (!extended && rx_put(X, 3, key, X->ns + 1)) {
        X->oom = 1;
        return UINT32_MAX;
    }
    return X->ns++;
}

/* A parity for a column c >= col of flex ii (a peer's plan, not razor's
 * sender): the flex moves to the shape with that column added, its
 * registered parities carried over by index.  Returns the column's line in
 * the new shape, or -1 (no room: the parity stays unmodelled). */
static int rx_extend(rx_sim* X, uint32_t ii, uint32_t c)
{
    rx_touch(X, ii);
    rx_inst* g = &X->G[ii];
    uint64_t xcol[2] = {X->S[g->shape].xcol[0], X->S[g->shape].xcol[1]};
    xcol[c >> 6] |= 1ull << (c & 63);
    const uint32_t ns = rx_shape_of(X, g->count, g->row, g->col, xcol);
    if (ns == UINT32_MAX)
        return -1;
    const rx_shape* nsh = &X->S[ns]; /* (X->S may have moved) */
    const rx_shape* osh = &X->S[g->shape];
    RX_GROW(X->line_par, X->nline, X->linecap, nsh->n_lines, int32_t);
    if (X->oom)
        return -1;
    uint64_t ppm = 0;
    for (uint32_t l = 0; l < nsh->n_lines; ++l) {
        const int ol = osh->line_of[nsh->huge ? l : nsh->plan.line[l].index];
        X->line_par[X->nline + l] = ol >= 0 && ((g->ppm >> ol) & 1ull) ? X->line_par[g->line0 + ol] : -1;
        if (ol >= 0 && ((g->ppm >> ol) & 1ull) && !nsh->huge)
            ppm |= 1ull << l;
    }
    if (nsh->huge) /* more than RFEC_MAX_LINES lines now: membership moves to the slot headers (rx_has) */
        for (uint32_t t = 0; t < g->count; ++t)
            if (!((g->have[t >> 6] >> (t & 63)) & 1ull))
                X->slot_hdr[g->slot0 + t].seq = ~(g->base + t);
    g->line0 = X->nline;
    X->nline += nsh->n_lines;
    g->ppm = ppm;
    g->shape = ns;
    return nsh->line_of[0x80u | c];
}

/* sim_fec_put_fec_packet (sim_fec.c:141-169) -> flex_fec_receiver_on_fec (flex_fec_receiver.c:208-241) */
static void rx_put_fec(rx_sim* X, uint32_t a)
{
    const rfec_wire_rec* f = &X->R[a];
    if (f->base_id + f->count == 0u || f->send_ts + 3000u < X->max_ts) {
        X->dropped++;
        return;
    }
    uint32_t fi = pm_get(&X->flex_of, f->fec_id);
    if (!fi) { /* flex_fec_receiver_active (flex_fec_receiver.c:69-88) */
        RX_GROW(X->G, X->ng, X->gcap, 1, rx_inst);
        if (X->oom)
            return;
        rx_inst* g = &X->G[X->ng];
        memset(g, 0, sizeof(*g));
        g->fec_id = f->fec_id;
        g->base = f->base_id;
        g->count = f->count;
        g->row = f->row;
        g->col = f->col;
        g->fec_ts = f->send_ts;
        g->ref_ok = g->col >= 2 && g->row >= 1 && g->count >= 1;
        static const uint64_t no_xcol[2] = {0, 0};
        g->shape = g->ref_ok ? rx_shape_of(X, g->count, g->row, g->col, no_xcol) : UINT32_MAX;
        if (g->shape != UINT32_MAX) {
            const rx_shape* sh = &X->S[g->shape];
            RX_GROW(X->slot_src, X->nslot, X->slotcap, g->count, int32_t);
            RX_GROW(X->slot_hdr, X->nslot, X->slothcap, g->count, rfec_hdr);
            RX_GROW(X->line_par, X->nline, X->linecap, sh->n_lines, int32_t);
            if (X->oom)
                return;
            g->slot0 = X->nslot;
            g->line0 = X->nline;
            for (uint32_t i = 0; i < g->count; ++i) {
                X->slot_src[X->nslot + i] = -1;
                X->slot_hdr[X->nslot + i].seq = ~(g->base + i); /* rx_has: not in the flex */
            }
            for (uint32_t l = 0; l < sh->n_lines; ++l)
                X->line_par[X->nline + l] = -1;
            X->nslot += g->count;
            X->nline += sh->n_lines;
        } else if (g->ref_ok) {
            X->unmodelled++;
        }
        fi = ++X->ng;
        if (rx_put(X, 2, f->fec_id, fi)) {
            X->oom = 1;
            return;
        }
        for (uint32_t i = 0; i < g->count && g->shape != UINT32_MAX; ++i) { /* sim_fec_add_segment_to_flex */
            const uint32_t c = pm_get(&X->cache, g->base + i);
            if (!c)
                continue;
            if (c & 0x80000000u) {
                rx_on_segment(X, fi - 1, &X->rh[c & 0x7FFFFFFFu], -1, 0);
            } else {
                const rfec_hdr h = rec_hdr(&X->R[c - 1]);
                rx_on_segment(X, fi - 1, &h, (int32_t)(c - 1), 0);
            }
        }
    }
    rx_inst* g = &X->G[fi - 1];
    if (!g->ref_ok || g->shape == UINT32_MAX)
        return;
    rx_touch(X, fi - 1);
    g = &X->G[fi - 1];
    int l = X->S[g->shape].line_of[f->index];
    if (X->S[g->shape].huge) { /* line = index; the parity registered once */
        uint32_t first, stride;
        if (rx_line_members(g->count, g->row, g->col, f->index, &first, &stride) < 2 ||
            X->line_par[g->line0 + l] >= 0)
            return;
        X->line_par[g->line0 + l] = (int32_t)a;
        rx_check_line(X, fi - 1, l);
        return;
    }
    if (l < 0) {
        uint32_t first, stride;
        if (rx_line_members(g->count, g->row, g->col, f->index, &first, &stride) < 2)
            return; /* a line that can never recover (flex_fec_receiver.c:133-134, 189-190) */
        /* a column c >= col (razor's sender never emits one; a peer may) */
        if ((l = rx_extend(X, fi - 1, f->index & 0x7Fu)) < 0) {
            X->unmodelled++;
            return;
        }
        g = &X->G[fi - 1];
    }
    if (X->S[g->shape].huge) { /* (the extension took it past RFEC_MAX_LINES lines) */
        if (X->line_par[g->line0 + l] >= 0)
            return;
    } else {
        if ((g->ppm >> l) & 1ull)
            return;
        g->ppm |= 1ull << l;
    }
    X->line_par[g->line0 + l] = (int32_t)a;
    rx_check_line(X, fi - 1, l);
}

/* sim_receiver_recover (sim_receiver.c:780-804): lowest packet_id first,
 * cascading; the recoveries of record a.  In a sharded batch each delivered
 * packet must lie in its flex's range (so its id stays in this shard) and,
 * in the parallel replay, raise max_ts no higher than any later parity of
 * the batch can take (smin): else the batch is replayed otherwise. */
static void rx_drain(rx_sim* X, uint32_t a)
{
    while (X->npend && !X->oom) {
        uint32_t b = 0;
        for (uint32_t i = 1; i < X->npend; ++i)
            if (X->pend[i].hdr.seq < X->pend[b].hdr.seq)
                b = i;
        const rx_event e = X->pend[b];
        X->pend[b] = X->pend[--X->npend];
        if (pm_get(&X->seen, e.hdr.seq))
            continue;
        if (X->P) {
            const rx_inst* g = &X->G[e.inst];
            if (e.hdr.seq - g->base >= g->count) {
                rx_conflict(X, RX_CONFLICT_OWNER);
                return;
            }
            if (X->P->ts_check && e.hdr.ts > X->smin_cur) {
                rx_conflict(X, RX_CONFLICT_TS);
                return;
            }
        }
        RX_GROW(X->out, X->nout, X->outcap, 1, rx_event);
        RX_GROW(X->rh, X->nrh, X->rhcap, 1, rfec_hdr);
        if (X->oom || rx_put_new(X, 0, e.hdr.seq, 1)) {
            X->oom = 1;
            return;
        }
        X->out[X->nout++] = e;
        X->rh[X->nrh] = e.hdr;
        const uint32_t idx = X->nrh++;
        rx_put_segment(X, &e.hdr, (uint16_t)X->G[e.inst].fec_id, 0x80000000u | idx, -1);
    }
}

static void rx_sim_free(rx_sim* X)
{
    pm_free(&X->seen);
    pm_free(&X->cache);
    pm_free(&X->flex_of);
    hm_free(&X->shape_of);
    free(X->G);
    free(X->S);
    free(X->slot_src);
    free(X->slot_hdr);
    free(X->line_par);
    free(X->pend);
    free(X->out);
    free(X->rh);
    free(X->jops);
    free(X->jsave);
    free(X->claims);
    free(X->mine);
    free(X->mine_sm);
    free(X->cpos);
    free(X->csm);
    free(X->cpart);
    free(X->claimed);
}

/* sim_fec_evict (sim_fec.c:209-241) past its 300 ms wall-clock gate: flexes in
 * fec_id order while stale (fec_ts + 3000 <= max_ts) or full, removed with
 * their members' cache entries; then cached segments in packet_id order while
 * older than 6 s (timestamp + 6000 < max_ts).  Both walks stop at the first
 * entry that stays, as the skiplist walks do (pmap: key order; each step
 * looks up the next key afresh, so removals are safe). */
static void rx_evict(rx_sim* X)
{
    uint32_t key = 0, done = 0;
    for (uint32_t* v; (v = pm_next(&X->flex_of, &key, &done)) != NULL;) {
        const uint32_t fi = *v - 1;
        const rx_inst* g = &X->G[fi];
        if (!(g->fec_ts + 3000u <= X->max_ts || g->nsegs >= g->count))
            break;
        rx_remove(X, fi);
        if (key == UINT32_MAX)
            break;
        ++key;
    }
    key = done = 0;
    for (uint32_t* v; (v = pm_next(&X->cache, &key, &done)) != NULL;) {
        const uint32_t c = *v;
        const uint32_t ts = (c & 0x80000000u) ? X->rh[c & 0x7FFFFFFFu].ts : X->R[c - 1].hdr.ts;
        if (!(ts + 6000u < X->max_ts))
            break;
        pm_del(&X->cache, key);
        if (key == UINT32_MAX)
            break;
        ++key;
    }
}

static int cmp_event(const void* a, const void* b)
{
    const uint32_t x = ((const rx_event*)a)->hdr.seq, y = ((const rx_event*)b)->hdr.seq;
    return x < y ? -1 : x > y;
}

typedef struct {
    uint8_t* h;  /* pinned, device-mapped */
    uint8_t* hd; /* h as the device addresses it */
    size_t hb;
    uint8_t* d;
    size_t db;
} rx_ctx;
static __thread rx_ctx t_rx;

/* The device address of host memory the device can read directly (pinned:
 * rfec_pinned_alloc, hipHostMalloc, registered), else NULL (pageable: the
 * caller copies).  A failed query leaves no pending HIP error behind. */
static const uint8_t* host_mapped(const void* p)
{
    hipPointerAttribute_t a;
    void* d = NULL;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost ||
        hipHostGetDevicePointer(&d, (void*)p, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return NULL;
    }
    return (const uint8_t*)d;
}

/* Grows the per-thread pinned / device areas.  The first `keep` bytes of the
 * pinned area survive a grow (copied into the new block before the old one is
 * freed: the allocator may hand back the same address, so callers cannot tell
 * a grow from the pointer). */
static int rx_reserve(size_t host_bytes, size_t dev_bytes, size_t keep)
{
    hipError_t e;
    if (t_rx.hb < host_bytes) {
        uint8_t* nh = NULL;
        host_bytes += host_bytes / 4;
        void* nd = NULL;
        if ((e = hipHostMalloc((void**)&nh, host_bytes, hipHostMallocMapped)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx staging (host)", e);
        if ((e = hipHostGetDevicePointer(&nd, nh, 0)) != hipSuccess) {
            (void)hipHostFree(nh);
            return set_err(RFEC_EDEVICE, "rx staging (host): device view", e);
        }
        if (t_rx.h) {
            if (keep)
                memcpy(nh, t_rx.h, keep < t_rx.hb ? keep : t_rx.hb);
            (void)hipHostFree(t_rx.h);
        }
        t_rx.h = nh;
        t_rx.hd = (uint8_t*)nd;
        t_rx.hb = host_bytes;
    }
    if (t_rx.db < dev_bytes) {
        if (t_rx.d)
            (void)hipFree(t_rx.d);
        t_rx.d = NULL;
        t_rx.db = 0;
        dev_bytes += dev_bytes / 4;
        if ((e = hipMalloc((void**)&t_rx.d, dev_bytes)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx workspace (device)", e);
        t_rx.db = dev_bytes;
    }
    return RFEC_OK;
}

#define RX_ALIGN(x) (((x) + 255) & ~(size_t)255)

static int rx_tables_init(rx_sim* X, uint32_t n)
{
    (void)n;
    return pm_init(&X->seen) || pm_init(&X->cache) || pm_init(&X->flex_of) || hm_init(&X->shape_of, 64);
}

/* One record of X->R in arrival order: sim_receiver_put /
 * sim_receiver_put_fec and the recovery cascade.  In a sharded batch the
 * record first claims its packet ids for its fec_id. */
static void rx_arrival(rx_sim* X, uint32_t a)
{
    const rfec_wire_rec* r = &X->R[a];
    if (r->status != RFEC_WIRE_OK)
        return;
    if (r->mid == RFEC_WIRE_SEG) { /* sim_receiver_put (sim_receiver.c:811-827) */
        if (X->P) /* (a segment outside FEC claims its id for fec_id 0) */
            rx_claim(X, r->hdr.seq, (uint32_t)r->fec_id + 1u);
        if (pm_get(&X->seen, r->hdr.seq))
            return;
        if (rx_put_new(X, 0, r->hdr.seq, 1)) {
            X->oom = 1;
            return;
        }
        if (r->fec_id == 0)
            return;
        const rfec_hdr h = rec_hdr(r);
        rx_put_segment(X, &h, r->fec_id, a + 1, (int32_t)a);
    } else if (r->mid == RFEC_WIRE_FEC) {
        if (X->P)
            rx_claim_range(X, r);
        rx_put_fec(X, a);
    }
    rx_drain(X, a);
}

/* The control plane over records [a0, a0 + n) of X->R. */
static void rx_run(rx_sim* X, uint32_t a0, uint32_t n)
{
    for (uint32_t a = a0; a < a0 + n && !X->oom; ++a)
        rx_arrival(X, a);
}

/* The device side of one ingestion call over T shards (one for rfec_rx_recover
 * and a merged session): the shards' deliveries merged in packet-id order, the
 * delivering groups laid out by device shape (the same geometry on several
 * shards is one launch), the line jobs of the large groups. */
typedef struct {
    const rx_shape* sh; /* any shard's shape of this geometry (plans are a function of it) */
    uint32_t n_groups, row0, prow0, group0;
    uint32_t E, dense0; /* dense output slots per group, the shape's first dense row */
} rx_dclass;

typedef struct {
    rx_event* ev;          /* this call's deliveries, all shards, ascending packet id */
    uint32_t nev, evcap;
    uint64_t* dl;          /* delivering groups: shard << 32 | instance */
    uint32_t ndl, dlcap;
    rx_dclass* C;          /* device shapes */
    uint32_t nc, ccap;
    uint32_t* cls;         /* per (shard, shape): its device shape */
    uint32_t clscap;
    rfec_line_job* jobs;   /* groups above RFEC_MAX_K: this call's line jobs (rx_big_peel) */
    uint32_t njobs, jobcap;
    uint16_t* jlevel;      /* a job's dependency level (1 = arrived members only) */
    uint32_t jlevelcap;
    int32_t* jmem;         /* member codes: record >= 0, job j as -1 - j */
    uint32_t njmem, jmemcap;
    uint32_t unmodelled;
    int oom;
} rx_dev;

/* D->ev by packet id: an LSD radix sort of (packet id, position) keys, 4 x 8
 * bits, then one permutation (qsort's comparisons were ~20 % of the device
 * tables' host time at ~900 deliveries a batch); stable */
static int rx_sort_events(rx_dev* D)
{
    const uint32_t n = D->nev;
    uint64_t* k = (uint64_t*)malloc((size_t)n * 2 * sizeof(uint64_t));
    rx_event* tmp = (rx_event*)malloc((size_t)n * sizeof(rx_event));
    if (!k || !tmp) {
        free(k);
        free(tmp);
        return -1;
    }
    uint64_t* src = k;
    uint64_t* dst = k + n;
    for (uint32_t i = 0; i < n; ++i)
        src[i] = (uint64_t)D->ev[i].hdr.seq << 32 | i;
    for (uint32_t sh = 32; sh < 64; sh += 8) {
        uint32_t cnt[257] = {0};
        for (uint32_t i = 0; i < n; ++i)
            cnt[((src[i] >> sh) & 0xFFu) + 1]++;
        for (uint32_t b = 1; b <= 256; ++b)
            cnt[b] += cnt[b - 1];
        for (uint32_t i = 0; i < n; ++i)
            dst[cnt[(src[i] >> sh) & 0xFFu]++] = src[i];
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    for (uint32_t i = 0; i < n; ++i)
        tmp[i] = D->ev[(uint32_t)src[i]];
    memcpy(D->ev, tmp, (size_t)n * sizeof(rx_event));
    free(k);
    free(tmp);
    return 0;
}

static void rx_dev_free(rx_dev* D)
{
    free(D->ev);
    free(D->dl);
    free(D->C);
    free(D->cls);
    free(D->jobs);
    free(D->jlevel);
    free(D->jmem);
    memset(D, 0, sizeof(*D));
}

/* A group recovered by line jobs (rx_line_jobs: above RFEC_MAX_K segments or a
 * huge shape -- a foreign peer's flex): the canonical
 * peel (lines in plan order -- rows, then columns -- to a fixpoint, with
 * flex_fec_recover's header checks, flex_fec_xor.c:60-99) from its arrived
 * members and registered parities, over headers on the host; each firing
 * becomes a line job the device runs (rfec_launch_line_jobs).  job_of[t]: the
 * job recovering member t, or -1.  Returns -1 when out of memory. */
static int rx_big_peel(const rx_sim* X, rx_dev* D, uint32_t gi, int32_t* job_of)
{
    const rx_inst* g = &X->G[gi];
    const rx_shape* sh = &X->S[g->shape];
    const uint32_t k = g->count, NL = sh->n_lines;
    rfec_hdr* hd = (rfec_hdr*)malloc((size_t)k * sizeof(rfec_hdr));
    int32_t* src = (int32_t*)malloc((size_t)k * sizeof(int32_t));
    uint16_t* lvl = (uint16_t*)malloc((size_t)k * sizeof(uint16_t));
    uint8_t* have = (uint8_t*)malloc(k);
    if (!hd || !src || !lvl || !have) {
        free(hd);
        free(src);
        free(lvl);
        free(have);
        return -1;
    }
    for (uint32_t i = 0; i < k; ++i) {
        job_of[i] = -1;
        lvl[i] = 0;
        src[i] = X->slot_src[g->slot0 + i];
        have[i] = src[i] >= 0; /* the peel starts from the arrived members */
        if (have[i])
            hd[i] = X->slot_hdr[g->slot0 + i];
    }
    for (int progress = 1; progress && !D->oom;) {
        progress = 0;
        for (uint32_t l = 0; l < NL && !D->oom; ++l) {
            uint32_t first, stride;
            int reg;
            const uint32_t n = rx_line(X, g, l, &first, &stride, &reg);
            if (!reg)
                continue;
            uint32_t miss = 0, present = 0, t = 0;
            for (uint32_t q = 0; q < n; ++q) {
                const uint32_t i = first + q * stride;
                if (have[i]) {
                    present++;
                } else {
                    miss++;
                    t = i;
                }
            }
            if (miss != 1 || present == 0)
                continue;
            const rfec_wire_rec* f = &X->R[X->line_par[g->line0 + l]];
            const uint32_t L = f->data_size;
            if (L > X->capacity)
                continue;
            rfec_hdr h = f->hdr;
            int ok = 1;
            uint16_t level = 0;
            for (uint32_t q = 0; q < n && ok; ++q) {
                const uint32_t i = first + q * stride;
                if (i == t)
                    continue;
                const rfec_hdr* m = &hd[i];
                ok = m->size <= L;
                h.seq ^= m->seq;
                h.fid ^= m->fid;
                h.ts ^= m->ts;
                h.index ^= m->index;
                h.total ^= m->total;
                h.ftype ^= m->ftype;
                h.payload_type ^= m->payload_type;
                h.size ^= m->size;
                level = lvl[i] > level ? lvl[i] : level;
            }
            if (!ok || h.size > L)
                continue;
            RX_GROW_F(D->oom, D->jobs, D->njobs, D->jobcap, 1, rfec_line_job);
            RX_GROW_F(D->oom, D->jlevel, D->njobs, D->jlevelcap, 1, uint16_t);
            RX_GROW_F(D->oom, D->jmem, D->njmem, D->jmemcap, present, int32_t);
            if (D->oom)
                break;
            rfec_line_job* J = &D->jobs[D->njobs];
            J->out = (int32_t)D->njobs;
            J->parity = X->line_par[g->line0 + l];
            J->member0 = D->njmem;
            J->n_members = present;
            for (uint32_t q = 0; q < n; ++q) {
                const uint32_t i = first + q * stride;
                if (i != t)
                    D->jmem[D->njmem++] = src[i];
            }
            D->jlevel[D->njobs] = (uint16_t)(level + 1);
            job_of[t] = (int32_t)D->njobs;
            src[t] = -1 - (int32_t)D->njobs;
            lvl[t] = (uint16_t)(level + 1);
            hd[t] = h;
            have[t] = 1;
            D->njobs++;
            progress = 1;
        }
    }
    free(hd);
    free(src);
    free(lvl);
    free(have);
    return D->oom ? -1 : 0;
}

#define RX_MAX_LEVEL 256u

/* A group whose device recovery runs as the host peel's line jobs: above
 * RFEC_MAX_K segments (the batched peel's masks hold 128 members), or a huge
 * shape of any count (no device plan: more than RFEC_MAX_LINES lines, e.g. a
 * peer's 128-segment flex of 64 rows x 2 columns, or one rx_extend took past
 * 64 lines; its parity rows sit at a 256-line stride). */
static int rx_line_jobs(const rx_shape* sh) { return sh->count > RFEC_MAX_K || sh->huge; }

static int same_geometry(const rx_shape* a, const rx_shape* b)
{
    return a->count == b->count && a->row == b->row && a->col == b->col && a->xcol[0] == b->xcol[0] &&
           a->xcol[1] == b->xcol[1];
}

/* The device tables of one call (rx_device), for the delivering groups and
 * the deliveries of shard t (UINT32_MAX: all): member and parity row maps,
 * header records, masks, sizes, and each delivery's output row -- the
 * recovering group's dense slot (its rank among the group's erased members)
 * or the line job that recovers it.  Sharded sessions fill them on the
 * replay threads, each over the state its own thread wrote. */
typedef struct {
    rx_sim* const* XS;
    const rx_dev* D;
    const uint32_t* sbase; /* per shard: its first entry in D->cls */
    const int32_t* job_of;
    int32_t* map;
    rfec_hdr *hh, *mh;
    uint16_t* fsz;
    uint64_t *pres, *ppm;
    int32_t* omap;
    uint32_t r_job, r_par, r_dense;
} rx_tabs;

static void rx_fill(const rx_tabs* A, uint32_t only)
{
    const rx_dev* D = A->D;
#define RX_CLS(t, g) (&D->C[D->cls[A->sbase[t] + (g)->shape] - 1])
    for (uint32_t d = 0; d < D->ndl; ++d) {
        const uint32_t t = (uint32_t)(D->dl[d] >> 32);
        if (only != UINT32_MAX && t != only)
            continue;
        const rx_sim* X = A->XS[t];
        const rx_inst* g = &X->G[(uint32_t)D->dl[d]];
        const rx_shape* sh = &X->S[g->shape];
        if (rx_line_jobs(sh))
            continue;
        const rx_dclass* C = RX_CLS(t, g);
        const uint32_t gg = C->group0 + g->gslot, r0 = C->row0 + g->gslot * sh->count;
        const uint32_t p0 = C->prow0 + g->gslot * sh->n_lines;
        A->pres[2 * gg] = g->arrived[0];
        A->pres[2 * gg + 1] = g->arrived[1];
        A->ppm[gg] = g->ppm;
        for (uint32_t i = 0; i < sh->count; ++i) {
            const int32_t src = X->slot_src[g->slot0 + i];
            A->map[r0 + i] = src;
            if (src >= 0)
                A->hh[r0 + i] = X->slot_hdr[g->slot0 + i];
            else
                memset(&A->hh[r0 + i], 0, sizeof(rfec_hdr));
        }
        for (uint32_t l = 0; l < sh->n_lines; ++l) {
            const int32_t src = X->line_par[g->line0 + l];
            A->map[A->r_par + p0 + l] = src;
            if (src >= 0) {
                A->mh[p0 + l] = X->R[src].hdr;
                A->fsz[p0 + l] = X->R[src].data_size;
            } else {
                memset(&A->mh[p0 + l], 0, sizeof(rfec_hdr));
                A->fsz[p0 + l] = 0;
            }
        }
    }
    for (uint32_t q = 0; q < D->nev; ++q) {
        const rx_event* ev = &D->ev[q];
        if (only != UINT32_MAX && ev->shard != only)
            continue;
        const rx_sim* X = A->XS[ev->shard];
        const rx_inst* g = &X->G[ev->inst];
        const rx_shape* sh = &X->S[g->shape];
        const uint32_t t = ev->hdr.seq - g->base;
        if (rx_line_jobs(sh)) { /* the job that recovers t */
            A->omap[q] = t < g->count && A->job_of[g->gslot + t] >= 0
                             ? (int32_t)(A->r_job + (uint32_t)A->job_of[g->gslot + t]) : -1;
            continue;
        }
        const rx_dclass* C = RX_CLS(ev->shard, g);
        uint32_t e = UINT32_MAX;
        if (t < g->count && !((g->arrived[t >> 6] >> (t & 63)) & 1ull)) {
            const uint64_t lo = t >= 64 ? ~g->arrived[0] : ~g->arrived[0] & ((1ull << t) - 1);
            const uint64_t hi = t >= 64 ? ~g->arrived[1] & ((1ull << (t - 64)) - 1) : 0;
            e = (uint32_t)(__builtin_popcountll(lo) + __builtin_popcountll(hi));
        }
        A->omap[q] = e < C->E ? (int32_t)(A->r_dense + C->dense0 + g->gslot * C->E + e) : -1;
    }
#undef RX_CLS
}

static void rx_fill_job(void* arg, uint32_t t) { rx_fill((const rx_tabs*)arg, t); }

typedef struct rx_pool rx_pool;
static void pool_run(rx_pool* P, void (*fn)(void*, uint32_t), void* arg);

/* The device side of one call: the groups that delivered something in this
 * call (over the T shards XS), rebuilt from their arrived members and
 * registered parities (rows of `rows`, DEVICE, indexed by record), peeled by
 * rfec_recover_batch, and the delivered rows copied out.  The pinned tables
 * go after the first `hoff` bytes of t_rx.h, which survive a grow (the
 * shards' R may live there: `r_stage`). */
static int rx_device(rx_sim* const* XS, uint32_t T, rx_pool* pool, rx_dev* D, const uint8_t* rows, uint32_t stride,
                     uint32_t capacity, size_t hoff, int r_stage, rfec_rx_seg* out, uint8_t* out_payload,
                     uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep, hipStream_t sm)
{
    hipError_t e = hipSuccess;
    int rc = RFEC_OK, ke = 0;
    const double th = now_us();
    *n_out = 0;
    D->nev = D->ndl = D->nc = D->njobs = D->njmem = 0;
    /* 1. the deliveries of every shard, ascending packet id */
    uint32_t total = 0, nshape = 0;
    for (uint32_t t = 0; t < T; ++t) {
        total += XS[t]->nout;
        nshape += XS[t]->ns;
    }
    if (total == 0) { /* nothing recovered: no device work */
        rep->host_us += now_us() - th;
        return RFEC_OK;
    }
    RX_GROW_F(D->oom, D->ev, 0, D->evcap, total, rx_event);
    RX_GROW_F(D->oom, D->cls, 0, D->clscap, nshape + 1, uint32_t);
    if (D->oom)
        return set_err(RFEC_ENOMEM, "rx: delivery list", 0);
    uint32_t sbase[RX_MAX_THREADS + 1];
    sbase[0] = 0;
    for (uint32_t t = 0; t < T; ++t) {
        const rx_sim* X = XS[t];
        for (uint32_t q = 0; q < X->nout; ++q) {
            D->ev[D->nev] = X->out[q];
            D->ev[D->nev++].shard = t;
        }
        sbase[t + 1] = sbase[t] + X->ns;
    }
    if (D->nev > 1 && rx_sort_events(D)) /* ascending packet id (each shard's list is in its arrival order) */
        return set_err(RFEC_ENOMEM, "rx: delivery list", 0);
    memset(D->cls, 0, (size_t)nshape * sizeof(uint32_t));
    /* 2. delivering groups, by device shape (work proportional to the deliveries, not to the open flexes) */
    for (uint32_t t = 0; t < T; ++t) {
        rx_sim* X = XS[t];
        if (++X->epoch == 0) { /* wrapped: no instance may carry a stale stamp */
            for (uint32_t gi = 0; gi < X->ng; ++gi)
                X->G[gi].gstamp = 0;
            X->epoch = 1;
        }
    }
    for (uint32_t q = 0; q < D->nev; ++q) {
        rx_sim* X = XS[D->ev[q].shard];
        rx_inst* g = &X->G[D->ev[q].inst];
        if (g->gstamp == X->epoch)
            continue;
        g->gstamp = X->epoch;
        RX_GROW_F(D->oom, D->dl, D->ndl, D->dlcap, 1, uint64_t);
        if (D->oom)
            return set_err(RFEC_ENOMEM, "rx: delivery list", 0);
        D->dl[D->ndl++] = (uint64_t)D->ev[q].shard << 32 | D->ev[q].inst;
        uint32_t* c = &D->cls[sbase[D->ev[q].shard] + g->shape];
        if (!*c) { /* this shard's shape: an existing device shape of the same geometry, or a new one */
            const rx_shape* sh = &X->S[g->shape];
            uint32_t k = 0;
            while (k < D->nc && !same_geometry(D->C[k].sh, sh))
                ++k;
            if (k == D->nc) {
                RX_GROW_F(D->oom, D->C, D->nc, D->ccap, 1, rx_dclass);
                if (D->oom)
                    return set_err(RFEC_ENOMEM, "rx: device shapes", 0);
                D->C[D->nc++] = (rx_dclass){sh, 0, 0, 0, 0, 0, 0};
            }
            *c = k + 1;
        }
        g->gslot = D->C[*c - 1].n_groups++;
    }
    uint32_t nrows = 0, prows = 0, ngs = 0;
    for (uint32_t k = 0; k < D->nc; ++k) {
        rx_dclass* C = &D->C[k];
        C->row0 = nrows;
        C->prow0 = prows;
        C->group0 = ngs;
        if (rx_line_jobs(C->sh)) /* line jobs instead (below) */
            continue;
        nrows += C->n_groups * C->sh->count;
        prows += C->n_groups * C->sh->n_lines;
        ngs += C->n_groups;
    }
#define RX_CLASS(t, g) (&D->C[D->cls[sbase[t] + (g)->shape] - 1])
    /* groups above RFEC_MAX_K: the host peel's line jobs, output rows after
     * the batched peel's rows, launched level by level (jobs sorted by level) */
    uint32_t nbig = 0, maxlvl = 0;
    for (uint32_t d = 0; d < D->ndl; ++d) {
        const rx_sim* X = XS[D->dl[d] >> 32];
        const rx_inst* g = &X->G[(uint32_t)D->dl[d]];
        if (rx_line_jobs(&X->S[g->shape]))
            nbig += g->count;
    }
    int32_t* job_of = nbig ? (int32_t*)malloc((size_t)nbig * sizeof(int32_t)) : NULL;
    uint32_t* jperm = NULL;
    if (nbig && !job_of)
        return set_err(RFEC_ENOMEM, "rx: large groups", 0);
    for (uint32_t d = 0, off = 0; d < D->ndl; ++d) {
        rx_sim* X = XS[D->dl[d] >> 32];
        rx_inst* g = &X->G[(uint32_t)D->dl[d]];
        if (!rx_line_jobs(&X->S[g->shape]))
            continue;
        g->gslot = off; /* (a large group's slot: its job_of range) */
        if (rx_big_peel(X, D, (uint32_t)D->dl[d], job_of + off))
            D->oom = 1;
        off += g->count;
    }
    if (D->oom) {
        free(job_of);
        return set_err(RFEC_ENOMEM, "rx: line jobs", 0);
    }
    /* a line fires at most once, so a chain is at most as deep as a group has lines (256 FEC indices) */
    uint32_t lvl_n[RX_MAX_LEVEL + 1] = {0};
    if (D->njobs) { /* stable sort by level; codes and job_of follow */
        for (uint32_t j = 0; j < D->njobs; ++j) {
            if (D->jlevel[j] > RX_MAX_LEVEL) {
                free(job_of);
                return set_err(RFEC_EINVAL, "rx: line job chain too deep", 0);
            }
            maxlvl = D->jlevel[j] > maxlvl ? D->jlevel[j] : maxlvl;
            lvl_n[D->jlevel[j]]++;
        }
        uint32_t start[RX_MAX_LEVEL + 2] = {0};
        for (uint32_t v = 1; v <= maxlvl; ++v)
            start[v + 1] = start[v] + lvl_n[v];
        jperm = (uint32_t*)malloc((size_t)D->njobs * sizeof(uint32_t));
        rfec_line_job* sorted = (rfec_line_job*)malloc((size_t)D->njobs * sizeof(rfec_line_job));
        if (!jperm || !sorted) {
            free(jperm);
            free(sorted);
            free(job_of);
            return set_err(RFEC_ENOMEM, "rx: line jobs", 0);
        }
        for (uint32_t j = 0; j < D->njobs; ++j)
            jperm[j] = start[D->jlevel[j]]++;
        for (uint32_t j = 0; j < D->njobs; ++j) {
            sorted[jperm[j]] = D->jobs[j];
            sorted[jperm[j]].out = (int32_t)jperm[j];
        }
        memcpy(D->jobs, sorted, (size_t)D->njobs * sizeof(rfec_line_job));
        free(sorted);
        for (uint32_t m = 0; m < D->njmem; ++m)
            if (D->jmem[m] < 0)
                D->jmem[m] = -1 - (int32_t)jperm[-1 - D->jmem[m]];
        for (uint32_t i = 0; i < nbig; ++i)
            if (job_of[i] >= 0)
                job_of[i] = (int32_t)jperm[job_of[i]];
    }
    /* dense output per device shape: E slots per group, the shape's largest erasure count among its
       delivering groups (the e-th erased member of a group, index order, goes to slot e) */
    for (uint32_t k = 0; k < D->nc; ++k)
        D->C[k].E = 0;
    for (uint32_t d = 0; d < D->ndl; ++d) {
        const uint32_t t = (uint32_t)(D->dl[d] >> 32);
        const rx_sim* X = XS[t];
        const rx_inst* g = &X->G[(uint32_t)D->dl[d]];
        if (rx_line_jobs(&X->S[g->shape]))
            continue;
        rx_dclass* C = RX_CLASS(t, g);
        const uint32_t er = g->count - (uint32_t)(__builtin_popcountll(g->arrived[0]) + __builtin_popcountll(g->arrived[1]));
        C->E = er > C->E ? er : C->E;
    }
    uint32_t ndense = 0;
    for (uint32_t k = 0; k < D->nc; ++k) {
        rx_dclass* C = &D->C[k];
        if (rx_line_jobs(C->sh) || !C->n_groups)
            continue;
        C->E = C->E < 1 ? 1 : C->E > C->sh->count ? C->sh->count : C->E;
        C->dense0 = ndense;
        ndense += C->n_groups * C->E;
    }
    /* rows on the device, one region: [nrows members][njobs line-job outputs][prows parities][ndense] */
    const uint32_t r_job = nrows, r_par = nrows + D->njobs, r_dense = r_par + prows, nmap = r_dense;
    const size_t o_map = 0, o_hdr = RX_ALIGN((size_t)nmap * 4);
    const size_t o_meta = RX_ALIGN(o_hdr + (size_t)nrows * sizeof(rfec_hdr));
    const size_t o_fs = RX_ALIGN(o_meta + (size_t)prows * sizeof(rfec_hdr));
    const size_t o_pres = RX_ALIGN(o_fs + (size_t)prows * 2), o_pp = RX_ALIGN(o_pres + (size_t)ngs * 16);
    const size_t o_omap = RX_ALIGN(o_pp + (size_t)ngs * 8), o_jobs = RX_ALIGN(o_omap + (size_t)D->nev * 4);
    const size_t o_jmem = RX_ALIGN(o_jobs + (size_t)D->njobs * sizeof(rfec_line_job));
    const size_t o_in_end = RX_ALIGN(o_jmem + (size_t)D->njmem * 4);
    const size_t o_rec = o_in_end, host_bytes = RX_ALIGN(o_rec + (size_t)ngs * 16);
    size_t ws_bytes = 0;
    for (uint32_t k = 0; k < D->nc; ++k)
        if (!rx_line_jobs(D->C[k].sh))
            ws_bytes += RX_ALIGN(rfec_recover_workspace_size(&D->C[k].sh->plan, D->C[k].n_groups));
    const size_t d_rows = o_in_end, d_ws = RX_ALIGN(d_rows + ((size_t)r_dense + ndense) * stride);
    const size_t d_ohdr = RX_ALIGN(d_ws + ws_bytes), d_oidx = RX_ALIGN(d_ohdr + (size_t)ndense * sizeof(rfec_hdr));
    const size_t d_out = RX_ALIGN(d_oidx + ndense), dev_bytes = RX_ALIGN(d_out + (size_t)D->nev * stride);
    if ((rc = rx_reserve(hoff + host_bytes, dev_bytes, hoff))) {
        free(job_of);
        free(jperm);
        return rc;
    }
    if (r_stage) /* the records live at the start of the pinned block, which may have moved */
        for (uint32_t t = 0; t < T; ++t)
            XS[t]->R = (const rfec_wire_rec*)t_rx.h;
    uint8_t* H = t_rx.h + hoff;
    uint8_t* Hd = t_rx.hd + hoff; /* H as the device addresses it */
    int32_t* map = (int32_t*)(H + o_map);
    rfec_hdr* hh = (rfec_hdr*)(H + o_hdr);
    rfec_hdr* mh = (rfec_hdr*)(H + o_meta);
    uint16_t* fsz = (uint16_t*)(H + o_fs);
    uint64_t* pres = (uint64_t*)(H + o_pres);
    uint64_t* ppm = (uint64_t*)(H + o_pp);
    int32_t* omap = (int32_t*)(H + o_omap);
    for (uint32_t j = 0; j < D->njobs; ++j)
        map[r_job + j] = -1;
    if (D->njobs) {
        memcpy(H + o_jobs, D->jobs, (size_t)D->njobs * sizeof(rfec_line_job));
        memcpy(H + o_jmem, D->jmem, (size_t)D->njmem * 4);
    }
    rx_tabs A = {XS, D, sbase, job_of, map, hh, mh, fsz, pres, ppm, omap, r_job, r_par, r_dense};
    if (pool && T > 1)
        pool_run(pool, rx_fill_job, &A); /* each shard's groups by the thread that replayed them */
    else
        rx_fill(&A, UINT32_MAX);
    uint32_t nok = 0;
    free(job_of);
    free(jperm);
    rep->host_us += now_us() - th;
    rep->n_groups = ngs;
    for (uint32_t k = 0; k < D->nc; ++k)
        rep->n_shapes += D->C[k].n_groups != 0;
    /* the device: rows and tables staged in one launch, one dense peel per device shape writing its
       recovered masks into pinned memory, the delivered rows gathered out; one synchronisation */
    uint8_t* Dv = t_rx.d;
    uint8_t* rows_d = Dv + d_rows;
    double tt = now_us();
    ke = rfec_launch_rx_stage(rows_d, rows, (const int32_t*)(Hd + o_map), nmap, stride, Dv, Hd, o_in_end, sm);
    for (uint32_t v = 1, lo = 0; v <= maxlvl && !ke; lo += lvl_n[v], ++v) /* the large groups' line jobs */
        ke = rfec_launch_line_jobs((const rfec_line_job*)(Dv + o_jobs) + lo, lvl_n[v], (const int32_t*)(Dv + o_jmem),
                                   rows, rows_d + (size_t)r_job * stride, stride, sm);
    size_t wso = 0;
    uint64_t* rec_d = (uint64_t*)(Hd + o_rec);
    for (uint32_t k = 0; k < D->nc && !ke; ++k) {
        const rx_dclass* C = &D->C[k];
        if (!C->n_groups || rx_line_jobs(C->sh))
            continue;
        rfec_kmask M;
        make_masks(&C->sh->plan, &M);
        const rfec_dense_out DO = {rows_d + ((size_t)r_dense + C->dense0) * stride,
                                   (rfec_hdr*)(Dv + d_ohdr) + C->dense0, Dv + d_oidx + C->dense0, C->E};
        ke = rfec_launch_recover_out(&M, C->n_groups, stride, capacity, rows_d + (size_t)C->row0 * stride,
                                     (const rfec_hdr*)(Dv + o_hdr) + C->row0, (const uint64_t*)(Dv + o_pres) + 2 * C->group0,
                                     rows_d + ((size_t)r_par + C->prow0) * stride, (const rfec_hdr*)(Dv + o_meta) + C->prow0,
                                     (const uint16_t*)(Dv + o_fs) + C->prow0, (const uint64_t*)(Dv + o_pp) + C->group0,
                                     rec_d + 2 * C->group0, Dv + d_ws + wso, sm, g_tuning, &DO);
        wso += RX_ALIGN(rfec_recover_workspace_size(&C->sh->plan, C->n_groups));
    }
    /* delivered rows: straight into the caller's output when it is pinned and
       large enough (no second round trip; rows the peel did not cover are
       squeezed out on the host below), else into the device staging */
    uint8_t* outd = D->nev && D->nev <= max_out ? (uint8_t*)host_mapped(out_payload) : NULL;
    if (!ke && D->nev)
        ke = rfec_launch_gather_rows(outd ? outd : Dv + d_out, rows_d, (const int32_t*)(Dv + o_omap), D->nev, stride,
                                     sm);
    uint64_t* rec = (uint64_t*)(H + o_rec);
    if (ke || (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: recover", ke ? ke : (int)e);
    rep->kernel_us += now_us() - tt;
    /* the device peel covers every packet the arrival-order pass delivered (same lines, a superset of
       the members at each firing); anything else is reported, not delivered */
    for (uint32_t q = 0; q < D->nev; ++q) {
        const rx_event* ev = &D->ev[q];
        const rx_sim* X = XS[ev->shard];
        const rx_inst* g = &X->G[ev->inst];
        const int big = rx_line_jobs(&X->S[g->shape]);
        const uint32_t t = ev->hdr.seq - g->base;
        const uint32_t gg = big ? 0 : RX_CLASS(ev->shard, g)->group0 + g->gslot;
        if (omap[q] < 0 || (!big && !((rec[2 * gg + (t >> 6)] >> (t & 63)) & 1ull))) {
            D->unmodelled++;
            omap[q] = -1;
            continue;
        }
        nok++;
    }
#undef RX_CLASS
    if (nok > max_out) {
        *n_out = nok;
        return set_err(RFEC_EINVAL, "rx: output too small", 0);
    }
    tt = now_us();
    uint32_t o = 0;
    if (outd) { /* the rows are in out_payload already (the sync above) */
        for (uint32_t q = 0; q < D->nev; ++q) {
            if (omap[q] < 0)
                continue;
            if (o != q)
                memmove(out_payload + (size_t)o * stride, out_payload + (size_t)q * stride, stride);
            D->ev[o++] = D->ev[q];
        }
    } else if (nok == D->nev) { /* the usual case: one copy */
        if (nok)
            e = hipMemcpyAsync(out_payload, Dv + d_out, (size_t)nok * stride, hipMemcpyDeviceToHost, sm);
        o = nok;
    }
    for (uint32_t q = 0; q < D->nev && !outd && nok != D->nev && e == hipSuccess; ++q) {
        if (omap[q] < 0)
            continue;
        e = hipMemcpyAsync(out_payload + (size_t)o * stride, Dv + d_out + (size_t)q * stride, stride,
                           hipMemcpyDeviceToHost, sm);
        D->ev[o++] = D->ev[q];
    }
    for (uint32_t q = 0; q < o; ++q) {
        out[q].hdr = D->ev[q].hdr;
        out[q].fec_id = (uint16_t)XS[D->ev[q].shard]->G[D->ev[q].inst].fec_id;
        out[q].reserved = 0;
    }
    if (e == hipSuccess && !outd)
        e = hipStreamSynchronize(sm);
    if (e != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: output D2H", e);
    rep->d2h_us += now_us() - tt;
    *n_out = o;
    rep->n_recovered = o;
    return RFEC_OK;
}

int rfec_rx_recover(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                    uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out,
                    uint32_t* n_out, rfec_rx_report* rep, void* stream)
{
    const double t0 = now_us();
    if (!max_ts || !n_out || !rep || (n && (!recs || !payload)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx: bad argument", 0);
    if (stride == 0 || stride % 16 || capacity > stride)
        return set_err(RFEC_EINVAL, "rx: stride must be a multiple of 16 and >= capacity", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    hipStream_t sm = (hipStream_t)stream;
    hipError_t e;
    int rc = RFEC_OK;
    /* 1. the records to the host (headers only: 64 B each) */
    const size_t rec_bytes = RX_ALIGN((size_t)n * sizeof(rfec_wire_rec));
    if ((rc = rx_reserve(rec_bytes, 0, 0)))
        return rc;
    double tt = now_us();
    if ((e = hipMemcpyAsync(t_rx.h, recs, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost, sm)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx: records D2H", e);
    rep->d2h_us += now_us() - tt;
    /* 2. the control plane, in arrival order */
    const double th = now_us();
    rx_sim X;
    memset(&X, 0, sizeof(X));
    X.R = (const rfec_wire_rec*)t_rx.h;
    X.capacity = capacity;
    X.max_ts = *max_ts;
    if (rx_tables_init(&X, n)) {
        rx_sim_free(&X);
        return set_err(RFEC_ENOMEM, "rx: host tables", 0);
    }
    rx_run(&X, 0, n);
    if (X.oom) {
        rx_sim_free(&X);
        return set_err(RFEC_ENOMEM, "rx: host tables", 0);
    }
    *max_ts = X.max_ts;
    rep->n_fec_dropped = X.dropped;
    rep->host_us += now_us() - th;
    /* 3. the device: the records stay at the start of the pinned block */
    rx_sim* XS[1] = {&X};
    rx_dev D;
    memset(&D, 0, sizeof(D));
    rc = rx_device(XS, 1, NULL, &D, payload, stride, capacity, rec_bytes, 1, out, out_payload, max_out, n_out, rep,
                   sm);
    rep->n_unmodelled = X.unmodelled + D.unmodelled;
    rx_dev_free(&D);
    rx_sim_free(&X);
    rep->total_us = now_us() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Received datagrams (host) -> recovered segments (host)                    */
/* ------------------------------------------------------------------------ */
/* rfec_pinned_alloc / rfec_pinned_free: rfec_hostmem.c (the registry of pinned blocks the device maps) */

typedef struct {
    uint8_t* d;
    size_t db;
    hipStream_t sm;
} rv_ctx;
static __thread rv_ctx t_rv;

int rfec_host_recv_datagrams(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                             uint32_t stride, uint32_t capacity, uint32_t* max_ts, rfec_wire_rec* recs_out,
                             rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                             rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!max_ts || !n_out || !rep || (n && (!dgram || !dlen)))
        return set_err(RFEC_EINVAL, "recv: bad argument", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    if (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16 || stride == 0 || stride % 16 ||
        capacity > stride)
        return set_err(RFEC_EINVAL, "recv: dstride must be a multiple of 16 in [64, 2048], stride >= capacity", 0);
    hipError_t e;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    const size_t o_dl = RX_ALIGN((size_t)n * dstride), o_rec = RX_ALIGN(o_dl + (size_t)n * 2);
    const size_t o_pay = RX_ALIGN(o_rec + (size_t)n * sizeof(rfec_wire_rec));
    const size_t need = RX_ALIGN(o_pay + (size_t)n * stride);
    if (t_rv.db < need) {
        if (t_rv.d)
            (void)hipFree(t_rv.d);
        t_rv.d = NULL;
        t_rv.db = 0;
        const size_t b = need + need / 4;
        if ((e = hipMalloc((void**)&t_rv.d, b)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "recv: device staging", e);
        t_rv.db = b;
    }
    uint8_t* D = t_rv.d;
    double tt = now_us();
    if ((e = hipMemcpyAsync(D, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
        (e = hipMemcpyAsync(D + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
        (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: datagrams H2D", e);
    const double h2d = now_us() - tt;
    tt = now_us();
    int ke = rfec_launch_wire_parse(n, dstride, D, (const uint16_t*)(D + o_dl), stride, capacity,
                                    (rfec_wire_rec*)(D + o_rec), D + o_pay, max_dlen(dlen, n), t_rv.sm);
    if (ke || (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: parse", ke ? ke : (int)e);
    const double parse = now_us() - tt;
    if (recs_out) {
        tt = now_us();
        if ((e = hipMemcpyAsync(recs_out, D + o_rec, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost,
                                t_rv.sm)) != hipSuccess ||
            (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "recv: records D2H", e);
        rep->d2h_us += now_us() - tt;
    }
    const double d2h_recs = rep->d2h_us;
    const int rc = rfec_rx_recover(n, (const rfec_wire_rec*)(D + o_rec), D + o_pay, stride, capacity, max_ts, out,
                                   out_payload, max_out, n_out, rep, t_rv.sm);
    rep->h2d_us += h2d;
    rep->kernel_us += parse;
    rep->d2h_us += d2h_recs;
    rep->total_us = now_us() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Receiver session: the control plane kept across calls, sharded by fec_id   */
/* (above: rx_owners, the journal) over T shards replayed by a thread pool;   */
/* records by id in a host store, their payload rows by id in an HBM arena    */
/* ------------------------------------------------------------------------ */
/* a batch of the pipelined push: its parse in flight on the session's stream */
typedef struct {
    rfec_rx_split* sum;  /* pinned, device-mapped: the batch's split summary (k_rx_split) */
    rfec_rx_split* sumd; /* sum as the device addresses it */
    uint32_t sumcap;
    uint8_t* dg; /* device copy of pageable datagram slots + lengths */
    size_t dgb;
    hipEvent_t done;
} rx_stage;

/* The replay threads: T - 1 workers beside the calling thread, woken per
 * batch (a generation counter; a short spin, then a condition variable). */
typedef struct {
    rx_pool* pool;
    uint32_t idx;
} rx_worker;
struct rx_pool {
    pthread_t th[RX_MAX_THREADS];
    rx_worker w[RX_MAX_THREADS];
    uint32_t nth; /* workers started */
    uint32_t base; /* the first worker's index: 1 (the caller runs fn(arg, 0)) or 0 (workers run every index) */
    pthread_mutex_t mu;
    pthread_cond_t go, fin;
    uint32_t gen, done; /* atomics */
    int stop;
    void (*fn)(void*, uint32_t);
    void* arg;
};

/* how long a worker (or the caller) spins before sleeping on the condition
 * variable: RFEC_RX_SPIN_US, default 50 us (spinning threads share the
 * process's CPU quota and cores with the caller's serial work) */
static double rx_spin_us(void)
{
    static double v = -1.0;
    if (v < 0) {
        const char* e = getenv("RFEC_RX_SPIN_US");
        v = e ? atof(e) : 50.0;
    }
    return v;
}
#define RX_SPIN_US rx_spin_us()

static void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

static void* pool_main(void* p)
{
    rx_worker* W = (rx_worker*)p;
    rx_pool* P = W->pool;
    uint32_t seen = 0;
    for (;;) {
        const double t0 = now_us();
        for (uint32_t i = 0; __atomic_load_n(&P->gen, __ATOMIC_ACQUIRE) == seen && !P->stop; ++i) {
            cpu_relax();
            if ((i & 63) == 63 && now_us() - t0 > RX_SPIN_US) {
                pthread_mutex_lock(&P->mu);
                while (__atomic_load_n(&P->gen, __ATOMIC_ACQUIRE) == seen && !P->stop)
                    pthread_cond_wait(&P->go, &P->mu);
                pthread_mutex_unlock(&P->mu);
            }
        }
        if (P->stop)
            return NULL;
        seen = __atomic_load_n(&P->gen, __ATOMIC_ACQUIRE);
        P->fn(P->arg, W->idx);
        if (__atomic_add_fetch(&P->done, 1u, __ATOMIC_ACQ_REL) == P->nth) {
            pthread_mutex_lock(&P->mu);
            pthread_cond_broadcast(&P->fin);
            pthread_mutex_unlock(&P->mu);
        }
    }
}

/* The CPUs the replay threads run on: RFEC_RX_CPUS ("a-b,c,..."), else those
 * sharing the last-level cache with the creating thread's CPU (one CCD of an
 * EPYC: the records, the shards and the device tables pass between the
 * threads through that L3; across CCDs every such line is a fabric round
 * trip, and the replay ran slower in parallel than alone), within the
 * process's affinity.  RFEC_RX_PIN=0: no placement.  0 when nothing applies. */
static int parse_cpus(const char* s, cpu_set_t* set)
{
    CPU_ZERO(set);
    int n = 0;
    while (s && *s) {
        char* e;
        long a = strtol(s, &e, 10), b = a;
        if (e == s)
            break;
        if (*e == '-')
            b = strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c, ++n)
            CPU_SET((int)c, set);
        s = *e == ',' ? e + 1 : e;
        if (*s == '\n')
            break;
    }
    return n;
}

static int rx_worker_cpus(cpu_set_t* set)
{
    const char* pin = getenv("RFEC_RX_PIN");
    if (pin && pin[0] == '0')
        return 0;
    const char* cpus = getenv("RFEC_RX_CPUS");
    if (cpus)
        return parse_cpus(cpus, set) > 0;
    const int cpu = sched_getcpu();
    if (cpu < 0)
        return 0;
    char path[96], buf[512];
    snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
    FILE* f = fopen(path, "r");
    if (!f)
        return 0;
    const int ok = fgets(buf, sizeof(buf), f) != NULL;
    fclose(f);
    if (!ok || parse_cpus(buf, set) < 2)
        return 0;
    cpu_set_t mine;
    if (pthread_getaffinity_np(pthread_self(), sizeof(mine), &mine))
        return 0;
    CPU_AND(set, set, &mine);
    return CPU_COUNT(set) >= 2;
}

static int pool_start(rx_pool* P, uint32_t workers, uint32_t base)
{
    memset(P, 0, sizeof(*P));
    P->base = base;
    pthread_mutex_init(&P->mu, NULL);
    pthread_cond_init(&P->go, NULL);
    pthread_cond_init(&P->fin, NULL);
    cpu_set_t cpus;
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    /* one CPU per worker, in the set's order (a CCD's physical cores come first in its list), so a shard's
       state stays in one core's L2 from batch to batch; the set as a whole if it has fewer CPUs */
    int list[CPU_SETSIZE], ncpu = 0;
    const int pinned = rx_worker_cpus(&cpus);
    for (int c = 0; pinned && c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &cpus))
            list[ncpu++] = c;
    for (uint32_t i = 0; i < workers; ++i) {
        if (pinned) {
            cpu_set_t one;
            CPU_ZERO(&one);
            if ((uint32_t)ncpu >= workers + P->base)
                CPU_SET(list[i + P->base], &one);
            else
                one = cpus;
            pthread_attr_setaffinity_np(&attr, sizeof(one), &one);
        }
        P->w[i] = (rx_worker){P, i + P->base};
        if (pthread_create(&P->th[i], &attr, pool_main, &P->w[i])) {
            pthread_attr_destroy(&attr);
            return -1;
        }
        P->nth = i + 1;
    }
    pthread_attr_destroy(&attr);
    return 0;
}

static void pool_stop(rx_pool* P)
{
    pthread_mutex_lock(&P->mu);
    P->stop = 1;
    pthread_cond_broadcast(&P->go);
    pthread_mutex_unlock(&P->mu);
    for (uint32_t i = 0; i < P->nth; ++i)
        pthread_join(P->th[i], NULL);
    pthread_mutex_destroy(&P->mu);
    pthread_cond_destroy(&P->go);
    pthread_cond_destroy(&P->fin);
    P->nth = 0;
}

/* fn(arg, 0) here (base 1) and fn(arg, i) on the workers; returns when all are done */
static void pool_run(rx_pool* P, void (*fn)(void*, uint32_t), void* arg)
{
    P->fn = fn;
    P->arg = arg;
    __atomic_store_n(&P->done, 0u, __ATOMIC_RELEASE);
    pthread_mutex_lock(&P->mu);
    __atomic_add_fetch(&P->gen, 1u, __ATOMIC_ACQ_REL);
    pthread_cond_broadcast(&P->go);
    pthread_mutex_unlock(&P->mu);
    if (P->base)
        fn(arg, 0);
    const double t0 = now_us();
    for (uint32_t i = 0; __atomic_load_n(&P->done, __ATOMIC_ACQUIRE) < P->nth; ++i) {
        cpu_relax();
        if ((i & 63) == 63 && now_us() - t0 > RX_SPIN_US) {
            pthread_mutex_lock(&P->mu);
            while (__atomic_load_n(&P->done, __ATOMIC_ACQUIRE) < P->nth)
                pthread_cond_wait(&P->fin, &P->mu);
            pthread_mutex_unlock(&P->mu);
        }
    }
}

struct rfec_rx_session {
    rx_sim* XS[RX_MAX_THREADS]; /* the shards: fec_id % T (T = 1: one serial state) */
    uint32_t T;
    uint32_t max_ts;            /* sim_receiver_fec_t.max_ts, over the shards */
    rx_pool pool;
    int pool_on;
    pmap vown[RX_MAX_THREADS];  /* sharded: packet id -> fec_id + 1, partition (seq >> 8) % T */
    int vown_on;
    rx_par par;
    uint8_t* pshard;            /* per batch record: its shard (0xFF: no control-plane effect) */
    uint32_t* lst;              /* per shard, its records of the batch in arrival order */
    uint32_t* smin;
    uint32_t lcap;
    uint32_t loff[RX_MAX_THREADS + 1];
    uint8_t shard_of[65536];    /* fec_id % T (no division per record) */
    uint32_t n_parallel, n_serial, n_rollback; /* batches by replay (rfec_rx_session_info) */
    double t_split, t_replay, t_verify, t_tables, t_compact; /* host time split (rfec_rx_session_info) */
    rx_dev dev;
    rfec_wire_rec* store;   /* every shard's R: pinned, the parse writes the records straight in */
    rfec_wire_rec* store_d; /* store as the device addresses it */
    uint32_t nstore, storecap;
    uint8_t* arena; /* [arows][stride]: rows [0, nstore) ingested, then the pending batch's */
    uint32_t arows;
    uint8_t* spare; /* the previous arena ([sprows][stride]): the next compaction's target when large enough */
    uint32_t sprows;
    int32_t* dmap;  /* compaction's row map on the device, [dmapcap] */
    uint32_t dmapcap;
    uint32_t stride, capacity;
    /* pipelined push (rfec_rx_session_push_datagrams_async) */
    hipStream_t sa;
    rx_stage st[2];
    uint32_t pend_n; /* rows of the pending batch (arena rows [nstore, nstore + pend_n)) */
    int pend;        /* its stage, -1: none */
};

/* a shard's state on cache lines of its own: the replay threads write their
 * shard's counters on every record (two shards on one line ping-pong it) */
static rx_sim* rx_sim_alloc(void)
{
    const size_t sz = (sizeof(rx_sim) + 127) & ~(size_t)127;
    void* p = NULL;
    if (posix_memalign(&p, 128, sz))
        return NULL;
    memset(p, 0, sz);
    return (rx_sim*)p;
}

static int rx_compact(rfec_rx_session* S, uint32_t extra, hipStream_t sm);

static void rx_shards_free(rfec_rx_session* S)
{
    for (uint32_t t = 0; t < S->T; ++t)
        if (S->XS[t]) {
            rx_sim_free(S->XS[t]);
            free(S->XS[t]);
            S->XS[t] = NULL;
        }
}

/* T empty shards (and, for T > 1, the replay threads) */
static int rx_shards_init(rfec_rx_session* S, uint32_t T)
{
    if (S->pool_on) {
        pool_stop(&S->pool);
        S->pool_on = 0;
    }
    rx_shards_free(S);
    S->T = T;
    for (uint32_t f = 0; f < 65536; ++f)
        S->shard_of[f] = (uint8_t)(f % T);
    for (uint32_t t = 0; t < T; ++t) {
        rx_sim* X = rx_sim_alloc();
        S->XS[t] = X;
        if (!X || rx_tables_init(X, 1024))
            return -1;
        X->capacity = S->capacity;
    }
    if (T > 1) {
        /* RFEC_RX_CALLER=0: the calling thread replays no shard (every shard on the pinned workers, which
           share one last-level cache; the caller may run elsewhere) */
        const char* c = getenv("RFEC_RX_CALLER");
        const uint32_t base = c && c[0] == '0' ? 0u : 1u;
        if (pool_start(&S->pool, T - base, base)) {
            S->pool_on = 1;
            return -1;
        }
        S->pool_on = 1;
    }
    return 0;
}

static uint32_t rx_default_threads(void)
{
    const char* v = getenv("RFEC_RX_THREADS");
    const int t = v ? atoi(v) : 8;
    return t < 1 ? 1u : t > RX_MAX_THREADS ? (uint32_t)RX_MAX_THREADS : (uint32_t)t;
}

rfec_rx_session* rfec_rx_session_create(uint32_t stride, uint32_t capacity)
{
    if (stride == 0 || stride % 16 || capacity > stride) {
        set_err(RFEC_EINVAL, "rx session: stride must be a multiple of 16 and >= capacity", 0);
        return NULL;
    }
    rfec_rx_session* s = (rfec_rx_session*)calloc(1, sizeof(*s));
    if (!s) {
        set_err(RFEC_ENOMEM, "rx session", 0);
        return NULL;
    }
    s->stride = stride;
    s->capacity = capacity;
    s->pend = -1;
    if (rx_shards_init(s, rx_default_threads())) {
        rfec_rx_session_destroy(s);
        set_err(RFEC_ENOMEM, "rx session: host tables / threads", 0);
        return NULL;
    }
    /* the row arena and the record store now (RFEC_RX_ARENA_ROWS), not inside the first push */
    if (rx_compact(s, 0, NULL)) {
        rfec_rx_session_destroy(s);
        return NULL;
    }
    s->t_compact = 0;
    return s;
}

int rfec_rx_session_set_threads(rfec_rx_session* s, uint32_t threads)
{
    if (!s || threads < 1 || threads > RX_MAX_THREADS)
        return set_err(RFEC_EINVAL, "rx session: threads must be in [1, 64]", 0);
    if (s->nstore || s->pend >= 0 || s->max_ts)
        return set_err(RFEC_EINVAL, "rx session: threads are set before the first push", 0);
    if (threads == s->T)
        return RFEC_OK;
    if (rx_shards_init(s, threads))
        return set_err(RFEC_ENOMEM, "rx session: host tables / threads", 0);
    return RFEC_OK;
}

void rfec_rx_session_destroy(rfec_rx_session* s)
{
    if (!s)
        return;
    if (s->sa) /* a pending parse still writes into the arena */
        (void)hipStreamSynchronize(s->sa);
    for (int i = 0; i < 2; ++i) {
        if (s->st[i].sum)
            (void)hipHostFree(s->st[i].sum);
        if (s->st[i].dg)
            (void)hipFree(s->st[i].dg);
        if (s->st[i].done)
            (void)hipEventDestroy(s->st[i].done);
    }
    if (s->sa)
        (void)hipStreamDestroy(s->sa);
    if (s->pool_on)
        pool_stop(&s->pool);
    if (getenv("RFEC_RX_TRACE"))
        for (uint32_t t = 0; t < s->T; ++t)
            if (s->XS[t] && s->XS[t]->tw_n)
                fprintf(stderr, "rx shard %u: %u replays, start +%.1f us, run %.1f us (before the first arrival %.1f), "
                        "%.1f records (per replay)\n", t, s->XS[t]->tw_n, s->XS[t]->tw_wake / s->XS[t]->tw_n,
                        s->XS[t]->tw_run / s->XS[t]->tw_n, s->XS[t]->tw_pre / s->XS[t]->tw_n,
                        (double)s->XS[t]->tw_recs / s->XS[t]->tw_n);
    rx_shards_free(s);
    rx_dev_free(&s->dev);
    if (s->vown_on)
        for (uint32_t t = 0; t < s->T; ++t)
            pm_free(&s->vown[t]);
    free(s->pshard);
    free(s->lst);
    free(s->smin);
    if (s->store)
        (void)hipHostFree(s->store);
    if (s->arena)
        (void)hipFree(s->arena);
    if (s->spare)
        (void)hipFree(s->spare);
    if (s->dmap)
        (void)hipFree(s->dmap);
    free(s);
}

/* The shards merged into one serial state, for good: a batch broke the
 * partition (a packet id under two fec_ids, a recovery outside its flex, or
 * parity ranges too large to claim).  Instances, shapes, slot / line tables
 * and recovered headers are concatenated; map values follow. */
static int rx_merge(rfec_rx_session* S)
{
    const uint32_t T = S->T;
    if (T == 1)
        return RFEC_OK;
    rx_sim* M = rx_sim_alloc();
    uint32_t ng = 0, nslot = 0, nline = 0, ns = 0, nrh = 0;
    for (uint32_t t = 0; t < T; ++t) {
        const rx_sim* X = S->XS[t];
        ng += X->ng, nslot += X->nslot, nline += X->nline, ns += X->ns, nrh += X->nrh;
    }
    if (!M || rx_tables_init(M, 0))
        goto oom;
    M->R = S->store;
    M->capacity = S->capacity;
    M->max_ts = S->max_ts;
    M->G = (rx_inst*)malloc(((size_t)ng + 1) * sizeof(rx_inst));
    M->S = (rx_shape*)malloc(((size_t)ns + 1) * sizeof(rx_shape));
    M->slot_src = (int32_t*)malloc(((size_t)nslot + 1) * sizeof(int32_t));
    M->slot_hdr = (rfec_hdr*)malloc(((size_t)nslot + 1) * sizeof(rfec_hdr));
    M->line_par = (int32_t*)malloc(((size_t)nline + 1) * sizeof(int32_t));
    M->rh = (rfec_hdr*)malloc(((size_t)nrh + 1) * sizeof(rfec_hdr));
    if (!M->G || !M->S || !M->slot_src || !M->slot_hdr || !M->line_par || !M->rh)
        goto oom;
    M->gcap = ng + 1, M->scap = ns + 1, M->slotcap = M->slothcap = nslot + 1, M->linecap = nline + 1;
    M->rhcap = nrh + 1;
    for (uint32_t t = 0; t < T; ++t) {
        const rx_sim* X = S->XS[t];
        const uint32_t og = M->ng, os = M->ns, oslot = M->nslot, oline = M->nline, orh = M->nrh;
        for (uint32_t i = 0; i < X->ng; ++i) {
            rx_inst g = X->G[i];
            g.slot0 += oslot;
            g.line0 += oline;
            if (g.shape != UINT32_MAX)
                g.shape += os;
            g.gstamp = g.jstamp = 0;
            M->G[M->ng++] = g;
        }
        for (uint32_t i = 0; i < X->ns; ++i) {
            const rx_shape* sh = &X->S[i];
            M->S[M->ns++] = *sh;
            const uint32_t key = sh->count << 16 | sh->row << 8 | sh->col;
            if (!sh->xcol[0] && !sh->xcol[1] && !hm_get(&M->shape_of, key) && hm_put(&M->shape_of, key, os + i + 1))
                goto oom;
        }
        memcpy(M->slot_src + oslot, X->slot_src, (size_t)X->nslot * sizeof(int32_t));
        memcpy(M->slot_hdr + oslot, X->slot_hdr, (size_t)X->nslot * sizeof(rfec_hdr));
        memcpy(M->line_par + oline, X->line_par, (size_t)X->nline * sizeof(int32_t));
        memcpy(M->rh + orh, X->rh, (size_t)X->nrh * sizeof(rfec_hdr));
        M->nslot += X->nslot, M->nline += X->nline, M->nrh += X->nrh;
        for (PM_EACH(&X->seen, k, v))
            if (pm_put(&M->seen, k, *v))
                goto oom;
        for (PM_EACH(&X->cache, k, v))
            if (pm_put(&M->cache, k, (*v & 0x80000000u) ? (0x80000000u | ((*v & 0x7FFFFFFFu) + orh)) : *v))
                goto oom;
        for (PM_EACH(&X->flex_of, k, v))
            if (pm_put(&M->flex_of, k, *v + og))
                goto oom;
    }
    if (S->vown_on)
        for (uint32_t t = 0; t < T; ++t)
            pm_free(&S->vown[t]);
    S->vown_on = 0;
    rx_shards_free(S);
    if (S->pool_on) {
        pool_stop(&S->pool);
        S->pool_on = 0;
    }
    S->XS[0] = M;
    S->T = 1;
    return RFEC_OK;
oom:
    if (M) {
        rx_sim_free(M);
        free(M);
    }
    return set_err(RFEC_ENOMEM, "rx session: merge", 0);
}

/* Phase 0 of a sharded batch, serial over the records [a0, a0 + n): each
 * record's shard, the per-shard lists, smin, whether a parity of the batch
 * could meet the 3 s drop through a segment timestamp before it (`risky`). */
static int rx_phase0(rfec_rx_session* S, uint32_t a0, uint32_t n, const rfec_rx_split* sum, int* risky)
{
    if (S->lcap < n) {
        const uint32_t c = n + n / 4 + 64;
        uint8_t* ps = (uint8_t*)realloc(S->pshard, c);
        if (ps)
            S->pshard = ps;
        uint32_t* l = (uint32_t*)realloc(S->lst, (size_t)c * 4);
        if (l)
            S->lst = l;
        uint32_t* m = (uint32_t*)realloc(S->smin, (size_t)c * 4);
        if (m)
            S->smin = m;
        if (!ps || !l || !m)
            return set_err(RFEC_ENOMEM, "rx session: batch lists", 0);
        S->lcap = c;
    }
    const uint32_t T = S->T;
    const rfec_wire_rec* R = S->store + a0;
    uint32_t cnt[RX_MAX_THREADS] = {0};
    uint32_t pm = S->max_ts;
    int rk = 0;
    if (sum) { /* the device's split (k_rx_split): 8 bytes per record */
        for (uint32_t p = 0; p < n; ++p) {
            const rfec_rx_split e = sum[p];
            if (e.kind == RX_SPLIT_SEG_TS && e.value > pm)
                pm = e.value;
            else if (e.kind == RX_SPLIT_FEC && e.value < pm)
                rk = 1;
            S->pshard[p] = e.shard;
            if (e.shard != 0xFF)
                cnt[e.shard]++;
        }
        uint32_t m = UINT32_MAX;
        for (uint32_t p = n; p-- > 0;) {
            S->smin[p] = m;
            if (sum[p].kind == RX_SPLIT_FEC && sum[p].value < m)
                m = sum[p].value;
        }
    }
    for (uint32_t p = 0; p < n && !sum; ++p) {
        const rfec_wire_rec* r = &R[p];
        uint32_t t = 0xFF;
        if (r->status == RFEC_WIRE_OK && r->mid == RFEC_WIRE_SEG) {
            t = r->fec_id ? S->shard_of[r->fec_id] : r->hdr.seq % T;
            if (r->fec_id && r->hdr.seq && r->hdr.ts > pm) /* (an upper bound of what raises max_ts) */
                pm = r->hdr.ts;
        } else if (r->status == RFEC_WIRE_OK && r->mid == RFEC_WIRE_FEC) {
            t = S->shard_of[r->fec_id];
            if (r->send_ts + 3000u < pm) /* sim_fec.c:148 could drop it */
                rk = 1;
        }
        S->pshard[p] = (uint8_t)t;
        if (t != 0xFF)
            cnt[t]++;
    }
    uint32_t m = UINT32_MAX;
    for (uint32_t p = n; !sum && p-- > 0;) {
        S->smin[p] = m;
        const rfec_wire_rec* r = &R[p];
        if (r->status == RFEC_WIRE_OK && r->mid == RFEC_WIRE_FEC && r->send_ts + 3000u < m)
            m = r->send_ts + 3000u;
    }
    S->loff[0] = 0;
    for (uint32_t t = 0; t < T; ++t)
        S->loff[t + 1] = S->loff[t] + cnt[t];
    uint32_t pos[RX_MAX_THREADS];
    memcpy(pos, S->loff, T * sizeof(uint32_t));
    for (uint32_t p = 0; p < n; ++p)
        if (S->pshard[p] != 0xFF)
            S->lst[pos[S->pshard[p]]++] = a0 + p;
    *risky = rk;
    return RFEC_OK;
}

/* shard t replays its records of the batch in arrival order */
static void rx_shard_replay(rfec_rx_session* S, rx_sim* X, const rx_par* P, uint32_t t);
static void rx_split_job(void* arg, uint32_t j);
static void rx_shard_job(void* arg, uint32_t t)
{
    rfec_rx_session* S = (rfec_rx_session*)arg;
    rx_sim* X = S->XS[t];
    const rx_par* P = &S->par;
    const double ts = now_us();
    X->tw_wake += ts - P->t0;
    X->tw_n++;
    X->tw_start = ts;
    rx_shard_replay(S, X, P, t);
    X->tw_run += now_us() - ts;
}

static void rx_shard_replay(rfec_rx_session* S, rx_sim* X, const rx_par* P, uint32_t t)
{
    if (P->sum) {
        /* the device's split, taken apart in chunks by rx_split_job: the drop check over the chunks (a
           parity's limit against max_ts at the batch's start and the segment timestamps before it), then
           this shard's records of every chunk, in arrival order, each with its smin */
        const uint32_t T = S->T;
        uint32_t run = P->max0, suf[RX_MAX_THREADS + 1], nm = 0;
        for (uint32_t j = 0; j < T; ++j) {
            const rx_sim* C = S->XS[j];
            if (C->c_flag || C->c_minfec < run) {
                rx_conflict(X, RX_CONFLICT_RISKY);
                return;
            }
            run = C->c_maxseg > run ? C->c_maxseg : run;
        }
        suf[T] = UINT32_MAX;
        for (uint32_t j = T; j-- > 0;)
            suf[j] = S->XS[j]->c_minfec < suf[j + 1] ? S->XS[j]->c_minfec : suf[j + 1];
        RX_GROW(X->mine, 0, X->minecap, P->n, uint32_t);
        if (X->oom)
            return;
        if (!(X->mine_sm = (uint32_t*)realloc(X->mine_sm, (size_t)X->minecap * 4))) {
            X->oom = 1;
            return;
        }
        for (uint32_t j = 0; j < T; ++j) {
            const rx_sim* C = S->XS[j];
            for (uint32_t q = C->cof[t]; q < C->cof[t + 1]; ++q) {
                X->mine[nm] = P->a0 + C->cpos[q];
                X->mine_sm[nm++] = C->csm[q] < suf[j + 1] ? C->csm[q] : suf[j + 1];
            }
        }
        /* the records, prefetched a few arrivals ahead: the device wrote them (cache-cold here) and a shard's
           records are scattered over the batch, so the hardware prefetcher does not follow them (each one a
           DRAM round trip: a shard replayed 3-4 x slower per arrival than one thread over the whole batch) */
        const rfec_wire_rec* R = X->R;
        const uint32_t pf = rx_prefetch();
        for (uint32_t i = 0; i < nm && i < pf; ++i)
            __builtin_prefetch(&R[X->mine[i]]);
        X->tw_pre += now_us() - X->tw_start;
        X->tw_recs += nm;
        for (uint32_t i = 0; i < nm && !X->oom; ++i) {
            if (i + pf < nm)
                __builtin_prefetch(&R[X->mine[i + pf]]);
            if ((i & 15) == 0 && __atomic_load_n(&S->par.conflict, __ATOMIC_RELAXED))
                return;
            X->smin_cur = X->mine_sm[i];
            rx_arrival(X, X->mine[i]);
        }
    } else {
        const uint32_t* L = S->lst + S->loff[t];
        const uint32_t n = S->loff[t + 1] - S->loff[t];
        X->tw_pre += now_us() - X->tw_start;
        for (uint32_t i = 0; i < n && !X->oom; ++i) {
            if ((i & 15) == 0 && __atomic_load_n(&S->par.conflict, __ATOMIC_RELAXED))
                return;
            X->smin_cur = P->smin[L[i] - P->a0];
            rx_arrival(X, L[i]);
        }
    }
    rx_bucket_claims(X, S->T);
}

/* Chunk j of the batch's split summary (positions [j n / T, (j + 1) n / T)),
 * on shard j's thread before the replay: its positions grouped by shard (a
 * counting pass, then a backward fill that keeps each shard's arrival order
 * and carries the chunk-local suffix min of the parity limits), and the
 * chunk's drop-check figures.  Every replay thread then reads only its own
 * records' positions (each thread walking the whole summary cost ~25 us a
 * batch: 4,096 records, two passes, branchy). */
static void rx_split_job(void* arg, uint32_t j)
{
    rfec_rx_session* S = (rfec_rx_session*)arg;
    rx_sim* X = S->XS[j];
    const rx_par* P = &S->par;
    const uint32_t T = S->T, n = P->n;
    const uint32_t p0 = (uint32_t)((uint64_t)n * j / T), p1 = (uint32_t)((uint64_t)n * (j + 1) / T);
    const rfec_rx_split* sum = P->sum;
    uint32_t cnt[RX_MAX_THREADS + 1] = {0};
    uint32_t pm = 0, mf = UINT32_MAX;
    int flag = 0;
    if (X->ccap < p1 - p0) {
        const uint32_t c = p1 - p0 + (p1 - p0) / 4 + 64;
        uint32_t* a = (uint32_t*)realloc(X->cpos, (size_t)c * 4);
        if (a)
            X->cpos = a;
        uint32_t* b = (uint32_t*)realloc(X->csm, (size_t)c * 4);
        if (b)
            X->csm = b;
        if (!a || !b) {
            X->oom = 1;
            X->c_flag = 1;
            return;
        }
        X->ccap = c;
    }
    for (uint32_t p = p0; p < p1; ++p) {
        const rfec_rx_split e = sum[p];
        if (e.kind == RX_SPLIT_SEG_TS) {
            pm = e.value > pm ? e.value : pm;
        } else if (e.kind == RX_SPLIT_FEC) {
            flag |= e.value < pm;
            mf = e.value < mf ? e.value : mf;
        }
        cnt[e.shard == 0xFF ? T : e.shard]++;
    }
    X->cof[0] = 0;
    for (uint32_t u = 0; u < T; ++u)
        X->cof[u + 1] = X->cof[u] + cnt[u];
    uint32_t end[RX_MAX_THREADS];
    memcpy(end, X->cof + 1, T * sizeof(uint32_t));
    uint32_t m = UINT32_MAX;
    for (uint32_t p = p1; p-- > p0;) {
        const rfec_rx_split e = sum[p];
        if (e.shard != 0xFF) {
            const uint32_t q = --end[e.shard];
            X->cpos[q] = p;
            X->csm[q] = m;
        }
        if (e.kind == RX_SPLIT_FEC && e.value < m)
            m = e.value;
    }
    X->c_maxseg = pm;
    X->c_minfec = mf;
    X->c_flag = flag;
}

/* the batch's packet-id claims into the owner tables: thread j takes the ids
 * of its partition from every shard's log; an id under two fec_ids is a
 * conflict */
static void rx_verify_job(void* arg, uint32_t j)
{
    rfec_rx_session* S = (rfec_rx_session*)arg;
    pmap* V = &S->vown[j];
    const uint32_t T = S->T;
    for (uint32_t u = 0; u < T; ++u) {
        const rx_sim* X = S->XS[u];
        for (uint32_t q = X->coff[j]; q < X->coff[j + 1]; ++q) {
            const uint32_t seq = (uint32_t)(X->cpart[q] >> 32), code = (uint32_t)X->cpart[q];
            const uint32_t v = pm_get(V, seq);
            if (!v) {
                if (pm_put(V, seq, code))
                    __atomic_fetch_or(&S->par.conflict, RX_CONFLICT_OWNER, __ATOMIC_RELAXED); /* (no memory: serial) */
            } else if (v != code) {
                __atomic_fetch_or(&S->par.conflict, RX_CONFLICT_OWNER, __ATOMIC_RELAXED);
                return;
            }
        }
    }
}

/* the batch in arrival order over the shards, one max_ts (then the claims bucketed) */
static void rx_serial_over_shards(rfec_rx_session* S, uint32_t a0, uint32_t n)
{
    uint32_t m = S->max_ts;
    const rfec_rx_split* sum = S->par.sum;
    for (uint32_t p = 0; p < n; ++p) {
        const uint32_t t = sum ? sum[p].shard : S->pshard[p];
        if (t == 0xFF)
            continue;
        rx_sim* X = S->XS[t];
        X->max_ts = m;
        rx_arrival(X, a0 + p);
        m = X->max_ts;
        if (X->oom || __atomic_load_n(&S->par.conflict, __ATOMIC_RELAXED))
            break;
    }
    for (uint32_t t = 0; t < S->T; ++t)
        rx_bucket_claims(S->XS[t], S->T);
}

static int rx_any_oom(const rfec_rx_session* S)
{
    for (uint32_t t = 0; t < S->T; ++t)
        if (S->XS[t]->oom)
            return 1;
    return 0;
}

/* The control plane over the session's records [a0, a0 + n). */
static int rx_ingest(rfec_rx_session* S, uint32_t a0, uint32_t n, const rfec_rx_split* sum)
{
    for (uint32_t t = 0; t < S->T; ++t) {
        rx_sim* X = S->XS[t];
        X->R = S->store;
        X->nout = X->dropped = X->unmodelled = 0;
    }
    int rc, risky = 0;
    if (S->T > 1) {
        if (!S->vown_on) {
            for (uint32_t t = 0; t < S->T; ++t)
                if (pm_init(&S->vown[t]))
                    return set_err(RFEC_ENOMEM, "rx session: packet ids", 0);
            S->vown_on = 1;
        }
        for (uint32_t t = 0; t < S->T; ++t) {
            rx_sim* X = S->XS[t];
            if (!X->claimed && !(X->claimed = (uint32_t*)calloc(2u * (65536u / S->T + 1u), sizeof(uint32_t))))
                return set_err(RFEC_ENOMEM, "rx session: claims", 0);
            X->nclaims = 0;
        }
        if (!sum) { /* (with the device's split the replay threads take the batch apart themselves) */
            const double ts = now_us();
            if ((rc = rx_phase0(S, a0, n, NULL, &risky)))
                return rc;
            S->t_split += now_us() - ts;
        }
    }
    const double tr = now_us();
    if (S->T == 1) {
        rx_sim* X = S->XS[0];
        X->P = NULL;
        X->R = S->store;
        X->nout = X->dropped = X->unmodelled = 0;
        X->max_ts = S->max_ts;
        rx_run(X, a0, n);
        S->max_ts = X->max_ts;
        S->n_serial++;
        S->t_replay += now_us() - tr;
        return X->oom ? set_err(RFEC_ENOMEM, "rx session: host tables", 0) : RFEC_OK;
    }
    rx_par* P = &S->par;
    P->T = S->T;
    P->sum = sum;
    P->n = n;
    P->max0 = S->max_ts;
    P->smin = sum ? NULL : S->smin;
    P->a0 = a0;
    P->ts_check = !risky;
    P->conflict = 0;
    P->t0 = now_us();
    for (uint32_t t = 0; t < S->T; ++t) {
        rx_sim* X = S->XS[t];
        X->P = P;
        X->max_ts = S->max_ts;
        rx_journal_begin(X);
    }
    if (!risky) {
        if (sum)
            pool_run(&S->pool, rx_split_job, S);
        P->t0 = now_us();
        pool_run(&S->pool, rx_shard_job, S);
    } else {
        rx_serial_over_shards(S, a0, n);
    }
    int c = __atomic_load_n(&P->conflict, __ATOMIC_RELAXED);
    S->t_replay += now_us() - tr;
    if (!c && !rx_any_oom(S)) {
        const double tv = now_us();
        pool_run(&S->pool, rx_verify_job, S); /* every packet id under one fec_id? */
        S->t_verify += now_us() - tv;
        c = __atomic_load_n(&P->conflict, __ATOMIC_RELAXED);
        if (!c)
            ++*(risky ? &S->n_serial : &S->n_parallel);
    } else if ((c & (RX_CONFLICT_TS | RX_CONFLICT_RISKY)) && !(c & RX_CONFLICT_OWNER) && !rx_any_oom(S)) {
        /* a recovery raised max_ts past a later parity's limit, or a parity could meet the drop through a
           segment timestamp before it: again, in arrival order */
        S->n_rollback++;
        for (uint32_t t = 0; t < S->T; ++t) {
            rx_rollback(S->XS[t]);
            rx_journal_begin(S->XS[t]);
        }
        P->ts_check = 0;
        P->conflict = 0;
        rx_serial_over_shards(S, a0, n); /* (the claim logs keep the first try's claims too) */
        c = __atomic_load_n(&P->conflict, __ATOMIC_RELAXED);
        if (!c && !rx_any_oom(S)) {
            pool_run(&S->pool, rx_verify_job, S);
            c = __atomic_load_n(&P->conflict, __ATOMIC_RELAXED);
        }
        if (!c)
            S->n_serial++;
    }
    if (rx_any_oom(S))
        return set_err(RFEC_ENOMEM, "rx session: host tables", 0);
    if (c) { /* a packet id crossed fec_ids: back to the batch's start, one serial state from here on */
        S->n_rollback++;
        for (uint32_t t = 0; t < S->T; ++t) {
            rx_rollback(S->XS[t]);
            S->XS[t]->P = NULL;
        }
        if (rx_any_oom(S) || (rc = rx_merge(S)))
            return set_err(RFEC_ENOMEM, "rx session: merge", 0);
        rx_sim* X = S->XS[0];
        X->nout = X->dropped = X->unmodelled = 0;
        X->max_ts = S->max_ts;
        rx_run(X, a0, n);
        S->max_ts = X->max_ts;
        S->n_serial++;
        return X->oom ? set_err(RFEC_ENOMEM, "rx session: host tables", 0) : RFEC_OK;
    }
    uint32_t m = S->max_ts;
    for (uint32_t t = 0; t < S->T; ++t) {
        rx_sim* X = S->XS[t];
        rx_journal_end(X);
        X->P = NULL;
        m = X->max_ts > m ? X->max_ts : m;
    }
    S->max_ts = m;
    return RFEC_OK;
}

/* Keeps only what the open state refers to: the flexes still registered (with
 * their slot / line tables), the records of cached segments and of those
 * flexes' members and parities (their rows gathered into a fresh arena with
 * room for `extra` more), the headers of cached recovered segments -- over
 * every shard; records are renumbered in arrival order.  The rows of a
 * pending pipelined batch (parsed, not ingested) move along behind the kept
 * ones. */
typedef struct {
    rx_inst* NG;
    int32_t* nsrc;
    rfec_hdr* nhdr;
    int32_t* npar;
    uint32_t* hmap_; /* old rh -> new + 1 */
    uint32_t ng, ns, nl, nh;
} rx_kept;

static uint32_t rx_min_rows(void)
{
    const char* v = getenv("RFEC_RX_ARENA_ROWS");
    const long r = v ? atol(v) : 1l << 18;
    return r < 4096 ? 4096u : r > (1l << 26) ? (1u << 26) : (uint32_t)r;
}

static int rx_compact_(rfec_rx_session* S, uint32_t extra, hipStream_t sm);
static int rx_compact(rfec_rx_session* S, uint32_t extra, hipStream_t sm)
{
    const double t0 = now_us();
    const int rc = rx_compact_(S, extra, sm);
    S->t_compact += now_us() - t0;
    return rc;
}

static int rx_compact_(rfec_rx_session* S, uint32_t extra, hipStream_t sm)
{
    const uint32_t tail = S->pend >= 0 ? S->pend_n : 0;
    hipError_t e;
    if (tail && (e = hipEventSynchronize(S->st[S->pend].done)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: pending parse", e);
    const uint32_t T = S->T;
    int rc = RFEC_OK;
    rx_kept K[RX_MAX_THREADS];
    memset(K, 0, sizeof(K));
    uint32_t* rmap = (uint32_t*)calloc((size_t)S->nstore + 1, sizeof(uint32_t)); /* old record -> new + 1 */
    uint32_t* gmap = NULL;
    uint8_t* arena = NULL;
    if (!rmap)
        goto oom;
    /* 1. per shard: live flexes and their tables; mark the records they refer to */
    for (uint32_t t = 0; t < T; ++t) {
        const rx_sim* X = S->XS[t];
        rx_kept* k = &K[t];
        uint32_t nslot = 0, nline = 0;
        for (PM_EACH(&X->flex_of, fk, fv)) {
            const rx_inst* g = &X->G[*fv - 1];
            if (g->shape != UINT32_MAX) {
                nslot += g->count;
                nline += X->S[g->shape].n_lines;
            }
        }
        k->NG = (rx_inst*)malloc(((size_t)X->flex_of.n + 1) * sizeof(rx_inst));
        k->nsrc = (int32_t*)malloc(((size_t)nslot + 1) * sizeof(int32_t));
        k->nhdr = (rfec_hdr*)malloc(((size_t)nslot + 1) * sizeof(rfec_hdr));
        k->npar = (int32_t*)malloc(((size_t)nline + 1) * sizeof(int32_t));
        k->hmap_ = (uint32_t*)calloc((size_t)X->nrh + 1, sizeof(uint32_t));
        if (!k->NG || !k->nsrc || !k->nhdr || !k->npar || !k->hmap_)
            goto oom;
        /* the records the live state refers to (read only: nothing changes before the arena is allocated) */
        for (PM_EACH(&X->flex_of, fk, fv)) {
                const rx_inst* g = &X->G[*fv - 1];
                if (g->shape == UINT32_MAX)
                    continue;
                for (uint32_t q = 0; q < g->count; ++q)
                    if (X->slot_src[g->slot0 + q] >= 0)
                        rmap[X->slot_src[g->slot0 + q]] = 1;
                for (uint32_t q = 0; q < X->S[g->shape].n_lines; ++q)
                    if (X->line_par[g->line0 + q] >= 0)
                        rmap[X->line_par[g->line0 + q]] = 1;
            }
        for (PM_EACH(&X->cache, ck, cv))
            if (!(*cv & 0x80000000u))
                rmap[*cv - 1] = 1;
    }
    uint32_t nr = 0;
    for (uint32_t r = 0; r < S->nstore; ++r)
        nr += rmap[r] != 0;
    gmap = (uint32_t*)malloc(((size_t)nr + tail + 1) * sizeof(uint32_t)); /* new -> old */
    /* room for 4 x what stays (compaction's host work is proportional to the open state: it comes back
       after >= 3 x that many records), at least RFEC_RX_ARENA_ROWS rows (default 2^18: ~320 MB of HBM at
       1,216-B rows; with razor's 300 ms evictions the open state stays far below it) */
    const uint64_t want = 4ull * (nr + tail + extra);
    const uint32_t arows = (uint32_t)(want > rx_min_rows() ? (want < 0xFFFFFFFFull ? want : 0xFFFFFFFFull) : rx_min_rows());
    if (!gmap)
        goto oom;
    /* the previous arena when it is large enough (no allocation per compaction: an eviction per batch
       compacts per batch), else a fresh one */
    if (S->spare && S->sprows >= arows) {
        arena = S->spare;
        S->spare = NULL;
    } else if ((e = hipMalloc((void**)&arena, (size_t)arows * S->stride)) != hipSuccess) {
        rc = set_err(RFEC_ENOMEM, "rx session: arena", e);
        goto done;
    }
    /* the record store: the same capacity, pinned and device-mapped (the parse writes records in) */
    rfec_wire_rec* nst = S->store;
    rfec_wire_rec* nst_d = S->store_d;
    if (S->storecap < arows) {
        void* d = NULL;
        nst = NULL;
        if ((e = hipHostMalloc((void**)&nst, (size_t)arows * sizeof(rfec_wire_rec), hipHostMallocMapped)) !=
                hipSuccess ||
            (e = hipHostGetDevicePointer(&d, nst, 0)) != hipSuccess) {
            if (nst)
                (void)hipHostFree(nst);
            rc = set_err(RFEC_ENOMEM, "rx session: record store", e);
            goto oom_arena;
        }
        nst_d = (rfec_wire_rec*)d;
    }
    for (uint32_t t = 0; t < T; ++t) {
        rx_sim* X = S->XS[t];
        rx_kept* k = &K[t];
        for (PM_EACH(&X->flex_of, fk, fv)) {
            rx_inst g = X->G[*fv - 1];
            if (g.shape != UINT32_MAX) {
                const uint32_t nlines = X->S[g.shape].n_lines;
                memcpy(k->nsrc + k->ns, X->slot_src + g.slot0, g.count * sizeof(int32_t));
                memcpy(k->nhdr + k->ns, X->slot_hdr + g.slot0, g.count * sizeof(rfec_hdr));
                memcpy(k->npar + k->nl, X->line_par + g.line0, nlines * sizeof(int32_t));
                g.slot0 = k->ns;
                g.line0 = k->nl;
                k->ns += g.count;
                k->nl += nlines;
            }
            k->NG[k->ng] = g;
            *fv = ++k->ng;
        }
        /* 2. cached recovered segments keep their header */
        for (PM_EACH(&X->cache, ck, cv))
            if (*cv & 0x80000000u)
                k->hmap_[*cv & 0x7FFFFFFFu] = 1;
    }
    /* 3. new ids, in arrival order */
    nr = 0;
    for (uint32_t r = 0; r < S->nstore; ++r)
        if (rmap[r])
            rmap[r] = ++nr;
    for (uint32_t t = 0; t < T; ++t) {
        rx_sim* X = S->XS[t];
        rx_kept* k = &K[t];
        for (uint32_t h = 0; h < X->nrh; ++h)
            if (k->hmap_[h])
                k->hmap_[h] = ++k->nh;
        for (uint32_t q = 0; q < k->ns; ++q)
            if (k->nsrc[q] >= 0)
                k->nsrc[q] = (int32_t)rmap[k->nsrc[q]] - 1;
        for (uint32_t q = 0; q < k->nl; ++q)
            if (k->npar[q] >= 0)
                k->npar[q] = (int32_t)rmap[k->npar[q]] - 1;
        for (PM_EACH(&X->cache, ck, cv))
            *cv = (*cv & 0x80000000u) ? (0x80000000u | (k->hmap_[*cv & 0x7FFFFFFFu] - 1)) : rmap[*cv - 1];
        for (uint32_t h = 0; h < X->nrh; ++h)
            if (k->hmap_[h])
                X->rh[k->hmap_[h] - 1] = X->rh[h];
        X->nrh = k->nh;
        /* the group tables */
        free(X->G);
        free(X->slot_src);
        free(X->slot_hdr);
        free(X->line_par);
        X->G = k->NG;
        X->ng = X->gcap = k->ng;
        X->slot_src = k->nsrc;
        X->slot_hdr = k->nhdr;
        X->nslot = X->slotcap = X->slothcap = k->ns;
        X->line_par = k->npar;
        X->nline = X->linecap = k->nl;
        k->NG = NULL;
        k->nsrc = k->npar = NULL;
        k->nhdr = NULL;
    }
    /* 4. records (host: in place, rmap[r] - 1 <= r, ascending, or into the larger store) and rows (device) */
    for (uint32_t r = 0; r < S->nstore; ++r)
        if (rmap[r]) {
            gmap[rmap[r] - 1] = r;
            nst[rmap[r] - 1] = S->store[r];
        }
    for (uint32_t t = 0; t < tail; ++t) { /* the pending batch's records and rows follow */
        gmap[nr + t] = S->nstore + t;
        nst[nr + t] = S->store[S->nstore + t];
    }
    if (nst != S->store) {
        if (S->store)
            (void)hipHostFree(S->store);
        S->store = nst;
        S->store_d = nst_d;
        S->storecap = arows;
    }
    S->nstore = nr;
    for (uint32_t t = 0; t < T; ++t)
        S->XS[t]->R = S->store;
    if (nr + tail) {
        int ke = 0;
        const uint32_t nm = nr + tail;
        if (S->dmapcap < nm) {
            if (S->dmap)
                (void)hipFree(S->dmap);
            S->dmap = NULL;
            S->dmapcap = 0;
            if ((e = hipMalloc((void**)&S->dmap, ((size_t)nm + nm / 2) * sizeof(int32_t))) == hipSuccess)
                S->dmapcap = nm + nm / 2;
        }
        if (!S->dmap ||
            (e = hipMemcpyAsync(S->dmap, gmap, (size_t)nm * sizeof(int32_t), hipMemcpyHostToDevice, sm)) != hipSuccess ||
            (ke = rfec_launch_gather_rows(arena, S->arena, S->dmap, nm, S->stride, sm)) != 0 ||
            (e = hipStreamSynchronize(sm)) != hipSuccess) {
            (void)hipFree(arena);
            arena = NULL;
            rc = set_err(RFEC_EDEVICE, "rx session: row compaction", ke ? ke : (int)e);
            goto done;
        }
    }
    if (S->arena) { /* the old arena is the next compaction's target (the larger of it and the spare) */
        if (S->spare && S->sprows >= S->arows) {
            (void)hipFree(S->arena);
        } else {
            if (S->spare)
                (void)hipFree(S->spare);
            S->spare = S->arena;
            S->sprows = S->arows;
        }
    }
    S->arena = arena;
    S->arows = arows;
    goto done;
oom:
    rc = set_err(RFEC_ENOMEM, "rx session: compaction", 0);
oom_arena:
    if (arena)
        (void)hipFree(arena);
done:
    for (uint32_t t = 0; t < T; ++t) {
        free(K[t].NG);
        free(K[t].nsrc);
        free(K[t].nhdr);
        free(K[t].npar);
        free(K[t].hmap_);
    }
    free(gmap);
    free(rmap);
    return rc;
}

/* room for n more arena rows and records: drop what the open state no longer
 * refers to (and grow) */
static int rx_session_room(rfec_rx_session* S, uint32_t n, hipStream_t sm)
{
    int rc;
    const uint32_t tail = S->pend >= 0 ? S->pend_n : 0; /* a pending pipelined batch's rows */
    if ((S->nstore + tail + n > S->arows || S->nstore + tail + n > S->storecap) && (rc = rx_compact(S, n, sm)))
        return rc; /* (compaction sizes both: room for 4 x what stays) */
    return RFEC_OK;
}

static int rx_stage_reserve(rx_stage* st, uint32_t n, size_t dg_bytes);

/* The batch's records are at store[nstore, nstore + n) already (the parse or
 * the D2H wrote them there); payload rows on the device at `payload`, or
 * already in the arena's next n rows (payload NULL; the caller made the
 * room); `sum`: the batch's split summary (k_rx_split), or NULL (split on the
 * host from the records) */
static int rx_session_push_staged(rfec_rx_session* S, uint32_t n, const uint8_t* payload, const rfec_rx_split* sum,
                                  rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                                  rfec_rx_report* rep, hipStream_t sm)
{
    hipError_t e;
    int rc;
    if (payload) {
        double tt = now_us();
        if ((e = hipMemcpyAsync(S->arena + (size_t)S->nstore * S->stride, payload, (size_t)n * S->stride,
                                hipMemcpyDeviceToDevice, sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: rows", e);
        rep->kernel_us += now_us() - tt;
    }
    const uint32_t a0 = S->nstore;
    S->nstore += n;
    const double th = now_us();
    if ((rc = rx_ingest(S, a0, n, sum)))
        return rc;
    uint32_t dropped = 0, unmod = 0;
    for (uint32_t t = 0; t < S->T; ++t) {
        dropped += S->XS[t]->dropped;
        unmod += S->XS[t]->unmodelled;
    }
    rep->n_fec_dropped = dropped;
    rep->host_us += now_us() - th;
    const double h0 = rep->host_us;
    rc = rx_device(S->XS, S->T, S->pool_on ? &S->pool : NULL, &S->dev, S->arena, S->stride, S->capacity, 0, 0, out, out_payload, max_out, n_out,
                   rep, sm);
    S->t_tables += rep->host_us - h0;
    rep->n_unmodelled = unmod + S->dev.unmodelled;
    return rc;
}

/* where a batch's split summary goes (sharded sessions), or NULL (one serial state; a huge push: split on the host) */
static rfec_rx_split* rx_split_of(const rfec_rx_session* S, rx_stage* st, uint32_t n)
{
    return S->T == 1 || n > (1u << 20) ? NULL : st->sumd;
}

/* the split summary of records the device can read at `recs_d` into stage st (sharded sessions) */
static int rx_split_launch(rfec_rx_session* S, rx_stage* st, const rfec_wire_rec* recs_d, uint32_t n, hipStream_t sm)
{
    if (S->T == 1 || n > (1u << 20)) /* (one serial state; or a huge push: split on the host) */
        return 0;
    return rfec_launch_rx_split(recs_d, n, S->T, st->sumd, sm);
}

int rfec_rx_session_push(rfec_rx_session* S, uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload,
                         rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                         rfec_rx_report* rep, void* stream)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!recs || !payload)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    if (S->pend >= 0)
        return set_err(RFEC_EINVAL, "rx session: a pipelined batch is pending (flush it: async push with n = 0)", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    hipStream_t sm = (hipStream_t)stream;
    hipError_t e;
    int rc, ke = 0;
    if ((rc = rx_session_room(S, n, sm)) || (rc = rx_stage_reserve(&S->st[0], n, 0)))
        return rc;
    double tt = now_us();
    /* the records into the store, their split beside */
    if ((e = hipMemcpyAsync(S->store + S->nstore, recs, (size_t)n * sizeof(rfec_wire_rec), hipMemcpyDeviceToHost,
                            sm)) != hipSuccess ||
        (ke = rx_split_launch(S, &S->st[0], recs, n, sm)) != 0 || (e = hipStreamSynchronize(sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: records D2H", ke ? ke : (int)e);
    rep->d2h_us += now_us() - tt;
    rc = rx_session_push_staged(S, n, payload, S->T > 1 && n <= (1u << 20) ? S->st[0].sum : NULL, out, out_payload,
                                max_out, n_out, rep, sm);
    rep->total_us = now_us() - t0;
    return rc;
}

int rfec_rx_session_push_datagrams(rfec_rx_session* S, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                   const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                   uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!dgram || !dlen)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    if (S->pend >= 0)
        return set_err(RFEC_EINVAL, "rx session: a pipelined batch is pending (flush it: async push with n = 0)", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n == 0)
        return RFEC_OK;
    if (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16)
        return set_err(RFEC_EINVAL, "rx session: dstride must be a multiple of 16 in [64, 2048]", 0);
    hipError_t e;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    const uint32_t stride = S->stride;
    const size_t o_dl = RX_ALIGN((size_t)n * dstride);
    int rc;
    /* the records are parsed straight into the store, the payload rows into the arena's next n rows */
    if ((rc = rx_session_room(S, n, t_rv.sm)) || (rc = rx_stage_reserve(&S->st[0], n, o_dl + (size_t)n * 2)))
        return rc;
    rx_stage* st = &S->st[0];
    double tt = now_us();
    /* datagrams in pinned memory (the UDP batch slots) are read by the parse
     * itself; pageable ones are copied first */
    const uint8_t* dg = host_mapped(dgram);
    const uint8_t* dl = host_mapped(dlen);
    if (!dg || !dl) {
        if ((e = hipMemcpyAsync(st->dg, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess ||
            (e = hipMemcpyAsync(st->dg + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, t_rv.sm)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "recv: datagrams H2D", e);
        dg = st->dg;
        dl = st->dg + o_dl;
    }
    const double h2d_issue = now_us() - tt;
    const int ke = rfec_launch_wire_parse_split(n, dstride, dg, (const uint16_t*)dl, stride, S->capacity,
                                                S->store_d + S->nstore, S->arena + (size_t)S->nstore * stride,
                                                max_dlen(dlen, n), rx_split_of(S, st, n), S->T, t_rv.sm);
    if (ke || (e = hipStreamSynchronize(t_rv.sm)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: parse", ke ? ke : (int)e);
    const double staged = now_us() - tt;
    if (recs_out)
        memcpy(recs_out, S->store + S->nstore, (size_t)n * sizeof(rfec_wire_rec));
    rc = rx_session_push_staged(S, n, NULL, S->T > 1 && n <= (1u << 20) ? st->sum : NULL, out, out_payload, max_out,
                                n_out, rep, t_rv.sm);
    rep->h2d_us += h2d_issue;
    rep->kernel_us += staged - h2d_issue; /* the H2D completes inside this interval too */
    rep->total_us = now_us() - t0;
    return rc;
}

/* The pipelined push: this call starts batch i (H2D if pageable, parse into
 * the store's records and the arena's rows after the pending batch's, its
 * split summary into its stage, on the session's own stream) and then
 * ingests batch i-1 (control plane, peel on the thread's stream) while the
 * device parses batch i. */
static int rx_stage_reserve(rx_stage* st, uint32_t n, size_t dg_bytes)
{
    hipError_t e;
    if (!st->done && (e = hipEventCreateWithFlags(&st->done, hipEventDisableTiming)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: event", e);
    if (st->sumcap < n) {
        const uint32_t c = n + n / 4 + 64;
        void* h = NULL;
        void* d = NULL;
        if ((e = hipHostMalloc(&h, (size_t)c * sizeof(rfec_rx_split), hipHostMallocMapped)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx session: split stage", e);
        if ((e = hipHostGetDevicePointer(&d, h, 0)) != hipSuccess) {
            (void)hipHostFree(h);
            return set_err(RFEC_EDEVICE, "rx session: split stage device view", e);
        }
        if (st->sum)
            (void)hipHostFree(st->sum);
        st->sum = (rfec_rx_split*)h;
        st->sumd = (rfec_rx_split*)d;
        st->sumcap = c;
    }
    if (dg_bytes > st->dgb) {
        if (st->dg)
            (void)hipFree(st->dg);
        st->dg = NULL;
        st->dgb = 0;
        const size_t b = dg_bytes + dg_bytes / 4;
        if ((e = hipMalloc((void**)&st->dg, b)) != hipSuccess)
            return set_err(RFEC_ENOMEM, "rx session: datagram stage", e);
        st->dgb = b;
    }
    return RFEC_OK;
}

int rfec_rx_session_push_datagrams_async(rfec_rx_session* S, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                         const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                         uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* rep)
{
    const double t0 = now_us();
    if (!S || !n_out || !rep || (n && (!dgram || !dlen)) || (max_out && (!out || !out_payload)))
        return set_err(RFEC_EINVAL, "rx session: bad argument", 0);
    memset(rep, 0, sizeof(*rep));
    *n_out = 0;
    if (n && (dstride < 64 || dstride > RFEC_WIRE_MAX_DSTRIDE || dstride % 16))
        return set_err(RFEC_EINVAL, "rx session: dstride must be a multiple of 16 in [64, 2048]", 0);
    hipError_t e;
    int rc;
    if (!t_rv.sm && (e = hipStreamCreateWithFlags(&t_rv.sm, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "recv: stream", e);
    if (!S->sa && (e = hipStreamCreateWithFlags(&S->sa, hipStreamNonBlocking)) != hipSuccess)
        return set_err(RFEC_EDEVICE, "rx session: stream", e);
    const int prev = S->pend;
    const uint32_t p = prev >= 0 ? S->pend_n : 0;
    int cur = -1;
    if (n) {
        /* 1. start batch i behind the pending one's rows */
        cur = prev == 0 ? 1 : 0;
        rx_stage* st = &S->st[cur];
        const size_t o_dl = RX_ALIGN((size_t)n * dstride);
        if ((rc = rx_session_room(S, n, t_rv.sm)) || (rc = rx_stage_reserve(st, n, o_dl + (size_t)n * 2)))
            return rc;
        double tt = now_us();
        const uint8_t* dg = host_mapped(dgram);
        const uint8_t* dl = host_mapped(dlen);
        if (!dg || !dl) {
            if ((e = hipMemcpyAsync(st->dg, dgram, (size_t)n * dstride, hipMemcpyHostToDevice, S->sa)) != hipSuccess ||
                (e = hipMemcpyAsync(st->dg + o_dl, dlen, (size_t)n * 2, hipMemcpyHostToDevice, S->sa)) != hipSuccess)
                return set_err(RFEC_EDEVICE, "rx session: datagrams H2D", e);
            dg = st->dg;
            dl = st->dg + o_dl;
        }
        rep->h2d_us += now_us() - tt;
        /* the parse writes the split entries beside the records (k_parse_q; the wave parses: k_rx_split) */
        const int ke = rfec_launch_wire_parse_split(n, dstride, dg, (const uint16_t*)dl, S->stride, S->capacity,
                                                    S->store_d + S->nstore + p,
                                                    S->arena + (size_t)(S->nstore + p) * S->stride, max_dlen(dlen, n),
                                                    rx_split_of(S, st, n), S->T, S->sa);
        if (ke || (e = hipEventRecord(st->done, S->sa)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: parse", ke ? ke : (int)e);
    }
    /* 2. ingest batch i-1 while the device parses batch i */
    if (prev >= 0) {
        rx_stage* ps = &S->st[prev];
        double tt = now_us();
        if ((e = hipEventSynchronize(ps->done)) != hipSuccess)
            return set_err(RFEC_EDEVICE, "rx session: parse", e);
        rep->kernel_us += now_us() - tt;
        if (recs_out)
            memcpy(recs_out, S->store + S->nstore, (size_t)p * sizeof(rfec_wire_rec));
        S->pend = -1; /* its records and rows are the store's and the arena's next p now */
        rc = rx_session_push_staged(S, p, NULL, S->T > 1 && p <= (1u << 20) ? ps->sum : NULL, out, out_payload,
                                    max_out, n_out, rep, t_rv.sm);
        if (rc) {
            S->pend = cur; /* batch i stays pending behind whatever was ingested */
            S->pend_n = n;
            return rc;
        }
    }
    S->pend = cur;
    S->pend_n = n;
    rep->total_us = now_us() - t0;
    return RFEC_OK;
}

/* One eviction walk over the union of the shards' maps m (2 flex_of, 1
 * cache), in key order: the shards' own walks (each in key order) merged, so
 * the cost is the entries evicted, not the open state (a sort of every
 * shard's keys per eviction cost ~10-20 % of a batch's host time).  Stops at
 * the first entry that stays, as the skiplist walks do. */
static void rx_evict_walk(rfec_rx_session* S, int m)
{
    const uint32_t T = S->T;
    uint32_t key[RX_MAX_THREADS], done[RX_MAX_THREADS];
    uint32_t* val[RX_MAX_THREADS];
    for (uint32_t t = 0; t < T; ++t) {
        key[t] = done[t] = 0;
        val[t] = pm_next(rx_map(S->XS[t], m), &key[t], &done[t]);
    }
    for (;;) {
        uint32_t b = UINT32_MAX;
        for (uint32_t t = 0; t < T; ++t)
            if (val[t] && (b == UINT32_MAX || key[t] < key[b]))
                b = t;
        if (b == UINT32_MAX)
            return;
        rx_sim* X = S->XS[b];
        const uint32_t v = *val[b];
        if (m == 2) {
            const rx_inst* g = &X->G[v - 1];
            if (!(g->fec_ts + 3000u <= S->max_ts || g->nsegs >= g->count))
                return;
            rx_remove(X, v - 1);
        } else {
            const uint32_t ts = (v & 0x80000000u) ? X->rh[v & 0x7FFFFFFFu].ts : X->R[v - 1].hdr.ts;
            if (!(ts + 6000u < S->max_ts))
                return;
            pm_del(&X->cache, key[b]);
        }
        if (key[b] == UINT32_MAX) {
            val[b] = NULL;
            continue;
        }
        ++key[b];
        val[b] = pm_next(rx_map(X, m), &key[b], &done[b]);
    }
}

/* sim_fec_evict (sim_fec.c:209-241) over the shards: flexes in fec_id order
 * while stale (fec_ts + 3000 <= max_ts) or full, removed with their members'
 * cache entries; then cached segments in packet_id order while older than 6 s
 * (timestamp + 6000 < max_ts); both walks stop at the first entry that stays
 * (rx_evict's rules over the union of the shards).  The records and rows the
 * evicted state held are dropped by the next compaction: here once the
 * session holds more than half its arena (an eviction per batch compacted per
 * batch, ~50 us of host time and a device gather each), else when a push
 * needs the room. */
int rfec_rx_session_evict(rfec_rx_session* S, void* stream)
{
    if (!S)
        return set_err(RFEC_EINVAL, "rx session: NULL", 0);
    for (uint32_t t = 0; t < S->T; ++t)
        S->XS[t]->max_ts = S->max_ts;
    if (S->T == 1) {
        rx_evict(S->XS[0]);
    } else {
        rx_evict_walk(S, 2);
        rx_evict_walk(S, 1);
    }
    for (uint32_t t = 0; t < S->T; ++t)
        if (S->XS[t]->oom)
            return set_err(RFEC_ENOMEM, "rx session: evict", 0);
    const uint32_t tail = S->pend >= 0 ? S->pend_n : 0;
    if (2ull * (S->nstore + tail) < S->arows)
        return RFEC_OK;
    return rx_compact(S, 0, (hipStream_t)stream);
}

int rfec_rx_session_get_info(const rfec_rx_session* S, rfec_rx_session_info* info)
{
    if (!S || !info)
        return set_err(RFEC_EINVAL, "rx session: NULL", 0);
    memset(info, 0, sizeof(*info));
    info->max_ts = S->max_ts;
    for (uint32_t t = 0; t < S->T; ++t) {
        info->open_flexes += S->XS[t]->flex_of.n;
        info->cached_segments += S->XS[t]->cache.n;
    }
    info->records_held = S->nstore;
    info->rows_held = S->arows;
    info->pending = S->pend >= 0 ? S->pend_n : 0;
    info->threads = S->T;
    info->batches_parallel = S->n_parallel;
    info->batches_serial = S->n_serial;
    info->batches_rolled_back = S->n_rollback;
    info->split_us = S->t_split;
    info->replay_us = S->t_replay;
    info->verify_us = S->t_verify;
    info->tables_us = S->t_tables;
    info->compact_us = S->t_compact;
    return RFEC_OK;
}
