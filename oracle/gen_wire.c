/*
 * gen_wire.c -- wire-codec golden vectors (own code, TEST INFRASTRUCTURE ONLY).
 * Links the reference's sim_proto.c, cf_stream.c and cf_crc32.c compiled out
 * of tree (oracle/Makefile) and writes, under tests/golden/:
 *
 *   wire_fec.bin    SIM_FEC messages: input fields + fec_data, then the
 *                   datagram sim_encode_msg produced (sim_proto.c:40-95)
 *   wire_seg.bin    SIM_SEG messages, same shape (sim_proto.inl:83-125)
 *   wire_parse.bin  datagrams (valid, corrupted, truncated, re-checksummed
 *                   with bad lengths / ids) and what sim_decode_header +
 *                   sim_decode_msg made of them (sim_proto.c:21-37, 99-146)
 *   wire_manifest.json
 *
 * Record layouts are mirrored by oracle/pyoracle.py (WIRE_* dtypes).
 * Usage: gen_wire <outdir>
 */
#include "cf_crc32.h"
#include "sim_proto.h"
#include "razor_fec.h" /* rfec_wire_rec, RFEC_WIRE_* (its sim types yield to the reference's) */

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void sim_encode_msg(bin_stream_t* strm, sim_header_t* header, void* body);
int sim_decode_header(bin_stream_t* strm, sim_header_t* header);
int sim_decode_msg(bin_stream_t* strm, sim_header_t* header, void* body);
uint64_t oracle_xs_next(uint64_t* state);
uint32_t oracle_xs_rand(uint64_t* state, uint32_t t);

#pragma pack(push, 1)
typedef struct {
    uint32_t uid, base_id, send_ts;
    uint16_t fec_id, count, transport_seq;
    uint8_t row, col, index, pad0;
    uint8_t meta[20];
    uint16_t fec_data_size, dlen;
    uint8_t pad1[2];
} wire_fec_in; /* 48 B, then fec_data[fec_data_size], then dgram[dlen] */

typedef struct {
    uint32_t uid, packet_id, fid, timestamp;
    uint16_t index, total;
    uint8_t ftype, payload_type, remb, pad0;
    uint16_t fec_id, send_ts, transport_seq, data_size, dlen;
    uint8_t pad1[2];
} wire_seg_in; /* 36 B, then data[data_size], then dgram[dlen] */

typedef struct {
    uint16_t len;
    uint8_t kind; /* 0 valid, 1 corrupted byte, 2 truncated + re-CRC, 3 length field + re-CRC,
                     4 mid + re-CRC, 5 trailing bytes + re-CRC, 6 random body + re-CRC */
    uint8_t pad[5];
    rfec_wire_rec rec; /* expected */
} wire_parse_in; /* 72 B, then dgram[len], then payload[rec.data_size] */
#pragma pack(pop)

static uint64_t g_st = 0x57495245ull; /* "WIRE" */
static uint32_t rnd(uint32_t t) { return oracle_xs_rand(&g_st, t); }
static uint32_t rnd32(void) { return (uint32_t)oracle_xs_next(&g_st); }

static FILE* out_file(const char* dir, const char* name)
{
    char p[512];
    snprintf(p, sizeof(p), "%s/%s", dir, name);
    FILE* f = fopen(p, "wb");
    if (!f) {
        perror(p);
        exit(1);
    }
    return f;
}

static uint16_t pick_size(int i)
{
    static const uint16_t edge[] = {0, 1, 2, 3, 4, 13, 15, 16, 17, 31, 32, 33, 63, 64, 999, 1000};
    if (i < (int)(sizeof(edge) / sizeof(edge[0])))
        return edge[i];
    return (uint16_t)rnd(SIM_VIDEO_SIZE);
}

/* encode with the reference into a fresh stream; returns its length */
static size_t ref_encode(uint8_t mid, uint32_t uid, void* body, uint8_t* out)
{
    bin_stream_t s;
    bin_stream_init(&s);
    sim_header_t h;
    INIT_SIM_HEADER(h, mid, uid);
    sim_encode_msg(&s, &h, body);
    memcpy(out, s.data, s.used);
    size_t n = s.used;
    bin_stream_destroy(&s);
    return n;
}

/* ---- parse cases ------------------------------------------------------------ */
typedef struct {
    uint8_t d[2048];
    size_t n;
} dgram_t;

static dgram_t* g_valid;
static int g_nvalid;

static void recrc(uint8_t* d, size_t n)
{
    uint32_t c = crc32(0x0e3dfc0a, d, n - 4);
    d[n - 4] = (uint8_t)(c >> 24);
    d[n - 3] = (uint8_t)(c >> 16);
    d[n - 2] = (uint8_t)(c >> 8);
    d[n - 1] = (uint8_t)c;
}

static void ref_parse(FILE* f, const uint8_t* d, size_t n, uint8_t kind)
{
    assert(n >= 4 && n <= 2048);
    bin_stream_t s;
    bin_stream_init(&s);
    bin_stream_resize(&s, 2048);
    memcpy(s.data, d, n);
    s.used = n; /* sim_session.c:338-345 */
    wire_parse_in r;
    memset(&r, 0, sizeof(r));
    r.len = (uint16_t)n;
    r.kind = kind;
    static sim_segment_t seg;
    static sim_fec_t fec;
    memset(&seg, 0, sizeof(seg));
    memset(&fec, 0, sizeof(fec));
    const uint8_t* payload = NULL;
    sim_header_t h;
    memset(&h, 0, sizeof(h));
    if (sim_decode_header(&s, &h) != 0) {
        r.rec.status = RFEC_WIRE_EBADCRC;
    } else {
        r.rec.ver = h.ver;
        r.rec.mid = h.mid;
        r.rec.uid = h.uid;
        if (h.mid < MIN_MSG_ID || h.mid > MAX_MSG_ID) { /* sim_session.c:594 */
            r.rec.status = RFEC_WIRE_EMID;
        } else if (h.mid == SIM_SEG) {
            int rc = sim_decode_msg(&s, &h, &seg);
            assert(rc == 0);
            r.rec.status = RFEC_WIRE_OK;
            r.rec.hdr.seq = seg.packet_id;
            r.rec.hdr.fid = seg.fid;
            r.rec.hdr.ts = seg.timestamp;
            r.rec.hdr.index = seg.index;
            r.rec.hdr.total = seg.total;
            r.rec.hdr.ftype = seg.ftype;
            r.rec.hdr.payload_type = seg.payload_type;
            r.rec.hdr.size = seg.data_size;
            r.rec.remb = seg.remb;
            r.rec.fec_id = seg.fec_id;
            r.rec.send_ts = seg.send_ts;
            r.rec.transport_seq = seg.transport_seq;
            r.rec.data_size = seg.data_size;
            payload = seg.data;
        } else if (h.mid == SIM_FEC) {
            int rc = sim_decode_msg(&s, &h, &fec);
            r.rec.status = rc == 0 ? RFEC_WIRE_OK : RFEC_WIRE_EBODY;
            r.rec.fec_id = fec.fec_id;
            r.rec.row = fec.row;
            r.rec.col = fec.col;
            r.rec.index = fec.index;
            r.rec.count = fec.count;
            r.rec.base_id = fec.base_id;
            r.rec.transport_seq = fec.transport_seq;
            r.rec.send_ts = fec.send_ts;
            r.rec.hdr.seq = fec.fec_meta.seq;
            r.rec.hdr.fid = fec.fec_meta.fid;
            r.rec.hdr.ts = fec.fec_meta.ts;
            r.rec.hdr.index = fec.fec_meta.index;
            r.rec.hdr.total = fec.fec_meta.total;
            r.rec.hdr.ftype = fec.fec_meta.ftype;
            r.rec.hdr.payload_type = fec.fec_meta.payload_type;
            r.rec.hdr.size = fec.fec_meta.size;
            r.rec.data_size = fec.fec_data_size;
            payload = fec.fec_data;
        } else {
            r.rec.status = RFEC_WIRE_OTHER;
        }
    }
    fwrite(&r, sizeof(r), 1, f);
    fwrite(d, 1, n, f);
    if (r.rec.data_size)
        fwrite(payload, 1, r.rec.data_size, f);
    bin_stream_destroy(&s);
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: gen_wire <outdir>\n");
        return 2;
    }
    const char* dir = argv[1];
    enum { NFEC = 160, NSEG = 240 };
    g_valid = (dgram_t*)calloc(NFEC + NSEG, sizeof(dgram_t));
    static uint8_t buf[4096];

    FILE* f = out_file(dir, "wire_fec.bin");
    static sim_fec_t fec;
    for (int i = 0; i < NFEC; ++i) {
        memset(&fec, 0, sizeof(fec));
        wire_fec_in in;
        memset(&in, 0, sizeof(in));
        in.uid = rnd32();
        fec.fec_id = in.fec_id = (uint16_t)rnd32();
        fec.row = in.row = (uint8_t)rnd32();
        fec.col = in.col = (uint8_t)rnd32();
        fec.index = in.index = (uint8_t)(i & 1 ? 0x80 | rnd(19) : rnd(19));
        fec.count = in.count = (uint16_t)(i % 5 == 0 ? rnd32() : rnd(100));
        fec.base_id = in.base_id = i % 3 == 0 ? rnd(65535) : rnd32();
        fec.send_ts = in.send_ts = rnd32();
        fec.transport_seq = in.transport_seq = (uint16_t)rnd32();
        fec.fec_meta.seq = rnd32();
        fec.fec_meta.fid = rnd32();
        fec.fec_meta.ts = rnd32();
        fec.fec_meta.index = (uint16_t)rnd32();
        fec.fec_meta.total = (uint16_t)rnd32();
        fec.fec_meta.ftype = (uint8_t)rnd32();
        fec.fec_meta.payload_type = (uint8_t)rnd32();
        fec.fec_meta.size = (uint16_t)rnd32();
        memcpy(in.meta, &fec.fec_meta, 20);
        fec.fec_data_size = in.fec_data_size = pick_size(i);
        for (int b = 0; b < fec.fec_data_size; ++b)
            fec.fec_data[b] = (uint8_t)rnd32();
        size_t n = ref_encode(SIM_FEC, in.uid, &fec, buf);
        in.dlen = (uint16_t)n;
        fwrite(&in, sizeof(in), 1, f);
        fwrite(fec.fec_data, 1, fec.fec_data_size, f);
        fwrite(buf, 1, n, f);
        memcpy(g_valid[g_nvalid].d, buf, n);
        g_valid[g_nvalid++].n = n;
    }
    fclose(f);

    f = out_file(dir, "wire_seg.bin");
    static sim_segment_t seg;
    for (int i = 0; i < NSEG; ++i) {
        memset(&seg, 0, sizeof(seg));
        wire_seg_in in;
        memset(&in, 0, sizeof(in));
        in.uid = rnd32();
        /* every combination of the mask's width bits (sim_proto.inl:85-98) */
        seg.packet_id = in.packet_id = (i & 1) ? 65536 + rnd32() % 0xFFFEFFFFu : rnd(65535);
        seg.fid = in.fid = (i & 2) ? 65536 + rnd32() % 0xFFFEFFFFu : rnd(65535);
        seg.total = in.total = (uint16_t)((i & 4) ? 256 + rnd(65279) : rnd(255));
        seg.index = in.index = (uint16_t)(seg.total ? rnd(seg.total - 1u) : 0);
        seg.remb = in.remb = (uint8_t)((i & 8) ? 0 : 1 + rnd(254));
        seg.ftype = in.ftype = (uint8_t)rnd(3);
        seg.payload_type = in.payload_type = (uint8_t)rnd32();
        seg.timestamp = in.timestamp = rnd32();
        seg.fec_id = in.fec_id = (uint16_t)rnd32();
        seg.send_ts = in.send_ts = (uint16_t)rnd32();
        seg.transport_seq = in.transport_seq = (uint16_t)rnd32();
        seg.data_size = in.data_size = pick_size(i >> 4 ? i - 16 : i);
        for (int b = 0; b < seg.data_size; ++b)
            seg.data[b] = (uint8_t)rnd32();
        size_t n = ref_encode(SIM_SEG, in.uid, &seg, buf);
        in.dlen = (uint16_t)n;
        fwrite(&in, sizeof(in), 1, f);
        fwrite(seg.data, 1, seg.data_size, f);
        fwrite(buf, 1, n, f);
        memcpy(g_valid[g_nvalid].d, buf, n);
        g_valid[g_nvalid++].n = n;
    }
    fclose(f);

    f = out_file(dir, "wire_parse.bin");
    long np = 0;
    for (int v = 0; v < g_nvalid; ++v) {
        dgram_t* s = &g_valid[v];
        ref_parse(f, s->d, s->n, 0);
        np++;
        uint8_t d[2048];
        /* 1: one byte flipped (CRC mismatch) */
        memcpy(d, s->d, s->n);
        d[rnd((uint32_t)s->n - 1)] ^= (uint8_t)(1 + rnd(254));
        ref_parse(f, d, s->n, 1);
        np++;
        /* 2: truncated, CRC recomputed: fields past the end read as 0 */
        if (v % 2 == 0) {
            size_t t = 4 + rnd((uint32_t)(s->n - 5));
            memcpy(d, s->d, t);
            recrc(d, t);
            ref_parse(f, d, t, 2);
            np++;
        }
        /* 3: data length field rewritten, CRC recomputed */
        if (v % 3 == 0) {
            memcpy(d, s->d, s->n);
            const int is_fec = s->d[1] == SIM_FEC;
            size_t lp;
            if (is_fec) {
                lp = 6 + 37;
            } else {
                const uint8_t m = s->d[6];
                lp = 6 + 2 + ((m & 0x80) ? 4 : 2) + ((m & 0x40) ? 4 : 2) + 4 + ((m & 0x20) ? 4 : 2) + 6;
            }
            const uint16_t cur = (uint16_t)(s->d[lp] << 8 | s->d[lp + 1]);
            static const uint16_t choices[] = {0xFFFF, 1001, 0};
            uint16_t nl = (v % 4 < 3) ? choices[v % 4] : (uint16_t)(cur + 1 + rnd(8));
            if (v % 7 == 0 && cur > 1)
                nl = (uint16_t)rnd(cur - 1u);
            d[lp] = (uint8_t)(nl >> 8);
            d[lp + 1] = (uint8_t)nl;
            recrc(d, s->n);
            ref_parse(f, d, s->n, 3);
            np++;
        }
        /* 4: message id rewritten, CRC recomputed */
        if (v % 5 == 0) {
            static const uint8_t mids[] = {0x0f, 0x1e, 0x1d, 0x15, 0x17, 0x1c, 0x10, 0x18};
            memcpy(d, s->d, s->n);
            d[1] = mids[(v / 5) % 8];
            recrc(d, s->n);
            ref_parse(f, d, s->n, 4);
            np++;
        }
        /* 5: trailing bytes appended, CRC recomputed */
        if (v % 4 == 1 && s->n + 40 <= 1500) {
            memcpy(d, s->d, s->n - 4);
            const size_t extra = 1 + rnd(35);
            for (size_t b = 0; b < extra; ++b)
                d[s->n - 4 + b] = (uint8_t)rnd32();
            const size_t t = s->n + extra;
            recrc(d, t);
            ref_parse(f, d, t, 5);
            np++;
        }
    }
    /* 6: random bodies under a SEG / FEC header, CRC valid */
    for (int i = 0; i < 200; ++i) {
        uint8_t d[2048];
        const size_t t = 6 + 4 + rnd(i < 100 ? 60 : 1100);
        for (size_t b = 0; b < t; ++b)
            d[b] = (uint8_t)rnd32();
        d[0] = 1;
        d[1] = (i & 1) ? SIM_FEC : SIM_SEG;
        if (i % 4 >= 2 && t > 50) { /* plausible data length field */
            const size_t lp = (i & 1) ? 43 : 26;
            const uint16_t nl = (uint16_t)rnd((uint32_t)(t - lp));
            d[lp] = (uint8_t)(nl >> 8);
            d[lp + 1] = (uint8_t)nl;
        }
        recrc(d, t);
        ref_parse(f, d, t, 6);
        np++;
    }
    fclose(f);

    f = out_file(dir, "wire_manifest.json");
    fprintf(f,
            "{\"generator\": \"oracle/gen_wire.c (reference sim_proto.c + cf_stream.c + cf_crc32.c)\",\n"
            " \"sim_video_size\": %d, \"crc_seed\": %u,\n"
            " \"fec\": {\"file\": \"wire_fec.bin\", \"count\": %d, \"record_bytes\": %zu},\n"
            " \"seg\": {\"file\": \"wire_seg.bin\", \"count\": %d, \"record_bytes\": %zu},\n"
            " \"parse\": {\"file\": \"wire_parse.bin\", \"count\": %ld, \"record_bytes\": %zu}}\n",
            SIM_VIDEO_SIZE, 0x0e3dfc0au, NFEC, sizeof(wire_fec_in), NSEG, sizeof(wire_seg_in), np,
            sizeof(wire_parse_in));
    fclose(f);
    fprintf(stderr, "wire fixtures: %d fec, %d seg, %ld parse\n", NFEC, NSEG, np);
    return 0;
}
