/*
 * razor_fec.h -- C ABI of the MI355X-native flex-FEC engine.
 *
 * Two layers, both exported from librazor_fec.so:
 *
 *  1. Drop-in symbols with the reference signatures (link-compatible with the
 *     callers in sim_transport/fec/flex_fec_sender.c:175,219 and
 *     flex_fec_receiver.c:144,200):
 *        flex_fec_generate   replaces sim_transport/fec/flex_fec_xor.h:7 (.c:4-53)
 *        flex_fec_recover    replaces sim_transport/fec/flex_fec_xor.h:8 (.c:55-104)
 *     Each call runs on the GPU (one launch over a zero-copy staging area).
 *
 *  2. A batched, device-resident API (rfec_*): many independent FEC groups laid
 *     out structure-of-arrays in HBM, encoded / recovered by one kernel launch
 *     each.  The plan (which segments every parity line covers) restates
 *     flex_fec_sender_num_packets / flex_fec_sender_update
 *     (sim_transport/fec/flex_fec_sender.c:81-135, 146-245).
 *
 * All pointers passed to rfec_*_batch are DEVICE pointers; `stream` is a
 * hipStream_t passed as void* (NULL = the default stream).  Nothing in this
 * header needs HIP headers.
 */
#ifndef RAZOR_FEC_H_
#define RAZOR_FEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Reference ABI types (sim_transport/sim_proto.h:54, 80-99, 145-174).       */
/* When the reference's own sim_proto.h is already included, its definitions */
/* are used and these are skipped; the layouts are identical.                */
/* ------------------------------------------------------------------------ */
#ifndef SIM_VIDEO_SIZE
#define SIM_VIDEO_SIZE 1000 /* sim_proto.h:54 */
#endif

#ifndef __sim_proto_h_001__
typedef struct {
    uint32_t packet_id;     /* offset  0 */
    uint32_t fid;           /* offset  4 */
    uint32_t timestamp;     /* offset  8 */
    uint16_t index;         /* offset 12 */
    uint16_t total;         /* offset 14 */
    uint8_t ftype;          /* offset 16 */
    uint8_t payload_type;   /* offset 17 */
    uint8_t remb;           /* offset 18 */
    uint16_t fec_id;        /* offset 20 */
    uint16_t send_ts;       /* offset 22 */
    uint16_t transport_seq; /* offset 24 */
    uint32_t send_id;       /* offset 28 */
    uint16_t data_size;     /* offset 32 */
    uint8_t data[SIM_VIDEO_SIZE]; /* offset 34 (not 16-B aligned) */
} sim_segment_t;

typedef struct {
    uint32_t seq;  /* XOR of packet_id */
    uint32_t fid;
    uint32_t ts;   /* XOR of timestamp */
    uint16_t index;
    uint16_t total;
    uint8_t ftype;
    uint8_t payload_type;
    uint16_t size; /* XOR of data_size */
} sim_fec_meta_t;

typedef struct {
    uint16_t fec_id;        /* offset  0 */
    uint8_t row;            /* offset  2 */
    uint8_t col;            /* offset  3 */
    uint8_t index;          /* offset  4: row r, or 0x80|c for column c */
    uint16_t count;         /* offset  6 */
    uint32_t base_id;       /* offset  8 */
    uint32_t send_ts;       /* offset 12 */
    uint16_t transport_seq; /* offset 16 */
    sim_fec_meta_t fec_meta; /* offset 20 */
    uint16_t fec_data_size; /* offset 40 */
    uint8_t fec_data[SIM_VIDEO_SIZE]; /* offset 42 */
} sim_fec_t;
#endif /* __sim_proto_h_001__ */

/* Drop-in entry points: same names, argument meaning and 0 / -1 returns as
 * flex_fec_xor.c:4-53 and :55-104 (see DESIGN.md for the side effects kept). */
int flex_fec_generate(sim_segment_t* segs[], int segs_count, sim_fec_t* fec);
int flex_fec_recover(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, sim_segment_t* out_seg);

/* SIM_VIDEO_SIZE this library's drop-in symbols were compiled with. */
int rfec_sim_video_size(void);

/* ABI version of this header / library.  A caller compiled against one
 * header checks rfec_abi_version() == RFEC_ABI_VERSION before using structs
 * whose size changed.  History: 5 -- rfec_host_timing grew from 48 to 56
 * bytes (zero_copy, reserved); 6 -- rfec_abi_version, rfec_rx_session_info grew
 * from 24 to 88 bytes (threads, batches_*, the host time split),
 * rfec_rx_session_set_threads; 7 -- rfec_send_report grew from 64 to 72 bytes
 * (zero_copy, reserved). */
#define RFEC_ABI_VERSION 7
uint32_t rfec_abi_version(void);

/* ------------------------------------------------------------------------ */
/* Batched device API                                                        */
/* ------------------------------------------------------------------------ */
#define RFEC_MAX_K 128     /* segments per group in recovery (sim_sender.c:370 flushes at 100) */
#define RFEC_MAX_K_ENCODE 255 /* segments per group in an encode plan (rfec_line's 8-bit fields; razor's
                                 flex sender keeps row and col in uint8_t, so no line exceeds it) */
#define RFEC_MAX_LINES 64  /* parity lines per group */

#define RFEC_OK 0
#define RFEC_EINVAL (-1)
#define RFEC_EDEVICE (-2)
#define RFEC_ENOMEM (-3)

/* 20-byte header record.  Field order and widths are sim_fec_meta_t's, so the
 * XOR of several records, taken as five 32-bit words, is the record of the
 * XORed fields (flex_fec_xor.c:13-20, 37-44, 64-85). */
typedef struct {
    uint32_t seq;   /* packet_id */
    uint32_t fid;
    uint32_t ts;    /* timestamp */
    uint16_t index;
    uint16_t total;
    uint8_t ftype;
    uint8_t payload_type;
    uint16_t size;  /* data_size */
} rfec_hdr;

/* One parity line: members first, first+stride, ..., first+(count-1)*stride. */
typedef struct {
    uint8_t first;
    uint8_t stride;
    uint8_t count;
    uint8_t index; /* sim_fec_t.index: row r, or 0x80|c (flex_fec_sender.c:180,224) */
} rfec_line;

#define RFEC_LAYER_ROWS 1u
#define RFEC_LAYER_COLS 2u

typedef struct {
    uint16_t k;        /* segments per group */
    uint8_t row, col;  /* matrix shape (flex_fec_sender_t.row/.col) */
    uint8_t rc;        /* 1 when the planner chose matrix mode */
    uint8_t n_lines;   /* parity lines emitted (lines with <2 members dropped) */
    uint8_t n_row_lines;
    uint8_t reserved;
    rfec_line line[RFEC_MAX_LINES]; /* rows first, then columns, reference order */
} rfec_plan;

/* Restates flex_fec_sender_num_packets (flex_fec_sender.c:81-135).  Writes
 * row/col and returns rc (0 strip mode, 1 matrix mode); k==0 -> (0,0). */
int rfec_num_packets(uint16_t k, uint8_t protect_fraction, uint8_t* row, uint8_t* col);

/* Plan of flex_fec_sender_update (flex_fec_sender.c:146-245) for a group of
 * k segments at the given protect_fraction, restricted to `layers`.  Lines
 * whose flex_fec_generate would fail (fewer than 2 members) are dropped, as
 * the reference drops them.  Returns RFEC_OK or RFEC_EINVAL. */
int rfec_plan_from_fraction(uint16_t k, uint8_t protect_fraction, unsigned layers, rfec_plan* plan);

/* Plan for an explicit row x col matrix over k segments (rows of `col`
 * consecutive segments, columns strided by `col`). */
int rfec_plan_matrix(uint16_t k, uint8_t row, uint8_t col, unsigned layers, rfec_plan* plan);

/*
 * Device layout (G groups, k segments, n = plan->n_lines):
 *   shards  [G][k][stride] u8    payloads, bytes beyond data_size MUST be 0
 *   hdr     [G][k]         rfec_hdr
 *   parity  [G][n][stride] u8    fec_data; bytes beyond fec_data_size are 0
 *   meta    [G][n]         rfec_hdr  (fec_meta)
 *   fec_size[G][n]         u16   (fec_data_size)
 *   status  [G][n]         i8    0, or -1 where flex_fec_generate returns -1
 * stride is a multiple of 16 and >= capacity; capacity plays SIM_VIDEO_SIZE.
 */
int rfec_encode_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                      const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                      uint16_t* fec_size, int8_t* status, void* stream);

/*
 * Peeling recovery (flex_fec_receiver.c:105-206 + the cascade of
 * sim_receiver.c:780-804), batched:
 *   shards/hdr       in/out: erased slots are filled with the recovered segment
 *   present          [G][2] u64: bit i = segment i was received
 *   parity/meta/fec_size as produced by rfec_encode_batch
 *   parity_present   [G] u64: bit l = parity line l was received
 *   recovered        [G][2] u64 out: bit i = segment i was recovered here
 *   workspace        rfec_recover_workspace_size(plan, G) bytes of device memory
 *                    (one peeling-schedule record per group, used by the
 *                    generic peel + replay), 16-byte aligned; its contents
 *                    need no initialisation
 * A line recovers its single missing member only under the conditions of
 * flex_recover_row/col and flex_fec_recover (sizes within fec_data_size).
 * `recovered` is authoritative: an erased slot whose bit stays clear holds
 * unspecified bytes afterwards (the fused decode may have written it).
 */
size_t rfec_recover_workspace_size(const rfec_plan* plan, uint32_t groups);
int rfec_recover_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                       uint8_t* shards, rfec_hdr* hdr, const uint64_t* present,
                       const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                       const uint64_t* parity_present, uint64_t* recovered, void* workspace,
                       void* stream);

/*
 * Recovery into a dense output, as flex_fec_recover writes each recovered
 * segment into a caller-allocated out_seg (flex_fec_xor.c:55-104,
 * flex_fec_receiver.c:142-143): the shards and headers are only read.  The
 * e-th erased segment of group g (e-th in segment-index order among the
 * segments whose present bit is clear, e < per_group) goes to
 *   out_shards [g*per_group + e][stride]   payload bytes [0, fec_data_size)
 *   out_hdr    [g*per_group + e]           its recovered header record
 *   out_index  [g*per_group + e]           its segment index, or 0xFF where
 *                                          that erased segment was not recovered
 *                                          (its out_shards slot then holds
 *                                          unspecified bytes)
 * and `recovered` gets its bit as in rfec_recover_batch.  Any plan: where
 * lines cascade (rows + columns), a recovered segment feeds the lines after
 * it as in place.  Only erased segments of rank < per_group are recovered
 * (they are the ones with an output slot), so with per_group at least the
 * group's erasure count the result is rfec_recover_batch's; with fewer slots
 * the peel runs as if the segments of higher rank could not be recovered.
 * Same workspace as rfec_recover_batch.
 */
int rfec_recover_batch_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                           const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                           const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                           const uint64_t* parity_present, uint64_t* recovered, uint32_t per_group,
                           uint8_t* out_shards, rfec_hdr* out_hdr, uint8_t* out_index, void* workspace,
                           void* stream);

/*
 * Packed erasure records: the header input of rfec_recover_batch_out for row
 * layouts (rows of `col` consecutive segments and no columns -- strip mode or
 * the row layer alone, flex_fec_sender.c:166-190; k <= 64, col <= 4) laid out
 * per erased segment, so a decode reads one contiguous run per group instead
 * of the present / parity_present / fec_size / meta / hdr arrays, whose
 * sectors it shares with the rows that do not fire.  Group g's record,
 * rfec_packed_stride(plan, per_group) bytes (a multiple of 64) at
 * packed + g * stride:
 *   +0   u64 present         bit i = segment i was received
 *   +8   u64 parity_present  bit r = row r's parity was received
 *   +16 + e * S, e < per_group, S = 24 + 20 (col - 1): the group's e-th erased
 *        segment (index order), in row r:
 *        rfec_hdr meta of row r; u16 fec_data_size of row r; u16 0;
 *        rfec_hdr of row r's other members in index order (zeros past the
 *        row's end).  All zeros where the group has fewer than e + 1 erasures.
 *   zeros up to the stride.
 * A receiver that knows the plan can write these as segments and parities
 * arrive (each segment's record goes to the slot of every erased segment of
 * its row); rfec_pack_erasures builds them from the batch layout.
 * rfec_recover_packed_out then gives rfec_recover_batch_out's results for the
 * same batch (out_shards, out_hdr, out_index, recovered) with no workspace.
 * rfec_packed_stride returns 0 for a plan outside the row layouts above or a
 * per_group outside [1, k].  (razor's flex_fec_receiver.c:105-206 reads the
 * same fields per line; the layout is this library's.)
 */
size_t rfec_packed_stride(const rfec_plan* plan, uint32_t per_group);
int rfec_pack_erasures(const rfec_plan* plan, uint32_t groups, const rfec_hdr* hdr, const uint64_t* present,
                       const rfec_hdr* meta, const uint16_t* fec_size, const uint64_t* parity_present,
                       uint32_t per_group, uint8_t* packed, void* stream);
int rfec_recover_packed_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                            const uint8_t* shards, const uint8_t* parity, const uint8_t* packed,
                            uint64_t* recovered, uint32_t per_group, uint8_t* out_shards, rfec_hdr* out_hdr,
                            uint8_t* out_index, void* stream);

/*
 * Host-resident batch: the path that starts and ends in host memory (segments
 * built from UDP socket buffers, sim_session.c).  Gathers G groups of
 * sim_segment_t (segs[g*k + i], this library's SIM_VIDEO_SIZE layout) into a
 * pinned structure-of-arrays staging area, copies it to HBM, runs
 * rfec_encode_batch, copies the parities back and scatters them into the
 * caller's sim_fec_t (fecs[g*n + l]) stamped like flex_fec_sender_update
 * (flex_fec_sender.c:176-181, 220-225: fec_id = fec_id0 + g, base_id = the
 * group's smallest packet_id, row, col, index, count).  A line whose
 * flex_fec_generate would fail gets fec_data_size = 0xFFFF and no payload.
 * `timing` (may be NULL) receives the per-stage wall times in microseconds.
 * Staging is per calling thread and grows on demand.
 *
 * Zero copy: when every segs / fecs pointer lies inside one block from
 * rfec_pinned_alloc (and RFEC_HOST_ZEROCOPY is not "0"), no host gather or
 * scatter runs -- the device reads the sim_segment_t and writes the sim_fec_t
 * through the block's device mapping over PCIe, and only the pointer tables
 * are staged (timing->zero_copy = 1; gather_us is then the host's table
 * build, h2d_us the device's gathers over PCIe, kernel_us the encode / decode,
 * d2h_us the device's scatter, scatter_us the copy of out_index / recovered).
 */
typedef struct {
    double gather_us, h2d_us, kernel_us, d2h_us, scatter_us, total_us;
    uint32_t zero_copy, reserved;
} rfec_host_timing;

int rfec_host_encode_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                            sim_fec_t* const* fecs, uint16_t fec_id0, rfec_host_timing* timing);

/*
 * The receive direction of rfec_host_encode_groups: G groups in host memory,
 * segs[g*k + i] the received sim_segment_t of member i or NULL where it was
 * lost, fecs[g*n + l] the received sim_fec_t of line l or NULL.  Gathers them
 * into the pinned staging (payload slots, header records, the present and
 * parity-present masks, the parities' meta / fec_data_size / payload), copies
 * it to HBM, runs rfec_recover_batch_out with per_group dense slots, copies
 * the recovered slots back and scatters them like flex_fec_recover's out_seg
 * (flex_fec_xor.c:64-101): out[g*per_group + e] receives the group's e-th
 * erased segment (index order) when the peel recovered it -- header fields,
 * data_size, SIM_VIDEO_SIZE bytes of data (zero past the recovering line's
 * fec_data_size), fec_id of the group's parities -- and out_index[g*per_group
 * + e] its member index, 0xFF when it was not recovered (out[...] untouched).
 * recovered (may be NULL): [G][2] masks.  Chunked and double-buffered as the
 * encode; k <= RFEC_MAX_K.  timing: gather = staging, scatter = delivery.
 */
int rfec_host_recover_groups(const rfec_plan* plan, uint32_t groups, sim_segment_t* const* segs,
                             sim_fec_t* const* fecs, uint32_t per_group, sim_segment_t* const* out,
                             uint8_t* out_index, uint64_t* recovered, rfec_host_timing* timing);

/* Kernel timing for benches: the next kernel this thread launches through the
 * batched API (rfec_encode_batch, rfec_recover_batch[_out], rfec_zero_tails,
 * rfec_wire_frame_fec / _seg, rfec_wire_parse) records its own start / stop on these hipEvent_t (either may be NULL), via
 * hipExtLaunchKernel; the setting is consumed by that launch.
 * rfec_timing_launches: kernels launched by this thread since the last
 * rfec_timing_events (a call that launched more than one kernel timed only
 * its first). */
int rfec_timing_events(void* start, void* stop);
uint32_t rfec_timing_launches(void);

/* Zero bytes [data_size, stride) of every shard (establishes the layout
 * invariant for callers that cannot guarantee it). */
int rfec_zero_tails(uint32_t groups, uint32_t k, uint32_t stride, uint8_t* shards,
                    const rfec_hdr* hdr, void* stream);

/* ------------------------------------------------------------------------ */
/* Wire codec, batched on the device: the SIM_FEC / SIM_SEG datagrams of     */
/* sim_encode_msg / sim_decode_header + sim_decode_msg (sim_proto.c:13-146,  */
/* sim_proto.inl:83-179, 244-307), big-endian fields (cf_stream.c:328-414),  */
/* CRC32 trailer (cf_crc32.c:56-68, seed 0x0e3dfc0a, sim_proto.c:11).        */
/*                                                                          */
/* A datagram is: ver, mid, uid (6 B, sim_proto.c:13-18) | body | crc32 of   */
/* everything before it, big-endian (sim_proto.c:92-94).  Datagram slots are */
/* [N][dstride] bytes, dstride a multiple of 16 in [64, 2048]; lengths are   */
/* u16 per slot.  Bytes of a slot beyond its length are written as 0.        */
/* ------------------------------------------------------------------------ */
#define RFEC_WIRE_VER 0x01        /* protocol_ver, sim_proto.h:39 */
#define RFEC_WIRE_SEG 0x17        /* SIM_SEG, sim_proto.h:17-29 */
#define RFEC_WIRE_FEC 0x1c        /* SIM_FEC, sim_proto.h:34 */
#define RFEC_WIRE_MIN_MID 0x10    /* MIN_MSG_ID */
#define RFEC_WIRE_MAX_MID 0x1d    /* MAX_MSG_ID (accepted, sim_session.c:594) */
#define RFEC_WIRE_CRC_SEED 0x0e3dfc0au
#define RFEC_WIRE_FEC_OVERHEAD 49 /* 6 + 17 + 20 + 2 + 4 bytes around fec_data */
#define RFEC_WIRE_MAX_DSTRIDE 2048

/* Per-datagram fields of a SIM_FEC the FEC engine does not produce: the
 * session uid (sim_proto.c:13-18) and the sim_fec_t stamps of the sender
 * (flex_fec_sender.c:176-181, 220-225; sim_sender.c:112-113). */
typedef struct {
    uint32_t uid;
    uint32_t base_id;
    uint32_t send_ts;
    uint16_t fec_id;
    uint16_t count;
    uint16_t transport_seq;
    uint8_t row, col, index;
    uint8_t reserved;
    uint8_t pad[2];
} rfec_fec_stamp; /* 24 bytes */

/* Per-datagram fields of a SIM_SEG beyond rfec_hdr (sim_sender.c:88-91, 335-351). */
typedef struct {
    uint32_t uid;
    uint16_t fec_id;
    uint16_t send_ts;
    uint16_t transport_seq;
    uint8_t remb;
    uint8_t reserved;
} rfec_seg_stamp; /* 12 bytes */

/* SIM_FEC datagrams (sim_sender.c:118-119 + sim_fec_encode,
 * sim_proto.inl:270-285) of `count` parity slots laid out as rfec_encode_batch
 * wrote them (slot g*n + l = line l of group g): datagram i -> dgram slot i.
 * `status` may be NULL; a slot with status -1 gets length 0 (the reference
 * never emits that parity).  `order` may be NULL; otherwise datagram i is
 * written to slot order[i] of dgram / dlen (a permutation).  Needs
 * fec_size <= capacity <= stride and dstride >= capacity + 49.  Datagram
 * slots whose stride is a multiple of 128 bytes (1,280 for 1,200-byte
 * payloads) are written in whole 128-byte lines: 0.60 of HBM peak against
 * 0.52 for the minimal 16-byte multiples, whose slot edges split lines
 * (DESIGN.md §4). */
int rfec_wire_frame_fec(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                        const rfec_fec_stamp* stamps, const uint32_t* order, uint32_t dstride, uint8_t* dgram,
                        uint16_t* dlen, void* stream);

/* SIM_SEG datagrams (sim_sender.c:96-97 + sim_segment_encode,
 * sim_proto.inl:83-125; header widths follow the value ranges) of `count`
 * segments: shards [count][stride], hdr [count]; `order` as for
 * rfec_wire_frame_fec.  Needs data_size <= capacity <= stride and
 * dstride >= capacity + 36. */
int rfec_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                        const rfec_hdr* hdr, const rfec_seg_stamp* stamps, const uint32_t* order, uint32_t dstride,
                        uint8_t* dgram, uint16_t* dlen, void* stream);

/* Parse status (rfec_wire_rec.status). */
#define RFEC_WIRE_OK 0         /* SIM_SEG / SIM_FEC decoded (a SEG with a bad data length decodes
                                  with data_size 0, as sim_segment_decode does) */
#define RFEC_WIRE_OTHER 1      /* valid control message (CONNECT, PING, ...): header only */
#define RFEC_WIRE_EBADCRC (-1) /* sim_decode_header: CRC mismatch, or shorter than the trailer */
#define RFEC_WIRE_EMID (-2)    /* mid outside [MIN_MSG_ID, MAX_MSG_ID] (sim_session.c:594) */
#define RFEC_WIRE_EBODY (-3)   /* sim_fec_decode returned -1 (fec_data length invalid) */

/* One parsed datagram.  SIM_SEG: hdr = the segment's header (seq=packet_id,
 * fid, ts=timestamp, index, total, ftype, payload_type, size=data_size),
 * fec_id, send_ts (u16 widened), transport_seq, remb.  SIM_FEC: hdr = fec_meta,
 * the sim_fec_t fields, data_size = fec_data_size. */
typedef struct {
    int8_t status;
    uint8_t ver, mid, remb;
    uint32_t uid;
    rfec_hdr hdr;
    uint32_t base_id;
    uint32_t send_ts;
    uint16_t fec_id;
    uint16_t count;
    uint16_t transport_seq;
    uint16_t data_size;
    uint8_t row, col, index;
    uint8_t reserved[17];
} rfec_wire_rec; /* 64 bytes */

/* Decode N received datagrams (sim_session.c:587-653 -> sim_decode_header,
 * sim_decode_msg) into recs [N] and their payloads into slots [N][stride]
 * (zero beyond data_size: the layout rfec_recover_batch expects).  `capacity`
 * plays SIM_VIDEO_SIZE in the length checks (cf_stream.c:342-355,
 * sim_proto.inl:301-305); capacity <= stride. */
int rfec_wire_parse(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                    uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                    void* stream);

/* ------------------------------------------------------------------------ */
/* Sender staging: sim_sender_put (sim_sender.c:306-377) with sim_split_frame */
/* (:254-284) and the flex sender's grouping (flex_fec_sender.c:49-78,       */
/* 137-245), as a plan over a batch of frames, then frame bytes copied       */
/* straight into pinned structure-of-arrays slots.                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t* data;      /* frame bytes (host) */
    uint32_t size;
    uint8_t payload_type, ftype;
    uint8_t protect_fraction; /* s->loss_fraction when the frame is put (sim_sender.c:291) */
    uint8_t reserved;
    int64_t now_ms;           /* GET_SYS_MS() during sim_sender_put */
} rfec_frame;

/* The sim_sender_t / flex_fec_sender_t fields that shape segments and groups. */
typedef struct {
    uint32_t packet_id_seed, send_id_seed, frame_id_seed;
    int64_t first_ts;   /* -1 before the first frame (sim_sender.c:333-338) */
    int64_t fec_ts;     /* flex->fec_ts (0 = unset) */
    uint32_t base_id;   /* flex->base_id */
    int32_t open_seg;   /* the open group's first segment, relative to the next batch (<= 0) */
    uint16_t fec_id;    /* flex->fec_id, starts at 1, skips 0 */
    uint16_t segs_count;
    int32_t first;      /* flex->first */
    uint32_t transport_seq_seed; /* sender->transport_seq_seed (sim_sender.c:90, 112), u16 on the wire */
} rfec_sender_state;

/* One segment the sender builds (sim_sender.c:341-363). */
typedef struct {
    uint32_t frame;        /* index into the frame batch */
    uint32_t offset;       /* byte offset in the frame */
    uint32_t packet_id, send_id, fid, timestamp;
    uint16_t index, total, data_size, fec_id;
    uint8_t ftype, payload_type;
    uint8_t reserved[2];
    int32_t group;         /* group index in this batch, -1 if never protected */
} rfec_seg_plan; /* 40 bytes */

/* One protected group: a flex_fec_sender_update that emitted parities. */
typedef struct {
    int32_t first_seg;     /* segments [first_seg, first_seg + count) of the batch; negative:
                              the first -first_seg were planned by the previous call */
    uint16_t count, fec_id;
    uint32_t base_id;      /* smallest packet_id of the group */
    uint32_t fec_send_id0; /* send ids of its parities: fec_send_id0 + line (sim_sender.c:295-296) */
    uint32_t fec_ts;       /* now_ms - first_ts when it closed (sim_sender.c:299) */
    uint8_t protect_fraction, n_lines;
    uint8_t reserved[2];
} rfec_group_plan; /* 24 bytes */

void rfec_sender_init(rfec_sender_state* st);
/* Plans `n` frames: the segments sim_sender_put builds (segs, at most
 * max_segs) and the groups flex_fec_sender_update protects (groups, at most
 * max_groups), in creation order; `st` carries the sender across calls.  A
 * group still open after the last frame stays open in `st` (its segments have
 * group -2); the call that closes it reports a negative first_seg.
 * seg_size = the sender's SIM_VIDEO_SIZE.  Returns RFEC_OK, or RFEC_EINVAL
 * when an output array is too small (nothing is consumed then). */
int rfec_sender_plan(rfec_sender_state* st, const rfec_frame* frames, uint32_t n, uint32_t seg_size,
                     rfec_seg_plan* segs, uint32_t max_segs, uint32_t* n_segs, rfec_group_plan* groups,
                     uint32_t max_groups, uint32_t* n_groups);

/* Frames in, datagrams out (host memory both ends): rfec_sender_plan, the
 * frame bytes copied once into pinned structure-of-arrays slots (groups of
 * one shape contiguous, so each shape is one rfec_encode_batch), one H2D
 * copy, the encode, rfec_wire_frame_seg / _fec, one D2H copy per datagram
 * kind.  Datagrams come out in creation order: seg_dgram[i] is segs[i]'s
 * SIM_SEG, fec_dgram holds the parities group by group, lines in plan order.
 * transport_seq counts datagrams in creation order (a group's parities right
 * after the segment that closed it); send_ts is that of an immediate send
 * (sim_sender.c:88-91, 111-113).  seg_size is this library's SIM_VIDEO_SIZE;
 * the segments of a group still open at the end are kept (per calling thread)
 * and encoded by the call that closes it.
 *
 * Zero copy (RFEC_HOST_ZEROCOPY not "0"): when every frame's bytes lie inside
 * one rfec_pinned_alloc block, the device reads the segments out of the frames
 * itself (no host copy into the staging slots, no bulk H2D: h2d_us is then the
 * tables' copy and the device's reads); when the four datagram outputs lie in
 * such blocks, the framing writes the datagrams there (no D2H; the writes fall
 * in kernel_us).  report->zero_copy: bit 0 input, bit 1 output. */
typedef struct {
    uint32_t n_segs, n_groups, n_parities, n_shapes;
    double plan_us, stage_us, h2d_us, kernel_us, d2h_us, total_us;
    uint32_t zero_copy, reserved;
} rfec_send_report;

int rfec_host_send_frames(rfec_sender_state* st, const rfec_frame* frames, uint32_t n_frames, uint32_t uid,
                          rfec_seg_plan* segs, uint32_t max_segs, rfec_group_plan* groups, uint32_t max_groups,
                          uint32_t dstride, uint8_t* seg_dgram, uint16_t* seg_dlen, uint8_t* fec_dgram,
                          uint16_t* fec_dlen, uint32_t max_parities, rfec_send_report* report);

/* ------------------------------------------------------------------------ */
/* Receiver ingestion: the receiver-side FEC of one session over a batch of */
/* parsed datagrams in arrival order (sim_receiver_put / _put_fec,          */
/* sim_receiver.c:780-838 -> sim_fec_put_segment / sim_fec_put_fec_packet,  */
/* sim_fec.c:104-207 -> flex receiver, flex_fec_receiver.c:69-280).         */
/* The control plane replays the reference event by event over the 64-byte  */
/* records on the host: first-arrival dedupe, max_ts (raised by recovered   */
/* segments too), the 3000 ms parity drop (sim_fec.c:148), flex creation    */
/* from the first admitted parity and removal when full, and which line     */
/* recovers which packet and when (so a packet recovered before its own     */
/* late arrival is delivered, as the reference does).  The bytes stay on    */
/* the device: every group is peeled by rfec_recover_batch from its arrived */
/* members and registered parities, and the delivered rows are gathered.    */
/* Not modelled (counted in n_unmodelled, never delivered wrong): the       */
/* wall-clock eviction of sim_fec_evict, parity lines outside the sender's  */
/* row/column plan, geometries the planner cannot express (count > 128 or   */
/* row * col < count) and parities inconsistent with their members.         */
/* Output: the recovered segments, ascending packet_id.                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    rfec_hdr hdr;     /* recovered header (flex_fec_xor.c:64-85) */
    uint16_t fec_id;  /* out_seg->fec_id = fec->fec_id (:101) */
    uint16_t reserved;
} rfec_rx_seg; /* 24 bytes */

typedef struct {
    uint32_t n_groups, n_shapes, n_recovered, n_fec_dropped, n_unmodelled, reserved;
    double host_us, h2d_us, kernel_us, d2h_us, total_us;
} rfec_rx_report;

/* recs / payload: DEVICE (rfec_wire_parse output), n records in arrival
 * order, payload rows of `stride` bytes.  max_ts: in/out
 * (sim_receiver_fec_t.max_ts).  out / out_payload: HOST, up to max_out
 * recovered segments (payload rows of `stride`, zero beyond data_size). */
int rfec_rx_recover(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                    uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out,
                    uint32_t* n_out, rfec_rx_report* report, void* stream);

/* ------------------------------------------------------------------------ */
/* Batched UDP I/O: the datagram path of sim_session (sim_session.c:286-296 */
/* send, :321-364 receive loop) over posix.c's socket calls (su_udp_create  */
/* :133-170, su_udp_send :240-243, su_udp_recv :245-275), moved from one    */
/* sendto / select+recvfrom per datagram to sendmmsg / recvmmsg over the    */
/* [N][dstride] datagram slots the wire codec reads and writes.  Host-only  */
/* (no HIP); slot buffers are best pinned (hipHostMalloc) so the same block */
/* is the DMA source / target of the H2D / D2H copies.                      */
/* ------------------------------------------------------------------------ */
#define RFEC_EAGAIN (-4)           /* the socket stayed blocked for wait_ms */
#define RFEC_EIO (-5)              /* a socket call failed (errno in rfec_last_error) */
#define RFEC_UDP_SERVER 1u         /* SU_SERVER build: 1 MiB buffers, non-blocking (posix.c:135-160) */
#define RFEC_UDP_RECV_BYTES 1500u  /* receive buffer per datagram (sim_session.c:333) */
#define RFEC_UDP_MIN_DGRAM 6u      /* SIM_HEADER_SIZE: shorter datagrams are ignored (sim_session.c:339) */

typedef struct {
    uint32_t ip;   /* host byte order */
    uint16_t port; /* host byte order */
    uint16_t reserved;
} rfec_udp_addr;

typedef struct {
    uint64_t datagrams;  /* sent / received (kept) datagrams: s->scount / s->rcount */
    uint64_t bytes;      /* their bytes: s->sbandwidth / s->rbandwidth (sim_session.c:291, 343) */
    uint64_t skipped;    /* send: slots of length 0 (sim_session_network_send returns -1, :287-288) */
    uint64_t dropped;    /* recv: datagrams shorter than RFEC_UDP_MIN_DGRAM */
    uint64_t truncated;  /* recv: datagrams longer than the slot (MSG_TRUNC; their CRC then fails) */
    uint64_t syscalls;   /* sendmmsg / recvmmsg calls */
    uint64_t stalls;     /* send: waits for buffer space; recv: waits for data */
} rfec_udp_stats;

/* su_udp_create (posix.c:133-170): a UDP socket bound to ip:port (ip NULL or
 * "" = INADDR_ANY, port 0 = any), SO_SNDBUF / SO_RCVBUF = buf_bytes (0 = the
 * reference's 1 MiB with RFEC_UDP_SERVER, 128 KiB without), non-blocking
 * with RFEC_UDP_SERVER.  `bound` (may be NULL) receives the bound address. */
int rfec_udp_open(const char* ip, uint16_t port, unsigned flags, uint32_t buf_bytes, int* fd, rfec_udp_addr* bound);
void rfec_udp_close(int fd);
/* su_set_addr (posix.c:282-288) */
int rfec_udp_addr_of(const char* ip, uint16_t port, rfec_udp_addr* addr);

/* Sends slots [0, n) of dgram ([n][dstride], lengths dlen) to `peer` in slot
 * order, up to 1024 per sendmmsg; slots of length 0 are skipped.  When the
 * socket is full it waits for space up to wait_ms per stall (0: no wait) and
 * then returns RFEC_EAGAIN; *n_done (may be NULL) = slots consumed so far, so
 * the call can be resumed at that slot.  `st` (may be NULL) accumulates. */
int rfec_udp_send_batch(int fd, const rfec_udp_addr* peer, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                        const uint16_t* dlen, uint32_t wait_ms, uint32_t* n_done, rfec_udp_stats* st);

/* Receives up to `max` datagrams into consecutive slots of dgram ([max][dstride],
 * at most RFEC_UDP_RECV_BYTES of each datagram; slot bytes past the length
 * are not written) with their lengths in dlen and sources in `from` (may be
 * NULL).  Waits up to wait_ms for the first datagram, as su_udp_recv's select
 * does (0: no wait), then takes what is queued without waiting.  Datagrams
 * shorter than RFEC_UDP_MIN_DGRAM are dropped, as the session loop does.
 * *n = datagrams stored (0 after a quiet wait_ms: RFEC_OK). */
int rfec_udp_recv_batch(int fd, uint32_t max, uint32_t dstride, uint8_t* dgram, uint16_t* dlen, rfec_udp_addr* from,
                        uint32_t wait_ms, uint32_t* n, rfec_udp_stats* st);

/* Received datagrams in host memory -> recovered segments in host memory: one
 * H2D of the slots, rfec_wire_parse, rfec_rx_recover (arrival order = slot
 * order).  recs_out (HOST, may be NULL) receives the n parse records.  The
 * device staging is per calling thread.  rfec_rx_report.h2d_us includes the
 * datagram H2D; parse time is in kernel_us. */
int rfec_host_recv_datagrams(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                             uint32_t stride, uint32_t capacity, uint32_t* max_ts, rfec_wire_rec* recs_out,
                             rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                             rfec_rx_report* report);

/* Pinned host memory the device maps (hipHostMalloc / hipHostFree): datagram
 * slots, and struct pools for the zero-copy form of rfec_host_encode_groups /
 * rfec_host_recover_groups (each block is registered with its device address
 * until rfec_pinned_free). */
void* rfec_pinned_alloc(size_t bytes);
void rfec_pinned_free(void* p);

/* ------------------------------------------------------------------------ */
/* Receiver session: the receiver-side FEC state of one sim_session          */
/* (sim_receiver_fec_t, sim_fec.c) kept from one batch of datagrams to the   */
/* next -- open flex receivers, the segment cache, max_ts, first-arrival     */
/* dedupe -- with every cached segment's and registered parity's payload row */
/* held in HBM, so a group whose datagrams straddle batches recovers exactly */
/* as in one stream.  rfec_rx_session_evict is sim_fec_evict (sim_fec.c:    */
/* 209-241) for the caller's heartbeat (sim_receiver_timer, sim_receiver.c: */
/* 880, every >= 300 ms): stale or full flexes in fec_id order, cached      */
/* segments older than 6 s in packet_id order; then the held rows are       */
/* compacted.  Pushing a stream in any batches, with evictions between      */
/* batches, delivers what rfec_rx_recover delivers on the whole stream with */
/* the same evictions.  One session per calling thread at a time.           */
/* ------------------------------------------------------------------------ */
typedef struct rfec_rx_session rfec_rx_session;

typedef struct {
    uint32_t max_ts;          /* sim_receiver_fec_t.max_ts */
    uint32_t open_flexes;     /* skiplist_size(f->flexes) */
    uint32_t cached_segments; /* skiplist_size(f->segs_cache) */
    uint32_t records_held;    /* parsed records kept for open state */
    uint32_t rows_held;       /* HBM payload rows allocated */
    uint32_t pending;         /* datagrams of the batch the last _async call
                                 started: the records its next call writes */
    uint32_t threads;         /* control-plane shards (1: serial) */
    uint32_t batches_parallel;    /* batches replayed by the shards in parallel */
    uint32_t batches_serial;      /* batches replayed in arrival order */
    uint32_t batches_rolled_back; /* parallel replays undone (then replayed in order) */
    uint32_t reserved;
    /* host time, microseconds, summed over the session's batches: */
    double split_us;   /* the batch split over the shards (serial) */
    double replay_us;  /* the control plane's replay (the shards in parallel, or in order) */
    double verify_us;  /* the packet-id ownership check (parallel) */
    double tables_us;  /* the device tables of the delivering groups (rx_device, host part) */
    double compact_us; /* record / row compaction (rfec_rx_session_evict, and when the arena fills) */
} rfec_rx_session_info;

/* NULL on bad arguments (stride % 16, capacity > stride) or no memory.
 *
 * The control plane is sharded by fec_id over RFEC_RX_THREADS (default 8)
 * shards, each replayed in arrival order by its own thread: groups are
 * independent in the reference (sim_fec.c:141-207 keys a flex by fec_id).
 * Deliveries are those of the serial replay, always: a batch runs in parallel
 * only while every packet id belongs to one fec_id and no parity of the batch
 * can meet the 3 s drop (sim_fec.c:148) through max_ts; one that breaks either
 * is rolled back and replayed in arrival order (a packet id under two fec_ids
 * merges the shards into one for the rest of the session). */
rfec_rx_session* rfec_rx_session_create(uint32_t stride, uint32_t capacity);
/* Control-plane shards / threads (1..64) of a session that has not been
 * pushed to yet; 1 = the serial replay. */
int rfec_rx_session_set_threads(rfec_rx_session* s, uint32_t threads);
void rfec_rx_session_destroy(rfec_rx_session* s);
/* recs / payload: DEVICE (rfec_wire_parse output, rows of the session's
 * stride), n records in arrival order; out / out_payload: HOST, the segments
 * recovered by this batch, ascending packet_id.  As rfec_rx_recover. */
int rfec_rx_session_push(rfec_rx_session* s, uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload,
                         rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                         rfec_rx_report* report, void* stream);
/* Received datagram slots in HOST memory (rfec_udp_recv_batch's output):
 * rfec_wire_parse, rfec_rx_session_push.  Pinned slots (rfec_pinned_alloc)
 * are read by the parse kernel itself, pageable ones copied first; a pinned
 * out_payload is gathered into directly.  recs_out (HOST, may be NULL)
 * receives the n parse records.  Refused while a pipelined batch is pending. */
int rfec_rx_session_push_datagrams(rfec_rx_session* s, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                   const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                   uint8_t* out_payload, uint32_t max_out, uint32_t* n_out, rfec_rx_report* report);
/* Pipelined form, one batch of latency: starts the parse of these n
 * datagrams on the session's own stream, then ingests the batch the previous
 * call started (control plane, peel) while the device parses this one, and
 * returns THAT batch's recovered segments.  recs_out (HOST, may be NULL)
 * receives THAT batch's records too, so it must hold the PREVIOUS call's n
 * records (rfec_rx_session_get_info's `pending`), not this call's.  dgram /
 * dlen must stay unchanged until the next call on the session returns.
 * n == 0 only ingests the pending batch (the flush).  Deliveries, in total
 * and in order, equal rfec_rx_session_push_datagrams over the same batches;
 * rfec_rx_session_evict may come between calls. */
int rfec_rx_session_push_datagrams_async(rfec_rx_session* s, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                                         const uint16_t* dlen, rfec_wire_rec* recs_out, rfec_rx_seg* out,
                                         uint8_t* out_payload, uint32_t max_out, uint32_t* n_out,
                                         rfec_rx_report* report);
int rfec_rx_session_evict(rfec_rx_session* s, void* stream);
int rfec_rx_session_get_info(const rfec_rx_session* s, rfec_rx_session_info* info);

/* Kernel selection, for tests: 0 = the default kernels (specialised where the
 * plan allows); RFEC_TUNE_GENERIC = the plan-driven kernels for every plan
 * (encode: one lane per (group, chunk column) over the plan's lines; recover
 * in place: the LDS peel + schedule replay), the cross-check of the
 * specialised ones.  Other bits: below, or ignored. */
#define RFEC_TUNE_GENERIC 1u
/* RFEC_TUNE_PLAN_CASCADE: a dense recover of the sender's matrix plan
 * (k = 6..16) takes the plan-driven cascade kernel instead of the one
 * compiled for its shape (the A/B and cross-check of the latter). */
#define RFEC_TUNE_PLAN_CASCADE (1u << 2)
/* RFEC_TUNE_WAVE_PARSE: rfec_wire_parse takes the wave-per-datagram kernel
 * instead of the quarter-wave one (the A/B and cross-check of the latter). */
#define RFEC_TUNE_WAVE_PARSE (1u << 3)
/* RFEC_TUNE_NO_SERVICE: the drop-in symbols (flex_fec_generate / _recover, the
 * group-level sender and receiver) launch their kernels per call instead of
 * posting to the resident service (process-wide; also RFEC_SERVICE=0 in the
 * environment).  Bit 30, so that no value of the round-1/2 tuning bits
 * (1u << 1 .. 1u << 24, now ignored) turns the service off. */
#define RFEC_TUNE_NO_SERVICE (1u << 30)
void rfec_set_tuning(unsigned flags);
unsigned rfec_get_tuning(void);

/* The drop-in's resident service: RFEC_SERVICE_GROUPS (default 1, at most 8)
 * workgroups that stay on the device and take the drop-in symbols' jobs from
 * a doorbell (no launch, no stream synchronisation per call), each on its
 * share of a job's 16-byte columns.  It starts on the
 * first drop-in call and leaves the device by itself after RFEC_SERVICE_IDLE_US
 * (default 2000) microseconds without a job, after RFEC_SERVICE_LIFE_US (default
 * 4000) in total (the next call starts it again) and at exit.  The request side
 * (doorbell, job, staged segments) sits in device memory the host writes
 * through its mapping when the runtime maps it (large-BAR hosts), else in
 * pinned host memory (also with RFEC_SERVICE_STAGE=host).  rfec_service_stop() makes it leave
 * now and waits for it; it returns RFEC_OK (also when it was not running) or
 * RFEC_EDEVICE.  rfec_service_get_info reports the calls served, the
 * launches made and where a call's time goes (means over the calls served). */
typedef struct {
    uint64_t jobs;       /* drop-in calls served */
    uint64_t launches;   /* workgroup launches (the first call, then after each idle exit) */
    double stage_host_us; /* mean, per job: the host copying the segments next to the doorbell */
    double wait_us;      /* doorbell written -> `done` seen by the host */
    double dev_stage_us; /* on the device: doorbell seen -> the job's slots in LDS */
    double dev_work_us;  /* -> results stored */
    double dev_release_us; /* -> the results' stores acknowledged, before `done` */
    uint32_t request_in_device; /* 1: the request side is in host-mapped device memory */
    uint32_t reserved;
} rfec_service_info;
int rfec_service_stop(void);
int rfec_service_get_info(rfec_service_info* info);

/* HBM ceiling probes (measurement only, not on the FEC path): streaming
 * read / copy / write of `bytes` (multiple of 16) in the FEC kernels' access
 * shape.  flags bit0 = non-temporal, bit1 = 4 vectors per lane.  `sink` of
 * rfec_probe_read needs 16 KiB.  Return 0 or a HIP error code. */
int rfec_probe_read(const void* src, size_t bytes, void* sink, unsigned flags, void* stream);
int rfec_probe_copy(const void* src, void* dst, size_t bytes, unsigned flags, void* stream);
int rfec_probe_write(void* dst, size_t bytes, unsigned flags, void* stream);
/* r read streams : w write streams of stream_bytes each (src holds r, dst w
 * streams back to back), lane i XORs chunk i of every read stream into chunk
 * i of every write stream, non-temporal: the ceiling of the encodes' read /
 * write mixes.  (r, w) in {(10, 3), (10, 7), (4, 1), (1, 1)}, else -1. */
int rfec_probe_mix(const void* src, void* dst, size_t stream_bytes, unsigned r, unsigned w, void* stream);

/* Synthetic inputs of SURVEY.md §8(d) (bench and tests only, not on the FEC
 * path): payload slots of groups [g0, g0 + groups) of the xorshift64*
 * stream seeded 0x52415A4F52464543 ^ config_id, filled group-major and
 * shard-major, S bytes per slot from ceil(S / 8) outputs (little endian),
 * zero to `stride`.  The slice is reached by jump-ahead, so a rank fills its
 * own part of a batch without the outputs before it.  Synchronises `stream`.
 * Returns RFEC_OK, RFEC_EINVAL or RFEC_EDEVICE. */
int rfec_fill_xorshift(uint8_t* shards, uint64_t config_id, uint64_t g0, uint32_t groups, uint32_t k, uint32_t S,
                       uint32_t stride, void* stream);
/* The xorshift64* state n steps after x (GF(2) jump-ahead; host only). */
uint64_t rfec_xorshift_jump(uint64_t x, uint64_t n);

/* Last HIP error string seen by this thread (for diagnostics). */
const char* rfec_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* RAZOR_FEC_H_ */
