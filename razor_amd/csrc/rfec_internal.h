/* rfec_internal.h -- contract between the C host layer (rfec_host.c) and the
 * HIP launch shim (rfec_kernels.hip).  Not installed. */
#ifndef RFEC_INTERNAL_H_
#define RFEC_INTERNAL_H_

#include "razor_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef rfec_plan rfec_kplan;

/* plan + per-line member bitmasks (bit i of mask[l] = segment i on line l) */
typedef struct {
    rfec_kplan plan;
    uint64_t mask[RFEC_MAX_LINES][2];
} rfec_kmask;

/* kernel flags == the RFEC_TUNE_* bits of razor_fec.h */
#define RFEC_KFLAG_GENERIC RFEC_TUNE_GENERIC
#define RFEC_KFLAG_MATRIX_GENERIC RFEC_TUNE_PLAN_CASCADE

int rfec_launch_encode(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                       const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                       uint16_t* fsize, int8_t* status, void* stream, unsigned flags);
int rfec_launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                        uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fsize, const uint64_t* parity_present,
                        uint64_t* recovered, void* ws, void* stream, unsigned flags);

/* dense output of rfec_recover_batch_out (device pointers; per_group > 0) */
typedef struct {
    uint8_t* shards;  /* [G][per_group][stride] */
    rfec_hdr* hdr;    /* [G][per_group] */
    uint8_t* index;   /* [G][per_group] */
    uint32_t per_group;
} rfec_dense_out;
int rfec_launch_recover_out(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                            const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                            const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                            const uint64_t* parity_present, uint64_t* recovered, void* ws, void* stream,
                            unsigned flags, const rfec_dense_out* out);

/* recover workspace, per group: the generic peel's schedule record (step
 * count, single-level flag, then a (line, target) byte pair per step), or the
 * cascade decode's 16-byte schedule record followed by one 4-byte task word
 * per output slot (max(k, n_lines) of them); 16-byte multiple */
static inline uint32_t rfec_sched_record_bytes(uint32_t k, uint32_t n_lines)
{
    const uint32_t peel = 2u + 2u * n_lines, casc = 16u + 4u * (k > n_lines ? k : n_lines);
    return ((peel > casc ? peel : casc) + 15u) & ~15u;
}
static inline size_t rfec_ws_bytes(uint32_t k, uint32_t n_lines, uint32_t groups)
{
    return (size_t)groups * rfec_sched_record_bytes(k, n_lines);
}
/* packed erasure records (rfec_pack_erasures / rfec_recover_packed_out): row layouts, rows of `col` <= 4,
 * k <= 64; group records of pk_stride bytes, slot records of pk_slot = 24 + 20 (col - 1) bytes */
int rfec_launch_pack_rows(const rfec_kplan* P, uint32_t col, uint32_t groups, const rfec_hdr* hdr,
                          const uint64_t* present, const rfec_hdr* meta, const uint16_t* fsize,
                          const uint64_t* parity_present, uint32_t per_group, uint8_t* packed, uint32_t pk_stride,
                          uint32_t pk_slot, void* stream);
int rfec_launch_recover_packed(const rfec_kmask* M, uint32_t col, uint32_t groups, uint32_t stride,
                               uint32_t capacity, const uint8_t* shards, const uint8_t* parity, const uint8_t* packed,
                               uint32_t pk_stride, uint32_t pk_slot, uint64_t* recovered,
                               const rfec_dense_out* out, void* stream);
int rfec_launch_wire_frame_fec(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                               const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                               const rfec_fec_stamp* stamps, const uint32_t* order, uint32_t dstride,
                               uint8_t* dgram, uint16_t* dlen, void* stream);
int rfec_launch_wire_frame_seg(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                               const rfec_hdr* hdr, const rfec_seg_stamp* stamps, const uint32_t* order,
                               uint32_t dstride, uint8_t* dgram, uint16_t* dlen, uint32_t rows_out, void* stream);
/* max_len: the longest datagram when the caller knows it (host-side lengths), else 0; slots
 * wider than 1,280 B still take the 20-byte-lane parse when every datagram fits 1,280 B */
int rfec_launch_wire_parse(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                           uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                           uint32_t max_len, void* stream);
int rfec_launch_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                            void* stream);
/* the receiver session's device stage (rfec_rx.c rx_device): dst row r <- src row map[r] (zeros for
 * map[r] < 0; `map` may be pinned host memory), and tbytes (a multiple of 16) of tables tsrc -> tdst */
int rfec_launch_rx_stage(uint8_t* dst, const uint8_t* src, const int32_t* map, uint32_t rows, uint32_t stride,
                         void* tdst, const void* tsrc, size_t tbytes, void* stream);
/* The receiver session's batch split, per parsed record (rfec_rx.c rx_phase0): its shard (fec_id % T, a
 * segment outside FEC by packet id; 0xFF: no effect on the control plane), its kind (RX_SPLIT_*) and the
 * value the replay's max_ts rules read (a segment's timestamp, a parity's send_ts + 3000). */
#define RX_SPLIT_NONE 0
#define RX_SPLIT_SEG_TS 1 /* SIM_SEG with fec_id and packet id: may raise max_ts */
#define RX_SPLIT_SEG 2
#define RX_SPLIT_FEC 3
typedef struct {
    uint8_t shard, kind;
    uint16_t reserved;
    uint32_t value;
} rfec_rx_split; /* 8 bytes */
int rfec_launch_rx_split(const rfec_wire_rec* recs, uint32_t n, uint32_t T, rfec_rx_split* out, void* stream);
/* rfec_launch_wire_parse with the receiver session's split entries of the parsed records (T shards) written
 * beside them (the quarter-wave parse writes them itself; the wave parses are followed by k_rx_split) */
int rfec_launch_wire_parse_split(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                                 uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload,
                                 uint32_t max_len, rfec_rx_split* split, uint32_t shards, void* stream);
/* receiver groups above RFEC_MAX_K segments: out row = parity row ^ member rows (one dependency level per call) */
typedef struct {
    int32_t out;       /* output row */
    int32_t parity;    /* row of `rows` holding the line's parity */
    uint32_t member0;  /* first member code in the member list */
    uint32_t n_members;
} rfec_line_job;
int rfec_launch_line_jobs(const rfec_line_job* jobs, uint32_t n_jobs, const int32_t* members, const uint8_t* rows,
                          uint8_t* outrows, uint32_t stride, void* stream);
int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream);
/* rfec_hostio.hip: razor's structs in device-mapped host memory <-> the slot
 * layout (pointer tables hold device addresses, 0 = a lost struct, bit 0 set =
 * header only: the payload is not read and its slot is zeroed).  One launch
 * gathers ns sim_segment_t (-> shards + header records) and nf sim_fec_t (->
 * parity slots + fec_meta records + fec_data_size + fec_id; nf may be 0) and
 * copies aux_n u64 words aux_src -> aux_dst (may be 0: none). */
int rfec_launch_host_gather(const uint64_t* sptrs, uint32_t ns, uint8_t* shards, rfec_hdr* hdr,
                            const uint64_t* fptrs, uint32_t nf, uint8_t* parity, rfec_hdr* meta, uint16_t* fsize,
                            uint16_t* fecid, uint32_t stride, uint32_t video, const uint64_t* aux_src,
                            uint64_t* aux_dst, uint32_t aux_n, void* stream);
/* sender staging (rfec_sender.c): slot s of `stride` bytes <- src[s] (device address of host bytes, any
 * alignment; 0: zeros) for size[s] bytes, zeros past them */
int rfec_launch_send_gather(const uint64_t* src, const uint16_t* size, uint32_t slots, uint32_t stride, uint8_t* dst,
                            void* stream);
/* parity slots of `groups` groups -> their sim_fec_t, stamped as flex_fec_sender_update does */
int rfec_launch_host_scatter_fec(const uint64_t* fptrs, uint32_t groups, const rfec_kplan* P, uint32_t stride,
                                 const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fsize,
                                 const int8_t* status, const rfec_hdr* hdr, uint16_t fec_id0, uint32_t g0,
                                 uint32_t video, void* stream);
/* dense recover output -> the callers' out_seg structs (flex_fec_recover's
 * fields + fec_id); out_index and the recovered masks into oidx_host / rec_host */
int rfec_launch_host_scatter_seg(const uint64_t* optrs, uint32_t groups, uint32_t E, uint32_t stride,
                                 const uint8_t* out_shards, const rfec_hdr* out_hdr, const uint8_t* out_index,
                                 const uint16_t* fecid, const uint64_t* ppm, uint32_t n_lines, uint32_t video,
                                 uint8_t* oidx_host, const uint64_t* recovered, uint64_t* rec_host, void* stream);
const char* rfec_hip_error_string(int code);

/* Group-level drop-in (rfec_flex.c) over the per-thread pinned, device-mapped
 * staging area of the single-call path (rfec_host.c): one launch and one
 * stream sync per call.  Both return RFEC_OK once the device work is done
 * (per-item results in rets[]), or an error code with rfec_last_error set. */
#define RFEC_DI_GROUPS 8 /* one-line recover jobs per launch */
typedef struct {
    sim_segment_t* const* segs; /* the present members */
    int count;
    sim_fec_t* fec;
    sim_segment_t* out;
} rfec_di_recover_job;
__attribute__((visibility("hidden"))) int rfec_di_generate_group(sim_segment_t* const* segs, int k,
                                                                 const rfec_plan* plan, sim_fec_t* const* outs,
                                                                 int* rets);
__attribute__((visibility("hidden"))) int rfec_di_recover_lines(const rfec_di_recover_job* jobs, int n, int* rets);
/* The resident service (rfec_service.hip): one workgroup polling a doorbell for
 * the drop-in's jobs.  Two control blocks of this layout: the request side
 * (bell, stop, quit, job; the staging slots follow it) in host-mapped device
 * memory or pinned host memory, the results side (done, alive, out; the output
 * slots follow it) in pinned host memory; with a host-memory request side
 * they are one block.  A job's payloads sit in staging slots 0..n_slots-1
 * (LDS slot s = staging slot s), zero-filled to the slot's end; its outputs go
 * to the output slots (encode: line l, recover: job g). */
#define RFEC_SVC_ENCODE 1u
#define RFEC_SVC_RECOVER 2u
#define RFEC_SVC_SLOTS 264 /* an encode group (<= 255 members) or the recover jobs' members + parities */
#define RFEC_SVC_MAX_GROUPS 8 /* workgroups of the service, each on its share of the chunk columns */
/* the doorbell word: job sequence number | n_slots << 32 | op << 48 */
#define RFEC_SVC_BELL(seq, ns, op) ((uint64_t)(uint32_t)(seq) | (uint64_t)(ns) << 32 | (uint64_t)(op) << 48)
typedef struct {
    uint32_t op, n_slots, groups, capacity;
    rfec_kplan plan;                   /* encode: the group's lines over slots 0..k-1 */
    uint16_t slot0[RFEC_DI_GROUPS];    /* recover job g: its first slot (members, then its parity) and the
                                        * first of its header records (the parity's meta, then the members') */
    uint16_t count[RFEC_DI_GROUPS];    /* present members */
    uint16_t fsize[RFEC_DI_GROUPS];    /* fec_data_size */
    uint16_t pad[RFEC_DI_GROUPS];
    uint8_t slot_nck[RFEC_SVC_SLOTS];  /* 16-byte chunks of the slot that hold its bytes (zeros follow) */
    uint32_t hdr[RFEC_SVC_SLOTS * 5];  /* encode: member i at 5 i; recover: as slot0 */
} rfec_svc_job;
typedef struct {
    uint64_t bell;                 /* host-written: RFEC_SVC_BELL, written last */
    uint32_t stop, pad0[13];       /* host-written: leave now */
    uint32_t done[RFEC_SVC_MAX_GROUPS], pad1[16 - RFEC_SVC_MAX_GROUPS]; /* device-written: workgroup w's last job */
    uint32_t alive, quit, pad2[14]; /* alive: 1 set by the host before a launch, 0 by workgroup 0 as it leaves;
                                     * quit: set by workgroup 0 before that, the others leave on it */
    struct {
        uint32_t meta[RFEC_MAX_LINES][5]; /* encode: line l's meta; recover: job g's recovered header */
        uint16_t fsize[RFEC_MAX_LINES];
        int8_t status[RFEC_MAX_LINES];    /* flex_fec_generate / flex_fec_recover's 0 / -1 */
        uint64_t t[2][4]; /* s_memrealtime of job seq at [seq & 1]: bell seen, job staged, results stored,
                           * drained; written after its `done` (the next job's drain lands it) */
    } out;
    rfec_svc_job job;
} rfec_svc_ctl;
int rfec_launch_service(rfec_svc_ctl* ctl, rfec_svc_ctl* in, const uint8_t* shards, uint8_t* out, uint32_t stride,
                        uint64_t idle_ticks, uint64_t life_ticks, uint32_t groups, void* stream);

__attribute__((visibility("hidden"))) int rfec_set_error(int code, const char* what);
/* sets rfec_last_error() from an errno value (0: `what` alone); returns code */
int rfec_set_error_sys(int code, const char* what, int err);

#ifdef __cplusplus
}
#endif

#endif
