/*
 * rfec_oracle.h -- CPU restatement of razor's flex-FEC path.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / CPU baseline.  The product
 * (librazor_fec.so) never links or calls anything in oracle/.
 *
 * Parity pinning: checked bit-for-bit against the reference C compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref/) through the golden
 * fixtures in tests/golden/ (generator: oracle/gen_golden.c).
 */
#ifndef RFEC_ORACLE_H_
#define RFEC_ORACLE_H_

#include "razor_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* xorshift64* as in test/common_test.c:10-16 */
uint64_t oracle_xs_next(uint64_t* state);
/* cf_rand (test/common_test.c:18-26): uniform integer in [0, t] */
uint32_t oracle_xs_rand(uint64_t* state, uint32_t t);

/* Synthetic group fill.  shards [G][k][stride], hdr [G][k].
 * ragged==0: data_size = S; else data_size = 1 + cf_rand(S-1) from a second
 * stream, bytes beyond data_size zeroed.  seed = 0x52415A4F52464543 ^ config_id. */
void oracle_fill_groups(uint64_t config_id, uint32_t groups, uint32_t k, uint32_t S, uint32_t stride,
                        int ragged, uint8_t* shards, rfec_hdr* hdr);
/* The same stream in pieces: groups [g0, g0+groups) written at shards/hdr[0];
 * state = {0, 0} before the first piece, carried between pieces. */
void oracle_fill_stream(uint64_t config_id, uint64_t state[2], uint32_t g0, uint32_t groups, uint32_t k,
                        uint32_t S, uint32_t stride, int ragged, uint8_t* shards, rfec_hdr* hdr);

/* flex_fec_xor.c:4-53 with SIM_VIDEO_SIZE replaced by `capacity`. */
int oracle_generate(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, int capacity);
/* flex_fec_xor.c:55-104 */
int oracle_recover(sim_segment_t* segs[], int segs_count, sim_fec_t* fec, sim_segment_t* out_seg);

/* flex_fec_sender.c:81-135 */
int oracle_num_packets(int segs_count, int protect_fraction, int* row, int* col);
/* flex_fec_sender.c:146-245 line layout */
int oracle_plan_from_fraction(int k, int protect_fraction, unsigned layers, rfec_plan* plan);
int oracle_plan_matrix(int k, int row, int col, unsigned layers, rfec_plan* plan);

/* Batched restatements over the device layout (include/razor_fec.h). */
void oracle_encode_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                         const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                         uint16_t* fec_size, int8_t* status);
void oracle_recover_batch(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                          uint8_t* shards, rfec_hdr* hdr, const uint64_t* present,
                          const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                          const uint64_t* parity_present, uint64_t* recovered);
/* rfec_recover_batch_out's semantics (include/razor_fec.h): the same peel on a
 * copy of each group in which only erased segments of rank < per_group may be
 * recovered; out slot e = the e-th erased segment (bytes, header, index or 0xFF). */
void oracle_recover_batch_out(const rfec_plan* plan, uint32_t groups, uint32_t stride, uint32_t capacity,
                              const uint8_t* shards, const rfec_hdr* hdr, const uint64_t* present,
                              const uint8_t* parity, const rfec_hdr* meta, const uint16_t* fec_size,
                              const uint64_t* parity_present, uint64_t* recovered, uint32_t per_group,
                              uint8_t* out_shards, rfec_hdr* out_hdr, uint8_t* out_index);

/* Reference-shaped CPU path for the baseline: per group, builds sim_segment_t*
 * arrays over AoS segments (segs[G*k], each sizeof(sim_segment_t) at this
 * build's SIM_VIDEO_SIZE) and calls oracle_generate once per plan line,
 * exactly as flex_fec_sender_update does.  Returns parities produced. */
long oracle_encode_aos(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs);
/* Same, split over `threads` pthreads by contiguous group ranges. */
long oracle_encode_aos_mt(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                          int threads);
/* Per group, recover the erased segments of `present` from row/col parities
 * with oracle_recover (canonical peel order).  Returns segments recovered. */
long oracle_recover_aos(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs,
                        sim_fec_t* fecs, const uint64_t* present, sim_segment_t* out);
long oracle_recover_aos_mt(const rfec_plan* plan, uint32_t groups, sim_segment_t* segs, sim_fec_t* fecs,
                           const uint64_t* present, sim_segment_t* out, int threads);

/* wire codec (sim_proto.c, sim_proto.inl, cf_stream.c, cf_crc32.c) */
uint32_t oracle_crc32(uint32_t crc, const void* buf, size_t size);
size_t oracle_wire_frame_fec(const sim_fec_t* f, uint32_t uid, uint8_t* out);
size_t oracle_wire_frame_seg(const sim_segment_t* s, uint32_t uid, uint8_t* out);
int oracle_wire_parse(const uint8_t* d, size_t len, uint32_t capacity, rfec_wire_rec* rec, uint8_t* payload);
void oracle_wire_frame_fec_batch(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* parity,
                                 const rfec_hdr* meta, const uint16_t* fec_size, const int8_t* status,
                                 const rfec_fec_stamp* stamps, uint32_t dstride, uint8_t* dgram, uint16_t* dlen);
void oracle_wire_frame_seg_batch(uint32_t count, uint32_t stride, uint32_t capacity, const uint8_t* shards,
                                 const rfec_hdr* hdr, const rfec_seg_stamp* stamps, uint32_t dstride, uint8_t* dgram,
                                 uint16_t* dlen);
void oracle_wire_parse_batch(uint32_t n, uint32_t dstride, const uint8_t* dgram, const uint16_t* dlen,
                             uint32_t stride, uint32_t capacity, rfec_wire_rec* recs, uint8_t* payload);

/* sender staging (sim_sender.c:254-377, flex_fec_sender.c:49-245) */
void oracle_sender_init(rfec_sender_state* st);
int oracle_sender_plan(rfec_sender_state* st, const rfec_frame* frames, uint32_t n, uint32_t seg_size,
                       rfec_seg_plan* segs, uint32_t max_segs, uint32_t* n_segs, rfec_group_plan* groups,
                       uint32_t max_groups, uint32_t* n_groups);

/* receiver ingestion, event by event (sim_fec.c:104-207, flex_fec_receiver.c:69-280,
 * sim_receiver.c:780-838); out in delivery order */
int oracle_rx_recover(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                      uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload, uint32_t max_out,
                      uint32_t* n_out, uint32_t* dropped);
/* the same with sim_fec_evict (sim_fec.c:209-241) after every evict_every arrivals (0: never) */
int oracle_rx_recover_ev(uint32_t n, const rfec_wire_rec* recs, const uint8_t* payload, uint32_t stride,
                         uint32_t capacity, uint32_t* max_ts, rfec_rx_seg* out, uint8_t* out_payload,
                         uint32_t max_out, uint32_t* n_out, uint32_t* dropped, uint32_t evict_every);

int oracle_sim_video_size(void);
size_t oracle_segment_size(void);
size_t oracle_fec_size(void);

#ifdef __cplusplus
}
#endif

#endif
