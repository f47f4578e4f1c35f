/*
 * razor_flex.h -- group-level drop-in of razor's flex FEC sender / receiver
 * (sim_transport/fec/flex_fec_sender.h, flex_fec_receiver.h), exported from
 * librazor_fec.so next to the line-level flex_fec_generate / flex_fec_recover
 * of razor_fec.h.
 *
 * Linking razor with librazor_fec.so in place of flex_fec_xor.c,
 * flex_fec_sender.c AND flex_fec_receiver.c keeps every
 * caller unchanged (sim_sender.c:150-370, sim_fec.c:93-241, test_func.c) and
 * moves the FEC work from one GPU round trip per parity line to one per call:
 *
 *   flex_fec_sender_update       all row + column parities of the group in one
 *                                launch (was: one flex_fec_generate per line,
 *                                flex_fec_sender.c:158-233)
 *   flex_fec_receiver_on_segment the row and the column recovery an arriving
 *                                segment triggers in one launch (was: two
 *                                flex_fec_recover calls, flex_fec_receiver.c:243-280)
 *
 * Same names, argument meaning, return values, ownership (the receiver frees
 * the parities it holds; recovered segments are malloc'd for the caller) and
 * struct layouts as the reference headers; the receiver keeps its member /
 * parity tables in its own storage behind the public struct, so `segs` and
 * `fecs` are NULL (no caller of the reference touches them).
 *
 * The outputs go into the caller's cf_list (common/cf_list.h): this library
 * calls the application's list_push / list_clear when it links cf_list.c, or
 * an equivalent push onto the same base_list_t layout when it does not.
 */
#ifndef RAZOR_FLEX_H_
#define RAZOR_FLEX_H_

#include "razor_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef __WB_LIST_H_ /* common/cf_list.h:17-27 */
typedef struct base_list_unit_t {
    struct base_list_unit_t* next;
    void* pdata;
} base_list_unit_t;

typedef struct {
    base_list_unit_t* head;
    base_list_unit_t* tailer;
    size_t size;
} base_list_t;
#endif

#ifndef __flex_fec_sender_h_ /* flex_fec_sender.h:7-24 */
typedef struct {
    uint16_t fec_id;
    uint8_t row;
    uint8_t col;
    uint32_t base_id;
    int first;
    int64_t fec_ts;
    uint16_t seg_size;
    uint16_t segs_count; /* read by sim_sender.c:370 */
    sim_segment_t** segs;
    uint16_t cache_size;
    sim_segment_t** cache;
} flex_fec_sender_t;
#endif

/* flex_fec_sender.c:8-19, 21-36, 38-46, 49-78, 146-245, 247-260, 81-135 */
flex_fec_sender_t* flex_fec_sender_create(void);
void flex_fec_sender_destroy(flex_fec_sender_t* fec);
void flex_fec_sender_reset(flex_fec_sender_t* fec);
void flex_fec_sender_add_segment(flex_fec_sender_t* fec, sim_segment_t* seg);
void flex_fec_sender_update(flex_fec_sender_t* fec, uint8_t protect_fraction, base_list_t* out_fecs);
void flex_fec_sender_release(flex_fec_sender_t* fec, base_list_t* out_fecs);
int flex_fec_sender_num_packets(flex_fec_sender_t* fec, uint8_t protect_fraction);

#ifndef __flex_fec_receiver_h_ /* flex_fec_receiver.h:8-35 */
typedef void (*flex_fec_free_f)(sim_fec_t* fec, void* args);
typedef void (*flex_segment_free_f)(sim_segment_t* fec, void* args);

typedef struct {
    uint16_t fec_id;
    uint8_t col;
    uint8_t row;
    uint32_t base_id;
    uint16_t count;
    int inited;
    void* segs; /* skiplist_t* in the reference; NULL here */
    void* fecs; /* skiplist_t* in the reference; NULL here */
    uint16_t cache_size;
    sim_segment_t** cache;
    uint32_t fec_ts; /* set by sim_fec.c:159, read by sim_fec_evict (:225) */
    flex_fec_free_f flex_fec_free_cb;
    flex_segment_free_f flex_seg_free_cb;
    void* args;
} flex_fec_receiver_t;
#endif

/* flex_fec_receiver.c:15-30, 32-51, 53-67, 69-88, 90-96, 208-241, 243-280
 * ("desotry" is the reference's spelling) */
flex_fec_receiver_t* flex_fec_receiver_create(flex_segment_free_f seg_free, flex_fec_free_f fec_free, void* args);
void flex_fec_receiver_desotry(flex_fec_receiver_t* r);
void flex_fec_receiver_reset(flex_fec_receiver_t* r);
void flex_fec_receiver_active(flex_fec_receiver_t* r, uint16_t fec_id, uint8_t col, uint8_t row, uint32_t base_id,
                              uint16_t count);
int flex_fec_receiver_full(flex_fec_receiver_t* r);
sim_segment_t* flex_fec_receiver_on_fec(flex_fec_receiver_t* r, sim_fec_t* fec);
int flex_fec_receiver_on_segment(flex_fec_receiver_t* r, sim_segment_t* seg, base_list_t* out);

#ifdef __cplusplus
}
#endif

#endif
