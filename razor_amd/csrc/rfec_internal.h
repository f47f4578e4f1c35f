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

/* one peeling step replayed by the recovery XOR kernel; slot 0 of a group's
 * record holds the step count in `first` */
typedef struct {
    uint8_t first, stride, count, q; /* line geometry, q = target's position on it */
    uint8_t line, target;
    uint8_t pad[2];
} rfec_step;

#define RFEC_KFLAG_GENERIC 1u  /* never use the specialised row kernels */
#define RFEC_KFLAG_TEMPORAL 2u /* plain (not non-temporal) loads/stores */

int rfec_launch_encode(const rfec_kplan* P, uint32_t groups, uint32_t stride, uint32_t capacity,
                       const uint8_t* shards, const rfec_hdr* hdr, uint8_t* parity, rfec_hdr* meta,
                       uint16_t* fsize, int8_t* status, void* stream, unsigned flags);
int rfec_launch_recover(const rfec_kmask* M, uint32_t groups, uint32_t stride, uint32_t capacity,
                        uint8_t* shards, rfec_hdr* hdr, const uint64_t* present, const uint8_t* parity,
                        const rfec_hdr* meta, const uint16_t* fsize, const uint64_t* parity_present,
                        uint64_t* recovered, void* ws, uint32_t ws_stride, void* stream, unsigned flags);
int rfec_launch_zero_tails(uint32_t slots, uint32_t stride, uint8_t* shards, const rfec_hdr* hdr, void* stream);
const char* rfec_hip_error_string(int code);

#ifdef __cplusplus
}
#endif

#endif
