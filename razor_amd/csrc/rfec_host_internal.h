/*
 * rfec_host_internal.h -- declarations shared by the C host layer's
 * translation units (rfec_host.c, rfec_dropin.c, rfec_hostmem.c,
 * rfec_sender.c, rfec_rx.c).  Internal: hidden from the shared library's
 * exports.
 */
#ifndef RFEC_HOST_INTERNAL_H
#define RFEC_HOST_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "razor_fec.h"
#include "rfec_internal.h"

#pragma GCC visibility push(hidden)

/* rfec_host.c: the thread's last error (rfec_last_error), with the HIP error
 * string when hip_code != 0; returns code */
int set_err(int code, const char* what, int hip_code);
extern unsigned g_tuning; /* rfec_set_tuning */
int check_plan(const rfec_plan* p, uint32_t max_k);
int check_geometry(uint32_t groups, uint32_t stride, uint32_t capacity, uint32_t rows_per_group);
void make_masks(const rfec_plan* p, rfec_kmask* M);
uint32_t max_dlen(const uint16_t* dlen, uint32_t n);
double now_us(void); /* CLOCK_MONOTONIC, microseconds */
/* a tiny fork/join for the host gathers / scatters: fn(arg, lo, hi) over
 * [0, n) split across `threads` (RFEC_HOST_THREADS, default 8) */
typedef void (*pf_fn)(void* arg, size_t lo, size_t hi);
int host_threads(void);
void parallel_for(size_t n, int threads, pf_fn fn, void* arg);

/* rfec_dropin.c: the per-thread staging of the drop-in path, also used by the
 * host-memory batch paths and the sender staging */
#define DI_STRIDE ((SIM_VIDEO_SIZE + 15) & ~15)
#define DI_MAXK RFEC_MAX_K_ENCODE /* staging slots: a whole encode group, or the recover jobs' slots */

/* one pinned, device-mapped staging area per calling thread */
/* staging slots of the host-memory batch paths: 2 for the staged forms, 3
 * for the zero-copy forms (chunk c+2 is queued while chunk c still decodes
 * and scatters) */
#define RFEC_HB_SLOTS 3
typedef struct {
    int device;
    hipStream_t stream;
    uint8_t* host;   /* host view */
    uint8_t* dev;    /* device view of the same bytes */
    size_t bytes;
    /* rfec_host_encode_groups: two pinned host staging slots + their HBM
     * mirrors, one stream and four events per slot */
    uint8_t* bh;
    uint8_t* bh_dev; /* the device's address of bh (the zero-copy kernels read / write it) */
    uint8_t* bd;
    size_t bh_bytes, bd_bytes; /* the two pinned / device staging slots, together */
    hipStream_t bstream[2];
    hipEvent_t ev[RFEC_HB_SLOTS][4];
    int have_ev;
} di_ctx;
di_ctx* di_get(void);
/* rfec_hostmem.c: the pinned-block registry (rfec_pinned_alloc): 1 when [lo, hi) lies inside one block,
 * its device offset (device address - host address) in *delta; RFEC_HOST_ZEROCOPY != "0" */
int pinned_range(uintptr_t lo, uintptr_t hi, intptr_t* delta);
int zerocopy_on(void);
void seg_to_hdr(const sim_segment_t* s, rfec_hdr* h);
void stage_payload(uint8_t* slot, const uint8_t* data, uint32_t size);

#pragma GCC visibility pop

#endif
