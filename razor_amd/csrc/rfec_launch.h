// rfec_launch.h -- kernel launch of the HIP sources (C++ only).  Not installed.
//
// Kernel timing (rfec_timing_events, razor_fec.h): the next launch of the
// calling thread records its own start and stop on the caller's events
// (hipExtLaunchKernel: the kernel's dispatch timestamps), so the measured
// window is the kernel alone, without the dispatch gap a stream-event bracket
// around the call also holds.
#ifndef RFEC_LAUNCH_H_
#define RFEC_LAUNCH_H_

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

// counts the launch; true with the events (consumed) when the caller set them
bool rfec_timing_take(hipEvent_t* start, hipEvent_t* stop);

#define RFEC_LAUNCH(K, G, B, SH, ST, ...)                                                                          \
    do {                                                                                                           \
        hipEvent_t ev_a_, ev_z_;                                                                                   \
        if (rfec_timing_take(&ev_a_, &ev_z_))                                                                      \
            hipExtLaunchKernelGGL(K, G, B, SH, ST, ev_a_, ev_z_, 0u, __VA_ARGS__);                                 \
        else                                                                                                       \
            hipLaunchKernelGGL(K, G, B, SH, ST, __VA_ARGS__);                                                      \
    } while (0)

#endif
