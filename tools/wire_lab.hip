// wire_lab.hip -- cost breakdown of the wire kernels (measurement only, not on
// the product path): the product source compiled with one RFEC_WIRE_DIAG_*
// switch, k_frame_seg and k_parse timed on the bench workload (655,360 SIM_SEG
// datagrams of 1,200-byte payloads, 1,248-byte slots).
//
// build (tools/wire_lab.sh does all variants):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Irazor_amd/csrc [-DRFEC_WIRE_DIAG_NO_CRC ...] \
//         tools/wire_lab.hip -o tools/bin/wire_lab_<variant>
// run:   tools/bin/wire_lab_<variant> [reps=20] [dstride=1248] [payload stride=1200]
#include "bin/wire_lab_src/rfec_wire.hip"

// (the product's kernel-own timing hook, rfec_kernels.hip: no events here)
bool rfec_timing_take(hipEvent_t*, hipEvent_t*) { return false; }

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint32_t N = 655360, S = 1200, DS = argc > 2 ? (uint32_t)atoi(argv[2]) : 1248; // datagram slot stride
    const uint32_t PS = argc > 3 ? (uint32_t)atoi(argv[3]) : S;                       // parse payload slot stride
    std::vector<uint8_t> sh((size_t)N * S);
    uint64_t x = 0x52415A4F52464543ull;
    for (size_t i = 0; i < sh.size(); i += 8) {
        x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
        const uint64_t v = x * 2685821657736338717ull;
        std::memcpy(&sh[i], &v, std::min<size_t>(8, sh.size() - i));
    }
    std::vector<rfec_hdr> hdr(N);
    std::vector<rfec_seg_stamp> st(N);
    for (uint32_t i = 0; i < N; ++i) {
        hdr[i] = rfec_hdr{};
        hdr[i].seq = 1 + i;
        hdr[i].fid = 1 + i / 10;
        hdr[i].ts = 33 * (i / 10);
        hdr[i].index = (uint16_t)(i % 10);
        hdr[i].total = 10;
        hdr[i].payload_type = 96;
        hdr[i].size = (uint16_t)S;
        st[i] = rfec_seg_stamp{};
        st[i].uid = 7;
        st[i].fec_id = (uint16_t)(1 + i / 10);
        st[i].transport_seq = (uint16_t)i;
    }
    uint8_t *d_sh, *d_dg, *d_pay;
    rfec_hdr* d_hdr;
    rfec_seg_stamp* d_st;
    uint16_t* d_len;
    rfec_wire_rec* d_rec;
    CK(hipMalloc(&d_sh, sh.size()));
    CK(hipMalloc(&d_dg, (size_t)N * DS));
    CK(hipMalloc(&d_pay, (size_t)N * PS));
    CK(hipMalloc(&d_hdr, N * sizeof(rfec_hdr)));
    CK(hipMalloc(&d_st, N * sizeof(rfec_seg_stamp)));
    CK(hipMalloc(&d_len, N * 2));
    CK(hipMalloc(&d_rec, N * sizeof(rfec_wire_rec)));
    CK(hipMemcpy(d_sh, sh.data(), sh.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_hdr, hdr.data(), N * sizeof(rfec_hdr), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_st, st.data(), N * sizeof(rfec_seg_stamp), hipMemcpyHostToDevice));
    hipStream_t sm;
    CK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto fn) {
        std::vector<float> t;
        for (int r = 0; r < reps + 3; ++r) {
            CK(hipEventRecord(a, sm));
            fn();
            CK(hipEventRecord(b, sm));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 3)
                t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    // the frame kernel first in any case: the parse reads its datagrams
    const float tf = time([&] {
        CK((hipError_t)rfec_launch_wire_frame_seg(N, S, S, d_sh, d_hdr, d_st, nullptr, DS, d_dg, d_len, sm));
    });
    const float tp = time([&] {
        CK((hipError_t)rfec_launch_wire_parse(N, DS, d_dg, d_len, PS, S, d_rec, d_pay, 0, sm));
    });
    const double bf = (double)N * ((S + 32) + (S + 36 + 2)), bp = (double)N * ((S + 36 + 2) + (64 + S));
    printf("frame_seg %8.1f us %6.4f   parse_seg %8.1f us %6.4f\n", tf, bf / tf / 1e3 / 8000, tp,
           bp / tp / 1e3 / 8000);
    return 0;
}
