// Probe: LDS read THROUGHPUT by alignment on gfx950 (16 waves per CU, 256 workgroups),
// each lane reading at its own pseudo-random address (the value windows of the bitmap
// expansion): ds_read_b64 8-B aligned / 4-B aligned / 2-B aligned, ds_read_b96 4-B
// aligned, ds_read_b32 2-B aligned, ds_read2_b32.  Reads only (plus the sink store).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(1024) void k_lds(uint32_t iters, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[16384];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 16384; i += 1024) lds[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0, h = tid * 2654435761u + 12345u;
    for (uint32_t it = 0; it < iters; it++) {
        h = h * 1664525u + 1013904223u;
        const uint32_t halves = (h >> 8) & 8191u;  // half index in the first 16 KB
        uint32_t a;
        if constexpr (MODE == 0) a = (halves & ~3u) * 2u;      // 8-B aligned
        else if constexpr (MODE == 1 || MODE == 4 || MODE == 5) a = (halves & ~1u) * 2u;  // 4-B aligned
        else a = halves * 2u;                                   // 2-B aligned
        const unsigned char *p = reinterpret_cast<const unsigned char *>(lds) + a;
        if constexpr (MODE <= 2) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p);
            acc += v.x ^ v.y;
        } else if constexpr (MODE == 3) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(p);
            acc += v;
        } else if constexpr (MODE == 4) {
            typedef uint32_t u3v __attribute__((ext_vector_type(3)));
            u3v x;
            asm volatile("ds_read_b96 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(x) : "v"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const unsigned char *)p) : "memory");
            acc += x.x ^ x.y ^ x.z;
        } else {
            const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
            acc += q[0] ^ q[1] ^ q[2];
        }
    }
    if (acc == 0x9e3779b9u) sink[tid] = acc;
}

int main() {
    uint32_t *sink;
    hipMalloc(&sink, 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"ds_read_b64 8B-aligned", "ds_read_b64 4B-aligned", "ds_read_b64 2B-aligned",
                           "ds_read_b32 2B-aligned", "ds_read_b96 4B-aligned", "3x b32 4B-aligned"};
    void (*ks[])(uint32_t, uint32_t *) = {k_lds<0>, k_lds<1>, k_lds<2>, k_lds<3>, k_lds<4>, k_lds<5>};
    const uint32_t iters = 4096;
    for (int m = 0; m < 6; m++) {
        ks[m]<<<256, 1024>>>(iters, sink);
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++) ks[m]<<<256, 1024>>>(iters, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1000.0 / 5;
        // wave-instructions per CU = 16 waves * iters
        printf("%-24s %8.1f us   %6.2f ns per wave-instruction per CU\n", names[m], us, us * 1000.0 / (16.0 * iters));
    }
    return 0;
}
