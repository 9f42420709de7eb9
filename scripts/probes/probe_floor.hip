// Probe: memory floor of a C2-shaped row-block SpMM on gfx950 (diagnostic, not product).
// 256 workgroups; workgroup b streams its private slice of an "A" buffer (HBM, rotated over
// copies so it never sits in the Infinity Cache) and a "B" slice of Bsz/S bytes that S-groups
// of workgroups share (L2-resident), both by global_load_dwordx4 into VGPRs, DEPTH loads in
// flight per lane.  Prints us per launch (events over back-to-back launches) for:
//   A bytes in {31.5 MB (u16 CSR), 19.0 MB (bitmap)}, S in {1,2,4,8}, W in {8,16}.
// Also the empty-launch floor of the same grid.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

template <int DEPTH>
__global__ void k_floor(const uint4 *A, const uint4 *B, uint32_t a_units, uint32_t b_units, uint32_t S,
                        uint32_t *sink) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint4 *a = A + (size_t)blockIdx.x * a_units;
    const uint4 *b = B + (size_t)((blockIdx.x / 8) % S) * b_units;  // S slices of B
    uint4 acc = make_uint4(0, 0, 0, 0);
    const uint32_t total = a_units + b_units;
    for (uint32_t base = 0; base < total; base += nt * DEPTH) {
        uint4 x[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            const uint32_t u = base + d * nt + tid;
            // B interleaved with the first A units (both streams in flight together), then the rest of A
            if (u < 2 * b_units) x[d] = (u & 1) ? b[u >> 1] : a[u >> 1];
            else if (u < total) x[d] = a[u - b_units];
            else x[d] = make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int d = 0; d < DEPTH; d++) { acc.x ^= x[d].x; acc.y ^= x[d].y; acc.z ^= x[d].z; acc.w ^= x[d].w; }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[tid] = 1;
}

__global__ void k_empty(uint32_t *sink) {
    if (threadIdx.x == 1023u && blockIdx.x == 100000u) sink[0] = 1;
}

int main() {
    const size_t copies = 16;
    const size_t a_max = 31457280;  // 31.5 MB
    uint4 *A, *B;
    uint32_t *sink;
    hipMalloc(&A, a_max * copies + (1 << 20));
    hipMalloc(&B, 327680 + (1 << 16));
    hipMalloc(&sink, 8192);
    hipMemset(A, 1, a_max * copies);
    hipMemset(B, 2, 327680);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](auto launch) {
        for (int r = 0; r < 10; r++) launch(r);
        hipDeviceSynchronize();
        const int R = 64;
        hipEventRecord(e0);
        for (int r = 0; r < R; r++) launch(r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return ms * 1000.0 / R;
    };
    for (int W : {8, 16}) {
        const double us = timeit([&](int) { k_empty<<<256, 64 * W>>>(sink); });
        printf("empty 256 x %4d: %6.2f us\n", 64 * W, us);
    }
    for (size_t abytes : {a_max, (size_t)19005440}) {
        for (uint32_t S : {1u, 2u, 4u, 8u}) {
            for (int W : {8, 16}) {
                for (int depth : {4, 8}) {
                    const uint32_t a_units = (uint32_t)(abytes / 256 / 16);
                    const uint32_t b_units = 327680 / S / 16;
                    auto kern = depth == 4 ? k_floor<4> : k_floor<8>;
                    const double us = timeit([&](int r) {
                        kern<<<256, 64 * W>>>((const uint4 *)((char *)A + (size_t)(r % copies) * a_max), B, a_units,
                                              b_units, S, sink);
                    });
                    const double bytes = (double)abytes + 327680.0;
                    printf("A %5.1f MB  S=%u (B %3u KB/WG)  W=%2d depth=%d: %6.2f us  %5.2f TB/s (A+B once)\n",
                           abytes / 1e6, S, 327680 / S / 1024, W, depth, us, bytes / (us * 1e-6) / 1e12);
                }
            }
        }
    }
    return 0;
}
