// Probe: fixed cost of a launch geometry on gfx950 (no memory traffic but the output):
// 256 x 1024-thread workgroups with 138 KB of dynamic LDS (k_mfma_rows' shape) vs smaller
// workgroups, with 0 or 10 workgroup barriers.  Back-to-back launches timed with events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_empty(uint32_t nbar, uint32_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    lds[threadIdx.x] = threadIdx.x;
    for (uint32_t i = 0; i < nbar; i++) {
        __syncthreads();
        lds[threadIdx.x] += lds[(threadIdx.x + 1) % blockDim.x];
    }
    if (threadIdx.x == 0) out[blockIdx.x] = lds[0];
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipFuncSetAttribute((const void *)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    struct { int wgs, threads; size_t lds; } shapes[] = {
        {256, 1024, 138 * 1024}, {256, 1024, 16 * 1024}, {256, 512, 138 * 1024}, {256, 256, 16 * 1024},
        {1024, 256, 32 * 1024}, {512, 512, 64 * 1024}};
    for (auto s : shapes) {
        for (uint32_t nbar : {0u, 10u, 40u}) {
            for (int r = 0; r < 50; r++) k_empty<<<s.wgs, s.threads, s.lds>>>(nbar, out);
            hipEventRecord(e0);
            const int R = 500;
            for (int r = 0; r < R; r++) k_empty<<<s.wgs, s.threads, s.lds>>>(nbar, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%5d WGs x %4d threads, %3zu KB LDS, %2u barriers: %6.2f us per launch\n", s.wgs, s.threads,
                   s.lds / 1024, nbar, ms * 1000.0 / R);
        }
    }
    return 0;
}
