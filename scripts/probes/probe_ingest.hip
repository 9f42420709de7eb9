// Probe: per-CU ingest rate of the load paths a row-block SpMM kernel can use on
// gfx950, one workgroup per CU (256 workgroups), W waves each:
//   mode 0  LDS-DMA (global_load_lds_dwordx4) of a buffer every workgroup shares (L2-resident, like B)
//   mode 1  global_load_dwordx4 to VGPRs of the shared buffer
//   mode 2  LDS-DMA of a private per-workgroup region (HBM stream, like A)
//   mode 3  global_load_dwordx4 of the private region
//   mode 4  LDS-DMA, shared buffer, only 16 lanes active per instruction (256 B)
// Each wave keeps DEPTH wave-instructions in flight (counted vmcnt).  Vector loads only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ void dma16(const void *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <int DEPTH>
__global__ void k_ingest(const uint4 *shared_buf, const uint4 *priv, uint32_t shared_units, uint32_t priv_units,
                         int mode, uint32_t iters, uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t W = blockDim.x >> 6;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)lds;
    const uint32_t slot = __builtin_amdgcn_readfirstlane(lds0 + wv * 8u * 1024u);
    uint4 acc = make_uint4(0, 0, 0, 0);
    const uint4 *src = (mode == 2 || mode == 3 || mode == 6) ? priv + (size_t)blockIdx.x * priv_units : shared_buf;
    uint32_t units = (mode == 2 || mode == 3) ? priv_units : shared_units;
    if (mode == 6) units = 64 * 1024 / 16;  // 64 KB private region re-read: L2-resident, unshared
    const uint32_t rot = (blockIdx.x >> 3) * 64u * 13u;
    for (uint32_t i = 0; i < iters; i++) {
        const uint32_t piece = (wv + i * W) * 64u + rot;  // 1 KB pieces, interleaved over the waves
        const uint32_t u = (piece + lane) % units;
        if (mode == 0 || mode == 2 || mode == 6) {
            dma16(src + u, slot + (i % 8u) * 1024u);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
        } else if (mode == 5) {
            if ((i & 3u) == 0) {  // four 1-KB pieces per M0 write: instruction offsets 0/1/2/3 KB
                uint32_t keep;
                const uint4 *g4 = src + ((wv * 64u + i * W * 64u + rot) % (units - 256u)) + lane;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                    "global_load_lds_dwordx4 %1, off\n\t"
                    "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                    "global_load_lds_dwordx4 %1, off offset:2048\n\t"
                    "global_load_lds_dwordx4 %1, off offset:3072\n\t"
                    "s_mov_b32 m0, %0"
                    : "=&s"(keep) : "v"(g4), "s"(slot + ((i >> 2) % (DEPTH / 4 > 0 ? DEPTH / 4 : 1)) * 4096u) : "memory");
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
            }
        } else if (mode == 4) {
            if (lane < 16) dma16(src + u, slot + (i % 8u) * 1024u);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
        } else if ((i % DEPTH) == 0) {
            // compiler-visible loads (no inline asm with a VGPR destination): DEPTH
            // wave-instructions issued together, then consumed
            uint4 x[DEPTH];
#pragma unroll
            for (int d = 0; d < DEPTH; d++) {
                const uint32_t pd = (wv + (i + d) * W) * 64u + rot;
                x[d] = src[(pd + lane) % units];
            }
#pragma unroll
            for (int d = 0; d < DEPTH; d++) { acc.x ^= x[d].x; acc.y ^= x[d].y; acc.z ^= x[d].z; acc.w ^= x[d].w; }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

// does the instruction offset move the LDS destination with the global address?
__global__ void k_offset_check(const uint4 *src, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint4 lds[64 * 4];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 256; i += 64) lds[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4 *)lds);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\t"
                 "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                 "global_load_lds_dwordx4 %1, off offset:2048\n\t"
                 "global_load_lds_dwordx4 %1, off offset:3072\n\t"
                 "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
                 : "=&s"(keep) : "v"(src + lane), "s"(lds0) : "memory");
    __syncthreads();
    for (uint32_t i = lane; i < 256; i += 64) out[i] = lds[i].x;
}

int main() {
    const uint32_t shared_units = 512 * 1024 / 16, priv_units = 128 * 1024 / 16;
    uint4 *sb, *pv;
    uint32_t *sink;
    hipMalloc(&sb, (size_t)shared_units * 16);
    hipMalloc(&pv, (size_t)priv_units * 16 * 256 * 8);  // 8 rotating copies of the private regions
    hipMalloc(&sink, 4096);
    hipMemset(sb, 1, (size_t)shared_units * 16);
    hipMemset(pv, 2, (size_t)priv_units * 16 * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"lds-dma shared(L2)", "vgpr   shared(L2)", "lds-dma private(HBM)", "vgpr   private(HBM)",
                           "lds-dma shared 256B", "lds-dma x4 per M0"};
    {
        std::vector<uint4> h(256);
        for (uint32_t i = 0; i < 256; i++) h[i] = make_uint4(i * 7 + 1, 0, 0, 0);
        hipMemcpy(sb, h.data(), 4096, hipMemcpyHostToDevice);
        k_offset_check<<<1, 64>>>(sb, sink);
        std::vector<uint32_t> o(256);
        hipMemcpy(o.data(), sink, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (uint32_t i = 0; i < 256; i++) bad += o[i] != i * 7 + 1;
        printf("offset DMA: %d of 256 LDS units wrong (0: inst offset moves LDS dest too)\n", bad);
        hipMemset(sb, 1, (size_t)shared_units * 16);
    }
    names[5] = "lds-dma private 64K(L2)";
    for (int mode : {0, 6}) {
        for (int W : {8, 16}) {
            for (int depth : {4, 16, 32}) {
                // bytes per workgroup per launch: 512 KB (shared) or 128 KB (private)
                const uint32_t per_wg = (mode == 2 || mode == 3) ? 128 * 1024 : 512 * 1024;
                const uint32_t iters = per_wg / 1024 / W;
                auto kern = depth == 4 ? k_ingest<4> : (depth == 16 ? k_ingest<16> : k_ingest<32>);
                
                const size_t lds = (size_t)W * 8 * 1024;
                hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                for (int rep = 0; rep < 3; rep++)
                    kern<<<256, 64 * W, lds>>>(sb, pv, shared_units, priv_units, mode, iters, sink);
                const int R = 20;
                hipEventRecord(e0);
                for (int rep = 0; rep < R; rep++)
                    kern<<<256, 64 * W, lds>>>(sb, pv + (size_t)(rep % 8) * priv_units * 256, shared_units, priv_units,
                                               mode, iters, sink);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                const double us = ms * 1000.0 / R;
                const double bytes = (mode == 4 ? 256.0 : 1024.0) * iters * W;
                printf("%-24s W=%2d depth=%d  %7.2f us  %6.1f GB/s per CU  (%.2f TB/s chip)\n", (mode == 6 ? names[5] : names[mode]), W, depth, us,
                       bytes / (us * 1e-6) / 1e9, bytes * 256 / (us * 1e-6) / 1e12);
            }
        }
    }
    return 0;
}
