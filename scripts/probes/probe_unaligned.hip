// Probe: do LDS and global vector loads at 2-byte-aligned addresses return the
// right bytes on gfx950 (and at what cost)?  Decides the value-window reads of
// the bitmap-panel MFMA kernel.  Vector loads only; stores are ordinary.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_probe(const uint16_t *g, uint32_t *out, int mode, int reps, uint64_t *cyc) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = g[i];
    __syncthreads();
    const uint32_t off = (uint32_t)(lane * 7 + 1);  // halves: odd and even, crossing 4/8/16-B lines
    const uint32_t addr = (uint32_t)(uintptr_t)(lds) + off * 2u;
    uint32_t a = 0, b = 0, c = 0, d = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        const uint32_t ad = addr + (uint32_t)(r & 1) * 0u;
        if (mode == 0) {
            uint32_t x;
            asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(ad) : "memory");
            a ^= x;
        } else if (mode == 1) {
            uint2 x;
            asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(ad) : "memory");
            a ^= x.x; b ^= x.y;
        } else if (mode == 2) {
            uint4 x;
            asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(ad) : "memory");
            a ^= x.x; b ^= x.y; c ^= x.z; d ^= x.w;
        } else if (mode == 3) {
            uint2 x;
            const uint16_t *p = g + off;
            asm volatile("global_load_dwordx2 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
            a ^= x.x; b ^= x.y;
        } else if (mode == 4) {
            uint4 x;
            const uint16_t *p = g + off;
            asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
            a ^= x.x; b ^= x.y; c ^= x.z; d ^= x.w;
        } else {  // aligned reference: ds_read_b64 at 8-B aligned
            uint2 x;
            const uint32_t al = (uint32_t)(uintptr_t)(lds) + (uint32_t)lane * 8u;
            asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(al) : "memory");
            a ^= x.x; b ^= x.y;
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[lane * 4 + 0] = a; out[lane * 4 + 1] = b; out[lane * 4 + 2] = c; out[lane * 4 + 3] = d;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    std::vector<uint16_t> h(4096);
    for (int i = 0; i < 4096; i++) h[i] = (uint16_t)(i * 2654435761u >> 7);
    uint16_t *dg; uint32_t *dout; uint64_t *dc;
    hipMalloc(&dg, 8192 + 64); hipMalloc(&dout, 64 * 16); hipMalloc(&dc, 8);
    hipMemcpy(dg, h.data(), 8192, hipMemcpyHostToDevice);
    const char *names[] = {"ds_read_b32 @2B", "ds_read_b64 @2B", "ds_read_b128 @2B", "global_load_dwordx2 @2B",
                           "global_load_dwordx4 @2B", "ds_read_b64 aligned"};
    const int words[] = {1, 2, 4, 2, 4, 2};
    for (int mode = 0; mode < 6; mode++) {
        k_probe<<<1, 64>>>(dg, dout, mode, 1, dc);
        std::vector<uint32_t> o(256);
        hipMemcpy(o.data(), dout, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; l++) {
            const uint32_t off = mode == 5 ? (uint32_t)l * 4u : (uint32_t)(l * 7 + 1);
            for (int w = 0; w < words[mode]; w++) {
                const uint32_t want = (uint32_t)h[off + 2 * w] | ((uint32_t)h[off + 2 * w + 1] << 16);
                if (o[l * 4 + w] != want) bad++;
            }
        }
        k_probe<<<1, 64>>>(dg, dout, mode, 1000, dc);
        uint64_t c = 0;
        hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        printf("%-26s wrong words %4d / %4d   %.1f cycles per dependent load\n", names[mode], bad, 64 * words[mode],
               c / 1000.0);
    }
    return 0;
}
