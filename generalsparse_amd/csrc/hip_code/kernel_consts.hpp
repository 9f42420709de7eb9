// hip_code/kernel_consts.hpp -- compile-time shapes of the gfx950 kernels in
// kernel_lib.hpp that the host-side layout builders (host/device_layout.cc) size
// their tiles by.  Plain C++ (no device code): included by both sides.
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifndef __HIPCC__
#define GSK_HD
#else
#define GSK_HD __host__ __device__
#endif

namespace gsk {

// k_mfma_rows: waves per role: compute 0..5, B loaders 6..9, entry loaders 10..15
constexpr int kMfmaWaves = 16, kMfmaCompute = 6, kMfmaBWaves = 4, kMfmaAWaves = 6;
// GLDS = g > 0: g waves issue the B rows (LDS-DMA), the other 10 - g load and scatter entries
constexpr int kMfmaBWavesG = 2, kMfmaAWavesG = 8;

// k_mfma_ks_group: entries of one grouped launch (kernel arguments, ~3.2 KB of the 4 KB)
constexpr int kKsGroupMax = 32;

// k_mfma_ks: wave image row stride (conflict-free ds_read_b128 fragment reads)
constexpr uint32_t kKsStride = 96;

template <int RT>
GSK_HD constexpr uint32_t ks_image_bytes() {
    return (16u * RT + 1u) * kKsStride;
}

// dynamic LDS of k_mfma_ks: W x (wave image + one k-step of B rows), or the W partial
// tiles of the final reduction (+ the arrival flag), whichever is larger
// (the reduction runs in two halves of W/2 waves when W tiles would exceed the 160 KB)
GSK_HD constexpr bool ks_red_halves(uint32_t CT, uint32_t RT, uint32_t W) {
    return (size_t)W * RT * CT * 1024u + 16u > 160u * 1024u;
}
GSK_HD constexpr size_t ks_stage_bytes(uint32_t CT, uint32_t RT, uint32_t W) {
    return (size_t)W * ((16u * RT + 1u) * kKsStride + 32u * 32u * CT);
}
// the W partial tiles (+ the ticket word) fit beside the wave images: each wave stores its
// tile when its own loop ends, with no barrier before
// (ap = false: never apart -- the partial tiles reuse the stage LDS after a barrier, so more
// workgroups fit a CU: KS_APART)
GSK_HD constexpr bool ks_red_apart(uint32_t CT, uint32_t RT, uint32_t W, bool ap = true) {
    return ap && ks_stage_bytes(CT, RT, W) + (size_t)W * RT * CT * 1024u + 16u <= 160u * 1024u;
}
GSK_HD constexpr size_t ks_lds_bytes(uint32_t CT, uint32_t RT, uint32_t W, bool ap = true) {
    const size_t stage = ks_stage_bytes(CT, RT, W);
    if (ks_red_apart(CT, RT, W, ap)) return stage + (size_t)W * RT * CT * 1024u + 16u;
    const size_t red = (size_t)(ks_red_halves(CT, RT, W) ? W / 2 : W) * RT * CT * 1024u + 16u;
    return stage > red ? stage : red;
}

// k_mfma_kb: the selector table (128 B) + W wave slots (one k-step of B rows + NVB KB of
// values), then the W partial tiles (+ the ticket word) when they fit beside them
GSK_HD constexpr size_t kb_stage_bytes(uint32_t CT, uint32_t W, uint32_t NVB) {
    return 128u + (size_t)W * (32u * 32u * CT + 1024u * NVB);
}
GSK_HD constexpr bool kb_red_apart(uint32_t CT, uint32_t RT, uint32_t W, uint32_t NVB) {
    return kb_stage_bytes(CT, W, NVB) + (size_t)W * RT * CT * 1024u + 16u <= 160u * 1024u;
}
GSK_HD constexpr size_t kb_lds_bytes(uint32_t CT, uint32_t RT, uint32_t W, uint32_t NVB) {
    const size_t st = kb_stage_bytes(CT, W, NVB);
    if (kb_red_apart(CT, RT, W, NVB)) return st + (size_t)W * RT * CT * 1024u + 16u;
    const size_t red = (size_t)(ks_red_halves(CT, RT, W) ? W / 2 : W) * RT * CT * 1024u + 16u;
    return st > red ? st : red;
}

// k_mfma_bm: per (row block, K range, 32-column k-step) one 8-byte record per lane (RT <= 6
// mask bytes, u16 value offset in bytes 6..7); B by LDS-DMA into NBT k-step slots per wave.
// NBT (k-steps a wave keeps in flight): the value windows take 4 VGPRs per tile per step
// (<= ~100 VGPRs), the slots W * NBT * 1 KB * CT of LDS.  bm_sel: the v_perm_b32 selector
// that expands the packed halves of mask nibble n into output halves 2w, 2w+1 (0x0c: zero)
GSK_HD constexpr uint32_t bm_nbt(uint32_t CT, uint32_t RT) {
    const uint32_t by_vgpr = 25u / RT < 12u ? 25u / RT : 12u;
    const uint32_t by_lds = 18u / CT;
    return by_vgpr < by_lds ? by_vgpr : by_lds;
}
GSK_HD constexpr uint32_t bm_sel(uint32_t n, uint32_t w) {
    uint32_t sel = 0;
    for (uint32_t j = 0; j < 2; j++) {
        const uint32_t h = 2 * w + j;
        uint32_t b0 = 0x0c, b1 = 0x0c;
        if ((n >> h) & 1u) {
            uint32_t src = 0;
            for (uint32_t b = 0; b < h; b++) src += (n >> b) & 1u;
            b0 = 2 * src;
            b1 = 2 * src + 1;
        }
        sel |= (b0 | (b1 << 8)) << (16 * j);
    }
    return sel;
}
GSK_HD constexpr bool bm_red_halves(uint32_t CT, uint32_t RT, uint32_t W) {
    return (size_t)W * RT * CT * 1024u + 16u > 64u * 1024u;
}
// dynamic LDS of k_mfma_bm: selector table + W x NBT k-step slots, or the partial tiles of
// the final reduction (+ the arrival flag)
GSK_HD constexpr size_t bm_lds_bytes(uint32_t CT, uint32_t RT, uint32_t W) {
    const size_t ring = 128u + (size_t)W * bm_nbt(CT, RT) * 32u * 32u * CT;
    const size_t red = (size_t)(bm_red_halves(CT, RT, W) ? W / 2 : W) * RT * CT * 1024u + 16u;
    return ring > red ? ring : red;
}

// k_nm_mfma: 8 waves, 4,608-B blocks per (64 rows, 64-column k-step), B chunks of 256 rows
constexpr int kNmWaves = 8;
constexpr uint32_t kNmBlockBytes = 4608, kNmKC = 256;
// bytes per (workgroup of T 16-row tiles, 64-column k-step): two wave sets of ceil(T/2) and T/2
// tiles, each 512 B of positions + 1 KB of values per tile (T = 8: two 4,608-B blocks).  Set rh's
// blocks of all k-steps are contiguous: set 0 at w * S * this, set 1 after set 0's S blocks.
GSK_HD constexpr uint32_t nm_wg_block_bytes(uint32_t T) { return 1024u + 1024u * T; }
// k_nm_mfma4: two B chunk buffers, or the four q = 1 wave tiles of the k-phase sum (+ ticket)
GSK_HD constexpr size_t nm4_lds_bytes(uint32_t CT) {
    const size_t bufs = (size_t)2 * kNmKC * 32u * CT, red = (size_t)4 * 4 * CT * 64 * 16 + 16;
    return bufs > red ? bufs : red;
}

}  // namespace gsk
