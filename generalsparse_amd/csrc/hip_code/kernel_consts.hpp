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
GSK_HD constexpr size_t ks_lds_bytes(uint32_t CT, uint32_t RT, uint32_t W) {
    const size_t stage = (size_t)W * ((16u * RT + 1u) * kKsStride + 32u * 32u * CT);
    const size_t red = (size_t)(ks_red_halves(CT, RT, W) ? W / 2 : W) * RT * CT * 1024u + 16u;
    return stage > red ? stage : red;
}

// k_nm_mfma: 8 waves, 4,608-B blocks per (64 rows, 64-column k-step), B chunks of 256 rows
constexpr int kNmWaves = 8;
constexpr uint32_t kNmBlockBytes = 4608, kNmKC = 256;

}  // namespace gsk
