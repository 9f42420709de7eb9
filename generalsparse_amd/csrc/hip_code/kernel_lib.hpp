// hip_code/kernel_lib.hpp -- hand-written gfx950 (MI355X, CDNA4) SpMM kernel families.
//
// Replaces cuda_code/kernel_lib.hpp of the reference (Load()/__ldg helpers,
// kernel_lib.hpp:1006-1148) and the kernels its reduction tokens print
// (SURVEY.md §2.2 K1-K7).  C = A * B, B row-major K x N, C row-major M x N.
// Written for 64-lane waves: a wave is split into S = 64/X "slots" of X column
// lanes; every lane owns CF consecutive dense columns (one 16-byte load of a B
// row segment when CF*sizeof(VT) == 16).  A (cols/vals) is streamed once,
// vector-loaded; B rows are gathered through L1/L2 (B is small and shared).
// Accumulation is always fp32 (the reference accumulates fp16 in half).
//
// Families (selected by code_generator::compile from the reduction tokens):
//   k_thread_total   K1: X lanes per BMT row, rows sorted + col-padded (SCF-aligned)
//   k_warp_rows      K4: one wave per BMW, nnz split over S slots, xor-shuffle reduce
//                       (+ optional BMTB grouping = one workgroup per BMTB)
//   k_block_rows     K6: one 256-thread workgroup per BMTB, wave reduce + LDS reduce
//   k_bitmap_segment K2+K3: fixed 32-nnz BMTs, row segments from bitmaps, open
//                       head/tail partials combined per wave, then atomics
//   k_row_chunks     K5/K7: col-direction BMTs (chunks of one row), segmented
//                       slot tree + a row carry per wave
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "idx_formula.hpp"
#include "kernel_consts.hpp"

namespace gsk {

typedef _Float16 f16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int BYTES> struct raw_vec;
template <> struct raw_vec<2> { typedef uint16_t t; };
template <> struct raw_vec<4> { typedef uint32_t t; };
template <> struct raw_vec<8> { typedef uint2 t; };
template <> struct raw_vec<16> { typedef uint4 t; };
struct alignas(16) u32x8 { uint4 lo, hi; };
template <> struct raw_vec<32> { typedef u32x8 t; };

// CF contiguous values -> fp32 (one vector load)
template <class VT, int CF>
__device__ __forceinline__ void load_f32(const VT *__restrict__ p, float (&out)[CF]) {
    typedef typename raw_vec<CF * sizeof(VT)>::t R;
    R r = *reinterpret_cast<const R *>(p);
    VT tmp[CF];
    __builtin_memcpy(tmp, &r, sizeof(R));
#pragma unroll
    for (int k = 0; k < CF; k++) out[k] = (float)tmp[k];
}

template <class VT, int CF>
__device__ __forceinline__ void store_f32(VT *__restrict__ p, const float (&in)[CF]) {
    typedef typename raw_vec<CF * sizeof(VT)>::t R;
    VT tmp[CF];
#pragma unroll
    for (int k = 0; k < CF; k++) tmp[k] = (VT)in[k];
    R r;
    __builtin_memcpy(&r, tmp, sizeof(R));
    *reinterpret_cast<R *>(p) = r;
}

// Loads of the operand a launch reads exactly once (A's entries, groups, panels).  GS_A_NT=1
// (make A_NT=1): the non-temporal form (global_load ... nt), which the XCD's L2 holds at low
// retention, so the stream does not push out the rows of B that other workgroups re-read.
template <class T>
__device__ __forceinline__ T ld_once(const T *p) {
#if defined(GS_A_NT) && GS_A_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
// the same, chosen per instantiation (k_mfma_ks KS_NT, k_nm_mfma NM_NT): NT loads bypass the CU's
// L1 and stream through L2 (MI355X_MICROARCH.md: nt loads are L2-served)
template <bool NT, class T>
__device__ __forceinline__ T ld_once_if(const T *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return ld_once(p);
}
template <int BYTES> struct raw_ext;
template <> struct raw_ext<1> { typedef uint8_t t; };
template <> struct raw_ext<2> { typedef uint16_t t; };
template <> struct raw_ext<4> { typedef uint32_t t; };
template <> struct raw_ext<8> { typedef u32x2 t; };
template <> struct raw_ext<16> { typedef u32x4 t; };

// SCF contiguous sparse entries (cols or vals) in one load (read once: ld_once)
template <class T, int SCF>
__device__ __forceinline__ void load_raw(const T *__restrict__ p, T (&out)[SCF]) {
    if constexpr (SCF * sizeof(T) <= 16) {
        typedef typename raw_ext<SCF * sizeof(T)>::t R;
        R r = ld_once(reinterpret_cast<const R *>(p));
        __builtin_memcpy(out, &r, sizeof(R));
    } else {
        static_assert(SCF * sizeof(T) == 32, "8 to 32 bytes");
        u32x4 r[2] = {ld_once(reinterpret_cast<const u32x4 *>(p)), ld_once(reinterpret_cast<const u32x4 *>(p) + 1)};
        __builtin_memcpy(out, r, 32);
    }
}

template <int CF>
__device__ __forceinline__ void wave_reduce_slots(float (&acc)[CF], int X) {
    for (int off = X; off < 64; off <<= 1) {
#pragma unroll
        for (int k = 0; k < CF; k++) acc[k] += __shfl_xor(acc[k], off, 64);
    }
}

template <class VT, int CF>
__device__ __forceinline__ void atomic_add_vals(VT *p, const float (&v)[CF]);

template <>
__device__ __forceinline__ void atomic_add_vals<float, 1>(float *p, const float (&v)[1]) {
    unsafeAtomicAdd(p, v[0]);
}
template <>
__device__ __forceinline__ void atomic_add_vals<float, 4>(float *p, const float (&v)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) unsafeAtomicAdd(p + k, v[k]);
}
template <>
__device__ __forceinline__ void atomic_add_vals<float, 8>(float *p, const float (&v)[8]) {
#pragma unroll
    for (int k = 0; k < 8; k++) unsafeAtomicAdd(p + k, v[k]);
}
template <>
__device__ __forceinline__ void atomic_add_vals<f16, 8>(f16 *p, const float (&v)[8]) {
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        __half2 h = __floats2half2_rn(v[k], v[k + 1]);
        unsafeAtomicAdd(reinterpret_cast<__half2 *>(p + k), h);
    }
}
template <>
__device__ __forceinline__ void atomic_add_vals<f16, 1>(f16 *p, const float (&v)[1]) {
    unsafeAtomicAdd(reinterpret_cast<__half *>(p), __float2half(v[0]));
}

// XCD-aware block numbering (cdna_hip_programming.md §5.5 T1): blocks b and b + 8 are
// observed to share an XCD (round-robin dispatch, MI355X_MICROARCH.md §Workgroup dispatch),
// so consecutive blockIdx read the neighbouring cache lines of A's streams from eight
// different L2s.  The bijective renumbering gives each XCD one contiguous range of
// logical block ids instead; a speed choice only, any placement stays correct.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
#ifdef GS_NO_XCD_SWIZZLE  // A/B diagnostic builds only
    return b;
#endif
    const uint32_t q = n >> 3, r = n & 7u, x = b & 7u;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + (b >> 3);
}

// one sparse entry times a CF-wide B segment
template <class VT, int CF>
__device__ __forceinline__ void fma_row(float (&acc)[CF], float v, const VT *__restrict__ brow) {
    float b[CF];
    load_f32<VT, CF>(brow, b);
#pragma unroll
    for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(v, b[k], acc[k]);
}

// ---------------------------------------------------------------------------
// K1 thread_total: the row-sorted, col-padded plan (sort_operator +
// fixed_interval_row_direction_thread_blocking_operator(1,...,scf) +
// thread_total_reduce_operator).  BMT b covers sorted row b; X lanes own its
// dense columns; the row's nnz are walked SCF at a time with one vector load
// of cols and one of vals (the reference's Load() of col4/val4,
// total_BMT_result_reduce_to_one_register_token.cc:807-898).  Sorted rows
// b >= n_bmt are the trailing empty rows: their C rows are zero-filled here
// instead of relying on a memset.
// ---------------------------------------------------------------------------
template <class VT, class CT, int CF, int SCF, bool FX>
__device__ __forceinline__ void thread_total_body(const uint32_t *__restrict__ first_nz,  // n_bmt+1
                                                      const idx_formula f_nz,
                                                      const uint32_t *__restrict__ order,     // n_rows: sorted->orig
                                                      const idx_formula f_order,
                                                      const CT *__restrict__ col, const VT *__restrict__ val,
                                                      const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmt,
                                                      uint32_t n_rows, uint32_t N, uint32_t X, uint32_t row_base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t xl = lane & (X - 1u);
    const uint32_t groups_per_block = blockDim.x / X;
    // plain block order: the rows are sorted by length, so XCD-contiguous ranges would
    // give one XCD all the longest rows (measured slower on C1)
    const uint32_t g = blockIdx.x * groups_per_block + threadIdx.x / X;
    const uint32_t stride = gridDim.x * groups_per_block;
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t rr = g; rr < n_rows; rr += stride) {
            float acc[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) acc[k] = 0.f;
            if (rr < n_bmt) {
                uint32_t b, e;
                idx_range<FX>(first_nz, f_nz, rr, b, e);
                typedef typename raw_vec<CF * sizeof(VT)>::t RB;
                for (uint32_t p = b; p < e; p += SCF) {
                    CT cc[SCF];
                    VT vv[SCF];
                    load_raw<CT, SCF>(col + p, cc);
                    load_raw<VT, SCF>(val + p, vv);
                    RB braw[SCF];
#pragma unroll
                    for (int j = 0; j < SCF; j++) braw[j] = *reinterpret_cast<const RB *>(B + (size_t)cc[j] * N + c0);
#pragma unroll
                    for (int j = 0; j < SCF; j++) {
                        VT bt[CF];
                        __builtin_memcpy(bt, &braw[j], sizeof(RB));
                        const float v = (float)vv[j];
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(v, (float)bt[k], acc[k]);
                    }
                }
            }
            if (cok) store_f32<VT, CF>(C + (size_t)(idx_at<FX>(order, f_order, rr) + row_base) * N + c0, acc);
        }
    }
}

template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) void k_thread_total(const uint32_t *__restrict__ first_nz, const idx_formula f_nz,
                                                      const uint32_t *__restrict__ order, const idx_formula f_order,
                                                      const CT *__restrict__ col, const VT *__restrict__ val,
                                                      const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmt,
                                                      uint32_t n_rows, uint32_t N, uint32_t X, uint32_t row_base) {
    if (f_nz.kind == IDX_ARRAY && f_order.kind == IDX_ARRAY)
        thread_total_body<VT, CT, CF, SCF, false>(first_nz, f_nz, order, f_order, col, val, B, C, n_bmt, n_rows, N, X, row_base);
    else
        thread_total_body<VT, CT, CF, SCF, true>(first_nz, f_nz, order, f_order, col, val, B, C, n_bmt, n_rows, N, X, row_base);
}

// ---------------------------------------------------------------------------
// K4 warp_total over BMWs (fixed_interval_row_direction_warp_blocking_operator
// or balanced_interval_row_direction_warp_blocking_operator, optionally inside
// BMTBs) + warp_total_reduce_operator.  One wave per BMW; the BMW's rows are
// processed in order; each row's nnz are split over the S = 64/X slots in
// SCF-aligned chunks (row_ptr is padded so the aligned over-read stays in
// bounds and is masked), then reduced with xor shuffles.  With a BMTB level,
// workgroup g owns BMWs [bmw_of_bmtb[g], bmw_of_bmtb[g+1]) and its waves stride
// over them (keeps a BMTB's rows on one CU / XCD).
// ---------------------------------------------------------------------------
template <class VT, class CT, int CF, int SCF>
__device__ __forceinline__ void wave_row(const uint32_t b, const uint32_t e, const CT *__restrict__ col,
                                         const VT *__restrict__ val, const VT *__restrict__ B, uint32_t N,
                                         uint32_t c0, uint32_t slot, uint32_t S, float (&acc)[CF]) {
    // Slot-owned SCF-entry chunks, SCF-aligned so cols and vals come in one
    // 16-byte load each; entries outside [b, e) (aligned over-read into the
    // neighbouring rows / zero padding, always valid column indices) are
    // masked by zeroing their value, never by a branch, so all SCF B-row
    // gathers of a chunk are in flight together.  The next chunk's A loads are
    // issued before this chunk's gathers (software pipelining).
    typedef typename raw_vec<CF * sizeof(VT)>::t RB;
    const uint32_t a = b & ~(uint32_t)(SCF - 1);
    uint32_t p0 = a + slot * SCF;
    CT cn[SCF];
    VT vn[SCF];
    if (p0 < e) {
        load_raw<CT, SCF>(col + p0, cn);
        load_raw<VT, SCF>(val + p0, vn);
    }
    while (p0 < e) {
        CT cc[SCF];
        VT vv[SCF];
#pragma unroll
        for (int j = 0; j < SCF; j++) { cc[j] = cn[j]; vv[j] = vn[j]; }
        const uint32_t pn = p0 + S * SCF;
        if (pn < e) {
            load_raw<CT, SCF>(col + pn, cn);
            load_raw<VT, SCF>(val + pn, vn);
        }
        RB braw[SCF];
#pragma unroll
        for (int j = 0; j < SCF; j++) braw[j] = *reinterpret_cast<const RB *>(B + (size_t)cc[j] * N + c0);
#pragma unroll
        for (int j = 0; j < SCF; j++) {
            const uint32_t p = p0 + j;
            const float v = (p >= b && p < e) ? (float)vv[j] : 0.f;
            VT bt[CF];
            __builtin_memcpy(bt, &braw[j], sizeof(RB));
#pragma unroll
            for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(v, (float)bt[k], acc[k]);
        }
        p0 = pn;
    }
}

#ifndef GS_WR_MAXCH  // A/B builds only (make var VAR_FLAGS=...): chunk capacity and waves per SIMD of k_warp_rows_mc
#define GS_WR_MAXCH 3
#endif
#ifndef GS_WR_WPE
#define GS_WR_WPE 4
#endif
constexpr uint32_t kWarpRowsMaxChunks = GS_WR_MAXCH;  // k_warp_rows_mc: SCF-chunks per slot in one grouped pass (WARP_ROWS_CHUNKS)

template <class VT, class CT, int CF, int SCF, bool FX, uint32_t MC = 1>
__device__ __forceinline__ void warp_rows_body(const uint32_t *__restrict__ bmw_first_row,  // n_bmw+1
                                                   const idx_formula f_row,
                                                   const uint32_t *__restrict__ bmw_of_bmtb,    // n_bmtb+1 or null
                                                   const idx_formula f_bmw,                     // kind ARRAY + null: no BMTB level
                                                   const uint32_t *__restrict__ row_ptr,        // rows+1 (CSR)
                                                   const CT *__restrict__ col, const VT *__restrict__ val,
                                                   const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmw,
                                                   uint32_t N, uint32_t X, uint32_t row_base, uint32_t G, uint32_t nch) {
    // G slots per row (a power of two <= S): the wave takes S/G consecutive rows of the BMW at
    // a time, so rows much shorter than S*SCF nonzeros do not leave most slots idle (C1: rows
    // of ~37 nonzeros against 128-nonzero wave passes at N = 8)
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t xl = lane & (X - 1u);
    const uint32_t S0 = 64u / X;
    const uint32_t S = G < S0 ? G : S0, RP = S0 / S;
    const uint32_t slot = (lane / X) % S, grp = (lane / X) / S;
    const uint32_t wib = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint32_t w_begin, w_end, w_step;
    if (bmw_of_bmtb || f_bmw.kind != IDX_ARRAY) {
        const uint32_t t = xcd_block(blockIdx.x, gridDim.x);
        idx_range<FX>(bmw_of_bmtb, f_bmw, t, w_begin, w_end);
        w_begin += wib;
        w_step = wpb;
    } else {
        w_begin = xcd_block(blockIdx.x, gridDim.x) * wpb + wib;
        w_end = n_bmw;
        w_step = gridDim.x * wpb;
    }
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t w = w_begin; w < w_end; w += w_step) {
            uint32_t r_begin, r_end;
            idx_range<FX>(bmw_first_row, f_row, w, r_begin, r_end);
            if (RP > 1 && r_end - r_begin <= 63u) {
                // grouped passes, software-pipelined: the BMW's row starts in one load (lane i
                // holds row_ptr[r_begin + i]); a pass gives each slot up to nch SCF-chunks of its
                // row at once (all their A loads, then all their B gathers in flight: one gather
                // round trip per pass, not one per chunk), and pass ps+1's chunks are loaded before
                // the gathers of pass ps, so a pass waits on one gather latency, not three
                typedef typename raw_vec<CF * sizeof(VT)>::t RB;
                const uint32_t nr = r_end - r_begin, npass = (nr + RP - 1) / RP;
                const uint32_t rpv = lane <= nr ? row_ptr[r_begin + lane] : 0u;
                auto bounds = [&](uint32_t ps, uint32_t &b, uint32_t &e) {  // rows past the end: b == e
                    const uint32_t i = ps * RP + grp;
                    b = (uint32_t)__shfl((int)rpv, (int)min(i, nr), 64);
                    e = (uint32_t)__shfl((int)rpv, (int)min(i + 1u, nr), 64);
                };
                auto fma_chunk = [&](uint32_t q, uint32_t b, uint32_t e, const VT (&vv)[SCF], const RB (&braw)[SCF],
                                     float (&acc)[CF]) {
#pragma unroll
                    for (int j = 0; j < SCF; j++) {
                        const float v = (q + j >= b && q + j < e) ? (float)vv[j] : 0.f;
                        VT bt[CF];
                        __builtin_memcpy(bt, &braw[j], sizeof(RB));
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(v, (float)bt[k], acc[k]);
                    }
                };
                auto chunk = [&](uint32_t q, uint32_t b, uint32_t e, const CT (&cc)[SCF], const VT (&vv)[SCF],
                                 float (&acc)[CF]) {
                    RB braw[SCF];
#pragma unroll
                    for (int j = 0; j < SCF; j++) braw[j] = *reinterpret_cast<const RB *>(B + (size_t)cc[j] * N + c0);
                    fma_chunk(q, b, e, vv, braw, acc);
                };
                // chunk c of a pass: entries p + c*S*SCF .. (chunks past the row: column 0, value 0)
                CT cn[MC][SCF];
                VT vn[MC][SCF];
                auto load_pass = [&](uint32_t p, uint32_t e) {
#pragma unroll
                    for (uint32_t c = 0; c < MC; c++) {
                        if (c >= nch) break;
                        const uint32_t q = p + c * S * SCF;
                        if (q < e) {
                            load_raw<CT, SCF>(col + q, cn[c]);
                            load_raw<VT, SCF>(val + q, vn[c]);
                        } else {
#pragma unroll
                            for (int j = 0; j < SCF; j++) { cn[c][j] = (CT)0; vn[c][j] = (VT)0.f; }
                        }
                    }
                };
                uint32_t b, e;
                bounds(0u, b, e);
                uint32_t p = (b & ~(uint32_t)(SCF - 1)) + slot * SCF;
                load_pass(p, e);
                for (uint32_t ps = 0; ps < npass; ps++) {
                    CT cc[MC][SCF];
                    VT vv[MC][SCF];
#pragma unroll
                    for (uint32_t c = 0; c < MC; c++)
#pragma unroll
                        for (int j = 0; j < SCF; j++) { cc[c][j] = cn[c][j]; vv[c][j] = vn[c][j]; }
                    const uint32_t cb = b, ce = e, cp = p;
                    if (ps + 1 < npass) {
                        bounds(ps + 1u, b, e);
                        p = (b & ~(uint32_t)(SCF - 1)) + slot * SCF;
                        load_pass(p, e);
                    }
                    float acc[CF];
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] = 0.f;
                    if (cp < ce) {
                        // every chunk's gathers before any chunk's FMAs
                        RB braw[MC][SCF];
#pragma unroll
                        for (uint32_t c = 0; c < MC; c++) {
                            if (c >= nch) break;
#pragma unroll
                            for (int j = 0; j < SCF; j++)
                                braw[c][j] = *reinterpret_cast<const RB *>(B + (size_t)cc[c][j] * N + c0);
                        }
#pragma unroll
                        for (uint32_t c = 0; c < MC; c++) {
                            if (c >= nch) break;
                            fma_chunk(cp + c * S * SCF, cb, ce, vv[c], braw[c], acc);
                        }
                        for (uint32_t q = cp + nch * S * SCF; q < ce; q += S * SCF) {  // rest of a long row
                            CT cq[SCF];
                            VT vq[SCF];
                            load_raw<CT, SCF>(col + q, cq);
                            load_raw<VT, SCF>(val + q, vq);
                            chunk(q, cb, ce, cq, vq, acc);
                        }
                    }
                    for (uint32_t off = X; off < X * S; off <<= 1) {
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] += __shfl_xor(acc[k], (int)off, 64);
                    }
                    const uint32_t r = r_begin + ps * RP + grp;
                    if (slot == 0 && cok && r < r_end) store_f32<VT, CF>(C + (size_t)(r + row_base) * N + c0, acc);
                }
                continue;
            }
            for (uint32_t r0 = r_begin; r0 < r_end; r0 += RP) {
                const uint32_t r = r0 + grp;
                const bool live = r < r_end;
                float acc[CF];
#pragma unroll
                for (int k = 0; k < CF; k++) acc[k] = 0.f;
                if (live) wave_row<VT, CT, CF, SCF>(row_ptr[r], row_ptr[r + 1], col, val, B, N, c0, slot, S, acc);
                for (uint32_t off = X; off < X * S; off <<= 1) {
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] += __shfl_xor(acc[k], (int)off, 64);
                }
                if (slot == 0 && cok && live) store_f32<VT, CF>(C + (size_t)(r + row_base) * N + c0, acc);
            }
        }
    }
}

template <class VT, class CT, int CF, int SCF, uint32_t MC>
__device__ __forceinline__ void warp_rows_kernel(const uint32_t *__restrict__ bmw_first_row, const idx_formula f_row,
                                                 const uint32_t *__restrict__ bmw_of_bmtb, const idx_formula f_bmw,
                                                 const uint32_t *__restrict__ row_ptr, const CT *__restrict__ col,
                                                 const VT *__restrict__ val, const VT *__restrict__ B, VT *__restrict__ C,
                                                 uint32_t n_bmw, uint32_t N, uint32_t X, uint32_t row_base, uint32_t G,
                                                 uint32_t nch) {
    nch = nch < 1u ? 1u : (nch > MC ? MC : nch);
    if (f_row.kind == IDX_ARRAY && f_bmw.kind == IDX_ARRAY)
        warp_rows_body<VT, CT, CF, SCF, false, MC>(bmw_first_row, f_row, bmw_of_bmtb, f_bmw, row_ptr, col, val, B, C, n_bmw,
                                                   N, X, row_base, G, nch);
    else
        warp_rows_body<VT, CT, CF, SCF, true, MC>(bmw_first_row, f_row, bmw_of_bmtb, f_bmw, row_ptr, col, val, B, C, n_bmw,
                                                  N, X, row_base, G, nch);
}

// one SCF-chunk per slot and pass (registers as the plan needs them)
template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) void k_warp_rows(const uint32_t *__restrict__ bmw_first_row, const idx_formula f_row,
                                                   const uint32_t *__restrict__ bmw_of_bmtb, const idx_formula f_bmw,
                                                   const uint32_t *__restrict__ row_ptr, const CT *__restrict__ col,
                                                   const VT *__restrict__ val, const VT *__restrict__ B, VT *__restrict__ C,
                                                   uint32_t n_bmw, uint32_t N, uint32_t X, uint32_t row_base,
                                                   uint32_t G = 64) {
    warp_rows_kernel<VT, CT, CF, SCF, 1>(bmw_first_row, f_row, bmw_of_bmtb, f_bmw, row_ptr, col, val, B, C, n_bmw, N, X,
                                         row_base, G, 1u);
}

// up to kWarpRowsMaxChunks SCF-chunks per slot and pass, at most 128 VGPRs (four waves per SIMD):
// launched for fp32 values, u16 columns and 4-entry chunks of 16-B B pieces (C1: fp32, N = 8), the
// instantiations that fit 128 registers without spilling
template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS_WR_WPE))) void k_warp_rows_mc(
    const uint32_t *__restrict__ bmw_first_row, const idx_formula f_row, const uint32_t *__restrict__ bmw_of_bmtb,
    const idx_formula f_bmw, const uint32_t *__restrict__ row_ptr, const CT *__restrict__ col, const VT *__restrict__ val,
    const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmw, uint32_t N, uint32_t X, uint32_t row_base, uint32_t G,
    uint32_t nch) {
    static_assert(SCF <= 4 && CF * sizeof(VT) <= 16, "k_warp_rows_mc: 4-entry chunks, B pieces of at most 16 B");
    warp_rows_kernel<VT, CT, CF, SCF, kWarpRowsMaxChunks>(bmw_first_row, f_row, bmw_of_bmtb, f_bmw, row_ptr, col, val, B, C,
                                                          n_bmw, N, X, row_base, G, nch);
}

// ---------------------------------------------------------------------------
// K6 tblock_total: one 256-thread workgroup per BMTB (fixed row-direction
// TBLOCK blocking + tblock_total_reduce_operator; the reference reduces every
// row of the BMTB over blockDim.y with __syncthreads,
// total_block_reduce_to_one_register_token.cc:374-480).  Here the BMTB's rows
// are taken in windows of kBrWindow: the 4S slots (X column lanes each) walk the
// window's rows slot-per-row and store the short ones (<= kBrSlot nonzeros)
// directly; medium rows (<= solo) are listed and each taken by one wave (its S
// slots split the row, one xor-shuffle reduction, no barrier); longer rows are
// listed in LDS and then reduced by the whole workgroup (all 4S slots split the
// row, registers, then one LDS round of four wave partials).  Short-row BMTBs
// (balanced_block_total on power-law graphs: hundreds of 1-10 nnz rows) cost three
// barriers per window instead of two per row; a medium row no longer serialises
// its slot's wave (one dependent gather round per 4 nonzeros); long-row BMTBs keep
// the cooperative path.
// ---------------------------------------------------------------------------
constexpr uint32_t kBrWindow = 1024;  // rows per window (the long/medium row lists' capacity)
constexpr uint32_t kBrSlot = 8;       // a row of at most this many nonzeros is one slot's
constexpr uint32_t kBrSolo = 512;     // ... at most this many one wave's (more: the workgroup's)

template <class VT, class CT, int CF, int SCF, bool FX>
__device__ __forceinline__ void block_rows_body(const uint32_t *__restrict__ bmtb_first_row,  // n_bmtb+1
                                                    const idx_formula f_row,
                                                    const uint32_t *__restrict__ row_ptr,
                                                    const CT *__restrict__ col, const VT *__restrict__ val,
                                                    const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmtb,
                                                    uint32_t N, uint32_t X, uint32_t row_base,
                                                    float (*part)[64][CF],  // [4][64][CF] in LDS
                                                    uint32_t *long_rows,    // [kBrWindow + 1] in LDS
                                                    uint32_t *med_rows,     // [kBrWindow + 1] in LDS
                                                    uint32_t solo) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t xl = lane & (X - 1u);
    const uint32_t S = 64u / X;
    const uint32_t slot = wib * S + lane / X;  // 0 .. 4S-1
    uint32_t *n_long = long_rows + kBrWindow;
    uint32_t *n_med = med_rows + kBrWindow;
    const uint32_t one = min(solo, kBrSlot);  // slot-per-row bound
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t t = xcd_block(blockIdx.x, gridDim.x); t < n_bmtb; t += gridDim.x) {
            uint32_t r_begin, r_end;
            idx_range<FX>(bmtb_first_row, f_row, t, r_begin, r_end);
            for (uint32_t w0 = r_begin; w0 < r_end; w0 += kBrWindow) {
                const uint32_t w1 = min(r_end, w0 + kBrWindow);
                if (threadIdx.x == 0) {
                    *n_long = 0u;
                    *n_med = 0u;
                }
                __syncthreads();
                // slot-per-row over the window; medium and long rows are listed.  The next
                // row's bounds are loaded before this row's entries (one dependent round trip
                // less per row: a slot walks hundreds of short rows in a 17,864-row BMTB)
                uint32_t rbn = 0, ren = 0;
                if (w0 + slot < w1) {
                    rbn = row_ptr[w0 + slot];
                    ren = row_ptr[w0 + slot + 1];
                }
                for (uint32_t r = w0 + slot; r < w1; r += 4u * S) {
                    const uint32_t rb = rbn, re = ren;
                    if (r + 4u * S < w1) {
                        rbn = row_ptr[r + 4u * S];
                        ren = row_ptr[r + 4u * S + 1];
                    }
                    if (re - rb <= one) {
                        float acc[CF];
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] = 0.f;
                        wave_row<VT, CT, CF, SCF>(rb, re, col, val, B, N, c0, 0u, 1u, acc);
                        if (cok) store_f32<VT, CF>(C + (size_t)(r + row_base) * N + c0, acc);
                    } else if (xl == 0u) {
                        if (re - rb <= solo) med_rows[atomicAdd(n_med, 1u)] = r;
                        else long_rows[atomicAdd(n_long, 1u)] = r;
                    }
                }
                __syncthreads();
                // medium rows: one wave each (its S slots split the row)
                const uint32_t nm = *n_med;
                for (uint32_t i = wib; i < nm; i += 4u) {
                    const uint32_t r = med_rows[i];
                    float acc[CF];
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] = 0.f;
                    wave_row<VT, CT, CF, SCF>(row_ptr[r], row_ptr[r + 1], col, val, B, N, c0, lane / X, S, acc);
                    wave_reduce_slots<CF>(acc, (int)X);
                    if (lane < X && cok) store_f32<VT, CF>(C + (size_t)(r + row_base) * N + c0, acc);
                }
                const uint32_t nl = *n_long;
                for (uint32_t i = 0; i < nl; i++) {  // the window's long rows, the whole workgroup each
                    const uint32_t r = long_rows[i];
                    float acc[CF];
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] = 0.f;
                    wave_row<VT, CT, CF, SCF>(row_ptr[r], row_ptr[r + 1], col, val, B, N, c0, slot, 4 * S, acc);
                    wave_reduce_slots<CF>(acc, (int)X);
                    if (lane < X) {
#pragma unroll
                        for (int k = 0; k < CF; k++) part[wib][lane][k] = acc[k];
                    }
                    __syncthreads();
                    if (wib == 0 && lane < X && cok) {
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] = part[0][lane][k] + part[1][lane][k] + part[2][lane][k] + part[3][lane][k];
                        store_f32<VT, CF>(C + (size_t)(r + row_base) * N + c0, acc);
                    }
                    __syncthreads();
                }
                __syncthreads();  // every thread has read n_long before the next window resets it
            }
        }
    }
}

template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) void k_block_rows(const uint32_t *__restrict__ bmtb_first_row, const idx_formula f_row,
                                                    const uint32_t *__restrict__ row_ptr, const CT *__restrict__ col,
                                                    const VT *__restrict__ val, const VT *__restrict__ B, VT *__restrict__ C,
                                                    uint32_t n_bmtb, uint32_t N, uint32_t X, uint32_t row_base,
                                                    uint32_t solo = kBrSolo) {
    __shared__ float part[4][64][CF];
    __shared__ uint32_t long_rows[kBrWindow + 1];
    __shared__ uint32_t med_rows[kBrWindow + 1];
    if (f_row.kind == IDX_ARRAY)
        block_rows_body<VT, CT, CF, SCF, false>(bmtb_first_row, f_row, row_ptr, col, val, B, C, n_bmtb, N, X, row_base, part,
                                                long_rows, med_rows, solo);
    else
        block_rows_body<VT, CT, CF, SCF, true>(bmtb_first_row, f_row, row_ptr, col, val, B, C, n_bmtb, N, X, row_base, part,
                                               long_rows, med_rows, solo);
}

// ---------------------------------------------------------------------------
// K2 + K3 bitmap segments (fixed_interval_nnz_direction_thread_blocking_operator
// (32) + thread_bit_map_operator (+ warp_segment_reduce_operator)).  Slot s of
// wave w walks BMT w*S+s.  Row starts come from the BMT's row-start mask (the
// plan's thread_bit_map without the forced BMW heads, thread_bit_map.cc:45-71),
// segment rows from segment_ptr + segment_empty_row_indices
// (segment_ptr.cc / segment_empty_row_indices.cc).  Segments that start and
// end inside the BMT are complete and stored; the open head/tail partials of
// the wave's slots are merged in slot order through LDS (the K3 segmented
// combine, warp_segment_reduce_token.cc:26-444) and added with one atomic per
// row run.  C must be zeroed first.
// ---------------------------------------------------------------------------
template <class VT, class CT, int CF, int SCF, bool FX>
__device__ __forceinline__ void bitmap_segment_body(const uint32_t *__restrict__ bmt_first_nz,   // n_bmt+1
                                                        const idx_formula f_nz,
                                                        const uint32_t *__restrict__ bmt_first_row,  // n_bmt+1
                                                        const idx_formula f_row,
                                                        const uint64_t *__restrict__ row_start_mask, // n_bmt
                                                        const uint32_t *__restrict__ seg_ptr,        // n_bmt
                                                        const uint32_t *__restrict__ seg_row_off,    // segments
                                                        const CT *__restrict__ col, const VT *__restrict__ val,
                                                        const VT *__restrict__ B, VT *__restrict__ C, uint32_t n_bmt,
                                                        uint32_t N, uint32_t X, uint32_t row_base,
                                                        float *__restrict__ ws,
                                                        uint32_t (*open_row)[64][2]) {  // [4][64][2] in LDS
    // ws != nullptr (fp16 C): rows shared between BMTs accumulate in an fp32
    // workspace (k_finalize_rows rounds them to C once); else atomics go to C.
    // per wave: up to 2 open partials per slot (head, tail), S <= 64
    extern __shared__ float dyn[];  // [4 waves][S slots][2][X lanes][CF]
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t xl = lane & (X - 1u);
    const uint32_t slot = lane / X;
    const uint32_t S = 64u / X;
    float *my_dyn = dyn + (size_t)wib * S * 2 * X * CF;
    const uint32_t waves_total = gridDim.x * (blockDim.x >> 6);
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t w = xcd_block(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wib; w * S < n_bmt; w += waves_total) {
            const uint32_t bt = w * S + slot;
            uint32_t head_row = 0xffffffffu, tail_row = 0xffffffffu;
            float head_acc[CF], acc[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) { acc[k] = 0.f; head_acc[k] = 0.f; }
            if (bt < n_bmt) {
                uint32_t b, e;
                idx_range<FX>(bmt_first_nz, f_nz, bt, b, e);
                const uint64_t mask = row_start_mask[bt];
                const bool next_continues = (bt + 1 < n_bmt) && !(row_start_mask[bt + 1] & 1ull);
                const uint32_t r0 = idx_at<FX>(bmt_first_row, f_row, bt);
                const uint32_t sbase = seg_ptr[bt];
                uint32_t seg = 0, cur_row = r0;
                bool cur_open_head = !(mask & 1ull);
                typedef typename raw_vec<CF * sizeof(VT)>::t RB;
                for (uint32_t p0 = b; p0 < e; p0 += SCF) {
                    CT cc[SCF];
                    VT vv[SCF];
                    load_raw<CT, SCF>(col + p0, cc);
                    load_raw<VT, SCF>(val + p0, vv);
                    RB braw[SCF];  // all gathers of the chunk in flight before any use
#pragma unroll
                    for (int j = 0; j < SCF; j++) braw[j] = *reinterpret_cast<const RB *>(B + (size_t)cc[j] * N + c0);
#pragma unroll
                    for (int j = 0; j < SCF; j++) {
                        const uint32_t i = p0 + j - b;
                        if (i > 0 && ((mask >> i) & 1ull)) {  // a new row starts: flush the current segment
                            if (cur_open_head) {
                                head_row = cur_row;
#pragma unroll
                                for (int k = 0; k < CF; k++) head_acc[k] = acc[k];
                            } else if (cok) {
                                store_f32<VT, CF>(C + (size_t)(cur_row + row_base) * N + c0, acc);
                            }
#pragma unroll
                            for (int k = 0; k < CF; k++) acc[k] = 0.f;
                            seg++;
                            cur_row = r0 + seg_row_off[sbase + seg];
                            cur_open_head = false;
                        }
                        VT bt[CF];
                        __builtin_memcpy(bt, &braw[j], sizeof(RB));
                        const float v = (float)vv[j];
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(v, (float)bt[k], acc[k]);
                    }
                }
                // last segment
                if (cur_open_head || next_continues) {
                    if (cur_open_head && !next_continues) {
                        head_row = cur_row;
#pragma unroll
                        for (int k = 0; k < CF; k++) head_acc[k] = acc[k];
                    } else {
                        tail_row = cur_row;  // open at the tail (and maybe at the head too)
                        if (cur_open_head) head_row = 0xffffffffu;
                    }
                } else if (cok) {
                    store_f32<VT, CF>(C + (size_t)(cur_row + row_base) * N + c0, acc);
                }
            }
            // publish open partials: [slot][0] = head, [slot][1] = tail
            if (xl == 0) {
                open_row[wib][slot][0] = head_row;
                open_row[wib][slot][1] = tail_row;
            }
            float *hp = my_dyn + ((size_t)(slot * 2 + 0) * X + xl) * CF;
            float *tp = my_dyn + ((size_t)(slot * 2 + 1) * X + xl) * CF;
#pragma unroll
            for (int k = 0; k < CF; k++) { hp[k] = head_acc[k]; tp[k] = acc[k]; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // slot 0's lanes merge the 2S open partials in order, one atomic per row run
            if (slot == 0 && cok) {
                uint32_t run_row = 0xffffffffu;
                float run[CF];
#pragma unroll
                for (int k = 0; k < CF; k++) run[k] = 0.f;
                for (uint32_t q = 0; q < 2 * S; q++) {
                    const uint32_t r = open_row[wib][q >> 1][q & 1];
                    if (r == 0xffffffffu) continue;
                    const float *src = my_dyn + ((size_t)q * X + xl) * CF;
                    if (r != run_row) {
                        if (run_row != 0xffffffffu) {
                            if (ws) atomic_add_vals<float, CF>(ws + (size_t)(run_row + row_base) * N + c0, run);
                            else atomic_add_vals<VT, CF>(C + (size_t)(run_row + row_base) * N + c0, run);
                        }
                        run_row = r;
#pragma unroll
                        for (int k = 0; k < CF; k++) run[k] = src[k];
                    } else {
#pragma unroll
                        for (int k = 0; k < CF; k++) run[k] += src[k];
                    }
                }
                if (run_row != 0xffffffffu) {
                    if (ws) atomic_add_vals<float, CF>(ws + (size_t)(run_row + row_base) * N + c0, run);
                    else atomic_add_vals<VT, CF>(C + (size_t)(run_row + row_base) * N + c0, run);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) void k_bitmap_segment(const uint32_t *__restrict__ bmt_first_nz, const idx_formula f_nz,
                                                        const uint32_t *__restrict__ bmt_first_row, const idx_formula f_row,
                                                        const uint64_t *__restrict__ row_start_mask,
                                                        const uint32_t *__restrict__ seg_ptr,
                                                        const uint32_t *__restrict__ seg_row_off, const CT *__restrict__ col,
                                                        const VT *__restrict__ val, const VT *__restrict__ B,
                                                        VT *__restrict__ C, uint32_t n_bmt, uint32_t N, uint32_t X,
                                                        uint32_t row_base, float *__restrict__ ws) {
    __shared__ uint32_t open_row[4][64][2];
    if (f_nz.kind == IDX_ARRAY && f_row.kind == IDX_ARRAY)
        bitmap_segment_body<VT, CT, CF, SCF, false>(bmt_first_nz, f_nz, bmt_first_row, f_row, row_start_mask, seg_ptr,
                                                    seg_row_off, col, val, B, C, n_bmt, N, X, row_base, ws, open_row);
    else
        bitmap_segment_body<VT, CT, CF, SCF, true>(bmt_first_nz, f_nz, bmt_first_row, f_row, row_start_mask, seg_ptr,
                                                   seg_row_off, col, val, B, C, n_bmt, N, X, row_base, ws, open_row);
}

// ---------------------------------------------------------------------------
// K5 / K7 on col-direction plans (fixed_interval_col_direction_thread_blocking_
// operator + thread_total_reduce + warp_bit_map_operator / tblock_thread_bit_map_
// operator; token_test.cc:1250-1315, 1515-1582).  Every BMT is a chunk of ONE
// row, so a row is a run of consecutive BMTs.  A wave owns U consecutive BMTs
// and walks them S = 64/X at a time, one BMT per X-lane slot.  Equal-row slots
// are summed by a segmented shuffle tree (the row-equality-guarded __shfl_down
// of warp_bit_map_reduce_token.cc), the run reaching the end of a group is
// carried in registers into the next group, and a row is written once it
// closes: a plain store when the row lies inside the wave's range, fp32 atomics
// into `ws` when a neighbouring wave shares it (k_finalize_rows then rounds
// those rows and writes the empty ones).
// ---------------------------------------------------------------------------
template <class VT, class CT, int CF, int SCF, bool FX>
__device__ __forceinline__ void row_chunks_body(const uint32_t *__restrict__ bmt_nz,   // n_bmt+1
                                                    const idx_formula f_nz,
                                                    const uint32_t *__restrict__ bmt_row,  // n_bmt
                                                    const idx_formula f_row,
                                                    const CT *__restrict__ col, const VT *__restrict__ val,
                                                    const VT *__restrict__ B, VT *__restrict__ C,
                                                    float *__restrict__ ws, uint32_t n_bmt, uint32_t U, uint32_t N,
                                                    uint32_t X, uint32_t row_base, uint32_t ilv = 0,
                                                    const uint32_t *__restrict__ ilv_base = nullptr,
                                                    const uint32_t *__restrict__ ilv_stride = nullptr) {
    // ilv > 0: interleaved storage (interlance_storage_operator, GLOBAL parent): every BMT
    // has ilv nonzeros and the i-th of BMT b sits at b + i * n_bmt, so the slots of a wave
    // read consecutive addresses (total_BMT_result_reduce_to_one_register_token.cc:581-624).
    // ilv_base: interleaved per TBLOCK / WARP parent (modify_col_indices_by_interlance_storage.cc
    // :73-118): the i-th nonzero of BMT b sits at ilv_base[b] + i * ilv_stride[b] = the parent's
    // first nonzero + (b - its first BMT) + i * its BMT count; BMT b keeps its own size
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t xl = lane & (X - 1u);
    const uint32_t slot = lane / X;
    const uint32_t S = 64u / X;
    const uint32_t waves_total = gridDim.x * (blockDim.x >> 6);
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t w = xcd_block(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); (size_t)w * U < n_bmt;
             w += waves_total) {
            const uint32_t r0 = w * U, r1 = min(r0 + U, n_bmt);
            const uint32_t first_row = idx_at<FX>(bmt_row, f_row, r0), last_row = idx_at<FX>(bmt_row, f_row, r1 - 1);
            const bool head_shared = r0 > 0 && idx_at<FX>(bmt_row, f_row, r0 - 1) == first_row;
            const bool tail_shared = r1 < n_bmt && idx_at<FX>(bmt_row, f_row, r1) == last_row;
            float carry[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) carry[k] = 0.f;
            uint32_t carry_row = 0xffffffffu;
            for (uint32_t g = r0; g < r1; g += S) {
                const uint32_t bt = g + slot;
                const bool valid = bt < r1;
                const uint32_t row = valid ? idx_at<FX>(bmt_row, f_row, bt) : 0xfffffffeu;
                float acc[CF];
#pragma unroll
                for (int k = 0; k < CF; k++) acc[k] = 0.f;
                if (valid) {
                    if (ilv_base) {
                        uint32_t b, e;
                        idx_range<FX>(bmt_nz, f_nz, bt, b, e);
                        const uint32_t q0 = ilv_base[bt], st = ilv_stride[bt];
#pragma unroll 4
                        for (uint32_t i = 0; i < e - b; i++) {
                            const size_t p = (size_t)q0 + (size_t)i * st;
                            fma_row<VT, CF>(acc, (float)val[p], B + (size_t)col[p] * N + c0);
                        }
                    } else if (ilv) {
#pragma unroll 8
                        for (uint32_t i = 0; i < ilv; i++) {
                            const size_t p = (size_t)bt + (size_t)i * n_bmt;
                            fma_row<VT, CF>(acc, (float)val[p], B + (size_t)col[p] * N + c0);
                        }
                    } else {
                        uint32_t b, e;
                        idx_range<FX>(bmt_nz, f_nz, bt, b, e);
                        wave_row<VT, CT, CF, SCF>(b, e, col, val, B, N, c0, 0u, 1u, acc);
                    }
                }
                // segmented suffix sums: the first slot of each run ends with the run total
                for (uint32_t off = 1; off < S; off <<= 1) {
                    const uint32_t rn = __shfl_down(row, off * X, 64);
                    float v[CF];
#pragma unroll
                    for (int k = 0; k < CF; k++) v[k] = __shfl_down(acc[k], off * X, 64);
                    if (slot + off < S && rn == row) {
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] += v[k];
                    }
                }
                const uint32_t rp = __shfl_up(row, X, 64);
                const bool is_head = valid && (slot == 0 || rp != row);
                if (slot == 0 && row == carry_row) {
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] += carry[k];
                }
                const uint32_t nv = min(S, r1 - g);
                const uint32_t lr = __shfl(row, (nv - 1) * X, 64);
                const bool cont = g + S < r1 && idx_at<FX>(bmt_row, f_row, g + S) == lr;
                const unsigned long long hm = __ballot(is_head && row == lr);
                const uint32_t hs = (uint32_t)__builtin_ctzll(hm) / X;
#pragma unroll
                for (int k = 0; k < CF; k++) carry[k] = __shfl(acc[k], hs * X + xl, 64);
                carry_row = cont ? lr : 0xffffffffu;
                if (is_head && !(cont && row == lr) && cok) {
                    const size_t o = (size_t)(row_base + row) * N + cw;
                    if ((row == first_row && head_shared) || (row == last_row && tail_shared))
                        atomic_add_vals<float, CF>(ws + o, acc);
                    else
                        store_f32<VT, CF>(C + o, acc);
                }
            }
        }
    }
}

template <class VT, class CT, int CF, int SCF>
__global__ __launch_bounds__(256) void k_row_chunks(const uint32_t *__restrict__ bmt_nz, const idx_formula f_nz,
                                                    const uint32_t *__restrict__ bmt_row, const idx_formula f_row,
                                                    const CT *__restrict__ col, const VT *__restrict__ val,
                                                    const VT *__restrict__ B, VT *__restrict__ C,
                                                    float *__restrict__ ws, uint32_t n_bmt, uint32_t U, uint32_t N,
                                                    uint32_t X, uint32_t row_base, uint32_t ilv = 0,
                                                    const uint32_t *__restrict__ ilv_base = nullptr,
                                                    const uint32_t *__restrict__ ilv_stride = nullptr) {
    if (f_nz.kind == IDX_ARRAY && f_row.kind == IDX_ARRAY)
        row_chunks_body<VT, CT, CF, SCF, false>(bmt_nz, f_nz, bmt_row, f_row, col, val, B, C, ws, n_bmt, U, N, X, row_base, ilv,
                                                ilv_base, ilv_stride);
    else
        row_chunks_body<VT, CT, CF, SCF, true>(bmt_nz, f_nz, bmt_row, f_row, col, val, B, C, ws, n_bmt, U, N, X, row_base, ilv,
                                               ilv_base, ilv_stride);
}

// ---------------------------------------------------------------------------
// rows listed (shared between BMTs, or empty): C = fp16(workspace), workspace
// re-zeroed for the next launch (companion of k_bitmap_segment with ws and of
// k_row_chunks)
// parent-indexed sub-matrices (row_nz_matrix_div_operator): C row r of the divided range is
// the sum, in sub-matrix order, of row r of every scratch output that has a row r
template <class VT>
__global__ __launch_bounds__(256) void k_combine_parts(const VT *const *__restrict__ parts,
                                                       const uint32_t *__restrict__ rows, uint32_t n,
                                                       VT *__restrict__ C, uint64_t total, uint32_t N) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (uint64_t)gridDim.x * 256) {
        const uint64_t r = e / N;
        float s = 0.f;
        for (uint32_t q = 0; q < n; q++)
            if (r < rows[q]) s += (float)parts[q][e];
        C[e] = (VT)s;
    }
}

// MP_COL_PARTS: C += the fp32 outputs of column partitions 1..n-1, added in partition order
// (deterministic), C rounded once
struct mp_part_outs {
    const float *p[8];
};
template <class VT>
__global__ __launch_bounds__(256) void k_add_parts(VT *__restrict__ C, mp_part_outs parts, uint32_t n, uint64_t total) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (uint64_t)gridDim.x * 256) {
        float s = (float)C[e];
        for (uint32_t q = 0; q < n; q++) s += parts.p[q][e];
        C[e] = (VT)s;
    }
}

template <class VT>
__global__ __launch_bounds__(256) void k_finalize_rows(const uint32_t *__restrict__ rows, uint32_t n_rows,
                                                       float *__restrict__ ws, VT *__restrict__ C, uint32_t N) {
    const size_t total = (size_t)n_rows * N;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const size_t idx = (size_t)rows[e / N] * N + e % N;
        C[idx] = (VT)ws[idx];
        ws[idx] = 0.f;
    }
}

// ---------------------------------------------------------------------------
// v_fma_mix_f32: fp32 += fp16 * fp16 with the conversions folded into the FMA
// (no v_cvt_f32_f16).  VS/BS select the low (0) or high (1) half of the packed
// operand.
// ---------------------------------------------------------------------------
template <int VS, int BS>
__device__ __forceinline__ float fma_mix(uint32_t v_h2, uint32_t b_h2, float c) {
    float d;
    if constexpr (VS == 0 && BS == 0)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(v_h2), "v"(b_h2), "v"(c));
    else if constexpr (VS == 0 && BS == 1)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(v_h2), "v"(b_h2), "v"(c));
    else if constexpr (VS == 1 && BS == 0)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(v_h2), "v"(b_h2), "v"(c));
    else
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(v_h2), "v"(b_h2), "v"(c));
    return d;
}

// acc[0..CF) += v * b (CF fp16 values packed in b_words), v = half VS of v_word
template <int CF, int VS>
__device__ __forceinline__ void fma_row_mix(float (&acc)[CF], uint32_t v_word, const uint32_t *b_words) {
#pragma unroll
    for (int m = 0; m < CF / 2; m++) {
        acc[2 * m] = fma_mix<VS, 0>(v_word, b_words[m], acc[2 * m]);
        acc[2 * m + 1] = fma_mix<VS, 1>(v_word, b_words[m], acc[2 * m + 1]);
    }
}

// ---------------------------------------------------------------------------
// K4 on an LDS-stationary B (tblock_warp_total plan, MI355X layout):
// workgroup g owns BMTB g (<= rpw_max rows); wave w owns BMW g.first_BMW + w
// (<= MAXR rows).  K is cut into nc chunks of KC columns.  Per chunk the
// workgroup stages
//   * B[kc0 : kc0+KC, 0:N]   -> LDS, rows padded to RSB bytes (bank spread),
//   * the BMTB's A entries whose columns fall in the chunk -> LDS, right after
//     it: [cols u16 | vals].  They are stored chunk-major at upload (tile
//     layout [BMTB][chunk][row][entries], 16-bit chunk-local columns, rows
//     padded to 4 entries, segments to 8), so staging is one contiguous copy,
// with the global loads of chunk j+1 issued into registers before computing
// chunk j and written to LDS after the compute barrier.  Every B-row read of
// the inner loop is then an LDS ds_read_b128 instead of an L1/L2 gather: B
// crosses L2->CU once per workgroup instead of once per nonzero.  Accumulators
// of the wave's rows stay in registers across all chunks.
// ---------------------------------------------------------------------------
// compile-time unrolled loop: the index is a constant in every body, so
// register arrays indexed by it stay in VGPRs (no scratch)
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

typedef float f4v __attribute__((ext_vector_type(4)));
// K split (ksp > 1, LDS_KSPLIT): workgroup u = g * ksp + q walks the chunks [q * ncs, +ncs) of
// BMTB g only, publishes its rows' fp32 partials and the last of the ksp workgroups sums them in q
// order (deterministic) -- for plans with too few BMTBs to fill the CUs (upload rule).
template <class VT, int CF, int MAXR, int MAXU>
__global__ __launch_bounds__(1024) void k_lds_rows(
    const uint32_t *__restrict__ bmtb_first_row,  // n_bmtb+1
    const uint32_t *__restrict__ bmw_of_bmtb,     // n_bmtb+1
    const uint32_t *__restrict__ bmw_first_row,   // n_bmw+1
    const uint32_t *__restrict__ seg_start,       // n_bmtb*nc+1: entry offset of (g, j)
    const uint32_t *__restrict__ seg_row_off,     // n_bmtb*nc*(rpw_max+1): row starts inside (g, j)
    const uint16_t *__restrict__ tcol, const VT *__restrict__ tval, const VT *__restrict__ B, VT *__restrict__ C,
    uint32_t K, uint32_t N, uint32_t X, uint32_t KC, uint32_t nc, uint32_t RSB, uint32_t rpw_max, uint32_t seg_cap,
    uint32_t row_base, uint32_t ksp = 1, uint32_t ncs = 0, float *__restrict__ slabs = nullptr,
    uint32_t *__restrict__ arrivals = nullptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef typename raw_vec<CF * sizeof(VT)>::t RB;
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    const uint32_t lane = tid & 63u, wib = tid >> 6;
    const uint32_t xl = lane & (X - 1u), slot = lane / X, S = 64u / X;
    // K split (LDS_KSPLIT): workgroup u = g * ksp + q walks chunks [q * ncs, +ncs) of BMTB g
    const uint32_t g = ksp > 1u ? blockIdx.x / ksp : blockIdx.x, q = ksp > 1u ? blockIdx.x % ksp : 0u;
    const uint32_t j0 = q * (ksp > 1u ? ncs : 0u), j1 = ksp > 1u ? min(nc, j0 + ncs) : nc;
    const uint32_t r_first = bmtb_first_row[g];
    const uint32_t bmw = bmw_of_bmtb[g] + wib;
    uint32_t t0 = 0, nt = 0;
    if (bmw < bmw_of_bmtb[g + 1]) {
        t0 = bmw_first_row[bmw] - r_first;
        nt = bmw_first_row[bmw + 1] - bmw_first_row[bmw];
    }
    const uint32_t UB = X;  // 16-B units per B row (CF * sizeof(VT) == 16)
    const uint32_t lgUB = __builtin_ctz(UB);
    const uint32_t lA = KC * RSB;                        // LDS byte offset of the A segment
    const uint32_t lR = lA + seg_cap * (2u + (uint32_t)sizeof(VT));  // row offsets
    uint32_t *lRp = reinterpret_cast<uint32_t *>(lds + lR);
    const uint32_t c0 = xl * CF;
    const uint32_t cb = c0 * (uint32_t)sizeof(VT);
    const uint32_t ridx = min(tid, rpw_max);

    u32x4 stage[MAXU];  // native vectors (HIP's uint4 is a union struct that defeats SROA)
    uint32_t stage_r;
    uint32_t s_lo = seg_start[g * nc + j0], s_hi = seg_start[g * nc + j0 + 1];

    float acc[MAXR][CF];
#pragma unroll
    for (int t = 0; t < MAXR; t++)
#pragma unroll
        for (int k = 0; k < CF; k++) acc[t][k] = 0.f;

    // issue the global loads of chunk j into registers.  Branch-free: the three
    // source streams are one base per unit picked by a select (B rows, A cols,
    // A vals); units past the end re-read B's first unit.
#define GS_STAGE_LOAD(j, s0, s1)                                                                         \
    {                                                                                                  \
        const uint32_t kc0_ = (j) * KC;                                                                \
        const uint32_t UBt_ = min(KC, K - kc0_) * UB;                                                  \
        const uint32_t len_ = (s1) - (s0);                                                             \
        const uint32_t UAc_ = UBt_ + len_ / 8u, UAe_ = UAc_ + len_ * (uint32_t)sizeof(VT) / 16u;       \
        const unsigned char *pB_ = reinterpret_cast<const unsigned char *>(B + (size_t)kc0_ * N);      \
        const unsigned char *pC_ = reinterpret_cast<const unsigned char *>(tcol + (s0));               \
        const unsigned char *pV_ = reinterpret_cast<const unsigned char *>(tval + (s0));               \
        _Pragma("unroll") for (int I = 0; I < MAXU; I++) {                                             \
            const uint32_t u = tid + I * nthr;                                                         \
            const bool inB = u < UBt_, inC = u < UAc_, live = u < UAe_;                                \
            const unsigned char *base = inB ? static_cast<const unsigned char *>(pB_)                  \
                                      : inC ? static_cast<const unsigned char *>(pC_)                  \
                                      : live ? static_cast<const unsigned char *>(pV_)                 \
                                             : static_cast<const unsigned char *>(pB_);                \
            const uint32_t off = inB ? u : inC ? u - UBt_ : live ? u - UAc_ : 0u;                      \
            stage[I] = *reinterpret_cast<const u32x4 *>(base + (size_t)off * 16u);                     \
        }                                                                                              \
        stage_r = seg_row_off[(size_t)(g * nc + (j)) * (rpw_max + 1) + ridx];                          \
    }

    GS_STAGE_LOAD(j0, s_lo, s_hi);
    for (uint32_t j = j0; j < j1; j++) {
        // registers -> LDS (B rows at RSB stride, A segment contiguous)
        {
            const uint32_t UBt = min(KC, K - j * KC) * UB;
            const uint32_t UAe = UBt + (s_hi - s_lo) * (2u + (uint32_t)sizeof(VT)) / 16u;
#pragma unroll
            for (int I = 0; I < MAXU; I++) {
                const uint32_t u = tid + I * nthr;
                const uint32_t db = (u >> lgUB) * RSB + (u & (UB - 1u)) * 16u;
                const uint32_t da = lA + (u - UBt) * 16u;
                if (u < UAe) *reinterpret_cast<u32x4 *>(lds + (u < UBt ? db : da)) = stage[I];
            }
            if (tid <= rpw_max) lRp[tid] = stage_r;
        }
        __syncthreads();
        const uint32_t len = s_hi - s_lo;
        if (j + 1 < j1) {  // in flight during this chunk's compute
            const uint32_t n_lo = s_hi, n_hi = seg_start[g * nc + j + 2];
            GS_STAGE_LOAD(j + 1, n_lo, n_hi);
            s_lo = n_lo;
            s_hi = n_hi;
        }
        const unsigned char *lAc = lds + lA;
        const unsigned char *lAv = lds + lA + len * 2u;
#pragma unroll
        for (int t = 0; t < MAXR; t++) {
            if ((uint32_t)t < nt) {
                const uint32_t e0 = lRp[t0 + t], e1 = lRp[t0 + t + 1];
                for (uint32_t p0 = e0 + slot * 4u; p0 < e1; p0 += S * 4u) {
                    const uint2 craw = *reinterpret_cast<const uint2 *>(lAc + p0 * 2u);
                    const uint32_t cc[4] = {craw.x & 0xffffu, craw.x >> 16, craw.y & 0xffffu, craw.y >> 16};
                    RB braw[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        // 24-bit LDS byte offsets (KC * RSB <= 160 KB): one v_mad_u32_u24
                        const uint32_t ob = __umul24(cc[q], RSB) + cb;
                        braw[q] = *reinterpret_cast<const RB *>(lds + ob);
                    }
                    if constexpr (sizeof(VT) == 2) {
                        const uint2 vraw = *reinterpret_cast<const uint2 *>(lAv + p0 * 2u);
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            uint32_t bw[CF / 2];
                            __builtin_memcpy(bw, &braw[q], sizeof(RB));
                            const uint32_t vw = (q < 2) ? vraw.x : vraw.y;
                            if (q & 1) fma_row_mix<CF, 1>(acc[t], vw, bw);
                            else fma_row_mix<CF, 0>(acc[t], vw, bw);
                        }
                    } else {
                        const float4 vv = *reinterpret_cast<const float4 *>(lAv + p0 * 4u);
                        const float vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            float bt[CF];
                            __builtin_memcpy(bt, &braw[q], sizeof(RB));
#pragma unroll
                            for (int k = 0; k < CF; k++) acc[t][k] = __builtin_fmaf(vq[q], bt[k], acc[t][k]);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
#undef GS_STAGE_LOAD
#pragma unroll
    for (int t = 0; t < MAXR; t++)
        if ((uint32_t)t < nt) wave_reduce_slots<CF>(acc[t], (int)X);
    if (ksp <= 1u) {
#pragma unroll
        for (int t = 0; t < MAXR; t++)
            if ((uint32_t)t < nt && slot == 0) store_f32<VT, CF>(C + (size_t)(r_first + t0 + t + row_base) * N + c0, acc[t]);
        return;
    }
    // K-split hand-off (k_mfma_ks's drain form, MI355X_MICROARCH.md §Correctness boundaries: sc1
    // stores, every storing wave's vmcnt(0), a barrier, one agent-scope arrival add; the last
    // adder loads the other slabs with sc1 loads): slab (g, q) holds the BMTB's rows x N fp32
    // partials of K range q; the last of the S workgroups sums them in q order (its own from
    // registers: the same bits it stored), so C is the same whichever workgroup arrives last
    const size_t slab_rows = (size_t)rpw_max;
    if (slot == 0) {
#pragma unroll
        for (int t = 0; t < MAXR; t++) {
            if ((uint32_t)t < nt) {
                float *dst = slabs + (((size_t)g * ksp + q) * slab_rows + t0 + t) * N + c0;
#pragma unroll
                for (int k = 0; k < CF; k += 4) {
                    const f4v v = {acc[t][k], acc[t][k + 1], acc[t][k + 2], acc[t][k + 3]};
                    __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + k), "v"(v) : "memory");
                }
            }
        }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t *flag = lRp;  // the row offsets are no longer read
    if (tid == 0) *flag = __hip_atomic_fetch_add(arrivals + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag != ksp - 1u) return;
    if (tid == 0) __hip_atomic_store(arrivals + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (slot != 0) return;
#pragma unroll
    for (int t = 0; t < MAXR; t++) {
        if ((uint32_t)t < nt) {
            float sum[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) sum[k] = 0.f;
            for (uint32_t qq = 0; qq < ksp; qq++) {
                if (qq == q) {
#pragma unroll
                    for (int k = 0; k < CF; k++) sum[k] += acc[t][k];
                    continue;
                }
                const float *src = slabs + (((size_t)g * ksp + qq) * slab_rows + t0 + t) * N + c0;
#pragma unroll
                for (int k = 0; k < CF; k++) sum[k] += __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            store_f32<VT, CF>(C + (size_t)(r_first + t0 + t + row_base) * N + c0, sum);
        }
    }
}


// ---------------------------------------------------------------------------
// k_lds_rows_dma -- k_lds_rows for fp32 B at N = 32 (LDS_DMA): B rows sit in LDS at 128 B, exactly
// their HBM image, so each chunk's B rows and A segment (u16 columns, fp32 values) go to LDS by
// LDS-DMA (global_load_lds_dwordx4: no register staging, no ds_write phase) into one of two
// buffers: chunk j+1 lands while chunk j is computed, one barrier per chunk.  A wave's row offsets
// in the chunk come from scalar loads.  Same compute loop, K split and slab combine as k_lds_rows;
// entries are in the parity-paired order (conflict-free B reads).
// ---------------------------------------------------------------------------
template <int MAXR>
__global__ __launch_bounds__(1024) void k_lds_rows_dma(
    const uint32_t *__restrict__ bmtb_first_row, const uint32_t *__restrict__ bmw_of_bmtb,
    const uint32_t *__restrict__ bmw_first_row, const uint32_t *__restrict__ seg_start,
    const uint32_t *__restrict__ seg_row_off, const uint16_t *__restrict__ tcol, const float *__restrict__ tval,
    const float *__restrict__ B, float *__restrict__ C, uint32_t K, uint32_t KC, uint32_t nc, uint32_t rpw_max,
    uint32_t seg_cap, uint32_t row_base, uint32_t ksp, uint32_t ncs, float *__restrict__ slabs,
    uint32_t *__restrict__ arrivals) {
    constexpr uint32_t N = 32, CF = 4, X = 8, S = 8, RSB = 128;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, nthr = blockDim.x, nwv = nthr >> 6;
    const uint32_t lane = tid & 63u, wib = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t xl = lane & (X - 1u), slot = lane / X;
    const uint32_t g = ksp > 1u ? blockIdx.x / ksp : blockIdx.x, q = ksp > 1u ? blockIdx.x % ksp : 0u;
    const uint32_t j0 = q * (ksp > 1u ? ncs : 0u), j1 = ksp > 1u ? min(nc, j0 + ncs) : nc;
    const uint32_t r_first = bmtb_first_row[g];
    const uint32_t bmw = bmw_of_bmtb[g] + wib;
    uint32_t t0 = 0, nt = 0;
    if (bmw < bmw_of_bmtb[g + 1]) {
        t0 = bmw_first_row[bmw] - r_first;
        nt = bmw_first_row[bmw + 1] - bmw_first_row[bmw];
    }
    t0 = __builtin_amdgcn_readfirstlane(t0);
    nt = __builtin_amdgcn_readfirstlane(nt);
    // one buffer: B rows [0, KC*128), columns [cap*2), values [cap*4)
    const uint32_t lB = KC * RSB, lV = lB + seg_cap * 2u, szBuf = lV + seg_cap * 4u;
    const uint32_t c0 = xl * CF, cb = c0 * 4u;
    float acc[MAXR][CF];
#pragma unroll
    for (int t = 0; t < MAXR; t++)
#pragma unroll
        for (int k = 0; k < CF; k++) acc[t][k] = 0.f;
    // LDS-DMA of chunk j into buffer b: every wave takes 1 KB blocks (64 lanes x 16 B) of the three
    // contiguous source ranges in turn; lanes past a range's end are masked off
    auto issue = [&](uint32_t j, uint32_t b) {
        unsigned char *dst = lds + b * szBuf;
        const uint32_t kc0 = j * KC, rows = min(KC, K - kc0);
        const uint32_t s0 = seg_start[g * nc + j], len = seg_start[g * nc + j + 1] - s0;
        const unsigned char *srcs[3] = {reinterpret_cast<const unsigned char *>(B + (size_t)kc0 * N),
                                        reinterpret_cast<const unsigned char *>(tcol + s0),
                                        reinterpret_cast<const unsigned char *>(tval + s0)};
        const uint32_t units[3] = {rows * (RSB / 16u), len / 8u, len / 4u};
        const uint32_t dofs[3] = {0u, lB, lV};
#pragma unroll
        for (int r = 0; r < 3; r++) {
            for (uint32_t ib = wib; ib * 64u < units[r]; ib += nwv) {
                const uint32_t u = ib * 64u + lane;
                if (u < units[r])
                    __builtin_amdgcn_global_load_lds((const void *)(srcs[r] + (size_t)u * 16u),
                                                     (__attribute__((address_space(3))) void *)(dst + dofs[r] + ib * 1024u), 16, 0, 0);
            }
        }
    };
    issue(j0, 0u);
    __syncthreads();  // vmcnt(0): chunk j0 landed
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t b = (j - j0) & 1u;
        if (j + 1 < j1) issue(j + 1, b ^ 1u);  // lands while chunk j is computed
        const unsigned char *lAc = lds + b * szBuf + lB;
        const unsigned char *lAv = lds + b * szBuf + lV;
        const unsigned char *lBb = lds + b * szBuf;
        const uint32_t *ro = seg_row_off + (size_t)(g * nc + j) * (rpw_max + 1) + t0;  // this wave's row offsets
#pragma unroll
        for (int t = 0; t < MAXR; t++) {
            if ((uint32_t)t < nt) {
                const uint32_t e0 = ro[t], e1 = ro[t + 1];
                for (uint32_t p0 = e0 + slot * 4u; p0 < e1; p0 += S * 4u) {
                    const uint2 craw = *reinterpret_cast<const uint2 *>(lAc + p0 * 2u);
                    const uint32_t cc[4] = {craw.x & 0xffffu, craw.x >> 16, craw.y & 0xffffu, craw.y >> 16};
                    uint4 braw[4];
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) braw[qq] = *reinterpret_cast<const uint4 *>(lBb + cc[qq] * RSB + cb);
                    const float4 vv = *reinterpret_cast<const float4 *>(lAv + p0 * 4u);
                    const float vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) {
                        float bt[CF];
                        __builtin_memcpy(bt, &braw[qq], 16);
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[t][k] = __builtin_fmaf(vq[qq], bt[k], acc[t][k]);
                    }
                }
            }
        }
        __syncthreads();  // chunk j+1 landed (every wave's vmcnt(0)), chunk j consumed
    }
#pragma unroll
    for (int t = 0; t < MAXR; t++)
        if ((uint32_t)t < nt) wave_reduce_slots<CF>(acc[t], (int)X);
    if (ksp <= 1u) {
#pragma unroll
        for (int t = 0; t < MAXR; t++)
            if ((uint32_t)t < nt && slot == 0) store_f32<float, CF>(C + (size_t)(r_first + t0 + t + row_base) * N + c0, acc[t]);
        return;
    }
    // K-split hand-off: as k_lds_rows (sc1 slab stores, vmcnt(0), barrier, one arrival add)
    const size_t slab_rows = (size_t)rpw_max;
    if (slot == 0) {
#pragma unroll
        for (int t = 0; t < MAXR; t++) {
            if ((uint32_t)t < nt) {
                float *dst = slabs + (((size_t)g * ksp + q) * slab_rows + t0 + t) * N + c0;
                const f4v v = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
                __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
            }
        }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds);
    if (tid == 0) *flag = __hip_atomic_fetch_add(arrivals + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag != ksp - 1u) return;
    if (tid == 0) __hip_atomic_store(arrivals + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (slot != 0) return;
#pragma unroll
    for (int t = 0; t < MAXR; t++) {
        if ((uint32_t)t < nt) {
            float sum[CF] = {0.f, 0.f, 0.f, 0.f};
            for (uint32_t qq = 0; qq < ksp; qq++) {
                if (qq == q) {
#pragma unroll
                    for (int k = 0; k < CF; k++) sum[k] += acc[t][k];
                    continue;
                }
                const float *src = slabs + (((size_t)g * ksp + qq) * slab_rows + t0 + t) * N + c0;
#pragma unroll
                for (int k = 0; k < CF; k++) sum[k] += __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            store_f32<float, CF>(C + (size_t)(r_first + t0 + t + row_base) * N + c0, sum);
        }
    }
}

// ---------------------------------------------------------------------------
// k_lds_rows_rs -- k_lds_rows_dma with one row per slot (fp32, N = 32, BMWs of 5..8 rows): slot s of
// a wave walks row s of its BMW four entries at a time (its 8 lanes x 16 B cover the row of C), so
// a row's chunk segment costs ceil(len / 4) iterations of the slot instead of ceil(len / 32) of the
// whole wave per row (k_lds_rows_dma: a 72-entry segment runs 3 iterations = 96 slots, 75% used),
// and no cross-slot reduction is left at the end.  Taller BMTBs (64 rows in 8-row BMWs) also cut
// the B rows a CU stages per nonzero.  Bank order (device_plan.hip, rowslot): slots {0, 1, 4, 5}
// take entries of column parity k & 1, slots {2, 3, 6, 7} the opposite, so the ds_read_b128 lane
// groups (slots {0,3} and {1,2} of each half-wave) read rows of opposite parity while both kinds
// last.  A slot's row offsets in the chunk come by vector loads (one per chunk, issued with the
// chunk's DMA).  The columns arrive as LDS byte offsets of their B rows (column x 128, device_plan.hip).
// Same DMA double buffer, K split and slab combine as k_lds_rows_dma.
// The chunks' DMA is issued by inline asm (lds_dma16): with the builtin, hipcc's wait inserter puts a
// vmcnt(0) before every LDS read of the issuing wave (the DMA writes LDS), so each wave would wait
// for its share of chunk j+1 before computing chunk j; the kernel retires the DMA itself with
// vmcnt(0) right before each chunk barrier, the only point where the other buffer changes hands.
// (RS: rows per slot, 1; a template so that every translation unit's copy is one symbol)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_dma16(const void *src, const unsigned char *dst) {
    const uint32_t la = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)dst);
    __asm__ volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory");
}
template <int RS = 1>
__global__ __launch_bounds__(1024) void k_lds_rows_rs(
    const uint32_t *__restrict__ bmtb_first_row, const uint32_t *__restrict__ bmw_of_bmtb,
    const uint32_t *__restrict__ bmw_first_row, const uint32_t *__restrict__ seg_start,
    const uint32_t *__restrict__ seg_row_off, const uint16_t *__restrict__ tcol, const float *__restrict__ tval,
    const float *__restrict__ B, float *__restrict__ C, uint32_t K, uint32_t KC, uint32_t nc, uint32_t rpw_max,
    uint32_t seg_cap, uint32_t row_base, uint32_t ksp, uint32_t ncs, float *__restrict__ slabs,
    uint32_t *__restrict__ arrivals) {
    constexpr uint32_t N = 32, CF = 4, X = 8, RSB = 128;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, nthr = blockDim.x, nwv = nthr >> 6;
    const uint32_t lane = tid & 63u, wib = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t xl = lane & (X - 1u), slot = lane / X;
    const uint32_t g = ksp > 1u ? blockIdx.x / ksp : blockIdx.x, q = ksp > 1u ? blockIdx.x % ksp : 0u;
    const uint32_t j0 = q * (ksp > 1u ? ncs : 0u), j1 = ksp > 1u ? min(nc, j0 + ncs) : nc;
    const uint32_t r_first = bmtb_first_row[g];
    const uint32_t bmw = bmw_of_bmtb[g] + wib;
    uint32_t t0 = 0, nt = 0;
    if (bmw < bmw_of_bmtb[g + 1]) {
        t0 = bmw_first_row[bmw] - r_first;
        nt = bmw_first_row[bmw + 1] - bmw_first_row[bmw];
    }
    t0 = __builtin_amdgcn_readfirstlane(t0);
    nt = __builtin_amdgcn_readfirstlane(nt);
    const bool has_row = slot < nt;
    const uint32_t rl = t0 + (has_row ? slot : 0u);  // this slot's row in the BMTB (rl + 1 <= rpw_max)
    const uint32_t lB = KC * RSB, lV = lB + seg_cap * 2u, szBuf = lV + seg_cap * 4u;
    const uint32_t cb = xl * 16u;
    float acc[CF] = {0.f, 0.f, 0.f, 0.f};
    auto issue = [&](uint32_t j, uint32_t b) {
        unsigned char *dst = lds + b * szBuf;
        const uint32_t kc0 = j * KC, rows = min(KC, K - kc0);
        const uint32_t s0 = seg_start[g * nc + j], len = seg_start[g * nc + j + 1] - s0;
        const unsigned char *srcs[3] = {reinterpret_cast<const unsigned char *>(B + (size_t)kc0 * N),
                                        reinterpret_cast<const unsigned char *>(tcol + s0),
                                        reinterpret_cast<const unsigned char *>(tval + s0)};
        const uint32_t units[3] = {rows * (RSB / 16u), len / 8u, len / 4u};
        const uint32_t dofs[3] = {0u, lB, lV};
#pragma unroll
        for (int r = 0; r < 3; r++) {
            for (uint32_t ib = wib; ib * 64u < units[r]; ib += nwv) {
                const uint32_t u = ib * 64u + lane;
                if (u < units[r]) lds_dma16(srcs[r] + (size_t)u * 16u, dst + dofs[r] + ib * 1024u);
            }
        }
    };
    // the slot's row bounds in chunk j (segment-relative entry indices)
    auto row_off = [&](uint32_t j) {
        const uint32_t *ro = seg_row_off + (size_t)(g * nc + j) * (rpw_max + 1) + rl;
        return make_uint2(ro[0], ro[1]);
    };
    uint2 ro_n = row_off(j0);
    issue(j0, 0u);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // chunk j0 landed
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t b = (j - j0) & 1u;
        const uint2 ro = ro_n;
        if (j + 1 < j1) {
            ro_n = row_off(j + 1);
            issue(j + 1, b ^ 1u);  // lands while chunk j is computed
        }
        const unsigned char *lAc = lds + b * szBuf + lB;
        const unsigned char *lAv = lds + b * szBuf + lV;
        const unsigned char *lBb = lds + b * szBuf + cb;
        if (has_row) {
            for (uint32_t p0 = ro.x; p0 < ro.y; p0 += 4u) {
                const uint2 craw = *reinterpret_cast<const uint2 *>(lAc + p0 * 2u);
                const uint32_t cc[4] = {craw.x & 0xffffu, craw.x >> 16, craw.y & 0xffffu, craw.y >> 16};
                uint4 braw[4];
#pragma unroll
                for (int qq = 0; qq < 4; qq++) braw[qq] = *reinterpret_cast<const uint4 *>(lBb + cc[qq]);  // byte offsets
                const float4 vv = *reinterpret_cast<const float4 *>(lAv + p0 * 4u);
                const float vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    float bt[CF];
                    __builtin_memcpy(bt, &braw[qq], 16);
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] = __builtin_fmaf(vq[qq], bt[k], acc[k]);
                }
            }
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk j+1 landed (every wave's vmcnt(0)), chunk j consumed
    }
    const uint32_t c0 = xl * CF;
    if (ksp <= 1u) {
        if (has_row) store_f32<float, CF>(C + (size_t)(r_first + rl + row_base) * N + c0, acc);
        return;
    }
    // K-split hand-off: as k_lds_rows_dma (sc1 slab stores, vmcnt(0), barrier, one arrival add)
    const size_t slab_rows = (size_t)rpw_max;
    if (has_row) {
        float *dst = slabs + (((size_t)g * ksp + q) * slab_rows + rl) * N + c0;
        const f4v v = {acc[0], acc[1], acc[2], acc[3]};
        __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds);
    if (tid == 0) *flag = __hip_atomic_fetch_add(arrivals + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag != ksp - 1u) return;
    if (tid == 0) __hip_atomic_store(arrivals + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!has_row) return;
    float sum[CF] = {0.f, 0.f, 0.f, 0.f};
    for (uint32_t qq = 0; qq < ksp; qq++) {
        if (qq == q) {
#pragma unroll
            for (int k = 0; k < CF; k++) sum[k] += acc[k];
            continue;
        }
        const float *src = slabs + (((size_t)g * ksp + qq) * slab_rows + rl) * N + c0;
#pragma unroll
        for (int k = 0; k < CF; k++) sum[k] += __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    store_f32<float, CF>(C + (size_t)(r_first + rl + row_base) * N + c0, sum);
}

// ---------------------------------------------------------------------------
// BMTB row blocks on the matrix cores (MI355X layout of a tblock/warp/block-
// total plan whose row blocks are dense enough).  Workgroup g owns BMTB g
// (R <= RMAX <= 16*RT rows) and walks K in chunks of KC = 2^LGKC columns.
// 16 waves in three roles, each role its own loop with one barrier per chunk
// (so hipcc's vmcnt analysis of a role sees only that role's loads):
//   compute waves 0-5: v_mfma_f32_16x16x32_f16 over chunk j (A rows by
//     ds_read_b128 from the dense image, B by ds_read_b64_tr_b16, fp32
//     accumulators), then clear the dense image of chunk j+2;
//   B waves 6-9: B rows of chunk j+3 -> registers (three sets), each load
//     next to the LDS store of chunk j+1's rows;
//   entry waves 10-15: compressed entries of chunk j+4 -> registers (four
//     sets: HBM latency is the longest), scatter of chunk j+1's entries
//     (upload layout: per group of 8, [8 x u16 h = row*RS/2 + col, the
//     entry's halfword index in the dense image] in one array and [8 x f16
//     value] in another, so both loads are coalesced and the LDS address is
//     one shift; padding entries write 0 to row R) into its dense image.
// Register set indices are compile-time constants (each role's loop is
// unrolled by its set count).  LDS: two B buffers (row k at k*N*2 bytes, 32-B
// pieces permuted by b_piece() so the transposed reads are conflict-free) and
// three dense images (RMAX+1 rows of RS = 2*KC+32 bytes, conflict-free
// ds_read_b128; row R stays zero and stands in for every MFMA row >= R).  At
// the end the compute waves' partial tiles are summed in a fixed order through
// LDS (deterministic) and rows < R are stored.  A zero of the dense image
// times a non-finite B value gives NaN: the kernel multiplies the row block's
// whole tile.
// ---------------------------------------------------------------------------
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

template <int CT>
__device__ __forceinline__ uint32_t b_piece(uint32_t k, uint32_t p) {
    uint32_t sw;
    if constexpr (CT == 1) sw = 0;
    else if constexpr (CT == 2) sw = (k >> 3) & 1u;
    else if constexpr (CT == 4) sw = ((k >> 1) & 1u) | (((k >> 3) & 1u) << 1);
    else sw = (k & 3u) | (((k >> 3) & 1u) << 2);
    return p ^ (sw & (uint32_t)(CT - 1));
}


// STAMPS (diagnostic build only, gs_debug_mfma_timeline): lane 0 of the first
// compute / B / entry wave records s_memtime at phase boundaries
// NBG (GLDS only): B buffers, the B rows of chunk j + NBG - 1 issued in period j
// WCT: compute waves (the entry waves are the other 16 - WCT - B waves)
// DBG (diagnostic timing builds only, wrong results): 1 no B DMA, 2 no scatter, 4 no compute-wave
// LDS reads or clears, 8 no entry loads
// FLG (round 3, MFMA_FLAGS, LDS-DMA variant only): the roles hand buffers over through three
// LDS counters instead of one workgroup barrier per chunk -- B full (B waves, after the
// chunk's DMA retired), image full (entry waves, after the scatter), chunk consumed (compute
// waves, after their reads and clears); each wave waits (s_sleep polling) only for what
// it consumes, so a role runs ahead of the others by the ring depth
template <int CT, int RT, int LGKC, int MAXA, bool STAMPS = false, int GLDS = 0, int NBG = 3, int WCT = kMfmaCompute,
          int DBG = 0, bool FLG = false>
__global__ __launch_bounds__(64 * kMfmaWaves) void k_mfma_rows(
    const uint32_t *__restrict__ bmtb_first_row,  // n_bmtb+1
    const uint32_t *__restrict__ seg_start,       // n_bmtb*nc+1 (groups)
    const u32x4 *__restrict__ tP,                 // per group: 8 x u16 pos (+1 spare group)
    const u32x4 *__restrict__ tV,                 // per group: 8 x f16 value (+1 spare group)
    const f16 *__restrict__ B, f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t nc, uint32_t RMAX,
    uint32_t row_base, uint32_t nsplit, uint32_t ncs, float *__restrict__ slabs, uint32_t *__restrict__ arrivals,
    uint64_t *__restrict__ stamps = nullptr, uint32_t krot = 0) {
    constexpr uint32_t KC = 1u << LGKC;
    constexpr uint32_t RB = 32 * CT;                  // bytes per LDS B row (N <= 16*CT)
    constexpr uint32_t UB = 2 * CT;                   // 16-B units per B row
    constexpr uint32_t RS = 2 * KC + 32;              // dense image row stride
    constexpr uint32_t NT = 64 * kMfmaWaves;
    constexpr uint32_t WC = WCT;
    constexpr uint32_t BWV = GLDS ? GLDS : kMfmaBWaves;
    constexpr uint32_t NBT = 64 * BWV, NAT = 64 * (kMfmaWaves - WC - BWV);  // B / entry threads
    constexpr uint32_t szB = KC * RB;
    constexpr uint32_t NB = szB / 16 / NBT;           // B units per B thread per chunk
    static_assert(szB % (16 * NBT) == 0, "whole B units per B thread");
    constexpr int MAXS = (int)((KC / 32 + WC - 1) / WC);  // k-steps per compute wave per chunk
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t szD = (RMAX + 1) * RS;
    // register-staged B: two B buffers + three dense images; GLDS (B by LDS-DMA, two
    // chunks ahead): three B buffers + two dense images, each compute wave clearing the
    // k-step columns it read
    constexpr uint32_t NBUF = GLDS ? (uint32_t)NBG : 2u, NDI = GLDS ? 2u : 3u;
    static_assert(!GLDS || NBG >= 3, "LDS-DMA B ring of at least three buffers");
    static_assert(!FLG || (GLDS && !STAMPS), "counter hand-offs: LDS-DMA variant, no stamps");
    const uint32_t oD = NBUF * szB;                   // dense images follow the B buffers
    constexpr uint32_t NAW = kMfmaWaves - WCT - (GLDS ? GLDS : kMfmaBWaves);  // entry waves
    // FLG counters (in the launch's 1 KB tail slack): [0] B chunks full x BWV, [1] images full
    // x NAW, [2] chunks consumed x WC
    uint32_t *flg = reinterpret_cast<uint32_t *>(lds + oD + NDI * ((RMAX + 1) * (2u * KC + 32u)) + 768u);
    auto flg_wait = [&](uint32_t idx, uint32_t target) {
        if constexpr (FLG) {
            while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flg + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
                   target)
                __builtin_amdgcn_s_sleep(1);
            __asm__ volatile("" ::: "memory");
        }
    };
    auto flg_arrive = [&](uint32_t idx) {
        if constexpr (FLG) {
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if ((threadIdx.x & 63u) == 0u) __hip_atomic_fetch_add(flg + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __asm__ volatile("" ::: "memory");
        }
    };
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t role = wv < WC ? 0u : (wv < WC + BWV ? 1u : 2u);  // wave-uniform
    const uint32_t bt = tid - 64 * WC;                // B thread index (role 1)
    const uint32_t at = tid - 64 * (WC + BWV);         // entry thread index (role 2)
    // K-split: workgroup (g, sp) takes chunks [j0, j0 + ncl) of BMTB g
    const uint32_t g = blockIdx.x / nsplit, sp = blockIdx.x % nsplit;
    const uint32_t j0 = sp * ncs, ncl = min(nc, j0 + ncs) - j0;
    const uint32_t r0 = bmtb_first_row[g], R = bmtb_first_row[g + 1] - r0;
    const u32x4 zero4 = {0u, 0u, 0u, 0u};
    // this BMTB's segment starts, lane t holding chunk t's (nc <= 63, host-checked);
    // GS_SEG takes a local chunk index
    const uint32_t segv = seg_start[g * nc + min(lane, nc)];
#define GS_SEG(j) __builtin_amdgcn_readlane(segv, j0 + (j))
    // chunk order: period j works on chunk jr(j); with krot every workgroup starts at its
    // own chunk (g mod ncl) and wraps, so the 256 workgroups are not all pulling the same
    // B rows from the same L2 channels at once (wave-uniform; the k order of a row block's
    // partial sums changes, the result stays deterministic per plan)
    const uint32_t rot = krot ? g % ncl : 0u;
    auto jr = [&](uint32_t j) -> uint32_t { const uint32_t x = j + rot; return x >= ncl ? x - ncl : x; };
    uint64_t *lst = reinterpret_cast<uint64_t *>(lds + oD + NDI * szD);  // STAMPS only
    // first lane of each role -> slots [21*role, 21*role + 21): 0 start, 1 chunk 0 staged,
    // 2+2j chunk j's work done, 3+2j after its barrier (j < 9); slot 63 end
#define GS_STAMP(i)                                                                               \
    if constexpr (STAMPS) {                                                                       \
        if ((tid == 0 || tid == 64 * WC || tid == 64 * (WC + BWV)) && (i) < 21u)                  \
            lst[(i) + 21u * role] = __builtin_amdgcn_s_memtime();                                 \
    }
    GS_STAMP(0u);

    for (uint32_t u = tid; u < NDI * szD / 16u; u += NT) *reinterpret_cast<u32x4 *>(lds + oD + u * 16u) = zero4;
    if constexpr (FLG) {
        if (tid < 4u) flg[tid] = 0u;
    }

    if (role == 0) {
        // ---------------------------------------------------------------- compute
        f4v acc[RT][CT];
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
        uint32_t arow[RT];
#pragma unroll
        for (int rt = 0; rt < RT; rt++) {
            const uint32_t row = 16u * rt + (lane & 15u);
            arow[rt] = (row < R ? row : R) * RS;
        }
        __syncthreads();  // dense images cleared
        GS_STAMP(1u);
        __syncthreads();  // chunk 0 staged
        for (uint32_t j = 0; j < ncl; j++) {
            flg_wait(0, BWV * j);  // chunk j's B rows landed (FLG)
            flg_wait(1, NAW * j);  // ... and its dense image scattered
            const uint32_t kr = min(KC, K - (j0 + jr(j)) * KC);
            const uint32_t nsteps = (kr + 31u) / 32u;
            const unsigned char *la = lds + oD + (j % NDI) * szD;
            const unsigned char *lb = lds + (j % NBUF) * szB;
            // all of this wave's k-steps of the chunk: every fragment read issued
            // before the first MFMA (steps past the chunk's end read step 0 and
            // multiply a zeroed A fragment: no branch around the reads)
            h8v av[MAXS][RT], bv[MAXS][CT];
#pragma unroll
            for (int q = 0; q < MAXS; q++) {
                const uint32_t st = wv + q * WC;
                const uint32_t kb = (st < nsteps ? st : 0u) * 32u + 8u * (lane >> 4);
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
                    av[q][rt] = (DBG & 4) ? h8v{} : *reinterpret_cast<const h8v *>(la + arow[rt] + kb * 2u);
#pragma unroll
                for (int ct = 0; ct < CT; ct++) {
                    s4v t[2];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint32_t k = kb + 4u * h + ((lane & 15u) >> 2);
                        t[h] = (DBG & 4) ? s4v{} : __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s4v *)(lb + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                    }
                    __builtin_memcpy(&bv[q][ct], t, 16);
                }
            }
#pragma unroll
            for (int q = 0; q < MAXS; q++) {
                const bool live = wv + q * WC < nsteps;
#pragma unroll
                for (int rt = 0; rt < RT; rt++) {
                    const h8v a = live ? av[q][rt] : h8v{};
#pragma unroll
                    for (int ct = 0; ct < CT; ct++)
                        acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bv[q][ct], acc[rt][ct], 0, 0, 0);
                }
            }
            if constexpr (GLDS) {
                // image j%2 holds chunk j+2 next: clear the k-step columns this wave read
                // (its MFMAs consumed the reads; no other wave reads these columns)
                if (j + 2 < ncl && !(DBG & 4)) {
                    unsigned char *dj = lds + oD + (j & 1u) * szD;
#pragma unroll
                    for (int q = 0; q < MAXS; q++) {
                        const uint32_t st = wv + q * WC;
                        if (st < nsteps)
                            for (uint32_t u = lane; u < R * 4u; u += 64u)
                                *reinterpret_cast<u32x4 *>(dj + (u >> 2) * RS + st * 64u + (u & 3u) * 16u) = zero4;
                    }
                }
            } else if (j + 2 < ncl) {
                for (uint32_t u = tid; u < R * RS / 16u; u += 64u * WC)
                    *reinterpret_cast<u32x4 *>(lds + oD + ((j + 2) % 3u) * szD + u * 16u) = zero4;
            }
            GS_STAMP(2u + 2u * j);
            if constexpr (FLG) flg_arrive(2);  // reads and clears of chunk j done
            else __syncthreads();
            GS_STAMP(3u + 2u * j);
        }
        // partial tiles -> LDS for the fixed-order reduction below
        __syncthreads();
        float *red = reinterpret_cast<float *>(lds);
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++)
                *reinterpret_cast<f4v *>(red + (((wv * RT + rt) * CT + ct) * 64u + lane) * 4u) = acc[rt][ct];
    } else if (role == 1 && GLDS) {
        // ---------------------------------------------------------------- B rows, LDS-DMA
        // global_load_lds_dwordx4: no VGPR round trip, no ds_write transfer cycles.
        // Wave-instruction i of B wave bw fills the 1 KB at unit (bw*NB + i)*64 (the
        // destination is lane-linear); b_piece's permutation rides on the source address
        // (an XOR with a per-row constant: its own inverse).  Period j issues chunk j+2
        // into the buffer period j-1 finished reading and retires chunk j+1 with a
        // counted vmcnt before a raw s_barrier (__syncthreads would drain to vmcnt(0)).
        const uint32_t bw = wv - WC;
        auto issue = [&](uint32_t jl) {
            const uint32_t kc0 = (j0 + jr(jl)) * KC;
#pragma unroll
            for (uint32_t i = 0; i < NB; i++) {
                const uint32_t u0 = (bw * NB + i) * 64u, u = u0 + lane;
                const uint32_t k = u / UB, s = u % UB;
                const uint32_t kk = kc0 + k < K ? kc0 + k : kc0;
                // N < 16*CT (N = 8): the tile's columns past N copy column 0; their outputs are not stored
                const uint32_t cu = (b_piece<CT>(k, s >> 1) * 2u + (s & 1u)) * 8u;
                const f16 *src = B + (size_t)kk * N + (cu < N ? cu : 0u);
                __builtin_amdgcn_global_load_lds(
                    (const void *)src, (__attribute__((address_space(3))) void *)(lds + (jl % NBUF) * szB + u0 * 16u),
                    16, 0, 0);
            }
        };
        for (uint32_t jl = 0; jl + 1 < NBUF && jl < ncl; jl++)
            if (!(DBG & 1)) issue(jl);
        __syncthreads();  // dense images cleared (its vmcnt(0) retires the first chunks)
        GS_STAMP(1u);
        __syncthreads();  // chunk 0 staged
        for (uint32_t j = 0; j < ncl; j++) {
            flg_wait(2, WC * j);  // chunk j-1 consumed: its buffer takes chunk j+NBUF-1 (FLG)
            if (j + NBUF - 1 < ncl) {
                if (!(DBG & 1)) issue(j + NBUF - 1);
                // chunk j+1 retired, chunks j+2 .. j+NBUF-1 left in flight
                // (vmcnt holds at most 63: a larger count waits for more than chunk j+1)
                __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * NB < 63u ? (NBUF - 2) * NB : 63u) : "memory");
            } else {
                // tail: chunks j+2 .. ncl-1 are in flight
                const uint32_t left = ncl > j + 2 ? ncl - j - 2 : 0u;
                if constexpr (NBUF >= 5) {
                    if (left >= 3) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NB < 63u ? 3 * NB : 63u) : "memory");
                    else if (left == 2) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NB < 63u ? 2 * NB : 63u) : "memory");
                    else if (left == 1) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NB < 63u ? NB : 63u) : "memory");
                    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                } else if constexpr (NBUF == 4) {
                    if (left >= 2) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NB < 63u ? 2 * NB : 63u) : "memory");
                    else if (left == 1) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NB < 63u ? NB : 63u) : "memory");
                    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                } else {
                    if (left >= 1) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NB < 63u ? NB : 63u) : "memory");
                    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            GS_STAMP(2u + 2u * j);
            if constexpr (FLG) flg_arrive(0);  // chunk j+1 landed
            else __builtin_amdgcn_s_barrier();
            GS_STAMP(3u + 2u * j);
        }
        __syncthreads();
    } else if (role == 1) {
        // ---------------------------------------------------------------- B rows
        u32x4 s0[NB], s1[NB], s2[NB];
#define GS_BLOAD(j, S)                                                                              \
    {                                                                                             \
        const uint32_t kc0_ = (j0 + jr(min((uint32_t)(j), ncl - 1u))) * KC;                      \
        _Pragma("unroll") for (uint32_t i = 0; i < NB; i++) {                                     \
            const uint32_t u = bt + i * NBT;                                                      \
            const uint32_t k = u / UB;                                                            \
            const uint32_t kk = kc0_ + k < K ? kc0_ + k : kc0_;                                   \
            S[i] = *reinterpret_cast<const u32x4 *>(B + (size_t)kk * N + ((u % UB) * 8u < N ? (u % UB) * 8u : 0u)); \
        }                                                                                         \
    }
#define GS_BSTORE_UNIT(jb, S, i)                                                                    \
    {                                                                                             \
        const uint32_t u = bt + (i) * NBT;                                                        \
        const uint32_t k = u / UB, s = u % UB;                                                    \
        *reinterpret_cast<u32x4 *>(lds + ((jb) & 1u) * szB + k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u) = S[i]; \
    }
        // chunk j: fetch j+3 into set j%3 next to staging j+1 from set (j+1)%3 (the
        // store is unconditional: B[(nc)&1] is free at the last chunk)
#define GS_BITER(j, Sn, Ss)                                                                         \
    {                                                                                             \
        const uint32_t kc0_ = (j0 + jr(min((uint32_t)(j) + 3u, ncl - 1u))) * KC;                 \
        _Pragma("unroll") for (uint32_t i = 0; i < NB; i++) {                                     \
            const uint32_t u = bt + i * NBT;                                                      \
            const uint32_t k = u / UB;                                                            \
            const uint32_t kk = kc0_ + k < K ? kc0_ + k : kc0_;                                   \
            Sn[i] = *reinterpret_cast<const u32x4 *>(B + (size_t)kk * N + ((u % UB) * 8u < N ? (u % UB) * 8u : 0u)); \
            GS_BSTORE_UNIT((j) + 1u, Ss, i);                                                      \
        }                                                                                         \
        GS_STAMP(2u + 2u * (j));                                                                  \
        __syncthreads();                                                                          \
        GS_STAMP(3u + 2u * (j));                                                                  \
    }
        GS_BLOAD(0u, s0);
        GS_BLOAD(1u, s1);
        GS_BLOAD(2u, s2);
        __syncthreads();  // dense images cleared
#pragma unroll
        for (uint32_t i = 0; i < NB; i++) GS_BSTORE_UNIT(0u, s0, i);
        GS_STAMP(1u);
        __syncthreads();  // chunk 0 staged
        uint32_t j = 0;
        for (; j + 2 < ncl; j += 3) {
            GS_BITER(j, s0, s1);
            GS_BITER(j + 1, s1, s2);
            GS_BITER(j + 2, s2, s0);
        }
        if (j < ncl) GS_BITER(j, s0, s1);
        if (j + 1 < ncl) GS_BITER(j + 1, s1, s2);
#undef GS_BITER
#undef GS_BSTORE_UNIT
#undef GS_BLOAD
        __syncthreads();
    } else {
        // ---------------------------------------------------------------- entries
        u32x4 p0[MAXA], v0[MAXA], p1[MAXA], v1[MAXA], p2[MAXA], v2[MAXA], p3[MAXA], v3[MAXA];
#define GS_ALOAD(j, P, V)                                                                           \
    {                                                                                             \
        const uint32_t jj_ = jr(min((uint32_t)(j), ncl - 1u));                                    \
        const uint32_t s0_ = GS_SEG(jj_);                                                         \
        const uint32_t G_ = (uint32_t)(j) < ncl ? GS_SEG(jj_ + 1) - s0_ : 0u;                     \
        _Pragma("unroll") for (int I = 0; I < MAXA; I++) {                                        \
            const uint32_t q = at + I * NAT;                                                      \
            const size_t qq = (size_t)s0_ + (q < G_ ? q : 0u);                                    \
            P[I] = tP[qq];                                                                        \
            V[I] = tV[qq];                                                                        \
        }                                                                                         \
    }
#define GS_SCATTER(j, P, V)                                                                         \
    {                                                                                             \
        const uint32_t G_ = GS_SEG(jr(j) + 1) - GS_SEG(jr(j));                                    \
        unsigned char *ld_ = lds + oD + ((j) % NDI) * szD;                                        \
        _Pragma("unroll") for (int I = 0; I < MAXA; I++) {                                        \
            const uint32_t q = at + I * NAT;                                                      \
            if (q < G_) {                                                                         \
                _Pragma("unroll") for (int e = 0; e < 8; e++) {                                   \
                    const uint32_t h = (P[I][e >> 1] >> (16 * (e & 1))) & 0xffffu;                \
                    const uint16_t v = (uint16_t)((V[I][e >> 1] >> (16 * (e & 1))) & 0xffffu);    \
                    *reinterpret_cast<uint16_t *>(ld_ + h * 2u) = v;                              \
                }                                                                                 \
            }                                                                                     \
        }                                                                                         \
    }
        // chunk j: fetch j+4 into set j%4, scatter j+1 from set (j+1)%4
#define GS_AITER(j, Pn, Vn, Ps, Vs)                                                                 \
    {                                                                                             \
        if (!(DBG & 8)) GS_ALOAD((j) + 4, Pn, Vn);                                                \
        GS_STAMP(2u + 2u * (j)); /* entry role: loads issued, then scatter done */                \
        flg_wait(2, WC * (uint32_t)(j)); /* FLG: chunk j-1 consumed, its image cleared */         \
        if ((j) + 1 < ncl && !(DBG & 2)) GS_SCATTER((j) + 1, Ps, Vs);                             \
        GS_STAMP(3u + 2u * (j));                                                                  \
        if constexpr (FLG) flg_arrive(1);                                                         \
        else __syncthreads();                                                                     \
    }
        GS_ALOAD(0u, p0, v0);
        GS_ALOAD(1u, p1, v1);
        GS_ALOAD(2u, p2, v2);
        GS_ALOAD(3u, p3, v3);
        __syncthreads();  // dense images cleared
        GS_SCATTER(0u, p0, v0);
        GS_STAMP(1u);
        __syncthreads();  // chunk 0 staged
        uint32_t j = 0;
        for (; j + 3 < ncl; j += 4) {
            GS_AITER(j, p0, v0, p1, v1);
            GS_AITER(j + 1, p1, v1, p2, v2);
            GS_AITER(j + 2, p2, v2, p3, v3);
            GS_AITER(j + 3, p3, v3, p0, v0);
        }
        if (j < ncl) GS_AITER(j, p0, v0, p1, v1);
        if (j + 1 < ncl) GS_AITER(j + 1, p1, v1, p2, v2);
        if (j + 2 < ncl) GS_AITER(j + 2, p2, v2, p3, v3);
#undef GS_AITER
#undef GS_SCATTER
#undef GS_ALOAD
        __syncthreads();
    }
#undef GS_SEG
    __syncthreads();
    // fixed-order reduction of the compute waves' partial tiles (all threads)
    const float *red = reinterpret_cast<const float *>(lds);
    auto tile_sum = [&](uint32_t e, uint32_t &row, uint32_t &colx) {
        const uint32_t cc = e & 15u, rr = (e >> 4) & 15u, tt = e >> 8;
        const uint32_t rt = tt / CT, ct = tt % CT;
        const uint32_t ln = 16u * (rr >> 2) + cc, i = rr & 3u;
        float sum = 0.f;
#pragma unroll
        for (uint32_t w = 0; w < WC; w++) sum += red[(((w * RT + rt) * CT + ct) * 64u + ln) * 4u + i];
        row = 16u * rt + rr;
        colx = 16u * ct + cc;
        return sum;
    };
    if (nsplit == 1) {
        for (uint32_t e = tid; e < RT * CT * 256u; e += NT) {
            uint32_t row, colx;
            const float sum = tile_sum(e, row, colx);
            if (row < R && colx < N) C[(size_t)(row_base + r0 + row) * N + colx] = (f16)sum;
        }
    } else {
        // K-split: this workgroup's fp32 slab, then the last of the row block's
        // nsplit workgroups sums the slabs in split order (deterministic) and stores C.
        // Slabs and the arrival counter use agent-scope relaxed atomics: the stores and
        // loads themselves are device-coherent (no L2 write-back / invalidate fences
        // across the XCDs); the stores are complete (vmcnt 0) before the counter moves,
        // and the combining workgroup loads only after it has seen the count.
        float *slab = slabs + ((size_t)g * nsplit + sp) * RMAX * N;
        for (uint32_t e = tid; e < RT * CT * 256u; e += NT) {
            uint32_t row, colx;
            const float sum = tile_sum(e, row, colx);
            if (row < R && colx < N)
                __hip_atomic_store(slab + (size_t)row * N + colx, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        uint32_t *flag = reinterpret_cast<uint32_t *>(lds + oD + NDI * szD + 512);
        if (tid == 0)
            *flag = __hip_atomic_fetch_add(&arrivals[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (*flag == nsplit - 1u) {
            if (tid == 0) __hip_atomic_store(&arrivals[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float *base = slabs + (size_t)g * nsplit * RMAX * N;
            for (uint32_t e = tid; e < R * N; e += NT) {
                float sum = 0.f;
                for (uint32_t q = 0; q < nsplit; q++)
                    sum += __hip_atomic_load(base + (size_t)q * RMAX * N + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                C[(size_t)(row_base + r0) * N + e] = (f16)sum;
            }
        }
    }
    if constexpr (STAMPS) {
        __syncthreads();
        if (tid == 0) {
            lst[63] = __builtin_amdgcn_s_memtime();
            for (uint32_t i = 0; i < 64; i++) stamps[(size_t)blockIdx.x * 64 + i] = lst[i];
        }
    }
#undef GS_STAMP
}

// ---------------------------------------------------------------------------
// k_mfma_ks -- BMTB row blocks on the matrix cores with K split over S workgroups
// and every wave running on its own (the default matrix-core kernel for row blocks of
// >= 40 rows).
// Why: a workgroup that owns a row block over all of K streams all of B (327 KB on C2)
// for its ~120 KB of A; one CU takes in ~50-70 GB/s, so B, not A, set the time
// (scripts/probes/probe_floor.hip: loading A + B alone takes 10.9 us at S = 1, 7.2 us at
// S = 4).  Here workgroup (g, q) owns row block g over the K range [q*KR, q*KR + KR) and
// reads only that slice of B (KR rows).
// Wave w owns the range's 32-column k-steps w, w+W, ... and runs them with no
// workgroup barrier until the end: per k-step it loads (D steps ahead, into registers)
// the step's 32 B rows and its entries (upload layout: the step's groups back to back,
// each 8 x [u16 halfword position in the wave's dense image] + 8 x [f16 value], found by
// the step's {first group, group count} record, loaded D steps ahead of the groups;
// padding inside a group writes 0 into the image's zero row; NT: the groups by non-temporal
// loads when NTL & 1 (KS_NT; B's rows when NTL & 2, not instantiated: slower), stores the B rows into its private stage (32-B pieces
// permuted by b_piece so the ds_read_b64_tr_b16 fragment reads are conflict-free),
// scatters the entries into its private image of 16*RT+1 rows x 96 B (conflict-free
// ds_read_b128), reads the RT A fragments and the CT B fragments, writes zeros back at
// the entries' positions, and runs RT x CT v_mfma_f32_16x16x32_f16 into fp32
// accumulators.  Every step issues the same loads (steps past the wave's last read the
// first B rows and the spare group: one cached line each), so the compiler's waits
// stay counted ones.  At the end the W partial tiles are summed through LDS in wave
// order; with S > 1 each workgroup publishes its fp32 slab (16-B sc1 write-through
// stores, drained by every storing wave, then one arrival add), and the last of the row
// block's S workgroups sums the S slabs in q order (deterministic, whichever arrives
// last) and writes C: the hand-off form of MI355X_MICROARCH.md §Workgroup dispatch,
// table row 1 (sc1 stores + vmcnt(0) + barrier + one agent add; the last adder, told by
// the returned value, loads with sc1 loads after a barrier).  Workgroup order: unit
// u = g*S + q, XCD-contiguous (xcd_block), so a row block's S workgroups are normally on
// one XCD (speed only).  Rows of B past K are stored as zeros; a zero of the dense tile
// times a non-finite in-range B value gives NaN for the row block (DESIGN.md deviation,
// as for k_mfma_rows).
// ---------------------------------------------------------------------------
// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt <= N only (expcnt / lgkmcnt at their maxima)
template <int N>
__device__ constexpr int vmcnt_imm() {
    static_assert(N >= 0 && N < 64, "vmcnt is six bits");
    return (N & 0xF) | ((N >> 4) << 14) | 0x70 | 0xF00;
}

// kKsStride, ks_image_bytes, ks_lds_bytes: kernel_consts.hpp
// 8 bytes at a 2-byte-aligned address (k_mfma_kb / k_mfma_bm value windows)
typedef uint32_t u32x2_a2 __attribute__((ext_vector_type(2), aligned(2)));

// K-split combine: the last ticket holder's read of 4 words of another workgroup's slab
// (each word tagged in its low mantissa bit): agent-scope (sc1) loads until every tag reads
// `tag`.  The writer holds an earlier ticket, so it is resident and its stores are issued or
// about to be; the wait is bounded by wall time (s_memrealtime, 100 MHz: 0.2 s) all the same.
// Past the bound the words read as NaN and bit 0 of the plan replica's device error word
// (`err`, the word after the arrival counters) is set: gs_plan_device_status reports it as
// GS_ERR_DEVICE, so a lost slab is an error at the C ABI, not silent NaNs in C.  `force`
// (experiments build, KS_FORCE_TIMEOUT) takes the timeout path at once (the test of that chain).
__device__ __forceinline__ u32x4 ks_slab_wait(const uint32_t *src, uint32_t tag, uint32_t *err, bool force) {
    u32x4 w;
    auto load4 = [&]() {
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto stale = [&]() { return (((w[0] ^ tag) | (w[1] ^ tag) | (w[2] ^ tag) | (w[3] ^ tag)) & 1u) != 0u; };
    bool lost = force;
    if (!lost) {
        load4();
        if (stale()) {
            // the bound needs 0.2 s of wall time AND 1024 polls since the last gap: a gap of
            // over 1 ms between two polls means this wave was switched out (CWSR time slicing),
            // so the bound restarts rather than counting the time the writer could not run
            uint64_t t0 = __builtin_amdgcn_s_memrealtime(), prev = t0;
            uint32_t polls = 0;
            do {
                const uint64_t t = __builtin_amdgcn_s_memrealtime();
                if (t - prev > 100000ull) {
                    t0 = t;
                    polls = 0;
                }
                prev = t;
                if (t - t0 > 20000000ull && polls >= 1024u) {
                    lost = true;
                    break;
                }
                polls++;
                __builtin_amdgcn_s_sleep(2);
                load4();
            } while (stale());
        }
    }
    if (lost) {
        w = u32x4{0x7fc00000u | tag, 0x7fc00000u | tag, 0x7fc00000u | tag, 0x7fc00000u | tag};
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return w;
}
#ifdef GS_EXPERIMENTS
#define GS_KS_FORCE(prio) (((prio) & 16u) != 0u)
#else
#define GS_KS_FORCE(prio) false
#endif

// STAMPS (diagnostic build only, gs_debug_mfma_timeline): lane 0 of every wave records
// s_memtime into stamps[(workgroup * W + wave) * 32 + slot]: 0 start, 1 loads issued,
// 3 + i after step i (i < 16), 20 loop done, 21 reduced, 22 end
// the body of k_mfma_ks for workgroup bx of a launch of nwg workgroups (k_mfma_ks: the
// whole grid; k_mfma_ks_group: one entry's share of it)
// P8 (KS_POS8, device_layout.cc pos8_step): tP holds 8 bytes per group -- byte e = bit e of the
// group's 8 x 16 segment id in bit 7, the entry's (row % 8) << 4 | column % 16 below; the image
// halfword of a segment sg's entry is 384 * (sg >> 1) + 16 * (sg & 1) + 48 * (b >> 4) + (b & 15)
template <int CT, int RT, int W, int D, int MAXG, bool STAMPS, bool AP = true, bool P8 = false, int NTL = 0>
__device__ __forceinline__ void ks_body(const uint32_t *__restrict__ bmtb_first_row, const u32x4 *__restrict__ tP,
                                        const u32x4 *__restrict__ tV, const u32x2 *__restrict__ steps,
                                        const f16 *__restrict__ B, f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                        uint32_t NS, uint32_t nwg, uint32_t row_base, float *__restrict__ slabs,
                                        uint32_t *__restrict__ arrivals, uint64_t *__restrict__ stamps, uint32_t bx,
                                        uint32_t prio) {
    constexpr uint32_t RB = 32 * CT;  // bytes per LDS B row (a 16*CT-column tile)
    constexpr uint32_t UB = 2 * CT;   // 16-B units per B row
    constexpr uint32_t IMG = ks_image_bytes<RT>();
    constexpr uint32_t STG = 32u * RB;  // one k-step of B rows
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t u = xcd_block(bx, nwg);
    const uint32_t g = u / S, q = u - g * S;
#define GS_KS_STAMP(slot)                                                                          \
    if constexpr (STAMPS) {                                                                        \
        if (lane == 0) stamps[((size_t)blockIdx.x * W + wv) * 32u + (slot)] = __builtin_amdgcn_s_memtime(); \
    }
    GS_KS_STAMP(0u);
    const uint32_t k0 = q * NS * 32u;
    // column tile blockIdx.y: columns [col0, col0 + nv) of B and C (N > 16*CT: several
    // tiles; N = 8: one partial tile)
    const uint32_t col0 = blockIdx.y * 16u * CT, nv = min(16u * CT, N - col0);
    unsigned char *img = lds + wv * (IMG + STG);
    unsigned char *bst = img + IMG;
    const u32x4 zero4 = {0u, 0u, 0u, 0u};

    // ---- this wave's k-steps w, w+W, ...: step s of unit u is record steps[u*NS + s] =
    // {first group, group count}; a slot's next record is loaded one round (D steps) before
    // its groups, so the groups' addresses wait on a load issued a round earlier
    const uint32_t nsw = NS > wv ? (NS - wv + W - 1u) / W : 0u;
    const size_t ubase = (size_t)u * NS;
    using PV = typename std::conditional<P8, u32x2, u32x4>::type;
    const PV *tPp = reinterpret_cast<const PV *>(tP);
    PV P[D][MAXG];
    u32x4 V[D][MAXG], BR[D][CT];
    u32x2 NX[D];      // per slot: record of the step the slot loads next
    uint32_t CN[D];   // per slot: group count of the step whose groups it holds
    // the record is read by a vector load (vmcnt, in order with the groups): a scalar load
    // would share lgkmcnt with the LDS traffic, and every step's lgkmcnt(0) before its
    // fragments would then wait for the newest record as well (80% sparsity: +3-9%)
    uint32_t vz;
    __asm__ volatile("v_mov_b32 %0, 0" : "=v"(vz));
    auto rec_of = [&](uint32_t i) -> u32x2 {
        const uint32_t st = __builtin_amdgcn_readfirstlane(i < nsw ? wv + i * W : 0u);
        return steps[ubase + st + vz];
    };
    // steps past the wave's last re-read the unit's first step (cached; the same lane-varying
    // load form as a live step, so no path of the loop issues a different count).  The B rows
    // of a step need no record: they are issued apart from (and, in the prologue, before) the
    // groups, whose addresses wait for the step's record
    auto load_b = [&](uint32_t i, u32x4 (&B_)[CT]) {
        const uint32_t st = __builtin_amdgcn_readfirstlane(i < nsw ? wv + i * W : 0u);
        const uint32_t kr = k0 + st * 32u;  // first B row of the step
#pragma unroll
        for (int c = 0; c < CT; c++) {
            const uint32_t un = lane + 64u * c;  // 16-B unit of the step's 32 rows
            const uint32_t k = kr + un / UB, cu = (un % UB) * 8u;
            // columns past N (a partial column tile: N = 8, 24, ...) read column 0 and are
            // stored as zeros below
            B_[c] = ld_once_if<(NTL & 2) != 0>(
                reinterpret_cast<const u32x4 *>(B + (size_t)(k < K ? k : K - 1u) * N + col0 + (cu < nv ? cu : 0u)));
        }
    };
    // the groups of step i (b0: first group, gc: count), then the record of step i + D
    auto load_g_at = [&](uint32_t i, uint32_t b0, uint32_t gc, u32x2 &NX_, uint32_t &CN_, PV (&P_)[MAXG],
                         u32x4 (&V_)[MAXG]) {
        CN_ = gc;
        NX_ = rec_of(i + D);
#pragma unroll
        for (int j = 0; j < MAXG; j++) {
            const uint32_t qg = lane + 64u * j;
            const size_t at = (size_t)b0 + (qg < gc ? qg : 0u);
            P_[j] = ld_once_if<(NTL & 1) != 0>(tPp + at);
            V_[j] = ld_once_if<(NTL & 1) != 0>(tV + at);
        }
    };
    auto load_g = [&](uint32_t i, u32x2 &NX_, uint32_t &CN_, PV (&P_)[MAXG], u32x4 (&V_)[MAXG]) {
        load_g_at(i, __builtin_amdgcn_readfirstlane(NX_[0]), __builtin_amdgcn_readfirstlane(NX_[1]), NX_, CN_, P_, V_);
    };
    // head steps (device_layout.cc ks_tiles::GH, prio bits 8..17): the first D steps of every wave
    // sit at (unit * min(W * D, NS) + step) * GH, padded with zero-row groups, so the prologue issues their
    // groups with the B rows at once instead of a record round trip later
    const uint32_t GH = (prio >> 8) & 0x3ffu;
    if (GH) {
#pragma unroll
        for (int d = 0; d < D; d++) load_b((uint32_t)d, BR[d]);
#pragma unroll
        for (int d = 0; d < D; d++) {
            const uint32_t st = (uint32_t)d < nsw ? wv + (uint32_t)d * W : 0u;
            load_g_at((uint32_t)d, (u * min((uint32_t)(W * D), NS) + st) * GH, GH, NX[d], CN[d], P[d], V[d]);
        }
        for (uint32_t x = lane; x < IMG / 16u; x += 64u) *reinterpret_cast<u32x4 *>(img + x * 16u) = zero4;
    } else {
#pragma unroll
        for (int d = 0; d < D; d++) NX[d] = rec_of((uint32_t)d);
#pragma unroll
        for (int d = 0; d < D; d++) load_b((uint32_t)d, BR[d]);
        for (uint32_t x = lane; x < IMG / 16u; x += 64u) *reinterpret_cast<u32x4 *>(img + x * 16u) = zero4;
#pragma unroll
        for (int d = 0; d < D; d++) load_g((uint32_t)d, NX[d], CN[d], P[d], V[d]);
    }
    GS_KS_STAMP(1u);

    f4v acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    uint32_t arow[RT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++) arow[rt] = (16u * rt + (lane & 15u)) * kKsStride + 16u * (lane >> 4);

    // step i on its set, then the set is reloaded with step i + D (issued whether or not
    // step i exists: every loop iteration issues the same loads)
    // image halfword of entry e of a group (u16 position, or P8's segment + 7-bit position)
    auto ent_h = [&](const PV &p, uint32_t hb, int e) -> uint32_t {
        if constexpr (P8) {
            const uint32_t b = (p[e >> 2] >> (8 * (e & 3))) & 0x7fu;
            return hb + 48u * (b >> 4) + (b & 15u);
        } else {
            return (p[e >> 1] >> (16 * (e & 1))) & 0xffffu;
        }
    };
    auto grp_hb = [&](const PV &p) -> uint32_t {
        if constexpr (P8) {
            const uint32_t x = p[0], y = p[1];
            const uint32_t sg = ((x >> 7) & 1u) | ((x >> 14) & 2u) | ((x >> 21) & 4u) | ((x >> 28) & 8u) | ((y >> 3) & 16u);
            return 384u * (sg >> 1) + 16u * (sg & 1u);
        } else {
            return 0u;
        }
    };
    auto step = [&](uint32_t i, u32x2 &NX_, uint32_t &CN_, PV (&P_)[MAXG], u32x4 (&V_)[MAXG], u32x4 (&B_)[CT]) {
        const bool live = i < nsw;  // wave-uniform
        const uint32_t gc = CN_;
        h8v av[RT], bv[CT];
        if (live) {
            const uint32_t kr = k0 + (wv + i * W) * 32u;
            // the step's B rows into the stage (rows past K as zeros)
#pragma unroll
            for (int c = 0; c < CT; c++) {
                const uint32_t un = lane + 64u * c, k = un / UB, s = un % UB;
                *reinterpret_cast<u32x4 *>(bst + k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u) =
                    kr + k < K && s * 8u < nv ? B_[c] : zero4;
            }
            // scatter the step's entries into the image
#pragma unroll
            for (int j = 0; j < MAXG; j++) {
                if (lane + 64u * j < gc) {
                    const uint32_t hb = grp_hb(P_[j]);
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const uint32_t h = ent_h(P_[j], hb, e);
                        const uint16_t v = (uint16_t)((V_[j][e >> 1] >> (16 * (e & 1))) & 0xffffu);
                        *reinterpret_cast<uint16_t *>(img + h * 2u) = v;
                    }
                }
            }
            // fragments (LDS runs a wave's operations in order: the reads see the stores)
#pragma unroll
            for (int rt = 0; rt < RT; rt++) av[rt] = *reinterpret_cast<const h8v *>(img + arow[rt]);
            const uint32_t kb = 8u * (lane >> 4);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                s4v t[2];
#pragma unroll
                for (int hh = 0; hh < 2; hh++) {
                    const uint32_t k = kb + 4u * hh + ((lane & 15u) >> 2);
                    t[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s4v *)(bst + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                }
                __builtin_memcpy(&bv[ct], t, 16);
            }
            // the image back to zero at the entries' positions
#pragma unroll
            for (int j = 0; j < MAXG; j++) {
                if (lane + 64u * j < gc) {
                    const uint32_t hb = grp_hb(P_[j]);
#pragma unroll
                    for (int e = 0; e < 8; e++) *reinterpret_cast<uint16_t *>(img + ent_h(P_[j], hb, e) * 2u) = (uint16_t)0;
                }
            }
        }
        load_b(i + D, B_);
        load_g(i + D, NX_, CN_, P_, V_);
        if (live) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++)
                    acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[rt], bv[ct], acc[rt][ct], 0, 0, 0);
            if (i < 16u) GS_KS_STAMP(3u + i);
        }
    };
    // prio (KS_PRIO): the younger half of the waves (the second wave of each SIMD, the one
    // that loses issue arbitration) at s_setprio 1 -- prio & 3 = 1: for its whole loop, 2: for the
    // first half of its steps
    const bool young = wv >= W / 2u;
    if ((prio & 3u) && young) __builtin_amdgcn_s_setprio(1);
    for (uint32_t i0 = 0; i0 < nsw; i0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) step(i0 + d, NX[d], CN[d], P[d], V[d], BR[d]);
        if ((prio & 3u) == 2u && young && i0 + D >= nsw / 2u && i0 < nsw / 2u) __builtin_amdgcn_s_setprio(0);
    }
    if ((prio & 3u) && young) __builtin_amdgcn_s_setprio(0);
    GS_KS_STAMP(20u);
    // ---- K-split ticket: wave 0 takes its row block's arrival ticket as soon as its own
    // loop ends, so the add's round trip overlaps the partial-tile reduction below
    uint32_t *arr = arrivals + (size_t)g * gridDim.y + blockIdx.y;
    uint32_t ticket = 0;
    if (S > 1 && wv == 0 && lane == 0) ticket = __hip_atomic_fetch_add(arr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- wave partial tiles -> LDS (the trailing loads write registers only), summed in
    // wave order.  Item t = (tile, lane) of a 16x16 tile: the 4 rows 4*(lane/16)+i of
    // column lane%16.  When the W partial tiles fit LDS beside the wave images (APART), each
    // wave stores its tile as soon as its loop ends, without waiting for the others
    constexpr bool APART = ks_red_apart(CT, RT, W, AP);
    f4v *red = reinterpret_cast<f4v *>(lds + (APART ? (size_t)W * (IMG + STG) : 0u));
    constexpr bool HALVES = !APART && ks_red_halves(CT, RT, W);
    constexpr uint32_t WR = HALVES ? W / 2 : W;  // partial tiles summed from LDS
    uint32_t *flag = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(red) + (size_t)WR * RT * CT * 1024u);
    if constexpr (!APART) {
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    }
    if constexpr (HALVES) {
        if (wv >= WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) red[(((wv - WR) * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
        if (wv < WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) acc[rt][ct] += red[((wv * RT + rt) * CT + ct) * 64u + lane];
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    }
    if (wv < WR) {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[((wv * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
    }
    if (S > 1 && wv == 0 && lane == 0) *flag = ticket;  // (waits for the add's return)
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
    constexpr uint32_t NI = RT * CT * 64u, NT = 64u * W;
    const uint32_t r0 = bmtb_first_row[g], R = bmtb_first_row[g + 1] - r0;
    auto item_sum = [&](uint32_t t) {
        f4v sum = red[t];
#pragma unroll
        for (uint32_t w = 1; w < WR; w++) sum += red[w * NI + t];
        return sum;
    };
    auto store_item = [&](uint32_t t, const f4v &v) {
        const uint32_t ln = t & 63u, tt = t >> 6, rt = tt / CT, ct = tt % CT;
        const uint32_t col = 16u * ct + (ln & 15u), rb = 16u * rt + 4u * (ln >> 4);
        if (col >= nv) return;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (rb + i < R) C[(size_t)(row_base + r0 + rb + i) * N + col0 + col] = (f16)v[i];
    };
    GS_KS_STAMP(21u);
    if (S == 1) {
        for (uint32_t t = tid; t < NI; t += NT) store_item(t, item_sum(t));
        GS_KS_STAMP(22u);
        return;
    }
    // ---- K-split combine by tagged slabs.  Every fp32 word of a published slab carries
    // its own validity tag in the low mantissa bit (the reader drops the bit, a 2^-24
    // relative truncation), so no store needs to be drained before a signal: every workgroup
    // stores its slab with 16-B write-through (sc1) stores, and the one that drew the last
    // ticket loads each other slab word with agent-scope (sc1) loads until its tag reads
    // this launch's value -- its writer holds an earlier ticket, so it is running and its
    // stores are issued or about to be -- sums the S partials in q order (deterministic) and
    // writes C.  The tag alternates from launch to launch: the arrival counter holds
    // (epoch << 16) | arrivals, the tag is epoch ^ 1, and the last workgroup re-arms the
    // counter with the epoch flipped and no arrivals.  Every slab word then holds the
    // previous launch's tag when a launch starts (the last workgroup stores its own slab
    // too), and the zero-filled first state reads as "tag 0, epoch 0" -- so no slab is
    // cleared after use ((S - 1) fewer slab stores than clearing, the last workgroup's own
    // store issued before it waits).  Every access to the slabs is sc1 (MI355X_MICROARCH.md
    // Workgroup dispatch, Valid forms: the R2 granule, here one naturally aligned word).
    // The next launch on the stream starts after these stores complete.
    const uint32_t tk = *flag & 0xffffu, tag = ((*flag >> 16) & 1u) ^ 1u;
    f4v *slab = reinterpret_cast<f4v *>(slabs) + ((size_t)u * gridDim.y + blockIdx.y) * NI;
    auto tagged = [&](const f4v &v) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        w[0] = (w[0] & ~1u) | tag; w[1] = (w[1] & ~1u) | tag; w[2] = (w[2] & ~1u) | tag; w[3] = (w[3] & ~1u) | tag;
        return w;
    };
    for (uint32_t t = tid; t < NI; t += NT) {
        const u32x4 w = tagged(item_sum(t));
        __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(slab + t), "v"(w) : "memory");
    }
    if (tk != S - 1u) {
        GS_KS_STAMP(22u);
        return;
    }
    if (tid == 0) __hip_atomic_store(arr, tag << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const f4v *base = reinterpret_cast<const f4v *>(slabs) + blockIdx.y * NI;
    const size_t qstride = (size_t)gridDim.y * NI;  // slab of (g, qq) = base + (g*S + qq) * qstride
    uint32_t *err = arrivals + (size_t)(nwg / S) * gridDim.y;  // the replica's device error word
    for (uint32_t t = tid; t < NI; t += NT) {
        f4v sum = {0.f, 0.f, 0.f, 0.f};
        for (uint32_t qq = 0; qq < S; qq++) {
            u32x4 w;
            if (qq == q) {  // truncated as a published word is (whichever workgroup is last: deterministic)
                w = tagged(item_sum(t));
            } else {
                w = ks_slab_wait(reinterpret_cast<const uint32_t *>(base + ((size_t)g * S + qq) * qstride + t), tag, err,
                                 GS_KS_FORCE(prio));
            }
            w[0] &= ~1u; w[1] &= ~1u; w[2] &= ~1u; w[3] &= ~1u;
            f4v x;
            __builtin_memcpy(&x, &w, 16);
            sum += x;
        }
        store_item(t, sum);
    }
    GS_KS_STAMP(22u);
#undef GS_KS_STAMP
}

template <int CT, int RT, int W, int D, int MAXG, bool STAMPS = false, bool AP = true, bool P8 = false, int NTL = 0>
__global__ __launch_bounds__(64 * W) void k_mfma_ks(const uint32_t *__restrict__ bmtb_first_row,  // nb+1
                                                    const u32x4 *__restrict__ tP,  // 8 x u16 position per group
                                                    const u32x4 *__restrict__ tV,  // 8 x f16 value per group
                                                    const u32x2 *__restrict__ steps,  // per (unit, k-step): first group, count
                                                    const f16 *__restrict__ B, f16 *__restrict__ C, uint32_t K,
                                                    uint32_t N, uint32_t S, uint32_t NS, uint32_t nwg,
                                                    uint32_t row_base, float *__restrict__ slabs,
                                                    uint32_t *__restrict__ arrivals, uint64_t *__restrict__ stamps = nullptr,
                                                    uint32_t prio = 0) {
    // nwg == gridDim.x (an argument: kernarg preload)
    ks_body<CT, RT, W, D, MAXG, STAMPS, AP, P8, NTL>(bmtb_first_row, tP, tV, steps, B, C, K, N, S, NS, nwg, row_base, slabs,
                                                arrivals, stamps, blockIdx.x, prio);
}

#ifdef GS_EXPERIMENTS
// ---------------------------------------------------------------------------
// k_mfma_ks_persist (KS_PERSIST = the grid): a persistent grid over
// the plan's units (row block, K range) -- workgroup b runs unit b, then units pulled from its
// XCD's head (queue[xcc]: unit grid + xcc + 8 n), until the units run out.  The pull for the next
// unit is issued as the current one starts (its round trip overlaps the unit's first loads);
// the units' K-range combine is k_mfma_ks's (tickets + tagged slabs in q order), so C is the
// same bits as the static launch's whichever workgroup runs a unit.  The last workgroup out
// re-arms the nine queue words (8 heads + the exit count).
// ---------------------------------------------------------------------------
template <int CT, int RT, int W, int D, int MAXG, int NTL = 0>
__global__ __launch_bounds__(64 * W) void k_mfma_ks_persist(const uint32_t *__restrict__ bmtb_first_row,
                                                            const u32x4 *__restrict__ tP, const u32x4 *__restrict__ tV,
                                                            const u32x2 *__restrict__ steps, const f16 *__restrict__ B,
                                                            f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                                            uint32_t NS, uint32_t nunits, uint32_t row_base,
                                                            float *__restrict__ slabs, uint32_t *__restrict__ arrivals,
                                                            uint32_t prio, uint32_t *__restrict__ queue) {
    __shared__ uint32_t next_sh;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    xcc &= 7u;
    const uint32_t grid = gridDim.x;
    uint32_t u = blockIdx.x, qx = xcc, tried = 0;
    while (u < nunits) {
        uint32_t pulled = 0;
        if (threadIdx.x == 0) pulled = __hip_atomic_fetch_add(queue + qx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ks_body<CT, RT, W, D, MAXG, false, true, false, NTL>(bmtb_first_row, tP, tV, steps, B, C, K, N, S, NS, nunits,
                                                          row_base, slabs, arrivals, nullptr, u, prio);
        __syncthreads();
        if (threadIdx.x == 0) next_sh = pulled;
        __syncthreads();
        u = grid + qx + 8u * next_sh;
        __syncthreads();
        // this XCD's units are done: take the other heads' in turn (correct whatever the placement)
        while (u >= nunits && ++tried < 8u) {
            qx = (qx + 1u) & 7u;
            if (threadIdx.x == 0) next_sh = __hip_atomic_fetch_add(queue + qx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            u = grid + qx + 8u * next_sh;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0 && __hip_atomic_fetch_add(queue + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == grid - 1u) {
        for (int i = 0; i < 9; i++) __hip_atomic_store(queue + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
#endif  // GS_EXPERIMENTS (k_mfma_ks_persist)

// ---------------------------------------------------------------------------
// k_mfma_ks_group -- several k_mfma_ks launches of one instantiation as one grid (a layer's
// or a batch's SpMMs; gs_spmm_batch): entry i owns workgroups [begin[i], begin[i] + nwg_i) and
// runs them as its own launch would (begin[i] a multiple of 8: the entry's block numbers keep
// the XCD residues xcd_block assumes; the blocks up to begin[i+1] exit at once).  One launch instead of one per matrix: no kernel boundary
// between the matrices, and one matrix's last workgroups overlap the next one's first.  The
// entries are kernel arguments (ks_group_args, read through the kernarg segment with scalar
// loads); every entry has its own plan replica (distinct K-range tickets and slabs).
// ---------------------------------------------------------------------------
struct ks_entry {  // 96 B
    const uint32_t *tbr;
    const u32x4 *tP, *tV;
    const u32x2 *steps;
    const f16 *B;
    f16 *C;
    float *slabs;
    uint32_t *arrivals;
    uint32_t K, S, NS, nwg, row_base, pad0, pad1, pad2;
};
// kKsGroupMax: kernel_consts.hpp
struct ks_group_args {
    uint32_t begin[kKsGroupMax + 1];  // first workgroup of each entry (+ the total)
    uint32_t n, N, pad[2];  // pad[0]: k_mfma_ks's prio
    ks_entry e[kKsGroupMax];
};

template <int CT, int RT, int W, int D, int MAXG, bool P8 = false, bool AP = true, int NTL = 0>
__global__ __launch_bounds__(64 * W) void k_mfma_ks_group(ks_group_args args) {
    const uint32_t bx = blockIdx.x, n = args.n;
    uint32_t sel = 0;
#pragma unroll
    for (int i = 1; i < kKsGroupMax; i++)
        if ((uint32_t)i < n && args.begin[i] <= bx) sel = (uint32_t)i;
    sel = __builtin_amdgcn_readfirstlane(sel);
    const ks_entry &e = args.e[sel];  // kernel arguments: scalar loads at a computed offset
    if (bx - args.begin[sel] >= e.nwg) return;  // padding up to the next entry's multiple of 8
    ks_body<CT, RT, W, D, MAXG, false, AP, P8, NTL>(e.tbr, e.tP, e.tV, e.steps, e.B, e.C, e.K, args.N, e.S, e.NS, e.nwg, e.row_base,
                                       e.slabs, e.arrivals, nullptr, bx - args.begin[sel], args.pad[0] | (e.pad0 << 8));
}

// ---------------------------------------------------------------------------
// k_mfma_kb -- k_mfma_ks's K split and per-wave pipeline on k_mfma_bm's bitmap layout: no
// dense image, no entry scatter.  Per (unit u = row block g x K range q, 32-column k-step s)
// one 8-byte record per lane l (byte t < RT: the occupancy of row 16t + l%16, columns
// 32s + 8(l/16) + [0, 8) -- exactly the 8 halves lane l holds of tile t's A operand of
// v_mfma_f32_16x16x32_f16 -- bytes 6..7: the lane's first value from the step's base
// sbase[u*NS + s]) and the step's values, lane after lane, tile after tile (host layout:
// device_layout.cc build_bm_tiles).  A is ~2.4 B per nonzero at 30% density (k_mfma_ks:
// 4 B).  Wave w runs steps w, w+W, ...: a slot's record and value bounds are loaded one
// round (D steps) ahead of its values; the values are fetched as whole 16-B units (the
// step's run from its 16-B-aligned start, NVB KB at most: one full wave load per KB, lanes
// past the run re-read the first unit) and staged through the wave's LDS slot with B's rows
// (b_piece-permuted, ds_read_b64_tr_b16 fragments); each lane reads its two 8-byte windows
// per tile there and expands them into the tile's fragment by four v_perm_b32 with
// selectors from a 16-entry LDS table.  (The first version loaded the windows straight from
// HBM: 2 x RT 8-byte loads per lane and step at 2-byte alignment, ~40% of each request
// used -- C2 21.1 us; the windows alone cost 11.5 us of it.)  Epilogue as k_mfma_ks (wave
// partial tiles summed in wave order, tagged-slab K-range combine).
// ---------------------------------------------------------------------------
// DBG (experiments diagnostics, wrong results): 2 = no value loads, 3 = no B loads
template <int CT, int RT, int W, int D, int NVB, bool STAMPS, int DBG = 0>
__device__ __forceinline__ void kb_body(const uint32_t *__restrict__ bmtb_first_row, const uint2 *__restrict__ rec,
                                        const uint32_t *__restrict__ sbase, const f16 *__restrict__ vals,
                                        const f16 *__restrict__ B, f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                        uint32_t NS, uint32_t nwg, uint32_t row_base, float *__restrict__ slabs,
                                        uint32_t *__restrict__ arrivals, uint64_t *__restrict__ stamps, uint32_t bx,
                                        uint32_t prio) {
    static_assert(RT >= 1 && RT <= 6, "six mask bytes per record");
    static_assert(NVB >= 1 && NVB <= 4, "1..4 KB of values per step");
    constexpr uint32_t RB = 32 * CT;  // bytes per LDS B row (a 16*CT-column tile)
    constexpr uint32_t UB = 2 * CT;   // 16-B units per B row
    constexpr uint32_t STG = 32u * RB;  // one k-step of B rows
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t u = xcd_block(bx, nwg);
    const uint32_t g = u / S, q = u - g * S;
#define GS_KB_STAMP(slot)                                                                          \
    if constexpr (STAMPS) {                                                                        \
        if (lane == 0) stamps[((size_t)blockIdx.x * W + wv) * 32u + (slot)] = __builtin_amdgcn_s_memtime(); \
    }
    GS_KB_STAMP(0u);
    const uint32_t k0 = q * NS * 32u;
    const uint32_t col0 = blockIdx.y * 16u * CT, nv = min(16u * CT, N - col0);
    uint2 *lut = reinterpret_cast<uint2 *>(lds);
    unsigned char *bst = lds + 128u + wv * (STG + NVB * 1024u);
    unsigned char *vst = bst + STG;  // the step's values (16-B-aligned run start at byte 0)
    const u32x4 zero4 = {0u, 0u, 0u, 0u};
    if (tid < 16u) lut[tid] = make_uint2(bm_sel(tid, 0), bm_sel(tid, 1));

    const uint32_t nsw = NS > wv ? (NS - wv + W - 1u) / W : 0u;
    const size_t ubase = (size_t)u * NS;
    u32x4 BR[D][CT];
    u32x4 VR[D][NVB];  // per slot: the values of the step it holds (16-B units)
    uint2 RC[D];       // ... its record
    uint32_t RL[D];    // ... and its first value's offset (halves) from the run's aligned start
    uint2 NX[D];       // per slot: record of the step the slot loads next
    uint32_t NB[D], NE[D];  // ... and its value bounds [sbase[s], sbase[s+1])
    uint32_t vz;
    __asm__ volatile("v_mov_b32 %0, 0" : "=v"(vz));
    auto st_of = [&](uint32_t i) -> uint32_t { return __builtin_amdgcn_readfirstlane(i < nsw ? wv + i * W : 0u); };
    auto mbyte = [](const uint2 &r, int t) -> uint32_t {
        return t < 4 ? (r.x >> (8 * t)) & 0xffu : (r.y >> (8 * (t - 4))) & 0xffu;
    };
    // record + value bounds of step i (vector loads, in order with the values: see k_mfma_ks)
    auto load_rec = [&](uint32_t i, uint2 &NX_, uint32_t &NB_, uint32_t &NE_) {
        const uint32_t st = st_of(i);
        NX_ = rec[(ubase + st) * 64u + lane + vz];
        NB_ = sbase[ubase + st + vz];
        NE_ = sbase[ubase + st + 1u + vz];
    };
    auto load_b = [&](uint32_t i, u32x4 (&B_)[CT]) {
        const uint32_t kr = k0 + st_of(i) * 32u;
#pragma unroll
        for (int c = 0; c < CT; c++) {
            const uint32_t un = lane + 64u * c;
            const uint32_t k = kr + un / UB, cu = (un % UB) * 8u;
            if constexpr (DBG == 3) B_[c] = u32x4{k, cu, k, cu};
            else B_[c] = *reinterpret_cast<const u32x4 *>(B + (size_t)(k < K ? k : K - 1u) * N + col0 + (cu < nv ? cu : 0u));
        }
    };
    // the slot takes over the record it loaded a round ago, issues its step's values, and
    // loads the record of its step a round ahead
    auto load_v = [&](uint32_t i, uint2 &NX_, uint32_t &NB_, uint32_t &NE_, uint2 &RC_, uint32_t &RL_,
                      u32x4 (&VR_)[NVB]) {
        RC_ = NX_;
        const uint32_t b0 = NB_ & ~7u, len = NE_ - b0;  // halves from the aligned start
        RL_ = NB_ - b0;
#pragma unroll
        for (int j = 0; j < NVB; j++) {
            const uint32_t h = 8u * (lane + 64u * j);
            if constexpr (DBG == 2) VR_[j] = u32x4{RC_.x, RC_.y, RC_.x, RC_.y};
            else VR_[j] = *reinterpret_cast<const u32x4 *>(vals + b0 + (h < len ? h : 0u));
        }
        load_rec(i + D, NX_, NB_, NE_);
    };
#pragma unroll
    for (int d = 0; d < D; d++) load_rec((uint32_t)d, NX[d], NB[d], NE[d]);
#pragma unroll
    for (int d = 0; d < D; d++) load_b((uint32_t)d, BR[d]);
#pragma unroll
    for (int d = 0; d < D; d++) load_v((uint32_t)d, NX[d], NB[d], NE[d], RC[d], RL[d], VR[d]);
    // the selector table (written by wave 0) before any wave expands a fragment
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
    GS_KB_STAMP(1u);

    f4v acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};

    auto step = [&](uint32_t i, uint2 &NX_, uint32_t &NB_, uint32_t &NE_, uint2 &RC_, uint32_t &RL_,
                    u32x4 (&VR_)[NVB], u32x4 (&B_)[CT]) {
        const bool live = i < nsw;  // wave-uniform
        h8v av[RT], bv[CT];
        if (live) {
            const uint32_t kr = k0 + (wv + i * W) * 32u;
#pragma unroll
            for (int c = 0; c < CT; c++) {
                const uint32_t un = lane + 64u * c, k = un / UB, s = un % UB;
                *reinterpret_cast<u32x4 *>(bst + k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u) =
                    kr + k < K && s * 8u < nv ? B_[c] : zero4;
            }
#pragma unroll
            for (int j = 0; j < NVB; j++) *reinterpret_cast<u32x4 *>(vst + (lane + 64u * j) * 16u) = VR_[j];
            const uint32_t kb = 8u * (lane >> 4);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                s4v t2[2];
#pragma unroll
                for (int hh = 0; hh < 2; hh++) {
                    const uint32_t k = kb + 4u * hh + ((lane & 15u) >> 2);
                    t2[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s4v *)(bst + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                }
                __builtin_memcpy(&bv[ct], t2, 16);
            }
            uint32_t p = RL_ + (RC_.y >> 16);
#pragma unroll
            for (int t = 0; t < RT; t++) {
                const uint32_t m = mbyte(RC_, t);
                const uint2 sl = lut[m & 15u], sh = lut[m >> 4];
                const u32x2_a2 lo = *reinterpret_cast<const u32x2_a2 *>(vst + 2u * p);
                const u32x2_a2 hi = *reinterpret_cast<const u32x2_a2 *>(vst + 2u * (p + __builtin_popcount(m & 15u)));
                p += __builtin_popcount(m);
                uint32_t w4[4];
                w4[0] = __builtin_amdgcn_perm(lo.y, lo.x, sl.x);
                w4[1] = __builtin_amdgcn_perm(lo.y, lo.x, sl.y);
                w4[2] = __builtin_amdgcn_perm(hi.y, hi.x, sh.x);
                w4[3] = __builtin_amdgcn_perm(hi.y, hi.x, sh.y);
                __builtin_memcpy(&av[t], w4, 16);
            }
        }
        load_b(i + D, B_);
        load_v(i + D, NX_, NB_, NE_, RC_, RL_, VR_);
        if (live) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++)
                    acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[rt], bv[ct], acc[rt][ct], 0, 0, 0);
            if (i < 16u) GS_KB_STAMP(3u + i);
        }
    };
    const bool young = wv >= W / 2u;
    if ((prio & 3u) && young) __builtin_amdgcn_s_setprio(1);
    for (uint32_t i0 = 0; i0 < nsw; i0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) step(i0 + d, NX[d], NB[d], NE[d], RC[d], RL[d], VR[d], BR[d]);
    }
    if ((prio & 3u) && young) __builtin_amdgcn_s_setprio(0);
    GS_KB_STAMP(20u);
    // ---- K-split ticket: wave 0 takes its row block's arrival ticket as soon as its own
    // loop ends, so the add's round trip overlaps the partial-tile reduction below
    uint32_t *arr = arrivals + (size_t)g * gridDim.y + blockIdx.y;
    uint32_t ticket = 0;
    if (S > 1 && wv == 0 && lane == 0) ticket = __hip_atomic_fetch_add(arr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- wave partial tiles -> LDS (the trailing loads write registers only), summed in
    // wave order.  Item t = (tile, lane) of a 16x16 tile: the 4 rows 4*(lane/16)+i of
    // column lane%16.  When the W partial tiles fit LDS beside the wave images (APART), each
    // wave stores its tile as soon as its loop ends, without waiting for the others
    constexpr bool APART = kb_red_apart(CT, RT, W, NVB);
    f4v *red = reinterpret_cast<f4v *>(lds + (APART ? kb_stage_bytes(CT, W, NVB) : 0u));
    constexpr bool HALVES = !APART && ks_red_halves(CT, RT, W);
    constexpr uint32_t WR = HALVES ? W / 2 : W;  // partial tiles summed from LDS
    uint32_t *flag = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(red) + (size_t)WR * RT * CT * 1024u);
    if constexpr (!APART) {
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    }
    if constexpr (HALVES) {
        if (wv >= WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) red[(((wv - WR) * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
        if (wv < WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) acc[rt][ct] += red[((wv * RT + rt) * CT + ct) * 64u + lane];
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    }
    if (wv < WR) {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[((wv * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
    }
    if (S > 1 && wv == 0 && lane == 0) *flag = ticket;  // (waits for the add's return)
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
    constexpr uint32_t NI = RT * CT * 64u, NT = 64u * W;
    const uint32_t r0 = bmtb_first_row[g], R = bmtb_first_row[g + 1] - r0;
    auto item_sum = [&](uint32_t t) {
        f4v sum = red[t];
#pragma unroll
        for (uint32_t w = 1; w < WR; w++) sum += red[w * NI + t];
        return sum;
    };
    auto store_item = [&](uint32_t t, const f4v &v) {
        const uint32_t ln = t & 63u, tt = t >> 6, rt = tt / CT, ct = tt % CT;
        const uint32_t col = 16u * ct + (ln & 15u), rb = 16u * rt + 4u * (ln >> 4);
        if (col >= nv) return;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (rb + i < R) C[(size_t)(row_base + r0 + rb + i) * N + col0 + col] = (f16)v[i];
    };
    GS_KB_STAMP(21u);
    if (S == 1) {
        for (uint32_t t = tid; t < NI; t += NT) store_item(t, item_sum(t));
        GS_KB_STAMP(22u);
        return;
    }
    // ---- K-split combine by tagged slabs.  Every fp32 word of a published slab carries
    // its own validity tag in the low mantissa bit (the reader drops the bit, a 2^-24
    // relative truncation), so no store needs to be drained before a signal: every workgroup
    // stores its slab with 16-B write-through (sc1) stores, and the one that drew the last
    // ticket loads each other slab word with agent-scope (sc1) loads until its tag reads
    // this launch's value -- its writer holds an earlier ticket, so it is running and its
    // stores are issued or about to be -- sums the S partials in q order (deterministic) and
    // writes C.  The tag alternates from launch to launch: the arrival counter holds
    // (epoch << 16) | arrivals, the tag is epoch ^ 1, and the last workgroup re-arms the
    // counter with the epoch flipped and no arrivals.  Every slab word then holds the
    // previous launch's tag when a launch starts (the last workgroup stores its own slab
    // too), and the zero-filled first state reads as "tag 0, epoch 0" -- so no slab is
    // cleared after use ((S - 1) fewer slab stores than clearing, the last workgroup's own
    // store issued before it waits).  Every access to the slabs is sc1 (MI355X_MICROARCH.md
    // Workgroup dispatch, Valid forms: the R2 granule, here one naturally aligned word).
    // The next launch on the stream starts after these stores complete.
    const uint32_t tk = *flag & 0xffffu, tag = ((*flag >> 16) & 1u) ^ 1u;
    f4v *slab = reinterpret_cast<f4v *>(slabs) + ((size_t)u * gridDim.y + blockIdx.y) * NI;
    auto tagged = [&](const f4v &v) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        w[0] = (w[0] & ~1u) | tag; w[1] = (w[1] & ~1u) | tag; w[2] = (w[2] & ~1u) | tag; w[3] = (w[3] & ~1u) | tag;
        return w;
    };
    for (uint32_t t = tid; t < NI; t += NT) {
        const u32x4 w = tagged(item_sum(t));
        __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(slab + t), "v"(w) : "memory");
    }
    if (tk != S - 1u) {
        GS_KB_STAMP(22u);
        return;
    }
    if (tid == 0) __hip_atomic_store(arr, tag << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const f4v *base = reinterpret_cast<const f4v *>(slabs) + blockIdx.y * NI;
    const size_t qstride = (size_t)gridDim.y * NI;  // slab of (g, qq) = base + (g*S + qq) * qstride
    uint32_t *err = arrivals + (size_t)(nwg / S) * gridDim.y;  // the replica's device error word
    for (uint32_t t = tid; t < NI; t += NT) {
        f4v sum = {0.f, 0.f, 0.f, 0.f};
        for (uint32_t qq = 0; qq < S; qq++) {
            u32x4 w;
            if (qq == q) {  // truncated as a published word is (whichever workgroup is last: deterministic)
                w = tagged(item_sum(t));
            } else {
                w = ks_slab_wait(reinterpret_cast<const uint32_t *>(base + ((size_t)g * S + qq) * qstride + t), tag, err,
                                 GS_KS_FORCE(prio));
            }
            w[0] &= ~1u; w[1] &= ~1u; w[2] &= ~1u; w[3] &= ~1u;
            f4v x;
            __builtin_memcpy(&x, &w, 16);
            sum += x;
        }
        store_item(t, sum);
    }
    GS_KB_STAMP(22u);
#undef GS_KB_STAMP
}

template <int CT, int RT, int W, int D, int NVB, bool STAMPS = false, int DBG = 0>
__global__ __launch_bounds__(64 * W) void k_mfma_kb(const uint32_t *__restrict__ bmtb_first_row,  // nb+1
                                                    const uint2 *__restrict__ rec,       // (u*NS + step)*64 + lane
                                                    const uint32_t *__restrict__ sbase,  // u*NS + step (+1)
                                                    const f16 *__restrict__ vals, const f16 *__restrict__ B,
                                                    f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                                    uint32_t NS, uint32_t nwg, uint32_t row_base,
                                                    float *__restrict__ slabs, uint32_t *__restrict__ arrivals,
                                                    uint64_t *__restrict__ stamps = nullptr, uint32_t prio = 0) {
    kb_body<CT, RT, W, D, NVB, STAMPS, DBG>(bmtb_first_row, rec, sbase, vals, B, C, K, N, S, NS, nwg, row_base, slabs, arrivals,
                                  stamps, blockIdx.x, prio);
}

#ifdef GS_EXPERIMENTS  // opt-in, measured slower than k_mfma_rows / k_mfma_ks (make EXPERIMENTS=1)
// ---------------------------------------------------------------------------
// k_mfma_bm -- BMTB row blocks on the matrix cores from a bitmap layout, with the
// dense A fragments built in registers (no dense image, no LDS scatter).
// Why: k_mfma_rows / k_mfma_ks move 4 B per nonzero ([u16 position][f16 value]) and
// scatter every entry into a dense LDS image (two LDS stores per entry, one to clear
// it); at 30% density a bitmap costs 0.42 B per nonzero, so A is ~2.4 B per nonzero
// and no entry ever passes through LDS.
// Layout (host/device_layout.cc build_bm_tiles): unit u = (row block g, K range q) of
// NS 32-column k-steps; per (u, step) one 8-byte record per lane l: byte t (t < RT) is
// the occupancy of row 16t + l%16, columns 32*step + 8*(l/16) + [0, 8) -- exactly the 8
// halves lane l holds of the A operand of v_mfma_f32_16x16x32_f16 for row tile t --
// and bytes 6..7 the lane's first value (halves, from the step's base sbase[u*NS+step]);
// a step's values are stored lane after lane, tile after tile, ascending columns.
// Wave w of the workgroup owns the range's k-steps w, w+W, ...: per k-step it loads the
// 32 B rows into registers and stores them into its own LDS ring slot (32-B pieces
// permuted by b_piece, so the ds_read_b64_tr_b16 fragment reads are conflict-free; not
// LDS-DMA: the compiler then waits for every DMA in flight before each LDS read of the
// same wave), loads the record, then per row tile two 8-byte
// value windows (at the tile's first value and past the low nibble's values; 2-byte
// aligned loads) that two v_perm_b32 each expand into the tile's dense fragment with
// selectors from a 16-entry table in LDS, and runs RT x CT MFMAs.  Pipeline per wave:
// B + record two steps ahead, B store + values one step ahead (counted waits); no
// workgroup barrier until the end.  Epilogue as k_mfma_ks: the W partial tiles summed in
// wave order through LDS, then C (S = 1) or a write-through fp32 slab + one arrival add,
// the last of the row block's S workgroups summing the slabs in q order (deterministic).
// Rows of B past K are read as row K-1 against zero A columns (a non-finite B value
// there gives NaN: the documented matrix-core deviation).
// ---------------------------------------------------------------------------

// STAMPS (diagnostic build only, gs_debug_mfma_timeline): lane 0 of every wave records
// s_memtime into stamps[(workgroup * W + wave) * 16 + slot]: 0 start, 1 B + records issued,
// 2 values issued, 3 B stored (all landed), 4 MFMAs done (first batch), 5 loop done,
// 6 reduced, 7 slab published, 8 end
template <int CT, int RT, int W, int NBT, bool STAMPS = false>
__global__ __launch_bounds__(64 * W) void k_mfma_bm(const uint32_t *__restrict__ bmtb_first_row,  // nb+1
                                                    const uint2 *__restrict__ rec,       // (u*NS + step)*64 + lane
                                                    const uint32_t *__restrict__ sbase,  // u*NS + step (+1)
                                                    const f16 *__restrict__ vals, const f16 *__restrict__ B,
                                                    f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                                    uint32_t NS, uint32_t nwg, uint32_t row_base,
                                                    float *__restrict__ slabs, uint32_t *__restrict__ arrivals,
                                                    uint64_t *__restrict__ stamps = nullptr) {
    static_assert(RT >= 1 && RT <= 6, "six mask bytes per record");
#define GS_BM_STAMP(slot)                                                                          \
    if constexpr (STAMPS) {                                                                        \
        if ((threadIdx.x & 63u) == 0) stamps[((size_t)blockIdx.x * W + (threadIdx.x >> 6)) * 16u + (slot)] = __builtin_amdgcn_s_memtime(); \
    }
    GS_BM_STAMP(0u);
    constexpr uint32_t RB = 32 * CT;     // bytes per LDS B row (a 16*CT-column tile)
    constexpr uint32_t UB = 2 * CT;      // 16-B units per B row
    constexpr uint32_t STG = 32u * RB;   // one k-step of B rows = CT LDS-DMA wave-instructions
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t u = xcd_block(blockIdx.x, nwg);  // nwg == gridDim.x
    const uint32_t g = u / S, q = u - g * S;
    const uint32_t col0 = blockIdx.y * 16u * CT, nv = min(16u * CT, N - col0);
    uint2 *lut = reinterpret_cast<uint2 *>(lds);
    unsigned char *ring = lds + 128u + wv * NBT * STG;  // this wave's NBT k-step slots
    if (tid < 16u) lut[tid] = make_uint2(bm_sel(tid, 0), bm_sel(tid, 1));
    const uint32_t k0 = q * NS * 32u;
    const uint32_t nsw = NS > wv ? (NS - wv + W - 1u) / W : 0u;  // this wave's k-steps
    const size_t ub = (size_t)u * NS;
    // steps past the wave's last re-read its first (cached)
    auto step_of = [&](uint32_t i) -> uint32_t { return i < nsw ? wv + i * W : wv; };
    // B rows of step i -> registers (16-B units, lane-linear over the step's 32 rows), then into
    // slot j with the 32-B pieces permuted by b_piece (conflict-free transposed reads).  Not
    // LDS-DMA: the compiler then waits for all DMA in flight before the wave's next
    // dependent load, which serialises the records and the value windows behind the B rows
    auto load_b = [&](uint32_t i, u32x4 (&BR)[CT]) {
        const uint32_t kr = k0 + step_of(i) * 32u;
#pragma unroll
        for (uint32_t c = 0; c < CT; c++) {
            const uint32_t un = c * 64u + lane, k = un / UB, cu = (un % UB) * 8u;
            const uint32_t kk = kr + k < K ? kr + k : K - 1u;
            BR[c] = *reinterpret_cast<const u32x4 *>(B + (size_t)kk * N + col0 + (cu < nv ? cu : 0u));
        }
    };
    auto store_b = [&](uint32_t j, const u32x4 (&BR)[CT]) {
        unsigned char *dst = ring + j * STG;
#pragma unroll
        for (uint32_t c = 0; c < CT; c++) {
            const uint32_t un = c * 64u + lane, k = un / UB, s = un % UB;
            *reinterpret_cast<u32x4 *>(dst + k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u) = BR[c];
        }
    };
    auto mbyte = [](const uint2 &r, int t) -> uint32_t {
        return t < 4 ? (r.x >> (8 * t)) & 0xffu : (r.y >> (8 * (t - 4))) & 0xffu;
    };
    f4v acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t kb = 8u * (lane >> 4);
    bool first = true;
    // batches of NBT k-steps: every load of the batch in flight at once (records, then the B
    // rows by DMA, then -- once each record is in -- the value windows), then the MFMAs
    for (uint32_t i0 = 0; i0 < nsw; i0 += NBT) {
        // B rows first (L2-served: they return before the records from HBM, and loads retire
        // in order, so waiting for the records costs nothing extra)
        u32x4 br[NBT][CT];
#pragma unroll
        for (int j = 0; j < NBT; j++) load_b(i0 + j, br[j]);
        uint2 rc[NBT];
        uint32_t sb[NBT];
#pragma unroll
        for (int j = 0; j < NBT; j++) {
            sb[j] = sbase[ub + step_of(i0 + j)];  // wave-uniform: a scalar load
            rc[j] = rec[(ub + step_of(i0 + j)) * 64u + lane];
        }
        if (first) GS_BM_STAMP(1u);
        u32x2_a2 vv[NBT][RT][2];
#pragma unroll
        for (int j = 0; j < NBT; j++) {
            uint32_t p = sb[j] + (rc[j].y >> 16);
#pragma unroll
            for (int t = 0; t < RT; t++) {
                const uint32_t m = mbyte(rc[j], t);
                vv[j][t][0] = *reinterpret_cast<const u32x2_a2 *>(vals + p);
                vv[j][t][1] = *reinterpret_cast<const u32x2_a2 *>(vals + p + __builtin_popcount(m & 15u));
                p += __builtin_popcount(m);
            }
        }
        if (first) GS_BM_STAMP(2u);
#pragma unroll
        for (int j = 0; j < NBT; j++) store_b(j, br[j]);
        if (first) {  // the selector table (its stores, once)
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __asm__ volatile("" ::: "memory");
            GS_BM_STAMP(3u);
        }
#pragma unroll
        for (int j = 0; j < NBT; j++) {
            if (i0 + j < nsw) {
                const unsigned char *bst = ring + j * STG;
                h8v bv[CT];
#pragma unroll
                for (int ct = 0; ct < CT; ct++) {
                    s4v t2[2];
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        const uint32_t k = kb + 4u * hh + ((lane & 15u) >> 2);
                        t2[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s4v *)(bst + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                    }
                    __builtin_memcpy(&bv[ct], t2, 16);
                }
#pragma unroll
                for (int t = 0; t < RT; t++) {
                    const uint32_t m = mbyte(rc[j], t);
                    const uint2 sl = lut[m & 15u], sh = lut[m >> 4];
                    const u32x2_a2 lo = vv[j][t][0], hi = vv[j][t][1];
                    uint32_t w[4];
                    w[0] = __builtin_amdgcn_perm(lo.y, lo.x, sl.x);
                    w[1] = __builtin_amdgcn_perm(lo.y, lo.x, sl.y);
                    w[2] = __builtin_amdgcn_perm(hi.y, hi.x, sh.x);
                    w[3] = __builtin_amdgcn_perm(hi.y, hi.x, sh.y);
                    h8v a;
                    __builtin_memcpy(&a, w, 16);
#pragma unroll
                    for (int ct = 0; ct < CT; ct++)
                        acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bv[ct], acc[t][ct], 0, 0, 0);
                }
            }
        }
        if (first) {
            GS_BM_STAMP(4u);
            first = false;
        }
    }
    GS_BM_STAMP(5u);
    if (first) {  // a wave with no k-steps still meets the table barrier
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    }
    // every wave is done with its ring before it is reused for the partial tiles
    __syncthreads();
    f4v *red = reinterpret_cast<f4v *>(lds);
    constexpr bool HALVES = bm_red_halves(CT, RT, W);
    constexpr uint32_t WR = HALVES ? W / 2 : W;
    if constexpr (HALVES) {
        if (wv >= WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) red[(((wv - WR) * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
        }
        __syncthreads();
        if (wv < WR) {
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int ct = 0; ct < CT; ct++) acc[rt][ct] += red[((wv * RT + rt) * CT + ct) * 64u + lane];
        }
        __syncthreads();
    }
    if (wv < WR) {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[((wv * RT + rt) * CT + ct) * 64u + lane] = acc[rt][ct];
    }
    __syncthreads();
    constexpr uint32_t NI = RT * CT * 64u, NT = 64u * W;
    const uint32_t r0 = bmtb_first_row[g], R = bmtb_first_row[g + 1] - r0;
    auto item_sum = [&](uint32_t t) {
        f4v sum = red[t];
#pragma unroll
        for (uint32_t w = 1; w < WR; w++) sum += red[w * NI + t];
        return sum;
    };
    auto store_item = [&](uint32_t t, const f4v &v) {
        const uint32_t ln = t & 63u, tt = t >> 6, rt = tt / CT, ct = tt % CT;
        const uint32_t col = 16u * ct + (ln & 15u), rb = 16u * rt + 4u * (ln >> 4);
        if (col >= nv) return;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (rb + i < R) C[(size_t)(row_base + r0 + rb + i) * N + col0 + col] = (f16)v[i];
    };
    GS_BM_STAMP(6u);
    if (S == 1) {
        for (uint32_t t = tid; t < NI; t += NT) store_item(t, item_sum(t));
        GS_BM_STAMP(8u);
        return;
    }
    // K-split hand-off (k_mfma_ks's form): 16-B write-through slab stores, every storing
    // wave's vmcnt(0), a barrier, one agent-scope arrival add; the last adder (told by the
    // returned count) loads the other slabs with agent-scope (sc1) loads
    f4v *slab = reinterpret_cast<f4v *>(slabs) + ((size_t)u * gridDim.y + blockIdx.y) * NI;
    for (uint32_t t = tid; t < NI; t += NT) {
        const f4v v = item_sum(t);
        __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(slab + t), "v"(v) : "memory");
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds + (size_t)WR * NI * 16u);
    uint32_t *arr = arrivals + (size_t)g * gridDim.y + blockIdx.y;
    if (tid == 0) *flag = __hip_atomic_fetch_add(arr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    GS_BM_STAMP(7u);
    if (*flag != S - 1u) {
        GS_BM_STAMP(8u);
        return;
    }
    if (tid == 0) __hip_atomic_store(arr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const f4v *base = reinterpret_cast<const f4v *>(slabs) + blockIdx.y * NI;
    const size_t qstride = (size_t)gridDim.y * NI;
    for (uint32_t t = tid; t < NI; t += NT) {
        const f4v own = item_sum(t);
        f4v sum = {0.f, 0.f, 0.f, 0.f};
        for (uint32_t qq = 0; qq < S; qq++) {
            if (qq == q) {
                sum += own;
                continue;
            }
            const float *src = reinterpret_cast<const float *>(base + ((size_t)g * S + qq) * qstride + t);
            f4v x;
#pragma unroll
            for (int i = 0; i < 4; i++) x[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sum += x;
        }
        store_item(t, sum);
    }
    GS_BM_STAMP(8u);
#undef GS_BM_STAMP
}

// ---------------------------------------------------------------------------
// k_mfma_bm2 -- k_mfma_bm's layout with one wave per 16-row tile (RT waves per
// workgroup): no cross-wave reduction, and every wave streams its tile's records and
// value windows through register rings (records 16 k-steps ahead, values 8 ahead) while
// the workgroup's B slice (NS k-steps, staged once by all waves, one barrier) stays in
// LDS.  K split: each wave publishes its 16 x N fp32 tile (8-B agent-scope stores), one
// agent-scope add per (row block, tile), the last adder sums the slabs in K-range order
// (deterministic) and stores C.
// ---------------------------------------------------------------------------
template <int CT, int RT>
__global__ __launch_bounds__(64 * RT) void k_mfma_bm2(const uint32_t *__restrict__ bmtb_first_row,  // nb+1
                                                     const uint2 *__restrict__ rec, const uint32_t *__restrict__ sbase,
                                                     const f16 *__restrict__ vals, const f16 *__restrict__ B,
                                                     f16 *__restrict__ C, uint32_t K, uint32_t N, uint32_t S,
                                                     uint32_t NS, uint32_t nwg, uint32_t row_base,
                                                     float *__restrict__ slabs, uint32_t *__restrict__ arrivals) {
    constexpr uint32_t RB = 32 * CT, UB = 2 * CT, STG = 32u * RB;
    constexpr uint32_t DR = 16, DV = 8;  // look-ahead of the records / value windows (k-steps)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // = this wave's row tile
    const uint32_t u = xcd_block(blockIdx.x, nwg);
    const uint32_t g = u / S, q = u - g * S;
    const uint32_t col0 = blockIdx.y * 16u * CT, nv = min(16u * CT, N - col0);
    uint2 *lut = reinterpret_cast<uint2 *>(lds);
    unsigned char *bsl = lds + 128u;  // NS k-steps of B rows
    if (tid < 16u) lut[tid] = make_uint2(bm_sel(tid, 0), bm_sel(tid, 1));
    const uint32_t k0 = q * NS * 32u;
    const size_t ub = (size_t)u * NS;
    const uint32_t tsh = 8u * (wv & 3u);  // this tile's mask byte in the record word
    auto mask_of = [&](const uint2 &r) -> uint32_t { return ((wv < 4u ? r.x : r.y) >> tsh) & 0xffu; };
    // the value offset of this lane's run for this tile: the record's lane offset + the
    // values of the lower tiles (bytes below this tile's)
    auto vstart = [&](const uint2 &r, uint32_t sb) -> uint32_t {
        uint32_t lower = wv < 4u ? (wv ? r.x & ((1u << (8u * wv)) - 1u) : 0u)
                                 : r.x;
        uint32_t p = sb + (r.y >> 16) + (uint32_t)__builtin_popcount(lower);
        if (wv >= 4u) p += (uint32_t)__builtin_popcount(r.y & ((1u << (8u * (wv - 4u))) - 1u) & 0xffffu);
        return p;
    };
    auto ld_rec = [&](uint32_t s, uint32_t &sb) -> uint2 {
        const uint32_t ss = s < NS ? s : NS - 1u;
        sb = sbase[ub + ss];
        return rec[(ub + ss) * 64u + lane];
    };
    auto ld_vals = [&](const uint2 &r, uint32_t sb, u32x2_a2 (&V)[2]) {
        const uint32_t p = vstart(r, sb), m = mask_of(r);
        V[0] = *reinterpret_cast<const u32x2_a2 *>(vals + p);
        V[1] = *reinterpret_cast<const u32x2_a2 *>(vals + p + __builtin_popcount(m & 15u));
    };
    // records of the first DR steps (the critical HBM chain) before the B slice
    uint2 rr[DR];
    uint32_t rs[DR];
#pragma unroll
    for (uint32_t j = 0; j < DR; j++) rr[j] = ld_rec(j, rs[j]);
    // B slice: step s staged by wave s % RT (registers -> ds_write_b128, b_piece permutation)
    for (uint32_t s = wv; s < NS; s += RT) {
        const uint32_t kr = k0 + s * 32u;
        u32x4 br[CT];
#pragma unroll
        for (uint32_t c = 0; c < CT; c++) {
            const uint32_t un = c * 64u + lane, k = un / UB, cu = (un % UB) * 8u;
            const uint32_t kk = kr + k < K ? kr + k : K - 1u;
            br[c] = *reinterpret_cast<const u32x4 *>(B + (size_t)kk * N + col0 + (cu < nv ? cu : 0u));
        }
#pragma unroll
        for (uint32_t c = 0; c < CT; c++) {
            const uint32_t un = c * 64u + lane, k = un / UB, sx = un % UB;
            *reinterpret_cast<u32x4 *>(bsl + s * STG + k * RB + b_piece<CT>(k, sx >> 1) * 32u + (sx & 1u) * 16u) = br[c];
        }
    }
    // the value windows of the first DV steps
    u32x2_a2 vv[DV][2];
#pragma unroll
    for (uint32_t j = 0; j < DV; j++) ld_vals(rr[j], rs[j], vv[j]);
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the B slice and the selector table
    __asm__ volatile("" ::: "memory");
    f4v acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ct++) acc[ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t kb = 8u * (lane >> 4);
    // step i (ring slots i % DR, i % DV): compute i, then refill: values of i + DV (their
    // record is in slot (i + DV) % DR), record of i + DR
    for (uint32_t i0 = 0; i0 < NS; i0 += DR) {
#pragma unroll
        for (uint32_t d = 0; d < DR; d++) {
            const uint32_t i = i0 + d;
            if (i < NS) {
                const unsigned char *bst = bsl + i * STG;
                const uint32_t m = mask_of(rr[d]);
                const uint2 sl = lut[m & 15u], sh = lut[m >> 4];
                const u32x2_a2 lo = vv[d % DV][0], hi = vv[d % DV][1];
                uint32_t w[4];
                w[0] = __builtin_amdgcn_perm(lo.y, lo.x, sl.x);
                w[1] = __builtin_amdgcn_perm(lo.y, lo.x, sl.y);
                w[2] = __builtin_amdgcn_perm(hi.y, hi.x, sh.x);
                w[3] = __builtin_amdgcn_perm(hi.y, hi.x, sh.y);
                h8v a;
                __builtin_memcpy(&a, w, 16);
#pragma unroll
                for (int ct = 0; ct < CT; ct++) {
                    s4v t2[2];
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        const uint32_t k = kb + 4u * hh + ((lane & 15u) >> 2);
                        t2[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s4v *)(bst + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                    }
                    h8v bv;
                    __builtin_memcpy(&bv, t2, 16);
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bv, acc[ct], 0, 0, 0);
                }
            }
            // refill (past NS: re-reads of the last step, never used)
            ld_vals(rr[(d + DV) % DR], rs[(d + DV) % DR], vv[d % DV]);
            rr[d] = ld_rec(i + DR, rs[d]);
        }
    }
    const uint32_t r0 = bmtb_first_row[g], R = bmtb_first_row[g + 1] - r0;
    auto store_tile = [&](const f4v (&v)[CT]) {
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            const uint32_t col = 16u * ct + (lane & 15u);
            if (col >= nv) continue;
#pragma unroll
            for (uint32_t e = 0; e < 4; e++) {
                const uint32_t rw = 16u * wv + 4u * (lane >> 4) + e;
                if (rw < R) C[(size_t)(row_base + r0 + rw) * N + col0 + col] = (f16)v[ct][e];
            }
        }
    };
    if (S == 1) {
        store_tile(acc);
        return;
    }
    if (16u * wv >= R) return;  // a tile past the block's rows: no counter traffic
    // K split hand-off per (row block, tile, column tile)
    constexpr uint32_t TI = CT * 64u;
    const size_t tix = ((size_t)g * gridDim.y + blockIdx.y) * RT + wv;
    f4v *slab = reinterpret_cast<f4v *>(slabs) + (tix * S + q) * TI;
#pragma unroll
    for (int ct = 0; ct < CT; ct++) {
        uint64_t *dst = reinterpret_cast<uint64_t *>(slab + ct * 64u + lane);
        uint64_t w[2];
        __builtin_memcpy(w, &acc[ct], 16);
        __hip_atomic_store(dst, w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dst + 1, w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&arrivals[tix], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != S - 1u) return;
    if (lane == 0) __hip_atomic_store(&arrivals[tix], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f4v sum[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ct++) sum[ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const f4v *base = reinterpret_cast<const f4v *>(slabs) + tix * S * TI;
    for (uint32_t qq = 0; qq < S; qq++) {
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            if (qq == q) {
                sum[ct] += acc[ct];
            } else {
                const uint64_t *src = reinterpret_cast<const uint64_t *>(base + (size_t)qq * TI + ct * 64u + lane);
                uint64_t w[2];
                w[0] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                w[1] = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                f4v x;
                __builtin_memcpy(&x, w, 16);
                sum[ct] += x;
            }
        }
    }
    store_tile(sum);
}

#endif  // GS_EXPERIMENTS (k_mfma_bm, k_mfma_bm2)
// ---------------------------------------------------------------------------
// k_nm_mfma -- fixed_interval_col_direction BMTs that are 2:4 panels
//  on the sparse matrix cores:
// v_smfmac_f32_16x16x64_f16 multiplies a 16x64 A tile stored as 16x32 values
// plus 2-bit positions by a dense 64x16 B tile.
//
// Operand layout of the instruction (measured, scripts/probes/probe_smfmac.hip):
// lane l holds A row l%16, dense k [16*(l/16), +16) of the 64-wide k-step as 8
// values (two per aligned group of 4; idx bits [4g+1:4g] / [4g+3:4g+2] = the
// positions of group g's two values, ascending); B lane l holds column l%16,
// k [8*(l/16), +8) in elements 0-7 and k [32 + 8*(l/16), +8) in elements 8-15;
// the accumulator is the 16x16 MFMA layout (column l%16, rows 4*(l/16)+i).
//
// HBM layout (device_plan.hip build_nm_panels): per row group of 64 rows (four
// 16-row tiles) and k-step s a 4608-byte block: [lane] 8 B of positions (u16
// per tile: tiles 0/1 in the low dword, selected by abid 0/1, tiles 2/3 in the
// high dword), then [tile rt][lane] 16 B of values.  Every wave load is one
// coalesced 512 B / 1 KB request; A is read exactly once.
//
// Workgroup = 8 waves = two row groups (128 rows) x four k-phases: wave (rh, q)
// takes k-step 4c+q of every 256-row chunk c of B.  B chunks are staged in LDS
// (two buffers, 32-B pieces XOR-permuted by b_piece so the transposed reads
// are conflict-free) by all 512 threads through registers, one chunk ahead;
// each wave's A blocks are loaded two chunks ahead.  One barrier per chunk;
// sched_barriers keep the phases in issue order so each wait leaves the younger
// prefetches in flight.  The four k-phase partial tiles are summed in a fixed
// order through LDS ((q0 + q2) + (q1 + q3): deterministic) and stored as fp16.
// ---------------------------------------------------------------------------
typedef _Float16 h16v __attribute__((ext_vector_type(16)));
// kNmWaves, kNmBlockBytes, kNmKC: kernel_consts.hpp

// DBG (diagnostic builds only, GS_NM_DEBUG): 1 = no B loads in the loop, 2 = no A loads,
// 4 = s_memtime phase stamps of waves 0/4 of workgroups 0 and 100, printed, 8 = the transposed B
// fragment reads of odd n-tiles skipped (half the LDS reads; wrong results)
// NG: the dense width in HBM (B and C row length); NG = 8 runs one 16-column tile whose
// columns 8..15 are zeros in LDS and never stored (N = 8, the half-used tile of C3's N sweep)
// TT: 16-row tiles per workgroup (nm_tiles; kernel_consts.hpp nm_wg_block_bytes): the wave set rh
// = 0 takes the first G0 = ceil(TT/2) tiles, rh = 1 the other G1 = TT/2 (TT = 8: two 64-row groups,
// the original layout).  TT = 7 spreads C3's 1,792 tiles over exactly 256 workgroups (one per
// CU) where TT = 8 leaves 32 CUs idle; the guards `rt < G` fold away for the tiles both sets hold.
template <int CT, int DBG = 0, int NG = 16 * CT, bool NT = false, int TT = 8>
__global__ __launch_bounds__(64 * kNmWaves) void k_nm_mfma(const unsigned char *__restrict__ A,
                                                           const f16 *__restrict__ B, f16 *__restrict__ C,
                                                           uint32_t K, uint32_t S, uint32_t rows,
                                                           uint32_t row_base, uint32_t krot = 0) {
    static_assert(NG == 16 * CT || (CT == 1 && NG == 8), "NG: 16*CT, or 8 in one half-used tile");
    static_assert(TT >= 2 && TT <= 8, "2..8 tiles per workgroup");
    constexpr uint32_t G0 = (TT + 1) / 2, G1 = TT / 2;
    constexpr uint32_t N = NG, RB = 32 * CT, UB = 2 * CT;
    constexpr uint32_t RBG = 2 * NG, UBG = RBG / 16;  // B row bytes / 16-B units in HBM
    constexpr uint32_t szB = kNmKC * RB;
    constexpr uint32_t NTH = 64 * kNmWaves;
    constexpr uint32_t NBU = szB / 16 / NTH;  // 16-B units of B per thread per chunk
    constexpr uint32_t RPU = NTH / UB;        // B rows between a thread's units
    static_assert(szB % (16 * NTH) == 0 && NTH % UB == 0, "whole B units per thread");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t rh = wv >> 2, q = wv & 3u;
    const uint32_t G = rh ? G1 : G0;                             // this wave set's tiles
    const uint32_t r0 = blockIdx.x * 16u * TT + rh * 16u * G0;   // its first row
    const uint32_t BB = 512u + 1024u * G;                        // its block bytes per k-step
    const uint32_t nch = S / 4u;
    // chunk order (krot, as in k_mfma_rows): iteration c works on chunk jr(c), every
    // workgroup starting at its own chunk so they do not all pull the same B rows at once
    const uint32_t rot = krot ? blockIdx.x % nch : 0u;
    auto jr = [&](uint32_t c) -> uint32_t { const uint32_t x = c + rot; return x >= nch ? x - nch : x; };
    const unsigned char *arow = A + (size_t)blockIdx.x * S * nm_wg_block_bytes(TT) + (size_t)rh * S * (512u + 1024u * G0);
    const unsigned char *bbase = reinterpret_cast<const unsigned char *>(B);
    const uint32_t bk = tid / UB, boff = bk * RBG + (tid % UB) * 16u;  // this thread's first unit
    const bool bun = tid % UB < UBG;  // the unit exists in HBM (NG = 8: the tile's upper half is zeros)
    // LDS byte offset of unit i (row bk + i*RPU, 16-B unit tid%UB) in either buffer
    auto bdst = [&](uint32_t i) {
        const uint32_t k = bk + i * RPU, s = tid % UB;
        return k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u;
    };

    u32x4 a0v[4], a1v[4];
    uint2 a0i, a1i;
#define GS_NM_ALOAD(c, V, I)                                                                        \
    if (DBG != 2 || (uint32_t)(c) < 2u) {                                                         \
        const uint32_t cc_ = jr(min((uint32_t)(c), nch - 1u));                                    \
        const unsigned char *blk_ = arow + (size_t)(4u * cc_ + q) * BB;                           \
        const u32x2 i_ = ld_once_if<NT>(reinterpret_cast<const u32x2 *>(blk_ + lane * 8u));      \
        I = make_uint2(i_[0], i_[1]);                                                             \
        _Pragma("unroll") for (int rt = 0; rt < 4; rt++) if ((uint32_t)rt < G) V[rt] =            \
            ld_once_if<NT>(reinterpret_cast<const u32x4 *>(blk_ + 512u + rt * 1024u + lane * 16u)); \
    }
    u32x4 bs[NBU];
    // whole chunks: one lane offset, uniform bases; the last partial chunk clamps rows
#define GS_NM_BLOAD(c)                                                                              \
    if (DBG != 1 || (uint32_t)(c) < 2u) {                                                         \
        const uint32_t k0_ = jr(min((uint32_t)(c), nch - 1u)) * kNmKC;                            \
        if (k0_ + kNmKC <= K) {                                                                   \
            const unsigned char *src_ = bbase + (size_t)k0_ * RBG;                                \
            _Pragma("unroll") for (uint32_t i = 0; i < NBU; i++) bs[i] =                          \
                bun ? *reinterpret_cast<const u32x4 *>(src_ + i * RPU * RBG + boff) : u32x4{0u, 0u, 0u, 0u}; \
        } else {                                                                                  \
            _Pragma("unroll") for (uint32_t i = 0; i < NBU; i++) {                                \
                const uint32_t kk_ = min(k0_ + bk + i * RPU, K - 1u);                             \
                bs[i] = bun ? *reinterpret_cast<const u32x4 *>(bbase + (size_t)kk_ * RBG + (tid % UB) * 16u) \
                            : u32x4{0u, 0u, 0u, 0u};                                              \
            }                                                                                     \
        }                                                                                         \
    }
#define GS_NM_BSTORE(c)                                                                             \
    {                                                                                             \
        const uint32_t k0_ = jr(min((uint32_t)(c), nch - 1u)) * kNmKC;                            \
        unsigned char *lb_ = lds + ((uint32_t)(c) & 1u) * szB;                                    \
        if (k0_ + kNmKC <= K) {                                                                   \
            _Pragma("unroll") for (uint32_t i = 0; i < NBU; i++)                                  \
                *reinterpret_cast<u32x4 *>(lb_ + bdst(i)) = bs[i];                                \
        } else { /* rows past K: zeros */                                                         \
            _Pragma("unroll") for (uint32_t i = 0; i < NBU; i++) {                                \
                const uint32_t z_ = k0_ + bk + i * RPU < K ? ~0u : 0u;                            \
                *reinterpret_cast<u32x4 *>(lb_ + bdst(i)) = bs[i] & z_;                           \
            }                                                                                     \
        }                                                                                         \
    }
    f4v acc[4][CT];
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    // transposed-read offsets of this lane (h = 0..3: k +0/+4/+32/+36 of the step)
    const uint32_t kl = 64u * q + 8u * (lane >> 4) + ((lane & 15u) >> 2);
    // chunk c's k-step for this wave: B rows 64q + [0, 64) of LDS buffer c&1
#define GS_NM_BFRAG(lb_, ct, BF)                                                                    \
    {                                                                                             \
        s4v t_[4];                                                                                \
        _Pragma("unroll") for (int h = 0; h < 4; h++) {                                           \
            const uint32_t k = kl + 32u * (h >> 1) + 4u * (h & 1);                                \
            t_[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(                                      \
                (lds_s4v *)(lb_ + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));         \
        }                                                                                         \
        __builtin_memcpy(&BF, t_, 32);                                                            \
    }
    // B fragments double-buffered in registers: the reads of n-tile ct+1 are in
    // flight while the four smfmac of n-tile ct run.  A wave set with G < 4 tiles runs the
    // smfmac of its missing tiles on whatever their (never loaded) registers hold: no branch
    // splits the issue-ordered region, and those accumulators are never stored
#define GS_NM_COMPUTE(c, V, I)                                                                      \
    {                                                                                             \
        const unsigned char *lb_ = lds + ((uint32_t)(c) & 1u) * szB;                              \
        h8v av_[4];                                                                               \
        _Pragma("unroll") for (int rt = 0; rt < 4; rt++) __builtin_memcpy(&av_[rt], &V[rt], 16);  \
        const int ix0_ = (int)I.x, ix1_ = (int)I.y;                                               \
        h16v bf_[2];                                                                              \
        GS_NM_BFRAG(lb_, 0, bf_[0]);                                                              \
        _Pragma("unroll") for (int ct = 0; ct < CT; ct++) {                                       \
            if (ct + 1 < CT && !(DBG == 8 && ((ct + 1) & 1))) GS_NM_BFRAG(lb_, ct + 1, bf_[(ct + 1) & 1]); \
            const h16v b_ = bf_[ct & 1];                                                          \
            acc[0][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[0], b_, acc[0][ct], ix0_, 0, 0); \
            acc[1][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[1], b_, acc[1][ct], ix0_, 0, 1); \
            acc[2][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[2], b_, acc[2][ct], ix1_, 0, 0); \
            acc[3][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[3], b_, acc[3][ct], ix1_, 0, 1); \
        }                                                                                         \
        /* issue order: reads of n-tile 0, then (reads of ct+1, smfmac of ct) */                  \
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                        \
        _Pragma("unroll") for (int ct = 0; ct < CT; ct++) {                                       \
            if (ct + 1 < CT) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                   \
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                    \
        }                                                                                         \
    }
    // prologue in the loop's steady-state issue order (B of c+1, then A of c+1)
    GS_NM_BLOAD(0u);
    GS_NM_ALOAD(0u, a0v, a0i);
    __builtin_amdgcn_sched_barrier(0);
    GS_NM_BSTORE(0u);
    __builtin_amdgcn_sched_barrier(0);
    GS_NM_BLOAD(nch > 1u ? 1u : 0u);
    __builtin_amdgcn_sched_barrier(0);
    GS_NM_ALOAD(1u, a1v, a1i);
    __syncthreads();
    // iteration c: stage chunk c+1 (its buffer was last read in iteration c-1,
    // before the barrier), fetch B of c+2, compute c, fetch A of c+2
    uint64_t *stl = reinterpret_cast<uint64_t *>(lds + 2 * szB);  // DBG 4 only
#define GS_NM_STAMP(hc, k)                                                                          \
    if constexpr (DBG == 4) {                                                                     \
        if (lane == 0 && (hc) >= 4u && (hc) < 10u) stl[wv * 32u + ((hc) - 4u) * 5u + (k)] = __builtin_amdgcn_s_memtime(); \
    }
    uint32_t c = 0;
    for (; c + 1 < nch; c += 2) {
        GS_NM_BSTORE(c + 1u);
        GS_NM_STAMP(c, 0u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_BLOAD(c + 2u < nch ? c + 2u : c + 1u);
        GS_NM_STAMP(c, 1u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_COMPUTE(c, a0v, a0i);
        GS_NM_STAMP(c, 2u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_ALOAD(c + 2u, a0v, a0i);
        GS_NM_STAMP(c, 3u);
        __syncthreads();
        GS_NM_STAMP(c, 4u);
        GS_NM_BSTORE(c + 2u);  /* past the end: a buffer nobody reads again */
        GS_NM_STAMP(c + 1u, 0u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_BLOAD(c + 3u < nch ? c + 3u : c + 1u);
        GS_NM_STAMP(c + 1u, 1u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_COMPUTE(c + 1u, a1v, a1i);
        GS_NM_STAMP(c + 1u, 2u);
        __builtin_amdgcn_sched_barrier(0);
        GS_NM_ALOAD(c + 3u, a1v, a1i);
        GS_NM_STAMP(c + 1u, 3u);
        __syncthreads();
        GS_NM_STAMP(c + 1u, 4u);
    }
    if constexpr (DBG == 4) {
        __syncthreads();
        if ((blockIdx.x == 0 || blockIdx.x == 100) && lane == 0 && (wv == 0 || wv == 4)) {
            const uint64_t t0 = stl[wv * 32u];
            for (int hc = 0; hc < 6; hc++)
                printf("wg %u wave %u half %d: bstore %llu bload %llu compute %llu aload %llu barrier %llu\n",
                       blockIdx.x, wv, hc + 4, (unsigned long long)(stl[wv * 32u + hc * 5] - t0),
                       (unsigned long long)(stl[wv * 32u + hc * 5 + 1] - t0), (unsigned long long)(stl[wv * 32u + hc * 5 + 2] - t0),
                       (unsigned long long)(stl[wv * 32u + hc * 5 + 3] - t0), (unsigned long long)(stl[wv * 32u + hc * 5 + 4] - t0));
        }
    }
#undef GS_NM_STAMP
    if (c < nch) GS_NM_COMPUTE(c, a0v, a0i);
#undef GS_NM_COMPUTE
#undef GS_NM_BFRAG
#undef GS_NM_BSTORE
#undef GS_NM_BLOAD
#undef GS_NM_ALOAD
    // fixed-order k-phase reduction: pass 1 q2 -> q0, q3 -> q1; pass 2 q1 -> q0
    __syncthreads();
    f4v *red = reinterpret_cast<f4v *>(lds);
    constexpr uint32_t TW = 4 * CT * 64;  // f4v per wave
    if (q >= 2) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[(rh * 2 + (q - 2)) * TW + (rt * CT + ct) * 64 + lane] = acc[rt][ct];
    }
    __syncthreads();
    if (q < 2) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[rt][ct] += red[(rh * 2 + q) * TW + (rt * CT + ct) * 64 + lane];
    }
    __syncthreads();
    if (q == 1) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[rh * TW + (rt * CT + ct) * 64 + lane] = acc[rt][ct];
    }
    __syncthreads();
    if (q == 0) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++) {
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const f4v v = acc[rt][ct] + red[rh * TW + (rt * CT + ct) * 64 + lane];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t r = r0 + rt * 16u + 4u * (lane >> 4) + i;
                    if ((uint32_t)rt < G && r < rows && ct * 16u + (lane & 15u) < N)
                        C[(size_t)(row_base + r) * N + ct * 16u + (lane & 15u)] = (f16)v[i];
                }
            }
        }
    }
}

#ifdef GS_EXPERIMENTS  // opt-in, measured slower than k_nm_mfma (make EXPERIMENTS=1)
// ---------------------------------------------------------------------------
// k_nm_mfma_ks -- the same 2:4 panels (same HBM blocks as k_nm_mfma) with one 64-row
// group per wave, four waves = 256 rows per workgroup and K split over `nsplit`
// workgroups (config C3, N = 128).
// Why: a k_nm_mfma workgroup (128 rows) streams all of B (1.8 MB at N = 128) for its
// 1.0 MB of A, and one CU takes in only ~45-70 GB/s, so B is 64% of every CU's intake
// (C3 runs at 69% of HBM at N = 32 and 40% at N = 128, profiles/r03_n_sweep.json).  Here a
// workgroup owns 256 rows over half of K: B 0.9 MB + A 1.0 MB per CU (-32%).
// One wave per SIMD: each wave holds its 64 x N fp32 tile (4 x CT accumulators, 128
// registers at N = 128, the rest of the 512-register budget for the look-ahead), the A
// blocks of the next 256-column chunk (four k-steps) in registers while it computes the
// current one, and the B chunk is staged through registers by all 256 threads into a
// double-buffered LDS image (b_piece permutation, one raw s_barrier per chunk: global
// loads stay in flight across it).  No cross-wave reduction: every wave owns its rows.
// K split: each wave publishes its fp32 tile (8-B agent-scope stores, its own vmcnt(0),
// then one agent-scope add on its row group's counter); the wave whose add completes the
// count sums the slabs in split order with agent-scope loads and stores C
// (deterministic), then re-arms the counter.
// ---------------------------------------------------------------------------
template <int CT>
__global__ __launch_bounds__(256) void k_nm_mfma_ks(const unsigned char *__restrict__ A,
                                                   const f16 *__restrict__ B, f16 *__restrict__ C, uint32_t K,
                                                   uint32_t S, uint32_t rows, uint32_t row_base, uint32_t nsplit,
                                                   uint32_t ncs, float *__restrict__ slabs,
                                                   uint32_t *__restrict__ arrivals) {
    constexpr uint32_t N = 16 * CT, RB = 32 * CT, UB = 2 * CT;
    constexpr uint32_t szB = kNmKC * RB;
    constexpr uint32_t NTH = 256;
    constexpr uint32_t NBU = szB / 16 / NTH;  // 16-B units of B per thread per chunk
    constexpr uint32_t RPU = NTH / UB;        // B rows between a thread's units
    static_assert(szB % (16 * NTH) == 0 && NTH % UB == 0, "whole B units per thread");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t g = blockIdx.x / nsplit, sp = blockIdx.x - g * nsplit;
    const uint32_t rg = g * 4u + wv;  // this wave's 64-row group
    const uint32_t nch = S / 4u;
    const uint32_t c0 = sp * ncs, ncl = min(nch, c0 + ncs) - c0;  // this workgroup's chunks
    const unsigned char *arow = A + (size_t)rg * S * kNmBlockBytes;
    const unsigned char *bbase = reinterpret_cast<const unsigned char *>(B);
    const uint32_t bk = tid / UB, boff = bk * RB + (tid % UB) * 16u;  // this thread's first unit
    auto bdst = [&](uint32_t i) {
        const uint32_t k = bk + i * RPU, s = tid % UB;
        return k * RB + b_piece<CT>(k, s >> 1) * 32u + (s & 1u) * 16u;
    };
    // the four k-step blocks of chunk c (clamped: past the range re-reads the last)
    auto aload = [&](uint32_t i, u32x4 (&V)[4][4], uint2 (&I)[4]) {
        const uint32_t c = c0 + min(i, ncl - 1u);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const unsigned char *blk = arow + (size_t)(4u * c + q) * kNmBlockBytes;
            I[q] = *reinterpret_cast<const uint2 *>(blk + lane * 8u);
#pragma unroll
            for (int rt = 0; rt < 4; rt++) V[q][rt] = *reinterpret_cast<const u32x4 *>(blk + 512u + rt * 1024u + lane * 16u);
        }
    };
    u32x4 bs[NBU];
    auto bload = [&](uint32_t i) {
        const uint32_t k0 = (c0 + min(i, ncl - 1u)) * kNmKC;
        if (k0 + kNmKC <= K) {
            const unsigned char *src = bbase + (size_t)k0 * RB;
#pragma unroll
            for (uint32_t u = 0; u < NBU; u++) bs[u] = *reinterpret_cast<const u32x4 *>(src + u * RPU * RB + boff);
        } else {
#pragma unroll
            for (uint32_t u = 0; u < NBU; u++) {
                const uint32_t kk = min(k0 + bk + u * RPU, K - 1u);
                bs[u] = *reinterpret_cast<const u32x4 *>(bbase + (size_t)kk * RB + (tid % UB) * 16u);
            }
        }
    };
    auto bstore = [&](uint32_t i) {
        const uint32_t k0 = (c0 + min(i, ncl - 1u)) * kNmKC;
        unsigned char *lb = lds + (i & 1u) * szB;
        if (k0 + kNmKC <= K) {
#pragma unroll
            for (uint32_t u = 0; u < NBU; u++) *reinterpret_cast<u32x4 *>(lb + bdst(u)) = bs[u];
        } else {  // rows past K: zeros
#pragma unroll
            for (uint32_t u = 0; u < NBU; u++) {
                const uint32_t z = k0 + bk + u * RPU < K ? ~0u : 0u;
                *reinterpret_cast<u32x4 *>(lb + bdst(u)) = bs[u] & z;
            }
        }
    };
    f4v acc[4][CT];
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t kl0 = 8u * (lane >> 4) + ((lane & 15u) >> 2);
    auto compute = [&](uint32_t i, const u32x4 (&V)[4][4], const uint2 (&I)[4]) {
        const unsigned char *lb = lds + (i & 1u) * szB;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            h8v av[4];
#pragma unroll
            for (int rt = 0; rt < 4; rt++) __builtin_memcpy(&av[rt], &V[q][rt], 16);
            const int ix0 = (int)I[q].x, ix1 = (int)I[q].y;
            const uint32_t kl = 64u * q + kl0;
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                s4v t[4];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const uint32_t k = kl + 32u * (h >> 1) + 4u * (h & 1);
                    t[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s4v *)(lb + k * RB + b_piece<CT>(k, ct) * 32u + (lane & 3u) * 8u));
                }
                h16v b;
                __builtin_memcpy(&b, t, 32);
                acc[0][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av[0], b, acc[0][ct], ix0, 0, 0);
                acc[1][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av[1], b, acc[1][ct], ix0, 0, 1);
                acc[2][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av[2], b, acc[2][ct], ix1, 0, 0);
                acc[3][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av[3], b, acc[3][ct], ix1, 0, 1);
            }
        }
    };
    // LDS stores of this thread done, then a raw barrier (the look-ahead loads stay in flight)
    auto barrier = [&]() {
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __asm__ volatile("" ::: "memory");
    };
    u32x4 va[4][4], vb[4][4];
    uint2 ia[4], ib[4];
    aload(0, va, ia);
    bload(0);
    bstore(0);
    barrier();
    // chunk i: B of i+1 and A of i+1 in flight while i computes; B of i+1 staged after it
    uint32_t i = 0;
    // (sched_barriers keep the look-ahead loads in front of the MFMAs: the scheduler would
    // otherwise sink them past the compute to shorten register lifetimes)
    for (; i + 1 < ncl; i += 2) {
        bload(i + 1);
        aload(i + 1, vb, ib);
        __builtin_amdgcn_sched_barrier(0);
        compute(i, va, ia);
        __builtin_amdgcn_sched_barrier(0);
        bstore(i + 1);
        barrier();
        bload(i + 2);
        aload(i + 2, va, ia);
        __builtin_amdgcn_sched_barrier(0);
        compute(i + 1, vb, ib);
        __builtin_amdgcn_sched_barrier(0);
        bstore(i + 2);
        barrier();
    }
    if (i < ncl) compute(i, va, ia);
    // the trailing look-ahead loads land in registers only
    const bool live = rg * 64u < rows;
    auto store_tile = [&](const f4v (&v)[4][CT]) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const uint32_t r = rg * 64u + rt * 16u + 4u * (lane >> 4) + e;
                    if (r < rows) C[(size_t)(row_base + r) * N + ct * 16u + (lane & 15u)] = (f16)v[rt][ct][e];
                }
    };
    if (nsplit == 1) {
        if (live) store_tile(acc);
        return;
    }
    if (!live) return;  // a row group past the matrix has no counter traffic
    // K split: this wave's tile -> its slab (8-B agent-scope stores: write-through, and
    // compiler-visible, so the MFMA-result -> store wait states are inserted -- an inline-asm
    // 16-B store of the accumulators read one register before the smfmac had written it),
    // then one add
    constexpr uint32_t TI = 4u * CT * 64u;  // f4v per wave tile
    f4v *slab = reinterpret_cast<f4v *>(slabs) + ((size_t)rg * nsplit + sp) * TI;
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            uint64_t *dst = reinterpret_cast<uint64_t *>(slab + (rt * CT + ct) * 64u + lane);
            uint64_t w[2];
            __builtin_memcpy(w, &acc[rt][ct], 16);
            __hip_atomic_store(dst, w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(dst + 1, w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&arrivals[rg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != nsplit - 1u) return;
    if (lane == 0) __hip_atomic_store(&arrivals[rg], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const f4v *base = reinterpret_cast<const f4v *>(slabs) + (size_t)rg * nsplit * TI;
    f4v sum[4][CT];
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) sum[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    for (uint32_t qq = 0; qq < nsplit; qq++) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                if (qq == sp) {
                    sum[rt][ct] += acc[rt][ct];
                } else {
                    const uint64_t *src = reinterpret_cast<const uint64_t *>(base + (size_t)qq * TI + (rt * CT + ct) * 64u + lane);
                    uint64_t w[2];
                    w[0] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    w[1] = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    f4v x;
                    __builtin_memcpy(&x, w, 16);
                    sum[rt][ct] += x;
                }
            }
    }
    store_tile(sum);
}

#endif  // GS_EXPERIMENTS (k_nm_mfma_ks)

// ---------------------------------------------------------------------------
// k_nm_mfma4 -- the same 2:4 panels (build_nm_panels blocks) for wide B (N = 128, CT = 8),
// with a quarter of k_nm_mfma's B bytes per row.
// Why: a k_nm_mfma workgroup (128 rows, all of K) takes in 1.8 MB of B for its 1.0 MB of A,
// and one CU's intake is the sum of its A (HBM, ~24 GB/s per CU) and B (L2, ~70 GB/s)
// streams (DESIGN §4 model: 43 + 26 us on C3).  Here a workgroup owns 256 rows (four 64-row
// groups) over one of S K ranges: B per CU halves (0.9 MB at S = 2), A per CU is unchanged,
// the grid stays 224 workgroups on C3.
// Waves: 8 = four row groups x two k-phases; wave (rh, q) takes k-steps 4c+q and 4c+q+2 of
// every 256-row chunk c of its range (its 64 x 128 fp32 tile: 128 accumulator registers).
// B chunks go to LDS by LDS-DMA (global_load_lds_dwordx4: no register staging, no LDS store
// cycles; b_piece's XOR rides on the source address), two 64 KB buffers, one chunk ahead;
// A blocks two chunks ahead in registers.  One barrier per chunk.  Epilogue: the two
// k-phase tiles summed through LDS (q0 + q1), then, with S > 1, the tagged-slab K-split
// combine of k_mfma_ks (ks_slab_wait; sums in K-range order: deterministic).  K must be a
// multiple of 256 (whole chunks; the upload checks).
// ---------------------------------------------------------------------------
template <int CT>
__global__ __launch_bounds__(64 * kNmWaves) void k_nm_mfma4(const unsigned char *__restrict__ A,
                                                            const f16 *__restrict__ B, f16 *__restrict__ C,
                                                            uint32_t K, uint32_t S64, uint32_t rows, uint32_t row_base,
                                                            uint32_t S, uint32_t ncs, uint32_t nwg,
                                                            float *__restrict__ slabs, uint32_t *__restrict__ arrivals,
                                                            uint32_t flags) {
    constexpr uint32_t N = 16 * CT, RB = 32 * CT, UB = 2 * CT;
    constexpr uint32_t HR = kNmKC / 2;                       // B rows of a half chunk (two k-steps)
    constexpr uint32_t szH = HR * RB;                         // one ring slot
    constexpr uint32_t NBW = szH / 16u / (64u * kNmWaves);    // LDS-DMA wave-instructions per wave per half
    static_assert(CT == 8 || CT == 4, "k_nm_mfma4: 64- or 128-column tiles");
    static_assert(4 * szH <= 160u * 1024u, "four ring slots");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t rh = wv >> 1, q = wv & 1u;
    const uint32_t u = xcd_block(blockIdx.x, nwg);
    const uint32_t g = u / S, qs = u - g * S;
    const uint32_t rg = g * 4u + rh;
    const uint32_t nch = S64 / 4u, c0 = qs * ncs, nc = min(ncs, nch - c0);  // this range's chunks
    const uint32_t nh = 2u * nc;                                             // ... and half chunks
    const unsigned char *arow = A + (size_t)rg * S64 * kNmBlockBytes;

    // ---- B half chunk h (k-steps 2h, 2h+1 of the range) -> ring slot h & 3 by LDS-DMA:
    // wave-instruction i of wave wv fills the 1 KB at unit (wv*NBW + i)*64 (lane-linear), rows
    // k = (wv*NBW + i)*RPI + lane/UB of the half; the piece permutation rides on the source
    // address.  b_piece's swizzle of row k depends on i only through bit 3 of k (bit 1 of i at
    // RPI = 4 rows per instruction, CT = 8; bit 0 at RPI = 8, CT = 4): two per-lane offsets
    static_assert(64 % UB == 0, "whole B rows per wave-instruction");
    constexpr uint32_t RPI = 64u / UB;
    auto par_of = [](uint32_t i) -> uint32_t { return RPI == 4 ? (i >> 1) & 1u : i & 1u; };
    auto i0_of = [](uint32_t par) -> uint32_t { return RPI == 4 ? 2u * par : par; };
    uint32_t boff[2];
#pragma unroll
    for (uint32_t par = 0; par < 2; par++) {
        const uint32_t k = (wv * NBW + i0_of(par)) * RPI + lane / UB, sp = lane % UB;
        boff[par] = (k * N + (b_piece<CT>(k, sp >> 1) * 2u + (sp & 1u)) * 8u) * 2u;
    }
    auto issue_b = [&](uint32_t h) {
        const unsigned char *src0 = reinterpret_cast<const unsigned char *>(B) + ((size_t)c0 * kNmKC + (size_t)h * HR) * N * 2u;
        unsigned char *buf = lds + (h & 3u) * szH;
#pragma unroll
        for (uint32_t i = 0; i < NBW; i++) {
            const uint32_t par = par_of(i);
            const uint32_t u0 = (wv * NBW + i) * 64u;
            __builtin_amdgcn_global_load_lds((const void *)(src0 + boff[par] + (i - i0_of(par)) * RPI * N * 2u),
                                             (__attribute__((address_space(3))) void *)(buf + u0 * 16u), 16, 0, 0);
        }
    };
    // ---- A block of half h for this wave: k-step 2h + q of the range (positions + four tiles)
    u32x4 av[3][4];
    uint2 ai[3];
#define GS_NM4_ALOAD(h, V, I)                                                                       \
    {                                                                                             \
        const unsigned char *blk_ = arow + (size_t)(4u * c0 + 2u * (h) + q) * kNmBlockBytes;     \
        const u32x2 i_ = ld_once(reinterpret_cast<const u32x2 *>(blk_ + lane * 8u));              \
        I = make_uint2(i_[0], i_[1]);                                                             \
        _Pragma("unroll") for (int rt = 0; rt < 4; rt++) V[rt] =                                  \
            ld_once(reinterpret_cast<const u32x4 *>(blk_ + 512u + rt * 1024u + lane * 16u));      \
    }
    constexpr int NAL = 5;  // vector loads of one A block
    f4v acc[4][CT];
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    // transposed B reads: row k = 64*q + klane + {0, 4, 32, 36} keeps klane's swizzle bits
    // (k & 3 and bit 3: klane & 7 <= 3, so +4 carries nowhere), so piece ct of row k sits at
    // fb[h] ^ (ct << 5) + 64*q*RB, fb[h] = the row's byte offset + its swizzled piece 0
    const uint32_t klane = 8u * (lane >> 4) + ((lane & 15u) >> 2);
    uint32_t fb[4];
#pragma unroll
    for (int hh = 0; hh < 4; hh++) {
        const uint32_t k = klane + 32u * (hh >> 1) + 4u * (hh & 1);
        fb[hh] = 64u * q * RB + k * RB + b_piece<CT>(k, 0) * 32u + (lane & 3u) * 8u;
    }
#define GS_NM4_BFRAG(lb_, ct, BF)                                                                   \
    {                                                                                             \
        s4v t_[4];                                                                                \
        _Pragma("unroll") for (int hh = 0; hh < 4; hh++)                                          \
            t_[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v *)(lb_ + (fb[hh] ^ ((uint32_t)(ct) << 5)))); \
        __builtin_memcpy(&BF, t_, 32);                                                            \
    }
#define GS_NM4_COMPUTE(h, V, I)                                                                     \
    {                                                                                             \
        const unsigned char *lb_ = lds + ((uint32_t)(h) & 3u) * szH;                              \
        h8v av_[4];                                                                               \
        _Pragma("unroll") for (int rt = 0; rt < 4; rt++) __builtin_memcpy(&av_[rt], &V[rt], 16);  \
        const int ix0_ = (int)I.x, ix1_ = (int)I.y;                                               \
        h16v bf_[2];                                                                              \
        GS_NM4_BFRAG(lb_, 0, bf_[0]);                                                             \
        _Pragma("unroll") for (int ct = 0; ct < CT; ct++) {                                       \
            if (ct + 1 < CT) GS_NM4_BFRAG(lb_, ct + 1, bf_[(ct + 1) & 1]);                        \
            const h16v b_ = bf_[ct & 1];                                                          \
            acc[0][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[0], b_, acc[0][ct], ix0_, 0, 0); \
            acc[1][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[1], b_, acc[1][ct], ix0_, 0, 1); \
            acc[2][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[2], b_, acc[2][ct], ix1_, 0, 0); \
            acc[3][ct] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av_[3], b_, acc[3][ct], ix1_, 0, 1); \
        }                                                                                         \
    }
    // prologue: B halves 0, 1 and A blocks 0, 1, 2 in flight; half 0 retired (B(1), A(1), A(2)
    // left in flight: NBW + 2 * NAL loads)
    issue_b(0u);
    GS_NM4_ALOAD(0u, av[0], ai[0]);
    issue_b(1u);  // nh >= 2 (a range holds whole chunks)
    GS_NM4_ALOAD(1u, av[1], ai[1]);
    if (nh > 2u) {
        GS_NM4_ALOAD(2u, av[2], ai[2]);
        __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NBW + 2 * NAL) : "memory");
    } else {
        __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NBW + NAL) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    // half iteration h: B(h+2) -> slot (h+2)&3 (read last in h-2, two barriers ago), compute h,
    // A(h+3) into h's register set, retire B(h+1) and A(h+1) (B(h+2), A(h+2), A(h+3) left in
    // flight), barrier.  B is issued two half iterations ahead, A three.
#define GS_NM4_ITER(h, SET)                                                                         \
    {                                                                                             \
        const bool b2_ = (h) + 2u < nh, a3_ = (h) + 3u < nh;                                      \
        if (b2_) issue_b((h) + 2u);                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        GS_NM4_COMPUTE(h, av[SET], ai[SET]);                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (a3_) GS_NM4_ALOAD((h) + 3u, av[SET], ai[SET]);                                        \
        /* younger than B(h+1) and A(h+1): A(h+2) (if any), B(h+2), A(h+3) */                      \
        if (a3_) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NBW + 2 * NAL) : "memory");         \
        else if (b2_) __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(NBW + NAL) : "memory");        \
        else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");                                 \
        __builtin_amdgcn_s_barrier();                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                        \
    }
    uint32_t h = 0;
    for (; h + 2u < nh; h += 3u) {
        GS_NM4_ITER(h, 0);
        GS_NM4_ITER(h + 1u, 1);
        GS_NM4_ITER(h + 2u, 2);
    }
    if (h < nh) GS_NM4_ITER(h, 0);
    if (h + 1u < nh) GS_NM4_ITER(h + 1u, 1);
#undef GS_NM4_ITER
#undef GS_NM4_COMPUTE
#undef GS_NM4_BFRAG
#undef GS_NM4_ALOAD
    // ---- K-split ticket (wave 0), then the two k-phase tiles summed in LDS: q1 -> q0
    uint32_t *arr = arrivals + g;
    uint32_t ticket = 0;
    if (S > 1 && wv == 0 && lane == 0) ticket = __hip_atomic_fetch_add(arr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f4v *red = reinterpret_cast<f4v *>(lds);
    constexpr uint32_t TW = 4 * CT * 64;  // f4v per wave tile
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds + 4u * TW * 16u);  // (nm4_lds_bytes: after the tiles)
    if (q == 1u) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) red[rh * TW + (rt * CT + ct) * 64u + lane] = acc[rt][ct];
    }
    if (S > 1 && wv == 0 && lane == 0) *flag = ticket;
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
    if (q == 1u) return;
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[rt][ct] += red[rh * TW + (rt * CT + ct) * 64u + lane];
    auto store_c = [&](int rt, int ct, const f4v &v) {
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t r = rg * 64u + rt * 16u + 4u * (lane >> 4) + i;
            if (r < rows) C[(size_t)(row_base + r) * N + ct * 16u + (lane & 15u)] = (f16)v[i];
        }
    };
    if (S == 1) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) store_c(rt, ct, acc[rt][ct]);
        return;
    }
    // ---- tagged-slab combine (k_mfma_ks's protocol): slab of unit u = [rh][rt][ct][lane] f4v
    const uint32_t tk = *flag & 0xffffu, tag = ((*flag >> 16) & 1u) ^ 1u;
    auto tagged = [&](const f4v &v) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        w[0] = (w[0] & ~1u) | tag; w[1] = (w[1] & ~1u) | tag; w[2] = (w[2] & ~1u) | tag; w[3] = (w[3] & ~1u) | tag;
        return w;
    };
    f4v *slab = reinterpret_cast<f4v *>(slabs) + (size_t)u * 4u * TW + rh * TW;
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            const u32x4 w = tagged(acc[rt][ct]);
            __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(slab + (rt * CT + ct) * 64u + lane), "v"(w) : "memory");
        }
    if (tk != S - 1u) return;
    if (wv == 0 && lane == 0) __hip_atomic_store(arr, tag << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t *err = arrivals + nwg / S;  // the replica's device error word
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            f4v sum = {0.f, 0.f, 0.f, 0.f};
            for (uint32_t qq = 0; qq < S; qq++) {
                u32x4 w;
                if (qq == qs) {
                    w = tagged(acc[rt][ct]);
                } else {
                    const f4v *src = reinterpret_cast<const f4v *>(slabs) + (size_t)(g * S + qq) * 4u * TW + rh * TW +
                                     (rt * CT + ct) * 64u + lane;
                    w = ks_slab_wait(reinterpret_cast<const uint32_t *>(src), tag, err, GS_KS_FORCE(flags));
                }
                w[0] &= ~1u; w[1] &= ~1u; w[2] &= ~1u; w[3] &= ~1u;
                f4v x;
                __builtin_memcpy(&x, &w, 16);
                sum += x;
            }
            store_c(rt, ct, sum);
        }
}
// k_permute_rows -- B into a merge-path plan's column order (MP_COL_PERM): row i of Bp is row
// perm[i] of B (perm: the original column of renumbered column i, most nonzeros first), read
// by a gather; SCATTER: perm[i] is the new place of column i, B read in order and each row
// written to its place.  16 B per thread when a row is whole 16-B units, one element otherwise.
template <class VT, bool SCATTER>
__global__ __launch_bounds__(256) void k_permute_rows(const VT *__restrict__ B, VT *__restrict__ Bp,
                                                      const uint32_t *__restrict__ perm, uint32_t K, uint32_t N) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    if ((N * sizeof(VT)) % 16u == 0) {
        const uint32_t upr = N * (uint32_t)sizeof(VT) / 16u;
        const uint64_t total = (uint64_t)K * upr;
        for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < total; t += stride) {
            const uint32_t i = (uint32_t)(t / upr), u = (uint32_t)(t - (uint64_t)i * upr);
            if constexpr (SCATTER)
                reinterpret_cast<u32x4 *>(Bp)[(size_t)perm[i] * upr + u] = reinterpret_cast<const u32x4 *>(B)[t];
            else
                reinterpret_cast<u32x4 *>(Bp)[t] = reinterpret_cast<const u32x4 *>(B)[(size_t)perm[i] * upr + u];
        }
    } else {
        const uint64_t total = (uint64_t)K * N;
        for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < total; t += stride) {
            const uint32_t i = (uint32_t)(t / N), j = (uint32_t)(t - (uint64_t)i * N);
            if constexpr (SCATTER)
                Bp[(size_t)perm[i] * N + j] = B[t];
            else
                Bp[t] = B[(size_t)perm[i] * N + j];
        }
    }
}

// ---------------------------------------------------------------------------
// k_merge_path -- merge-path levels (merge_path_{thread,warp,tblock}_operator +
// the level's total-reduce token).  The plan's
// level starts (first_row_indices_without_ending / first_nz_indices,
// get_begin_{rows,nzs}_of_level_after_merge_path.cc) are decoded on the host
// into nz-exact wave ranges [wz[w], wz[w+1]) (gsk_host::merge_path_layout);
// rows are the non-empty rows in compact order: ends[j] = their CSR row ends,
// rid[j] = their output rows.  A wave walks its range in rounds of 8*S
// nonzeros (S = 64/X slots of X column lanes, 8 consecutive nonzeros per slot,
// one 16/32-B load of cols and of vals, all 8 B-row gathers in flight):
//   1. the rows closing in the round are staged in the wave's LDS and mark a
//      row-start flag per position (flag at e - zb for every row end e);
//   2. each slot walks its 8 positions with the flags as a bit mask: a run
//      that starts and closes inside the slot is stored at once; the slot's
//      head run (continuing from the left) is held back; its tail run is the
//      slot's carry;
//   3. a segmented scan over slots (stop = any row start/close in the slot)
//      gives every slot its carry-in; held-back heads add it and are stored;
//      the last slot's scan value is carried into the next round.
// Empty rows are zeroed from a list by the kernel's first fill_blocks
// workgroups, concurrently with the path waves (no memset of C, no extra
// launch).  Rows crossing waves: the wave the row is open at the end of writes
// its partial to rec[w], the wave that closes it writes its own partial to
// head_rec instead of C.  With `chain` (one column tile) the partials are
// combined in the same launch: every contributing wave publishes its partial
// with agent-scope (L2 write-through) stores, waits for them, and bumps the
// closing wave's arrival counter; the last arriver reads the chain's partials
// back in wave order, stores the row (one rounding, deterministic) and re-arms
// the counter.  No wave waits on another, so any dispatch order is safe.
// Without `chain`, rec_row[w] names the open row and k_merge_fixup sums them.
// ---------------------------------------------------------------------------
constexpr uint32_t kMpItems = 8;  // nonzeros per slot per round

// Rows split across waves, combined in the launch.  A partial is published to part[src]
// with agent-scope stores (written through the XCD's L2); its arrival (the X lanes of
// one slot; lane0 = the slot's first lane) waits for the wave's stores, then the slot's
// first lane bumps the closing wave's counter.  The arrival that completes the chain
// (parts = close - first + 1) sums rec[first .. close-1] and head_rec[close] in wave
// order with agent-scope loads, writes the row and re-arms the counter.
// Ordering: every access of the hand-off is an agent-scope atomic (sc1: written through
// to / read from the memory-side coherence point, no stale XCD-L2 copy), and the
// publisher's vmcnt(0) retires its stores before its counter add is issued; the reader
// loads only after its add returned the completing count (a control dependency).  That
// is MI355X_MICROARCH.md §Workgroup dispatch's hand-off form.  The language-level form
// (acq_rel on the add) is not used: on gfx950 an agent-scope release is a
// buffer_wbl2 sc1 (write-back of the XCD's whole L2) and the acquire a buffer_inv sc1,
// per arrival -- measured C4 merge_path(1024) 49 -> 84 us, r03 session 1.
template <int CF>
__device__ __forceinline__ void merge_chain_publish(const float (&a)[CF], float *part, uint32_t src, uint32_t N,
                                                    uint32_t c0, bool cok) {
    if (cok) {
#pragma unroll
        for (int k = 0; k < CF; k++)
            __hip_atomic_store(part + (size_t)src * N + c0 + k, a[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <class VT, int CF>
__device__ __forceinline__ void merge_chain_arrive(uint32_t close, uint32_t first, const float *rec, const float *head_rec,
                                                   uint32_t *cnt, uint32_t row, VT *C, uint32_t N, uint32_t c0, bool cok,
                                                   uint32_t lane0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if ((threadIdx.x & 63u) == lane0) old = __hip_atomic_fetch_add(cnt + close, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, (int)lane0, 64);
    if (old + 1u != close - first + 1u) return;
    if (cok) {
        float s[CF];
#pragma unroll
        for (int k = 0; k < CF; k++) s[k] = 0.f;
        for (uint32_t v = first; v < close; v++) {
#pragma unroll
            for (int k = 0; k < CF; k++)
                s[k] += __hip_atomic_load(rec + (size_t)v * N + c0 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < CF; k++)
            s[k] += __hip_atomic_load(head_rec + (size_t)close * N + c0 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        store_f32<VT, CF>(C + (size_t)row * N + c0, s);
    }
    if ((threadIdx.x & 63u) == lane0) __hip_atomic_store(cnt + close, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per wave: row-start flags (bytes 0..8S) and the staged output rows rid_l (cap + 2)
__host__ __device__ constexpr uint32_t merge_path_wave_lds_words(uint32_t S) {
    return (kMpItems * S) / 4u + 2u + (kMpItems * S + 64u) + 2u;
}

// STAMPS (diagnostic build only, gs_debug_mfma_timeline on a merge-path plan): lane 0 of
// every path wave records s_memtime into stamps[w * 16 + slot]: 0 start, 1 first loads
// issued, per round r < 4: 2 + 3r gathers issued, 3 + 3r rows staged, 4 + 3r walked and
// scanned; 14 loop done, 15 end (chain arrival)
template <class VT, class CT, int CF, bool STAMPS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_merge_path(const uint32_t *__restrict__ wz,   // n_waves+1
                                                    const uint32_t *__restrict__ wq,   // n_waves+1
                                                    const uint32_t *__restrict__ ends, // n_crow
                                                    const uint32_t *__restrict__ rid,  // n_crow
                                                    uint32_t n_crow, const CT *__restrict__ col,
                                                    const VT *__restrict__ val, const VT *__restrict__ B,
                                                    VT *__restrict__ C, float *__restrict__ rec,
                                                    uint32_t *__restrict__ rec_row, float *__restrict__ head_rec,
                                                    uint32_t n_waves, uint32_t N, uint32_t X, uint32_t row_lo,
                                                    uint32_t row_hi, const uint32_t *__restrict__ empty_rows,
                                                    uint32_t n_empty, uint32_t fill_blocks,
                                                    const uint32_t *__restrict__ chain,  // 2 n_waves or null
                                                    uint32_t *__restrict__ chain_cnt,    // n_waves, zero between launches
                                                    uint32_t dbg = 0, uint64_t *__restrict__ stamps = nullptr) {
    // dbg (diagnostic timing runs only, wrong results): bit 1 gathers B row 0 for every nonzero;
    // experiments build: bit 8 skips the slot scans (row-start prefix and the segmented carry
    // scan), bit 16 treats every position as inside a row (no row closes or emits in a round)
    const uint32_t lb = blockIdx.x;  // (XCD-contiguous numbering measured no faster cold on C4)
    if (lb < fill_blocks) {
        // the first fill_blocks workgroups zero the empty rows (listed; 16-B stores when a
        // C row is whole 16-B units) while the path waves run
        const uint32_t rbytes = N * (uint32_t)sizeof(VT);
        const uint32_t U = rbytes % 16u == 0 ? rbytes / 16u : N;
        const uint32_t tot = blockIdx.y == 0 ? n_empty * U : 0u;  // one column-tile row of blocks fills
        for (uint32_t i = lb * blockDim.x + threadIdx.x; i < tot; i += fill_blocks * blockDim.x) {
            const uint32_t er = empty_rows[i / U];
            if (rbytes % 16u == 0)
                *reinterpret_cast<uint4 *>(reinterpret_cast<unsigned char *>(C) + (size_t)er * rbytes + (i % U) * 16u) =
                    make_uint4(0u, 0u, 0u, 0u);
            else
                C[(size_t)er * N + i % U] = (VT)0.f;
        }
        return;
    }
    extern __shared__ uint32_t mp_lds[];
    const uint32_t lane = threadIdx.x & 63u, wib = threadIdx.x >> 6;
    const uint32_t xl = lane & (X - 1u), slot = lane / X, S = 64u / X;
    const uint32_t R8 = kMpItems * S;     // nonzeros per round
    const uint32_t fw = R8 / 4u + 2u;     // flag words: bytes 0..R8
    const uint32_t cap = R8 + 64u;        // staged rows per round
    uint32_t *wl = mp_lds + wib * merge_path_wave_lds_words(S);
    unsigned char *flags = reinterpret_cast<unsigned char *>(wl);
    uint32_t *rid_l = wl + fw;            // rid[qs - 1 + k]
    const uint32_t waves_total = (gridDim.x - fill_blocks) * (blockDim.x >> 6);
    typedef typename raw_vec<CF * sizeof(VT)>::t RB;
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t w = (lb - fill_blocks) * (blockDim.x >> 6) + wib; w < n_waves; w += waves_total) {
#define GS_MP_STAMP(slot)                                                                          \
    if constexpr (STAMPS) {                                                                        \
        if (lane == 0 && blockIdx.y == 0) stamps[(size_t)w * 16u + (slot)] = __builtin_amdgcn_s_memtime(); \
    }
            GS_MP_STAMP(0u);
            const uint32_t zlo = wz[w], wend = wz[w + 1], q0 = wq[w];
            uint32_t rnd = 0;
            // the wave starts inside row q0 (its partial goes to head_rec)
            const bool head_open = zlo > (q0 ? ends[q0 - 1] : 0u);
            const uint32_t head_first = chain && head_open ? chain[n_waves + w] : 0u;
            uint32_t qs = q0;
            float rc[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) rc[k] = 0.f;
            bool closed_end = false;
            bool head_done = false;  // chain mode: this slot published the head row's partial
            auto emit = [&](uint32_t qq, const float (&a)[CF]) {
                if (qq == q0 && head_open) {
                    if (chain) {  // published now (agent-scope stores), arrives after the walk
                        merge_chain_publish<CF>(a, head_rec, w, N, c0, cok);
                        head_done = true;
                        return;
                    }
                    if (!cok) return;
#pragma unroll
                    for (int k = 0; k < CF; k++) head_rec[(size_t)w * N + c0 + k] = a[k];
                } else {
                    if (!cok) return;
                    store_f32<VT, CF>(C + (size_t)rid_l[qq - qs + 1u] * N + c0, a);
                }
            };
            // software pipeline: round r+1's A entries and first staging batch are loaded
            // while round r walks; round r's gathers are issued before that prefetch, so
            // waiting for them leaves the prefetch in flight
            CT cn[kMpItems];
            VT vn[kMpItems];
            // the next round's first kMpPref x 64 rows (ends, output rows), prefetched a round
            // ahead; rows past the prefetched batches are loaded synchronously.  (Two batches,
            // for rounds of ~3-nonzero rows that close ~85 rows: C4 51.0 against 49.2 us.)
            constexpr uint32_t kMpPref = 1;
            uint32_t en[kMpPref], rn[kMpPref];
            auto load_a = [&](uint32_t zb_) {
                const uint32_t b_ = zb_ + kMpItems * slot;
                if (b_ < wend) {
                    load_raw<CT, kMpItems>(col + b_, cn);
                    load_raw<VT, kMpItems>(val + b_, vn);
                } else {
#pragma unroll
                    for (uint32_t k = 0; k < kMpItems; k++) { cn[k] = 0; vn[k] = (VT)0.f; }
                }
            };
            auto load_s = [&](uint32_t q_) {  // the first kMpPref x 64 rows a round stages
#pragma unroll
                for (uint32_t b = 0; b < kMpPref; b++) {
                    const uint32_t j = q_ + 64u * b + lane;
                    en[b] = j < n_crow ? ends[j] : 0xffffffffu;
                    rn[b] = j < n_crow ? rid[j] : 0u;
                }
            };
            const uint32_t zb0 = zlo & ~(kMpItems - 1u);
            load_a(zb0);
            load_s(qs);
            GS_MP_STAMP(1u);
            for (uint32_t zb = zb0; zb < wend; zb += R8) {
                const uint32_t zl = max(zb, zlo), ze = min(zb + R8, wend);
                const uint32_t base = zb + kMpItems * slot;
                CT cc[kMpItems];
                VT vv[kMpItems];
#pragma unroll
                for (uint32_t k = 0; k < kMpItems; k++) { cc[k] = cn[k]; vv[k] = vn[k]; }
                RB braw[kMpItems];  // all gathers of the round in flight before the walk
#pragma unroll
                for (uint32_t k = 0; k < kMpItems; k++) {
                    const uint32_t z = base + k;
                    const bool valid = z >= zl && z < ze;
                    braw[k] = *reinterpret_cast<const RB *>(B + (size_t)(valid && !(dbg & 2u) ? (uint32_t)cc[k] : 0u) * N + c0);
                }
                if (rnd < 4u) GS_MP_STAMP(2u + 3u * rnd);
                for (uint32_t i = lane; i < fw; i += 64u) wl[i] = 0u;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // stage the rows closing in this round and the one open at its end
                uint32_t nclose = 0;
                closed_end = false;
                uint32_t e = en[0], r = rn[0];
                for (uint32_t k0 = 0;; k0 += 64u) {
                    if (k0 && k0 < 64u * kMpPref) {
#pragma unroll
                        for (uint32_t b = 1; b < kMpPref; b++)
                            if (k0 == 64u * b) { e = en[b]; r = rn[b]; }
                    } else if (k0) {  // rows beyond the prefetched batches (short rows): synchronous
                        const uint32_t j = qs + k0 + lane;
                        e = j < n_crow ? ends[j] : 0xffffffffu;
                        r = j < n_crow ? rid[j] : 0u;
                    }
                    if (k0 + lane < cap) rid_l[k0 + lane + 1u] = r;
                    if (e > zl && e <= ze) flags[e - zb] = 1;
                    nclose += (uint32_t)__builtin_popcountll(__ballot(e <= ze));
                    closed_end = closed_end || __ballot(e == ze) != 0ull;
                    if (__ballot(e >= ze) != 0ull || k0 + 64u >= cap) break;
                }
                if (zb + R8 < wend) {
                    load_a(zb + R8);
                    load_s(qs + nclose);
                }
                if (rnd < 4u) GS_MP_STAMP(3u + 3u * rnd);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // this slot's row starts: bit k = position 8*slot + k (bit 8: the next slot's first)
                const uint32_t fo = kMpItems * slot;
                const uint2 f8 = *reinterpret_cast<const uint2 *>(flags + fo);
                uint32_t bits = (uint32_t)flags[fo + kMpItems] << 8;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) bits |= ((f8.x >> (8 * k)) & 1u) << k | ((f8.y >> (8 * k)) & 1u) << (k + 4);
#ifdef GS_EXPERIMENTS
                if (dbg & 16u) bits = 0u;
                const bool scans = !(dbg & 8u);
#else
                constexpr bool scans = true;
#endif
                const uint32_t pc = (uint32_t)__builtin_popcount(bits & 0xffu);
                uint32_t incl = pc;
                if (scans) {
#pragma unroll
                    for (uint32_t st = 0; st < 6; st++) {
                        const uint32_t off = X << st;
                        if (off >= 64u) break;
                        const uint32_t t = __shfl_up(incl, off, 64);
                        if (lane >= off) incl += t;
                    }
                }
                uint32_t qcur = qs + incl - pc;  // row open before this slot's first position
                float acc[CF], h[CF];
#pragma unroll
                for (int k = 0; k < CF; k++) { acc[k] = 0.f; h[k] = 0.f; }
                bool has_h = false, in_head = true;
                uint32_t hq = 0;
                const bool head_cont = !(bits & 1u);
                auto close = [&](uint32_t qq) {
                    if (in_head && head_cont) {
                        has_h = true;
                        hq = qq;
#pragma unroll
                        for (int k = 0; k < CF; k++) h[k] = acc[k];
                    } else {
                        emit(qq, acc);
                    }
                };
#pragma unroll
                for (uint32_t k = 0; k < kMpItems; k++) {
                    if ((bits >> k) & 1u) {
                        if (k > 0) close(qcur);
                        qcur++;
                        in_head = false;
#pragma unroll
                        for (int i = 0; i < CF; i++) acc[i] = 0.f;
                    }
                    const uint32_t z = base + k;
                    if (z >= zl && z < ze) {
                        VT bt[CF];
                        __builtin_memcpy(bt, &braw[k], sizeof(RB));
                        const float v = (float)vv[k];
#pragma unroll
                        for (int i = 0; i < CF; i++) acc[i] = __builtin_fmaf(v, (float)bt[i], acc[i]);
                    }
                }
                if ((bits >> kMpItems) & 1u) {
                    close(qcur);
#pragma unroll
                    for (int i = 0; i < CF; i++) acc[i] = 0.f;
                }
                // segmented inclusive scan of the slots' carries (stop: the slot starts or closes a row)
                uint32_t stop = bits != 0u;
                if (slot == 0 && !stop) {
#pragma unroll
                    for (int i = 0; i < CF; i++) acc[i] += rc[i];
                }
#pragma unroll
                for (uint32_t st = 0; st < 6; st++) {
                    const uint32_t off = X << st;
                    if (off >= 64u || !scans) break;
                    const uint32_t ts = __shfl_up(stop, off, 64);
                    float t[CF];
#pragma unroll
                    for (int i = 0; i < CF; i++) t[i] = __shfl_up(acc[i], off, 64);
                    if (lane >= off) {
                        if (!stop) {
#pragma unroll
                            for (int i = 0; i < CF; i++) acc[i] += t[i];
                        }
                        stop |= ts;
                    }
                }
                float cin[CF];
#pragma unroll
                for (int i = 0; i < CF; i++) {
                    const float t = __shfl_up(acc[i], X, 64);
                    cin[i] = slot ? t : rc[i];
                }
                if (has_h) {
#pragma unroll
                    for (int i = 0; i < CF; i++) h[i] += cin[i];
                    emit(hq, h);
                }
#pragma unroll
                for (int i = 0; i < CF; i++) rc[i] = __shfl(acc[i], (S - 1u) * X + xl, 64);
                qs += nclose;
                if (rnd < 4u) GS_MP_STAMP(4u + 3u * rnd);
                rnd++;
                __builtin_amdgcn_wave_barrier();
            }
            GS_MP_STAMP(14u);
            // the row open at the wave's end (if any): its partial joins the row's chain
            if (chain) {
                if (head_done)  // the slot that closed the head row
                    merge_chain_arrive<VT, CF>(w, head_first, rec, head_rec, chain_cnt, rid[q0], C, N, c0, cok, lane - xl);
                if (!closed_end && slot == 0) {
                    const uint32_t cw_ = chain[w];  // the wave closing the row
                    merge_chain_publish<CF>(rc, rec, w, N, c0, cok);
                    merge_chain_arrive<VT, CF>(cw_, chain[n_waves + cw_], rec, head_rec, chain_cnt, rid[qs], C, N, c0, cok,
                                               0u);
                }
            } else {
                if (lane == 0) rec_row[w] = closed_end ? 0xffffffffu : rid[qs];
                if (!closed_end && slot == 0 && cok) {
#pragma unroll
                    for (int k = 0; k < CF; k++) rec[(size_t)w * N + c0 + k] = rc[k];
                }
            }
            GS_MP_STAMP(15u);
#undef GS_MP_STAMP
        }
    }
}

#ifdef GS_EXPERIMENTS  // opt-in, measured slower than k_merge_path (make EXPERIMENTS=1)
// ---------------------------------------------------------------------------
// k_merge_rows -- the same merge-path plan (wave ranges wz/wq, compact rows
// ends/rid, split-row chains) with a two-phase walk per round of R = S*J
// nonzeros instead of k_merge_path's flag/scan machinery:
//   1. products: slot s owns the J consecutive nonzeros zb + s*J .. (one vector
//      load of cols and of vals, J B-row gathers in flight), multiplies them and
//      writes the fp32 products (X*CF columns per nonzero) to the wave's LDS;
//   2. rows: the rows meeting the round are dealt to the slots, S at a time; a
//      slot adds its row's products from LDS (rows of more than `solo` products
//      are summed by the whole wave, slot-strided, one xor-shuffle reduction)
//      and stores the row.  The row left open at the round's end carries its
//      partial into the next round's first row.
// Row bounds come from two 64-row batches of `ends` loaded at the wave's start
// (exchanged with shuffles; rows past them are loaded directly).  The head row
// (open at zlo) and the tail row (open at zhi) join the row's chain exactly as
// in k_merge_path (agent-scope publish, last arriver combines), or go to
// head_rec / rec + rec_row for k_merge_fixup when the launch has several column
// tiles.  Deterministic: every row is summed in a fixed order.
// ---------------------------------------------------------------------------
template <int CF>
__host__ __device__ constexpr uint32_t merge_rows_j() { return CF >= 8 ? 4u : 8u; }
// fp32 words of one wave's product buffer: R entries of X*CF words + 4 words per slot group
__host__ __device__ constexpr uint32_t merge_rows_wave_words(uint32_t X, uint32_t CF, uint32_t J) {
    return (64u / X) * J * X * CF + (64u / X) * 4u;
}

template <class VT, class CT, int CF>
__global__ __launch_bounds__(256) void k_merge_rows(const uint32_t *__restrict__ wz,   // n_waves+1
                                                    const uint32_t *__restrict__ wq,   // n_waves+1
                                                    const uint32_t *__restrict__ ends, // n_crow
                                                    const uint32_t *__restrict__ rid,  // n_crow
                                                    uint32_t n_crow, const CT *__restrict__ col,
                                                    const VT *__restrict__ val, const VT *__restrict__ B,
                                                    VT *__restrict__ C, float *__restrict__ rec,
                                                    uint32_t *__restrict__ rec_row, float *__restrict__ head_rec,
                                                    uint32_t n_waves, uint32_t N, uint32_t X,
                                                    const uint32_t *__restrict__ empty_rows, uint32_t n_empty,
                                                    uint32_t fill_blocks,
                                                    const uint32_t *__restrict__ chain,  // 2 n_waves or null
                                                    uint32_t *__restrict__ chain_cnt,    // n_waves, zero between launches
                                                    uint32_t solo) {
    constexpr uint32_t J = merge_rows_j<CF>();
    const uint32_t lb = blockIdx.x;
    if (lb < fill_blocks) {  // empty rows, as in k_merge_path
        const uint32_t rbytes = N * (uint32_t)sizeof(VT);
        const uint32_t U = rbytes % 16u == 0 ? rbytes / 16u : N;
        const uint32_t tot = blockIdx.y == 0 ? n_empty * U : 0u;
        for (uint32_t i = lb * blockDim.x + threadIdx.x; i < tot; i += fill_blocks * blockDim.x) {
            const uint32_t er = empty_rows[i / U];
            if (rbytes % 16u == 0)
                *reinterpret_cast<uint4 *>(reinterpret_cast<unsigned char *>(C) + (size_t)er * rbytes + (i % U) * 16u) =
                    make_uint4(0u, 0u, 0u, 0u);
            else
                C[(size_t)er * N + i % U] = (VT)0.f;
        }
        return;
    }
    extern __shared__ float mr_lds[];
    const uint32_t lane = threadIdx.x & 63u, wib = threadIdx.x >> 6;
    const uint32_t xl = lane & (X - 1u), slot = lane / X, S = 64u / X;
    const uint32_t R = S * J, TW = X * CF;
    float *P = mr_lds + wib * merge_rows_wave_words(X, CF, J);
    // float offset of product entry e (this lane's columns); 4 words of padding per slot group
    auto pofs = [&](uint32_t e) { return e * TW + (e / J) * 4u + xl * CF; };
    const uint32_t waves_total = (gridDim.x - fill_blocks) * (blockDim.x >> 6);
    const uint64_t slot_bits = X >= 64u ? ~0ull : ((1ull << X) - 1ull);
    typedef typename raw_vec<CF * sizeof(VT)>::t RB;
    for (uint32_t ct = blockIdx.y; ct * X * CF < N; ct += gridDim.y) {
        const uint32_t cw = ct * X * CF + xl * CF;
        const bool cok = cw < N;
        const uint32_t c0 = cok ? cw : 0u;
        for (uint32_t w = (lb - fill_blocks) * (blockDim.x >> 6) + wib; w < n_waves; w += waves_total) {
            const uint32_t zlo = wz[w], zhi = wz[w + 1], q0 = wq[w], qn = wq[w + 1];
            const uint32_t zb0 = zlo & ~(J - 1u);
            // A entries of the first round, and the first 128 rows' ends
            CT cn[J];
            VT vn[J];
            auto load_a = [&](uint32_t zb_) {
                const uint32_t b_ = zb_ + J * slot;
                if (b_ < zhi) {
                    load_raw<CT, (int)J>(col + b_, cn);
                    load_raw<VT, (int)J>(val + b_, vn);
                } else {
#pragma unroll
                    for (uint32_t k = 0; k < J; k++) { cn[k] = 0; vn[k] = (VT)0.f; }
                }
            };
            load_a(zb0);
            const uint32_t e0 = q0 + lane < n_crow ? ends[q0 + lane] : 0xffffffffu;
            const uint32_t e1 = q0 + 64u + lane < n_crow ? ends[q0 + 64u + lane] : 0xffffffffu;
            const uint32_t sq0 = q0 ? ends[q0 - 1u] : 0u;
            // end of wave row i (row q0 + i); i may differ per lane
            auto row_end = [&](uint32_t i) -> uint32_t {
                const uint32_t a0 = (uint32_t)__shfl((int)e0, (int)(i & 63u), 64);
                const uint32_t a1 = (uint32_t)__shfl((int)e1, (int)(i & 63u), 64);
                if (i < 64u) return a0;
                if (i < 128u) return a1;
                return q0 + i < n_crow ? ends[q0 + i] : 0xffffffffu;
            };
            const bool head_open = zlo > sq0;
            const uint32_t q_last = (qn < n_crow && (qn ? ends[qn - 1] : 0u) < zhi) ? qn : qn - 1u;
            const bool tail_open = ends[q_last] > zhi;
            bool head_mine = false;
            float carry[CF];
#pragma unroll
            for (int k = 0; k < CF; k++) carry[k] = 0.f;
            uint32_t qi0 = 0;  // wave row index of the round's first row
            for (uint32_t zb = zb0; zb < zhi; zb += R) {
                const uint32_t zl = max(zb, zlo), ze = min(zb + R, zhi);
                CT cc[J];
                VT vv[J];
#pragma unroll
                for (uint32_t k = 0; k < J; k++) { cc[k] = cn[k]; vv[k] = vn[k]; }
                RB braw[J];
#pragma unroll
                for (uint32_t k = 0; k < J; k++) {
                    const uint32_t z = zb + J * slot + k;
                    const bool valid = z >= zl && z < ze;
                    braw[k] = *reinterpret_cast<const RB *>(B + (size_t)(valid ? (uint32_t)cc[k] : 0u) * N + c0);
                }
                if (zb + R < zhi) load_a(zb + R);
#pragma unroll
                for (uint32_t k = 0; k < J; k++) {
                    const uint32_t z = zb + J * slot + k;
                    const float v = (z >= zl && z < ze) ? (float)vv[k] : 0.f;
                    VT bt[CF];
                    __builtin_memcpy(bt, &braw[k], sizeof(RB));
                    float pr[CF];
#pragma unroll
                    for (int i = 0; i < CF; i++) pr[i] = v * (float)bt[i];
                    float *dst = P + pofs(J * slot + k);
                    if constexpr (CF % 4 == 0) {
#pragma unroll
                        for (int i = 0; i < CF; i += 4)
                            *reinterpret_cast<float4 *>(dst + i) = make_float4(pr[i], pr[i + 1], pr[i + 2], pr[i + 3]);
                    } else {
#pragma unroll
                        for (int i = 0; i < CF; i++) dst[i] = pr[i];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // rows meeting [zl, ze), S at a time
                for (uint32_t bi = qi0;; bi += S) {
                    const uint32_t i = bi + slot;
                    const uint32_t q = q0 + i;
                    // (both shuffles with every lane active: a shuffle reads only active lanes)
                    const uint32_t en_ = row_end(i), st_ = row_end(i ? i - 1u : 0u);
                    const uint32_t en = q < n_crow ? en_ : 0xffffffffu;
                    const uint32_t st = i == 0u ? sq0 : st_;
                    const bool active = q < n_crow && st < ze;
                    const uint32_t rs = active ? max(st, zl) - zb : 0u, re = active ? min(en, ze) - zb : 0u;
                    const bool is_long = re - rs > solo;
                    float acc[CF];
#pragma unroll
                    for (int k = 0; k < CF; k++) acc[k] = 0.f;
                    if (active && !is_long) {
                        for (uint32_t e = rs; e < re; e++) {
                            const float *src = P + pofs(e);
#pragma unroll
                            for (int k = 0; k < CF; k++) acc[k] += src[k];
                        }
                    }
                    uint64_t lm = __ballot(is_long);
                    while (lm) {  // long rows: the whole wave, slot-strided, one at a time
                        const uint32_t l = (uint32_t)__builtin_ctzll(lm);
                        lm &= ~(slot_bits << l);
                        const uint32_t lrs = (uint32_t)__shfl((int)rs, (int)l, 64), lre = (uint32_t)__shfl((int)re, (int)l, 64);
                        float a2[CF];
#pragma unroll
                        for (int k = 0; k < CF; k++) a2[k] = 0.f;
                        for (uint32_t e = lrs + slot; e < lre; e += S) {
                            const float *src = P + pofs(e);
#pragma unroll
                            for (int k = 0; k < CF; k++) a2[k] += src[k];
                        }
                        wave_reduce_slots<CF>(a2, (int)X);
                        if (slot == l / X) {
#pragma unroll
                            for (int k = 0; k < CF; k++) acc[k] = a2[k];
                        }
                    }
                    if (bi == qi0 && slot == 0u) {  // the row carried in from the previous round
#pragma unroll
                        for (int k = 0; k < CF; k++) acc[k] += carry[k];
                    }
                    const bool closes = active && en <= ze;
                    if (closes) {
                        if (q == q0 && head_open) {
                            if (chain) {
                                merge_chain_publish<CF>(acc, head_rec, w, N, c0, cok);
                                head_mine = true;
                            } else if (cok) {
#pragma unroll
                                for (int k = 0; k < CF; k++) head_rec[(size_t)w * N + c0 + k] = acc[k];
                            }
                        } else if (cok) {
                            store_f32<VT, CF>(C + (size_t)rid[q] * N + c0, acc);
                        }
                    }
                    const uint64_t om = __ballot(active && !closes);  // the row left open at ze
                    const uint64_t am = __ballot(active);
                    if (om) {
                        const uint32_t l = (uint32_t)__builtin_ctzll(om);
#pragma unroll
                        for (int k = 0; k < CF; k++) carry[k] = __shfl(acc[k], (int)((l & ~(X - 1u)) + xl), 64);
                        qi0 = bi + l / X;
                        break;
                    }
                    if (am != ~0ull) {  // the round's rows are done; the next round opens a new row
#pragma unroll
                        for (int k = 0; k < CF; k++) carry[k] = 0.f;
                        qi0 = bi + (uint32_t)__builtin_popcountll(am) / X;
                        break;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            // carry = the tail row's partial when the wave ends inside a row
            if (chain) {
                if (head_mine && !(head_open && tail_open && q_last == q0))
                    merge_chain_arrive<VT, CF>(w, chain[n_waves + w], rec, head_rec, chain_cnt, rid[q0], C, N, c0, cok,
                                               lane - xl);
                if (tail_open && slot == 0u) {
                    const uint32_t cw_ = chain[w];  // the wave closing the row
                    merge_chain_publish<CF>(carry, rec, w, N, c0, cok);
                    merge_chain_arrive<VT, CF>(cw_, chain[n_waves + cw_], rec, head_rec, chain_cnt, rid[q_last], C, N, c0,
                                               cok, 0u);
                }
            } else {
                if (lane == 0) rec_row[w] = tail_open ? rid[q_last] : 0xffffffffu;
                if (tail_open && slot == 0u && cok) {
#pragma unroll
                    for (int k = 0; k < CF; k++) rec[(size_t)w * N + c0 + k] = carry[k];
                }
            }
        }
    }
}

#endif  // GS_EXPERIMENTS (k_merge_rows)
// rows open across waves: C[r] = (sum of the open partials in wave order) + the
// closing wave's partial, rounded once
template <class VT>
__global__ __launch_bounds__(256) void k_merge_fixup(const uint32_t *__restrict__ rec_row,
                                                     const float *__restrict__ rec,
                                                     const float *__restrict__ head_rec, VT *__restrict__ C,
                                                     uint32_t n_waves, uint32_t N) {
    const uint32_t total = n_waves * N;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const uint32_t g = e / N, c = e % N;
        // every load of the common case (a chain of <= 8 waves) is issued at once, before
        // any of them is tested: one memory latency instead of a chain of dependent ones
        // (the records were written by other XCDs' waves in the previous kernel)
        const uint32_t r = rec_row[g];
        const uint32_t rp = g > 0 ? rec_row[g - 1] : 0xffffffffu;
        uint32_t rr[8];
        float v[8], hv[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const bool in = g + k < n_waves, in1 = g + k + 1 < n_waves;
            rr[k] = in ? rec_row[g + k] : 0xffffffffu;
            v[k] = in ? rec[(size_t)(g + k) * N + c] : 0.f;
            hv[k] = in1 ? head_rec[(size_t)(g + k + 1) * N + c] : 0.f;
        }
        if (r == 0xffffffffu || rp == r) continue;
        // sum the open partials in wave order, then the closing wave's head partial
        float s = 0.f;
        uint32_t h = g;
        bool open = true;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (open && rr[k] == r) {
                s += v[k];
                h++;
            } else {
                open = false;
            }
        }
        while (open) {  // chains past 8 waves (long rows): 8 waves per step
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const bool in = h + k < n_waves;
                rr[k] = in ? rec_row[h + k] : 0xffffffffu;
                v[k] = in ? rec[(size_t)(h + k) * N + c] : 0.f;
            }
            const uint32_t h0 = h;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (open && rr[k] == r) {
                    s += v[k];
                    h++;
                } else {
                    open = false;
                }
            }
            if (h == h0) open = false;
        }
        if (h < n_waves) s += h - g <= 8 ? hv[h - g - 1] : head_rec[(size_t)h * N + c];
        C[(size_t)r * N + c] = (VT)s;
    }
}

}  // namespace gsk

// ---------------------------------------------------------------------------
// Host-side helpers shared by the library (kernels/device_plan.hip) and the
// programs code_generator emits: the kernel-side layouts derived from plan
// arrays.
// ---------------------------------------------------------------------------
#include <string>
#include <vector>

namespace gsk_host {

// CSR row pointer (u32) of a row-sorted COO row array
inline std::vector<uint32_t> csr_row_ptr(const std::vector<uint64_t> &row, uint64_t row_num) {
    std::vector<uint32_t> rp(row_num + 1, 0);
    for (uint64_t r : row) rp[r + 1]++;
    for (uint64_t i = 0; i < row_num; i++) rp[i + 1] += rp[i];
    return rp;
}

// per fixed-nnz BMT, bit i set iff its i-th nz starts a row (no forced BMW heads)
inline std::vector<uint64_t> row_start_masks(const std::vector<uint64_t> &row, const std::vector<uint64_t> &first_nz) {
    std::vector<uint64_t> mask(first_nz.size() - 1, 0);
    for (size_t i = 0; i + 1 < first_nz.size(); i++) {
        uint64_t mm = 0;
        for (uint64_t j = first_nz[i]; j < first_nz[i + 1]; j++)
            if (j == 0 || row[j] != row[j - 1]) mm |= 1ull << (j - first_nz[i]);
        mask[i] = mm;
    }
    return mask;
}

// k_row_chunks: BMTs per wave (enough waves to fill 256 CUs eight deep)
inline uint32_t row_chunk_span(size_t n_bmt) {
    const size_t u = (n_bmt + 8191) / 8192;
    return (uint32_t)(u < 8 ? 8 : u);
}

// rows k_row_chunks leaves to k_finalize_rows: rows without BMTs and rows whose
// BMTs straddle two waves' ranges (output rows = row_base + plan row)
inline std::vector<uint32_t> row_chunk_finalize_rows(const std::vector<uint32_t> &bmt_row, uint64_t M, uint32_t U,
                                                     uint32_t row_base) {
    std::vector<uint8_t> fin(M, 1);
    for (uint32_t r : bmt_row) fin[r + row_base] = 0;
    for (size_t i = U; i < bmt_row.size(); i += U)
        if (bmt_row[i] == bmt_row[i - 1]) fin[bmt_row[i] + row_base] = 1;
    std::vector<uint32_t> list;
    for (uint64_t r = 0; r < M; r++)
        if (fin[r]) list.push_back((uint32_t)r);
    return list;
}

// k_merge_path: nz-exact wave ranges from the plan's merge-path levels, and the
// compact non-empty rows.  Level w starts at path step p = w*work_size; the
// reference records (row j's index, p - j) for the first non-empty row j with
// total_path[j] > p (get_begin_{rows,nzs}_of_level_after_merge_path.cc:84-94).
// total_path[j] = ends[j] + j, so p == ends[j-1] + j - 1 is the step that
// closes row j-1: the nonzeros consumed there are ends[j-1] = (p - j) + 1;
// otherwise p - j.  Consecutive levels are grouped into waves of at least
// target_steps path steps; waves never have an empty nz range.  snap > 0: a wave
// boundary strictly inside a row of at most `snap` nonzeros moves to the nearer end of
// that row, so the row is summed by one wave (no cross-wave combine for it; the
// reference's own merge path splits such rows over threads and adds them atomically).
struct merge_path_layout {
    std::vector<uint32_t> wz, wq, ends, rid, empty;  // empty: output rows without nonzeros
    // rows split across waves: chain[w] = the wave closing the row open at w's end,
    // chain[W + w] = the first wave of the row w closes at its head (~0: none)
    std::vector<uint32_t> chain;
};

// the split-row chains of a layout (k_merge_path's in-launch combine)
inline void merge_path_chains(merge_path_layout &L) {
    const size_t W = L.wz.size() - 1;
    L.chain.assign(2 * W, 0xffffffffu);
    uint32_t start = 0xffffffffu;
    size_t q_last = 0;
    for (size_t w = 0; w < W; w++) {
        const uint32_t zlo = L.wz[w], zhi = L.wz[w + 1], q0 = L.wq[w];
        const bool head_open = zlo > (q0 ? L.ends[q0 - 1] : 0u);
        q_last = std::max<size_t>(q_last, q0);
        while (L.ends[q_last] < zhi) q_last++;  // the row holding position zhi - 1
        const bool end_open = L.ends[q_last] > zhi;
        const bool through = head_open && end_open && q_last == q0;  // the row spans the whole wave
        if (head_open && !through) {
            L.chain[W + w] = start;
            for (uint32_t v = start; v < w; v++) L.chain[v] = (uint32_t)w;
            start = 0xffffffffu;
        }
        if (end_open && !through) start = (uint32_t)w;
    }
}

inline bool merge_path_device_layout(const std::vector<uint64_t> &row, uint64_t row_num,
                                     const std::vector<uint64_t> &lvl_rows, const std::vector<uint64_t> &lvl_nzs,
                                     uint64_t work_size, uint32_t row_base, uint64_t target_steps,
                                     merge_path_layout &out, std::string &why, uint64_t out_rows = 0,
                                     uint64_t snap = 0) {
    out = merge_path_layout();
    std::vector<uint32_t> cnt(row_num, 0);
    for (uint64_t r : row) {
        if (r >= row_num) { why = "row index beyond the row count"; return false; }
        cnt[r]++;
    }
    std::vector<uint64_t> crow;  // plan row of compact row j
    uint64_t acc = 0;
    for (uint64_t r = 0; r < row_num; r++)
        if (cnt[r]) {
            acc += cnt[r];
            if (acc > 0xffffffffull) { why = "nnz exceeds 32 bits"; return false; }
            out.ends.push_back((uint32_t)acc);
            out.rid.push_back((uint32_t)(r + row_base));
            crow.push_back(r);
        } else {
            out.empty.push_back((uint32_t)(r + row_base));
        }
    for (uint64_t r = row_base + row_num; r < out_rows; r++) out.empty.push_back((uint32_t)r);
    const uint64_t R = crow.size();
    if (R == 0 || lvl_rows.empty() || lvl_nzs.size() != lvl_rows.size() + 1 || lvl_nzs.back() != acc || work_size == 0) {
        why = "merge-path level arrays do not match the matrix";
        return false;
    }
    uint64_t j = 0, gz = 0, gp = 0;
    out.wz.push_back(0);
    out.wq.push_back(0);
    for (uint64_t w = 0; w < lvl_rows.size(); w++) {
        while (j < R && crow[j] < lvl_rows[w]) j++;
        const uint64_t p = w * work_size;
        if (j == R || crow[j] != lvl_rows[w] || p < j || lvl_nzs[w] != p - j) {
            why = "merge-path level " + std::to_string(w) + " is not on the path";
            return false;
        }
        uint64_t z = (j >= 1 && p == (uint64_t)out.ends[j - 1] + j - 1) ? (uint64_t)out.ends[j - 1] : p - j;
        uint64_t q = j;
        if (w == 0 || p - gp < target_steps) continue;
        if (snap && q < R) {
            const uint64_t rs = q ? out.ends[q - 1] : 0, re = out.ends[q];
            if (z > rs && re - rs <= snap) {
                if (z - rs <= re - z) {
                    z = rs;
                } else {
                    z = re;
                    q++;
                }
            }
        }
        if (z <= gz || z >= acc) continue;
        out.wz.push_back((uint32_t)z);
        out.wq.push_back((uint32_t)q);
        gz = z;
        gp = p;
    }
    out.wz.push_back((uint32_t)acc);
    out.wq.push_back((uint32_t)R);
    merge_path_chains(out);
    return true;
}

}  // namespace gsk_host
