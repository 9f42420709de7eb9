// gather_launch.hip -- launches of the CUDA-core gather families (k_thread_total,
// k_warp_rows, k_block_rows, k_bitmap_segment, k_row_chunks, k_merge_path) and the
// LDS-staged k_lds_rows (hip_code/kernel_lib.hpp).
#include "../hip_code/kernel_lib.hpp"
#include "../host/gs_plan.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>

namespace gs {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) throw gs_error(std::string(#x) + ": " + hipGetErrorString(e_), -3); \
    } while (0)

namespace {

constexpr int kLdsMaxU = 12;  // 16-B staging registers per thread (k_lds_rows MAXU; device_plan.hip sizes the tiles)

#ifdef GS_EXPERIMENTS
uint64_t *g_mp_stamps = nullptr;  // set by debug_mp_timeline for one launch (diagnostic build only)
#endif

// GS_MP_DEBUG (diagnostic timing only): k_merge_path dbg bits
uint32_t mp_debug() {
#ifdef GS_EXPERIMENTS
    static const uint32_t v = getenv("GS_MP_DEBUG") ? (uint32_t)atoi(getenv("GS_MP_DEBUG")) : 0u;
    return v;
#else
    return 0u;
#endif
}

uint32_t pow2ceil(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

template <class VT, int CF>
void launch_lds(const plan_state &p, const device_arrays &a, const VT *B, VT *C, uint32_t N, hipStream_t s) {
    const device_plan &d = p.dev;
    const uint32_t X = N * (uint32_t)sizeof(VT) / 16u;
    const uint32_t nb = (uint32_t)d.n_rows_aux;
    const uint32_t ksp = d.ksplit > 1 ? d.ksplit : 1u;
    GS_CHECK(ksp == 1 || (a.ws && a.t3 && d.ncs > 0 && (ksp - 1) * d.ncs < d.nc), "k_lds_rows: K ranges disagree with the upload");
    const dim3 grid(nb * ksp), block(64 * d.waves);
    const uint32_t K = (uint32_t)p.K;
#define GS_LDS_ARGS                                                                                              \
    a.t0, a.a1, a.a0, a.t1, a.t2, (const uint16_t *)a.tcol, (const VT *)a.tval, B, C, K, N, X, d.KC, d.nc, d.RSB, \
        d.rpw_max, d.seg_cap, (uint32_t)d.row_base, ksp, d.ncs, a.ws, a.t3
    auto go = [&](auto kern) {
        // dynamic LDS above 64 KB must be opted into, once per kernel and device
        static std::mutex mu;
        static std::map<std::pair<int, const void *>, size_t> granted;
        {
            std::lock_guard<std::mutex> l(mu);
            size_t &g = granted[{d.device, reinterpret_cast<const void *>(kern)}];
            if (g < d.lds_bytes) {
                HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)d.lds_bytes));
                g = d.lds_bytes;
            }
        }
        hipLaunchKernelGGL(kern, grid, block, d.lds_bytes, s, GS_LDS_ARGS);
    };
    if constexpr (sizeof(VT) == 4 && CF == 4) {
        if (d.lds_dma) {  // LDS_DMA: fp32 N = 32, chunks by LDS-DMA into two buffers
            GS_CHECK(N == 32, "k_lds_rows_dma is built for N = 32");
            auto gd = [&](auto kern) {
                static std::mutex mu;
                static std::map<std::pair<int, const void *>, size_t> granted;
                {
                    std::lock_guard<std::mutex> l(mu);
                    size_t &g = granted[{d.device, reinterpret_cast<const void *>(kern)}];
                    if (g < d.lds_bytes) {
                        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)d.lds_bytes));
                        g = d.lds_bytes;
                    }
                }
                hipLaunchKernelGGL(kern, grid, block, d.lds_bytes, s, a.t0, a.a1, a.a0, a.t1, a.t2, (const uint16_t *)a.tcol,
                                   (const float *)a.tval, (const float *)B, (float *)C, K, d.KC, d.nc, d.rpw_max, d.seg_cap,
                                   (uint32_t)d.row_base, ksp, d.ncs, a.ws, a.t3);
            };
            if (d.maxr == 8) gd(gsk::k_lds_rows_rs<1>);  // one row per slot (BMWs of 5..8 rows)
            else if (d.maxr == 1) gd(gsk::k_lds_rows_dma<1>);
            else if (d.maxr == 2) gd(gsk::k_lds_rows_dma<2>);
            else gd(gsk::k_lds_rows_dma<4>);
            return;
        }
    }
    GS_CHECK(!d.lds_dma, "k_lds_rows_dma: fp32 plans at N = 32 only");
    if (d.maxr == 1) go(gsk::k_lds_rows<VT, CF, 1, kLdsMaxU>);
    else if (d.maxr == 2) go(gsk::k_lds_rows<VT, CF, 2, kLdsMaxU>);
    else go(gsk::k_lds_rows<VT, CF, 4, kLdsMaxU>);
#undef GS_LDS_ARGS
}

template <class VT, class CT, int CF, int SCF>
void launch_family(const plan_state &p, const device_arrays &a, const VT *B, VT *C, uint32_t N, hipStream_t s) {
    const device_plan &d = p.dev;
    const kernel_spec &sp = p.cg->get_kernel_spec();
    const uint32_t X = std::min<uint32_t>(64u, pow2ceil((N + CF - 1) / CF));
    const uint32_t tiles = (N + X * CF - 1) / (X * CF);
    const uint32_t row_base = (uint32_t)d.row_base;
    const CT *col = (const CT *)a.col;
    const VT *val = (const VT *)a.val;
    switch (sp.family) {
        case KF_THREAD_TOTAL: {
            uint32_t groups = 256 / X;
            uint32_t gx = (uint32_t)std::min<uint64_t>((d.n_rows_aux + groups - 1) / groups, 1u << 16);
            hipLaunchKernelGGL((gsk::k_thread_total<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256), 0,
                               s, a.a0, d.f0, a.a1, d.f1, col, val, B, C, (uint32_t)d.n_units, (uint32_t)d.n_rows_aux, N, X,
                               row_base);
            break;
        }
        case KF_WARP_TOTAL: {
            if constexpr (CF * sizeof(VT) == 16) {
                if (d.lds && N == d.lds_N) {
                    launch_lds<VT, CF>(p, a, B, C, N, s);
                    break;
                }
            }
            uint32_t gx;
            if (sp.tblock_parent) gx = (uint32_t)d.n_rows_aux;
            else gx = (uint32_t)std::min<uint64_t>((d.n_units + 3) / 4, 1u << 16);
            // slots per row: enough for the plan's mean row in WARP_ROWS_CHUNKS SCF-chunks per slot
            // (taken in one pass: one gather round trip), the rest of the wave on the next rows of
            // the BMW (only when BMWs hold several rows)
            uint32_t G = 64u / X, nch = 1;
            if (d.bmw_rows_max > 1 && get_config().WARP_ROWS_GROUPS) {
                nch = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(gsk::kWarpRowsMaxChunks, get_config().WARP_ROWS_CHUNKS));
                const uint32_t need = (uint32_t)std::max<double>(1.0, std::ceil(d.mean_row_nnz / (4.0 * nch)));
                G = std::min<uint32_t>(G, pow2ceil(need));
            }
            bool mc = false;
            if constexpr (SCF <= 4 && CF * sizeof(VT) == 16 && sizeof(VT) == 4 && sizeof(CT) == 2) {  // spill-free at 128 VGPRs
                if (nch > 1) {  // several chunks per slot and pass: the 128-VGPR multi-chunk kernel
                    hipLaunchKernelGGL((gsk::k_warp_rows_mc<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256), 0, s,
                                       a.a0, d.f0, sp.tblock_parent ? a.a1 : nullptr, sp.tblock_parent ? d.f1 : gsk::idx_formula(), a.a2, col,
                                       val, B, C, (uint32_t)d.n_units, N, X, row_base, G, nch);
                    mc = true;
                }
            }
            if (!mc) {
                // one chunk per slot and pass: slots per row for the mean row in one chunk each
                if (nch > 1) {
                    nch = 1;
                    if (d.bmw_rows_max > 1 && get_config().WARP_ROWS_GROUPS)
                        G = std::min<uint32_t>(64u / X, pow2ceil((uint32_t)std::max<double>(1.0, std::ceil(d.mean_row_nnz / 4.0))));
                }
                hipLaunchKernelGGL((gsk::k_warp_rows<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256), 0, s,
                                   a.a0, d.f0, sp.tblock_parent ? a.a1 : nullptr, sp.tblock_parent ? d.f1 : gsk::idx_formula(), a.a2, col, val, B, C, (uint32_t)d.n_units, N,
                                   X, row_base, G);
            }
            break;
        }
        case KF_BLOCK_TOTAL: {
            uint32_t gx = (uint32_t)std::min<uint64_t>(d.n_units, 1u << 16);
            hipLaunchKernelGGL((gsk::k_block_rows<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256), 0, s,
                               a.a0, d.f0, a.a2, col, val, B, C, (uint32_t)d.n_units, N, X, row_base);
            break;
        }
        case KF_BITMAP_SEGMENT: {
            const uint32_t S = 64 / X;
            uint32_t gx = (uint32_t)std::min<uint64_t>((d.n_units + 4 * S - 1) / (4 * S), 1u << 16);
            size_t lds = (size_t)4 * S * 2 * X * CF * sizeof(float);
            // the fp32 workspace is sized for the plan's dense width; other widths use fp16 atomics
            const bool use_ws = a.ws && N == d.ws_n;
            if (!use_ws)
                HIP_OK(hipMemsetAsync(C + (size_t)d.out_lo * N, 0, (size_t)(d.n_out_rows - d.out_lo) * N * sizeof(VT), s));
            hipLaunchKernelGGL((gsk::k_bitmap_segment<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256),
                               lds, s, a.a0, d.f0, a.a1, d.f1, a.m0, a.a2, a.a3, col, val, B, C, (uint32_t)d.n_units, N, X,
                               row_base, use_ws ? a.ws : (float *)nullptr);
            if (use_ws && d.n_fin) {
                HIP_OK(hipGetLastError());
                const uint32_t fx = (uint32_t)std::min<uint64_t>((d.n_fin * N + 255) / 256, 4096);
                hipLaunchKernelGGL((gsk::k_finalize_rows<VT>), dim3(fx), dim3(256), 0, s, a.a4, (uint32_t)d.n_fin,
                                   a.ws, C, N);
            }
            break;
        }
        case KF_ROW_CHUNKS: {
            GS_CHECK(N <= d.ws_n, "col-direction plan built for N=" + std::to_string(d.ws_n) +
                                      ": its workspace holds no wider B (re-run the pipeline for this N)");
            const uint32_t nw = (uint32_t)((d.n_units + d.span - 1) / d.span);
            const uint32_t gx = std::min<uint32_t>((nw + 3) / 4, 1u << 16);
            hipLaunchKernelGGL((gsk::k_row_chunks<VT, CT, CF, SCF>), dim3(std::max(gx, 1u), tiles), dim3(256), 0, s,
                               a.a0, d.f0, a.a1, d.f1, col, val, B, C, a.ws, (uint32_t)d.n_units, d.span, N, X, row_base, d.ilv,
                               a.a2, a.a3);
            if (d.n_fin) {
                HIP_OK(hipGetLastError());
                const uint32_t fx = (uint32_t)std::min<uint64_t>((d.n_fin * N + 255) / 256, 4096);
                hipLaunchKernelGGL((gsk::k_finalize_rows<VT>), dim3(fx), dim3(256), 0, s, a.a4, (uint32_t)d.n_fin,
                                   a.ws, C, N);
            }
            break;
        }
        case KF_MERGE_PATH: {
            GS_CHECK(N <= d.ws_n, "merge-path plan built for N=" + std::to_string(d.ws_n) +
                                      ": its carry buffers hold no wider B (re-run the pipeline for this N)");
            const uint32_t S = 64u / X;
            const size_t lds = (size_t)4 * gsk::merge_path_wave_lds_words(S) * sizeof(uint32_t);
            const uint32_t W = (uint32_t)d.n_units;
            const uint32_t gx = std::min<uint32_t>((W + 3) / 4, 1u << 16);
            GS_CHECK(d.n_fin * (uint64_t)N < 0xffffffffull, "merge-path empty-row fill exceeds 32-bit indices");
            const uint32_t fb = d.n_fin ? (uint32_t)std::min<uint64_t>(256, (d.n_fin * N / 4 + 1023) / 1024) : 0u;
            // one column tile: split rows are combined inside the launch (chain arrivals)
            const bool fused = tiles == 1 && !(mp_debug() & 4u);
            if (d.mp_parts > 1) {
                // MP_COL_PARTS: B gathered into partition order, one merge-path pass per column
                // partition (part 0 into C, the others into their fp32 outputs), then C += them
                GS_CHECK(fused && sizeof(VT) == 4 && a.pp.size() == (size_t)d.mp_parts * kMpPartPtrs && a.cperm && a.bperm,
                         "merge-path column partitions: fp32, one column tile, arrays uploaded");
                const uint64_t units = (uint64_t)p.K * N * sizeof(VT) / (N * sizeof(VT) % 16 == 0 ? 16u : sizeof(VT));
                const uint32_t pb = (uint32_t)std::min<uint64_t>((units + 255) / 256, 8192);
                hipLaunchKernelGGL((gsk::k_permute_rows<VT, false>), dim3(std::max(pb, 1u)), dim3(256), 0, s, B,
                                   (VT *)a.bperm, a.cperm, (uint32_t)p.K, N);
                HIP_OK(hipGetLastError());
                gsk::mp_part_outs outs{};
                for (uint32_t x = 0; x < d.mp_parts; x++) {
                    void *const *pp = &a.pp[(size_t)x * kMpPartPtrs];
                    const uint32_t Wx = d.mp_part_W[x], nfin = d.mp_part_fin[x];
                    const uint32_t gxx = std::min<uint32_t>((Wx + 3) / 4, 1u << 16);
                    const uint32_t fbx = nfin ? (uint32_t)std::min<uint64_t>(256, ((uint64_t)nfin * N / 4 + 1023) / 1024) : 0u;
                    VT *Cx = x == 0 ? C : (VT *)pp[MP_PART_OUT];
                    if (x > 0) outs.p[x - 1] = (const float *)pp[MP_PART_OUT];
                    hipLaunchKernelGGL((gsk::k_merge_path<VT, CT, CF>),
                                       dim3(gxx + fbx, 1), dim3(256), lds, s,
                                       (const uint32_t *)pp[MP_PART_WZ], (const uint32_t *)pp[MP_PART_WQ],
                                       (const uint32_t *)pp[MP_PART_ENDS], (const uint32_t *)pp[MP_PART_RID],
                                       d.mp_part_rows[x], (const CT *)pp[MP_PART_COL], (const VT *)pp[MP_PART_VAL],
                                       (const VT *)a.bperm, Cx, (float *)pp[MP_PART_WS], (uint32_t *)pp[MP_PART_T0],
                                       (float *)pp[MP_PART_WS2], Wx, N, X, row_base, (uint32_t)d.n_out_rows,
                                       (const uint32_t *)pp[MP_PART_EMPTY], nfin, fbx, (const uint32_t *)pp[MP_PART_CHAIN],
                                       (uint32_t *)pp[MP_PART_CNT], mp_debug(), nullptr);
                    HIP_OK(hipGetLastError());
                }
                const uint64_t total = (uint64_t)d.n_out_rows * N;
                const uint32_t ab = (uint32_t)std::min<uint64_t>((total + 255) / 256, 8192);
                hipLaunchKernelGGL((gsk::k_add_parts<VT>), dim3(std::max(ab, 1u)), dim3(256), 0, s, C, outs, d.mp_parts - 1, total);
                HIP_OK(hipGetLastError());
                break;
            }
            if (d.col_perm) {  // B into the plan's column order first (MP_COL_PERM, upload_csr)
                GS_CHECK(a.cperm && a.bperm, "merge-path column permutation without its device arrays");
                const uint64_t units = (uint64_t)p.K * N * sizeof(VT) / (N * sizeof(VT) % 16 == 0 ? 16u : sizeof(VT));
                const uint32_t pb = (uint32_t)std::min<uint64_t>((units + 255) / 256, 8192);
                if (d.perm_scatter)
                    hipLaunchKernelGGL((gsk::k_permute_rows<VT, true>), dim3(std::max(pb, 1u)), dim3(256), 0, s, B,
                                       (VT *)a.bperm, a.cperm, (uint32_t)p.K, N);
                else
                    hipLaunchKernelGGL((gsk::k_permute_rows<VT, false>), dim3(std::max(pb, 1u)), dim3(256), 0, s, B,
                                       (VT *)a.bperm, a.cperm, (uint32_t)p.K, N);
                HIP_OK(hipGetLastError());
                B = (const VT *)a.bperm;
            }
#ifdef GS_EXPERIMENTS
            if (d.mp_rows)
                hipLaunchKernelGGL((gsk::k_merge_rows<VT, CT, CF>), dim3(gx + fb, tiles), dim3(256),
                                   (size_t)4 * gsk::merge_rows_wave_words(X, CF, gsk::merge_rows_j<CF>()) * sizeof(float), s, a.a0,
                                   a.a1, a.a2, a.a3, (uint32_t)d.n_rows_aux, col, val, B, C, a.ws, a.t0, a.ws2, W, N, X,
                                   a.a4, (uint32_t)d.n_fin, fb, fused ? a.t1 : nullptr, fused ? a.t2 : nullptr,
                                   d.mp_solo);
            else
#else
            GS_CHECK(!d.mp_rows, "k_merge_rows is an experiments-build kernel");
#endif
#ifdef GS_EXPERIMENTS
            if (g_mp_stamps)
                    hipLaunchKernelGGL((gsk::k_merge_path<VT, CT, CF, true>), dim3(gx + fb, tiles), dim3(256), lds, s, a.a0, a.a1,
                                   a.a2, a.a3, (uint32_t)d.n_rows_aux, col, val, B, C, a.ws, a.t0, a.ws2, W, N, X, row_base,
                                   (uint32_t)d.n_out_rows, a.a4, (uint32_t)d.n_fin, fb, fused ? a.t1 : nullptr,
                                   fused ? a.t2 : nullptr, mp_debug(), g_mp_stamps);
            else
#endif
                    hipLaunchKernelGGL((gsk::k_merge_path<VT, CT, CF>),
                                   dim3(gx + fb, tiles), dim3(256), lds, s, a.a0, a.a1,
                                   a.a2, a.a3, (uint32_t)d.n_rows_aux, col, val, B, C, a.ws, a.t0, a.ws2, W, N, X, row_base,
                                   (uint32_t)d.n_out_rows, a.a4, (uint32_t)d.n_fin, fb, fused ? a.t1 : nullptr,
                                   fused ? a.t2 : nullptr, mp_debug(), nullptr);
            HIP_OK(hipGetLastError());
            if (fused) break;
            GS_CHECK((uint64_t)W * N < 0xffffffffull, "merge-path fix-up indices exceed 32 bits");
            const uint32_t fx = (uint32_t)std::min<uint64_t>(((uint64_t)W * N + 255) / 256, 1u << 16);
            hipLaunchKernelGGL((gsk::k_merge_fixup<VT>), dim3(std::max(fx, 1u)), dim3(256), 0, s, a.t0, a.ws, a.ws2, C,
                               W, N);
            break;
        }
        default:
            throw gs_error("no kernel family");
    }
    HIP_OK(hipGetLastError());
}

// compile-time shapes: CF = dense columns per lane (16 B of B when N allows),
// SCF = sparse entries per A load (16 B for the wave families; the plan's row
// alignment for thread_total)
template <class VT, class CT, int CF>
void dispatch_scf(const plan_state &p, const device_arrays &a, const VT *b, VT *c, uint32_t N, hipStream_t s) {
    constexpr int VEC = 16 / sizeof(VT);
    const kernel_spec &sp = p.cg->get_kernel_spec();
    if (sp.family == KF_THREAD_TOTAL) {
        if (p.dev.scf >= 8) launch_family<VT, CT, CF, 8>(p, a, b, c, N, s);
        else if (p.dev.scf >= 4) launch_family<VT, CT, CF, 4>(p, a, b, c, N, s);
        else launch_family<VT, CT, CF, 1>(p, a, b, c, N, s);
    } else {
        launch_family<VT, CT, CF, VEC>(p, a, b, c, N, s);
    }
}

template <class VT, int CFV>
void dispatch_vt(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    const VT *b = (const VT *)B;
    VT *c = (VT *)C;
    const bool vec = (N % CFV) == 0;
    if (p.dev.col_bytes == 2) {
        if (vec) dispatch_scf<VT, uint16_t, CFV>(p, a, b, c, N, s);
        else dispatch_scf<VT, uint16_t, 1>(p, a, b, c, N, s);
    } else {
        if (vec) dispatch_scf<VT, uint32_t, CFV>(p, a, b, c, N, s);
        else dispatch_scf<VT, uint32_t, 1>(p, a, b, c, N, s);
    }
}

}  // namespace


void launch_gather(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    if (p.dev.dtype == 0) dispatch_vt<float, 4>(p, a, B, C, N, s);
    else dispatch_vt<gsk::f16, 8>(p, a, B, C, N, s);
}

#ifdef GS_EXPERIMENTS
// diagnostic: one merge-path launch with s_memtime stamps per path wave (kernel_lib.hpp)
void debug_mp_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host) {
    const size_t n = (size_t)p.dev.n_units * 16;
    uint64_t *dst = nullptr;
    HIP_OK(hipMalloc(&dst, n * 8));
    HIP_OK(hipMemsetAsync(dst, 0, n * 8, s));
    g_mp_stamps = dst;
    try {
        launch_gather(p, p.dev.replicas[0], B, C, N, s);
    } catch (...) {
        g_mp_stamps = nullptr;
        (void)hipFree(dst);
        throw;
    }
    g_mp_stamps = nullptr;
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(host, dst, std::min(n, n_host) * 8, hipMemcpyDeviceToHost));
    (void)hipFree(dst);
}
#endif

}  // namespace gs
