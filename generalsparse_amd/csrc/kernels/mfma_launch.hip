// mfma_launch.hip -- launches of the dense-tile matrix-core kernels k_mfma_rows and
// k_nm_mfma (hip_code/kernel_lib.hpp); k_mfma_ks has ks_launch.hip.  Separate
// translation units so the kernel instantiations build in parallel.
#include "../hip_code/kernel_lib.hpp"
#include "../host/gs_plan.hpp"

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

template <int CT, int RT, int LGKC, int MAXA>
void launch_mfma_k(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N,
                   hipStream_t s) {
    const device_plan &d = p.dev;
    // the variant the upload fixed (device_layout.cc choose_matrix_core_layout): B rows by
    // LDS-DMA (GLDS 2 or 4 B waves, a ring of NBG buffers) or through registers (GLDS 0)
    const int gl = d.mfma_glds, nbg = d.mfma_nbg, wct = d.mfma_wct;
    GS_CHECK(mfma_rows_lds_need(LGKC, CT, RT, d.rpw_max, gl, nbg, wct) <= d.lds_bytes,
             "k_mfma_rows: the variant needs more LDS than the upload sized");
    auto kern = gl == 4 ? gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 4>
                        : (gl ? gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2> : gsk::k_mfma_rows<CT, RT, LGKC, MAXA>);
    if (gl == 2 && wct == 8) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 8>;
#ifdef GS_EXPERIMENTS
    // LDS counter hand-offs between the roles instead of per-chunk barriers (MFMA_FLAGS)
    if (gl == 2 && wct == 6 && nbg == 3 && d.mfma_flags) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 0, true>;
#endif
    if constexpr (LGKC == 8) {  // deeper B rings fit LDS with 256-column chunks
        if (gl == 2 && wct == 6 && nbg == 4) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 4>;
        if (gl == 2 && wct == 6 && nbg == 5) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 5>;
    }
#ifdef GS_EXPERIMENTS
    // GS_MFMA_DEBUG (diagnostic timing builds, wrong results): kernel_lib.hpp k_mfma_rows DBG bits, C2 shape only
    static const int mdbg = getenv("GS_MFMA_DEBUG") ? atoi(getenv("GS_MFMA_DEBUG")) : 0;
    if constexpr (CT == 2 && RT == 2 && LGKC == 9 && MAXA == 1) {
        if (gl == 2 && wct == 6 && mdbg == 1) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 1>;
        if (gl == 2 && wct == 6 && mdbg == 2) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 2>;
        if (gl == 2 && wct == 6 && mdbg == 4) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 4>;
        if (gl == 2 && wct == 6 && mdbg == 10) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 10>;
        if (gl == 2 && wct == 6 && mdbg == 11) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 11>;
        if (gl == 2 && wct == 6 && mdbg == 15) kern = gsk::k_mfma_rows<CT, RT, LGKC, MAXA, false, 2, 3, 6, 15>;
    }
#endif
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> granted;
    {
        std::lock_guard<std::mutex> l(mu);
        size_t &g = granted[{d.device, reinterpret_cast<const void *>(kern)}];
        if (g < d.lds_bytes) {
            HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)d.lds_bytes));
            g = d.lds_bytes;
        }
    }
    hipLaunchKernelGGL(kern, dim3((uint32_t)d.n_rows_aux * d.ksplit), dim3(kMfmaThreads), d.lds_bytes, s, a.t0,
                       a.t1, (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, B, C, (uint32_t)p.K, N, d.nc,
                       d.rpw_max, (uint32_t)d.row_base, d.ksplit, d.ncs, a.ws, a.t2, (uint64_t *)nullptr,
                       (uint32_t)get_config().MFMA_KROT);
    HIP_OK(hipGetLastError());
}

template <int CT, int RT>
void launch_mfma_rt(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N,
                    hipStream_t s) {
    const bool two = p.dev.mfma_maxa == 2;  // entry groups per thread per chunk (fixed at upload)
    switch (p.dev.RSB) {                  // log2 KC
        case 10: two ? launch_mfma_k<CT, RT, 10, 2>(p, a, B, C, N, s) : launch_mfma_k<CT, RT, 10, 1>(p, a, B, C, N, s); break;
        case 9: two ? launch_mfma_k<CT, RT, 9, 2>(p, a, B, C, N, s) : launch_mfma_k<CT, RT, 9, 1>(p, a, B, C, N, s); break;
        default: two ? launch_mfma_k<CT, RT, 8, 2>(p, a, B, C, N, s) : launch_mfma_k<CT, RT, 8, 1>(p, a, B, C, N, s); break;
    }
}

template <int CT>
void launch_mfma_ct(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N,
                    hipStream_t s) {
    switch (p.dev.maxr) {
        case 1: launch_mfma_rt<CT, 1>(p, a, B, C, N, s); break;
        case 2: launch_mfma_rt<CT, 2>(p, a, B, C, N, s); break;
        case 3: launch_mfma_rt<CT, 3>(p, a, B, C, N, s); break;
        default: launch_mfma_rt<CT, 4>(p, a, B, C, N, s); break;
    }
}

}  // namespace

#ifdef GS_EXPERIMENTS  // diagnostics (s_memtime stamps)
// diagnostic: N = 32 plans with 17..48-row BMTBs and KC 256 or 512
template <int RT, int LG>
auto timeline_kernel(bool two) {
    return two ? gsk::k_mfma_rows<2, RT, LG, 2, true, 2> : gsk::k_mfma_rows<2, RT, LG, 1, true, 2>;  // LDS-DMA B (default)
}

void debug_mfma_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                         size_t n_host) {
    const device_plan &d = p.dev;
    if (d.ks) {
        debug_ks_timeline(p, B, C, N, s, host, n_host);
        return;
    }
    if (d.bm) {
        debug_bm_timeline(p, B, C, N, s, host, n_host);
        return;
    }
    if (p.cg && p.cg->get_kernel_spec().family == KF_MERGE_PATH) {
        debug_mp_timeline(p, B, C, N, s, host, n_host);
        return;
    }
    GS_CHECK(p.uploaded && d.mfma && N == d.lds_N && N == 32 && (d.maxr == 2 || d.maxr == 3) &&
                 (d.RSB == 8 || d.RSB == 9),
             "timeline build exists for N=32 matrix-core plans with 17..48-row BMTBs, KC 256/512 only");
    const device_arrays &a = d.replicas[0];
    const bool two = d.seg_cap > 64u * gsk::kMfmaAWavesG;
    auto kern = d.maxr == 2 ? (d.RSB == 9 ? timeline_kernel<2, 9>(two) : timeline_kernel<2, 8>(two))
                            : (d.RSB == 9 ? timeline_kernel<3, 9>(two) : timeline_kernel<3, 8>(two));
    const size_t lds = d.lds_bytes;
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    uint64_t *dst = nullptr;
    const size_t n = (size_t)d.n_rows_aux * d.ksplit * 64;
    HIP_OK(hipMalloc(&dst, n * 8));
    hipLaunchKernelGGL(kern, dim3((uint32_t)d.n_rows_aux * d.ksplit), dim3(kMfmaThreads), lds, s, a.t0, a.t1,
                       (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, (const gsk::f16 *)B, (gsk::f16 *)C,
                       (uint32_t)p.K, N, d.nc, d.rpw_max, (uint32_t)d.row_base, d.ksplit, d.ncs, a.ws, a.t2, dst, 0u);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(host, dst, std::min(n, n_host) * 8, hipMemcpyDeviceToHost));
    (void)hipFree(dst);
}

#else
void debug_mfma_timeline(const plan_state &, const void *, void *, uint32_t, hipStream_t, uint64_t *, size_t) {
    throw gs_error("timeline builds are diagnostics of the experiments build (make -C generalsparse_amd/csrc exp)", -2);
}
#endif  // GS_EXPERIMENTS

namespace {

template <int CT, int NG, int TT>
void launch_nm_ctt(const plan_state &p, const device_arrays &a, const void *B, void *C, hipStream_t s) {
    const device_plan &d = p.dev;
#ifdef GS_EXPERIMENTS
    // GS_NM_DEBUG=1/2: diagnostic builds without the loop's B / A loads (wrong results)
    static const int dbg = getenv("GS_NM_DEBUG") ? atoi(getenv("GS_NM_DEBUG")) : 0;
    auto kern = dbg == 1 ? gsk::k_nm_mfma<CT, 1, NG, false, TT>
                         : (dbg == 2 ? gsk::k_nm_mfma<CT, 2, NG, false, TT>
                                     : (dbg == 4 ? gsk::k_nm_mfma<CT, 4, NG, false, TT> : gsk::k_nm_mfma<CT, 0, NG, false, TT>));
    if (dbg == 8) kern = gsk::k_nm_mfma<CT, 8, NG, false, TT>;
    if (d.nm_nt && dbg == 0) kern = gsk::k_nm_mfma<CT, 0, NG, true, TT>;
#else
    constexpr int dbg = 0;
    // NM_NT (fixed at upload): A's panel blocks by non-temporal loads
    auto kern = d.nm_nt ? gsk::k_nm_mfma<CT, 0, NG, true, TT> : gsk::k_nm_mfma<CT, 0, NG, false, TT>;
#endif
    const size_t lds = (size_t)2 * gsk::kNmKC * 32 * CT + (dbg == 4 ? 4096 : 0);
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, bool> granted;
    {
        std::lock_guard<std::mutex> l(mu);
        bool &g = granted[{d.device, reinterpret_cast<const void *>(kern)}];
        if (!g) {
            HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
            g = true;
        }
    }
#ifdef GS_EXPERIMENTS
    if (d.nm_ks) {
        GS_CHECK(d.nm_tiles == 8, "k_nm_mfma_ks reads the 64-row-group layout");
        auto kk = gsk::k_nm_mfma_ks<CT>;
        const size_t lds2 = (size_t)2 * gsk::kNmKC * 32 * CT;
        static std::mutex mu2;
        static std::map<std::pair<int, const void *>, bool> granted2;
        {
            std::lock_guard<std::mutex> l(mu2);
            bool &g = granted2[{d.device, reinterpret_cast<const void *>(kk)}];
            if (!g) {
                HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kk), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds2));
                g = true;
            }
        }
        const uint32_t nb = (uint32_t)((d.n_rows_aux + 255) / 256);
        hipLaunchKernelGGL(kk, dim3(nb * d.ksplit), dim3(256), lds2, s, (const unsigned char *)a.tcol, (const gsk::f16 *)B,
                           (gsk::f16 *)C, (uint32_t)p.K, d.KC, (uint32_t)d.n_rows_aux, (uint32_t)d.row_base, d.ksplit,
                           d.ncs, a.ws, a.t2);
        HIP_OK(hipGetLastError());
        return;
    }
#else
    GS_CHECK(!d.nm_ks, "k_nm_mfma_ks is an experiments-build kernel");
#endif
    const uint32_t wg = (uint32_t)((d.n_rows_aux + 16 * TT - 1) / (16 * TT));
    hipLaunchKernelGGL(kern, dim3(wg), dim3(64 * gsk::kNmWaves), lds, s, (const unsigned char *)a.tcol,
                       (const gsk::f16 *)B, (gsk::f16 *)C, (uint32_t)p.K, d.KC, (uint32_t)d.n_rows_aux,
                       (uint32_t)d.row_base, (uint32_t)get_config().NM_KROT);
    HIP_OK(hipGetLastError());
}

}  // namespace

#ifdef GS_EXPERIMENTS  // k_nm_mfma4: measured slower than k_nm_mfma on C3
template <int CT>
void launch_nm4(const plan_state &p, const device_arrays &a, const void *B, void *C, hipStream_t s) {
    const device_plan &d = p.dev;
    auto kern = gsk::k_nm_mfma4<CT>;
    const size_t lds = gsk::nm4_lds_bytes(CT);
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, bool> granted;
    {
        std::lock_guard<std::mutex> l(mu);
        bool &g = granted[{d.device, reinterpret_cast<const void *>(kern)}];
        if (!g) {
            HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
            g = true;
        }
    }
    const uint32_t nb = (uint32_t)((d.n_rows_aux + 255) / 256), nch = d.KC / 4;
    GS_CHECK(p.K % gsk::kNmKC == 0 && d.ksplit >= 1 && d.ncs >= 1 && (d.ksplit - 1) * d.ncs < nch &&
                 (d.ksplit == 1 || (a.ws && a.t2)),
             "k_nm_mfma4: K ranges disagree with the upload");
    const uint32_t nwg = nb * d.ksplit;
    const config_t cfg = get_config();
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * gsk::kNmWaves), lds, s, (const unsigned char *)a.tcol,
                       (const gsk::f16 *)B, (gsk::f16 *)C, (uint32_t)p.K, d.KC, (uint32_t)d.n_rows_aux,
                       (uint32_t)d.row_base, d.ksplit, d.ncs, nwg, a.ws, a.t2, cfg.KS_FORCE_TIMEOUT ? 16u : 0u);
    HIP_OK(hipGetLastError());
}

#endif

template <int CT, int NG = 16 * CT>
void launch_nm_ct(const plan_state &p, const device_arrays &a, const void *B, void *C, hipStream_t s) {
    switch (p.dev.nm_tiles) {  // 16-row tiles per workgroup (device_layout.cc nm_tiles_for)
        case 8: launch_nm_ctt<CT, NG, 8>(p, a, B, C, s); break;
        case 7: launch_nm_ctt<CT, NG, 7>(p, a, B, C, s); break;
        case 4: launch_nm_ctt<CT, NG, 4>(p, a, B, C, s); break;
        case 2: launch_nm_ctt<CT, NG, 2>(p, a, B, C, s); break;
        default: throw gs_error("k_nm_mfma: tiles per workgroup outside 2, 4, 7, 8");
    }
}

void launch_nm(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    if (p.dev.nm4) {
#ifdef GS_EXPERIMENTS
        switch (N) {
            case 64: launch_nm4<4>(p, a, B, C, s); return;
            case 128: launch_nm4<8>(p, a, B, C, s); return;
            default: throw gs_error("k_nm_mfma4 plan built for N = 64 / 128, not " + std::to_string(N), -2);
        }
#else
        throw gs_error("k_nm_mfma4 is an experiments-build kernel (make -C generalsparse_amd/csrc exp)", -2);
#endif
    }
    switch (N) {
        case 8: launch_nm_ct<1, 8>(p, a, B, C, s); break;  // one half-used 16-column tile
        case 16: launch_nm_ct<1>(p, a, B, C, s); break;
        case 32: launch_nm_ct<2>(p, a, B, C, s); break;
        case 64: launch_nm_ct<4>(p, a, B, C, s); break;
        case 128: launch_nm_ct<8>(p, a, B, C, s); break;
        default:
            throw gs_error("2:4 panel plan (k_nm_mfma) runs N = 8, 16, 32, 64 or 128, not " + std::to_string(N), -2);
    }
}

void launch_mfma(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    const gsk::f16 *b = (const gsk::f16 *)B;
    gsk::f16 *c = (gsk::f16 *)C;
    if (p.dev.ks) {
        launch_ks(p, a, B, C, N, s);  // ks_launch.hip
        return;
    }
    if (p.dev.bm) {
        launch_bm(p, a, B, C, N, s);  // ks_launch.hip
        return;
    }
    GS_CHECK(N % 8 == 0 && N <= 64, "k_mfma_rows runs N = 8..64, a multiple of 8");
    switch (ks_ct(N)) {  // 16-column tiles (device_layout.hpp)
        case 1: launch_mfma_ct<1>(p, a, b, c, N, s); break;
        case 2: launch_mfma_ct<2>(p, a, b, c, N, s); break;
        default: launch_mfma_ct<4>(p, a, b, c, N, s); break;
    }
}


}  // namespace gs
