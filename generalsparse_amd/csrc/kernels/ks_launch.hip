// ks_launch.hip -- launches of k_mfma_ks (hip_code/kernel_lib.hpp), the K-split,
// B-stationary matrix-core kernel for tall BMTB row blocks.  Its own translation unit
// so the kernel's instantiations build in parallel with device_plan.hip.
#include "../hip_code/kernel_lib.hpp"
#include "../host/gs_plan.hpp"

#include <cstring>
#include <map>
#include <mutex>

namespace gs {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) throw gs_error(std::string(#x) + ": " + hipGetErrorString(e_), -3); \
    } while (0)

namespace {

// k_mfma_ks's prio argument: KS_PRIO in bits 0..1; bit 4 (experiments build) forces the K-split
// combine's timeout path (KS_FORCE_TIMEOUT, the test of the device error word)
uint32_t ks_prio_arg() {
    const config_t c = get_config();
    return (uint32_t)(c.KS_PRIO & 3) | (c.KS_FORCE_TIMEOUT ? 16u : 0u);
}

template <class KERN>
void grant_lds(int device, KERN kern, size_t bytes) {
    // dynamic LDS above 64 KB is opted into once per kernel and device
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> granted;
    std::lock_guard<std::mutex> l(mu);
    size_t &g = granted[{device, reinterpret_cast<const void *>(kern)}];
    if (g < bytes) {
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)bytes));
        g = bytes;
    }
}

template <int CT, int RT, int MAXG, bool STAMPS = false, int W = (int)kKsWaves>
void launch_ks_k(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s,
                 uint64_t *stamps = nullptr) {
    const device_plan &d = p.dev;
#ifdef GS_EXPERIMENTS
    // KS_WAVES = 16 (fixed at upload): every instantiation spills (128 VGPRs at 4 waves per
    // SIMD; C2 48-98 us against 14-30 us with 8 waves, profiles/r04a), experiments build only
    if constexpr (W == (int)kKsWaves && !STAMPS) {
        if (d.waves == 16) {
            launch_ks_k<CT, RT, MAXG, false, 16>(p, a, B, C, N, s, stamps);
            return;
        }
        // KS_WAVES = 12 (N = 32, RT <= 5): three waves per SIMD (r06 A/B)
        if constexpr (CT == 2 && RT <= 5) {
            if (d.waves == 12) {
                launch_ks_k<CT, RT, MAXG, false, 12>(p, a, B, C, N, s, stamps);
                return;
            }
        }
    }
    // GS_KS_DEPTH=1/3/4 (look-ahead sweep against kKsDepth = 2, N = 32 on the C2 / attn / fc1 instantiations)
    if constexpr (W == (int)kKsWaves && !STAMPS && CT == 2 &&
                  ((RT == 3 && MAXG == 1) || (RT == 4 && MAXG == 2) || (RT == 5 && MAXG <= 2) || (RT == 7 && MAXG == 3))) {
        static const int dep = getenv("GS_KS_DEPTH") ? atoi(getenv("GS_KS_DEPTH")) : 0;
        if (dep == 1 || dep == 3 || dep == 4) {
            auto kd = dep == 1 ? gsk::k_mfma_ks<CT, RT, W, 1, MAXG, false>
                               : dep == 3 ? gsk::k_mfma_ks<CT, RT, W, 3, MAXG, false> : gsk::k_mfma_ks<CT, RT, W, 4, MAXG, false>;
            grant_lds(d.device, kd, d.lds_bytes);
            hipLaunchKernelGGL(kd, dim3((uint32_t)d.n_rows_aux * d.ksplit, ks_col_tiles_ct(N, CT)), dim3(64 * W), d.lds_bytes, s,
                               a.t0, (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, (const gsk::u32x2 *)a.t1, B, C,
                               (uint32_t)p.K, N, d.ksplit, d.ks_ns, (uint32_t)d.n_rows_aux * d.ksplit, (uint32_t)d.row_base,
                               a.ws, a.t2, stamps, ks_prio_arg());
            HIP_OK(hipGetLastError());
            return;
        }
    }
    // measured slower than the default form, experiments build only:
    // KS_WAVES = 4 (256-thread workgroups, overlapped LDS), KS_POS8 (8-bit positions), KS_APART = 0
    if constexpr (W == (int)kKsWaves && !STAMPS) {
        if (d.waves == 4) {
            if constexpr (CT == 2) {
                GS_CHECK(!d.ks_ap, "k_mfma_ks with 4 waves runs the overlapped LDS layout");
                auto k4 = d.ks_p8 ? gsk::k_mfma_ks<CT, RT, 4, (int)kKsDepth, MAXG, false, false, true>
                                  : gsk::k_mfma_ks<CT, RT, 4, (int)kKsDepth, MAXG, false, false, false>;
                GS_CHECK(gsk::ks_lds_bytes(CT, RT, 4, false) <= d.lds_bytes, "k_mfma_ks: LDS size disagrees with the upload");
                grant_lds(d.device, k4, d.lds_bytes);
                hipLaunchKernelGGL(k4, dim3((uint32_t)d.n_rows_aux * d.ksplit, ks_col_tiles_ct(N, CT)), dim3(256), d.lds_bytes,
                                   s, a.t0, (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, (const gsk::u32x2 *)a.t1, B,
                                   C, (uint32_t)p.K, N, d.ksplit, d.ks_ns, (uint32_t)d.n_rows_aux * d.ksplit,
                                   (uint32_t)d.row_base, a.ws, a.t2, stamps, ks_prio_arg() | (d.ks_gh << 8));
                HIP_OK(hipGetLastError());
                return;
            } else {
                throw gs_error("k_mfma_ks with 4 waves is built for N = 32");
            }
        }
    }
#else
    GS_CHECK(d.waves == kKsWaves && !d.ks_p8 && d.ks_ap,
             "k_mfma_ks with 4 or 16 waves, 8-bit positions or the overlapped LDS layout: experiments build");
#endif
    auto kern = gsk::k_mfma_ks<CT, RT, W, (int)kKsDepth, MAXG, STAMPS>;
    if (d.ks_nt) {  // KS_NT: A's groups by non-temporal loads (N = 32 / 128, 8 waves, the apart layout)
        if constexpr ((CT == 2 || CT == 8) && (W == (int)kKsWaves || W == 12) && !STAMPS) {
            GS_CHECK(d.ks_ap && !d.ks_p8, "k_mfma_ks: non-temporal loads are built for the apart layout, 16-bit positions");
            GS_CHECK(d.ks_nt == 1, "k_mfma_ks: KS_NT is built for A's groups (1)");
            kern = gsk::k_mfma_ks<CT, RT, W, (int)kKsDepth, MAXG, false, true, false, 1>;
        } else {
            throw gs_error("k_mfma_ks: non-temporal loads are built for N = 32 and 128-column tiles, 8 waves");
        }
    }
#ifdef GS_EXPERIMENTS
    if (d.ks_p8) {  // KS_POS8: 8-bit entry positions (N = 32, 8 waves, the apart layout)
        if constexpr (CT == 2 && W == (int)kKsWaves && !STAMPS) {
            GS_CHECK(d.ks_ap, "k_mfma_ks: 8-bit positions are built with the apart LDS layout");
            kern = gsk::k_mfma_ks<CT, RT, W, (int)kKsDepth, MAXG, false, true, true>;
        } else {
            throw gs_error("k_mfma_ks: 8-bit positions are built for N = 32, 8 waves");
        }
    }
    if (!d.ks_ap) {  // KS_APART = 0: the partial tiles reuse the stage LDS (N = 32, RT <= 5, MAXG <= 2)
        if constexpr (CT == 2 && RT <= 5 && MAXG <= 2 && W == (int)kKsWaves)
            kern = gsk::k_mfma_ks<CT, RT, W, (int)kKsDepth, MAXG, STAMPS, false>;
        else
            throw gs_error("k_mfma_ks: the overlapped-LDS layout is built for N = 32, RT <= 5, MAXG <= 2");
    }
#endif
#ifdef GS_EXPERIMENTS
    // KS_PERSIST (fixed at upload): a persistent grid of d.ks_persist workgroups pulling units
    if (d.ks_persist) {
        if constexpr (W == (int)kKsWaves && !STAMPS && (CT == 2 || CT == 8)) {
            GS_CHECK(d.ks_ap && !d.ks_p8 && a.t3 && ks_col_tiles_ct(N, CT) == 1, "k_mfma_ks_persist: 8 waves, apart layout, one column tile");
            auto kp = d.ks_nt ? gsk::k_mfma_ks_persist<CT, RT, W, (int)kKsDepth, MAXG, 1>
                              : gsk::k_mfma_ks_persist<CT, RT, W, (int)kKsDepth, MAXG, 0>;
            grant_lds(d.device, kp, d.lds_bytes);
            const uint32_t nunits = (uint32_t)d.n_rows_aux * d.ksplit;
            hipLaunchKernelGGL(kp, dim3(std::min(d.ks_persist, nunits)), dim3(64 * W), d.lds_bytes, s, a.t0,
                               (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, (const gsk::u32x2 *)a.t1, B, C,
                               (uint32_t)p.K, N, d.ksplit, d.ks_ns, nunits, (uint32_t)d.row_base, a.ws, a.t2,
                               ks_prio_arg() | (d.ks_gh << 8), a.t3);
            HIP_OK(hipGetLastError());
            return;
        } else {
            throw gs_error("k_mfma_ks_persist is built for N = 32 and 128-column tiles, 8 waves");
        }
    }
#else
    GS_CHECK(!d.ks_persist, "k_mfma_ks_persist is an experiments-build kernel");
#endif
    // the LDS this instantiation needs at the plan's range width, against what the upload sized
    GS_CHECK(gsk::ks_lds_bytes(CT, RT, W, d.ks_ap) <= d.lds_bytes, "k_mfma_ks: LDS size disagrees with the upload");
    grant_lds(d.device, kern, d.lds_bytes);
    hipLaunchKernelGGL(kern, dim3((uint32_t)d.n_rows_aux * d.ksplit, ks_col_tiles_ct(N, CT)), dim3(64 * W), d.lds_bytes, s, a.t0,
                       (const gsk::u32x4 *)a.tcol, (const gsk::u32x4 *)a.tval, (const gsk::u32x2 *)a.t1, B, C,
                       (uint32_t)p.K, N, d.ksplit, d.ks_ns, (uint32_t)d.n_rows_aux * d.ksplit, (uint32_t)d.row_base, a.ws, a.t2, stamps,
                       ks_prio_arg() | (d.ks_gh << 8));
    HIP_OK(hipGetLastError());
}

template <int CT, int RT>
void launch_ks_rt(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    if constexpr (CT == 8) {  // 128-column tiles: only the (RT, MAXG) pairs that do not spill (ks_ct8_fits)
        GS_CHECK(ks_ct8_fits(RT, p.dev.seg_cap), "k_mfma_ks: 128-column tile instantiation not built for this plan");
        if constexpr (RT == 2) {
            switch (p.dev.seg_cap) {
                case 1: launch_ks_k<CT, RT, 1>(p, a, B, C, N, s); break;
                case 2: launch_ks_k<CT, RT, 2>(p, a, B, C, N, s); break;
                default: launch_ks_k<CT, RT, 3>(p, a, B, C, N, s); break;
            }
        } else {
            launch_ks_k<CT, RT, 1>(p, a, B, C, N, s);
        }
    } else {
        switch (p.dev.seg_cap) {  // MAXG: entry groups per lane per k-step
            case 1: launch_ks_k<CT, RT, 1>(p, a, B, C, N, s); break;
            case 2: launch_ks_k<CT, RT, 2>(p, a, B, C, N, s); break;
            case 3: launch_ks_k<CT, RT, 3>(p, a, B, C, N, s); break;
            default: launch_ks_k<CT, RT, 4>(p, a, B, C, N, s); break;
        }
    }
}

template <int CT>
void launch_ks_ct(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    if constexpr (CT == 8) {  // 128 columns per workgroup: row blocks of up to 48 rows (ks_ct_rt)
        switch (p.dev.maxr) {
            case 2: launch_ks_rt<CT, 2>(p, a, B, C, N, s); return;
            case 3: launch_ks_rt<CT, 3>(p, a, B, C, N, s); return;
            default: throw gs_error("k_mfma_ks: 128-column tiles take row blocks of up to 48 rows");
        }
    } else {
        switch (p.dev.maxr) {  // RT: 16-row tiles per row block (the upload builds RT >= 2)
            case 2: launch_ks_rt<CT, 2>(p, a, B, C, N, s); break;
            case 3: launch_ks_rt<CT, 3>(p, a, B, C, N, s); break;
            case 4: launch_ks_rt<CT, 4>(p, a, B, C, N, s); break;
            case 5: launch_ks_rt<CT, 5>(p, a, B, C, N, s); break;
            case 6: if constexpr (CT <= 2) { launch_ks_rt<CT, 6>(p, a, B, C, N, s); break; } [[fallthrough]];
            case 7: if constexpr (CT <= 2) { launch_ks_rt<CT, 7>(p, a, B, C, N, s); break; } [[fallthrough]];
            case 8: if constexpr (CT <= 2) { launch_ks_rt<CT, 8>(p, a, B, C, N, s); break; } [[fallthrough]];
            default: throw gs_error("k_mfma_ks: row tiles outside 2..8 (6..8 for N <= 32)");
        }
    }
}

#ifdef GS_EXPERIMENTS
template <int CT, int RT, int W, bool STAMPS = false>
void launch_bm_k(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s,
                 uint64_t *stamps = nullptr) {
    const device_plan &d = p.dev;
    auto kern = gsk::k_mfma_bm<CT, RT, W, (int)gsk::bm_nbt(CT, RT), STAMPS>;
    GS_CHECK(gsk::bm_lds_bytes(CT, RT, W) <= d.lds_bytes, "k_mfma_bm: LDS size disagrees with the upload");
    grant_lds(d.device, kern, d.lds_bytes);
    const uint32_t nwg = (uint32_t)d.n_rows_aux * d.ksplit;
    hipLaunchKernelGGL(kern, dim3(nwg, ks_col_tiles(N)), dim3(64 * W), d.lds_bytes, s, a.t0, (const uint2 *)a.tcol, a.t1,
                       (const gsk::f16 *)a.tval, B, C, (uint32_t)p.K, N, d.ksplit, d.ks_ns, nwg, (uint32_t)d.row_base,
                       a.ws, a.t2, stamps);
    HIP_OK(hipGetLastError());
}

template <int CT, int RT>
void launch_bm2_k(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    const device_plan &d = p.dev;
    auto kern = gsk::k_mfma_bm2<CT, RT>;
    GS_CHECK(128u + (size_t)d.ks_ns * 32u * 32u * CT <= d.lds_bytes, "k_mfma_bm2: LDS size disagrees with the upload");
    grant_lds(d.device, kern, d.lds_bytes);
    const uint32_t nwg = (uint32_t)d.n_rows_aux * d.ksplit;
    hipLaunchKernelGGL(kern, dim3(nwg, ks_col_tiles(N)), dim3(64 * RT), d.lds_bytes, s, a.t0, (const uint2 *)a.tcol, a.t1,
                       (const gsk::f16 *)a.tval, B, C, (uint32_t)p.K, N, d.ksplit, d.ks_ns, nwg, (uint32_t)d.row_base,
                       a.ws, a.t2);
    HIP_OK(hipGetLastError());
}

template <int CT, int RT, int NVB>
void launch_kb_k(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    const device_plan &d = p.dev;
    // GS_KB_DEBUG=2/3 (diagnostics, wrong results): no value loads / no B loads
    static const int dbg = getenv("GS_KB_DEBUG") ? atoi(getenv("GS_KB_DEBUG")) : 0;
    auto kern = gsk::k_mfma_kb<CT, RT, (int)kKsWaves, (int)kKsDepth, NVB>;
    if constexpr (CT == 2 && NVB <= 2) {  // (N = 32 only)
        if (dbg == 2) kern = gsk::k_mfma_kb<CT, RT, (int)kKsWaves, (int)kKsDepth, NVB, false, 2>;
        if (dbg == 3) kern = gsk::k_mfma_kb<CT, RT, (int)kKsWaves, (int)kKsDepth, NVB, false, 3>;
    }
    GS_CHECK(d.waves == kKsWaves && gsk::kb_lds_bytes(CT, RT, kKsWaves, NVB) <= d.lds_bytes,
             "k_mfma_kb: LDS size disagrees with the upload");
    grant_lds(d.device, kern, d.lds_bytes);
    const uint32_t nwg = (uint32_t)d.n_rows_aux * d.ksplit;
    hipLaunchKernelGGL(kern, dim3(nwg, ks_col_tiles(N)), dim3(64 * kKsWaves), d.lds_bytes, s, a.t0, (const uint2 *)a.tcol,
                       a.t1, (const gsk::f16 *)a.tval, B, C, (uint32_t)p.K, N, d.ksplit, d.ks_ns, nwg,
                       (uint32_t)d.row_base, a.ws, a.t2, nullptr, ks_prio_arg());
    HIP_OK(hipGetLastError());
}

template <int CT, int RT>
void launch_bm_rt(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    if (p.dev.bmkb) {
        switch (p.dev.seg_cap) {  // NVB
            case 1: launch_kb_k<CT, RT, 1>(p, a, B, C, N, s); break;
            case 2: launch_kb_k<CT, RT, 2>(p, a, B, C, N, s); break;
            default: launch_kb_k<CT, RT, 4>(p, a, B, C, N, s); break;
        }
    }
    else if (p.dev.bm2) launch_bm2_k<CT, RT>(p, a, B, C, N, s);
    else if (p.dev.waves == 4) launch_bm_k<CT, RT, 4>(p, a, B, C, N, s);
    else launch_bm_k<CT, RT, 8>(p, a, B, C, N, s);
}

template <int CT>
void launch_bm_ct(const plan_state &p, const device_arrays &a, const gsk::f16 *B, gsk::f16 *C, uint32_t N, hipStream_t s) {
    switch (p.dev.maxr) {  // RT: 16-row tiles per row block
        case 1: launch_bm_rt<CT, 1>(p, a, B, C, N, s); break;
        case 2: launch_bm_rt<CT, 2>(p, a, B, C, N, s); break;
        case 3: launch_bm_rt<CT, 3>(p, a, B, C, N, s); break;
        case 4: launch_bm_rt<CT, 4>(p, a, B, C, N, s); break;
        case 5: launch_bm_rt<CT, 5>(p, a, B, C, N, s); break;
        case 6: launch_bm_rt<CT, 6>(p, a, B, C, N, s); break;
        default: throw gs_error("k_mfma_bm: row tiles outside 1..6");
    }
}

#endif  // GS_EXPERIMENTS

}  // namespace

#ifdef GS_EXPERIMENTS
void launch_bm(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    const gsk::f16 *b = (const gsk::f16 *)B;
    gsk::f16 *c = (gsk::f16 *)C;
    GS_CHECK(N == p.dev.lds_N, "k_mfma_bm runs the plan's dense width");
    switch (ks_ct(N)) {
        case 1: launch_bm_ct<1>(p, a, b, c, N, s); break;
        case 2: launch_bm_ct<2>(p, a, b, c, N, s); break;
        default: launch_bm_ct<4>(p, a, b, c, N, s); break;
    }
}

#else
void launch_bm(const plan_state &, const device_arrays &, const void *, void *, uint32_t, hipStream_t) {
    throw gs_error("k_mfma_bm is an experiments-build kernel (make -C generalsparse_amd/csrc exp)", -2);
}
#endif

// ---- grouped launches (gs_spmm_batch): N = 32 (CT = 2), 8 waves, one instantiation per group
namespace {
template <int RT, int MAXG, int W = (int)kKsWaves>
void launch_ks_group_k(const std::vector<ks_group_item> &it, uint32_t N, hipStream_t s) {
    constexpr bool AP = W == (int)kKsWaves;
#ifdef GS_EXPERIMENTS
    if constexpr (W == (int)kKsWaves) {
        if (it[0].p->dev.waves == 4) {  // KS_WAVES = 4: 256-thread workgroups, overlapped LDS
            launch_ks_group_k<RT, MAXG, 4>(it, N, s);
            return;
        }
    }
    auto kern = it[0].p->dev.ks_p8 ? gsk::k_mfma_ks_group<2, RT, W, (int)kKsDepth, MAXG, true, AP>
                                   : gsk::k_mfma_ks_group<2, RT, W, (int)kKsDepth, MAXG, false, AP>;
#else
    GS_CHECK(!it[0].p->dev.ks_p8, "k_mfma_ks_group: 8-bit positions are an experiments-build layout");
    auto kern = gsk::k_mfma_ks_group<2, RT, W, (int)kKsDepth, MAXG, false, AP>;
#endif
    if constexpr (AP) {
        if (it[0].p->dev.ks_nt) kern = gsk::k_mfma_ks_group<2, RT, W, (int)kKsDepth, MAXG, false, true, 1>;
    }
    GS_CHECK(!it.empty() && it.size() <= (size_t)gsk::kKsGroupMax, "k_mfma_ks_group: 1..32 entries");
    gsk::ks_group_args args;
    std::memset(&args, 0, sizeof(args));
    size_t lds = 0;
    uint32_t wg = 0;
    for (size_t i = 0; i < it.size(); i++) {
        const plan_state &p = *it[i].p;
        const device_plan &d = p.dev;
        const device_arrays &a = d.replicas[(size_t)it[i].replica];
        GS_CHECK(gsk::ks_lds_bytes(2, RT, W, AP) <= d.lds_bytes, "k_mfma_ks_group: LDS size disagrees with the upload");
        lds = std::max(lds, d.lds_bytes);
        gsk::ks_entry &e = args.e[i];
        e.tbr = a.t0;
        e.tP = (const gsk::u32x4 *)a.tcol;
        e.tV = (const gsk::u32x4 *)a.tval;
        e.steps = (const gsk::u32x2 *)a.t1;
        e.B = (const gsk::f16 *)it[i].B;
        e.C = (gsk::f16 *)it[i].C;
        e.slabs = a.ws;
        e.arrivals = a.t2;
        e.K = (uint32_t)p.K;
        e.S = d.ksplit;
        e.NS = d.ks_ns;
        e.nwg = (uint32_t)d.n_rows_aux * d.ksplit;
        e.row_base = (uint32_t)d.row_base;
        e.pad0 = d.ks_gh;  // the entry's head-step group count (ks_body's prio bits 8..17)
        args.begin[i] = wg;
        // each entry starts on a multiple of 8 workgroups (idle ones in between exit at once), so
        // its entry-relative block numbers share XCDs as the global ones do (xcd_block)
        wg += (e.nwg + 7u) & ~7u;
    }
    args.begin[it.size()] = wg;
    args.n = (uint32_t)it.size();
    args.N = N;
    args.pad[0] = ks_prio_arg();
    grant_lds(it[0].p->dev.device, kern, lds);
    hipLaunchKernelGGL(kern, dim3(wg, ks_col_tiles(N)), dim3(64 * W), lds, s, args);
    HIP_OK(hipGetLastError());
}

template <int RT>
void launch_ks_group_rt(const std::vector<ks_group_item> &it, uint32_t N, hipStream_t s) {
    switch (it[0].p->dev.seg_cap) {
        case 1: launch_ks_group_k<RT, 1>(it, N, s); break;
        case 2: launch_ks_group_k<RT, 2>(it, N, s); break;
        case 3: launch_ks_group_k<RT, 3>(it, N, s); break;
        default: launch_ks_group_k<RT, 4>(it, N, s); break;
    }
}
}  // namespace

uint32_t ks_group_key(const plan_state &p, uint32_t N) {
    const device_plan &d = p.dev;
    const bool w8 = d.waves == kKsWaves && d.ks_ap, w4 = d.waves == 4 && !d.ks_ap;
    if (!p.uploaded || !d.mfma || !d.ks || d.pad_rows || N != 32 || d.lds_N != 32 || !(w8 || w4) || d.ks_persist) return 0;
#ifndef GS_EXPERIMENTS
    // the release build instantiates the grouped kernel for 16-byte u16-position groups on 8
    // waves only: any other layout runs as single launches (which refuse it themselves)
    if (d.ks_p8 || !w8) return 0;
#endif
    return (d.ks_nt << 18) | (w4 ? 1u << 17 : 0u) | (d.ks_p8 ? 1u << 16 : 0u) | (d.maxr << 8) | d.seg_cap;  // NT, waves, P8, RT, MAXG
}

void launch_ks_group(const std::vector<ks_group_item> &it, uint32_t N, hipStream_t s) {
    GS_CHECK(!it.empty(), "empty group");
    const uint32_t key = ks_group_key(*it[0].p, N);
    GS_CHECK(key != 0, "k_mfma_ks_group: not a groupable k_mfma_ks plan");
    for (const auto &x : it) GS_CHECK(ks_group_key(*x.p, N) == key, "k_mfma_ks_group: entries of different instantiations");
    switch (it[0].p->dev.maxr) {
        case 2: launch_ks_group_rt<2>(it, N, s); break;
        case 3: launch_ks_group_rt<3>(it, N, s); break;
        case 4: launch_ks_group_rt<4>(it, N, s); break;
        case 5: launch_ks_group_rt<5>(it, N, s); break;
        case 6: launch_ks_group_rt<6>(it, N, s); break;
        case 7: launch_ks_group_rt<7>(it, N, s); break;
        case 8: launch_ks_group_rt<8>(it, N, s); break;
        default: throw gs_error("k_mfma_ks_group: row tiles outside 2..8");
    }
}

void launch_ks(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s) {
    const gsk::f16 *b = (const gsk::f16 *)B;
    gsk::f16 *c = (gsk::f16 *)C;
    GS_CHECK(N == p.dev.lds_N, "k_mfma_ks runs the plan's dense width");
    GS_CHECK(p.dev.ks_ctw == ks_ct_rt(N, p.dev.maxr) || (p.dev.ks_ctw == 4 && ks_ct_rt(N, p.dev.maxr) == 8 &&
                                                         !ks_ct8_fits(p.dev.maxr, p.dev.seg_cap)),
             "k_mfma_ks: column tiles disagree with the upload");
    switch (p.dev.ks_ctw) {  // 16-column tiles per workgroup; ks_col_tiles_ct(N, CT) workgroups across N
        case 1: launch_ks_ct<1>(p, a, b, c, N, s); break;
        case 2: launch_ks_ct<2>(p, a, b, c, N, s); break;
        case 4: launch_ks_ct<4>(p, a, b, c, N, s); break;
        case 8: launch_ks_ct<8>(p, a, b, c, N, s); break;
        default: throw gs_error("k_mfma_ks: bad column tile count");
    }
}

#ifdef GS_EXPERIMENTS  // diagnostics (s_memtime stamps)
// diagnostic: k_mfma_bm at N = 32, 65..80-row blocks, 8 waves (stamps: kernel_lib.hpp)
void debug_bm_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host) {
    const device_plan &d = p.dev;
    GS_CHECK(N == 32 && d.maxr == 5 && d.waves == 8, "k_mfma_bm timeline build: N=32, RT=5, 8 waves only");
    const size_t n = (size_t)d.n_rows_aux * d.ksplit * 8 * 16;
    uint64_t *dst = nullptr;
    HIP_OK(hipMalloc(&dst, n * 8));
    HIP_OK(hipMemsetAsync(dst, 0, n * 8, s));
    launch_bm_k<2, 5, 8, true>(p, d.replicas[0], (const gsk::f16 *)B, (gsk::f16 *)C, N, s, dst);
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(host, dst, std::min(n, n_host) * 8, hipMemcpyDeviceToHost));
    (void)hipFree(dst);
}

// diagnostic: the C2 shape (N = 32, 65..80-row blocks, <= 128 entry groups per k-step)
void debug_ks_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host) {
    const device_plan &d = p.dev;
    GS_CHECK(N == 32 && d.maxr >= 2 && d.maxr <= 5 && d.seg_cap <= 2 && d.waves == kKsWaves,
             "k_mfma_ks timeline build: N=32, RT 2..5, MAXG <= 2, 8 waves only");
    const size_t n = (size_t)d.n_rows_aux * d.ksplit * ks_col_tiles(N) * kKsWaves * 32;
    uint64_t *dst = nullptr;
    HIP_OK(hipMalloc(&dst, n * 8));
    HIP_OK(hipMemsetAsync(dst, 0, n * 8, s));
    const device_arrays &a = d.replicas[0];
    const gsk::f16 *b = (const gsk::f16 *)B;
    gsk::f16 *c = (gsk::f16 *)C;
    const bool g1 = d.seg_cap == 1;
    switch (d.maxr) {
        case 2: g1 ? launch_ks_k<2, 2, 1, true>(p, a, b, c, N, s, dst) : launch_ks_k<2, 2, 2, true>(p, a, b, c, N, s, dst); break;
        case 3: g1 ? launch_ks_k<2, 3, 1, true>(p, a, b, c, N, s, dst) : launch_ks_k<2, 3, 2, true>(p, a, b, c, N, s, dst); break;
        case 4: g1 ? launch_ks_k<2, 4, 1, true>(p, a, b, c, N, s, dst) : launch_ks_k<2, 4, 2, true>(p, a, b, c, N, s, dst); break;
        default: g1 ? launch_ks_k<2, 5, 1, true>(p, a, b, c, N, s, dst) : launch_ks_k<2, 5, 2, true>(p, a, b, c, N, s, dst); break;
    }
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(host, dst, std::min(n, n_host) * 8, hipMemcpyDeviceToHost));
    (void)hipFree(dst);
}

#else
void debug_bm_timeline(const plan_state &, const void *, void *, uint32_t, hipStream_t, uint64_t *, size_t) {
    throw gs_error("timeline builds are diagnostics of the experiments build (make -C generalsparse_amd/csrc exp)", -2);
}
void debug_ks_timeline(const plan_state &, const void *, void *, uint32_t, hipStream_t, uint64_t *, size_t) {
    throw gs_error("timeline builds are diagnostics of the experiments build (make -C generalsparse_amd/csrc exp)", -2);
}
#endif  // GS_EXPERIMENTS

}  // namespace gs
