// capi.cc -- extern "C" boundary (include/generalsparse.h) + the token_test pipelines.
#include "../../../include/generalsparse.h"
#include "gs_plan.hpp"
#include "index_compress.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>

// one plan per sub-matrix: st is sub-matrix 0 (the undivided matrix); a row division
// (fixed_interval_row_matrix_div_operator, §8f rank 3) adds sub-matrices, each with its
// own code generator / kernel / device arrays over the shared metadata set and operator
// history, run one after another by the multi-kernel executor (gs_spmm)
// Sub-matrices of row_nz_matrix_div_operator keep the divided sub-matrix's row indexing
// and a row can straddle two of them: each runs into a zeroed scratch output, and
// gs::combine_parts sums the scratch outputs into C's rows [base, base + rows).
// one plan replica's scratch outputs: one per sub-matrix (rows_of(sub) x N), so replicas
// (and gs_spmm_replica calls on different streams) never share a buffer
struct replica_scratch {
    std::vector<void *> bufs;
    void **ptrs_dev = nullptr;
    uint32_t N = 0;  // dense width the scratch outputs are sized for
};

struct parent_group {
    uint64_t base = 0, rows = 0;
    std::vector<gs::plan_state *> subs;
    std::vector<uint32_t> part_rows;
    std::vector<replica_scratch> rep;
    uint32_t *rows_dev = nullptr;
    int device = 0;
};

struct gs_plan {
    gs::plan_state st;
    std::map<int, std::unique_ptr<gs::plan_state>> subs;
    std::vector<std::pair<uint64_t, uint64_t>> gaps;  // output rows no sub-matrix writes
    std::vector<parent_group> groups;
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F &&f) {
    try {
        f();
        return GS_OK;
    } catch (const gs::gs_error &e) {
        g_err = e.what();
        return e.code < 0 ? e.code : GS_ERR;
    } catch (const std::exception &e) {
        g_err = e.what();
        return GS_ERR;
    }
}

void init_plan(gs::plan_state &s, std::shared_ptr<gs::meta_data_set> m) {
    s.meta = std::move(m);
    s.cg = std::make_shared<gs::code_generator>(s.meta, 0);
    s.exec = std::make_shared<gs::operator_executer>();
    s.M = s.meta->scalar(gs::GLOBAL_META, "origin_row_num", -1);
    s.K = s.meta->scalar(gs::GLOBAL_META, "origin_col_num", -1);
    s.nnz = s.meta->scalar(gs::GLOBAL_META, "origin_nnz_num", -1);
}

uint64_t global_scalar(const gs::plan_state &s, const char *n, int sub) { return s.meta->scalar(gs::GLOBAL_META, n, sub); }

bool sub_live(const gs::meta_data_set &m, int sub) { return m.is_exist(gs::GLOBAL_META, "nz_col_indices", sub); }

gs::plan_state &state_of(gs_plan *p, int sub) {
    GS_CHECK(sub >= 0, "sub-matrix id >= 0");
    if (sub == 0) return p->st;
    auto it = p->subs.find(sub);
    if (it != p->subs.end()) return *it->second;
    GS_CHECK(sub_live(*p->st.meta, sub), "no sub-matrix " + std::to_string(sub) + " in the plan");
    auto s = std::make_unique<gs::plan_state>();
    s->meta = p->st.meta;
    s->exec = p->st.exec;  // one operator history, keyed by sub-matrix id
    s->cg = std::make_shared<gs::code_generator>(s->meta, sub);
    s->M = p->st.M;
    s->K = p->st.K;
    s->nnz = p->st.nnz;
    auto &r = *s;
    p->subs.emplace(sub, std::move(s));
    return r;
}

// the kernels of the plan in sub-matrix order; every live sub-matrix needs one
std::vector<gs::plan_state *> kernel_states(gs_plan *p, bool strict = true) {
    const auto &m = *p->st.meta;
    std::vector<gs::plan_state *> out;
    const int mx = m.get_max_sub_matrix_id_of_data_item(gs::GLOBAL_META, "nz_col_indices");
    for (int sb = 0; sb <= mx; sb++) {
        if (!sub_live(m, sb)) continue;
        if (!strict && sb != 0 && !p->subs.count(sb)) continue;
        GS_CHECK(sb == 0 || p->subs.count(sb), "sub-matrix " + std::to_string(sb) + " has no plan (add its operators)");
        out.push_back(sb == 0 ? &p->st : p->subs[sb].get());
    }
    GS_CHECK(!out.empty(), "plan has no sub-matrix");
    return out;
}

bool divided(gs_plan *p) { return !p->subs.empty() || !sub_live(*p->st.meta, 0); }

#define GS_HIP(x) GS_CHECK((x) == hipSuccess, #x " failed")

void free_scratch(replica_scratch &r) {
    for (void *b : r.bufs) (void)hipFree(b);
    if (r.ptrs_dev) (void)hipFree(r.ptrs_dev);
    r.bufs.clear();
    r.ptrs_dev = nullptr;
    r.N = 0;
}

void free_group(parent_group &g) {
    bool any = g.rows_dev != nullptr;
    for (auto &r : g.rep) any |= r.ptrs_dev != nullptr || !r.bufs.empty();
    if (any) (void)hipSetDevice(g.device);
    for (auto &r : g.rep) free_scratch(r);
    g.rep.clear();
    if (g.rows_dev) (void)hipFree(g.rows_dev);
    g.rows_dev = nullptr;
}

void free_groups(gs_plan *p) {
    for (auto &g : p->groups) free_group(g);
    p->groups.clear();
}

// replica `replica`'s scratch outputs for dense width N (allocated on first use, grown for a
// wider N); the row counts are shared
// (the allocation and its synchronous copies are refused under stream capture: run one
// launch per replica and width before capturing, as for the deferred CSR upload)
replica_scratch &ensure_scratch(parent_group &g, int replica, uint32_t N, size_t e, hipStream_t stream) {
    if ((size_t)replica >= g.rep.size()) g.rep.resize((size_t)replica + 1);
    replica_scratch &r = g.rep[(size_t)replica];
    if (r.N >= N && g.rows_dev) return r;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    GS_HIP(hipStreamIsCapturing(stream, &cap));
    if (cap != hipStreamCaptureStatusNone)
        throw gs::gs_error("sub-matrix scratch outputs of replica " + std::to_string(replica) + " at N=" +
                               std::to_string(N) + " are allocated on first use: launch once before capturing",
                           -2);
    GS_HIP(hipSetDevice(g.device));
    free_scratch(r);
    for (size_t i = 0; i < g.subs.size(); i++) {
        void *b = nullptr;
        GS_HIP(hipMalloc(&b, std::max<size_t>(1, (size_t)g.part_rows[i] * N * e)));
        r.bufs.push_back(b);
    }
    GS_HIP(hipMalloc((void **)&r.ptrs_dev, r.bufs.size() * sizeof(void *)));
    GS_HIP(hipMemcpy(r.ptrs_dev, r.bufs.data(), r.bufs.size() * sizeof(void *), hipMemcpyHostToDevice));
    if (!g.rows_dev) {
        GS_HIP(hipMalloc((void **)&g.rows_dev, g.part_rows.size() * sizeof(uint32_t)));
        GS_HIP(hipMemcpy(g.rows_dev, g.part_rows.data(), g.part_rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    r.N = N;
    return r;
}

// multi-kernel executor: zero the output rows of empty row intervals, then run each
// sub-matrix's kernel on the same stream (each writes only its own rows); parent-indexed
// sub-matrices run into their scratch outputs, summed into C per divided range
void spmm_all(gs_plan *p, int replica, const void *B, void *C, uint32_t N, hipStream_t stream) {
    if (!divided(p)) {
        gs::launch_spmm(p->st, replica, B, C, N, stream);
        return;
    }
    auto ks = kernel_states(p);
    const int dtype = ks.front()->dev.dtype;
    const size_t e = dtype == 0 ? 4 : 2;
    for (auto &g : p->gaps)
        if (g.second > g.first)
            gs::memset_rows(C, g.first, g.second, N, e, stream);
    for (gs::plan_state *s : ks)
        if (s->parent_row_base < 0) gs::launch_spmm(*s, replica, B, C, N, stream);
    for (auto &g : p->groups) {
        replica_scratch &r = ensure_scratch(g, replica, N, e, stream);
        for (size_t i = 0; i < g.subs.size(); i++) {
            gs::memset_rows(r.bufs[i], 0, g.part_rows[i], N, e, stream);
            gs::launch_spmm(*g.subs[i], replica, B, r.bufs[i], N, stream);
        }
        gs::combine_parts(r.ptrs_dev, g.rows_dev, (uint32_t)g.subs.size(), C, g.base, g.rows, N, dtype, stream);
    }
}

}  // namespace

namespace gs {

// token_test.cc:1003-1582 -- the reference's end-to-end pipelines, same operators,
// same parameters and the same VECTOR_WIDTH / block rules.
void run_pipeline(plan_state &s, const std::string &name, int N, int p0, int p1) {
    set_config("DENSE_MATRIX_SIZE", N);
    auto cg = s.cg;
    auto &ex = *s.exec;
    auto ctx = ex.get_operator_context();
    // rows / nonzeros of the plan's sub-matrix (the whole matrix for sub-matrix 0)
    const int sb = cg->get_sub_matrix_id();
    const uint64_t rows = sb == 0 ? global_scalar(s, "origin_row_num", -1)
                                  : global_scalar(s, "end_row_index", sb) - global_scalar(s, "begin_row_index", sb) + 1;
    const uint64_t nnz = s.meta->u(GLOBAL_META, "nz_col_indices", sb).size();
    if (name.rfind("empty_pad_", 0) == 0) {
        // empty_row_pad_operator first (every empty row gets one zero entry), then the
        // named pipeline on the padded matrix
        ex.add_and_run(std::make_shared<empty_row_pad_operator>(cg, ctx));
        run_pipeline(s, name.substr(10), N, p0, p1);
        s.pipeline = name;
        return;
    }
    if (name == "thread_total") {  // token_test.cc:1003-1092, p0 = sparse_cf (4), p1 = cf (1)
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<sort_operator>(cg, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_thread_blocking_operator>(
            cg, 1, false, false, false, false, true, scf, ctx));
        int x = N / cf < 32 ? N / cf : 32;
        set_config("VECTOR_WIDTH", x);
        int y = 128 / std::max(1, x);
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, scf, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)(rows / y + 1),
                                                             std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "warp_total") {  // token_test.cc:1188-1249
        int cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, 1, false, false, false, ctx));
        int y = std::min(N / cf, 32), x = std::max(256 / std::max(1, y), 32);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "thread_bit_map") {  // token_test.cc:1319-1391
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_thread_blocking_operator>(cg, 32, false, false, true, ctx));
        int x = N / cf < 32 ? N / cf : 32;
        set_config("VECTOR_WIDTH", x);
        int y = 128 / std::max(1, x);
        cg->open_spec_level_of_paral(THREAD_META);
        ex.add_and_run(std::make_shared<thread_bit_map_operator>(cg, THREAD_META, (unsigned)x, (unsigned)scf, (unsigned)cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)(nnz / y + 1),
                                                             std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "nnz_warp_bitmap" || name == "nnz_tblock_bitmap" || name == "nnz_tblock_warp_bitmap") {
        // nnz-direction parents (fixed_interval_nnz_direction_{warp,tblock}_blocking_operator; p0 =
        // nnz per BMW / BMTB, padded, p1 = nnz per BMW inside the BMTBs), 32-nnz BMTs inside them
        // with indices relative to the parent (token_test.cc:851-870's composition), thread bitmaps
        const int cf = 1;
        if (name == "nnz_warp_bitmap") {
            ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_warp_blocking_operator>(cg, p0 > 0 ? p0 : 256, false,
                                                                                                 false, true, ctx));
        } else {
            ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_tblock_blocking_operator>(cg, p0 > 0 ? p0 : 1024,
                                                                                                   true, ctx));
            if (name == "nnz_tblock_warp_bitmap")
                ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_warp_blocking_operator>(cg, p1 > 0 ? p1 : 256,
                                                                                                     true, true, false, ctx));
        }
        ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_thread_blocking_operator>(cg, 32, true, true, false, ctx));
        int x = N / cf < 32 ? N / cf : 32;
        set_config("VECTOR_WIDTH", x);
        int y = 128 / std::max(1, x);
        cg->open_spec_level_of_paral(THREAD_META);
        ex.add_and_run(std::make_shared<thread_bit_map_operator>(cg, THREAD_META, (unsigned)x, 4u, (unsigned)cf, ctx));
        const uint64_t nz = s.meta->u(GLOBAL_META, "nz_col_indices", sb).size();
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)(nz / y + 1),
                                                             std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "warp_segment") {  // token_test.cc:1393-1455
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_nnz_direction_thread_blocking_operator>(cg, 32, false, false, true, ctx));
        int x = std::min(N, 32), y = 256 / std::max(1, x);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<thread_bit_map_operator>(cg, WARP_META, (unsigned)get_config().VECTOR_WIDTH,
                                                                 (unsigned)scf, (unsigned)cf, ctx));
        ex.add_and_run(std::make_shared<warp_segment_reduce_operator>(cg, (unsigned)cf, false, false, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)(nnz / 128 + 1),
                                                             std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "warp_bit_map") {  // token_test.cc:1250-1315 (p0 = sparse_cf 4, p1 = cf 1)
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, 64, false, false,
                                                                                               true, false, ctx));
        int y = std::min(std::max(1, N / cf), 32), x = std::max(128 / y, 32);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, true, scf, cf, ctx));
        ex.add_and_run(std::make_shared<warp_bit_map_operator>(cg, (unsigned)cf, true, true, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "tblock_bit_map") {  // token_test.cc:1515-1582 (p0 = sparse_cf 4, p1 = cf 1)
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, 64, false, false,
                                                                                               true, false, ctx));
        int x = std::min(std::max(1, N / cf), 32), y = 256 / x;
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, scf, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
        ex.add_and_run(std::make_shared<tblock_thread_bit_map_operator>(cg, (unsigned)cf, y, false, false, ctx));
    } else if (name == "warp_bit_map_interleaved" || name == "tblock_bit_map_interleaved") {
        // §8f rank 2: the warp_bit_map / tblock_bit_map plans with interleaved storage of the
        // equal-size (padded) col-direction BMTs (interlance_storage_operator, GLOBAL parent)
        int scf = p0 > 0 ? p0 : 4, cf = p1 > 0 ? p1 : 1;
        const bool warp = name == "warp_bit_map_interleaved";
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, 64, false, false,
                                                                                               true, false, ctx));
        ex.add_and_run(std::make_shared<interlance_storage_operator>(cg, ctx));
        if (warp) {
            int y = std::min(std::max(1, N / cf), 32), x = std::max(128 / y, 32);
            set_config("VECTOR_WIDTH", x);
            ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, true, scf, cf, ctx));
            ex.add_and_run(std::make_shared<warp_bit_map_operator>(cg, (unsigned)cf, true, true, ctx));
            ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
        } else {
            int x = std::min(std::max(1, N / cf), 32), y = 256 / x;
            set_config("VECTOR_WIDTH", x);
            ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, scf, cf, ctx));
            ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
            ex.add_and_run(std::make_shared<tblock_thread_bit_map_operator>(cg, (unsigned)cf, y, false, false, ctx));
        }
    } else if (name == "col_direction_nm") {
        // BASELINE.json configs[2] (C3): col-direction BMTs of p0 nnz (32 = one 64-column
        // k-step of a 2:4 row), no padding, summed per row (the warp_bit_map tokens);
        // rows that are 2:4 panels run on the sparse matrix cores (k_nm_mfma)
        int fcs = p0 > 0 ? p0 : 32, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, fcs, false, false,
                                                                                               false, false, ctx));
        int y = std::min(std::max(1, N / cf), 32), x = std::max(128 / y, 32);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, true, 4, cf, ctx));
        ex.add_and_run(std::make_shared<warp_bit_map_operator>(cg, (unsigned)cf, true, true, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "block_total_rowpad" || name == "warp_total_rowpad") {
        // row-direction BMTBs (BMWs) of p0 rows with is_padding: the row count padded up to a
        // multiple of p0 first (modify_*_by_row_pad_in_sub_matrix; one zero entry per added row)
        int rb = p0 > 0 ? p0 : 1, cf = p1 > 0 ? p1 : 1;
        int x = std::min(N, 32), y = 256 / std::max(1, x);
        set_config("VECTOR_WIDTH", x);
        if (name == "block_total_rowpad") {
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, true, ctx));
            ex.add_and_run(std::make_shared<tblock_total_reduce_operator>(cg, cf, ctx));
        } else {
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, rb, false, false, true, ctx));
            ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        }
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "block_total") {  // token_test.cc:1458-1514 (p0 = rows per BMTB, 1 there)
        int rb = p0 > 0 ? p0 : 1, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        int x = std::min(N, 32), y = 256 / std::max(1, x);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<tblock_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)rows, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "tblock_warp_total") {
        // headline plan (BASELINE.json configs[1]): row-direction BMTB blocking of
        // p0 rows, BMWs of p1 rows inside each BMTB, wave-level reduction
        int rb = p0 > 0 ? p0 : 4, wb = p1 > 0 ? p1 : 1, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, wb, false, false, false, ctx));
        ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "col_warp_total" || name == "col_tblock_total" || name == "tblock_col_warp_total") {
        // col-direction parents (fixed_interval_col_direction_{warp,tblock}_blocking_operator): BMWs /
        // BMTBs of p0 nonzeros of one row (tblock_col_warp_total: BMWs of p1 nonzeros inside
        // row-direction BMTBs of p0 rows, indices relative to the BMTB too), total-reduced
        const int cf = 1;
        if (name == "col_tblock_total") {
            ex.add_and_run(std::make_shared<fixed_interval_col_direction_tblock_blocking_operator>(cg, p0 > 0 ? p0 : 256, false,
                                                                                                   false, ctx));
            ex.add_and_run(std::make_shared<tblock_total_reduce_operator>(cg, cf, ctx));
        } else {
            int c = p0 > 0 ? p0 : 64;
            if (name == "tblock_col_warp_total") {
                ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, p0 > 0 ? p0 : 16,
                                                                                                       false, ctx));
                c = p1 > 0 ? p1 : 64;
            }
            const bool rel = name == "tblock_col_warp_total";
            ex.add_and_run(std::make_shared<fixed_interval_col_direction_warp_blocking_operator>(cg, c, rel, rel, false, false, ctx));
            ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        }
        const uint64_t units = s.meta->u(name == "col_tblock_total" ? TBLOCK_META : WARP_META, "first_nz_indices", sb).size() - 1;
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)std::max<uint64_t>(1, units),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_col_thread_maxpad" || name == "warp_col_thread_maxpad") {
        // col-direction BMTs of p1 nonzeros inside BMTBs (BMWs) of p0 rows, every non-empty row
        // first padded to its parent's longest row (is_col_padding_with_row_max_size_without_empty_row,
        // modify_*_by_col_pad_parent_blk_to_max_row_size; the parent level is then rebuilt)
        const int rb = p0 > 0 ? p0 : 16, c = p1 > 0 ? p1 : 32, cf = 1;
        if (name == "warp_col_thread_maxpad")
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, rb, false, false, false, ctx));
        else
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, c, true, true, false, true, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_col_thread_interleaved" || name == "warp_col_thread_interleaved") {
        // §8f rank 2 under a parent: tblock_col_thread_total_padded (every row padded to a
        // multiple of p1, BMTs of p1 nonzeros inside BMTBs of p0 rows), then
        // interlance_storage_operator, which takes the TBLOCK level from the distributing
        // operators before it (interlance_storage_operator.cc:12-45) and interleaves the BMTs of
        // each BMTB among themselves (modify_col_indices_by_interlance_storage.cc:73-118)
        // (warp_: the same inside BMWs of p0 rows, interleaved per BMW)
        const int rb = p0 > 0 ? p0 : 16, c = p1 > 0 ? p1 : 32, cf = 1;
        if (name == "warp_col_thread_interleaved")
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, rb, false, false, false, ctx));
        else
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, c, true, true, true, false, ctx));
        ex.add_and_run(std::make_shared<interlance_storage_operator>(cg, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_col_thread_total" || name == "warp_col_thread_total" || name == "tblock_col_thread_total_padded") {
        // col-direction BMTs of p1 nonzeros inside row-direction BMTBs (or BMWs) of p0 rows, row and
        // nz indices relative to the parent; _padded pads every row to a multiple of p1 first
        // (the parent level is rebuilt on the padded COO: the operator re-runs the former ones)
        const int rb = p0 > 0 ? p0 : 16, c = p1 > 0 ? p1 : 32, cf = 1;
        if (name == "warp_col_thread_total")
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, rb, false, false, false, ctx));
        else
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(
            cg, c, true, true, name == "tblock_col_thread_total_padded", false, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_thread_total" || name == "tblock_warp_thread_total") {
        // §8f rank 1: BMTs of p1 rows inside BMTBs of p0 rows (and inside BMWs of 8 rows),
        // row and nz indices relative to the parent as well
        int rb = p0 > 0 ? p0 : 16, tbr = p1 > 0 ? p1 : 1, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        if (name == "tblock_warp_thread_total")
            ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, 8, false, false, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_thread_blocking_operator>(
            cg, tbr, true, true, false, false, false, 0, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_thread_total_colpad") {
        // BMTs of one row inside BMTBs of p0 rows with is_col_padding_with_col_size (rows to a
        // multiple of p1; the BMTB level is rebuilt on the padded COO, :272-317 / :406-437)
        int rb = p0 > 0 ? p0 : 16, cs = p1 > 1 ? p1 : 2, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_thread_blocking_operator>(
            cg, 1, true, true, false, false, true, cs, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_thread_total_maxpad" || name == "thread_total_maxpad") {
        // row-direction BMTs with is_col_padding_with_row_max_size_with_empty_row: every row, empty
        // ones too, padded to its BMTB's (tblock_: p0 rows, BMTs of p1 rows) or the matrix's
        // (thread_total_maxpad: BMTs of p0 rows) longest row
        // (fixed_interval_row_direction_thread_blocking_operator.cc:369-437 / :506-521)
        const bool tb = name == "tblock_thread_total_maxpad";
        int rb = p0 > 0 ? p0 : 16, tbr = tb ? (p1 > 0 ? p1 : 1) : rb, cf = 1;
        if (tb) ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_thread_blocking_operator>(
            cg, tbr, tb, tb, false, true, false, 0, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_warp_total_relative") {
        // §8f rank 1: the C2 plan with BMW indices relative to their BMTB as well
        // (fixed_interval_row_direction_warp_blocking_operator with both relative flags)
        int rb = p0 > 0 ? p0 : 4, wb = p1 > 0 ? p1 : 1, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, wb, true, true, false, ctx));
        ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_balanced_thread_total") {
        // balanced BMTs of ~p1 nonzeros inside row-direction BMTBs of p0 rows, indices relative to
        // the BMTB as well (balanced_interval_row_direction_thread_blocking_operator.cc:207-249)
        int rb = p0 > 0 ? p0 : 64, per = p1 > 0 ? p1 : 64, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<balanced_interval_row_direction_thread_blocking_operator>(cg, per, true, true, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 1, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "tblock_balanced_warp_total") {
        // balanced BMWs of ~p1 nonzeros inside row-direction BMTBs of p0 rows, indices relative
        // to the BMTB as well (balanced_interval_row_direction_warp_blocking_operator.cc:165-207)
        int rb = p0 > 0 ? p0 : 64, per = p1 > 0 ? p1 : 256, cf = 1;
        ex.add_and_run(std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, rb, false, ctx));
        ex.add_and_run(std::make_shared<balanced_interval_row_direction_warp_blocking_operator>(cg, per, true, true, ctx));
        ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, (unsigned)((rows + rb - 1) / rb),
                                                             std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "balanced_warp_total") {
        // balanced row-direction BMWs (A11) + warp_total (the valid composition)
        int per = p0 > 0 ? p0 : 2048, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<balanced_interval_row_direction_warp_blocking_operator>(cg, per, false, false, ctx));
        ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, 1024u, std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else if (name == "balanced_block_total") {
        // balanced row-direction BMTBs (A11, TBLOCK level) + tblock_total (K6): the reference's
        // name rules accept it (tblock_total_reduce_operator.cc: "tblock" and not "nnz")
        int per = p0 > 0 ? p0 : 4096, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<balanced_interval_row_direction_tblock_blocking_operator>(cg, per, ctx));
        int x = std::min(N, 32), y = 256 / std::max(1, x);
        set_config("VECTOR_WIDTH", x);
        ex.add_and_run(std::make_shared<tblock_total_reduce_operator>(cg, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, 1024u, std::vector<unsigned>{(unsigned)x, (unsigned)y}, cf, ctx));
    } else if (name == "balanced_thread_total") {
        // balanced row-direction BMTs (A11, THREAD level) + thread_total (BMTs of whole rows)
        int per = p0 > 0 ? p0 : 64, cf = p1 > 0 ? p1 : 1;
        ex.add_and_run(std::make_shared<balanced_interval_row_direction_thread_blocking_operator>(cg, per, false, false, ctx));
        ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 4, cf, ctx));
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, 1024u, std::vector<unsigned>{32u, 4u}, cf, ctx));
    } else if (name == "merge_path") {
        // merge-path levels of p0 path steps (A11) at level p1 (WARP: 0 or 1, TBLOCK: 2,
        // THREAD: 3) + that level's total-reduce token -> k_merge_path (BASELINE.json configs[3])
        int ws = p0 > 0 ? p0 : 1024, lvl = p1 == 2 ? 2 : (p1 == 3 ? 0 : 1), cf = 1;
        if (lvl == 0) {
            ex.add_and_run(std::make_shared<merge_path_thread_operator>(cg, ws, ctx));
            ex.add_and_run(std::make_shared<thread_total_reduce_operator>(cg, false, 4, cf, ctx));
        } else if (lvl == 1) {
            ex.add_and_run(std::make_shared<merge_path_warp_operator>(cg, ws, ctx));
            ex.add_and_run(std::make_shared<warp_total_reduce_operator>(cg, cf, ctx));
        } else {
            ex.add_and_run(std::make_shared<merge_path_tblock_operator>(cg, ws, ctx));
            ex.add_and_run(std::make_shared<tblock_total_reduce_operator>(cg, cf, ctx));
        }
        ex.add_and_run(std::make_shared<grid_block_operator>(cg, 1024u, std::vector<unsigned>{64u, 4u}, cf, ctx));
    } else {
        throw gs_error("unknown pipeline " + name, GS_ERR_ARG);
    }
    s.pipeline = name;
}

}  // namespace gs

extern "C" {

const char *gs_last_error(void) { return g_err.c_str(); }
const char *gs_version(void) { return "generalsparse_amd 0.1 (gfx950)"; }

void gs_opts_default(gs_opts *o) {
    o->pipeline = "tblock_warp_total";
    o->dtype = GS_F16;
    o->dense_n = 32;
    o->p0 = 0;
    o->p1 = 0;
    o->ones_values = 0;
    o->device = 0;
}

int gs_plan_create_from_mtx(const char *path, int ones_values, gs_plan_t **out) {
    return guard([&] {
        GS_CHECK(path && out, "null argument");
        auto *p = new gs_plan;
        try {
            init_plan(p->st, gs::create_init_metadata_set_from_file(path, path, ones_values != 0));
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
    });
}

int gs_plan_create_from_coo(uint64_t n_rows, uint64_t n_cols, uint64_t nnz, const uint64_t *row, const uint64_t *col,
                            const float *val, gs_plan_t **out) {
    return guard([&] {
        GS_CHECK(row && col && out, "null argument");
        auto *p = new gs_plan;
        try {
            init_plan(p->st, gs::create_init_metadata_set_from_coo(n_rows, n_cols, nnz, row, col, val, "coo"));
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
    });
}

int gs_set_config_int(const char *key, long long value) {
    return guard([&] { gs::set_config(key, value); });
}

int gs_get_config_int(const char *key, long long *value) {
    return guard([&] {
        GS_CHECK(key && value, "null argument");
        *value = (long long)gs::get_config_int(key);
    });
}

int gs_plan_add_operator_sub(gs_plan_t *p, int sub, const char *op_name, const long long *args, int nargs) {
    return guard([&] {
        GS_CHECK(p && op_name && (nargs == 0 || args), "null argument");
        gs::plan_state &st = state_of(p, sub);
        std::vector<long long> a(args, args + nargs);
        auto op = gs::make_operator(op_name, a, st.cg, st.exec->get_operator_context());
        st.exec->add_and_run(op);
    });
}

int gs_plan_add_operator(gs_plan_t *p, const char *op_name, const long long *args, int nargs) {
    return gs_plan_add_operator_sub(p, 0, op_name, args, nargs);
}

int gs_plan_run_pipeline_sub(gs_plan_t *p, int sub, const char *name, int dense_n, int p0, int p1) {
    return guard([&] {
        GS_CHECK(p && name && dense_n > 0, "bad argument");
        gs::run_pipeline(state_of(p, sub), name, dense_n, p0, p1);
    });
}

int gs_plan_run_pipeline(gs_plan_t *p, const char *name, int dense_n, int p0, int p1) {
    return gs_plan_run_pipeline_sub(p, 0, name, dense_n, p0, p1);
}

int gs_plan_sub_matrices(gs_plan_t *p, int *ids, int cap) {
    int n = 0;
    int rc = guard([&] {
        GS_CHECK(p && (cap == 0 || ids), "bad argument");
        const auto &m = *p->st.meta;
        const int mx = m.get_max_sub_matrix_id_of_data_item(gs::GLOBAL_META, "nz_col_indices");
        for (int sb = 0; sb <= mx; sb++)
            if (sub_live(m, sb)) {
                if (n < cap) ids[n] = sb;
                n++;
            }
    });
    return rc ? rc : n;
}

int gs_plan_compile(gs_plan_t *p) {
    return guard([&] {
        GS_CHECK(p, "null plan");
        const auto &m = *p->st.meta;
        // sub-matrices of row_nz_matrix_div_operator keep the divided sub-matrix's row
        // indexing (div_row_indices_by_row_nnz.cc): their rows refer to its row range; a
        // fixed-interval division of such a sub-matrix has no row range to write to
        std::map<int, std::pair<uint64_t, uint64_t>> pidx;
        std::map<int, bool> unexec;
        for (auto &o : p->st.exec->get_operator_context()->read_operator_context_arr(gs::CONVERTING_OP, 0)) {
            const int t = o->get_target_matrix_id();
            if (auto *r = dynamic_cast<gs::row_nz_matrix_div_operator *>(o.get())) {
                const auto range = pidx.count(t) ? pidx[t] : std::make_pair(r->parent_row_base, r->parent_rows);
                for (int id : r->new_sub_matrix_ids) {
                    pidx[id] = range;
                    if (unexec.count(t)) unexec[id] = true;
                }
            } else if (auto *f = dynamic_cast<gs::fixed_interval_row_matrix_div_operator *>(o.get())) {
                if (pidx.count(t) || unexec.count(t))
                    for (int id : f->new_sub_matrix_ids) unexec[id] = true;
            }
        }
        for (gs::plan_state *s : kernel_states(p)) {
            const int sb = s->cg->get_sub_matrix_id();
            GS_CHECK(!unexec.count(sb), "sub-matrix " + std::to_string(sb) + ": a fixed-interval division of a row_nz "
                     "sub-matrix (rows in its parent's indexing) -- plan only, not executable");
            const uint64_t b = m.scalar(gs::GLOBAL_META, "begin_row_index", sb), e = m.scalar(gs::GLOBAL_META, "end_row_index", sb);
            const auto &r = m.u(gs::GLOBAL_META, "nz_row_indices", sb);
            auto it = pidx.find(sb);
            if (it != pidx.end()) {
                s->parent_row_base = (int64_t)it->second.first;
                s->parent_rows = it->second.second;
                GS_CHECK(r.empty() || r.back() < s->parent_rows, "sub-matrix " + std::to_string(sb) +
                         ": row indices lie past the divided sub-matrix's rows");
            } else {
                // a kernel writes C row begin_row_index + r: every row inside the sub-matrix
                // (an undivided row-padded matrix is the exception: its padding rows run into
                // the scratch output upload_plan gives it)
                GS_CHECK(r.empty() || b + r.back() <= e || (sb == 0 && !divided(p)),
                         "sub-matrix " + std::to_string(sb) + ": row indices lie past its end_row_index");
            }
            s->cg->compile();
        }
        // the reference asserts logical_check after every pipeline (token_test.cc:517-1541)
        const std::string bad = gs::logical_check(m);
        GS_CHECK(bad.empty(), "logical_check: " + bad);
    });
}

int gs_plan_logical_check(gs_plan_t *p, char *msg, int msg_len) {
    int rc = 0;
    const int g = guard([&] {
        GS_CHECK(p, "null plan");
        const std::string bad = gs::logical_check(*p->st.meta);
        if (msg && msg_len > 0) {
            std::strncpy(msg, bad.c_str(), msg_len - 1);
            msg[msg_len - 1] = 0;
        }
        rc = bad.empty() ? 0 : 1;
    });
    return g ? g : rc;
}

int gs_plan_array_set_u64(gs_plan_t *p, const char *key, uint64_t i, uint64_t value) {
    return guard([&] {
        GS_CHECK(p && key, "null argument");
        auto a = p->st.meta->get_element(key)->meta_data_arr;
        GS_CHECK(!a->is_float(), "array is a value array");
        GS_CHECK(i < a->get_len(), "index out of range");
        a->u_mut()[i] = value;
    });
}

int gs_plan_generate_program(gs_plan_t *p, const char *root_dir, int repeat, char *dir_out, int dir_out_len) {
    return guard([&] {
        GS_CHECK(p && root_dir, "null argument");
        GS_CHECK(!divided(p), "generated programs cover undivided plans (one kernel)");
        std::string dir;
        p->st.cg->generate_final_program(repeat, root_dir, &dir);
        if (dir_out && dir_out_len > 0) {
            std::strncpy(dir_out, dir.c_str(), dir_out_len - 1);
            dir_out[dir_out_len - 1] = 0;
        }
    });
}

int gs_plan_upload(gs_plan_t *p, int dtype, int device) {
    return guard([&] {
        GS_CHECK(p, "null plan");
        auto ks = kernel_states(p);
        for (gs::plan_state *s : ks) gs::upload_plan(*s, dtype, device);
        // parent-indexed sub-matrices, grouped by the row range they refer to
        free_groups(p);
        for (gs::plan_state *s : ks) {
            if (s->parent_row_base < 0) continue;
            auto g = std::find_if(p->groups.begin(), p->groups.end(), [&](const parent_group &x) {
                return x.base == (uint64_t)s->parent_row_base && x.rows == s->parent_rows;
            });
            if (g == p->groups.end()) {
                p->groups.emplace_back();
                g = p->groups.end() - 1;
                g->base = (uint64_t)s->parent_row_base;
                g->rows = s->parent_rows;
                g->device = device;
            }
            GS_CHECK(s->dev.n_out_rows <= g->rows && g->base + g->rows <= s->M, "parent-indexed sub-matrix outside its range");
            g->subs.push_back(s);
            g->part_rows.push_back((uint32_t)s->dev.n_out_rows);
        }
        // rows of C no sub-matrix owns (intervals without nonzeros): zeroed by the executor
        p->gaps.clear();
        if (divided(p)) {
            std::vector<std::pair<uint64_t, uint64_t>> own;
            for (gs::plan_state *s : ks)
                if (s->parent_row_base < 0) own.push_back({s->dev.out_lo, s->dev.n_out_rows});
            for (auto &g : p->groups) own.push_back({g.base, g.base + g.rows});
            std::sort(own.begin(), own.end());
            uint64_t at = 0;
            for (auto &o : own) {
                if (o.first > at) p->gaps.push_back({at, o.first});
                at = std::max(at, o.second);
            }
            if (at < p->st.M) p->gaps.push_back({at, p->st.M});
        }
    });
}

int gs_plan_add_replica(gs_plan_t *p) {
    return guard([&] {
        GS_CHECK(p, "null plan");
        for (gs::plan_state *s : kernel_states(p)) gs::add_replica(*s);
    });
}

int gs_spmm_replica(gs_plan_t *p, int replica, const void *B, void *C, int N, gs_stream_t stream) {
    return guard([&] {
        GS_CHECK(p && B && C && N > 0, "bad argument");
        spmm_all(p, replica, B, C, (uint32_t)N, (hipStream_t)stream);
    });
}

int gs_spmm_rotate(gs_plan_t *p, int count, int first, const void *const *B_ptrs, void *const *C_ptrs, int n_ptrs,
                   int N, gs_stream_t stream) {
    return guard([&] {
        GS_CHECK(p && B_ptrs && C_ptrs && n_ptrs > 0 && N > 0 && count >= 0, "bad argument");
        const int reps = (int)p->st.dev.replicas.size();
        GS_CHECK(reps > 0, "plan is not on the device");
        for (int i = 0; i < count; i++) {
            int k = first + i;
            spmm_all(p, k % reps, B_ptrs[k % n_ptrs], C_ptrs[k % n_ptrs], (uint32_t)N, (hipStream_t)stream);
        }
    });
}

namespace {
// the launches of a batch (gs_spmm_batch): runs of consecutive entries that are one grouped
// k_mfma_ks launch (key != 0; up to 32, each (plan, replica) once), single entries otherwise
struct batch_launch {
    uint32_t key;
    std::vector<int> idx;
};
std::vector<batch_launch> plan_batch(gs_plan_t *const *plans, const int *replicas, int n, int N) {
    std::vector<batch_launch> out;
    for (int i = 0; i < n; i++) {
        gs_plan *p = plans[i];
        GS_CHECK(p, "bad batch entry " + std::to_string(i));
        GS_CHECK(replicas[i] >= 0 && (size_t)replicas[i] < p->st.dev.replicas.size(),
                 "batch entry " + std::to_string(i) + ": bad replica index");
        const uint32_t k = divided(p) ? 0u : gs::ks_group_key(p->st, (uint32_t)N);
        bool join = k != 0 && !out.empty() && out.back().key == k && out.back().idx.size() < (size_t)gsk::kKsGroupMax;
        if (join)  // a (plan, replica) twice in one grid would share tickets and slabs
            for (int j : out.back().idx) join &= !(plans[j] == p && replicas[j] == replicas[i]);
        if (join)
            out.back().idx.push_back(i);
        else
            out.push_back({k, {i}});
    }
    return out;
}
}  // namespace

int gs_spmm_batch(gs_plan_t *const *plans, const int *replicas, const void *const *B, void *const *C, int n, int N,
                  gs_stream_t stream) {
    return guard([&] {
        GS_CHECK(plans && replicas && B && C && n >= 0 && N > 0, "bad argument");
        hipStream_t s = (hipStream_t)stream;
        for (int i = 0; i < n; i++) GS_CHECK(B[i] && C[i], "bad batch entry " + std::to_string(i));
        for (const batch_launch &l : plan_batch(plans, replicas, n, N)) {
            if (l.idx.size() == 1) {
                const int i = l.idx[0];
                if (l.key == 0)
                    spmm_all(plans[i], replicas[i], B[i], C[i], (uint32_t)N, s);
                else
                    gs::launch_spmm(plans[i]->st, replicas[i], B[i], C[i], (uint32_t)N, s);
                continue;
            }
            std::vector<gs::ks_group_item> grp;
            for (int i : l.idx) grp.push_back({&plans[i]->st, replicas[i], B[i], C[i]});
            gs::launch_ks_group(grp, (uint32_t)N, s);
        }
    });
}

int gs_batch_launches(gs_plan_t *const *plans, const int *replicas, int n, int N, int *entries_per_launch, int cap) {
    int count = 0;
    const int rc = guard([&] {
        GS_CHECK(plans && replicas && n >= 0 && N > 0 && (cap == 0 || entries_per_launch), "bad argument");
        const auto ls = plan_batch(plans, replicas, n, N);
        count = (int)ls.size();
        for (int i = 0; i < count && i < cap; i++) entries_per_launch[i] = (int)ls[(size_t)i].idx.size();
    });
    return rc < 0 ? rc : count;
}

int gs_plan_device_status(gs_plan_t *p, gs_stream_t stream) {
    return guard([&] {
        GS_CHECK(p, "null plan");
        // every stream of the device, not only `stream`: launches of this plan on side streams
        // (Rotation, Batch, multi-stream C5) must have finished before the words are read and
        // cleared, or a fault bit could be missed or cleared unreported
        (void)stream;
        GS_HIP(hipDeviceSynchronize());
        std::string what;
        for (gs::plan_state *k : kernel_states(p, false)) {
            if (!k->uploaded || !k->dev.err_at) continue;
            for (size_t r = 0; r < k->dev.replicas.size(); r++) {
                uint32_t *w = k->dev.replicas[r].t2 + k->dev.err_at;
                uint32_t v = 0;
                GS_HIP(hipMemcpy(&v, w, sizeof(v), hipMemcpyDeviceToHost));
                if (!v) continue;
                GS_HIP(hipMemset(w, 0, sizeof(v)));  // reported once
                what += (what.empty() ? "" : ", ") + k->dev.kernel + " replica " + std::to_string(r);
            }
        }
        if (!what.empty())
            throw gs::gs_error("K-split combine timed out waiting for a partial slab (" + what +
                                   "): the affected rows of C hold NaN", GS_ERR_DEVICE);
    });
}

int gs_spmm(gs_plan_t *p, const void *B, void *C, int N, gs_stream_t stream) {
    return gs_spmm_replica(p, 0, B, C, N, stream);
}

int gs_debug_mfma_timeline(gs_plan_t *p, const void *B, void *C, int N, gs_stream_t stream, uint64_t *stamps,
                           uint64_t n_stamps) {
    return guard([&] {
        GS_CHECK(p && B && C && stamps, "null argument");
        gs::debug_mfma_timeline(p->st, B, C, (uint32_t)N, (hipStream_t)stream, stamps, n_stamps);
    });
}

int gs_plan_info_get(gs_plan_t *p, gs_plan_info *info) {
    return guard([&] {
        GS_CHECK(p && info, "null argument");
        std::memset(info, 0, sizeof(*info));
        auto ks = kernel_states(p, false);
        auto &s = *ks.front();  // kernel fields: the first sub-matrix's kernel
        info->rows = s.M;
        info->cols = s.K;
        info->nnz = s.nnz;
        info->n_kernels = (int)ks.size();
        for (gs::plan_state *k : ks) info->nnz_stored += s.meta->u(gs::GLOBAL_META, "nz_col_indices", k->cg->get_sub_matrix_id()).size();
        if (s.cg->is_compiled()) {
            const auto &sp = s.cg->get_kernel_spec();
            info->family = sp.family;
            std::strncpy(info->kernel_name, sp.name().c_str(), sizeof(info->kernel_name) - 1);
        }
        if (s.uploaded) {
            info->n_units = s.dev.n_units;
            info->device_bytes_A = s.dev.bytes_A;
            info->col_bytes = s.dev.col_bytes;
            info->dtype = s.dev.dtype;
            info->replicas = (int)s.dev.replicas.size();
            info->needs_memset = s.dev.needs_memset ? 1 : 0;
            info->lds_stage = s.dev.nm ? 3 : (s.dev.mfma ? 2 : (s.dev.lds ? 1 : 0));
            info->lds_n = s.dev.lds_N;
            info->lds_kc = s.dev.KC;
            info->lds_chunks = s.dev.nc;
            info->lds_waves = s.dev.waves;
            info->lds_bytes = s.dev.lds_bytes;
            info->tile_bytes = s.dev.bytes_tile;
            info->ksplit = s.dev.ksplit;
            const std::string dk = !s.dev.kernel.empty() ? s.dev.kernel : s.cg->get_kernel_spec().name();
            std::strncpy(info->device_kernel, dk.c_str(), sizeof(info->device_kernel) - 1);
            info->index_formulas = s.dev.index_formulas;
            info->index_bytes_saved = s.dev.index_bytes_saved;
            info->ks_nt = s.dev.ks ? s.dev.ks_nt : 0;
            info->ks_head_groups = s.dev.ks ? s.dev.ks_gh : 0;
            info->nm_tiles = s.dev.nm ? s.dev.nm_tiles : 0;
        }
    });
}

int gs_plan_array_count(gs_plan_t *p) { return p ? (int)p->st.meta->keys().size() : GS_ERR_ARG; }

int gs_plan_array_key(gs_plan_t *p, int i, char *buf, int buf_len) {
    return guard([&] {
        GS_CHECK(p && buf && buf_len > 0, "bad argument");
        auto k = p->st.meta->keys();
        GS_CHECK(i >= 0 && (size_t)i < k.size(), "index out of range");
        std::strncpy(buf, k[i].c_str(), buf_len - 1);
        buf[buf_len - 1] = 0;
    });
}

long long gs_plan_array_len(gs_plan_t *p, const char *key) {
    if (!p || !key || !p->st.meta->is_exist(key)) return -1;
    return (long long)p->st.meta->get_element(key)->meta_data_arr->get_len();
}

int gs_plan_array_is_float(gs_plan_t *p, const char *key) {
    if (!p || !key || !p->st.meta->is_exist(key)) return GS_ERR_ARG;
    return p->st.meta->get_element(key)->meta_data_arr->is_float() ? 1 : 0;
}

int gs_plan_array_read_u64(gs_plan_t *p, const char *key, uint64_t *out, uint64_t n) {
    return guard([&] {
        GS_CHECK(p && key && out, "null argument");
        auto a = p->st.meta->get_element(key)->meta_data_arr;
        GS_CHECK(!a->is_float(), "array is a value array");
        GS_CHECK(n >= a->get_len(), "buffer too small");
        std::copy(a->u().begin(), a->u().end(), out);
    });
}

int gs_plan_array_read_f64(gs_plan_t *p, const char *key, double *out, uint64_t n) {
    return guard([&] {
        GS_CHECK(p && key && out, "null argument");
        auto a = p->st.meta->get_element(key)->meta_data_arr;
        GS_CHECK(n >= a->get_len(), "buffer too small");
        for (uint64_t i = 0; i < a->get_len(); i++) out[i] = a->read_float_from_arr(i);
    });
}

int gs_plan_log(gs_plan_t *p, char *buf, int buf_len) {
    return guard([&] {
        GS_CHECK(p && buf && buf_len > 0, "bad argument");
        std::string s;
        for (auto &l : p->st.exec->log()) s += l + "\n";
        std::strncpy(buf, s.c_str(), buf_len - 1);
        buf[buf_len - 1] = 0;
    });
}

int gs_plan_index_compression(gs_plan_t *p, const char *key, char *kind_out, int kind_len, char *expr_out,
                              int expr_len, int *exact) {
    return guard([&] {
        GS_CHECK(p && key && kind_out && kind_len > 0 && expr_out && expr_len > 0, "bad argument");
        std::string k = key;
        // "<POS>_<name>_<sub>": POS is two tokens (e.g. THREAD_META), sub the last
        const size_t a = k.find('_', k.find('_') + 1), b = k.rfind('_');
        GS_CHECK(a != std::string::npos && b > a, "key must be <POS>_<name>_<sub>");
        const std::string pos_s = k.substr(0, a), name = k.substr(a + 1, b - a - 1);
        const int sub = std::stoi(k.substr(b + 1));
        gs::POS_TYPE pos = pos_s == "GLOBAL_META" ? gs::GLOBAL_META
                         : pos_s == "TBLOCK_META" ? gs::TBLOCK_META
                         : pos_s == "WARP_META" ? gs::WARP_META : gs::THREAD_META;
        GS_CHECK(p->st.meta->is_exist(pos, name, sub), "no plan array " + k);
        auto c = gs::analyze_index_compression(*p->st.meta, pos, name, sub);
        const std::string e = gs::code_of_index_compression(c, "i", gs::get_metadata_item_name(pos, name + "_res", sub));
        std::strncpy(kind_out, c.kind.c_str(), kind_len - 1);
        kind_out[kind_len - 1] = 0;
        std::strncpy(expr_out, e.c_str(), expr_len - 1);
        expr_out[expr_len - 1] = 0;
        if (exact) *exact = c.exact ? 1 : 0;
    });
}

int gs_index_compression_of_array(const uint64_t *a, uint64_t n, int type_ori, int branch_max, char *kind_out,
                                  int kind_len, uint64_t *params, int *exact) {
    return guard([&] {
        GS_CHECK(a && kind_out && kind_len > 0 && params, "bad argument");
        auto c = gs::analyze_index_compression(std::vector<uint64_t>(a, a + n), (gs::data_type)type_ori, branch_max);
        std::strncpy(kind_out, c.kind.c_str(), kind_len - 1);
        kind_out[kind_len - 1] = 0;
        params[0] = c.coef;
        params[1] = c.intercept;
        params[2] = c.cycle;
        params[3] = (uint64_t)c.aa;
        params[4] = (uint64_t)c.bb;
        if (exact) *exact = c.exact ? 1 : 0;
    });
}

int gs_plan_save(gs_plan_t *p, const char *path) {
    return guard([&] {
        GS_CHECK(p && path, "null argument");
        std::vector<const gs::plan_state *> ks;
        for (gs::plan_state *s : kernel_states(p)) ks.push_back(s);
        gs::save_plan(ks, path);
    });
}

int gs_plan_load(const char *path, gs_plan_t **out) {
    return guard([&] {
        GS_CHECK(path && out, "null argument");
        auto *p = new gs_plan;
        try {
            std::vector<gs::loaded_kernel> specs;
            std::string pipeline;
            auto m = gs::load_plan(path, specs, pipeline);
            init_plan(p->st, m);
            p->st.pipeline = pipeline;
            for (auto &ks : specs) {
                gs::plan_state &st = state_of(p, ks.sub);
                st.pipeline = pipeline;
                st.parent_row_base = ks.parent_row_base;
                st.parent_rows = ks.parent_rows;
                st.cg->restore_compiled(ks.spec);
            }
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
    });
}

int gs_plan_from_mtx(const char *path, const gs_opts *opts, gs_plan_t **out) {
    gs_opts o;
    if (opts) o = *opts;
    else gs_opts_default(&o);
    gs_plan_t *p = nullptr;
    int rc = gs_plan_create_from_mtx(path, o.ones_values, &p);
    if (rc) return rc;
    rc = gs_plan_run_pipeline(p, o.pipeline ? o.pipeline : "tblock_warp_total", o.dense_n, o.p0, o.p1);
    if (!rc) rc = gs_plan_compile(p);
    if (!rc) rc = gs_plan_upload(p, o.dtype, o.device);
    if (rc) {
        gs_plan_free(p);
        return rc;
    }
    *out = p;
    return GS_OK;
}

void gs_plan_free(gs_plan_t *p) {
    if (!p) return;
    try {
        free_groups(p);
        gs::free_device(p->st);
        for (auto &kv : p->subs) gs::free_device(*kv.second);
    } catch (...) {
    }
    delete p;
}

}  // extern "C"
