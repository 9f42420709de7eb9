// code_generator.cc -- lowers the operators' reduction tokens to a gfx950 kernel
// family and emits a standalone HIP program for it.
#include "code_generator.hpp"
#include "device_layout.hpp"
#include "index_compress.hpp"

#include <cstdio>
#include <fstream>
#include <sstream>
#include <sys/stat.h>

#include <dlfcn.h>

namespace gs {

const char *reduction_kind_name(reduction_kind k) {
    switch (k) {
        case reduction_kind::TOTAL_BMT_RESULT: return "total_BMT_result_reduce_to_one_register_token";
        case reduction_kind::THREAD_BIT_MAP: return "thread_bit_map_reduce_to_two_register_token";
        case reduction_kind::TOTAL_WARP_RESULT: return "total_warp_result_reduce_to_one_register_token";
        case reduction_kind::WARP_SEGMENT: return "warp_segment_reduce_token";
        case reduction_kind::TOTAL_BLOCK_RESULT: return "total_block_reduce_to_one_register_token";
        case reduction_kind::WARP_BIT_MAP: return "warp_bit_map_reduce_token";
        case reduction_kind::TBLOCK_BIT_MAP: return "tblock_bit_map_reduce_token";
        default: return "none";
    }
}

const char *kernel_family_name(int f) {
    switch (f) {
        case KF_THREAD_TOTAL: return "k_thread_total";
        case KF_WARP_TOTAL: return "k_warp_rows";
        case KF_BLOCK_TOTAL: return "k_block_rows";
        case KF_BITMAP_SEGMENT: return "k_bitmap_segment";
        case KF_ROW_CHUNKS: return "k_row_chunks";
        case KF_MERGE_PATH: return "k_merge_path";  // the family; MP_ROWS picks the k_merge_rows walk
        default: return "none";
    }
}

std::string kernel_spec::name() const {
    std::string n = kernel_family_name(family);
    if (family == KF_BITMAP_SEGMENT && warp_segment) n += "+warp_segment";
    if (family == KF_WARP_TOTAL && tblock_parent) n += "+tblock";
    if (family == KF_ROW_CHUNKS && bitmap_parent == WARP_META) n += "+warp_bit_map";
    if (family == KF_ROW_CHUNKS && bitmap_parent == TBLOCK_META) n += "+tblock_bit_map";
    if (interleaved) n += "+interleaved";
    return n;
}

code_generator::code_generator(std::shared_ptr<meta_data_set> m, int sub_matrix_id) : meta(std::move(m)), sub(sub_matrix_id) {
    GS_CHECK(meta != nullptr, "code_generator needs a metadata set");
    GS_CHECK(sub_matrix_id >= 0, "sub_matrix_id >= 0");
}

void code_generator::set_reduction_token(POS_TYPE pos, const reduction_token &tok) {
    // code_generator.cc:2451-2485: a level holds one reduction token
    GS_CHECK(tokens.count(pos) == 0, "a reduction token is already set for " + convert_pos_type_to_string(pos));
    tokens[pos] = tok;
}

void code_generator::set_thread_grid(const std::vector<unsigned> &g, const std::vector<unsigned> &b) {
    grid = g;
    block = b;
}

// code_generator.cc:2586-2616 assembles the kernel text from the tokens; here the
// token set selects one of the hand-written families.
void code_generator::compile() {
    GS_CHECK(!compiled, "code_generator::compile may run once");
    kernel_spec s;
    const meta_data_set &m = *meta;
    auto tok = [&](POS_TYPE p) -> const reduction_token * { return tokens.count(p) ? &tokens.at(p) : nullptr; };
    const reduction_token *tt = tok(THREAD_META), *tw = tok(WARP_META), *tb = tok(TBLOCK_META);
    const reduction_token *tm = merge_level != GLOBAL_META ? tok(merge_level) : nullptr;
    if (tm && (tm->kind == reduction_kind::TOTAL_BMT_RESULT || tm->kind == reduction_kind::TOTAL_WARP_RESULT ||
               tm->kind == reduction_kind::TOTAL_BLOCK_RESULT)) {
        // merge-path levels + the level's total-reduce token (the compositions the
        // reference's name rules accept: merge_path_{thread,warp,tblock} followed by
        // {thread,warp,tblock}_total_reduce).  The reference emits no working kernel
        // for multi-row levels; here they map to k_merge_path.
        s.family = KF_MERGE_PATH;
        s.coarsen_factor = tm->coarsen_factor;
        s.merge_level = merge_level;
        s.work_size = merge_work_size;
        const std::string L = convert_pos_type_to_string(merge_level);
        s.arrays = {L + "_first_row_indices_without_ending_0", L + "_first_nz_indices_0"};
    } else if (tt && tt->kind == reduction_kind::TOTAL_BMT_RESULT &&
        m.is_exist(THREAD_META, "first_row_indices_without_ending", sub)) {
        // col-direction BMTs (A10) summed per row: K5 warp_bit_map / K7 tblock_bit_map
        s.family = KF_ROW_CHUNKS;
        s.coarsen_factor = tt->coarsen_factor;
        s.sparse_coarsen_factor = tt->sparse_coarsen_factor;
        s.arrays = {"THREAD_META_first_nz_indices_0", "THREAD_META_first_row_indices_without_ending_0"};
        if (tw && tw->kind == reduction_kind::WARP_BIT_MAP) {
            s.bitmap_parent = WARP_META;
            s.vector_width = tw->size;
            for (auto k : {"WARP_META_first_row_indices_0", "WARP_META_first_nz_indices_0", "WARP_META_first_BMT_indices_0",
                           "WARP_META_bit_map_of_thread_0"})
                s.arrays.push_back(k);
        } else if (tb && tb->kind == reduction_kind::TBLOCK_BIT_MAP) {
            s.bitmap_parent = TBLOCK_META;
            s.vector_width = tb->size;
            for (auto k : {"TBLOCK_META_first_row_indices_0", "TBLOCK_META_first_nz_indices_0",
                           "TBLOCK_META_first_BMT_indices_0", "THREAD_META_bit_map_of_thread_0",
                           "THREAD_META_segment_offset_0"})
                s.arrays.push_back(k);
        }
    } else if (tt && tt->kind == reduction_kind::THREAD_BIT_MAP) {
        s.family = KF_BITMAP_SEGMENT;
        s.warp_segment = tw && tw->kind == reduction_kind::WARP_SEGMENT;
        s.coarsen_factor = tt->coarsen_factor;
        s.sparse_coarsen_factor = tt->sparse_coarsen_factor;
        s.vector_width = tt->size;
        s.arrays = {"THREAD_META_first_nz_indices_0", "THREAD_META_first_row_indices_0", "THREAD_META_thread_bit_map_0",
                    "THREAD_META_segment_ptr_0", "THREAD_META_segment_empty_row_indices_0",
                    "THREAD_META_segment_empty_flag_0", "THREAD_META_segment_offset_0"};
        if (s.warp_segment)
            for (auto k : {"WARP_META_first_row_indices_0", "WARP_META_first_nz_indices_0", "WARP_META_first_BMT_indices_0"})
                s.arrays.push_back(k);
    } else if (tt && tt->kind == reduction_kind::TOTAL_BMT_RESULT && !tt->need_warp_reduction &&
               !m.is_exist(GLOBAL_META, "original_nz_row_indices", sub) &&
               m.is_exist(THREAD_META, "first_row_indices", sub) && [&] {
                   const auto &fr = m.u(THREAD_META, "first_row_indices", sub);
                   for (size_t i = 0; i < fr.size(); i++)
                       if (fr[i] != i) return true;
                   return false;
               }()) {
        // multi-row BMTs (balanced_interval_row_direction_thread_blocking_operator, or fixed
        // row blocking inside BMTB/BMW parents, whose absolute starts end with row_num / nnz
        // like the parentless arrays): every BMT is a run of whole rows, summed row by row ->
        // the wave-per-row-group kernel
        s.family = KF_WARP_TOTAL;
        s.group_level = THREAD_META;
        s.coarsen_factor = tt->coarsen_factor;
        s.arrays = {"THREAD_META_first_row_indices_0", "THREAD_META_first_nz_indices_0"};
    } else if (tt && tt->kind == reduction_kind::TOTAL_BMT_RESULT) {
        GS_CHECK(!tt->need_warp_reduction,
                 "thread_total with need_warp_reduction (col-direction warp_bit_map plans) is not built in this round");
        GS_CHECK(m.is_exist(THREAD_META, "first_row_indices", sub),
                 "thread_total over col-direction BMTs without a bit-map token is not built in this round");
        s.family = KF_THREAD_TOTAL;
        s.coarsen_factor = tt->coarsen_factor;
        s.sparse_coarsen_factor = tt->sparse_coarsen_factor;
        s.row_sorted = m.is_exist(GLOBAL_META, "original_nz_row_indices", sub);
        s.arrays = {"THREAD_META_first_nz_indices_0", "THREAD_META_first_row_indices_0"};
        if (s.row_sorted) s.arrays.push_back("GLOBAL_META_original_nz_row_indices_0");
    } else if ((tw && tw->kind == reduction_kind::TOTAL_WARP_RESULT &&
                m.is_exist(WARP_META, "first_row_indices_without_ending", sub)) ||
               (tb && tb->kind == reduction_kind::TOTAL_BLOCK_RESULT && !tw &&
                m.is_exist(TBLOCK_META, "first_row_indices_without_ending", sub))) {
        // col-direction BMWs / BMTBs (fixed_interval_col_direction_{warp,tblock}_blocking_operator):
        // chunks of one row, so a row's chunks are summed across units -> the row-chunk kernel
        // over that level's chunks.  The reference's total-reduce tokens read first_row_indices,
        // which these levels do not have (total_warp_result_reduce_to_one_register_token.cc:661)
        const bool w = tw && tw->kind == reduction_kind::TOTAL_WARP_RESULT;
        const std::string L = w ? "WARP_META" : "TBLOCK_META";
        s.family = KF_ROW_CHUNKS;
        s.coarsen_factor = w ? tw->coarsen_factor : tb->coarsen_factor;
        s.arrays = {L + "_first_nz_indices_0", L + "_first_row_indices_without_ending_0"};
    } else if (tw && tw->kind == reduction_kind::TOTAL_WARP_RESULT) {
        s.family = KF_WARP_TOTAL;
        s.coarsen_factor = tw->coarsen_factor;
        s.tblock_parent = m.is_exist(TBLOCK_META, "first_BMW_indices", sub);
        s.arrays = {"WARP_META_first_row_indices_0", "WARP_META_first_nz_indices_0"};
        if (s.tblock_parent) {
            s.arrays.push_back("TBLOCK_META_first_row_indices_0");
            s.arrays.push_back("TBLOCK_META_first_nz_indices_0");
            s.arrays.push_back("TBLOCK_META_first_BMW_indices_0");
        }
    } else if (tb && tb->kind == reduction_kind::TOTAL_BLOCK_RESULT) {
        s.family = KF_BLOCK_TOTAL;
        s.coarsen_factor = tb->coarsen_factor;
        s.arrays = {"TBLOCK_META_first_row_indices_0", "TBLOCK_META_first_nz_indices_0"};
    } else {
        throw gs_error("code_generator::compile: no reduction token set (or a combination not built in this round)");
    }
    if (interleave) {
        // interleaved storage is consumed by the col-direction chunk kernel over the BMTs,
        // interleaved as one run (GLOBAL parent) or per TBLOCK / WARP parent
        GS_CHECK(s.family == KF_ROW_CHUNKS && s.arrays[0].rfind("THREAD_META", 0) == 0,
                 "interleaved storage is built for col-direction BMT plans only");
        s.interleaved = true;
        s.interleave_parent = interleave_parent;
        for (auto k : {"GLOBAL_META_nz_col_indices_after_interlance_storage_0", "GLOBAL_META_nz_vals_after_interlance_storage_0"})
            s.arrays.push_back(k);
        const std::string L = interleave_parent == GLOBAL_META ? "GLOBAL_META"
                              : (interleave_parent == TBLOCK_META ? "TBLOCK_META" : "WARP_META");
        s.arrays.push_back(L + "_BMT_size_of_each_blk_0");
        if (interleave_parent != GLOBAL_META) {
            s.arrays.push_back(L + "_first_BMT_indices_0");
            s.arrays.push_back(L + "_first_nz_indices_0");
        }
    }
    for (auto k : {"GLOBAL_META_nz_row_indices_0", "GLOBAL_META_nz_col_indices_0", "GLOBAL_META_nz_vals_0"})
        s.arrays.push_back(k);
    // the keys above are written for sub-matrix 0; a divided matrix's sub-matrices carry their id
    if (sub != 0)
        for (auto &k : s.arrays)
            if (k.size() > 2 && k.compare(k.size() - 2, 2, "_0") == 0) k = k.substr(0, k.size() - 2) + "_" + std::to_string(sub);
    for (auto &k : s.arrays) GS_CHECK(m.is_exist(k), "compile: plan array missing: " + k);
    if (grid.size() == 2) s.ref_grid = {{grid[0], grid[1]}};
    if (block.size() == 2) s.ref_block = {{block[0], block[1]}};
    spec = s;
    compiled = true;
}

// ------------------------------------------------------------------ emission
namespace {

// the matrix-core program: the layout arrays (binary sidecars next to the plan's text
// arrays, code_generator.cc:311-336 writes the reference's as text) uploaded as they are,
// and the kernel launched with the template arguments and scalars gs_spmm uses
// (kernels/{ks,mfma}_launch.hip); the check and perf_result as for the other families
std::string matrix_core_source(const meta_data_set &m, const mc_layout &L, int repeat) {
    std::ostringstream o;
    const uint32_t N = L.N, CT = L.kind == mc_layout::NM ? std::max<uint32_t>(1, N / 16)
                                                         : (L.kind == mc_layout::KS ? L.ks.CT : ks_ct(N));
    const uint32_t NT = L.kind == mc_layout::KS ? ks_col_tiles_ct(N, CT) : ks_col_tiles(N);
    const char *kname = L.kind == mc_layout::KS ? "k_mfma_ks"
                        : L.kind == mc_layout::BM ? (L.bm.kb ? "k_mfma_kb" : L.bm.v2 ? "k_mfma_bm2" : "k_mfma_bm")
                        : L.kind == mc_layout::ROWS ? "k_mfma_rows"
                        : (L.nm_ks ? "k_nm_mfma_ks" : (L.nm4 ? "k_nm_mfma4" : "k_nm_mfma"));
    o << "// kernel_file.hip -- generated by generalsparse_amd code_generator: the matrix-core kernel " << kname << "\n"
      << "// build: sh make_kernel.sh; run: ./a.out [matrix.mtx] [N]  -> perf_result (ms, GFLOP/s)\n"
      << (L.kind == mc_layout::BM || L.nm_ks || L.rows_flags ? "#define GS_EXPERIMENTS  // an experiments-build kernel\n" : "")
      << "#include \"kernel_lib.hpp\"\n#include <cstdio>\n#include <cstdlib>\n#include <cstring>\n#include <fstream>\n"
      << "#include <string>\n#include <vector>\n\n"
      << "typedef gsk::f16 VT;\n"
      << "static std::vector<uint64_t> rd(const char *n) {\n"
      << "    std::ifstream f(n); std::vector<uint64_t> v; unsigned long long x; while (f >> x) v.push_back(x); return v; }\n"
      << "static std::vector<double> rdf(const char *n) {\n"
      << "    std::ifstream f(n); std::vector<double> v; double x; while (f >> x) v.push_back(x); return v; }\n"
      << "template <class T> static std::vector<T> rdb(const char *n) {  // binary sidecar\n"
      << "    std::ifstream f(n, std::ios::binary | std::ios::ate); std::vector<T> v((size_t)f.tellg() / sizeof(T));\n"
      << "    f.seekg(0); f.read(reinterpret_cast<char *>(v.data()), v.size() * sizeof(T)); return v; }\n"
      << "template <class T> static T *up(const std::vector<T> &h, size_t pad = 64) {\n"
      << "    T *p; hipMalloc(&p, (h.size() + pad) * sizeof(T)); hipMemset(p, 0, (h.size() + pad) * sizeof(T));\n"
      << "    hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); return p; }\n\n"
      << "int main(int argc, char **argv) {\n"
      << "    const uint32_t N = argc > 2 ? (uint32_t)atoi(argv[2]) : " << N << ";\n"
      << "    if (N != " << N << ") { printf(\"this program's " << kname << " layout is built for N = " << N
      << "\\n\"); return 2; }\n"
      << "    const int repeat = " << repeat << ";\n"
      << "    const uint64_t M = " << m.scalar(GLOBAL_META, "origin_row_num", -1) << ", K = "
      << m.scalar(GLOBAL_META, "origin_col_num", -1) << ", NNZ = " << m.scalar(GLOBAL_META, "origin_nnz_num", -1) << ";\n"
      << "    auto rows = rd(\"GLOBAL_META_nz_row_indices_0\");\n"
      << "    auto vals = rdf(\"GLOBAL_META_nz_vals_0\");\n"
      << "    uint64_t row_num = rows.back() + 1;\n";
    std::string launch, setup;
    if (L.kind == mc_layout::KS) {
        const ks_tiles &t = L.ks;
        const uint64_t nb = L.tbr.size() - 1, nwg = nb * t.S;
        o << "    auto tbr = rd(\"TBLOCK_META_first_row_indices_0\");\n"
          << "    std::vector<uint32_t> t32(tbr.begin(), tbr.end()); uint32_t *d_tbr = up(t32);\n"
          << (t.P8 ? "    uint8_t *d_pos = up(rdb<uint8_t>(\"TBLOCK_META_mfma_ks_entry_pos_0.bin\"));  // 8-bit positions\n"
                   : "    uint16_t *d_pos = up(rdb<uint16_t>(\"TBLOCK_META_mfma_ks_entry_pos_0.bin\"));\n")
          << "    uint16_t *d_val = up(rdb<uint16_t>(\"TBLOCK_META_mfma_ks_entry_val_0.bin\"));\n"
          << "    uint32_t *d_steps = up(rdb<uint32_t>(\"TBLOCK_META_mfma_ks_steps_0.bin\"));\n"
          << "    // the tagged slabs start (and are left by every launch) all 0\n"
          << "    float *d_ws; uint32_t *d_arr; hipMalloc(&d_ws, " << nwg * NT * 256 * t.RT * CT * 4 << "ull + 16);\n"
          << "    hipMemset(d_ws, 0, " << nwg * NT * 256 * t.RT * CT * 4 << "ull + 16);\n"
          << "    hipMalloc(&d_arr, " << nb * NT * 4 << "ull + 4); hipMemset(d_arr, 0, " << nb * NT * 4
          << "ull + 4);\n";
        const std::string k = "gsk::k_mfma_ks<" + std::to_string(CT) + ", " + std::to_string(t.RT) + ", " +
                              std::to_string(t.W) + ", " + std::to_string(kKsDepth) + ", " + std::to_string(t.MAXG) +
                              std::string(", false, ") + (t.AP ? "true" : "false") + ", " + (t.P8 ? "true" : "false") +
                              (t.NT ? ", " + std::to_string(t.NT) + ">" : ">");
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(t.lds_bytes) + ")";
        launch = k + "<<<dim3(" + std::to_string(nwg) + ", " + std::to_string(NT) + "), " +
                 std::to_string(64 * t.W) + ", " + std::to_string(t.lds_bytes) +
                 ">>>(d_tbr, (const gsk::u32x4 *)d_pos, (const gsk::u32x4 *)d_val, (const gsk::u32x2 *)d_steps, d_B, d_C, "
                 "(uint32_t)K, N, " + std::to_string(t.S) + "u, " + std::to_string(t.NS) + "u, " + std::to_string(nwg) + "u, 0u, d_ws, d_arr, nullptr, " +
                 std::to_string((uint32_t)get_config().KS_PRIO | (t.GH << 8)) + "u)";
    } else if (L.kind == mc_layout::BM) {
        const bm_tiles &t = L.bm;
        const uint64_t nb = L.tbr.size() - 1, nwg = nb * t.S;
        o << "    auto tbr = rd(\"TBLOCK_META_first_row_indices_0\");\n"
          << "    std::vector<uint32_t> t32(tbr.begin(), tbr.end()); uint32_t *d_tbr = up(t32);\n"
          << "    uint32_t *d_rec = up(rdb<uint32_t>(\"TBLOCK_META_mfma_bm_records_0.bin\"));\n"
          << "    uint32_t *d_sb = up(rdb<uint32_t>(\"TBLOCK_META_mfma_bm_step_base_0.bin\"));\n"
          << "    uint16_t *d_val = up(rdb<uint16_t>(\"TBLOCK_META_mfma_bm_values_0.bin\"));\n"
          << "    float *d_ws; uint32_t *d_arr; hipMalloc(&d_ws, " << nwg * ks_col_tiles(N) * 256 * t.RT * CT * 4 << "ull + 16);\n"
          << "    hipMalloc(&d_arr, " << nb * ks_col_tiles(N) * t.RT * 4 << "ull + 4); hipMemset(d_arr, 0, "
          << nb * ks_col_tiles(N) * t.RT * 4 << "ull + 4);\n";
        if (t.kb) o << "    hipMemset(d_ws, 0, " << nwg * ks_col_tiles(N) * 256 * t.RT * CT * 4 << "ull + 16);\n";
        const std::string k = t.kb ? "gsk::k_mfma_kb<" + std::to_string(CT) + ", " + std::to_string(t.RT) + ", " +
                                         std::to_string(t.W) + ", " + std::to_string(kKsDepth) + ", " +
                                         std::to_string(t.NVB) + ">"
                            : t.v2 ? "gsk::k_mfma_bm2<" + std::to_string(CT) + ", " + std::to_string(t.RT) + ">"
                                   : "gsk::k_mfma_bm<" + std::to_string(CT) + ", " + std::to_string(t.RT) + ", " +
                                         std::to_string(t.W) + ", " + std::to_string(gsk::bm_nbt(CT, t.RT)) + ">";
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(t.lds_bytes) + ")";
        launch = k + "<<<dim3(" + std::to_string(nwg) + ", " + std::to_string(ks_col_tiles(N)) + "), " +
                 std::to_string(64 * t.W) + ", " + std::to_string(t.lds_bytes) +
                 ">>>(d_tbr, (const uint2 *)d_rec, d_sb, (const gsk::f16 *)d_val, d_B, d_C, (uint32_t)K, N, " +
                 std::to_string(t.S) + "u, " + std::to_string(t.NS) + "u, " + std::to_string(nwg) + "u, 0u, d_ws, d_arr" +
                 (t.kb ? ", nullptr, " + std::to_string(get_config().KS_PRIO) + "u)" : std::string(")"));
    } else if (L.kind == mc_layout::ROWS) {
        const mfma_tiles &t = L.rows;
        const uint64_t nb = L.tbr.size() - 1;
        o << "    auto tbr = rd(\"TBLOCK_META_first_row_indices_0\");\n"
          << "    std::vector<uint32_t> t32(tbr.begin(), tbr.end()); uint32_t *d_tbr = up(t32);\n"
          << "    uint32_t *d_seg = up(rdb<uint32_t>(\"TBLOCK_META_mfma_seg_start_0.bin\"));\n"
          << "    uint16_t *d_pos = up(rdb<uint16_t>(\"TBLOCK_META_mfma_entry_pos_0.bin\"));\n"
          << "    uint16_t *d_val = up(rdb<uint16_t>(\"TBLOCK_META_mfma_entry_val_0.bin\"));\n"
          << "    float *d_ws = nullptr; uint32_t *d_arr = nullptr;\n";
        if (L.rows_ksplit > 1)
            o << "    hipMalloc(&d_ws, " << nb * L.rows_ksplit * t.RMAX * N * 4 << "ull); hipMalloc(&d_arr, " << nb * 4
              << "ull); hipMemset(d_arr, 0, " << nb * 4 << "ull);\n";
        const std::string k = "gsk::k_mfma_rows<" + std::to_string(CT) + ", " + std::to_string(t.RT) + ", " +
                              std::to_string(t.lgKC) + ", " + std::to_string(L.rows_maxa) + ", false, " +
                              std::to_string(L.rows_glds) + ", " + std::to_string(L.rows_nbg) + ", " +
                              std::to_string(L.rows_wct) + (L.rows_flags ? ", 0, true>" : ">");
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(t.lds_bytes) + ")";
        launch = k + "<<<" + std::to_string(nb * L.rows_ksplit) + ", " + std::to_string(kMfmaThreads) + ", " +
                 std::to_string(t.lds_bytes) + ">>>(d_tbr, d_seg, (const gsk::u32x4 *)d_pos, (const gsk::u32x4 *)d_val, d_B, d_C, " +
                 "(uint32_t)K, N, " + std::to_string(t.nc) + "u, " + std::to_string(t.RMAX) + "u, 0u, " +
                 std::to_string(L.rows_ksplit) + "u, " + std::to_string(L.rows_ncs) + "u, d_ws, d_arr, nullptr, 0u)";
    } else if (L.nm_ks) {
        const uint64_t nb = (L.nm_rows + 255) / 256, ngr = nb * 4;
        o << "    unsigned char *d_blk = up(rdb<unsigned char>(\"THREAD_META_nm_panels_0.bin\"));\n"
          << "    float *d_ws; uint32_t *d_arr; hipMalloc(&d_ws, " << ngr * L.nm_split * 64 * N * 4 << "ull + 16);\n"
          << "    hipMalloc(&d_arr, " << ngr * 4 << "ull); hipMemset(d_arr, 0, " << ngr * 4 << "ull);\n";
        const std::string k = "gsk::k_nm_mfma_ks<" + std::to_string(CT) + ">";
        const size_t lds = (size_t)2 * gsk::kNmKC * 32 * CT;
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(lds) + ")";
        launch = k + "<<<" + std::to_string(nb * L.nm_split) + ", 256, " + std::to_string(lds) +
                 ">>>(d_blk, d_B, d_C, (uint32_t)K, " + std::to_string(L.nm_S) + "u, " + std::to_string(L.nm_rows) +
                 "u, 0u, " + std::to_string(L.nm_split) + "u, " + std::to_string(L.nm_ncs) + "u, d_ws, d_arr)";
    } else if (L.nm4) {
        const uint64_t nb = (L.nm_rows + 255) / 256, nwg = nb * L.nm_split;
        o << "    unsigned char *d_blk = up(rdb<unsigned char>(\"THREAD_META_nm_panels_0.bin\"));\n"
          << "    // the tagged slabs and the arrival counters start all 0\n"
          << "    float *d_ws; uint32_t *d_arr; hipMalloc(&d_ws, " << nwg * 256 * N * 4 << "ull + 16); hipMemset(d_ws, 0, "
          << nwg * 256 * N * 4 << "ull + 16);\n"
          << "    hipMalloc(&d_arr, " << (nb + 1) * 4 << "ull); hipMemset(d_arr, 0, " << (nb + 1) * 4 << "ull);\n";
        const std::string k = "gsk::k_nm_mfma4<" + std::to_string(CT) + ">";
        const size_t lds = gsk::nm4_lds_bytes(CT);
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(lds) + ")";
        launch = k + "<<<" + std::to_string(nwg) + ", " + std::to_string(64 * gsk::kNmWaves) + ", " + std::to_string(lds) +
                 ">>>(d_blk, d_B, d_C, (uint32_t)K, " + std::to_string(L.nm_S) + "u, " + std::to_string(L.nm_rows) +
                 "u, 0u, " + std::to_string(L.nm_split) + "u, " + std::to_string(L.nm_ncs) + "u, " + std::to_string(nwg) +
                 "u, d_ws, d_arr, 0u)";
    } else {
        o << "    unsigned char *d_blk = up(rdb<unsigned char>(\"THREAD_META_nm_panels_0.bin\"));\n";
        // N = 8: one half-used 16-column tile (k_nm_mfma's NG)
        // TT: 16-row tiles per workgroup (the layout's nm_T)
        const std::string k = "gsk::k_nm_mfma<" + std::to_string(CT) + ", 0, " + std::to_string(N == 8 ? 8 : 16 * CT) +
                              (L.nm_nt ? ", true, " : ", false, ") + std::to_string(L.nm_T) + ">";
        const size_t lds = (size_t)2 * gsk::kNmKC * 32 * CT;
        setup = "hipFuncSetAttribute((const void *)" + k + ", hipFuncAttributeMaxDynamicSharedMemorySize, " +
                std::to_string(lds) + ")";
        launch = k + "<<<" + std::to_string((L.nm_rows + 16 * L.nm_T - 1) / (16 * L.nm_T)) + ", " +
                 std::to_string(64 * gsk::kNmWaves) + ", " +
                 std::to_string(lds) + ">>>(d_blk, d_B, d_C, (uint32_t)K, " + std::to_string(L.nm_S) + "u, " +
                 std::to_string(L.nm_rows) + "u, 0u, " + std::to_string((uint32_t)get_config().NM_KROT) + "u)";
    }
    o << "    std::vector<VT> hB(K * N, (VT)1.0f);  // x_arr = 1 (code_generator.cc:464-467)\n"
      << "    VT *d_B = up(hB, 0); VT *d_C; hipMalloc(&d_C, M * N * sizeof(VT)); hipMemset(d_C, 0, M * N * sizeof(VT));\n"
      << "    " << setup << ";\n"
      << "    auto run = [&]() { " << launch << "; };\n"
      << "    run(); if (hipDeviceSynchronize() != hipSuccess) { printf(\"launch failed\\n\"); return 3; }\n"
      << "    // check (kernel_lib.hpp:884-921 of the reference): all-ones B, C[i][j] = sum of row i's values\n"
      << "    std::vector<VT> hC(M * N); hipMemcpy(hC.data(), d_C, M * N * sizeof(VT), hipMemcpyDeviceToHost);\n"
      << "    std::vector<double> ref(M, 0.0);\n"
      << "    for (size_t i = 0; i < rows.size(); i++) ref[rows[i]] += vals[i];\n"
      << "    long wrong = 0;\n"
      << "    for (uint64_t i = 0; i < M; i++) for (uint32_t j = 0; j < N; j++) {\n"
      << "        double c = (double)(float)hC[i * N + j], r = (double)(float)(VT)(float)ref[i];\n"
      << "        const double tol = 1e-1 * (1 + (r < 0 ? -r : r));  // north_star fp16\n"
      << "        if (c - r > tol || r - c > tol) {\n"
      << "            if (wrong < 10) printf(\"Wrong result: i = %llu, j = %u, result = %f, reference = %f.\\n\", (unsigned long long)i, j, c, r);\n"
      << "            wrong++; } }\n"
      << "    printf(\"wrong number:%ld\\n\", wrong); if (!wrong) printf(\"correct\\n\");\n"
      << "    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);\n"
      << "    for (int i = 0; i < 20; i++) run();  // warm-up\n"
      << "    hipEventRecord(e0, 0); for (int i = 0; i < repeat; i++) run(); hipEventRecord(e1, 0); hipEventSynchronize(e1);\n"
      << "    float ms = 0; hipEventElapsedTime(&ms, e0, e1);\n"
      << "    double gflops = " << get_config().FLOAT_RATE << ".0 * (double)NNZ * N * repeat / (ms * 1e-3) / 1e9;\n"
      << "    FILE *pr = fopen(\"perf_result\", \"w\"); fprintf(pr, \"%f\\n%f\\n\", ms, gflops); fclose(pr);  // code_generator.cc:643-648\n"
      << "    printf(\"time %f ms for %d launches, %f GFLOP/s\\n\", ms, repeat, gflops);\n"
      << "    return wrong ? 1 : 0;\n}\n";
    return o.str();
}

template <class T>
void write_bin(const std::string &path, const std::vector<T> &v) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    GS_CHECK(f.good(), "cannot write " + path);
}

mc_layout emitted_layout(const meta_data_set &m, const kernel_spec &spec, int sub) {
    if (!get_config().HALF) return mc_layout();
    return choose_matrix_core_layout(m, spec, sub, m.scalar(GLOBAL_META, "origin_col_num", -1), 1);
}

}  // namespace

std::string code_generator::generate_kernel_file_source(int repeat) const {
    GS_CHECK(compiled, "compile() before emitting the program");
    GS_CHECK(sub == 0, "the standalone program is emitted for an undivided matrix");
    const mc_layout L = emitted_layout(*meta, spec, sub);
    if (L.kind != mc_layout::NONE) return matrix_core_source(*meta, L, repeat);
    return generate_gather_source(repeat);
}

std::string code_generator::generate_gather_source(int repeat) const {
    const bool half = get_config().HALF;
    // model-driven index compression (code_generator.cc:2618-3063): with
    // MODEL_DRIVEN_COMPRESS, integer plan arrays whose formula reproduces them exactly are
    // generated from the formula instead of read
    std::string formulas;
    if (get_config().MODEL_DRIVEN_COMPRESS)
        for (const auto &k : spec.arrays) {
            auto arr = meta->get_element(k)->meta_data_arr;
            if (arr->is_float()) continue;
            index_compression c = analyze_index_compression(arr->u(), arr->get_compress_data_type(),
                                                            get_config().BRANCH_COMPRESS_MAX_SIZE);
            if (!c.exact || c.kind == "residual") continue;
            formulas += "    if (!std::strcmp(n, \"" + k + "\")) { std::vector<uint64_t> v(" + std::to_string(arr->get_len()) +
                        "); for (uint64_t i = 0; i < v.size(); i++) v[i] = " + code_of_index_compression(c, "i", "") +
                        "; return v; }  // " + c.kind + "\n";
        }
    std::ostringstream o;
    o << "// kernel_file.hip -- generated by generalsparse_amd code_generator for plan family "
      << spec.name() << "\n"
      << "// build: sh make_kernel.sh; run: ./a.out [matrix.mtx] [N]  -> perf_result (ms, GFLOP/s)\n"
      << (get_config().MP_ROWS ? "#define GS_EXPERIMENTS  // an experiments-build kernel\n" : "")
      << "#include \"kernel_lib.hpp\"\n#include <cstdio>\n#include <cstdlib>\n#include <cstring>\n#include <fstream>\n"
      << "#include <string>\n#include <vector>\n\n"
      << "typedef " << (half ? "gsk::f16" : "float") << " VT;\n"
      << "static std::vector<uint64_t> rd(const char *n) {\n" << formulas
      << "    std::ifstream f(n); std::vector<uint64_t> v; unsigned long long x;\n"
      << "    while (f >> x) v.push_back(x); return v; }\n"
      << "static std::vector<double> rdf(const char *n) {\n"
      << "    std::ifstream f(n); std::vector<double> v; double x; while (f >> x) v.push_back(x); return v; }\n"
      << "template <class T> static T *up(const std::vector<T> &h, size_t pad = 64) {\n"
      << "    T *p; hipMalloc(&p, (h.size() + pad) * sizeof(T)); hipMemset(p, 0, (h.size() + pad) * sizeof(T));\n"
      << "    hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); return p; }\n"
      << "static std::vector<uint32_t> u32(const std::vector<uint64_t> &v) { return std::vector<uint32_t>(v.begin(), v.end()); }\n\n"
      << "int main(int argc, char **argv) {\n"
      << "    const uint32_t N = argc > 2 ? (uint32_t)atoi(argv[2]) : " << get_config().DENSE_MATRIX_SIZE << ";\n"
      << "    const int repeat = " << repeat << ";\n"
      << "    const uint64_t M = " << meta->scalar(GLOBAL_META, "origin_row_num", -1) << ", K = "
      << meta->scalar(GLOBAL_META, "origin_col_num", -1) << ", NNZ = " << meta->scalar(GLOBAL_META, "origin_nnz_num", -1)
      << ";\n"
      << "    auto rows = rd(\"GLOBAL_META_nz_row_indices_0\");\n"
      << "    auto cols = rd(\"GLOBAL_META_nz_col_indices_0\");\n"
      << "    auto vals = rdf(\"GLOBAL_META_nz_vals_0\");\n"
      << "    std::vector<uint32_t> c32(cols.begin(), cols.end());\n"
      << "    std::vector<VT> vv(vals.size()); for (size_t i = 0; i < vals.size(); i++) vv[i] = (VT)vals[i];\n"
      << "    uint32_t *d_col = up(c32); VT *d_val = up(vv);\n"
      << "    uint64_t row_num = rows.back() + 1;\n";
    // the index arrays the gather kernels read through gsk::idx_at: an exact formula is a
    // kernel argument and the array is not uploaded (the reference prints the expression
    // into the kernel instead, code_generator.cc:2618-3063)
    auto fml = [&](const std::string &key) {
        gsk::idx_formula f;
        if (!get_config().MODEL_DRIVEN_COMPRESS || !meta->is_exist(key)) return f;
        auto arr = meta->get_element(key)->meta_data_arr;
        index_compression c = analyze_index_compression(arr->u(), arr->get_compress_data_type(),
                                                        get_config().BRANCH_COMPRESS_MAX_SIZE);
        if (c.kind == "residual" || !device_formula_of(c, f)) f = gsk::idx_formula();
        return f;
    };
    auto decl = [&](const char *name, const gsk::idx_formula &f) {
        o << "    const gsk::idx_formula " << name << " = " << code_of_device_formula(f) << ";\n";
    };
    gsk::idx_formula identity;
    identity.kind = gsk::IDX_LINEAR;
    identity.coef = 1;
    const char *cf = half ? "8" : "4";
    std::string launch;
    switch (spec.family) {
        case KF_THREAD_TOTAL:
            decl("F0", fml("THREAD_META_first_nz_indices_0"));
            decl("F1", spec.row_sorted ? fml("GLOBAL_META_original_nz_row_indices_0")
                                       : (get_config().MODEL_DRIVEN_COMPRESS ? identity : gsk::idx_formula()));
            o << "    auto fn = rd(\"THREAD_META_first_nz_indices_0\");\n";
            if (spec.row_sorted) o << "    auto order = rd(\"GLOBAL_META_original_nz_row_indices_0\");\n";
            else o << "    std::vector<uint64_t> order(M); for (uint64_t i = 0; i < M; i++) order[i] = i;\n";
            o << "    uint32_t *d_a0 = F0.kind ? nullptr : up(u32(fn)), *d_a1 = F1.kind ? nullptr : up(u32(order));\n"
              << "    const uint32_t n_units = fn.size() - 1, n_aux = order.size();\n"
              << "    bool al = true; for (auto x : fn) al &= x % 4 == 0;\n";
            launch = "gsk::k_thread_total<VT, uint32_t, CF, SCF><<<dim3((n_aux + 256 / X - 1) / (256 / X), tiles), 256>>>("
                     "d_a0, F0, d_a1, F1, d_col, d_val, d_B, d_C, n_units, n_aux, N, X, 0)";
            break;
        case KF_WARP_TOTAL:
            decl("F0", fml(convert_pos_type_to_string(spec.group_level) + "_first_row_indices_0"));
            decl("F1", spec.tblock_parent ? fml("TBLOCK_META_first_BMW_indices_0") : gsk::idx_formula());
            o << "    auto wr = rd(\"" << convert_pos_type_to_string(spec.group_level) << "_first_row_indices_0\");\n"
              << "    uint32_t *d_a0 = F0.kind ? nullptr : up(u32(wr)), *d_a1 = nullptr;\n"
              << "    uint32_t *d_a2 = up(gsk_host::csr_row_ptr(rows, wr.back()));\n"
              << "    const uint32_t n_units = wr.size() - 1; uint32_t gx = (n_units + 3) / 4; const bool al = true;\n";
            if (spec.tblock_parent)
                o << "    auto tbw = rd(\"TBLOCK_META_first_BMW_indices_0\"); d_a1 = F1.kind ? nullptr : up(u32(tbw)); gx = tbw.size() - 1;\n";
            launch = "gsk::k_warp_rows<VT, uint32_t, CF, SCF><<<dim3(gx, tiles), 256>>>(d_a0, F0, d_a1, F1, d_a2, d_col, d_val, d_B, d_C, n_units, N, X, 0)";
            break;
        case KF_BLOCK_TOTAL:
            decl("F0", fml("TBLOCK_META_first_row_indices_0"));
            o << "    auto tr = rd(\"TBLOCK_META_first_row_indices_0\");\n"
              << "    uint32_t *d_a0 = F0.kind ? nullptr : up(u32(tr)); uint32_t *d_a2 = up(gsk_host::csr_row_ptr(rows, tr.back()));\n"
              << "    const uint32_t n_units = tr.size() - 1; const bool al = true;\n";
            launch = "gsk::k_block_rows<VT, uint32_t, CF, SCF><<<dim3(n_units, tiles), 256>>>(d_a0, F0, d_a2, d_col, d_val, d_B, d_C, n_units, N, X, 0)";
            break;
        case KF_BITMAP_SEGMENT:
            decl("F0", fml("THREAD_META_first_nz_indices_0"));
            decl("F1", fml("THREAD_META_first_row_indices_0"));
            o << "    auto fn = rd(\"THREAD_META_first_nz_indices_0\"), fr = rd(\"THREAD_META_first_row_indices_0\");\n"
              << "    auto sp = rd(\"THREAD_META_segment_ptr_0\"), so = rd(\"THREAD_META_segment_empty_row_indices_0\");\n"
              << "    uint32_t *d_a0 = F0.kind ? nullptr : up(u32(fn)), *d_a1 = F1.kind ? nullptr : up(u32(fr)), *d_a2 = up(u32(sp)), *d_a3 = up(u32(so));\n"
              << "    uint64_t *d_m0 = up(gsk_host::row_start_masks(rows, fn));\n"
              << "    const uint32_t n_units = fn.size() - 1; const bool al = true;\n";
            launch = "hipMemsetAsync(d_C, 0, M * N * sizeof(VT), 0); "
                     "gsk::k_bitmap_segment<VT, uint32_t, CF, SCF><<<dim3((n_units + 4 * (64 / X) - 1) / (4 * (64 / X)), tiles), 256, "
                     "4 * (64 / X) * 2 * X * CF * sizeof(float)>>>(d_a0, F0, d_a1, F1, d_m0, d_a2, d_a3, d_col, d_val, d_B, d_C, n_units, N, X, 0, "
                     "(float *)nullptr)";  // no workspace: open rows by atomics into the zeroed C
            break;
        case KF_ROW_CHUNKS: {
            // the chunk level: THREAD (col-direction BMTs) or a col-direction WARP / TBLOCK level
            const std::string L = spec.arrays[0].substr(0, spec.arrays[0].find("_META_") + 5);
            decl("F0", fml(L + "_first_nz_indices_0"));
            decl("F1", fml(L + "_first_row_indices_without_ending_0"));
            o << "    auto fn = rd(\"" << L << "_first_nz_indices_0\"), fr = rd(\"" << L << "_first_row_indices_without_ending_0\");\n"
              << "    uint32_t *d_a0 = F0.kind ? nullptr : up(u32(fn)), *d_a1 = F1.kind ? nullptr : up(u32(fr));\n"
              << "    const uint32_t n_units = fn.size() - 1, U = gsk_host::row_chunk_span(n_units); const bool al = true;\n"
              << "    auto fin = gsk_host::row_chunk_finalize_rows(u32(fr), M, U, 0); uint32_t *d_a4 = up(fin);\n"
              << "    float *d_ws; hipMalloc(&d_ws, M * N * sizeof(float)); hipMemset(d_ws, 0, M * N * sizeof(float));\n";
            launch = "gsk::k_row_chunks<VT, uint32_t, CF, SCF><<<dim3(((n_units + U - 1) / U + 3) / 4, tiles), 256>>>("
                     "d_a0, F0, d_a1, F1, d_col, d_val, d_B, d_C, d_ws, n_units, U, N, X, 0); "
                     "if (!fin.empty()) gsk::k_finalize_rows<VT><<<dim3((fin.size() * N + 255) / 256), 256>>>("
                     "d_a4, (uint32_t)fin.size(), d_ws, d_C, N)";
            break;
        }
        case KF_MERGE_PATH: {
            const std::string L = convert_pos_type_to_string(spec.merge_level);
            o << "    auto lr = rd(\"" << L << "_first_row_indices_without_ending_0\"), ln = rd(\"" << L
              << "_first_nz_indices_0\");\n"
              << "    gsk_host::merge_path_layout lay; std::string why;\n"
              << "    if (!gsk_host::merge_path_device_layout(rows, row_num, lr, ln, " << spec.work_size
              << ", 0, 256, lay, why, M)) { printf(\"%s\\n\", why.c_str()); return 2; }\n"
              << "    uint32_t *d_a0 = up(lay.wz), *d_a1 = up(lay.wq), *d_a2 = up(lay.ends), *d_a3 = up(lay.rid), *d_a4 = up(lay.empty);\n"
              << "    const uint32_t n_units = lay.wz.size() - 1, n_crow = lay.ends.size(); const bool al = true;\n"
              << "    float *d_r0, *d_r1; uint32_t *d_rr; hipMalloc(&d_r0, n_units * N * 4); hipMalloc(&d_r1, n_units * N * 4);\n"
              << "    hipMalloc(&d_rr, n_units * 4);\n";
            if (get_config().MP_ROWS)  // the walk gs_spmm runs (device_plan.hip fixes it at upload)
                launch = "gsk::k_merge_rows<VT, uint32_t, CF><<<dim3((n_units + 3) / 4 + 64, tiles), 256, "
                         "4 * gsk::merge_rows_wave_words(X, CF, gsk::merge_rows_j<CF>()) * 4>>>(d_a0, d_a1, "
                         "d_a2, d_a3, n_crow, d_col, d_val, d_B, d_C, d_r0, d_rr, d_r1, n_units, N, X, d_a4, "
                         "(uint32_t)lay.empty.size(), 64u, nullptr, nullptr, " + std::to_string(std::max<int64_t>(1, get_config().MP_SOLO)) + "u); "
                         "gsk::k_merge_fixup<VT><<<dim3((n_units * N + 255) / 256), 256>>>(d_rr, d_r0, d_r1, d_C, n_units, N)";
            else
                launch = "gsk::k_merge_path<VT, uint32_t, CF><<<dim3((n_units + 3) / 4 + 64, tiles), 256, "
                         "4 * gsk::merge_path_wave_lds_words(64 / X) * 4>>>(d_a0, d_a1, d_a2, d_a3, n_crow, d_col, d_val, d_B, d_C, "
                         "d_r0, d_rr, d_r1, n_units, N, X, 0, (uint32_t)M, d_a4, (uint32_t)lay.empty.size(), 64u, nullptr, nullptr); "
                         "gsk::k_merge_fixup<VT><<<dim3((n_units * N + 255) / 256), 256>>>(d_rr, d_r0, d_r1, d_C, n_units, N)";
            break;
        }
        default:
            throw gs_error("no family");
    }
    o << "    std::vector<VT> hB(K * N, (VT)1.0f);  // x_arr = 1 (code_generator.cc:464-467)\n"
      << "    VT *d_B = up(hB, 0); VT *d_C; hipMalloc(&d_C, M * N * sizeof(VT)); hipMemset(d_C, 0, M * N * sizeof(VT));\n"
      << "    auto run = [&]() {\n"
      << "        if (al && N % " << cf << " == 0) {\n"
      << "            constexpr int CF = " << cf << ", SCF = 4; uint32_t X = 1; while (X < 64 && X * CF < N) X <<= 1;\n"
      << "            uint32_t tiles = (N + X * CF - 1) / (X * CF); " << launch << ";\n"
      << "        } else {\n"
      << "            constexpr int CF = 1, SCF = 1; uint32_t X = 1; while (X < 64 && X * CF < N) X <<= 1;\n"
      << "            uint32_t tiles = (N + X * CF - 1) / (X * CF); " << launch << ";\n"
      << "        }\n"
      << "    };\n"
      << "    run(); hipDeviceSynchronize();\n"
      << "    // check (kernel_lib.hpp:884-921 of the reference): all-ones B, C[i][j] = sum of row i's values\n"
      << "    std::vector<VT> hC(M * N); hipMemcpy(hC.data(), d_C, M * N * sizeof(VT), hipMemcpyDeviceToHost);\n"
      << "    std::vector<double> ref(M, 0.0);\n"
      << "    std::vector<uint64_t> orig_of(row_num);\n";
    if (spec.row_sorted)
        o << "    { auto order = rd(\"GLOBAL_META_original_nz_row_indices_0\"); for (uint64_t i = 0; i < row_num; i++) orig_of[i] = order[i]; }\n";
    else
        o << "    for (uint64_t i = 0; i < row_num; i++) orig_of[i] = i;\n";
    o << "    for (size_t i = 0; i < rows.size(); i++) ref[orig_of[rows[i]]] += vals[i];\n"
      << "    long wrong = 0;\n"
      << "    for (uint64_t i = 0; i < M; i++) for (uint32_t j = 0; j < N; j++) {\n"
      << "        double c = (double)(float)hC[i * N + j], r = (double)(float)(VT)(float)ref[i];\n"
      << "        const double tol = " << (half ? "1e-1" : "1e-3") << " * (1 + (r < 0 ? -r : r));  // north_star fp16 / fp32\n"
      << "        if (c - r > tol || r - c > tol) {\n"
      << "            if (wrong < 10) printf(\"Wrong result: i = %llu, j = %u, result = %f, reference = %f.\\n\", (unsigned long long)i, j, c, r);\n"
      << "            wrong++; } }\n"
      << "    printf(\"wrong number:%ld\\n\", wrong); if (!wrong) printf(\"correct\\n\");\n"
      << "    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);\n"
      << "    hipEventRecord(e0, 0); for (int i = 0; i < repeat; i++) run(); hipEventRecord(e1, 0); hipEventSynchronize(e1);\n"
      << "    float ms = 0; hipEventElapsedTime(&ms, e0, e1);\n"
      << "    double gflops = " << get_config().FLOAT_RATE << ".0 * (double)NNZ * N * repeat / (ms * 1e-3) / 1e9;\n"
      << "    FILE *pr = fopen(\"perf_result\", \"w\"); fprintf(pr, \"%f\\n%f\\n\", ms, gflops); fclose(pr);  // code_generator.cc:643-648\n"
      << "    printf(\"time %f ms for %d launches, %f GFLOP/s\\n\", ms, repeat, gflops);\n"
      << "    return wrong ? 1 : 0;\n}\n";
    return o.str();
}

uint64_t code_generator::generate_final_program(int repeat, const std::string &root, std::string *dir_out) {
    GS_CHECK(compiled, "compile() before generate_final_program");
    GS_CHECK(sub == 0, "the standalone program is emitted for an undivided matrix");
    std::string dir;
    uint64_t id = meta->output_format_to_dir(root, spec.arrays, &dir);
    const mc_layout L = emitted_layout(*meta, spec, sub);
    if (L.kind == mc_layout::KS) {
        if (L.ks.P8)
            write_bin(dir + "/TBLOCK_META_mfma_ks_entry_pos_0.bin", L.ks.pos8);
        else
            write_bin(dir + "/TBLOCK_META_mfma_ks_entry_pos_0.bin", L.ks.pos);
        write_bin(dir + "/TBLOCK_META_mfma_ks_entry_val_0.bin", L.ks.val);
        write_bin(dir + "/TBLOCK_META_mfma_ks_steps_0.bin", L.ks.steps);
    } else if (L.kind == mc_layout::BM) {
        write_bin(dir + "/TBLOCK_META_mfma_bm_records_0.bin", L.bm.rec);
        write_bin(dir + "/TBLOCK_META_mfma_bm_step_base_0.bin", L.bm.sbase);
        write_bin(dir + "/TBLOCK_META_mfma_bm_values_0.bin", L.bm.val);
    } else if (L.kind == mc_layout::ROWS) {
        write_bin(dir + "/TBLOCK_META_mfma_seg_start_0.bin", L.rows.seg_start);
        write_bin(dir + "/TBLOCK_META_mfma_entry_pos_0.bin", L.rows.pos);
        write_bin(dir + "/TBLOCK_META_mfma_entry_val_0.bin", L.rows.val);
    } else if (L.kind == mc_layout::NM) {
        write_bin(dir + "/THREAD_META_nm_panels_0.bin", L.nm_blk);
    }
    {
        std::ofstream f(dir + "/kernel_file.hip");
        f << (L.kind != mc_layout::NONE ? matrix_core_source(*meta, L, repeat) : generate_gather_source(repeat));
    }
    // copy the device headers next to the program (code_generator.cc:686-694); they ship
    // next to the library: <pkg>/csrc/hip_code/{kernel_lib,idx_formula}.hpp
    std::string hdr_dir;
    Dl_info info;
    if (dladdr((void *)&kernel_family_name, &info) && info.dli_fname) {
        std::string so = info.dli_fname;
        hdr_dir = so.substr(0, so.find_last_of('/') + 1) + "csrc/hip_code/";
    }
    if (!hdr_dir.empty())
        for (const char *h : {"kernel_lib.hpp", "idx_formula.hpp", "kernel_consts.hpp"}) {
            std::ifstream in(hdr_dir + h, std::ios::binary);
            std::ofstream out(dir + "/" + h, std::ios::binary);
            out << in.rdbuf();
        }
    {
        std::ofstream f(dir + "/make_kernel.sh");
        f << "hipcc --offload-arch=gfx950 -O3 -std=c++17 kernel_file.hip -o a.out\n";
    }
    if (dir_out) *dir_out = dir;
    return id;
}

}  // namespace gs
