// operator.cc -- operators on the hot path; validity rules restate the
// reference's name-substring checks (cited per class).
#include "operator.hpp"

#include <algorithm>

namespace gs {

std::string convert_operator_stage_type_to_string(OPERATOR_STAGE_TYPE t) {
    switch (t) {
        case CONVERTING_OP: return "CONVERTING_OP";
        case DISTRIBUTING_OP: return "DISTRIBUTING_OP";
        case IMPLEMENTING_OP: return "IMPLEMENTING_OP";
        default: return "NONE_OP";
    }
}

void operator_context::add(const std::shared_ptr<basic_operator> &op) {
    switch (op->get_stage()) {
        case CONVERTING_OP: converting.push_back(op); break;
        case DISTRIBUTING_OP: distributing[op->get_target_matrix_id()].push_back(op); break;
        case IMPLEMENTING_OP: implementing[op->get_target_matrix_id()].push_back(op); break;
        default: break;
    }
}

std::vector<std::shared_ptr<basic_operator>> operator_context::read_operator_context_arr(OPERATOR_STAGE_TYPE stage,
                                                                                         int sub) const {
    if (stage == CONVERTING_OP) return converting;
    const auto &m = stage == DISTRIBUTING_OP ? distributing : implementing;
    auto it = m.find(sub);
    return it == m.end() ? std::vector<std::shared_ptr<basic_operator>>{} : it->second;
}

static bool any_name(const std::vector<std::shared_ptr<basic_operator>> &ops, const char *sub) {
    for (auto &o : ops)
        if (o->get_name().find(sub) != std::string::npos) return true;
    return false;
}

bool has_row_direction_blocking_in_specific_level(const meta_data_set &m, POS_TYPE pos, int sub) {
    if (m.is_exist(pos, "first_row_indices_without_ending", sub)) return false;
    const auto &fr = m.u(pos, "first_row_indices", sub);
    for (size_t i = 1; i < fr.size(); i++)
        if (fr[i] == fr[i - 1]) return false;
    return true;
}

static bool interlance_storage_existing(const meta_data_set &m, int s) {
    return m.is_exist(GLOBAL_META, "nz_row_indices_after_interlance_storage", s) ||
           m.is_exist(GLOBAL_META, "nz_col_indices_after_interlance_storage", s) ||
           m.is_exist(GLOBAL_META, "nz_vals_after_interlance_storage", s);
}

static bool coo_present(const meta_data_set &m, int s) {
    return m.is_exist(GLOBAL_META, "nz_row_indices", s) && m.is_exist(GLOBAL_META, "nz_col_indices", s) &&
           m.is_exist(GLOBAL_META, "nz_vals", s) && m.is_exist(GLOBAL_META, "begin_row_index", s) &&
           m.is_exist(GLOBAL_META, "end_row_index", s);
}

// ------------------------------------------------------------ sort_operator
sort_operator::sort_operator(cg_ptr cg, ctx_ptr)
    : basic_operator("sort_operator", cg->get_metadata_set(), CONVERTING_OP, cg->get_sub_matrix_id()) {}

// sort_operator.cc:20-45
bool sort_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    if (!h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty()) return false;
    for (auto &o : h->read_operator_context_arr(CONVERTING_OP, target_matrix_id))
        if (o->get_name().find("sort_operator") != std::string::npos && o->get_target_matrix_id() == target_matrix_id)
            return false;
    return true;
}

// sort_operator.cc:47-67
bool sort_operator::is_valid_according_to_metadata() {
    return coo_present(*meta_data_set_ptr, target_matrix_id) && !has(GLOBAL_META, "original_nz_row_indices");
}

// sort_operator.cc:70-108
void sort_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "sort_operator: invalid metadata");
    get_row_order_by_length a(meta_data_set_ptr, target_matrix_id);
    run_step(a, check);
    reorder_val_by_index b(meta_data_set_ptr, target_matrix_id);
    run_step(b, check);
    reorder_col_by_index c(meta_data_set_ptr, target_matrix_id);
    run_step(c, check);
    reorder_row_by_index d(meta_data_set_ptr, target_matrix_id);
    run_step(d, check);
    remove_empty_row_in_end_of_sub_matrix e(meta_data_set_ptr, target_matrix_id);
    run_step(e, check);
    is_run = true;
}

// -------------------------------------------- empty_row_pad_operator
empty_row_pad_operator::empty_row_pad_operator(cg_ptr cg, ctx_ptr)
    : basic_operator("empty_row_pad_operator", cg->get_metadata_set(), CONVERTING_OP, cg->get_sub_matrix_id()) {}

// empty_row_pad_operator.cc:25-55: no implementing or distributing operator yet, and no
// sort_operator or empty_row_pad_operator before it on this sub-matrix
bool empty_row_pad_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    if (!h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty()) return false;
    for (auto &o : h->read_operator_context_arr(CONVERTING_OP, target_matrix_id)) {
        if (o->get_target_matrix_id() != target_matrix_id) continue;
        if (o->get_name().find("sort_operator") != std::string::npos ||
            o->get_name().find("empty_row_pad_operator") != std::string::npos)
            return false;
    }
    return true;
}

// empty_row_pad_operator.cc:57-135: the COO and its row range, no interleaved arrays, no
// blocking metadata, at least one empty row in the (grown) row range, and the padding rate
// of one entry per empty row under PADDING_RATE_UP_BOUND
// (padding_rate_valid_empty_padding, data_transform_common.cc:600-643)
bool empty_row_pad_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    if (!coo_present(m, s) || interlance_storage_existing(m, s)) return false;
    if (m.count_of_metadata_of_diff_pos(THREAD_META, s) || m.count_of_metadata_of_diff_pos(WARP_META, s) ||
        m.count_of_metadata_of_diff_pos(TBLOCK_META, s))
        return false;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    if (row.empty()) return false;
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", s);
    if (row.back() > e - b) e = b + row.back();
    const auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, e - b, 0, row.size() - 1);
    const uint64_t zeros = (uint64_t)std::count(cnt.begin(), cnt.end(), 0ull);
    if (!zeros) return false;
    return (double)(row.size() + zeros) / (double)row.size() < (double)get_config().PADDING_RATE_UP_BOUND;
}

// empty_row_pad_operator.cc:137-170: the column, value and row transforms, in that order
void empty_row_pad_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "empty_row_pad_operator: invalid metadata");
    modify_col_indices_by_empty_pad_in_submatrix a(meta_data_set_ptr, target_matrix_id);
    run_step(a, check);
    modify_vals_by_empty_pad_in_submatrix b(meta_data_set_ptr, target_matrix_id);
    run_step(b, check);
    modify_row_indices_by_empty_pad_in_submatrix c(meta_data_set_ptr, target_matrix_id);
    run_step(c, check);
    is_run = true;
}

// -------------------------------------------- row-direction TBLOCK blocking
fixed_interval_row_direction_tblock_blocking_operator::fixed_interval_row_direction_tblock_blocking_operator(
    cg_ptr cg, int rb, bool pad, ctx_ptr)
    : basic_operator("fixed_interval_row_direction_tblock_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      fixed_row_block_size(rb), is_padding(pad), code_generator_ptr(cg) {
    GS_CHECK(rb > 0, "fixed_row_block_size > 0");
}

bool fixed_interval_row_direction_tblock_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    return h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
           h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty();
}

bool fixed_interval_row_direction_tblock_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    return coo_present(m, s) && !interlance_storage_existing(m, s) && m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0 &&
           m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0;
}

// modify_{col,vals,row}_*_by_row_pad_in_sub_matrix in the row-direction operators' order
static void run_row_pad(const std::shared_ptr<meta_data_set> &m, int s, int mult, bool check,
                        std::vector<std::string> &seq) {
    modify_col_indices_by_row_pad_in_sub_matrix a(m, s, mult);
    a.run(check);
    seq.push_back(a.convert_to_string());
    modify_vals_by_row_pad_in_sub_matrix b(m, s, mult);
    b.run(check);
    seq.push_back(b.convert_to_string());
    modify_row_indices_by_row_pad_in_sub_matrix r(m, s, mult);
    r.run(check);
    seq.push_back(r.convert_to_string());
}

// fixed_interval_row_direction_tblock_blocking_operator.cc:126-185
void fixed_interval_row_direction_tblock_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "tblock blocking: invalid metadata");
    if (is_padding) run_row_pad(meta_data_set_ptr, target_matrix_id, fixed_row_block_size, check, transform_seq);  // :142-158
    get_begin_rows_of_BMTBs_after_fixed_blocking_in_row_direction a(meta_data_set_ptr, target_matrix_id,
                                                                    fixed_row_block_size);
    run_step(a, check);
    get_begin_nzs_of_BMTBs_after_fixed_blocking_in_row_direction b(meta_data_set_ptr, target_matrix_id,
                                                                   fixed_row_block_size);
    run_step(b, check);
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

// ------------------------------------------- row matrix division (§8f rank 3)
fixed_interval_row_matrix_div_operator::fixed_interval_row_matrix_div_operator(cg_ptr cg, int size, ctx_ptr)
    : basic_operator("fixed_interval_row_matrix_div_operator", cg->get_metadata_set(), CONVERTING_OP,
                     cg->get_sub_matrix_id()),
      fixed_row_interval_size(size) {
    GS_CHECK(size > 0, "fixed_row_interval_size > 0");
}

// fixed_interval_row_matrix_div_operator.cc:30-60: invalid only when the target was
// divided before AND nothing was distributed / implemented on it (the reference's flag is
// only raised inside that branch)
bool fixed_interval_row_matrix_div_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return true;
    if (!h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty()) return true;
    for (auto &o : h->read_operator_context_arr(CONVERTING_OP, target_matrix_id))
        if (o->get_name().find("div_operator") != std::string::npos && o->get_target_matrix_id() == target_matrix_id)
            return false;
    return true;
}

// :61-150: boundaries + COO present, no interleaved storage, more rows than the interval
// and at most MAX_DIV_TIMES_OF_DIV non-empty intervals
bool fixed_interval_row_matrix_div_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    for (const char *n : {"begin_row_index", "end_row_index", "begin_col_index", "end_col_index"})
        if (!m.is_exist(GLOBAL_META, n, s)) return false;
    if (!coo_present(m, s) || interlance_storage_existing(m, s)) return false;
    const uint64_t row_num = m.scalar(GLOBAL_META, "end_row_index", s) - m.scalar(GLOBAL_META, "begin_row_index", s) + 1;
    const uint64_t g = (uint64_t)fixed_row_interval_size, nbin = (row_num + g - 1) / g;
    std::vector<uint8_t> used(nbin, 0);
    int64_t non_empty = 0;
    for (uint64_t r : m.u(GLOBAL_META, "nz_row_indices", s)) {
        if (r / g >= nbin) return false;
        if (!used[r / g]) non_empty++;
        used[r / g] = 1;
    }
    return row_num > g && non_empty <= get_config().MAX_DIV_TIMES_OF_DIV;
}

// :85-150: boundaries, then cols / vals (which read the parent's rows), then rows
void fixed_interval_row_matrix_div_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "row matrix division: invalid metadata");
    auto &m = *meta_data_set_ptr;
    const int first = m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices") + 1;
    const uint64_t g = (uint64_t)fixed_row_interval_size;
    modify_row_start_boundary_after_fixed_div_in_row_direction a(meta_data_set_ptr, target_matrix_id, g);
    run_step(a, check);
    modify_row_end_boundary_after_fixed_div_in_row_direction b(meta_data_set_ptr, target_matrix_id, g);
    run_step(b, check);
    modify_col_start_boundary_after_fixed_div_in_row_direction c(meta_data_set_ptr, target_matrix_id, g);
    run_step(c, check);
    modify_col_end_boundary_after_fixed_div_in_row_direction d(meta_data_set_ptr, target_matrix_id, g);
    run_step(d, check);
    fixed_div_col_indices_by_corr_row_indices e(meta_data_set_ptr, target_matrix_id, g);
    run_step(e, check);
    fixed_div_vals_by_corr_row_indices f(meta_data_set_ptr, target_matrix_id, g);
    run_step(f, check);
    fixed_div_row_indices h(meta_data_set_ptr, target_matrix_id, g);
    run_step(h, check);
    const int last = m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices");
    for (int k = first; k <= last; k++) new_sub_matrix_ids.push_back(k);
    is_run = true;
}

// ---------------------------------------- row division by row length (§8f rank 3)
row_nz_matrix_div_operator::row_nz_matrix_div_operator(cg_ptr cg, int init, int mx, int rate, ctx_ptr)
    : basic_operator("row_nz_matrix_div_operator", cg->get_metadata_set(), CONVERTING_OP, cg->get_sub_matrix_id()),
      init_row_size_upper_boundary(init), max_row_size_upper_boundary(mx), expansion_rate(rate) {
    GS_CHECK(init > 0 && rate > 0, "init_row_size_upper_boundary > 0 and expansion_rate > 0");
}

// row_nz_matrix_div_operator.cc:29-57: the same rule as the fixed-interval division
bool row_nz_matrix_div_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return true;
    if (!h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty()) return true;
    for (auto &o : h->read_operator_context_arr(CONVERTING_OP, target_matrix_id))
        if (o->get_name().find("div_operator") != std::string::npos && o->get_target_matrix_id() == target_matrix_id)
            return false;
    return true;
}

// :59-170: boundaries + COO present, no interleaved storage, at most MAX_DIV_TIMES_OF_DIV
// division positions
bool row_nz_matrix_div_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    for (const char *n : {"begin_row_index", "end_row_index", "begin_col_index", "end_col_index"})
        if (!m.is_exist(GLOBAL_META, n, s)) return false;
    if (!coo_present(m, s) || interlance_storage_existing(m, s)) return false;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const uint64_t rn = m.scalar(GLOBAL_META, "end_row_index", s) - m.scalar(GLOBAL_META, "begin_row_index", s) + 1;
    if (row.empty() || row.back() >= rn) return false;
    bool over = false;
    row_nz_div_positions(get_nnz_of_each_row_in_spec_range(row, 0, rn - 1, 0, row.size() - 1),
                         {(uint64_t)init_row_size_upper_boundary, (uint64_t)max_row_size_upper_boundary,
                          (uint64_t)expansion_rate},
                         (size_t)get_config().MAX_DIV_TIMES_OF_DIV, &over);
    return !over;
}

// :172-250: boundaries, cols, vals, then rows
void row_nz_matrix_div_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "row-length division: invalid metadata");
    const row_nz_window w{(uint64_t)init_row_size_upper_boundary, (uint64_t)max_row_size_upper_boundary,
                          (uint64_t)expansion_rate};
    auto &m = *meta_data_set_ptr;
    parent_row_base = m.scalar(GLOBAL_META, "begin_row_index", target_matrix_id);
    parent_rows = row_num_of_sub_matrix(m, target_matrix_id);
    const int first = m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices") + 1;
    modify_row_start_boundary_after_div_according_to_row_nz a(meta_data_set_ptr, target_matrix_id, w);
    run_step(a, check);
    modify_row_end_boundary_after_div_according_to_row_nz b(meta_data_set_ptr, target_matrix_id, w);
    run_step(b, check);
    modify_col_start_boundary_after_div_according_to_row_nz c(meta_data_set_ptr, target_matrix_id, w);
    run_step(c, check);
    modify_col_end_boundary_after_div_according_to_row_nz d(meta_data_set_ptr, target_matrix_id, w);
    run_step(d, check);
    div_col_indices_by_row_nnz e(meta_data_set_ptr, target_matrix_id, w);
    run_step(e, check);
    div_val_indices_by_row_nnz f(meta_data_set_ptr, target_matrix_id, w);
    run_step(f, check);
    div_row_indices_by_row_nnz g(meta_data_set_ptr, target_matrix_id, w);
    run_step(g, check);
    const int last = m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices");
    new_sub_matrix_ids.clear();
    for (int k = first; k <= last; k++) new_sub_matrix_ids.push_back(k);
    is_run = true;
}

// --------------------------------------------- row-direction WARP blocking
fixed_interval_row_direction_warp_blocking_operator::fixed_interval_row_direction_warp_blocking_operator(
    cg_ptr cg, int rb, bool rrel, bool nrel, bool pad, ctx_ptr)
    : basic_operator("fixed_interval_row_direction_warp_blocking_operator", cg->get_metadata_set(), DISTRIBUTING_OP,
                     cg->get_sub_matrix_id()),
      fixed_row_block_size(rb), row_index_is_relative_to_BMTB(rrel), nz_index_is_relative_to_BMTB(nrel),
      is_padding(pad), code_generator_ptr(cg) {
    GS_CHECK(rb > 0, "fixed_row_block_size > 0");
}

// fixed_interval_row_direction_warp_blocking_operator.cc (is_valid_according_to_operator)
bool fixed_interval_row_direction_warp_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "thread") && !any_name(d, "warp") && !any_name(d, "col") && !any_name(d, "interlance");
}

bool fixed_interval_row_direction_warp_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 &&
              m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 && !interlance_storage_existing(m, s);
    int tb = m.count_of_metadata_of_diff_pos(TBLOCK_META, s);
    if (tb != 0) ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s) && !is_padding;
    if (row_index_is_relative_to_BMTB) ok = ok && m.is_exist(TBLOCK_META, "first_row_indices", s);
    if (nz_index_is_relative_to_BMTB) ok = ok && m.is_exist(TBLOCK_META, "first_nz_indices", s);
    return ok;
}

void fixed_interval_row_direction_warp_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "warp blocking: invalid metadata");
    if ((row_index_is_relative_to_BMTB || nz_index_is_relative_to_BMTB) && !has(TBLOCK_META, "first_row_indices"))
        throw gs_error("relative BMW indices need a BMTB level (fixed_interval_row_direction_warp_blocking_operator.cc:100-101)");
    if (has(TBLOCK_META, "first_row_indices")) {
        get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB a(meta_data_set_ptr, target_matrix_id,
                                                                              fixed_row_block_size);
        run_step(a, check);
        if (row_index_is_relative_to_BMTB) {  // :52-58
            get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id,
                                                                                           fixed_row_block_size);
            run_step(r, check);
        }
        get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB b(meta_data_set_ptr, target_matrix_id,
                                                                             fixed_row_block_size);
        run_step(b, check);
        if (nz_index_is_relative_to_BMTB) {  // :66-72
            get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id,
                                                                                          fixed_row_block_size);
            run_step(r, check);
        }
        get_begin_BMWs_of_BMTB_after_blocking_in_row_direction c(meta_data_set_ptr, target_matrix_id);
        run_step(c, check);
    } else {
        if (is_padding) run_row_pad(meta_data_set_ptr, target_matrix_id, fixed_row_block_size, check, transform_seq);  // :287-302
        get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB a(meta_data_set_ptr,
                                                                                   target_matrix_id,
                                                                                   fixed_row_block_size);
        run_step(a, check);
        get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB b(meta_data_set_ptr,
                                                                                  target_matrix_id,
                                                                                  fixed_row_block_size);
        run_step(b, check);
    }
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// ------------------------------------------- row-direction THREAD blocking
static void run_max_row_pad(const std::shared_ptr<meta_data_set> &m, int s, POS_TYPE pos, bool check,
                            std::vector<std::string> &seq, bool with_empty);
static void col_pad_and_rerun(const std::shared_ptr<meta_data_set> &m, int s, int c, bool drop_tblock, bool drop_warp,
                              const std::vector<std::shared_ptr<basic_operator>> &former, bool check,
                              std::vector<std::string> &seq, bool col_size, bool max_pad, POS_TYPE max_pos);

fixed_interval_row_direction_thread_blocking_operator::fixed_interval_row_direction_thread_blocking_operator(
    cg_ptr cg, int rb, bool rrel, bool nrel, bool row_pad, bool colpad_max, bool colpad_size, int col_size, ctx_ptr history)
    : basic_operator("fixed_interval_row_direction_thread_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      fixed_row_block_size(rb), row_index_is_relative_to_parent(rrel), nz_index_is_relative_to_parent(nrel),
      is_row_padding(row_pad), is_col_padding_with_row_max_size_with_empty_row(colpad_max),
      is_col_padding_with_col_size(colpad_size), col_size(col_size), code_generator_ptr(cg) {
    GS_CHECK(rb > 0, "fixed_row_block_size > 0");
    if (row_pad) GS_CHECK(!rrel && !nrel, "row padding needs absolute indices");
    former_operator = history->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
}

// fixed_interval_row_direction_thread_blocking_operator.cc (is_valid_according_to_operator)
bool fixed_interval_row_direction_thread_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    bool balanced_and_max_pad = any_name(d, "balanced_interval") && is_col_padding_with_row_max_size_with_empty_row;
    return !any_name(d, "thread") && !any_name(d, "col") && !any_name(d, "interlance") && !balanced_and_max_pad;
}

bool fixed_interval_row_direction_thread_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
              !interlance_storage_existing(m, s);
    bool tb = m.is_exist(TBLOCK_META, "first_row_indices", s), wb = m.is_exist(WARP_META, "first_row_indices", s);
    if (row_index_is_relative_to_parent) ok = ok && (tb || wb);
    if (nz_index_is_relative_to_parent)
        ok = ok && (m.is_exist(TBLOCK_META, "first_nz_indices", s) || m.is_exist(WARP_META, "first_nz_indices", s));
    if (is_row_padding && (tb || wb)) ok = false;
    if (tb) ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s);
    if (wb) ok = ok && has_row_direction_blocking_in_specific_level(m, WARP_META, s);
    return ok;
}

// fixed_interval_row_direction_thread_blocking_operator.cc:198-575; the
// no-parent branch (:482-565) is the one token_test exercises
void fixed_interval_row_direction_thread_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "thread blocking: invalid metadata");
    if (has(TBLOCK_META, "first_row_indices") || has(WARP_META, "first_row_indices")) {
        // :198-480: BMTs inside the BMWs when there are BMWs, else inside the BMTBs;
        // absolute starts always, the relative arrays on request
        const POS_TYPE par = has(WARP_META, "first_row_indices") ? WARP_META : TBLOCK_META;
        const bool bmtb = has(TBLOCK_META, "first_row_indices"), bmw = has(WARP_META, "first_row_indices");
        // :225-317 / :369-437: every row (empty ones too) to the BMW's (else the BMTB's) longest
        // row, then to a multiple of col_size; each drops the parent levels and re-runs the
        // former operators on the padded COO
        if (is_col_padding_with_row_max_size_with_empty_row) {
            run_max_row_pad(meta_data_set_ptr, target_matrix_id, par, check, transform_seq, true);
            col_pad_and_rerun(meta_data_set_ptr, target_matrix_id, col_size, bmtb, bmw, former_operator, check,
                              transform_seq, false, false, GLOBAL_META);
        }
        if (is_col_padding_with_col_size)
            col_pad_and_rerun(meta_data_set_ptr, target_matrix_id, col_size, bmtb, bmw, former_operator, check,
                              transform_seq, true, false, GLOBAL_META);
        get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_in_parent a(meta_data_set_ptr, target_matrix_id, par,
                                                                              fixed_row_block_size);
        run_step(a, check);
        if (row_index_is_relative_to_parent) {
            get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent b(
                meta_data_set_ptr, target_matrix_id, par, fixed_row_block_size);
            run_step(b, check);
        }
        get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_in_parent c(meta_data_set_ptr, target_matrix_id, par,
                                                                             fixed_row_block_size);
        run_step(c, check);
        if (nz_index_is_relative_to_parent) {
            get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent d(
                meta_data_set_ptr, target_matrix_id, par, fixed_row_block_size);
            run_step(d, check);
        }
        get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction e(meta_data_set_ptr, target_matrix_id, par,
                                                                          fixed_row_block_size);
        run_step(e, check);
        code_generator_ptr->open_spec_level_of_paral(THREAD_META);
        code_generator_ptr->set_thread_for_row(true);
        is_run = true;
        return;
    }
    if (is_row_padding) run_row_pad(meta_data_set_ptr, target_matrix_id, fixed_row_block_size, check, transform_seq);  // :488-504
    if (is_col_padding_with_row_max_size_with_empty_row)  // :506-521, GLOBAL parent, empty rows too
        run_max_row_pad(meta_data_set_ptr, target_matrix_id, GLOBAL_META, check, transform_seq, true);
    if (is_col_padding_with_col_size) {
        modify_col_indices_by_col_pad_in_sub_matrix a(meta_data_set_ptr, target_matrix_id, col_size);
        run_step(a, check);
        modify_vals_by_col_pad_in_sub_matrix b(meta_data_set_ptr, target_matrix_id, col_size);
        run_step(b, check);
        modify_row_indices_by_col_pad_in_sub_matrix c(meta_data_set_ptr, target_matrix_id, col_size);
        run_step(c, check);
    }
    get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction d(meta_data_set_ptr, target_matrix_id,
                                                                  fixed_row_block_size);
    run_step(d, check);
    get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction e(meta_data_set_ptr, target_matrix_id,
                                                                 fixed_row_block_size);
    run_step(e, check);
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    code_generator_ptr->set_thread_for_row(true);
    is_run = true;
}

// ------------------------------------------- nnz-direction THREAD blocking
fixed_interval_nnz_direction_thread_blocking_operator::fixed_interval_nnz_direction_thread_blocking_operator(
    cg_ptr cg, int nnz_per_BMT, bool rrel, bool nrel, bool nnz_padding, ctx_ptr)
    : basic_operator("fixed_interval_nnz_direction_thread_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      nnz_per_BMT(nnz_per_BMT), row_index_is_relative_to_parent(rrel), nz_index_is_relative_to_parent(nrel),
      nnz_padding(nnz_padding), code_generator_ptr(cg) {
    GS_CHECK(nnz_per_BMT > 0 && nnz_per_BMT <= 64, "nnz_per_BMT in [1, 64] (bitmaps are 64-bit)");
}

// fixed_interval_nnz_direction_thread_blocking_operator.cc:40-96
// fixed_interval_nnz_direction_thread_blocking_operator.cc:40-96: only nnz-direction parents,
// whose sizes are multiples of nnz_per_BMT
bool fixed_interval_nnz_direction_thread_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    bool ok = true;
    for (auto &o : h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id)) {
        const auto &n = o->get_name();
        if (h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
            n.find("fixed_interval_nnz_direction_tblock_blocking_operator") == std::string::npos &&
            n.find("fixed_interval_nnz_direction_warp_blocking_operator") == std::string::npos)
            ok = false;
        if (auto t = std::dynamic_pointer_cast<fixed_interval_nnz_direction_tblock_blocking_operator>(o))
            if (t->get_nnz_per_BMTB() % nnz_per_BMT) ok = false;
        if (auto w = std::dynamic_pointer_cast<fixed_interval_nnz_direction_warp_blocking_operator>(o))
            if (w->get_nnz_per_BMW() % nnz_per_BMT) ok = false;
    }
    return ok;
}

// fixed_interval_nnz_direction_thread_blocking_operator.cc:98-150: relative indices need a
// parent; padding only without parents
bool fixed_interval_nnz_direction_thread_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    if (!coo_present(m, s) || m.count_of_metadata_of_diff_pos(THREAD_META, s) != 0 || interlance_storage_existing(m, s))
        return false;
    const bool bmtb = has(TBLOCK_META, "first_row_indices"), bmw = has(WARP_META, "first_row_indices");
    if ((row_index_is_relative_to_parent || nz_index_is_relative_to_parent) && !(bmtb || has(WARP_META, "first_nz_indices")))
        return false;
    if (nnz_padding && (bmtb || bmw)) return false;
    return true;
}

// fixed_interval_nnz_direction_thread_blocking_operator.cc:156-245
void fixed_interval_nnz_direction_thread_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "nnz blocking: invalid metadata");
    const bool bmtb = has(TBLOCK_META, "first_row_indices"), bmw = has(WARP_META, "first_row_indices");
    if (bmtb || bmw) {
        // BMTs inside the nearest parent: absolute starts, the relative ones, the parent's
        // first BMT of each block; the size step keeps the reference's GLOBAL parent
        const POS_TYPE par = bmw ? WARP_META : TBLOCK_META;
        get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction d(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
        run_step(d, check);
        if (row_index_is_relative_to_parent) {
            if (bmw) {
                get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW r(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
                run_step(r, check);
            } else {
                get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
                run_step(r, check);
            }
        }
        get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction e(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
        run_step(e, check);
        if (nz_index_is_relative_to_parent) {
            if (bmw) {
                get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW r(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
                run_step(r, check);
            } else {
                get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
                run_step(r, check);
            }
        }
        get_begin_BMTs_of_specific_parent_after_blocking g(meta_data_set_ptr, target_matrix_id, par);
        run_step(g, check);
        get_BMT_size_of_each_parent f(meta_data_set_ptr, GLOBAL_META, target_matrix_id, false);
        run_step(f, check);
        code_generator_ptr->open_spec_level_of_paral(THREAD_META);
        is_run = true;
        return;
    }
    if (nnz_padding) {
        modify_col_indices_by_nnz_pad a(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
        run_step(a, check);
        modify_vals_by_nnz_pad b(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
        run_step(b, check);
        modify_row_indices_by_nnz_pad c(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
        run_step(c, check);
    }
    get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction d(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
    run_step(d, check);
    get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction e(meta_data_set_ptr, target_matrix_id, nnz_per_BMT);
    run_step(e, check);
    get_BMT_size_of_each_parent f(meta_data_set_ptr, GLOBAL_META, target_matrix_id, false);
    run_step(f, check);
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    is_run = true;
}

// ------------------------------------------ nnz-direction TBLOCK / WARP blocking
fixed_interval_nnz_direction_tblock_blocking_operator::fixed_interval_nnz_direction_tblock_blocking_operator(
    cg_ptr cg, int nnz_per_BMTB, bool nnz_padding, ctx_ptr)
    : basic_operator("fixed_interval_nnz_direction_tblock_blocking_operator", cg->get_metadata_set(), DISTRIBUTING_OP,
                     cg->get_sub_matrix_id()),
      nnz_per_BMTB(nnz_per_BMTB), nnz_padding(nnz_padding), code_generator_ptr(cg) {
    GS_CHECK(nnz_per_BMTB > 0, "nnz_per_BMTB > 0");
}

// fixed_interval_nnz_direction_tblock_blocking_operator.cc:35-48: the first distributing operator
bool fixed_interval_nnz_direction_tblock_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    return h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
           h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty();
}

// :50-85: the COO, no blocking metadata at any level, no interleaved arrays
bool fixed_interval_nnz_direction_tblock_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    return coo_present(m, s) && !interlance_storage_existing(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
           m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 && m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0;
}

// :87-135
void fixed_interval_nnz_direction_tblock_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "nnz-direction tblock blocking: invalid metadata");
    if (nnz_padding) {
        modify_col_indices_by_nnz_pad a(meta_data_set_ptr, target_matrix_id, nnz_per_BMTB);
        run_step(a, check);
        modify_vals_by_nnz_pad b(meta_data_set_ptr, target_matrix_id, nnz_per_BMTB);
        run_step(b, check);
        modify_row_indices_by_nnz_pad c(meta_data_set_ptr, target_matrix_id, nnz_per_BMTB);
        run_step(c, check);
    }
    get_begin_rows_of_BMTB_after_fixed_blocking_in_nnz_direction d(meta_data_set_ptr, target_matrix_id, nnz_per_BMTB);
    run_step(d, check);
    get_begin_nzs_of_BMTB_after_fixed_blocking_in_nnz_direction e(meta_data_set_ptr, target_matrix_id, nnz_per_BMTB);
    run_step(e, check);
    if (nnz_padding) {
        get_BMTB_size f(meta_data_set_ptr, target_matrix_id);
        run_step(f, check);
    }
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

fixed_interval_nnz_direction_warp_blocking_operator::fixed_interval_nnz_direction_warp_blocking_operator(
    cg_ptr cg, int nnz_per_BMW, bool rrel, bool nrel, bool nnz_padding, ctx_ptr)
    : basic_operator("fixed_interval_nnz_direction_warp_blocking_operator", cg->get_metadata_set(), DISTRIBUTING_OP,
                     cg->get_sub_matrix_id()),
      nnz_per_BMW(nnz_per_BMW), row_index_is_relative_to_parent(rrel), nz_index_is_relative_to_parent(nrel),
      nnz_padding(nnz_padding), code_generator_ptr(cg) {
    GS_CHECK(nnz_per_BMW > 0, "nnz_per_BMW > 0");
}

// fixed_interval_nnz_direction_warp_blocking_operator.cc:40-85: only an nnz-direction BMTB
// before it, whose size is a multiple of nnz_per_BMW
bool fixed_interval_nnz_direction_warp_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    bool ok = true;
    for (auto &o : h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id)) {
        if (h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
            o->get_name().find("fixed_interval_nnz_direction_tblock_blocking_operator") == std::string::npos)
            ok = false;
        if (auto t = std::dynamic_pointer_cast<fixed_interval_nnz_direction_tblock_blocking_operator>(o))
            if (t->get_nnz_per_BMTB() % nnz_per_BMW) ok = false;
    }
    return ok;
}

// :87-130: no THREAD / WARP metadata yet; relative indices need the BMTB level; padding
// only without it; no interleaved arrays
bool fixed_interval_nnz_direction_warp_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    if (!coo_present(m, s) || interlance_storage_existing(m, s) || m.count_of_metadata_of_diff_pos(THREAD_META, s) != 0 ||
        m.count_of_metadata_of_diff_pos(WARP_META, s) != 0)
        return false;
    const bool bmtb = has(TBLOCK_META, "first_row_indices");
    if ((row_index_is_relative_to_parent || nz_index_is_relative_to_parent) && !bmtb) return false;
    if (nnz_padding && bmtb) return false;
    return true;
}

// :132-200
void fixed_interval_nnz_direction_warp_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "nnz-direction warp blocking: invalid metadata");
    const bool bmtb = has(TBLOCK_META, "first_row_indices");
    if (nnz_padding) {
        modify_col_indices_by_nnz_pad a(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
        run_step(a, check);
        modify_vals_by_nnz_pad b(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
        run_step(b, check);
        modify_row_indices_by_nnz_pad c(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
        run_step(c, check);
    }
    get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction d(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
    run_step(d, check);
    get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction e(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
    run_step(e, check);
    if (row_index_is_relative_to_parent) {
        get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
        run_step(r, check);
    }
    if (nz_index_is_relative_to_parent) {
        get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, nnz_per_BMW);
        run_step(r, check);
    }
    if (bmtb) {
        get_begin_BMWs_of_BMTB_after_blocking g(meta_data_set_ptr, target_matrix_id);
        run_step(g, check);
    }
    get_BMW_size_of_each_parent f(meta_data_set_ptr, target_matrix_id, GLOBAL_META);
    run_step(f, check);
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// --------------------------------------- balanced row-direction WARP blocking
balanced_interval_row_direction_warp_blocking_operator::balanced_interval_row_direction_warp_blocking_operator(
    cg_ptr cg, int per, bool rrel, bool nrel, ctx_ptr)
    : basic_operator("balanced_interval_row_direction_warp_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      nnz_per_interval(per), row_index_is_relative_to_BMTB(rrel), nz_index_is_relative_to_BMTB(nrel),
      code_generator_ptr(cg) {
    GS_CHECK(per > 0, "nnz_per_interval > 0");
}

bool balanced_interval_row_direction_warp_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "thread") && !any_name(d, "warp") && !any_name(d, "nnz_direction") && !any_name(d, "col") &&
           !any_name(d, "interlance");
}

bool balanced_interval_row_direction_warp_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
              m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 && !interlance_storage_existing(m, s);
    if (m.is_exist(TBLOCK_META, "first_row_indices", s))
        ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s);
    return ok;
}

// balanced_interval_row_direction_warp_blocking_operator.cc:177-227 (no-parent branch)
void balanced_interval_row_direction_warp_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "balanced warp blocking: invalid metadata");
    if (has(TBLOCK_META, "first_row_indices")) {  // :165-207
        const uint64_t per = (uint64_t)nnz_per_interval;
        get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB a(meta_data_set_ptr, target_matrix_id, per);
        run_step(a, check);
        if (row_index_is_relative_to_BMTB) {
            get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, per);
            run_step(r, check);
        }
        get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB b(meta_data_set_ptr, target_matrix_id, per);
        run_step(b, check);
        if (nz_index_is_relative_to_BMTB) {
            get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, per);
            run_step(r, check);
        }
        get_begin_BMWs_of_BMTB_after_blocking_in_row_direction c(meta_data_set_ptr, target_matrix_id);
        run_step(c, check);
        code_generator_ptr->open_spec_level_of_paral(WARP_META);
        is_run = true;
        return;
    }
    get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction a(meta_data_set_ptr, target_matrix_id,
                                                               (uint64_t)nnz_per_interval);
    run_step(a, check);
    get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction b(meta_data_set_ptr, target_matrix_id,
                                                              (uint64_t)nnz_per_interval);
    run_step(b, check);
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// -------------------------------------- balanced row-direction TBLOCK blocking
balanced_interval_row_direction_tblock_blocking_operator::balanced_interval_row_direction_tblock_blocking_operator(
    cg_ptr cg, int per, ctx_ptr)
    : basic_operator("balanced_interval_row_direction_tblock_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      nnz_per_interval(per), code_generator_ptr(cg) {
    GS_CHECK(per > 0, "nnz_per_interval > 0");
}

// balanced_interval_row_direction_tblock_blocking_operator.cc:29-45: nothing distributed or implemented yet
bool balanced_interval_row_direction_tblock_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    return h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
           h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty();
}

// :47-87: COO + row bounds, no THREAD / WARP / TBLOCK metadata, no interleaved storage
bool balanced_interval_row_direction_tblock_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    return coo_present(m, s) && !interlance_storage_existing(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
           m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 && m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0;
}

// :89-120
void balanced_interval_row_direction_tblock_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "balanced tblock blocking: invalid metadata");
    get_begin_rows_of_BMTB_after_nnz_blocking_in_row_direction a(meta_data_set_ptr, target_matrix_id,
                                                                (uint64_t)nnz_per_interval);
    run_step(a, check);
    get_begin_nzs_of_BMTB_after_nnz_blocking_in_row_direction b(meta_data_set_ptr, target_matrix_id,
                                                               (uint64_t)nnz_per_interval);
    run_step(b, check);
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

// -------------------------------------- balanced row-direction THREAD blocking
balanced_interval_row_direction_thread_blocking_operator::balanced_interval_row_direction_thread_blocking_operator(
    cg_ptr cg, int per, bool rrel, bool nrel, ctx_ptr)
    : basic_operator("balanced_interval_row_direction_thread_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      nnz_per_interval(per), row_index_is_relative_to_parent(rrel), nz_index_is_relative_to_parent(nrel),
      code_generator_ptr(cg) {
    GS_CHECK(per > 0, "nnz_per_interval > 0");
}

// balanced_interval_row_direction_thread_blocking_operator.cc:35-75: no implementing
// operator, no distributing one named thread / col / interlance / nnz_direction
bool balanced_interval_row_direction_thread_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "thread") && !any_name(d, "col") && !any_name(d, "interlance") && !any_name(d, "nnz_direction");
}

bool balanced_interval_row_direction_thread_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 && !interlance_storage_existing(m, s);
    if (m.is_exist(TBLOCK_META, "first_row_indices", s)) ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s);
    if (m.is_exist(WARP_META, "first_row_indices", s)) ok = ok && has_row_direction_blocking_in_specific_level(m, WARP_META, s);
    return ok;
}

// the no-parent branch of run() (BMT rows / nzs over the whole sub-matrix)
void balanced_interval_row_direction_thread_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "balanced thread blocking: invalid metadata");
    if (has(TBLOCK_META, "first_row_indices") || has(WARP_META, "first_row_indices")) {
        // :162-249: inside the BMWs when there are BMWs, else inside the BMTBs
        const POS_TYPE par = has(WARP_META, "first_row_indices") ? WARP_META : TBLOCK_META;
        const uint64_t per = (uint64_t)nnz_per_interval;
        get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_in_parent a(meta_data_set_ptr, target_matrix_id, par, per);
        run_step(a, check);
        if (row_index_is_relative_to_parent) {
            get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent r(meta_data_set_ptr, target_matrix_id, par, per);
            run_step(r, check);
        }
        get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_in_parent b(meta_data_set_ptr, target_matrix_id, par, per);
        run_step(b, check);
        if (nz_index_is_relative_to_parent) {
            get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent r(meta_data_set_ptr, target_matrix_id, par, per);
            run_step(r, check);
        }
        get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction e(meta_data_set_ptr, target_matrix_id, par, 1);
        run_step(e, check);
        code_generator_ptr->open_spec_level_of_paral(THREAD_META);
        is_run = true;
        return;
    }
    if (row_index_is_relative_to_parent || nz_index_is_relative_to_parent)
        throw gs_error("relative BMT indices need a parent level");
    get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction a(meta_data_set_ptr, target_matrix_id,
                                                               (uint64_t)nnz_per_interval);
    run_step(a, check);
    get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction b(meta_data_set_ptr, target_matrix_id,
                                                              (uint64_t)nnz_per_interval);
    run_step(b, check);
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    is_run = true;
}

// ------------------------------------------------------------- merge path
merge_path_operator_base::merge_path_operator_base(const char *name, POS_TYPE level, cg_ptr cg, int ws)
    : basic_operator(name, cg->get_metadata_set(), DISTRIBUTING_OP, cg->get_sub_matrix_id()), work_size(ws),
      level(level), code_generator_ptr(cg) {
    GS_CHECK(ws > 0, "work_size > 0");
}

// merge_path_{tblock,warp}_operator.cc is_valid_according_to_metadata: COO + row bounds,
// no interleaved storage, no metadata at the levels the operator may not follow
bool merge_path_operator_base::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && !interlance_storage_existing(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0;
    if (level != THREAD_META) ok = ok && m.count_of_metadata_of_diff_pos(WARP_META, s) == 0;
    if (level == TBLOCK_META) ok = ok && m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0;
    return ok;
}

// merge_path_warp_operator.cc:106-133 (same body at TBLOCK / THREAD)
void merge_path_operator_base::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), name + ": invalid metadata");
    get_begin_rows_of_level_after_merge_path a(meta_data_set_ptr, target_matrix_id, level, work_size);
    run_step(a, check);
    get_begin_nzs_of_level_after_merge_path b(meta_data_set_ptr, target_matrix_id, level, work_size);
    run_step(b, check);
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    code_generator_ptr->set_merge_path_level(level, work_size);
    is_run = true;
}

merge_path_tblock_operator::merge_path_tblock_operator(cg_ptr cg, int ws, ctx_ptr)
    : merge_path_operator_base("merge_path_tblock_operator", TBLOCK_META, cg, ws) {}
merge_path_warp_operator::merge_path_warp_operator(cg_ptr cg, int ws, ctx_ptr)
    : merge_path_operator_base("merge_path_warp_operator", WARP_META, cg, ws) {}
merge_path_thread_operator::merge_path_thread_operator(cg_ptr cg, int ws, ctx_ptr)
    : merge_path_operator_base("merge_path_thread_operator", THREAD_META, cg, ws) {}

// merge_path_tblock_operator.cc: nothing distributed or implemented yet
bool merge_path_tblock_operator::is_valid_according_to_operator(ctx_ptr h) {
    return h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
           h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty();
}

// merge_path_warp_operator.cc:26-63: no distributing op named thread / warp / col / interlance
bool merge_path_warp_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "thread") && !any_name(d, "warp") && !any_name(d, "col") && !any_name(d, "interlance");
}

// merge_path_thread_operator.cc: no distributing op named thread / col / interlance
bool merge_path_thread_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "thread") && !any_name(d, "col") && !any_name(d, "interlance");
}

// ------------------------------------------------ interleaved storage (§8f rank 2)
// interlance_storage_operator.cc:12-45: the parent level is the WARP / TBLOCK level a
// distributing operator opened before, else GLOBAL
interlance_storage_operator::interlance_storage_operator(cg_ptr cg, ctx_ptr history)
    : basic_operator("interlance_storage_operator", cg->get_metadata_set(), DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      code_generator_ptr(cg) {
    bool warp = false, tblock = false;
    for (auto &o : history->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id)) {
        if (o->get_name().find("warp") != std::string::npos) warp = true;
        else if (o->get_name().find("tblock") != std::string::npos) tblock = true;
    }
    pos = warp ? WARP_META : (tblock ? TBLOCK_META : GLOBAL_META);
}

// :56-97: no implementing op; a col-direction thread blocking WITH padding to a multiple
// of its size (or row-direction thread blocking padded to the row max) came before; once
bool interlance_storage_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    bool col_pad = false, row_pad = false;
    for (auto &o : h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id)) {
        if (o->get_name().find("interlance") != std::string::npos) return false;
        if (auto *c = dynamic_cast<fixed_interval_col_direction_thread_blocking_operator *>(o.get()))
            col_pad = col_pad || c->is_padding_with_col_size_in_bmt;
        if (auto *r = dynamic_cast<fixed_interval_row_direction_thread_blocking_operator *>(o.get()))
            row_pad = row_pad || r->is_col_padding_with_row_max_size_with_empty_row;
    }
    return col_pad || row_pad;
}

// :99-141
bool interlance_storage_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = !interlance_storage_existing(m, s) && m.is_exist(GLOBAL_META, "nz_row_indices", s) &&
              m.is_exist(GLOBAL_META, "nz_col_indices", s) && m.is_exist(GLOBAL_META, "nz_vals", s);
    if (pos != GLOBAL_META) ok = ok && m.is_exist(pos, "first_BMT_indices", s);
    return ok && m.is_exist(pos, "BMT_size_of_each_blk", s);
}

// :144-176
void interlance_storage_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "interlance_storage: invalid metadata (equal-size BMTs per parent needed)");
    modify_col_indices_by_interlance_storage a(meta_data_set_ptr, pos, target_matrix_id);
    run_step(a, check);
    modify_vals_by_interlance_storage b(meta_data_set_ptr, pos, target_matrix_id);
    run_step(b, check);
    modify_row_indices_by_interlance_storage c(meta_data_set_ptr, pos, target_matrix_id);
    run_step(c, check);
    code_generator_ptr->set_interleave_storage(pos);
    is_run = true;
}

// ------------------------------------------- col-direction THREAD blocking (A10)
fixed_interval_col_direction_thread_blocking_operator::fixed_interval_col_direction_thread_blocking_operator(
    cg_ptr cg, int fcs, bool rrel, bool nrel, bool pad_size, bool pad_max, ctx_ptr history)
    : basic_operator("fixed_interval_col_direction_thread_blocking_operator", cg->get_metadata_set(),
                     DISTRIBUTING_OP, cg->get_sub_matrix_id()),
      fixed_col_block_size(fcs), row_index_is_relative_to_BMTB(false), nz_index_is_relative_to_BMTB(false),
      is_padding_with_col_size_in_bmt(pad_size), is_col_padding_with_row_max_size_without_empty_row(pad_max),
      code_generator_ptr(cg) {
    GS_CHECK(fcs > 0, "fixed_col_block_size > 0");
    // ...col_direction_thread_blocking_operator.cc:25-85: the padding level and the
    // relative-index parent follow the distributing operators already run (a "warp" one
    // wins over a "tblock" one); with no parent the relative flags are unused
    former_operator = history->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    bool warp = false, tblock = false;
    for (auto &o : former_operator) {
        if (o->get_name().find("warp") != std::string::npos) warp = true;
        else if (o->get_name().find("tblock") != std::string::npos) tblock = true;
    }
    if (warp) {
        padding_pos = WARP_META;
        row_index_is_relative_to_BMW = rrel;
        nz_index_is_relative_to_BMW = nrel;
    } else if (tblock) {
        padding_pos = TBLOCK_META;
        row_index_is_relative_to_BMTB = rrel;
        nz_index_is_relative_to_BMTB = nrel;
    }
}

// ...col_direction_thread_blocking_operator.cc:97-138
bool fixed_interval_col_direction_thread_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    bool balanced_and_max_pad = any_name(d, "balanced_interval") && is_col_padding_with_row_max_size_without_empty_row;
    return !any_name(d, "thread") && !any_name(d, "col") && !any_name(d, "interlance") && !balanced_and_max_pad;
}

// data_transform_common.cc:644-690 (padding_rate_valid_col_direction_with_multiple)
static bool padding_rate_valid_col_direction_with_multiple(const meta_data_set &m, int fcs, int s) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    const uint64_t orig = row.size();
    uint64_t after = orig;
    for (uint64_t c : cnt)
        if (c % (uint64_t)fcs) {
            after += (c / fcs + 1) * fcs - c;
            if ((double)after / (double)orig >= (double)get_config().PADDING_RATE_UP_BOUND) return false;
        }
    return true;
}

// ...col_direction_thread_blocking_operator.cc:140-258
bool fixed_interval_col_direction_thread_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0;
    bool tb = m.is_exist(TBLOCK_META, "first_row_indices", s), wb = m.is_exist(WARP_META, "first_row_indices", s);
    if (row_index_is_relative_to_BMTB) ok = ok && tb;
    if (nz_index_is_relative_to_BMTB) ok = ok && m.is_exist(TBLOCK_META, "first_nz_indices", s);
    if (row_index_is_relative_to_BMW) ok = ok && wb;
    if (nz_index_is_relative_to_BMW) ok = ok && m.is_exist(WARP_META, "first_nz_indices", s);
    if (is_col_padding_with_row_max_size_without_empty_row) {
        if (padding_pos == TBLOCK_META) ok = ok && tb;
        else if (padding_pos == WARP_META) ok = ok && wb;
    }
    if (tb) ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s);
    if (wb) ok = ok && has_row_direction_blocking_in_specific_level(m, WARP_META, s);
    if (ok && is_padding_with_col_size_in_bmt)
        ok = padding_rate_valid_col_direction_with_multiple(m, fixed_col_block_size, s);
    return ok && !interlance_storage_existing(m, s);
}

// ...col_direction_thread_blocking_operator.cc:297-368 (shared by the WARP / THREAD col-direction
// operators): pad every row to a multiple of c, drop the parent levels and run the former
// operators again on the padded COO with their own padding off
// (max_pad: first every non-empty row to its max_pos parent's longest row, :297-310;
// col_size: then to a multiple of c, :313-326; either one drops and rebuilds the parents)
static void run_max_row_pad(const std::shared_ptr<meta_data_set> &m, int s, POS_TYPE pos, bool check,
                            std::vector<std::string> &seq, bool with_empty) {
    modify_col_indices_by_col_pad_parent_blk_to_max_row_size a(m, s, pos, with_empty);
    a.run(check);
    seq.push_back(a.convert_to_string());
    modify_vals_by_col_pad_parent_blk_to_max_row_size b(m, s, pos, with_empty);
    b.run(check);
    seq.push_back(b.convert_to_string());
    modify_row_indices_by_col_pad_parent_blk_to_max_row_size r(m, s, pos, with_empty);
    r.run(check);
    seq.push_back(r.convert_to_string());
}

static void col_pad_and_rerun(const std::shared_ptr<meta_data_set> &m, int s, int c, bool drop_tblock, bool drop_warp,
                              const std::vector<std::shared_ptr<basic_operator>> &former, bool check,
                              std::vector<std::string> &seq, bool col_size, bool max_pad, POS_TYPE max_pos) {
    if (max_pad) run_max_row_pad(m, s, max_pos, check, seq, false);
    if (col_size) {
        modify_col_indices_by_col_pad_in_sub_matrix a(m, s, c);
        a.run(check);
        seq.push_back(a.convert_to_string());
        modify_vals_by_col_pad_in_sub_matrix b(m, s, c);
        b.run(check);
        seq.push_back(b.convert_to_string());
        modify_row_indices_by_col_pad_in_sub_matrix r(m, s, c);
        r.run(check);
        seq.push_back(r.convert_to_string());
    }
    for (POS_TYPE pos : {TBLOCK_META, WARP_META}) {
        if ((pos == TBLOCK_META && !drop_tblock) || (pos == WARP_META && !drop_warp)) continue;
        for (const auto &n : m->all_item_of_metadata_of_diff_pos(pos, s)) {
            remove_item_of_metadata d(m, s, n, pos);
            d.run(check);
            seq.push_back(d.convert_to_string());
        }
    }
    for (auto &o : former) {
        const size_t before = o->get_data_transform_sequence().size();
        o->set_padding_to_false();
        o->run(check);
        const auto after = o->get_data_transform_sequence();
        for (size_t k = before; k < after.size(); k++) seq.push_back(after[k]);
    }
}

// ...col_direction_thread_blocking_operator.cc:260-487
void fixed_interval_col_direction_thread_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "col-direction thread blocking: invalid metadata");
    const bool bmtb = has(TBLOCK_META, "first_row_indices"), bmw = has(WARP_META, "first_row_indices");
    const int c = fixed_col_block_size;
    if (is_padding_with_col_size_in_bmt || is_col_padding_with_row_max_size_without_empty_row) {  // :297-368
        col_pad_and_rerun(meta_data_set_ptr, target_matrix_id, c, bmtb, bmw, former_operator, check, transform_seq,
                          is_padding_with_col_size_in_bmt, is_col_padding_with_row_max_size_without_empty_row, padding_pos);
    }
    get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction e(meta_data_set_ptr, target_matrix_id, c);
    run_step(e, check);
    get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction f(meta_data_set_ptr, target_matrix_id, c);
    run_step(f, check);
    if (row_index_is_relative_to_BMTB) {  // :381-395
        get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, c);
        run_step(r, check);
    }
    if (nz_index_is_relative_to_BMTB) {  // :397-412
        get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents r(meta_data_set_ptr, target_matrix_id, c, TBLOCK_META);
        run_step(r, check);
    }
    if (bmtb) {  // :414-420
        get_begin_BMTs_of_specific_parent_after_blocking g(meta_data_set_ptr, target_matrix_id, TBLOCK_META);
        run_step(g, check);
    }
    if (is_padding_with_col_size_in_bmt && bmtb) {  // :422-428
        get_BMT_size_of_each_parent g(meta_data_set_ptr, TBLOCK_META, target_matrix_id, false);
        run_step(g, check);
    }
    if (row_index_is_relative_to_BMW) {  // :430-444
        get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMW r(meta_data_set_ptr, target_matrix_id, c);
        run_step(r, check);
    }
    if (nz_index_is_relative_to_BMW) {  // :446-460
        get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents r(meta_data_set_ptr, target_matrix_id, c, WARP_META);
        run_step(r, check);
    }
    if (bmw) {  // :462-468
        get_begin_BMTs_of_specific_parent_after_blocking g(meta_data_set_ptr, target_matrix_id, WARP_META);
        run_step(g, check);
    }
    if (is_padding_with_col_size_in_bmt && bmw) {  // :470-476
        get_BMT_size_of_each_parent g(meta_data_set_ptr, WARP_META, target_matrix_id, false);
        run_step(g, check);
    }
    if (is_padding_with_col_size_in_bmt) {  // :478-483
        get_BMT_size_of_each_parent g(meta_data_set_ptr, GLOBAL_META, target_matrix_id, false);
        run_step(g, check);
    }
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    is_run = true;
}

// ------------------------------------------- col-direction TBLOCK blocking
fixed_interval_col_direction_tblock_blocking_operator::fixed_interval_col_direction_tblock_blocking_operator(
    cg_ptr cg, int fcs, bool pad_size, bool pad_max, ctx_ptr)
    : basic_operator("fixed_interval_col_direction_tblock_blocking_operator", cg->get_metadata_set(), DISTRIBUTING_OP,
                     cg->get_sub_matrix_id()),
      fixed_col_block_size(fcs), is_padding_with_col_size_in_bmtb(pad_size),
      is_col_padding_with_row_max_size_without_empty_row(pad_max), code_generator_ptr(cg) {
    GS_CHECK(fcs > 0, "fixed_col_block_size > 0");
}

// fixed_interval_col_direction_tblock_blocking_operator.cc:37-77: the first distributing operator
bool fixed_interval_col_direction_tblock_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    return h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty() &&
           h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id).empty();
}

// :80-128: the COO, no blocking at any level, the padding rates, no interleaved arrays
bool fixed_interval_col_direction_tblock_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
              m.count_of_metadata_of_diff_pos(WARP_META, s) == 0 && m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0;
    if (ok && is_padding_with_col_size_in_bmtb) ok = padding_rate_valid_col_direction_with_multiple(m, fixed_col_block_size, s);
    return ok && !interlance_storage_existing(m, s);
}

// :130-201
void fixed_interval_col_direction_tblock_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "col-direction tblock blocking: invalid metadata");
    const int c = fixed_col_block_size;
    if (is_col_padding_with_row_max_size_without_empty_row)  // :149-162, GLOBAL parent
        run_max_row_pad(meta_data_set_ptr, target_matrix_id, GLOBAL_META, check, transform_seq, false);
    if (is_padding_with_col_size_in_bmtb) {
        modify_col_indices_by_col_pad_in_sub_matrix a(meta_data_set_ptr, target_matrix_id, c);
        run_step(a, check);
        modify_vals_by_col_pad_in_sub_matrix b(meta_data_set_ptr, target_matrix_id, c);
        run_step(b, check);
        modify_row_indices_by_col_pad_in_sub_matrix r(meta_data_set_ptr, target_matrix_id, c);
        run_step(r, check);
    }
    get_begin_rows_of_BMTB_after_fixed_blocking_in_col_direction d(meta_data_set_ptr, target_matrix_id, c);
    run_step(d, check);
    get_begin_nzs_of_BMTB_after_fixed_blocking_in_col_direction e(meta_data_set_ptr, target_matrix_id, c);
    run_step(e, check);
    if (is_padding_with_col_size_in_bmtb) {
        get_BMTB_size f(meta_data_set_ptr, target_matrix_id);
        run_step(f, check);
    }
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

// ------------------------------------------- col-direction WARP blocking
fixed_interval_col_direction_warp_blocking_operator::fixed_interval_col_direction_warp_blocking_operator(
    cg_ptr cg, int fcs, bool rrel, bool nrel, bool pad_size, bool pad_max, ctx_ptr history)
    : basic_operator("fixed_interval_col_direction_warp_blocking_operator", cg->get_metadata_set(), DISTRIBUTING_OP,
                     cg->get_sub_matrix_id()),
      fixed_col_block_size(fcs), row_index_is_relative_to_BMTB(rrel), nz_index_is_relative_to_BMTB(nrel),
      is_padding_with_col_size_in_bmw(pad_size), is_col_padding_with_row_max_size_without_empty_row(pad_max),
      code_generator_ptr(cg) {
    GS_CHECK(fcs > 0, "fixed_col_block_size > 0");
    // fixed_interval_col_direction_warp_blocking_operator.cc:20-50
    former_operator = history->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    padding_pos = any_name(former_operator, "tblock") ? TBLOCK_META : GLOBAL_META;
}

// :60-100
bool fixed_interval_col_direction_warp_blocking_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    bool balanced_and_max_pad = any_name(d, "balanced_interval") && is_col_padding_with_row_max_size_without_empty_row;
    return !any_name(d, "thread") && !any_name(d, "warp") && !any_name(d, "col") && !any_name(d, "interlance") &&
           !balanced_and_max_pad;
}

// :102-190
bool fixed_interval_col_direction_warp_blocking_operator::is_valid_according_to_metadata() {
    auto &m = *meta_data_set_ptr;
    const int s = target_matrix_id;
    bool ok = coo_present(m, s) && m.count_of_metadata_of_diff_pos(THREAD_META, s) == 0 &&
              m.count_of_metadata_of_diff_pos(WARP_META, s) == 0;
    const bool tb = m.is_exist(TBLOCK_META, "first_row_indices", s);
    if (row_index_is_relative_to_BMTB) ok = ok && tb;
    if (nz_index_is_relative_to_BMTB) ok = ok && m.is_exist(TBLOCK_META, "first_nz_indices", s);
    if (is_col_padding_with_row_max_size_without_empty_row && padding_pos == TBLOCK_META) ok = ok && tb;
    if (tb) ok = ok && has_row_direction_blocking_in_specific_level(m, TBLOCK_META, s);
    if (ok && is_padding_with_col_size_in_bmw) ok = padding_rate_valid_col_direction_with_multiple(m, fixed_col_block_size, s);
    const bool balanced_and_max_pad = any_name(former_operator, "balanced_interval") && is_col_padding_with_row_max_size_without_empty_row;
    return ok && !interlance_storage_existing(m, s) && !balanced_and_max_pad;
}

// :192-372
void fixed_interval_col_direction_warp_blocking_operator::run(bool check) {
    if (check) GS_CHECK(is_valid_according_to_metadata(), "col-direction warp blocking: invalid metadata");
    const bool bmtb = has(TBLOCK_META, "first_row_indices");
    const int c = fixed_col_block_size;
    if (is_padding_with_col_size_in_bmw || is_col_padding_with_row_max_size_without_empty_row)  // :242-290
        col_pad_and_rerun(meta_data_set_ptr, target_matrix_id, c, bmtb, false, former_operator, check, transform_seq,
                          is_padding_with_col_size_in_bmw, is_col_padding_with_row_max_size_without_empty_row, padding_pos);
    get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction d(meta_data_set_ptr, target_matrix_id, c);
    run_step(d, check);
    get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction e(meta_data_set_ptr, target_matrix_id, c);
    run_step(e, check);
    if (row_index_is_relative_to_BMTB) {
        get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, c);
        run_step(r, check);
    }
    if (nz_index_is_relative_to_BMTB) {
        get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB r(meta_data_set_ptr, target_matrix_id, c);
        run_step(r, check);
    }
    if (bmtb) {
        get_begin_BMWs_of_BMTB_after_blocking g(meta_data_set_ptr, target_matrix_id);
        run_step(g, check);
    }
    if (is_padding_with_col_size_in_bmw && bmtb) {
        get_BMW_size_of_each_parent f(meta_data_set_ptr, target_matrix_id, TBLOCK_META);
        run_step(f, check);
    }
    if (is_padding_with_col_size_in_bmw) {
        get_BMW_size_of_each_parent f(meta_data_set_ptr, target_matrix_id, GLOBAL_META);
        run_step(f, check);
    }
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// ------------------------------------------------------------- implementing
thread_total_reduce_operator::thread_total_reduce_operator(cg_ptr cg, bool nwr, int scf, int cf, ctx_ptr)
    : basic_operator("thread_total_reduce_operator", cg->get_metadata_set(), IMPLEMENTING_OP,
                     cg->get_sub_matrix_id()),
      need_warp_reduction(nwr), sparse_coarsen_factor(scf), coarsen_factor(cf), code_generator_ptr(cg) {}

// thread_total_reduce_operator.cc:14-40
bool thread_total_reduce_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "nnz") && any_name(d, "thread");
}

bool thread_total_reduce_operator::is_valid_according_to_metadata() { return has(THREAD_META, "first_nz_indices"); }

// thread_total_reduce_operator.cc:57-79
void thread_total_reduce_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "thread_total_reduce: no THREAD first_nz_indices");
    reduction_token t;
    t.kind = reduction_kind::TOTAL_BMT_RESULT;
    t.need_warp_reduction = need_warp_reduction;
    t.sparse_coarsen_factor = sparse_coarsen_factor;
    t.coarsen_factor = coarsen_factor;
    code_generator_ptr->set_reduction_token(THREAD_META, t);
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    is_run = true;
}

warp_total_reduce_operator::warp_total_reduce_operator(cg_ptr cg, int cf, ctx_ptr)
    : basic_operator("warp_total_reduce_operator", cg->get_metadata_set(), IMPLEMENTING_OP, cg->get_sub_matrix_id()),
      coarsen_factor(cf), code_generator_ptr(cg) {}

// warp_total_reduce_operator.cc:14-38
bool warp_total_reduce_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "nnz") && any_name(d, "warp");
}

bool warp_total_reduce_operator::is_valid_according_to_metadata() { return has(WARP_META, "first_nz_indices"); }

void warp_total_reduce_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "warp_total_reduce: no WARP first_nz_indices");
    reduction_token t;
    t.kind = reduction_kind::TOTAL_WARP_RESULT;
    t.coarsen_factor = coarsen_factor;
    code_generator_ptr->set_reduction_token(WARP_META, t);
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

tblock_total_reduce_operator::tblock_total_reduce_operator(cg_ptr cg, int cf, ctx_ptr)
    : basic_operator("tblock_total_reduce_operator", cg->get_metadata_set(), IMPLEMENTING_OP,
                     cg->get_sub_matrix_id()),
      coarsen_factor(cf), code_generator_ptr(cg) {}

// tblock_total_reduce_operator.cc
bool tblock_total_reduce_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "nnz") && any_name(d, "tblock");
}

bool tblock_total_reduce_operator::is_valid_according_to_metadata() { return has(TBLOCK_META, "first_nz_indices"); }

void tblock_total_reduce_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "tblock_total_reduce: no TBLOCK first_nz_indices");
    reduction_token t;
    t.kind = reduction_kind::TOTAL_BLOCK_RESULT;
    t.coarsen_factor = coarsen_factor;
    code_generator_ptr->set_reduction_token(TBLOCK_META, t);
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

thread_bit_map_operator::thread_bit_map_operator(cg_ptr cg, POS_TYPE pos, unsigned size, unsigned scf, unsigned cf,
                                                 ctx_ptr)
    : basic_operator("thread_bit_map_operator", cg->get_metadata_set(), IMPLEMENTING_OP, cg->get_sub_matrix_id()),
      pos(pos), size(size), sparse_coarsen_factor(scf), coarsen_factor(cf), code_generator_ptr(cg) {
    GS_CHECK(cf <= 16, "coarsen_factor <= 16");
    GS_CHECK(size >= 1, "bitmap group size >= 1");
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
}

// thread_bit_map_operator.cc (is_valid_according_to_operator)
bool thread_bit_map_operator::is_valid_according_to_operator(ctx_ptr h) {
    if (!h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id).empty()) return false;
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return any_name(d, "thread") && any_name(d, "nnz");
}

bool thread_bit_map_operator::is_valid_according_to_metadata() { return has(THREAD_META, "first_nz_indices"); }

// thread_bit_map_operator.cc:60-101
void thread_bit_map_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "thread_bit_map: no THREAD first_nz_indices");
    bool parent_flag = pos != THREAD_META;
    thread_bit_map a(meta_data_set_ptr, parent_flag, (int)size, target_matrix_id);
    run_step(a, check);
    segment_empty_flag b(meta_data_set_ptr, pos, (int)size, target_matrix_id);
    run_step(b, check);
    segment_empty_row_indices c(meta_data_set_ptr, pos, target_matrix_id);
    run_step(c, check);
    segment_offset d(meta_data_set_ptr, false, (int)size, target_matrix_id);
    run_step(d, check);
    segment_ptr e(meta_data_set_ptr, pos, target_matrix_id);
    run_step(e, check);
    reduction_token t;
    t.kind = reduction_kind::THREAD_BIT_MAP;
    t.need_warp_reduction = pos == WARP_META;
    t.sparse_coarsen_factor = (int)sparse_coarsen_factor;
    t.coarsen_factor = (int)coarsen_factor;
    t.size = (int)size;
    code_generator_ptr->set_reduction_token(THREAD_META, t);
    code_generator_ptr->open_spec_level_of_paral(THREAD_META);
    is_run = true;
}

warp_segment_reduce_operator::warp_segment_reduce_operator(cg_ptr cg, unsigned cf, bool rnz, bool rrow, ctx_ptr)
    : basic_operator("warp_segment_reduce_operator", cg->get_metadata_set(), IMPLEMENTING_OP,
                     cg->get_sub_matrix_id()),
      coarsen_factor(cf), relative_nz(rnz), relative_row(rrow), code_generator_ptr(cg) {
    GS_CHECK(cf <= 16, "coarsen_factor <= 16");
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
}

// warp_segment_reduce_operator.cc:14-56
bool warp_segment_reduce_operator::is_valid_according_to_operator(ctx_ptr h) {
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    auto i = h->read_operator_context_arr(IMPLEMENTING_OP, target_matrix_id);
    return any_name(d, "thread") && any_name(d, "nnz") && !any_name(d, "warp") && any_name(i, "thread_bit_map");
}

bool warp_segment_reduce_operator::is_valid_according_to_metadata() {
    return has(THREAD_META, "first_nz_indices") && !has(WARP_META, "first_nz_indices");
}

// warp_segment_reduce_operator.cc:74-111; merge_num = VECTOR_WIDTH
void warp_segment_reduce_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "warp_segment_reduce: invalid metadata");
    int vw = (int)get_config().VECTOR_WIDTH;
    GS_CHECK(vw >= 1, "VECTOR_WIDTH >= 1");
    get_begin_rows_after_merge_thread a(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(a, check);
    get_begin_nzs_after_merge_thread b(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(b, check);
    if (relative_row) {  // :86-91
        get_begin_rows_relative_to_parent_after_merge_thread r(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
        run_step(r, check);
    }
    if (relative_nz) {  // :93-98
        get_begin_nzs_relative_to_parent_after_merge_thread r(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
        run_step(r, check);
    }
    get_begin_BMTs_after_merge_thread c(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(c, check);
    reduction_token t;
    t.kind = reduction_kind::WARP_SEGMENT;
    t.coarsen_factor = (int)coarsen_factor;
    t.size = vw;
    code_generator_ptr->set_reduction_token(WARP_META, t);
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// ------------------------------------------------ warp_bit_map_operator (K5)
warp_bit_map_operator::warp_bit_map_operator(cg_ptr cg, unsigned cf, bool rnz, bool rrow, ctx_ptr)
    : basic_operator("warp_bit_map_operator", cg->get_metadata_set(), IMPLEMENTING_OP, cg->get_sub_matrix_id()),
      coarsen_factor(cf), relative_nz(rnz), relative_row(rrow), code_generator_ptr(cg) {
    GS_CHECK(cf <= 16, "coarsen_factor <= 16");
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
}

// warp_bit_map_operator.cc:14-46: a thread-level distribution, no warp one, no nnz one
bool warp_bit_map_operator::is_valid_according_to_operator(ctx_ptr h) {
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "nnz") && any_name(d, "thread") && !any_name(d, "warp");
}

bool warp_bit_map_operator::is_valid_according_to_metadata() {
    return has(THREAD_META, "first_nz_indices") && !has(WARP_META, "first_nz_indices");
}

// warp_bit_map_operator.cc:69-109; merge_num = VECTOR_WIDTH
void warp_bit_map_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "warp_bit_map: invalid metadata");
    GS_CHECK(has(THREAD_META, "first_row_indices_without_ending"),
             "warp_bit_map needs col-direction BMTs (parent_bit_map_of_thread.cc reads first_row_indices_without_ending)");
    int vw = (int)get_config().VECTOR_WIDTH;
    GS_CHECK(vw >= 1, "VECTOR_WIDTH >= 1");
    get_begin_rows_after_merge_thread a(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(a, check);
    get_begin_nzs_after_merge_thread b(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(b, check);
    if (relative_row) {
        get_begin_rows_relative_to_parent_after_merge_thread c(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
        run_step(c, check);
    }
    if (relative_nz) {
        get_begin_nzs_relative_to_parent_after_merge_thread c(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
        run_step(c, check);
    }
    get_begin_BMTs_after_merge_thread e(meta_data_set_ptr, WARP_META, vw, target_matrix_id);
    run_step(e, check);
    parent_bit_map_of_thread f(meta_data_set_ptr, WARP_META, target_matrix_id);
    run_step(f, check);
    reduction_token t;
    t.kind = reduction_kind::WARP_BIT_MAP;
    t.coarsen_factor = (int)coarsen_factor;
    t.size = vw;
    code_generator_ptr->set_reduction_token(WARP_META, t);
    code_generator_ptr->open_spec_level_of_paral(WARP_META);
    is_run = true;
}

// ------------------------------------------ tblock_thread_bit_map_operator (K7)
tblock_thread_bit_map_operator::tblock_thread_bit_map_operator(cg_ptr cg, unsigned cf, int bs, bool rnz, bool rrow,
                                                               ctx_ptr)
    : basic_operator("tblock_thread_bit_map_operator", cg->get_metadata_set(), IMPLEMENTING_OP,
                     cg->get_sub_matrix_id()),
      coarsen_factor(cf), block_size(bs), relative_nz(rnz), relative_row(rrow), code_generator_ptr(cg) {
    GS_CHECK(cf <= 16, "coarsen_factor <= 16");
    GS_CHECK(bs >= 1, "block_size >= 1");
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
}

// tblock_thread_bit_map_operator.cc:14-46
bool tblock_thread_bit_map_operator::is_valid_according_to_operator(ctx_ptr h) {
    auto d = h->read_operator_context_arr(DISTRIBUTING_OP, target_matrix_id);
    return !any_name(d, "nnz") && any_name(d, "thread") && !any_name(d, "tblock");
}

bool tblock_thread_bit_map_operator::is_valid_according_to_metadata() { return has(THREAD_META, "first_nz_indices"); }

// tblock_thread_bit_map_operator.cc:62-109; merge_num = block_size
void tblock_thread_bit_map_operator::run(bool check) {
    GS_CHECK(is_valid_according_to_metadata(), "tblock_thread_bit_map: invalid metadata");
    GS_CHECK(has(THREAD_META, "first_row_indices_without_ending"),
             "tblock_thread_bit_map needs col-direction BMTs (parent_bit_map_of_thread.cc)");
    get_begin_rows_after_merge_thread a(meta_data_set_ptr, TBLOCK_META, block_size, target_matrix_id);
    run_step(a, check);
    get_begin_nzs_after_merge_thread b(meta_data_set_ptr, TBLOCK_META, block_size, target_matrix_id);
    run_step(b, check);
    if (relative_row) {
        get_begin_rows_relative_to_parent_after_merge_thread c(meta_data_set_ptr, TBLOCK_META, block_size,
                                                               target_matrix_id);
        run_step(c, check);
    }
    if (relative_nz) {
        get_begin_nzs_relative_to_parent_after_merge_thread c(meta_data_set_ptr, TBLOCK_META, block_size,
                                                              target_matrix_id);
        run_step(c, check);
    }
    get_begin_BMTs_after_merge_thread e(meta_data_set_ptr, TBLOCK_META, block_size, target_matrix_id);
    run_step(e, check);
    parent_bit_map_of_thread f(meta_data_set_ptr, TBLOCK_META, target_matrix_id);
    run_step(f, check);
    // segment_offset(meta, TBLOCK_META, block_size): the POS_TYPE argument lands in the
    // bool parent_flag parameter (TBLOCK_META = -98, i.e. true)
    segment_offset g(meta_data_set_ptr, true, block_size, target_matrix_id);
    run_step(g, check);
    reduction_token t;
    t.kind = reduction_kind::TBLOCK_BIT_MAP;
    t.coarsen_factor = (int)coarsen_factor;
    t.size = block_size;
    code_generator_ptr->set_reduction_token(TBLOCK_META, t);
    code_generator_ptr->open_spec_level_of_paral(TBLOCK_META);
    is_run = true;
}

grid_block_operator::grid_block_operator(cg_ptr cg, unsigned grid_x, std::vector<unsigned> blk, unsigned cf, ctx_ptr)
    : basic_operator("grid_block_operator", cg->get_metadata_set(), IMPLEMENTING_OP, cg->get_sub_matrix_id()),
      code_generator_ptr(cg) {
    // grid_block_operator.cc:13-25: grid_y covers the dense columns
    GS_CHECK(blk.size() == 2 && blk[0] > 0 && blk[1] > 0, "block must be {x, y}");
    if (blk[1] % 2 && blk[1] > 1) blk[1] += 1;
    unsigned N = (unsigned)get_config().DENSE_MATRIX_SIZE;
    unsigned per = std::max(1u, blk[0] * std::max(1u, cf));
    grid = {grid_x, std::max(1u, (N + per - 1) / per)};
    block = blk;
}

void grid_block_operator::run(bool) {
    code_generator_ptr->set_thread_grid(grid, block);
    is_run = true;
}

// -------------------------------------------------------------- executer
// operator_executer.cc:19-26
void operator_executer::add_and_run(const std::shared_ptr<basic_operator> &op) {
    if (!op->is_valid_according_to_operator(ctx))
        throw gs_error("operator_executer: " + op->get_name() + " is not valid after the operators already run");
    bool check = get_config().OPERATOR_RUNTIME_CHECK;
    op->run(check);
    ctx->add(op);
    history_log.push_back(op->convert_to_string());
    for (auto &s : op->get_data_transform_sequence()) history_log.push_back("  " + s);
}

// -------------------------------------------------------------- factory
std::shared_ptr<basic_operator> make_operator(const std::string &name, const std::vector<long long> &a, cg_ptr cg,
                                              ctx_ptr ctx) {
    auto need = [&](size_t n) {
        GS_CHECK(a.size() == n, name + ": expected " + std::to_string(n) + " arguments");
    };
    if (name == "sort_operator") { need(0); return std::make_shared<sort_operator>(cg, ctx); }
    if (name == "empty_row_pad_operator") { need(0); return std::make_shared<empty_row_pad_operator>(cg, ctx); }
    if (name == "fixed_interval_row_direction_tblock_blocking_operator") {
        need(2);
        return std::make_shared<fixed_interval_row_direction_tblock_blocking_operator>(cg, (int)a[0], a[1] != 0, ctx);
    }
    if (name == "fixed_interval_row_direction_warp_blocking_operator") {
        need(4);
        return std::make_shared<fixed_interval_row_direction_warp_blocking_operator>(cg, (int)a[0], a[1] != 0,
                                                                                     a[2] != 0, a[3] != 0, ctx);
    }
    if (name == "fixed_interval_row_direction_thread_blocking_operator") {
        need(7);
        return std::make_shared<fixed_interval_row_direction_thread_blocking_operator>(
            cg, (int)a[0], a[1] != 0, a[2] != 0, a[3] != 0, a[4] != 0, a[5] != 0, (int)a[6], ctx);
    }
    if (name == "fixed_interval_nnz_direction_tblock_blocking_operator") {
        need(2);
        return std::make_shared<fixed_interval_nnz_direction_tblock_blocking_operator>(cg, (int)a[0], a[1] != 0, ctx);
    }
    if (name == "fixed_interval_nnz_direction_warp_blocking_operator") {
        need(4);
        return std::make_shared<fixed_interval_nnz_direction_warp_blocking_operator>(cg, (int)a[0], a[1] != 0, a[2] != 0,
                                                                                     a[3] != 0, ctx);
    }
    if (name == "fixed_interval_nnz_direction_thread_blocking_operator") {
        need(4);
        return std::make_shared<fixed_interval_nnz_direction_thread_blocking_operator>(cg, (int)a[0], a[1] != 0,
                                                                                       a[2] != 0, a[3] != 0, ctx);
    }
    if (name == "fixed_interval_col_direction_thread_blocking_operator") {
        need(5);  // fixed_col_block_size, row_relative, nz_relative, pad_to_multiple, pad_to_parent_max
        return std::make_shared<fixed_interval_col_direction_thread_blocking_operator>(cg, (int)a[0], a[1] != 0,
                                                                                       a[2] != 0, a[3] != 0,
                                                                                       a[4] != 0, ctx);
    }
    if (name == "fixed_interval_col_direction_tblock_blocking_operator") {
        need(3);  // fixed_col_block_size, pad_to_multiple, pad_to_parent_max
        return std::make_shared<fixed_interval_col_direction_tblock_blocking_operator>(cg, (int)a[0], a[1] != 0, a[2] != 0,
                                                                                       ctx);
    }
    if (name == "fixed_interval_col_direction_warp_blocking_operator") {
        need(5);  // fixed_col_block_size, row_relative, nz_relative, pad_to_multiple, pad_to_parent_max
        return std::make_shared<fixed_interval_col_direction_warp_blocking_operator>(cg, (int)a[0], a[1] != 0, a[2] != 0,
                                                                                     a[3] != 0, a[4] != 0, ctx);
    }
    if (name == "warp_bit_map_operator") {
        need(3);
        return std::make_shared<warp_bit_map_operator>(cg, (unsigned)a[0], a[1] != 0, a[2] != 0, ctx);
    }
    if (name == "tblock_thread_bit_map_operator") {
        need(4);
        return std::make_shared<tblock_thread_bit_map_operator>(cg, (unsigned)a[0], (int)a[1], a[2] != 0, a[3] != 0,
                                                                ctx);
    }
    if (name == "balanced_interval_row_direction_warp_blocking_operator") {
        need(3);
        return std::make_shared<balanced_interval_row_direction_warp_blocking_operator>(cg, (int)a[0], a[1] != 0,
                                                                                        a[2] != 0, ctx);
    }
    if (name == "balanced_interval_row_direction_tblock_blocking_operator") {
        need(1);
        return std::make_shared<balanced_interval_row_direction_tblock_blocking_operator>(cg, (int)a[0], ctx);
    }
    if (name == "balanced_interval_row_direction_thread_blocking_operator") {
        need(3);
        return std::make_shared<balanced_interval_row_direction_thread_blocking_operator>(cg, (int)a[0], a[1] != 0,
                                                                                          a[2] != 0, ctx);
    }
    if (name == "row_nz_matrix_div_operator") {
        need(3);
        return std::make_shared<row_nz_matrix_div_operator>(cg, (int)a[0], (int)a[1], (int)a[2], ctx);
    }
    if (name == "fixed_interval_row_matrix_div_operator") {
        need(1);
        return std::make_shared<fixed_interval_row_matrix_div_operator>(cg, (int)a[0], ctx);
    }
    if (name == "interlance_storage_operator") { need(0); return std::make_shared<interlance_storage_operator>(cg, ctx); }
    if (name == "merge_path_tblock_operator") { need(1); return std::make_shared<merge_path_tblock_operator>(cg, (int)a[0], ctx); }
    if (name == "merge_path_warp_operator") { need(1); return std::make_shared<merge_path_warp_operator>(cg, (int)a[0], ctx); }
    if (name == "merge_path_thread_operator") { need(1); return std::make_shared<merge_path_thread_operator>(cg, (int)a[0], ctx); }
    if (name == "thread_total_reduce_operator") {
        need(3);
        return std::make_shared<thread_total_reduce_operator>(cg, a[0] != 0, (int)a[1], (int)a[2], ctx);
    }
    if (name == "warp_total_reduce_operator") {
        need(1);
        return std::make_shared<warp_total_reduce_operator>(cg, (int)a[0], ctx);
    }
    if (name == "tblock_total_reduce_operator") {
        need(1);
        return std::make_shared<tblock_total_reduce_operator>(cg, (int)a[0], ctx);
    }
    if (name == "thread_bit_map_operator") {
        need(4);  // pos (0 THREAD, 1 WARP, 2 TBLOCK), size, sparse_cf, cf
        POS_TYPE p = a[0] == 1 ? WARP_META : (a[0] == 2 ? TBLOCK_META : THREAD_META);
        return std::make_shared<thread_bit_map_operator>(cg, p, (unsigned)a[1], (unsigned)a[2], (unsigned)a[3], ctx);
    }
    if (name == "warp_segment_reduce_operator") {
        need(3);
        return std::make_shared<warp_segment_reduce_operator>(cg, (unsigned)a[0], a[1] != 0, a[2] != 0, ctx);
    }
    if (name == "grid_block_operator") {
        need(4);  // grid_x, block_x, block_y, cf
        return std::make_shared<grid_block_operator>(cg, (unsigned)a[0],
                                                     std::vector<unsigned>{(unsigned)a[1], (unsigned)a[2]},
                                                     (unsigned)a[3], ctx);
    }
    throw gs_error("unknown operator " + name);
}

}  // namespace gs
